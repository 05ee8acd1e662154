// TEST DOUBLE: the loader type registered beside a scorer (Mm::AbstractMixtureSetLoader)
#pragma once
namespace Mm {
class AbstractMixtureSetLoader {
public:
    virtual ~AbstractMixtureSetLoader() {}
};
}  // namespace Mm
