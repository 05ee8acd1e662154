// TEST DOUBLE: Mm::Module::instance().featureScorerFactory()
#pragma once
namespace Mm {
class FeatureScorerFactory;
class Module_ {
public:
    FeatureScorerFactory* featureScorerFactory();
};
struct Module {
    static Module_& instance() {
        static Module_ m;
        return m;
    }
};
}  // namespace Mm
