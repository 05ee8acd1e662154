// TEST DOUBLE: a feature with one stream (Mm::Feature::mainStream), and the feature description
#pragma once
#include <map>
#include <string>
#include <Core/ReferenceCounting.hh>
#include "Types.hh"
namespace Mm {
class Feature : public Core::ReferenceCounted {
public:
    struct Vector : public Core::ReferenceCounted, public FeatureVector {
        explicit Vector(const FeatureVector& v) : FeatureVector(v) {}
    };
    explicit Feature(const FeatureVector& v) : main_(new Vector(v)) {}
    Core::Ref<const Vector> mainStream() const { return main_; }

private:
    Core::Ref<const Vector> main_;
};

class FeatureDescription {
public:
    struct Stream {
        std::map<std::string, size_t> values;
        void setValue(const std::string& name, size_t v) { values[name] = v; }
    };
    static constexpr const char* nameDimension = "dimension";
    Stream& mainStream() { return main_; }

private:
    Stream main_;
};
}  // namespace Mm
