// TEST DOUBLE: Mm::FeatureScorerFactory -- registry of creation functions by id (and name), createInstance
// constructs T(config, Ref<const ModelType>) after a dynamic_cast of the model
#pragma once
#include <map>
#include <string>
#include <Core/Assertions.hh>
#include "FeatureScorer.hh"
#include "MixtureSet.hh"
#include "MixtureSetLoader.hh"
#include "Module.hh"
namespace Mm {
class FeatureScorerFactory {
    typedef FeatureScorer* (*CreationFunction)(const Core::Configuration&, Core::Ref<const AbstractMixtureSet>);

public:
    template <class T, class ModelType, class Loader>
    bool registerFeatureScorer(u32 id, const char* name) {
        if (registry_.count(id))
            return false;
        registry_[id] = &createInstance<T, ModelType>;
        names_[name]  = id;
        return true;
    }
    FeatureScorer* createFeatureScorer(u32 id, const Core::Configuration& c, Core::Ref<const AbstractMixtureSet> m) const {
        auto it = registry_.find(id);
        return it == registry_.end() ? 0 : it->second(c, m);
    }
    bool idOf(const std::string& name, u32& id) const {
        auto it = names_.find(name);
        if (it == names_.end())
            return false;
        id = it->second;
        return true;
    }

private:
    template <class T, class ModelType>
    static FeatureScorer* createInstance(const Core::Configuration& c, Core::Ref<const AbstractMixtureSet> m) {
        verify(m);
        const ModelType* casted = dynamic_cast<const ModelType*>(m.get());
        ensure(casted);
        return new T(c, Core::Ref<const ModelType>(casted));
    }
    std::map<u32, CreationFunction> registry_;
    std::map<std::string, u32>      names_;
};
inline FeatureScorerFactory* Module_::featureScorerFactory() {
    static FeatureScorerFactory f;
    return &f;
}
}  // namespace Mm
