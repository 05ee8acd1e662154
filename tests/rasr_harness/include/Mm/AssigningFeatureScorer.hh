// TEST DOUBLE: Mm::AssigningFeatureScorer (best density per emission)
#pragma once
#include <vector>
#include "FeatureScorer.hh"
namespace Mm {
class AssigningFeatureScorer : public FeatureScorer {
    typedef FeatureScorer Precursor;

public:
    class AssigningContextScorer : public ContextScorer {
    protected:
        AssigningContextScorer() {}

    public:
        virtual ~AssigningContextScorer() {}
        virtual EmissionIndex    nEmissions() const                                                                = 0;
        virtual Score            score(EmissionIndex e) const                                                      = 0;
        virtual DensityInMixture bestDensity(EmissionIndex e) const                                                = 0;
        virtual Score            score(EmissionIndex e, DensityIndex dnsInMix) const                               = 0;
        virtual void             getDensityPosteriorProbabilities(EmissionIndex e, std::vector<Weight>& r) const = 0;
    };

    explicit AssigningFeatureScorer(const Core::Configuration& c) : Core::Component(c), Precursor(c) {}
    virtual ~AssigningFeatureScorer() {}
    virtual void getFeatureDescription(FeatureDescription& description) const {
        description.mainStream().setValue(FeatureDescription::nameDimension, dimension());
    }
    virtual Scorer getScorer(Core::Ref<const Feature> f) const { return getAssigningScorer(f); }
    virtual Scorer getScorer(const FeatureVector& f) const { return getAssigningScorer(f); }
    typedef Core::Ref<const AssigningContextScorer> AssigningScorer;
    virtual AssigningScorer getAssigningScorer(Core::Ref<const Feature> f) const { return getAssigningScorer(*f->mainStream()); }
    virtual AssigningScorer getAssigningScorer(const FeatureVector&) const = 0;
    virtual ComponentIndex  dimension() const                              = 0;
};
}  // namespace Mm
