// TEST DOUBLE: Mm::FeatureScorerScaling -- the wrapper the acoustic model hands to the search:
// ScaledContextScorer::score(e) = scale * inner score(e); the buffered protocol forwarded
#pragma once
#include "AssigningFeatureScorer.hh"
#include "FeatureScorer.hh"
namespace Mm {
class FeatureScorerScaling : public FeatureScorer {
public:
    class ScaledContextScorer : public ContextScorer {
    public:
        ScaledContextScorer(Scorer s, Score scale) : scorer_(s), scale_(scale) {}
        virtual EmissionIndex nEmissions() const { return scorer_->nEmissions(); }
        virtual Score         score(EmissionIndex e) const { return scale_ * scorer_->score(e); }
        Scorer                getUnscaledScorer() const { return scorer_; }

    private:
        Scorer scorer_;
        Score  scale_;
    };
    FeatureScorerScaling(const Core::Configuration& c, Core::Ref<FeatureScorer> fs, Score scale)
            : Core::Component(c), FeatureScorer(c), featureScorer_(fs), scale_(scale) {}
    virtual EmissionIndex nMixtures() const { return featureScorer_->nMixtures(); }
    virtual void          getFeatureDescription(FeatureDescription& d) const { featureScorer_->getFeatureDescription(d); }
    virtual Scorer getScorer(Core::Ref<const Feature> f) const { return Scorer(new ScaledContextScorer(featureScorer_->getScorer(f), scale_)); }
    virtual Scorer getScorer(const FeatureVector& f) const { return Scorer(new ScaledContextScorer(featureScorer_->getScorer(f), scale_)); }
    virtual void   reset() const { featureScorer_->reset(); }
    virtual void   finalize() const { featureScorer_->finalize(); }
    virtual bool   isBuffered() const { return featureScorer_->isBuffered(); }
    virtual void   addFeature(const FeatureVector& f) const { featureScorer_->addFeature(f); }
    virtual void   addFeature(Core::Ref<const Feature> f) const { featureScorer_->addFeature(f); }
    virtual Scorer flush() const { return Scorer(new ScaledContextScorer(featureScorer_->flush(), scale_)); }
    virtual bool   bufferFilled() const { return featureScorer_->bufferFilled(); }
    virtual bool   bufferEmpty() const { return featureScorer_->bufferEmpty(); }
    virtual u32    bufferSize() const { return featureScorer_->bufferSize(); }
    Core::Ref<const AssigningFeatureScorer> assigningFeatureScorer() const {
        return Core::Ref<const AssigningFeatureScorer>(dynamic_cast<const AssigningFeatureScorer*>(featureScorer_.get()));
    }

private:
    Core::Ref<FeatureScorer> featureScorer_;
    Score                    scale_;
};
}  // namespace Mm
