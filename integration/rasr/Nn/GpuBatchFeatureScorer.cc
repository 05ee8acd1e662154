// GpuBatchFeatureScorer.cc -- the buffered protocol and the registration (see GpuBatchFeatureScorer.hh); the
// network upload is GpuBatchFeatureScorerNetwork.cc.
#include "GpuBatchFeatureScorer.hh"

#include <Mm/FeatureScorerFactory.hh>
#include <Mm/MixtureSetLoader.hh>
#include <Mm/Module.hh>

#include <cstring>

using namespace Nn;

const Core::ParameterInt GpuBatchFeatureScorer::paramBufferSize(
        "buffer-size", "buffer size (and also batch size) for the feature scorer", 8);
const Core::ParameterInt GpuBatchFeatureScorer::paramDevice(
        "device", "HIP device of this process (one process per GPU)", 0, 0);

namespace {

void* hostAlloc(size_t bytes) {
    void* p = 0;
    return gmm_host_alloc(bytes, &p) == GMM_OK ? p : 0;
}

}  // namespace

// BatchFeatureScorer::ContextScorer (BatchFeatureScorer.hh:52-72): (parent, buffer position)
class GpuBatchFeatureScorer::ContextScorer : public Mm::FeatureScorer::ContextScorer {
public:
    ContextScorer(const GpuBatchFeatureScorer* parent, u32 currentFeature)
            : parent_(parent), currentFeature_(currentFeature) {}
    virtual Mm::EmissionIndex nEmissions() const {
        return parent_->nMixtures();
    }
    virtual Mm::Score score(Mm::EmissionIndex e) const {
        return parent_->getScore(e, currentFeature_);
    }

private:
    const GpuBatchFeatureScorer* parent_;
    u32                          currentFeature_;
};

GpuBatchFeatureScorer::GpuBatchFeatureScorer(const Core::Configuration& c, Core::Ref<const Mm::MixtureSet> mixtureSet)
        : Core::Component(c),
          Precursor(c),
          bufferSize_(paramBufferSize(c)),
          nBufferedFeatures_(0),
          currentFeature_(0),
          scoreComputed_(bufferSize_, false),
          nClasses_(0),
          inputDimension_(0),
          nOutputs_(0),
          scorer_(0),
          buffer_(0),
          scores_(0) {
    initNetwork(mixtureSet);
    buffer_ = static_cast<float*>(hostAlloc(static_cast<size_t>(bufferSize_) * inputDimension_ * sizeof(float)));
    scores_ = static_cast<float*>(hostAlloc(static_cast<size_t>(bufferSize_) * nOutputs_ * sizeof(float)));
    if (!buffer_ || !scores_)
        criticalError("GPU nn scorer: %s", gmm_last_error());
    std::memset(buffer_, 0, static_cast<size_t>(bufferSize_) * inputDimension_ * sizeof(float));
}

GpuBatchFeatureScorer::~GpuBatchFeatureScorer() {
    nn_scorer_destroy(scorer_);
    gmm_host_free(buffer_);
    gmm_host_free(scores_);
}

// BatchFeatureScorer::setFeature (cc:81-90)
void GpuBatchFeatureScorer::setFeature(u32 position, const Mm::FeatureVector& f) const {
    require_lt(position, bufferSize_);
    require_eq(f.size(), inputDimension_);
    std::memcpy(buffer_ + static_cast<size_t>(position) * inputDimension_, &f[0], inputDimension_ * sizeof(float));
}

void GpuBatchFeatureScorer::addFeature(const Mm::FeatureVector& f) const {
    require(!bufferFilled());
    setFeature(nBufferedFeatures_, f);
    scoreComputed_[nBufferedFeatures_] = false;
    nBufferedFeatures_++;
}

void GpuBatchFeatureScorer::reset() const {
    scoreComputed_.assign(bufferSize_, false);
    nBufferedFeatures_ = 0;
    currentFeature_    = 0;
}

Mm::FeatureScorer::Scorer GpuBatchFeatureScorer::getScorer(const Mm::FeatureVector& f) const {
    require(bufferFilled());
    const u32 position = currentFeature_ ? (currentFeature_ - 1) % bufferSize_ : bufferSize_ - 1;
    setFeature(position, f);
    scoreComputed_[position] = false;
    Scorer scorer(new ContextScorer(this, currentFeature_));
    currentFeature_ = (currentFeature_ + 1) % bufferSize_;
    return scorer;
}

// BatchFeatureScorer::flush (cc:119-134).  Deliberate deviation: the reference clears the feature buffer when the
// last buffered frame is flushed, BEFORE that frame's context is read; when the frame was added after the last
// forward pass (its scores not computed yet) the reference then scores an all-zero frame for it.  Here the pending
// scores are computed first, so the last frame of a segment scores its own features.
Mm::FeatureScorer::Scorer GpuBatchFeatureScorer::flush() const {
    require(!bufferEmpty());
    const u32 position = currentFeature_;
    Scorer    scorer(new ContextScorer(this, position));
    currentFeature_ = (currentFeature_ + 1) % bufferSize_;
    nBufferedFeatures_--;
    if (bufferEmpty()) {
        if (!scoreComputed_[position])
            computeScores();
        currentFeature_ = 0;
        std::memset(buffer_, 0, static_cast<size_t>(bufferSize_) * inputDimension_ * sizeof(float));
    }
    return scorer;
}

// the whole buffer in one call (network_.forward(buffer_), cc:155-163)
void GpuBatchFeatureScorer::computeScores() const {
    if (nn_score_host_ex(scorer_, buffer_, bufferSize_, inputDimension_, scores_, nOutputs_, NN_HOST_FRAME_MAJOR) != GMM_OK)
        criticalError("GPU nn scorer: %s", nn_last_error());
    scoreComputed_.assign(bufferSize_, true);
}

// BatchFeatureScorer::getScore (cc:148-171): the whole buffer in one call when a position is out of date
Mm::Score GpuBatchFeatureScorer::getScore(Mm::EmissionIndex e, u32 position) const {
    require_lt(position, bufferSize_);
    require_lt(e, nClasses_);
    if (!scoreComputed_[position])
        computeScores();
    if (outputIndex_[e] < 0)  // !labelWrapper_->isClassToAccumulate(e)
        return Core::Type<Mm::Score>::max;
    // the table holds -output (nn_score_*: score = -(W^T h + b)), the reference's -getTopLayerOutput().at(e, position)
    return scores_[static_cast<size_t>(position) * nOutputs_ + static_cast<u32>(outputIndex_[e])];
}

// ---------------------------------------------------------------------------
// registration (Nn::Module_::Module_, src/Nn/Module.cc:39-67)
void Nn::registerGpuBatchFeatureScorer(u32 id) {
    Mm::Module::instance().featureScorerFactory()->registerFeatureScorer<GpuBatchFeatureScorer, Mm::MixtureSet,
                                                                          Mm::AbstractMixtureSetLoader>(
            id, "gpu-nn-batch-feature-scorer");
}
