// GpuBatchFeatureScorer.hh -- the RASR-side adapter for the hybrid-DNN scorer: an Mm::FeatureScorer with the
// buffered protocol of Nn::BatchFeatureScorer whose network is evaluated by the MI355X scorer library
// (librasr_gmm.so, include/rasr_nn.h: one bf16 MFMA GEMM per layer, bias and activation fused).  A maintainer
// copies integration/rasr/Nn/* into src/Nn/ of an RASR tree (plus -I<this repo>/include and -lrasr_gmm,
// INTEGRATION.md); `make check-integration` compiles it here -fsyntax-only against the reference's own headers.
//
// Interfaces implemented (reference file:line):
//   Mm::FeatureScorer (buffered protocol)  src/Mm/FeatureScorer.hh:28-164 (:70-134)
//   Nn::BatchFeatureScorer                 src/Nn/BatchFeatureScorer.hh:36-176, .cc:25-171: the same
//                                          configuration (network, "buffer-size", prior, class labels), the
//                                          same init checks, the same ring buffer and getScore
//   registration                           src/Nn/Module.cc:39-67 at the Nn id range (src/Nn/Module.hh:36-44)
//
// The network is built by the reference's own Nn::NeuralNetwork<f32> from the configuration (so parameter files,
// layer types and "gamma" are read exactly as the reference reads them), the log prior is removed from the top
// layer's bias by the reference's own LinearAndSoftmaxLayer::removeLogPriorFromBias, and then every layer's
// weights, bias and activation are handed to nn_scorer_create; the host copy of the network is released.
// Supported topologies: one feature stream, a chain of linear(+activation) layers (linear+sigmoid/tanh/
// rectified/elu/softmax, or linear followed by an activation layer), the top one linear+softmax.  Anything else
// is refused with criticalError at construction.
//
// Two translation units: GpuBatchFeatureScorer.cc (the buffered protocol and the registration; Mm headers only)
// and GpuBatchFeatureScorerNetwork.cc (initNetwork: the reference's NeuralNetwork, Prior and ClassLabelWrapper,
// whose headers pull in Math/Blas.hh and so <cblas.h>).
#ifndef _NN_GPU_BATCH_FEATURESCORER_HH
#define _NN_GPU_BATCH_FEATURESCORER_HH

#include <Core/Parameter.hh>
#include <Mm/Feature.hh>
#include <Mm/FeatureScorer.hh>
#include <Mm/MixtureSet.hh>
#include <Mm/Types.hh>

#include <rasr_nn.h>  // this repo's include/

#include <vector>

namespace Nn {

class GpuBatchFeatureScorer : public Mm::FeatureScorer {
    typedef Mm::FeatureScorer Precursor;

public:
    static const Core::ParameterInt paramBufferSize;  // "buffer-size" (BatchFeatureScorer.cc:21-22)
    static const Core::ParameterInt paramDevice;      // "device": HIP device of this process

    GpuBatchFeatureScorer(const Core::Configuration& c, Core::Ref<const Mm::MixtureSet> mixtureSet);
    virtual ~GpuBatchFeatureScorer();

    virtual Mm::EmissionIndex nMixtures() const {
        return nClasses_;
    }
    virtual void getFeatureDescription(Mm::FeatureDescription& description) const {
        description.mainStream().setValue(Mm::FeatureDescription::nameDimension, inputDimension_);
    }

    virtual FeatureScorer::Scorer getScorer(Core::Ref<const Mm::Feature> f) const {
        return getScorer(*f->mainStream());
    }
    virtual FeatureScorer::Scorer getScorer(const Mm::FeatureVector& f) const;  // BatchFeatureScorer.cc:105-117
    virtual Mm::Score             getScore(Mm::EmissionIndex e, u32 position) const;  // cc:148-171

    virtual void reset() const;  // cc:99-103
    virtual void finalize() const {}
    virtual bool isBuffered() const {
        return true;
    }
    virtual void addFeature(const Mm::FeatureVector& f) const;  // cc:92-97
    virtual void addFeature(Core::Ref<const Mm::Feature> f) const {
        addFeature(*f->mainStream());
    }
    virtual FeatureScorer::Scorer flush() const;  // cc:119-134 (scores a pending last frame before clearing)
    virtual bool                  bufferFilled() const {
        return nBufferedFeatures_ >= bufferSize_ - 1;
    }
    virtual bool bufferEmpty() const {
        return nBufferedFeatures_ == 0;
    }
    virtual u32 bufferSize() const {
        return bufferSize_;
    }

private:
    class ContextScorer;
    // BatchFeatureScorer::init (cc:45-79) with the reference's own network, prior and label objects, then the
    // upload (GpuBatchFeatureScorerNetwork.cc): sets nClasses_, inputDimension_, nOutputs_, outputIndex_, scorer_
    void initNetwork(Core::Ref<const Mm::MixtureSet> mixtureSet);
    void setFeature(u32 position, const Mm::FeatureVector& f) const;
    void computeScores() const;  // every buffer position in one nn_score_host_ex call

    const u32                 bufferSize_;
    mutable u32               nBufferedFeatures_;
    mutable u32               currentFeature_;
    mutable std::vector<bool> scoreComputed_;
    u32                       nClasses_, inputDimension_, nOutputs_;
    // ClassLabelWrapper: output index of each class, -1 where !isClassToAccumulate (BatchFeatureScorer.cc:164-170)
    std::vector<s32>          outputIndex_;
    nn_scorer*                scorer_;
    // page-locked (gmm_host_alloc): the [bufferSize][inputDimension] feature ring and the frame-major
    // [bufferSize][nOutputs] table of -output (the reference's output matrix holds a frame per column)
    float* buffer_;
    float* scores_;
};

// Registers "gpu-nn-batch-feature-scorer" with the reference factory (Mm::Module::instance().featureScorerFactory()),
// like Nn::Module_ registers "nn-batch-feature-scorer" (src/Nn/Module.cc:47-48); the default id sits after the Nn
// module's own range (Module_::FeatureScorerTypeOffset = 0x300 .. 0x306, src/Nn/Module.hh:36-44).
void registerGpuBatchFeatureScorer(u32 id = 0x310);

}  // namespace Nn

#endif  // _NN_GPU_BATCH_FEATURESCORER_HH
