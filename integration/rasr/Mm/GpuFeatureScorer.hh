// GpuFeatureScorer.hh -- the RASR-side adapter: an Mm::AssigningFeatureScorer whose scores come from the
// MI355X scorer library (librasr_gmm.so, include/rasr_gmm.h).  A maintainer copies integration/rasr/Mm/*
// into src/Mm/ of an RASR tree (plus -I<this repo>/include -I<this repo>/rasr_amd/csrc and
// -lrasr_gmm); `make check-integration` compiles it here -fsyntax-only against the
// reference's own headers.
//
// Interfaces implemented (reference file:line):
//   Mm::FeatureScorer                  src/Mm/FeatureScorer.hh:28-164 (buffered protocol :70-134)
//   Mm::AssigningFeatureScorer         src/Mm/AssigningFeatureScorer.hh:24-92 (bestDensity :36-48),
//                                      read by the aligners (src/Speech/AlignmentNode.cc:283-310)
//   BatchFeatureScorerBase protocol    src/Mm/BatchFeatureScorer.cc:40-105 (ring buffer, getScore)
//   registration                       src/Mm/FeatureScorerFactory.hh:54-66,114-122
//
// The ring buffer, the score cache and the launches are those of Mm::Gpu::GpuBatchFeatureScorer
// (rasr_amd/csrc/host/GpuFeatureScorer.hh), the class the GPU protocol tests drive: one launch scores
// every mixture of the buffered frames into a page-locked [mixtures][buffer-size] table that is reused
// for the scorer's lifetime.  buffer-size 1 gives the unbuffered behaviour of SIMD-diagonal-maximum
// (bufferFilled() is always true, every getScorer() scores its own frame).
#ifndef _MM_GPU_FEATURESCORER_HH
#define _MM_GPU_FEATURESCORER_HH

#include <Core/Parameter.hh>
#include <Mm/AssigningFeatureScorer.hh>
#include <Mm/MixtureSet.hh>

#include <memory>

#include <host/GpuFeatureScorer.hh>  // Mm::Gpu (this repo, rasr_amd/csrc/host)

namespace Mm {

class GpuFeatureScorer : public AssigningFeatureScorer {
    typedef AssigningFeatureScorer Precursor;

public:
    static const Core::ParameterInt   paramBufferSize;          // "buffer-size" (BatchFeatureScorer.cc:27-28)
    static const Core::ParameterInt   paramDevice;              // "device": HIP device of this process
    // "density-shard-devices": the model's densities split over these GPUs of the process (BASELINE config 4,
    // gmm_scorer_create_sharded; RCCL all-reduce for the mixtures split between GPUs); empty: all on "device"
    static const Core::ParameterIntVector paramShardDevices;
    static const Core::ParameterFloat paramMixtureWeightScale;  // GaussDiagonalMaximumFeatureScorer.cc:38-40
    static const Core::ParameterFloat paramGaussianScale;       // GaussDiagonalMaximumFeatureScorer.cc:42-44
    // the "density-clustering" sub-component of the preselection types (DensityClustering.cc:19-32)
    static const Core::ParameterInt   paramClusters;
    static const Core::ParameterInt   paramSelectClusters;
    static const Core::ParameterInt   paramClusteringIterations;
    static const Core::ParameterFloat paramBackoffScore;
    static const Core::ParameterString paramCacheArchive;

    // scorerType: a reference registration name ("SIMD-diagonal-maximum", "diagonal-maximum",
    // "batch-diagonal-maximum-int", ..., Mm::Gpu::createFeatureScorer)
    GpuFeatureScorer(const Core::Configuration& c, Core::Ref<const MixtureSet> mixtureSet, const char* scorerType);
    virtual ~GpuFeatureScorer();

    virtual EmissionIndex  nMixtures() const;
    virtual ComponentIndex dimension() const;

    using Precursor::getAssigningScorer;
    virtual Scorer getScorer(Core::Ref<const Feature> f) const {
        return getScorer(*f->mainStream());
    }
    virtual Scorer          getScorer(const FeatureVector& f) const;  // BatchFeatureScorer.cc:77-87
    virtual AssigningScorer getAssigningScorer(const FeatureVector& f) const;

    virtual void reset() const;  // BatchFeatureScorer.cc:40-44
    virtual void finalize() const;
    virtual bool isBuffered() const;
    virtual void addFeature(const FeatureVector& f) const;  // BatchFeatureScorer.cc:46-50
    virtual void addFeature(Core::Ref<const Feature> f) const {
        addFeature(*f->mainStream());
    }
    virtual Scorer flush() const;  // BatchFeatureScorer.cc:89-96
    virtual bool   bufferFilled() const;
    virtual bool   bufferEmpty() const;
    virtual u32    bufferSize() const;

private:
    class Context;
    friend class Context;
    AssigningScorer wrap(const Gpu::Scorer& s) const;

    std::unique_ptr<Gpu::FeatureScorer> impl_;
};

// Registers the GPU scorers with the reference factory (Mm::Module::instance().featureScorerFactory()),
// ids from `firstId` on (add-on modules use an offset range; the Nn module takes 0x300,
// src/Nn/Module.hh:36-44).  Names: "gpu-" + the reference name, e.g. "gpu-SIMD-diagonal-maximum".
void registerGpuFeatureScorers(u32 firstId = 0x500);

}  // namespace Mm

#endif  // _MM_GPU_FEATURESCORER_HH
