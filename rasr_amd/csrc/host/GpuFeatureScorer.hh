// GpuFeatureScorer.hh -- host-side C++ mirror of RASR's feature-scorer plugin surface on top of
// the MI355X C-ABI (include/rasr_gmm.h).
//
// Class and method names follow src/Mm/FeatureScorer.hh:28-164 (FeatureScorer, ContextScorer,
// the buffered protocol isBuffered/addFeature/flush/bufferFilled/bufferEmpty/bufferSize/reset),
// src/Mm/AssigningFeatureScorer.hh:29-48 (bestDensity) and src/Mm/BatchFeatureScorer.hh:34-199
// (ring buffer semantics).  Core::Ref<const ContextScorer> becomes std::shared_ptr; Core
// configuration parameters become a plain struct.  Inside an RASR build these classes are the
// bodies of Mm::FeatureScorer subclasses (INTEGRATION.md shows the registration).
//
// Errors: the constructors never throw; create() returns nullptr and sets *error (the reference
// calls criticalError(), src/Mm/Module.cc:305).  A failure while scoring (a device error) is never
// answered with stale or missing scores: it goes to the critical-error handler, which aborts with
// gmm_last_error() by default (Core::Component::criticalError); an RASR build routes it to the
// component's own criticalError (integration/rasr/Mm/GpuFeatureScorer.cc).  Methods keep the
// reference's require() preconditions as assertions.
#pragma once

#include <cstdint>
#include <memory>
#include <unordered_map>
#include <string>
#include <vector>

#include "../../../include/rasr_gmm.h"
#include "../../../include/rasr_gmm_io.h"

namespace Mm {
namespace Gpu {

typedef float                    Score;            // Mm::Score (src/Mm/Types.hh)
typedef uint32_t                 EmissionIndex;    // Mm::EmissionIndex
typedef uint32_t                 DensityInMixture; // Mm::DensityInMixture
typedef std::vector<float>       FeatureVector;    // Mm::FeatureVector

// Critical errors while scoring (Core::Component::criticalError, src/Core/Component.hh): the handler
// must not return normally into the scorer (abort, exit or throw); the default prints the message and
// aborts.  Returns the previous handler.
typedef void (*CriticalErrorHandler)(const std::string& message);
CriticalErrorHandler setCriticalErrorHandler(CriticalErrorHandler handler);

// Page-locked host table (gmm_host_alloc): gmm_score_host writes it by DMA directly.
template <class T>
class HostTable {
public:
    HostTable() {}
    HostTable(const HostTable&) = delete;
    HostTable& operator=(const HostTable&) = delete;
    ~HostTable() { gmm_host_free(p_); }
    bool allocate(size_t n, T fill) {
        gmm_host_free(p_);
        p_ = nullptr;
        void* q = nullptr;
        if (gmm_host_alloc(n * sizeof(T), &q) != GMM_OK)
            return false;
        p_ = static_cast<T*>(q);
        for (size_t i = 0; i < n; ++i)
            p_[i] = fill;
        return true;
    }
    T*       data() const { return p_; }
    T&       operator[](size_t i) const { return p_[i]; }

private:
    T* p_ = nullptr;
};

// ---------------------------------------------------------------------------
// MixtureSet: the tables of Mm::MixtureSet the scorers read (src/Mm/MixtureSet.hh:140-212)
// ---------------------------------------------------------------------------
class MixtureSet {
public:
    explicit MixtureSet(uint32_t dimension) : dimension_(dimension) {}

    uint32_t dimension() const { return dimension_; }
    uint32_t nMixtures() const { return static_cast<uint32_t>(mixtureOffsets_.size() - 1); }
    uint32_t nDensities() const { return static_cast<uint32_t>(densityMean_.size()); }

    uint32_t addMean(const std::vector<float>& mean);                 // MixtureSet::addMean
    uint32_t addCovariance(const std::vector<float>& diagonal);       // addCovariance(new DiagonalCovariance)
    uint32_t addDensity(uint32_t meanIndex, uint32_t covarianceIndex); // addDensity(new GaussDensity(m, c))
    // Mixture with its densities and log-weights (Mixture::addLogDensity, src/Mm/Mixture.hh:41)
    uint32_t addMixture(const std::vector<uint32_t>& densities, const std::vector<double>& logWeights);

    // descriptor of the C-ABI (valid while this object is alive and unchanged)
    gmm_mixture_set descriptor() const;

    // Module_::readMixtureSet (src/Mm/Module.cc:152-182) via gmm_mixture_set_read (include/rasr_gmm_io.h):
    // the text format for ".pms" / ".gz" names, a binary maximum-likelihood estimator file (estimated with the
    // default parameters) for any other name; nullptr and *error on failure
    static std::unique_ptr<MixtureSet> read(const std::string& filename, std::string* error,
                                            uint32_t dimensionOffset = 0, uint32_t reducedDimension = 0);

private:
    uint32_t              dimension_;
    std::vector<float>    means_, variances_;
    std::vector<uint32_t> densityMean_, densityCovariance_;
    std::vector<uint32_t> mixtureOffsets_{0}, mixtureDensities_;
    std::vector<double>   mixtureLogWeights_;
};

// ---------------------------------------------------------------------------
// ContextScorer: scores of one feature vector (FeatureScorer.hh:33-45, AssigningFeatureScorer.hh:36-48)
// ---------------------------------------------------------------------------
class ContextScorer {
public:
    virtual ~ContextScorer() {}
    virtual EmissionIndex    nEmissions() const                 = 0;
    virtual Score            score(EmissionIndex e) const       = 0;
    virtual bool             hasBestDensity() const             { return false; }
    virtual DensityInMixture bestDensity(EmissionIndex e) const { (void)e; return 0xffffffffu; }
};
typedef std::shared_ptr<const ContextScorer> Scorer;   // Core::Ref<const ContextScorer>

struct Configuration {
    std::string type               = "SIMD-diagonal-maximum";  // feature-scorer-type (src/Mm/Module.cc:78-80)
    // "buffer-size" (the reference's batch scorers default to 4, BatchFeatureScorer.cc:28-29): 512, the knee of the
    // measured drop-in throughput (bench.py drop_in_protocol: 64 -> 512 frames +12 %, 512 -> 32768 +1 %; below 64
    // each launch's ~170 us round trip dominates).  Online decoding that needs scores within a few frames sets 1..4.
    uint32_t    bufferSize         = 512;
    float       mixtureWeightScale = 1.0f;  // "mixture-weight-scale" (GDMFS.cc:38-40)
    float       gaussianScale      = 1.0f;  // "gaussian-scale" (GDMFS.cc:42-44)
    float       scale              = 1.0f;  // FeatureScorerScaling scale (ScaledFeatureScorer.hh:62-64)
    int         device             = 0;
    // more than one: the density-sharded scorer over these devices (gmm_scorer_create_sharded, exchange
    // GMM_EXCHANGE_AUTO: RCCL for distinct devices); device is then ignored
    std::vector<int> shardDevices;
    // "density-clustering" of the preselection scorers (DensityClustering.cc:19-32)
    uint32_t clusters             = 256;
    uint32_t selectClusters       = 32;
    uint32_t clusteringIterations = 5;
    float    backoffScore         = 40000.0f;
    // "cache-archive" of "density-clustering" (DensityClustering.cc:27-28), resolved to its file (the archive's
    // "file" / "read-only", Core/Application.cc:42-43): the clustering is read from / written to its item
    // "density-clustering"; empty: always built
    std::string cacheArchive;
    bool        cacheArchiveReadOnly = false;
};

// ---------------------------------------------------------------------------
// FeatureScorer (src/Mm/FeatureScorer.hh:28-164)
// ---------------------------------------------------------------------------
class FeatureScorer {
public:
    virtual ~FeatureScorer();

    EmissionIndex nMixtures() const { return nMixtures_; }
    uint32_t      dimension() const { return dimension_; }

    virtual Scorer getScorer(const FeatureVector& f) const = 0;
    virtual void   reset() const {}
    virtual void   finalize() const {}
    virtual bool   isBuffered() const { return false; }
    virtual void   addFeature(const FeatureVector& f) const { (void)f; }
    virtual Scorer flush() const { return Scorer(); }
    virtual bool   bufferFilled() const { return true; }
    virtual bool   bufferEmpty() const { return true; }
    virtual uint32_t bufferSize() const { return 0; }

    // SimdGaussDiagonalMaximumFeatureScorer::inverseQuantizationFactor (SimdFeatureScorer.hh:128-130)
    float inverseQuantizationFactor() const;
    // preselection types: where the density clustering came from (GMM_CLUSTERING_*, gmm_scorer_clustering_source);
    // -1 for the other types
    int densityClusteringSource() const;
    // SimdGaussDiagonalMaximumFeatureScorer::multiplyAndQuantize (SimdFeatureScorer.cc:37-52)
    std::vector<std::vector<uint8_t>> multiplyAndQuantize(const FeatureVector& f) const;

    gmm_scorer* handle() const { return handle_; }

protected:
    FeatureScorer() {}
    bool init(const MixtureSet& ms, const Configuration& c, uint32_t maxFrames, std::string* error);

    gmm_scorer*   handle_    = nullptr;
    EmissionIndex nMixtures_ = 0;
    uint32_t      dimension_ = 0;
    bool          assigning_ = false;  // scorer type reports best densities
    Configuration config_;
};

// Unbuffered scorer: every getScorer() scores one frame against all mixtures on the GPU
// (the SIMD / diagonal-maximum scorers' Context, SimdFeatureScorer.cc:22-35).  The contexts' tables are
// page-locked slots recycled when the caller drops a context (no allocation per frame).  Best densities:
// until the first bestDensity() the calls compute scores only (GMM_HOST_LAZY_BEST), and a context's
// bestDensity(e) is answered for that one emission (gmm_best_density_pairs, from the frame still on the device;
// past kSparseMax emissions of a context its whole table, gmm_fetch_best_density), or -- after a later frame
// replaced it there -- by scoring that frame again.  From the first bestDensity() on (an aligner) every call
// computes the best densities with the scores, in the same launch.  Contexts refer to their scorer, which must
// outlive them (as the reference's Context refers to its featureScorer_, SimdFeatureScorer.hh:51-68).
class GpuFeatureScorer : public FeatureScorer {
public:
    static std::unique_ptr<GpuFeatureScorer> create(const MixtureSet& ms, const Configuration& c,
                                                     std::string* error = nullptr);
    ~GpuFeatureScorer() override;
    Scorer getScorer(const FeatureVector& f) const override;

    struct Slot;     // a context's page-locked tables and frame
    struct SlotPool; // the free slots (shared with the contexts that return them)

    // host calls so far (tests: bestDensity() of the newest context copies, an older one re-scores)
    uint32_t nLaunches() const { return launches_; }
    uint32_t nBestFetches() const { return bestFetches_; }
    uint32_t nBestPairs() const { return bestPairs_; }  // bestDensity(e) answered by gmm_best_density_pairs
    // bestDensity of a context whose slot is `slot` (ContextScorer side)
    DensityInMixture slotBestDensity(Slot& slot, EmissionIndex e) const;

    // emissions of one score-only call answered one by one before its whole table is computed
    static constexpr uint32_t kSparseMax = 32;

private:
    GpuFeatureScorer() {}
    std::shared_ptr<SlotPool> pool_;
    mutable bool              bestEager_ = false;  // a bestDensity() was asked: calls compute best densities too
    mutable uint32_t          launches_ = 0, bestFetches_ = 0, bestPairs_ = 0;
};

// Buffered scorer: the BatchFeatureScorerBase ring-buffer protocol (BatchFeatureScorer.cc:40-116).
// When a score of a buffered position is requested and not cached, ALL mixtures of all buffered
// frames are scored in one GPU launch (the reference fills one mixture at a time).
class GpuBatchFeatureScorer : public FeatureScorer {
public:
    static std::unique_ptr<GpuBatchFeatureScorer> create(const MixtureSet& ms, const Configuration& c,
                                                          std::string* error = nullptr);
    ~GpuBatchFeatureScorer() override;
    Scorer   getScorer(const FeatureVector& f) const override;
    void     reset() const override;
    bool     isBuffered() const override { return true; }
    void     addFeature(const FeatureVector& f) const override;
    Scorer   flush() const override;
    bool     bufferFilled() const override { return buffered_ >= static_cast<int32_t>(bufferSize_) - 1; }
    bool     bufferEmpty() const override { return buffered_ <= 0; }
    uint32_t bufferSize() const override { return bufferSize_; }

    Score            getScore(EmissionIndex e, uint32_t featureIndex, uint32_t length) const;
    // the scores of every emission of the buffered position featureIndex (filled first if needed): nMixtures()
    // floats of the page-locked frame-major table, valid until the protocol reuses the position
    const float*     scoreRow(uint32_t featureIndex, uint32_t length) const;
    // changes whenever the position of featureIndex takes a new frame (or the ring is reset): a context that keeps
    // a scoreRow() pointer re-reads through scoreRow() once the generation moved, so it never reads a row that an
    // asynchronous call is still writing
    uint32_t         positionGeneration(uint32_t featureIndex) const { return generation_[featureIndex % bufferSize_]; }
    // 0xffffffff for the batch types, which have no assignment (as ContextScorer::bestDensity)
    DensityInMixture getBestDensity(EmissionIndex e, uint32_t featureIndex, uint32_t length) const;
    // the single-pair answer of (position, e) for the position's current frame, if one was given
    bool             sparseAnswer(uint32_t featureIndex, EmissionIndex e, DensityInMixture* v) const;
    // the best densities of every emission of the position (filled first if needed, with best densities), or NULL
    // while they are not in the table (a score-only call's position: getBestDensity answers); valid as scoreRow()
    const DensityInMixture* bestRow(uint32_t featureIndex, uint32_t length) const;

    // number of GPU launches so far (tests check that one launch serves a whole buffer, wrapped or not)
    uint32_t nLaunches() const { return launches_; }
    uint32_t nBestFetches() const { return bestFetches_; }
    uint32_t nBestPairs() const { return bestPairs_; }  // bestDensity(e) answered by gmm_best_density_pairs

    // (position, emission) pairs of one score-only call answered one by one before its whole table is computed
    static constexpr uint32_t kSparseMax = 32;

private:
    GpuBatchFeatureScorer() {}
    void     setFeature(size_t pos, const FeatureVector& f) const;
    // withBest: the call computes the best densities too (bestEager_), else scores only (GMM_HOST_LAZY_BEST)
    void     fill(uint32_t featureIndex, uint32_t length, bool withBest) const;
    void     submitPending() const;   // the pending run as a GMM_HOST_ASYNC call
    void     landInflight() const;    // wait for the asynchronous call; its positions become cached
    uint32_t rowStride() const { return nMixtures_ ? nMixtures_ : 1; }

    uint32_t bufferSize_ = 4;
    // [bufferSize][dimension] ring, row = buffer position (BatchFeatureScorerBase::features_), and the
    // score / best tables, all page-locked: a fill is ONE gmm_score_host_ring call over the buffered
    // positions, wrapped or not, whose frames and score rows move by DMA directly.  The tables are
    // frame-major, [bufferSize][nMixtures] (the reference's scores_ is [nMixtures][bufferSize],
    // BatchFeatureScorer.hh:177-186, filled one mixture at a time): a context's score(e) calls walk one
    // contiguous row instead of one cache line per emission.  Best densities (assigning types): until the
    // first bestDensity() the calls compute scores only (GMM_HOST_LAZY_BEST) -- a score-only caller (the
    // search) runs the score-only kernels and moves 4 B per (frame, mixture), not 8 -- and the positions of
    // such a call answer bestDensity(e) one pair at a time (gmm_best_density_pairs) up to kSparseMax pairs,
    // then from the call's whole table (gmm_fetch_best_density).  From the first bestDensity() on (an
    // aligner, a dump) every call, prefetches included, writes the best table with the scores (bestEager_).
    HostTable<float>          features_;
    HostTable<float>          scores_;
    HostTable<uint32_t>       best_;
    mutable std::vector<char> cached_;       // [bufferSize] scores of the position are in scores_
    mutable std::vector<uint32_t> generation_; // [bufferSize] frames the position has taken (positionGeneration)
    mutable std::vector<char> bestCached_;   // [bufferSize] best densities of the position are in best_
    mutable std::vector<uint64_t> bestCall_; // [bufferSize] host call that scored the position
    // Prefetch (buffers of kPrefetchMin frames and more): the newest frames not yet scored (pending: the ring run
    // [pendingFirst_, pendingFirst_ + pendingCount_)) go to the GPU as one GMM_HOST_ASYNC call once they number
    // prefetchChunk_ (half the ring), so the GPU scores them while the caller still consumes older positions; a position whose
    // score is asked for while its call is in flight waits for it (inflight_).
    static constexpr uint32_t kPrefetchMin = 64;
    uint32_t                  prefetchChunk_ = 0;  // 0: no prefetch
    mutable std::vector<char> inflight_;           // [bufferSize] scored by asyncCall_, not landed yet
    mutable uint64_t          asyncCall_    = 0;
    mutable uint32_t          pendingFirst_ = 0, pendingCount_ = 0;
    mutable bool              bestEager_    = false;  // a bestDensity() was asked: calls compute best densities
    mutable bool              asyncEager_   = false;  // the call in flight does
    // the score-only call whose pairs were answered one by one, how many, and the answers (key position << 32 | e)
    mutable uint64_t          sparseCall_ = 0;
    mutable uint32_t          sparseAsked_ = 0;
    // answers of single (position, e) pairs, with the position's generation: once answered, a pair keeps its
    // answer for that frame (CachedAssigningContextScorer memoizes, AssigningFeatureScorer.hh:110-121), even after
    // the position's whole table was fetched in the keyed scorer's arithmetic
    mutable std::unordered_map<uint64_t, std::pair<uint32_t, DensityInMixture>> sparse_;
    mutable std::vector<uint16_t> sparsePos_;  // [bufferSize] entries of sparse_ per position (0: no lookup)
    mutable int32_t           currentFeature_ = 0;
    mutable int32_t           buffered_       = 0;
    mutable uint32_t          launches_       = 0, bestFetches_ = 0, bestPairs_ = 0;
};

// Factory by reference type name ("SIMD-diagonal-maximum", "diagonal-maximum",
// "batch-diagonal-maximum-int", "batch-diagonal-maximum-float", "batch-diagonal-maximum-fast"):
// batch-* types (and bufferSize > 1) give the buffered scorer.
std::unique_ptr<FeatureScorer> createFeatureScorer(const MixtureSet& ms, const Configuration& c,
                                                   std::string* error = nullptr);

}  // namespace Gpu
}  // namespace Mm
