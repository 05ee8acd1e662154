// GpuFeatureScorer.cc -- see GpuFeatureScorer.hh.
#include "GpuFeatureScorer.hh"

#include <algorithm>
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace Mm {
namespace Gpu {

namespace {
void abortHandler(const std::string& message) {
    std::fprintf(stderr, "criticalError: GPU feature scorer: %s\n", message.c_str());
    std::fflush(stderr);
    std::abort();
}
CriticalErrorHandler gCriticalError = abortHandler;

[[noreturn]] void criticalError(const char* what) {
    gCriticalError(std::string(what) + ": " + gmm_last_error());
    std::abort();  // a handler that returns normally must not continue with missing scores
}
}  // namespace

CriticalErrorHandler setCriticalErrorHandler(CriticalErrorHandler handler) {
    CriticalErrorHandler prev = gCriticalError;
    gCriticalError            = handler ? handler : abortHandler;
    return prev;
}

// ---------------------------------------------------------------------------
// MixtureSet
// ---------------------------------------------------------------------------
uint32_t MixtureSet::addMean(const std::vector<float>& mean) {
    assert(mean.size() == dimension_);
    means_.insert(means_.end(), mean.begin(), mean.end());
    return static_cast<uint32_t>(means_.size() / dimension_ - 1);
}

uint32_t MixtureSet::addCovariance(const std::vector<float>& diagonal) {
    assert(diagonal.size() == dimension_);
    variances_.insert(variances_.end(), diagonal.begin(), diagonal.end());
    return static_cast<uint32_t>(variances_.size() / dimension_ - 1);
}

uint32_t MixtureSet::addDensity(uint32_t meanIndex, uint32_t covarianceIndex) {
    densityMean_.push_back(meanIndex);
    densityCovariance_.push_back(covarianceIndex);
    return static_cast<uint32_t>(densityMean_.size() - 1);
}

uint32_t MixtureSet::addMixture(const std::vector<uint32_t>& densities, const std::vector<double>& logWeights) {
    assert(densities.size() == logWeights.size());
    mixtureDensities_.insert(mixtureDensities_.end(), densities.begin(), densities.end());
    mixtureLogWeights_.insert(mixtureLogWeights_.end(), logWeights.begin(), logWeights.end());
    mixtureOffsets_.push_back(static_cast<uint32_t>(mixtureDensities_.size()));
    return nMixtures() - 1;
}

std::unique_ptr<MixtureSet> MixtureSet::read(const std::string& filename, std::string* error, uint32_t dimensionOffset,
                                             uint32_t reducedDimension) {
    gmm_mixture_set d;
    if (gmm_mixture_set_read(filename.c_str(), dimensionOffset, reducedDimension, &d) != GMM_OK) {
        if (error)
            *error = gmm_last_error();
        return nullptr;
    }
    std::unique_ptr<MixtureSet> ms(new MixtureSet(d.dimension));
    const size_t                D = d.dimension;
    ms->means_.assign(d.means, d.means + d.n_means * D);
    ms->variances_.assign(d.variances, d.variances + d.n_covariances * D);
    ms->densityMean_.assign(d.density_mean, d.density_mean + d.n_densities);
    ms->densityCovariance_.assign(d.density_covariance, d.density_covariance + d.n_densities);
    ms->mixtureOffsets_.assign(d.mixture_offsets, d.mixture_offsets + d.n_mixtures + 1);
    const uint32_t nEntries = d.mixture_offsets[d.n_mixtures];
    ms->mixtureDensities_.assign(d.mixture_densities, d.mixture_densities + nEntries);
    ms->mixtureLogWeights_.assign(d.mixture_log_weights, d.mixture_log_weights + nEntries);
    gmm_mixture_set_free(&d);
    return ms;
}

gmm_mixture_set MixtureSet::descriptor() const {
    gmm_mixture_set d;
    std::memset(&d, 0, sizeof(d));
    d.dimension           = dimension_;
    d.n_means             = dimension_ ? static_cast<uint32_t>(means_.size() / dimension_) : 0;
    d.means               = means_.data();
    d.n_covariances       = dimension_ ? static_cast<uint32_t>(variances_.size() / dimension_) : 0;
    d.variances           = variances_.data();
    d.n_densities         = nDensities();
    d.density_mean        = densityMean_.data();
    d.density_covariance  = densityCovariance_.data();
    d.n_mixtures          = nMixtures();
    d.mixture_offsets     = mixtureOffsets_.data();
    d.mixture_densities   = mixtureDensities_.data();
    d.mixture_log_weights = mixtureLogWeights_.data();
    return d;
}

// ---------------------------------------------------------------------------
// FeatureScorer
// ---------------------------------------------------------------------------
static bool typeOf(const std::string& name, gmm_scorer_type* t, bool* assigning, bool* batch) {
    struct {
        const char*     name;
        gmm_scorer_type type;
        bool            assigning, batch;
    } const table[] = {
            {"SIMD-diagonal-maximum", GMM_SIMD_DIAGONAL_MAXIMUM, true, false},
            {"diagonal-maximum", GMM_DIAGONAL_MAXIMUM, true, false},
            {"diagonal-sum", GMM_DIAGONAL_SUM, true, false},
            {"batch-diagonal-maximum-int", GMM_BATCH_DIAGONAL_MAXIMUM_INT, false, true},
            {"batch-diagonal-maximum-fast", GMM_BATCH_DIAGONAL_MAXIMUM_FAST, false, true},
            {"batch-diagonal-maximum-float", GMM_BATCH_DIAGONAL_MAXIMUM_FLOAT, false, true},
            {"preselection-batch-float", GMM_BATCH_PRESELECTION_FLOAT, false, true},
            {"preselection-batch-int", GMM_BATCH_PRESELECTION_INT, false, true},
    };
    for (const auto& e : table)
        if (name == e.name) {
            *t         = e.type;
            *assigning = e.assigning;
            *batch     = e.batch;
            return true;
        }
    return false;
}

FeatureScorer::~FeatureScorer() {
    gmm_scorer_destroy(handle_);
}

bool FeatureScorer::init(const MixtureSet& ms, const Configuration& c, uint32_t maxFrames, std::string* error) {
    gmm_scorer_type t;
    bool            batch = false;
    if (!typeOf(c.type, &t, &assigning_, &batch)) {
        if (error)
            *error = "unknown feature scorer type: " + c.type;
        return false;
    }
    config_ = c;
    gmm_scorer_config cfg;
    gmm_default_config(&cfg);
    cfg.mixture_weight_scale = c.mixtureWeightScale;
    cfg.gaussian_scale       = c.gaussianScale;
    cfg.score_scale          = c.scale;
    cfg.max_frames           = maxFrames;
    cfg.clusters              = c.clusters;
    cfg.select_clusters       = c.selectClusters;
    cfg.clustering_iterations = c.clusteringIterations;
    cfg.backoff_score         = c.backoffScore;
    cfg.cache_archive         = c.cacheArchive.empty() ? nullptr : c.cacheArchive.c_str();
    if (c.cacheArchiveReadOnly)
        cfg.flags |= GMM_FLAG_CACHE_ARCHIVE_READ_ONLY;
    const gmm_mixture_set d  = ms.descriptor();
    const int rc = c.shardDevices.size() > 1
                           ? gmm_scorer_create_sharded(&d, t, &cfg, c.shardDevices.data(),
                                                       static_cast<uint32_t>(c.shardDevices.size()), GMM_EXCHANGE_AUTO,
                                                       &handle_)
                           : gmm_scorer_create(&d, t, &cfg, c.device, &handle_);
    if (rc != GMM_OK) {
        if (error)
            *error = gmm_last_error();
        handle_ = nullptr;
        return false;
    }
    nMixtures_ = gmm_scorer_n_mixtures(handle_);
    dimension_ = gmm_scorer_dimension(handle_);
    return true;
}

int FeatureScorer::densityClusteringSource() const {
    int source = -1;
    return gmm_scorer_clustering_source(handle_, &source) == GMM_OK ? source : -1;
}

float FeatureScorer::inverseQuantizationFactor() const {
    float s = 0, q = 0;
    gmm_scorer_quantization(handle_, &s, &q);
    return q;
}

std::vector<std::vector<uint8_t>> FeatureScorer::multiplyAndQuantize(const FeatureVector& f) const {
    assert(f.size() == dimension_);
    const uint32_t                    dp = (dimension_ + 15) / 16 * 16;
    const uint32_t                    nc = gmm_scorer_n_covariances(handle_);
    std::vector<uint8_t>              buf(static_cast<size_t>(dp) * nc);
    std::vector<std::vector<uint8_t>> out;
    if (gmm_scorer_multiply_and_quantize(handle_, f.data(), buf.data()) != GMM_OK)
        return out;
    for (uint32_t c = 0; c < nc; ++c)
        out.emplace_back(buf.begin() + static_cast<size_t>(c) * dp, buf.begin() + static_cast<size_t>(c + 1) * dp);
    return out;
}

// ---------------------------------------------------------------------------
// ContextScorers
// ---------------------------------------------------------------------------
namespace {

// one frame, all mixtures (SimdGaussDiagonalMaximumFeatureScorer::Context): a recycled page-locked slot
class FrameScorer : public ContextScorer {
public:
    FrameScorer(const GpuFeatureScorer* parent, std::unique_ptr<GpuFeatureScorer::Slot> slot,
                std::shared_ptr<GpuFeatureScorer::SlotPool> pool, EmissionIndex n, bool assigning)
            : parent_(parent), slot_(std::move(slot)), pool_(std::move(pool)), n_(n), assigning_(assigning) {}
    ~FrameScorer() override;
    EmissionIndex nEmissions() const override { return n_; }
    Score         score(EmissionIndex e) const override;
    bool             hasBestDensity() const override { return assigning_; }
    DensityInMixture bestDensity(EmissionIndex e) const override {
        assert(e < n_);
        return assigning_ ? parent_->slotBestDensity(*slot_, e) : 0xffffffffu;
    }

private:
    const GpuFeatureScorer*                     parent_;
    std::unique_ptr<GpuFeatureScorer::Slot>     slot_;
    std::shared_ptr<GpuFeatureScorer::SlotPool> pool_;
    EmissionIndex                               n_;
    bool                                        assigning_;
};

// BatchFeatureScorerBase::ContextScorer (BatchFeatureScorer.hh:42-60)
class BufferedScorer : public ContextScorer {
public:
    BufferedScorer(const GpuBatchFeatureScorer* parent, uint32_t currentFeature, uint32_t buffered, bool assigning)
            : parent_(parent), currentFeature_(currentFeature), buffered_(buffered), assigning_(assigning) {}
    EmissionIndex nEmissions() const override { return parent_->nMixtures(); }
    // the first score(e) fills the position if needed and keeps its row of the frame-major table.  A later
    // getScorer() may reuse the position for a new frame (and a prefetch may then be writing that row): the
    // generation check sends such a context back through scoreRow(), which lands the call in flight first --
    // the reference's getScore() likewise answers from the position's current fill
    Score score(EmissionIndex e) const override {
        const uint32_t g = parent_->positionGeneration(currentFeature_);
        if (!row_ || g != gen_) {
            row_ = parent_->scoreRow(currentFeature_, buffered_);
            gen_ = g;
        }
        return row_[e];
    }
    bool             hasBestDensity() const override { return assigning_; }
    // the position's best-density row once its call carried one (the same generation check as score(e)); a
    // position of a score-only call answers through getBestDensity (one pair, or the call's whole table)
    DensityInMixture bestDensity(EmissionIndex e) const override {
        DensityInMixture v;
        if (parent_->sparseAnswer(currentFeature_, e, &v))  // answered alone before: that answer (memoized)
            return v;
        const uint32_t g = parent_->positionGeneration(currentFeature_);
        if (!bestRow_ || g != bestGen_) {
            bestRow_ = parent_->bestRow(currentFeature_, buffered_);
            bestGen_ = g;
        }
        return bestRow_ ? bestRow_[e] : parent_->getBestDensity(e, currentFeature_, buffered_);
    }

private:
    const GpuBatchFeatureScorer*    parent_;
    uint32_t                        currentFeature_, buffered_;
    bool                            assigning_;
    mutable const float*            row_ = nullptr;
    mutable uint32_t                gen_ = 0;
    mutable const DensityInMixture* bestRow_ = nullptr;
    mutable uint32_t                bestGen_ = 0;
};

}  // namespace

// ---------------------------------------------------------------------------
// GpuFeatureScorer
// ---------------------------------------------------------------------------
struct GpuFeatureScorer::Slot {
    HostTable<float>    scores;  // [nMixtures]
    HostTable<uint32_t> best;    // [nMixtures]
    HostTable<float>    frame;   // [dimension] the frame (page-locked: the library's small-call path reads it
                                 // on the device), kept for scoring it again
    std::vector<float>  scratch; // scores of that second scoring (the context keeps its first ones)
    uint64_t            call = 0;
    bool                bestValid = false;
    // bestDensity(e) of a score-only call answered one emission at a time (gmm_best_density_pairs)
    std::vector<std::pair<EmissionIndex, DensityInMixture>> sparse;
};

struct GpuFeatureScorer::SlotPool {
    std::vector<std::unique_ptr<Slot>> free;
};

FrameScorer::~FrameScorer() {
    pool_->free.push_back(std::move(slot_));
}

Score FrameScorer::score(EmissionIndex e) const {
    assert(e < n_);
    return slot_->scores[e];
}

std::unique_ptr<GpuFeatureScorer> GpuFeatureScorer::create(const MixtureSet& ms, const Configuration& c,
                                                           std::string* error) {
    std::unique_ptr<GpuFeatureScorer> s(new GpuFeatureScorer());
    if (!s->init(ms, c, 1, error))
        return nullptr;
    s->pool_ = std::make_shared<SlotPool>();
    return s;
}

GpuFeatureScorer::~GpuFeatureScorer() {}

Scorer GpuFeatureScorer::getScorer(const FeatureVector& f) const {
    assert(f.size() == dimension_);  // require(featureVector.size() == dimension()), SimdFeatureScorer.cc:26
    std::unique_ptr<Slot> slot;
    if (!pool_->free.empty()) {
        slot = std::move(pool_->free.back());
        pool_->free.pop_back();
    }
    else {
        slot.reset(new Slot());
        const size_t n = std::max<uint32_t>(nMixtures_, 1);
        if (!slot->scores.allocate(n, 0.0f) || (assigning_ && !slot->best.allocate(n, 0xffffffffu)) ||
            !slot->frame.allocate(std::max<uint32_t>(dimension_, 1), 0.0f))
            criticalError("gmm_host_alloc");
    }
    std::copy(f.begin(), f.end(), slot->frame.data());
    ++launches_;
    // an aligner (bestDensity() was asked before): the best densities come with the scores, in the same launch
    const bool eager = assigning_ && bestEager_;
    if (gmm_score_host_ring(handle_, slot->frame.data(), 1, 0, 1, dimension_, slot->scores.data(),
                            eager ? slot->best.data() : nullptr, 1, (assigning_ && !eager) ? GMM_HOST_LAZY_BEST : 0u,
                            &slot->call) != GMM_OK)
        criticalError("gmm_score_host_ring");
    slot->bestValid = eager;
    slot->sparse.clear();
    return std::make_shared<FrameScorer>(this, std::move(slot), pool_, nMixtures_, assigning_);
}

DensityInMixture GpuFeatureScorer::slotBestDensity(Slot& slot, EmissionIndex e) const {
    bestEager_ = true;  // from the next getScorer() on, the calls compute best densities too
    // an emission answered alone keeps that answer for this frame, also after the whole table was fetched
    // (the reference memoizes per (frame, emission), AssigningFeatureScorer.hh:110-121)
    for (const auto& kv : slot.sparse)
        if (kv.first == e)
            return kv.second;
    if (!slot.bestValid) {
        // the asked emission alone, while the frame is still on the device (its call is the newest)
        uint32_t pos = 0, v = 0;
        if (slot.sparse.size() < kSparseMax && gmm_best_density_pairs(handle_, slot.call, &pos, &e, 1, &v) == GMM_OK) {
            ++bestPairs_;
            slot.sparse.emplace_back(e, v);
            return v;
        }
        // computed from the frame the device still holds if no later frame was scored; otherwise score this
        // frame again, its best densities copied directly (its scores into scratch: the float types' keyed
        // scores carry fewer bits, and the context's scores stay the ones it already returned)
        if (gmm_fetch_best_density(handle_, slot.call, slot.best.data(), 1) == GMM_OK)
            ++bestFetches_;
        else {
            ++launches_;
            slot.scratch.resize(std::max<uint32_t>(nMixtures_, 1));
            if (gmm_score_host(handle_, slot.frame.data(), 1, dimension_, slot.scratch.data(), slot.best.data(), 1) != GMM_OK)
                criticalError("gmm_score_host");
        }
        slot.bestValid = true;
    }
    return slot.best[e];
}

// ---------------------------------------------------------------------------
// GpuBatchFeatureScorer
// ---------------------------------------------------------------------------
std::unique_ptr<GpuBatchFeatureScorer> GpuBatchFeatureScorer::create(const MixtureSet& ms, const Configuration& c,
                                                                     std::string* error) {
    std::unique_ptr<GpuBatchFeatureScorer> s(new GpuBatchFeatureScorer());
    const uint32_t                         b = c.bufferSize ? c.bufferSize : 1;
    if (!s->init(ms, c, b, error))
        return nullptr;
    s->bufferSize_ = b;
    const size_t n = std::max<size_t>(1, static_cast<size_t>(s->nMixtures_) * b);
    if (!s->features_.allocate(static_cast<size_t>(b) * std::max<uint32_t>(s->dimension_, 1), 0.0f) ||
        !s->scores_.allocate(n, 0.0f) || (s->assigning_ && !s->best_.allocate(n, 0xffffffffu))) {
        if (error)
            *error = gmm_last_error();
        return nullptr;
    }
    s->cached_.assign(b, 0);
    s->generation_.assign(b, 0);
    s->sparsePos_.assign(b, 0);
    s->bestCached_.assign(b, 0);
    s->bestCall_.assign(b, 0);
    s->inflight_.assign(b, 0);
    s->prefetchChunk_ = b >= kPrefetchMin ? b / 2 : 0;
    return s;
}

GpuBatchFeatureScorer::~GpuBatchFeatureScorer() {
    if (asyncCall_)  // no DMA into the tables after they are freed
        (void)gmm_host_call_wait(handle_, asyncCall_);
}

// BatchFeatureScorerBase::reset, BatchFeatureScorer.cc:40-44
void GpuBatchFeatureScorer::reset() const {
    if (asyncCall_)
        (void)gmm_host_call_wait(handle_, asyncCall_);
    asyncCall_ = 0;
    std::fill(inflight_.begin(), inflight_.end(), 0);
    std::fill(cached_.begin(), cached_.end(), 0);
    for (uint32_t& g : generation_)
        ++g;
    sparse_.clear();  // every position's frame is gone
    std::fill(sparsePos_.begin(), sparsePos_.end(), 0);
    pendingCount_   = 0;
    currentFeature_ = 0;
    buffered_       = 0;
}

void GpuBatchFeatureScorer::setFeature(size_t pos, const FeatureVector& f) const {
    assert(pos < bufferSize_ && f.size() == dimension_);
    if (inflight_[pos])  // its row may not have been read yet (a context whose scores were never asked for)
        landInflight();
    std::copy(f.begin(), f.end(), features_.data() + pos * dimension_);
    ++generation_[pos];
    // the position's single-pair answers belonged to its previous frame (once every position took a new frame
    // the map is empty and bestDensity() skips the lookup)
    if (sparsePos_[pos]) {
        for (auto i = sparse_.begin(); i != sparse_.end();)
            i = (i->first >> 32) == pos ? sparse_.erase(i) : std::next(i);
        sparsePos_[pos] = 0;
    }
    if (!prefetchChunk_)
        return;
    // the new frame joins the pending run (it is the newest buffered position)
    if (pendingCount_ == 0)
        pendingFirst_ = static_cast<uint32_t>(pos);
    if ((pendingFirst_ + pendingCount_) % bufferSize_ != pos || pendingCount_ >= bufferSize_) {
        pendingCount_ = 0;  // not contiguous with the run (cannot happen in the protocol's order): start over
        pendingFirst_ = static_cast<uint32_t>(pos);
    }
    ++pendingCount_;
    if (pendingCount_ >= prefetchChunk_)
        submitPending();
}

void GpuBatchFeatureScorer::landInflight() const {
    if (!asyncCall_)
        return;
    if (gmm_host_call_wait(handle_, asyncCall_) != GMM_OK)
        criticalError("gmm_host_call_wait");
    for (uint32_t q = 0; q < bufferSize_; ++q)
        if (inflight_[q]) {
            inflight_[q]   = 0;
            cached_[q]     = 1;
            bestCached_[q] = asyncEager_ ? 1 : 0;
            bestCall_[q]   = asyncCall_;
        }
    asyncCall_ = 0;
}

void GpuBatchFeatureScorer::submitPending() const {
    landInflight();  // one call in flight at a time (the library's staging)
    uint64_t   call  = 0;
    const bool eager = assigning_ && bestEager_;
    ++launches_;
    if (gmm_score_host_ring(handle_, features_.data(), bufferSize_, pendingFirst_, pendingCount_, dimension_, scores_.data(),
                            eager ? best_.data() : nullptr, rowStride(),
                            GMM_HOST_FRAME_MAJOR | GMM_HOST_ASYNC | ((assigning_ && !eager) ? GMM_HOST_LAZY_BEST : 0u),
                            &call) != GMM_OK)
        criticalError("gmm_score_host_ring");
    asyncEager_ = eager;
    for (uint32_t i = 0; i < pendingCount_; ++i) {
        const uint32_t q = (pendingFirst_ + i) % bufferSize_;
        inflight_[q]     = 1;
        cached_[q]       = 0;
    }
    asyncCall_    = call;
    pendingFirst_ = (pendingFirst_ + pendingCount_) % bufferSize_;
    pendingCount_ = 0;
}

// BatchFeatureScorerBase::addFeature, BatchFeatureScorer.cc:46-50
void GpuBatchFeatureScorer::addFeature(const FeatureVector& f) const {
    assert(!bufferFilled());
    setFeature(static_cast<size_t>(buffered_), f);
    cached_[static_cast<size_t>(buffered_)] = 0;
    ++buffered_;
}

// BatchFeatureScorerBase::getScorer, BatchFeatureScorer.cc:77-87
Scorer GpuBatchFeatureScorer::getScorer(const FeatureVector& f) const {
    assert(bufferFilled());
    const int32_t b        = static_cast<int32_t>(bufferSize_);
    const int32_t posToAdd = currentFeature_ ? (currentFeature_ - 1) % b : b - 1;
    setFeature(static_cast<size_t>(posToAdd), f);
    ++buffered_;
    cached_[static_cast<size_t>(posToAdd)] = 0;  // invalidateCache(posToAdd)
    Scorer result = std::make_shared<BufferedScorer>(this, currentFeature_, buffered_, assigning_);
    currentFeature_ = (currentFeature_ + 1) % b;
    --buffered_;
    return result;
}

// BatchFeatureScorerBase::flush, BatchFeatureScorer.cc:89-96
Scorer GpuBatchFeatureScorer::flush() const {
    assert(buffered_ > 0 && !bufferEmpty());
    Scorer result   = std::make_shared<BufferedScorer>(this, currentFeature_, buffered_, assigning_);
    currentFeature_ = (currentFeature_ + 1) % static_cast<int32_t>(bufferSize_);
    --buffered_;
    return result;
}

// Score all mixtures of the buffered positions featureIndex .. featureIndex+length-1 (mod buffer)
// and cache them (the reference's fillScoreCache does one mixture at a time): one gmm_score_host_ring call
// reads those rows of features_ and writes their rows of the page-locked frame-major tables in place,
// wrapped or not.
void GpuBatchFeatureScorer::fill(uint32_t featureIndex, uint32_t length, bool withBest) const {
    const uint32_t b = bufferSize_;
    length           = std::min(length, b);
    const uint32_t p = featureIndex % b;
    uint64_t       call  = 0;
    const bool     eager = assigning_ && withBest;
    landInflight();
    pendingCount_ = 0;  // this fill covers every buffered position from p on
    ++launches_;
    if (gmm_score_host_ring(handle_, features_.data(), b, p, length, dimension_, scores_.data(),
                            eager ? best_.data() : nullptr, rowStride(),
                            GMM_HOST_FRAME_MAJOR | ((assigning_ && !eager) ? GMM_HOST_LAZY_BEST : 0u), &call) != GMM_OK)
        criticalError("gmm_score_host_ring");
    for (uint32_t i = 0; i < length; ++i) {
        const uint32_t q = (p + i) % b;
        cached_[q]       = 1;
        bestCached_[q]   = eager ? 1 : 0;
        bestCall_[q]     = call;
    }
}

// BatchFeatureScorerBase::getScore, BatchFeatureScorer.cc:98-105
Score GpuBatchFeatureScorer::getScore(EmissionIndex e, uint32_t featureIndex, uint32_t length) const {
    assert(e < nMixtures_);
    return scoreRow(featureIndex, length)[e];
}

const float* GpuBatchFeatureScorer::scoreRow(uint32_t featureIndex, uint32_t length) const {
    const uint32_t p = featureIndex % bufferSize_;
    if (!cached_[p] && inflight_[p])
        landInflight();
    if (!cached_[p])
        fill(featureIndex, length, bestEager_);
    return scores_.data() + static_cast<size_t>(p) * rowStride();
}

const DensityInMixture* GpuBatchFeatureScorer::bestRow(uint32_t featureIndex, uint32_t length) const {
    if (!assigning_)
        return nullptr;
    bestEager_       = true;
    const uint32_t p = featureIndex % bufferSize_;
    if (!cached_[p] && inflight_[p])
        landInflight();
    if (!cached_[p])
        fill(featureIndex, length, true);
    return bestCached_[p] ? best_.data() + static_cast<size_t>(p) * rowStride() : nullptr;
}

bool GpuBatchFeatureScorer::sparseAnswer(uint32_t featureIndex, EmissionIndex e, DensityInMixture* v) const {
    const uint32_t p = featureIndex % bufferSize_;
    if (!sparsePos_[p])  // (one test per call: a full dump asks every emission's best density)
        return false;
    const auto     it = sparse_.find((static_cast<uint64_t>(p) << 32) | e);
    if (it == sparse_.end() || it->second.first != generation_[p])
        return false;
    *v = it->second.second;
    return true;
}

DensityInMixture GpuBatchFeatureScorer::getBestDensity(EmissionIndex e, uint32_t featureIndex, uint32_t length) const {
    assert(e < nMixtures_);
    if (!assigning_)
        return 0xffffffffu;
    bestEager_       = true;  // an aligner: from now on every call computes the best densities with the scores
    const uint32_t p = featureIndex % bufferSize_;
    if (!cached_[p] && inflight_[p])
        landInflight();
    if (!cached_[p])
        fill(featureIndex, length, true);
    const size_t o = static_cast<size_t>(p) * rowStride() + e;
    // a pair answered alone for this frame keeps its answer (memoized as the reference's context scorer does)
    const uint64_t   key = (static_cast<uint64_t>(p) << 32) | e;
    DensityInMixture memo;
    if (sparseAnswer(featureIndex, e, &memo))
        return memo;
    if (bestCached_[p])
        return best_[o];
    // a position of a score-only call (made before the first bestDensity()): the asked pair alone while that
    // call's asked set is small and its frames are still on the device
    const uint64_t call = bestCall_[p];
    if (call != sparseCall_) {
        sparseCall_  = call;
        sparseAsked_ = 0;
    }
    if (sparseAsked_ < kSparseMax) {
        uint32_t pos = p, v = 0;
        if (gmm_best_density_pairs(handle_, call, &pos, &e, 1, &v) == GMM_OK) {
            ++sparseAsked_;
            ++bestPairs_;
            if (sparse_.insert_or_assign(key, std::make_pair(generation_[p], v)).second)
                ++sparsePos_[p];
            return v;
        }
    }
    // past kSparseMax pairs: the call's whole table, computed from its frames on the device (every position of the
    // call); if a later call replaced them (a prefetch before the first bestDensity()), the buffered positions from
    // p are scored again, scores only (the values the contexts already returned), and their table computed from it
    bool ok = gmm_fetch_best_density(handle_, call, best_.data(), rowStride()) == GMM_OK;
    if (!ok) {
        fill(featureIndex, length, false);
        ok = gmm_fetch_best_density(handle_, bestCall_[p], best_.data(), rowStride()) == GMM_OK;
    }
    if (!ok)  // (not reached with this library: the fill above is the newest call)
        criticalError("gmm_fetch_best_density");
    ++bestFetches_;
    const uint64_t filled = bestCall_[p];
    for (uint32_t q = 0; q < bufferSize_; ++q)
        if (cached_[q] && bestCall_[q] == filled)
            bestCached_[q] = 1;
    return best_[o];
}

// ---------------------------------------------------------------------------
std::unique_ptr<FeatureScorer> createFeatureScorer(const MixtureSet& ms, const Configuration& c, std::string* error) {
    gmm_scorer_type t;
    bool            assigning = false, batch = false;
    if (!typeOf(c.type, &t, &assigning, &batch)) {
        if (error)
            *error = "unknown feature scorer type: " + c.type;
        return nullptr;
    }
    if (batch || c.bufferSize > 1)
        return GpuBatchFeatureScorer::create(ms, c, error);
    return GpuFeatureScorer::create(ms, c, error);
}

}  // namespace Gpu
}  // namespace Mm
