// GpuFeatureScorer.cc -- see GpuFeatureScorer.hh.
#include "GpuFeatureScorer.hh"

#include <Core/Application.hh>
#include <Mm/FeatureScorerFactory.hh>
#include <Mm/MixtureSetLoader.hh>
#include <Mm/Module.hh>

#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

using namespace Mm;

const Core::ParameterInt GpuFeatureScorer::paramBufferSize(
        "buffer-size",
        "frames scored per GPU launch (1: every frame on its own, unbuffered); default 4 as the reference batch "
        "scorers (BatchFeatureScorer.cc:28-29); 512 is the measured throughput knee for offline recognition",
        4, 1);
const Core::ParameterInt GpuFeatureScorer::paramDevice(
        "device", "HIP device of this process (one process per GPU)", 0, 0);
const Core::ParameterIntVector GpuFeatureScorer::paramShardDevices(
        "density-shard-devices", "HIP devices the model's densities are split over (empty: the whole model on device)",
        ",", 0);
const Core::ParameterFloat GpuFeatureScorer::paramMixtureWeightScale(
        "mixture-weight-scale", "scaling of the mixture weights", 1.0);
const Core::ParameterFloat GpuFeatureScorer::paramGaussianScale(
        "gaussian-scale", "scaling of the Gaussian densities", 1.0);
const Core::ParameterInt GpuFeatureScorer::paramClusters(
        "clusters", "number of density clusters", 256, 1, 256);
const Core::ParameterInt GpuFeatureScorer::paramSelectClusters(
        "select-clusters", "number of clusters selected per frame", 32, 1);
const Core::ParameterInt GpuFeatureScorer::paramClusteringIterations(
        "iterations", "density clustering iterations", 5, 0);
const Core::ParameterFloat GpuFeatureScorer::paramBackoffScore(
        "backoff-score", "score of a mixture without a selected density", 40000.0);
const Core::ParameterString GpuFeatureScorer::paramCacheArchive(
        "cache-archive", "cache-archive where to cache the clustering of the density preselection", "global-cache");

namespace {

// Scoring errors of the library reach the component that owns the call (one recognizer thread owns a
// scorer, src/Core/ReferenceCounting.hh:43-77): Core::Component::criticalError, which aborts.
thread_local const Core::Component* tOwner = 0;

void routeCriticalError(const std::string& message) {
    if (tOwner)
        tOwner->criticalError("GPU feature scorer: %s", message.c_str());
    std::abort();
}

// the library's handler is process-global: installed once (first scorer constructed or registration),
// never rewritten per call by several recognizer threads
std::once_flag gHandlerOnce;
void installCriticalErrorHandler() {
    std::call_once(gHandlerOnce, [] { Gpu::setCriticalErrorHandler(routeCriticalError); });
}

// the owner of the calls in this thread (thread_local: no shared state between recognizer threads)
struct CallScope {
    explicit CallScope(const Core::Component* c)
            : prev_(tOwner) {
        tOwner = c;
    }
    ~CallScope() {
        tOwner = prev_;
    }
    const Core::Component* prev_;
};

// Mm::MixtureSet -> the C-ABI tables (the reference scorers read the same fields in init():
// SimdFeatureScorer.cc:64-104, GaussDiagonalMaximumFeatureScorer.cc:64-86, BatchFeatureScorer.cc:59-75)
Gpu::MixtureSet convertMixtureSet(const MixtureSet& ms) {
    Gpu::MixtureSet out(ms.dimension());
    for (MeanIndex i = 0; i < ms.nMeans(); ++i) {
        const Mean& m = *ms.mean(i);
        out.addMean(std::vector<f32>(m.begin(), m.end()));
    }
    for (CovarianceIndex i = 0; i < ms.nCovariances(); ++i) {
        const std::vector<VarianceType>& v = ms.covariance(i)->diagonal();
        out.addCovariance(std::vector<f32>(v.begin(), v.end()));
    }
    for (DensityIndex i = 0; i < ms.nDensities(); ++i)
        out.addDensity(ms.density(i)->meanIndex(), ms.density(i)->covarianceIndex());
    for (MixtureIndex m = 0; m < ms.nMixtures(); ++m) {
        const Mixture*        x = ms.mixture(m);
        std::vector<u32>      dens;
        std::vector<f64>      logw;
        for (DensityIndex j = 0; j < x->nDensities(); ++j) {
            dens.push_back(x->densityIndex(j));
            logw.push_back(x->logWeight(j));
        }
        out.addMixture(dens, logw);
    }
    return out;
}

}  // namespace

// The ContextScorer handed to the search and the aligners: an AssigningContextScorer over the buffered
// scorer's context (BatchFeatureScorer.hh:42-60 holds (parent, currentFeature, bufferedFeatures) the same way).
class GpuFeatureScorer::Context : public AssigningFeatureScorer::AssigningContextScorer {
public:
    Context(const GpuFeatureScorer* parent, const Gpu::Scorer& s)
            : parent_(parent), s_(s) {}
    virtual EmissionIndex nEmissions() const {
        return s_->nEmissions();
    }
    virtual Score score(EmissionIndex e) const {
        require_(e < nEmissions());
        CallScope scope(parent_);
        return s_->score(e);
    }
    virtual DensityInMixture bestDensity(EmissionIndex e) const {
        require_(e < nEmissions());
        if (!s_->hasBestDensity())
            parent_->criticalError("bestDensity() not available for this feature scorer type");
        CallScope scope(parent_);
        return s_->bestDensity(e);
    }
    virtual Score score(EmissionIndex, DensityIndex) const {
        parent_->criticalError("This feature scorer does not support the calculation of scores given a density in the mixture");
        return Core::Type<Score>::max;
    }
    virtual void getDensityPosteriorProbabilities(EmissionIndex, std::vector<Mm::Weight>&) const {
        parent_->criticalError("This feature scorer does not support the calculation of density posterior probabilities");
    }

private:
    const GpuFeatureScorer* parent_;
    Gpu::Scorer             s_;
};

GpuFeatureScorer::GpuFeatureScorer(const Core::Configuration& c, Core::Ref<const MixtureSet> mixtureSet,
                                   const char* scorerType)
        : Core::Component(c), Precursor(c) {
    installCriticalErrorHandler();
    Gpu::Configuration cfg;
    cfg.type               = scorerType;
    cfg.bufferSize         = paramBufferSize(c);
    cfg.device             = paramDevice(c);
    for (s32 d : paramShardDevices(c))
        cfg.shardDevices.push_back(d);
    cfg.mixtureWeightScale = paramMixtureWeightScale(c);
    cfg.gaussianScale      = paramGaussianScale(c);
    const Core::Configuration dc(c, "density-clustering");
    cfg.clusters             = paramClusters(dc);
    cfg.selectClusters       = paramSelectClusters(dc);
    cfg.clusteringIterations = paramClusteringIterations(dc);
    cfg.backoffScore         = paramBackoffScore(dc);
    // the named archive's file and read-only flag, as Core::Application::getCacheArchive resolves them
    // (Application.cc:397-400); the library opens the file itself (gmm_scorer_config.cache_archive)
    {
        static const Core::ParameterString paramFile("file", "cache archive file");  // Application.cc:42-43
        static const Core::ParameterBool   paramReadOnly("read-only", "whether the cache archive is read-only", false);
        const Core::Configuration          ac(Core::Application::us()->getConfiguration(), paramCacheArchive(dc));
        cfg.cacheArchive         = paramFile(ac);
        cfg.cacheArchiveReadOnly = paramReadOnly(ac);
    }
    // the batched scorers take the whole buffer into one launch; buffer-size 1 keeps the unbuffered protocol
    // of SIMD-diagonal-maximum / diagonal-maximum (Gpu::createFeatureScorer)
    const Gpu::MixtureSet ms = convertMixtureSet(*mixtureSet);
    std::string           err;
    impl_ = Gpu::createFeatureScorer(ms, cfg, &err);
    if (!impl_)
        criticalError("GPU feature scorer: %s", err.c_str());
    // DensityClustering<F, D>::build's messages (DensityClustering.tcc:127-154)
    if (impl_->densityClusteringSource() == GMM_CLUSTERING_CACHED)
        log("using cached density clustering");
    else if (impl_->densityClusteringSource() == GMM_CLUSTERING_WRITTEN)
        log("density clustering written");
    if (cfg.shardDevices.size() > 1)
        log("GPU feature scorer \"%s\" density-sharded over %zu devices, buffer size %u", scorerType,
            cfg.shardDevices.size(), cfg.bufferSize);
    else
        log("GPU feature scorer \"%s\" on device %d, buffer size %u", scorerType, cfg.device, cfg.bufferSize);
}

GpuFeatureScorer::~GpuFeatureScorer() {}

EmissionIndex GpuFeatureScorer::nMixtures() const {
    return impl_->nMixtures();
}

ComponentIndex GpuFeatureScorer::dimension() const {
    return impl_->dimension();
}

AssigningFeatureScorer::AssigningScorer GpuFeatureScorer::wrap(const Gpu::Scorer& s) const {
    return AssigningScorer(new Context(this, s));
}

FeatureScorer::Scorer GpuFeatureScorer::getScorer(const FeatureVector& f) const {
    return getAssigningScorer(f);
}

AssigningFeatureScorer::AssigningScorer GpuFeatureScorer::getAssigningScorer(const FeatureVector& f) const {
    require(f.size() == dimension());
    CallScope scope(this);
    return wrap(impl_->getScorer(f));
}

void GpuFeatureScorer::reset() const {
    impl_->reset();
}

void GpuFeatureScorer::finalize() const {
    impl_->finalize();
}

bool GpuFeatureScorer::isBuffered() const {
    return impl_->isBuffered();
}

void GpuFeatureScorer::addFeature(const FeatureVector& f) const {
    require(f.size() == dimension());
    require(!bufferFilled());
    impl_->addFeature(f);
}

FeatureScorer::Scorer GpuFeatureScorer::flush() const {
    require(!bufferEmpty());
    CallScope scope(this);
    return Scorer(wrap(impl_->flush()));
}

bool GpuFeatureScorer::bufferFilled() const {
    return impl_->bufferFilled();
}

bool GpuFeatureScorer::bufferEmpty() const {
    return impl_->bufferEmpty();
}

u32 GpuFeatureScorer::bufferSize() const {
    return impl_->bufferSize();
}

// ---------------------------------------------------------------------------
// registration (FeatureScorerFactory::registerFeatureScorer<T, Model, Loader>, FeatureScorerFactory.hh:54-66)
// ---------------------------------------------------------------------------
namespace {

const char* const kTypes[] = {"SIMD-diagonal-maximum",        "diagonal-maximum",
                              "batch-diagonal-maximum-int",   "batch-diagonal-maximum-float",
                              "batch-diagonal-maximum-fast",  "preselection-batch-float",
                              "preselection-batch-int",       "diagonal-sum"};

// createInstance<T, MixtureSet> constructs T(config, Ref<const MixtureSet>) (FeatureScorerFactory.hh:114-122)
template<int I>
class GpuScorerOf : public GpuFeatureScorer {
public:
    GpuScorerOf(const Core::Configuration& c, Core::Ref<const MixtureSet> ms)
            : Core::Component(c), GpuFeatureScorer(c, ms, kTypes[I]) {}
};

template<int I>
void registerOne(FeatureScorerFactory* f, u32 firstId) {
    static const std::string name = std::string("gpu-") + kTypes[I];
    f->registerFeatureScorer<GpuScorerOf<I>, MixtureSet, AbstractMixtureSetLoader>(firstId + I, name.c_str());
}

}  // namespace

void Mm::registerGpuFeatureScorers(u32 firstId) {
    installCriticalErrorHandler();
    FeatureScorerFactory* f = Module::instance().featureScorerFactory();
    registerOne<0>(f, firstId);
    registerOne<1>(f, firstId);
    registerOne<2>(f, firstId);
    registerOne<3>(f, firstId);
    registerOne<4>(f, firstId);
    registerOne<5>(f, firstId);
    registerOne<6>(f, firstId);
    registerOne<7>(f, firstId);
}
