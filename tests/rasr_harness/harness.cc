// harness.cc -- TEST INFRASTRUCTURE ONLY: the RASR-side adapter (integration/rasr/Mm/GpuFeatureScorer.cc) linked
// and run inside test doubles of RASR's plugin machinery (tests/rasr_harness/include/README) together with the real
// host-side classes (rasr_amd/csrc/host), in two builds (Makefile):
//   rasr_adapter_harness      (CPU)  over the oracle-backed C-ABI stand-in (gmm_standin.cc);
//   rasr_adapter_harness_gpu  (GPU, -DHARNESS_PRODUCT) over the PRODUCT library librasr_gmm.so -- the HIP kernels;
//                                    the oracle is linked as the checker only.
//
//   1. Mm::registerGpuFeatureScorers(0x500) registers "gpu-<type>" with Mm::Module's FeatureScorerFactory
//      (src/Mm/FeatureScorerFactory.hh:54-66); the scorer is created by id from a configuration whose
//      "buffer-size" is set, through createInstance (:114-122), and wrapped in FeatureScorerScaling as the
//      acoustic model does (src/Mm/ScaledFeatureScorer.hh:56-153; scale 0.75).
//   2. Speech::OfflineRecognizer's sequence (src/Speech/Recognizer.cc:272-282 processFeature with
//      Core::Ref<const Feature>, :198-206 leaveSpeechSegment, reset per segment): every fed context is read
//      for all emissions -- once as the search does (score(e) only, SearchSpace.cc:1613-1659), and for the
//      assigning types once as an aligner does (score(e) and bestDensity(e) on the unscaled context,
//      AlignmentNode.cc:283-310).
//   3. Speech::FeatureScorerNode::work (src/Speech/FeatureScorerNode.cc:113-162): -score(e) of all nEmissions()
//      per frame, flush until empty, finalize(), reset().
//   Buffer sizes 1, 4, 64 and 512 (64 and 512: the ring's asynchronous prefetch), "density-shard-devices".
// Expected values: the oracle on all frames at once, the scaled score 0.75f * score.  SIMD-diagonal-maximum and
// batch-diagonal-maximum-int: bit for bit.  Float types: bit for bit against the stand-in (it IS the oracle); against
// the product library within the float contract, |got - want| <= 1e-4 max(1, |want|), and a different best density
// only where both densities' f64 scores agree within that tolerance.  Exit 0 = every check
// passed.  The CPU build also checks, in a forked child, that the adapter's criticalError routing aborts with the
// component's message when bestDensity() is asked of a type without assignments (the GPU build does not fork a
// process that may hold a GPU context; the routing is the adapter's own code, the same in both builds).
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <Core/Application.hh>
#include <Mm/FeatureScorerFactory.hh>
#include <Mm/ScaledFeatureScorer.hh>

#include "../../integration/rasr/Mm/GpuFeatureScorer.hh"
#include "../../oracle/gmm_oracle.h"

namespace {

struct Rng {
    uint64_t x;
    uint64_t next() {
        uint64_t z = (x += 0x9e3779b97f4a7c15ull);
        z          = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z          = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    float  normal() {
        const double u = uniform() + 1e-300, v = uniform();
        return static_cast<float>(std::sqrt(-2.0 * std::log(u)) * std::cos(6.283185307179586 * v));
    }
};

// a ragged model with random weights; one covariance (the batch types require pooled covariance)
struct Model {
    Core::Ref<Mm::MixtureSet> ms;
    std::vector<float>        means, vars;
    std::vector<uint32_t>     dMean, dCov, off{0}, dens;
    std::vector<double>       logw;
    orc_mixture_set           view() const {
        return orc_mixture_set{ms->dimension(), static_cast<uint32_t>(means.size() / ms->dimension()), means.data(),
                               static_cast<uint32_t>(vars.size() / ms->dimension()), vars.data(),
                               static_cast<uint32_t>(dMean.size()), dMean.data(), dCov.data(),
                               static_cast<uint32_t>(off.size() - 1), off.data(), dens.data(), logw.data()};
    }
};

Model makeModel(uint32_t D, uint32_t M, uint64_t seed) {
    Model m;
    Rng   rng{seed};
    m.ms = Core::Ref<Mm::MixtureSet>(new Mm::MixtureSet(D));
    std::vector<float> v(D);
    for (auto& x : v)
        x = 0.5f + std::fabs(rng.normal());
    m.vars = v;
    m.ms->addCovariance(v);
    for (uint32_t mix = 0; mix < M; ++mix) {
        const uint32_t      K = 1 + static_cast<uint32_t>(rng.next() % 12);
        std::vector<double> w(K);
        double              sum = 0;
        for (auto& x : w)
            sum += (x = 0.1 + rng.uniform());
        Mm::Mixture mixture;
        for (uint32_t j = 0; j < K; ++j) {
            for (auto& x : v)
                x = rng.normal();
            m.means.insert(m.means.end(), v.begin(), v.end());
            const Mm::DensityIndex d = m.ms->addDensity(m.ms->addMean(v), 0);
            m.dMean.push_back(d);
            m.dCov.push_back(0);
            m.dens.push_back(d);
            m.logw.push_back(std::log(w[j] / sum));
            mixture.addLogDensity(d, std::log(w[j] / sum));
        }
        m.off.push_back(static_cast<uint32_t>(m.dens.size()));
        m.ms->addMixture(mixture);
    }
    return m;
}

#ifdef HARNESS_PRODUCT
constexpr bool kProduct = true;
#else
constexpr bool kProduct = false;
#endif

// f64 score of entry j of mixture e for frame x (GaussDiagonalMaximumFeatureScorer, defaults mws = gs = 1:
// 0.5 (-2 log c + D log 2pi + sum log var + sum ((mu - x) / sigma)^2)), for the near-tie check of float best densities
double f64Score(const Model& m, const float* x, uint32_t e, uint32_t j) {
    const uint32_t D = m.ms->dimension(), entry = m.off[e] + j;
    const float*   mu = &m.means[static_cast<size_t>(m.dMean[m.dens[entry]]) * D];
    double         q = -2.0 * m.logw[entry] + D * std::log(2.0 * M_PI);
    for (uint32_t k = 0; k < D; ++k) {
        const double v = m.vars[k], d = (static_cast<double>(mu[k]) - x[k]);
        q += std::log(v) + d * d / v;
    }
    return 0.5 * q;
}

int gFailures = 0;
void check(bool ok, const std::string& what) {
    if (!ok) {
        ++gFailures;
        std::fprintf(stderr, "FAIL: %s\n", what.c_str());
    }
}

struct Expected {
    std::vector<float>    s;  // [M][F]
    std::vector<uint32_t> b;
    bool                  exact = true;  // false: the float contract (product library, float types)
};

bool sameScore(float want, float got, bool exact) {
    if (exact || !std::isfinite(want))
        return std::memcmp(&want, &got, sizeof(float)) == 0;  // bit for bit (and the "no score" values exactly)
    return std::fabs(static_cast<double>(got) - want) <= 1e-4 * std::max(1.0, std::fabs(static_cast<double>(want)));
}

Expected oracleScores(const Model& m, const std::string& type, const std::vector<float>& frames, uint32_t F) {
    const orc_mixture_set ms = m.view();
    const uint32_t        M = ms.n_mixtures, D = ms.dimension;
    Expected              x;
    x.s.assign(static_cast<size_t>(M) * F, 0.0f);
    x.b.assign(static_cast<size_t>(M) * F, 0xffffffffu);
    if (type == "SIMD-diagonal-maximum") {
        orc_simd_model sm;
        orc_simd_prepare(&ms, &sm);
        orc_simd_score(&sm, &ms, frames.data(), F, D, x.s.data(), x.b.data(), 0, 1);
        orc_simd_free(&sm);
    }
    else if (type == "diagonal-maximum") {
        orc_float_model fm;
        orc_float_prepare(&ms, 1.0f, 1.0f, &fm);
        orc_float_score(&fm, &ms, frames.data(), F, D, x.s.data(), x.b.data(), 1);
        orc_float_free(&fm);
    }
    else if (type == "batch-diagonal-maximum-int")
        orc_batch_int_score(&ms, frames.data(), F, D, x.s.data(), 1);
    else
        orc_batch_float_score(&ms, frames.data(), F, D, x.s.data(), 1);
    x.exact = !kProduct || type == "SIMD-diagonal-maximum" || type == "batch-diagonal-maximum-int";
    return x;
}

u32 idOf(const std::string& type) {
    u32 id = 0;
    verify(Mm::Module::instance().featureScorerFactory()->idOf("gpu-" + type, id));
    return id;
}

Core::Ref<Mm::FeatureScorerScaling> create(const Model& m, const std::string& type, u32 bufferSize,
                                           const std::string& shardDevices = "") {
    Core::Configuration root;
    root.set("acoustic-model.mixture-set.buffer-size", std::to_string(bufferSize));
    if (!shardDevices.empty())
        root.set("acoustic-model.mixture-set.density-shard-devices", shardDevices);
    const Core::Configuration c(Core::Configuration(root, "acoustic-model"), "mixture-set");
    Mm::FeatureScorer* fs = Mm::Module::instance().featureScorerFactory()->createFeatureScorer(
            idOf(type), c, Core::Ref<const Mm::AbstractMixtureSet>(m.ms.get()));
    verify(fs);
    return Core::Ref<Mm::FeatureScorerScaling>(new Mm::FeatureScorerScaling(c, Core::Ref<Mm::FeatureScorer>(fs), 0.75f));
}

const Mm::AssigningFeatureScorer::AssigningContextScorer* unscaled(const Mm::FeatureScorer::Scorer& s) {
    const auto* scaled = dynamic_cast<const Mm::FeatureScorerScaling::ScaledContextScorer*>(s.get());
    verify(scaled);
    return dynamic_cast<const Mm::AssigningFeatureScorer::AssigningContextScorer*>(scaled->getUnscaledScorer().get());
}

void runRecognizer(const Model& m, const std::string& type, u32 B, const std::vector<float>& frames, uint32_t F,
                   uint32_t segments, const Expected& ex, bool askBest, const std::string& shardDevices = "") {
    auto           scorer = create(m, type, B, shardDevices);
    const uint32_t M = m.ms->nMixtures(), D = m.ms->dimension();
    const bool     assigning = askBest && (type == "SIMD-diagonal-maximum" || type == "diagonal-maximum");
    uint32_t       t = 0, bad = 0, badBest = 0, nearTies = 0;
    check(scorer->isBuffered() == (B > 1 || type.rfind("batch", 0) == 0), type + ": isBuffered");
    check(scorer->bufferSize() == (scorer->isBuffered() ? B : 0u), type + ": bufferSize");
    auto feed = [&](const Mm::FeatureScorer::Scorer& s) {  // the search reads score(e); an aligner bestDensity(e)
        check(s->nEmissions() == M, type + ": nEmissions");
        for (uint32_t e = 0; e < M; ++e) {
            const float want = 0.75f * ex.s[static_cast<size_t>(e) * F + t], got = s->score(e);
            if (!sameScore(want, got, ex.exact))
                ++bad;
            if (!assigning)
                continue;
            const uint32_t gotB = unscaled(s)->bestDensity(e), wantB = ex.b[static_cast<size_t>(e) * F + t];
            if (gotB == wantB)
                continue;
            const float* x = &frames[static_cast<size_t>(t) * D];
            if (!ex.exact && gotB < m.off[e + 1] - m.off[e] &&
                std::fabs(f64Score(m, x, e, gotB) - f64Score(m, x, e, wantB)) <=
                        1e-4 * std::max(1.0, std::fabs(f64Score(m, x, e, wantB))))
                ++nearTies;  // the float contract: either of two densities whose scores agree within 1e-4
            else
                ++badBest;
        }
        ++t;
    };
    for (uint32_t seg = 0; seg < segments; ++seg) {
        scorer->reset();  // Recognizer.cc:186 (enterSpeechSegment)
        const uint32_t t0 = F * seg / segments, t1 = F * (seg + 1) / segments;
        for (uint32_t f = t0; f < t1; ++f) {
            Core::Ref<const Mm::Feature> feature(new Mm::Feature(
                    Mm::FeatureVector(frames.begin() + static_cast<size_t>(f) * D, frames.begin() + static_cast<size_t>(f + 1) * D)));
            if (scorer->isBuffered() && !scorer->bufferFilled())  // processFeature
                scorer->addFeature(feature);
            else
                feed(scorer->getScorer(feature));
        }
        if (scorer->isBuffered())  // leaveSpeechSegment
            while (!scorer->bufferEmpty())
                feed(scorer->flush());
    }
    check(t == F, type + ": every frame fed once");
    check(bad == 0, type + " buffer " + std::to_string(B) + ": " + std::to_string(bad) + " scaled scores differ");
    check(badBest == 0, type + " buffer " + std::to_string(B) + ": " + std::to_string(badBest) + " best densities differ");
    std::printf("recognizer %-30s buffer-size %5u%s %-7s: %u frames x %u emissions, scores %s, best densities %s%s\n",
                type.c_str(), B, shardDevices.empty() ? "" : (" density-shard-devices " + shardDevices).c_str(),
                askBest ? "aligner" : "search", F, M, bad ? "DIFFER" : (ex.exact ? "equal" : "within 1e-4"),
                assigning ? (badBest ? "DIFFER" : "equal") : "n/a",
                nearTies ? (" (" + std::to_string(nearTies) + " near ties)").c_str() : "");
}

void runScoreDump(const Model& m, const std::string& type, u32 B, const std::vector<float>& frames, uint32_t F,
                  const Expected& ex) {
    auto           scorer = create(m, type, B);
    const uint32_t M = m.ms->nMixtures(), D = m.ms->dimension();
    std::vector<float> dump;
    auto putData = [&](const Mm::FeatureScorer::Scorer& s) {  // FeatureScorerNode::putData: +log space
        for (uint32_t e = 0; e < s->nEmissions(); ++e)
            dump.push_back(-s->score(e));
    };
    for (int round = 0; round < 2; ++round) {  // two segments through the same node: finalize() + reset() between
        for (uint32_t f = 0; f < F; ++f) {
            Mm::FeatureVector v(frames.begin() + static_cast<size_t>(f) * D, frames.begin() + static_cast<size_t>(f + 1) * D);
            if (scorer->isBuffered() && !scorer->bufferFilled())
                scorer->addFeature(v);
            else
                putData(scorer->getScorer(v));
        }
        if (scorer->isBuffered())
            while (!scorer->bufferEmpty())
                putData(scorer->flush());
        scorer->finalize();
        scorer->reset();
    }
    uint32_t bad = 0;
    check(dump.size() == 2u * F * M, type + ": dump size");
    for (size_t i = 0; i < dump.size() && dump.size() == 2u * F * M; ++i) {
        const uint32_t f = static_cast<uint32_t>((i / M) % F), e = static_cast<uint32_t>(i % M);
        const float want = -(0.75f * ex.s[static_cast<size_t>(e) * F + f]);
        if (!sameScore(want, dump[i], ex.exact))
            ++bad;
    }
    check(bad == 0, type + " dump: " + std::to_string(bad) + " values differ");
    std::printf("score dump %-30s buffer-size %5u: 2 segments x %u frames, %s\n", type.c_str(), B, F,
                bad ? "DIFFER" : (ex.exact ? "equal" : "within 1e-4"));
}

#ifndef HARNESS_PRODUCT
// a type without assignments asked for bestDensity(): the adapter routes the error to the component's
// criticalError (Core::Component::criticalError aborts) -- run in a child
void checkCriticalErrorRouting(const Model& m, const std::vector<float>& frames) {
    std::fflush(stdout);
    int   pipefd[2];
    verify(pipe(pipefd) == 0);
    const pid_t pid = fork();
    if (pid == 0) {
        dup2(pipefd[1], 2);
        auto      scorer = create(m, "batch-diagonal-maximum-int", 1);
        const u32 D      = m.ms->dimension();
        Mm::FeatureVector v(frames.begin(), frames.begin() + D);
        while (!scorer->bufferFilled())
            scorer->addFeature(v);
        auto s = scorer->getScorer(v);
        unscaled(s)->bestDensity(0);  // must not return
        _exit(0);
    }
    close(pipefd[1]);
    std::string err;
    char        buf[512];
    ssize_t     k;
    while ((k = read(pipefd[0], buf, sizeof(buf))) > 0)
        err.append(buf, static_cast<size_t>(k));
    close(pipefd[0]);
    int status = 0;
    waitpid(pid, &status, 0);
    const bool aborted = WIFSIGNALED(status) && WTERMSIG(status) == SIGABRT;
    check(aborted && err.find("bestDensity() not available") != std::string::npos,
          "criticalError routing (status " + std::to_string(status) + "): " + err);
    std::printf("criticalError routing: batch type bestDensity() -> %s\n", aborted ? "component criticalError, abort" : "NOT ABORTED");
}

#endif

}  // namespace

#ifndef HARNESS_PRODUCT
extern std::vector<int> gStandinShardDevices;  // gmm_standin.cc
extern "C" std::string  gStandinCacheArchive;  // defined inside gmm_standin.cc's extern "C" block
extern "C" uint32_t     gStandinFlags;

// "density-clustering.cache-archive" names an archive of the application's configuration; its "file" and
// "read-only" reach gmm_scorer_config.cache_archive / GMM_FLAG_CACHE_ARCHIVE_READ_ONLY
// (DensityClustering.cc:27-28, Application.cc:397-400)
void checkCacheArchiveResolution(const Model& m) {
    Core::Configuration app = Core::Application::us()->getConfiguration();  // a copy sharing the resources
    create(m, "SIMD-diagonal-maximum", 1);
    check(gStandinCacheArchive.empty(), "no global-cache.file -> no cache archive");
    app.set("global-cache.file", "/tmp/global.cache");
    create(m, "SIMD-diagonal-maximum", 1);
    check(gStandinCacheArchive == "/tmp/global.cache" && !(gStandinFlags & GMM_FLAG_CACHE_ARCHIVE_READ_ONLY),
          "default archive global-cache -> its file");
    app.set("clustering-cache.file", "/tmp/clustering.cache");
    app.set("clustering-cache.read-only", "true");
    Core::Configuration root;
    root.set("acoustic-model.mixture-set.density-clustering.cache-archive", "clustering-cache");
    const Core::Configuration c(Core::Configuration(root, "acoustic-model"), "mixture-set");
    Mm::FeatureScorer* fs = Mm::Module::instance().featureScorerFactory()->createFeatureScorer(
            idOf("SIMD-diagonal-maximum"), c, Core::Ref<const Mm::AbstractMixtureSet>(m.ms.get()));
    verify(fs);
    Core::Ref<Mm::FeatureScorer> keep(fs);
    check(gStandinCacheArchive == "/tmp/clustering.cache" && (gStandinFlags & GMM_FLAG_CACHE_ARCHIVE_READ_ONLY),
          "density-clustering.cache-archive -> that archive's file, read-only");
    std::printf("cache-archive -> gmm_scorer_config.cache_archive \"%s\" read-only\n", gStandinCacheArchive.c_str());
}
#endif

int main() {
    Mm::registerGpuFeatureScorers(0x500);
    Mm::registerGpuFeatureScorers(0x500);  // a second registration of the same ids is refused by the factory
    u32 id = 0;
    check(Mm::Module::instance().featureScorerFactory()->idOf("gpu-SIMD-diagonal-maximum", id) && id == 0x500,
          "gpu-SIMD-diagonal-maximum at 0x500");
    check(Mm::Module::instance().featureScorerFactory()->idOf("gpu-batch-diagonal-maximum-int", id) && id == 0x502,
          "gpu-batch-diagonal-maximum-int at 0x502");
    // 3 segments of 700 frames: a 512-frame ring fills, wraps and prefetches inside every segment
    const uint32_t     D = 39, M = 40, F = 2100;
    const Model        model = makeModel(D, M, 7);
    std::vector<float> frames(static_cast<size_t>(F) * D);
    Rng                rng{11};
    for (auto& x : frames)
        x = rng.normal();
    std::printf("adapter over %s\n", kProduct ? "librasr_gmm.so (HIP)" : "the oracle-backed C-ABI stand-in");
    const char* types[] = {"SIMD-diagonal-maximum", "diagonal-maximum", "batch-diagonal-maximum-int",
                           "batch-diagonal-maximum-float"};
    for (const char* type : types) {
        const Expected ex        = oracleScores(model, type, frames, F);
        const bool     assigning = std::string(type) == "SIMD-diagonal-maximum" || std::string(type) == "diagonal-maximum";
        for (u32 B : {1u, 4u, 64u, 512u}) {
            if (B == 1 && std::string(type).rfind("batch", 0) == 0)
                continue;  // the batch types are always buffered
            runRecognizer(model, type, B, frames, F, 3, ex, false);
            if (assigning)
                runRecognizer(model, type, B, frames, F, 3, ex, true);
            runScoreDump(model, type, B, frames, F, ex);
        }
    }
    // "density-shard-devices" reaches gmm_scorer_create_sharded with the configured device list
    {
        const Expected ex = oracleScores(model, "SIMD-diagonal-maximum", frames, F);
#ifdef HARNESS_PRODUCT
        // three density parts on device 0 (the copy exchange; the library's one-GPU form of config 4)
        for (u32 B : {64u, 512u}) {
            runRecognizer(model, "SIMD-diagonal-maximum", B, frames, F, 3, ex, true, "0,0,0");
            runRecognizer(model, "SIMD-diagonal-maximum", B, frames, F, 3, ex, false, "0,0,0");
        }
        const Expected exi = oracleScores(model, "batch-diagonal-maximum-int", frames, F);
        runRecognizer(model, "batch-diagonal-maximum-int", 512, frames, F, 3, exi, false, "0,0,0");
#else
        gStandinShardDevices.clear();
        runRecognizer(model, "SIMD-diagonal-maximum", 64, frames, F, 3, ex, true, "0,1,2");
        check(gStandinShardDevices == std::vector<int>({0, 1, 2}), "density-shard-devices -> gmm_scorer_create_sharded");
        std::printf("density-shard-devices 0,1,2 -> gmm_scorer_create_sharded over %zu devices\n", gStandinShardDevices.size());
#endif
    }
#ifndef HARNESS_PRODUCT
    checkCriticalErrorRouting(model, frames);
    checkCacheArchiveResolution(model);
#endif
    std::printf("%s (%d failures)\n", gFailures ? "FAILED" : "PASSED", gFailures);
    return gFailures ? 1 : 0;
}
