// feature_scorer_driver.cc -- drives Mm::Gpu::FeatureScorer exactly as RASR's recognizer does
// (src/Speech/Recognizer.cc:198-206 leaveSpeechSegment, :272-282 processFeature) and dumps every
// ContextScorer's scores, so tests/test_host_protocol.py can compare them with the oracle.
//
// usage: feature_scorer_driver <model> <frames.bin> <out.bin> <type> <bufferSize> <segments> [protocol]
//   protocol  : "recognizer" (default): Speech::OfflineRecognizer, reset() before every segment,
//               scores as the search reads them;
//               "delayed": as "recognizer", but every context is consumed only after the next `kDelay`
//               frames were scored (a RecognizerDelayHandler-like consumer, src/Speech/DelayedRecognizer.cc:65-135;
//               unbuffered types: bestDensity() of such a context finds its best densities replaced on
//               the device and scores its frame again);
//               "node": Speech::FeatureScorerNode::work (src/Speech/FeatureScorerNode.cc:113-162), the
//               reference's score dump: every frame's -score(e) for ALL emissions (putData, :95-111),
//               finalize() and reset() after every segment
//   model     : a RASR mixture-set file read by Mm::Gpu::MixtureSet::read like the reference's MixtureSetReader:
//               text for *.pms / *.gz, a binary maximum-likelihood estimator file for any other name; or
//   model.drvmodel : (this test's own dump) u32 D, nMeans, nCov, nDens, nMix, nEntries; f32 means[nMeans*D]; f32 var[nCov*D];
//               u32 densMean[nDens]; u32 densCov[nDens]; u32 offsets[nMix+1]; u32 dens[nEntries];
//               f64 logw[nEntries]
//   frames.bin: u32 F, D; f32 frames[F*D]
//   out.bin   : u32 F, M, launches; f32 scores[F*M] (frame-major, as consumed); u32 best[F*M]
// The frames are split into `segments` equal speech segments with reset() between them.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <string>
#include <vector>

#include "../../rasr_amd/csrc/host/GpuFeatureScorer.hh"

template <class T>
static bool readVec(FILE* f, std::vector<T>& v, size_t n) {
    v.resize(n);
    return n == 0 || fread(v.data(), sizeof(T), n, f) == n;
}

// the binary dump written by tests/test_host_protocol.py, built through the MixtureSet::add* API
static std::unique_ptr<Mm::Gpu::MixtureSet> readBinaryModel(const std::string& path) {
    FILE* fm = fopen(path.c_str(), "rb");
    if (!fm)
        return nullptr;
    uint32_t h[6];
    if (fread(h, sizeof(uint32_t), 6, fm) != 6)
        return nullptr;
    const uint32_t        D = h[0], nMeans = h[1], nCov = h[2], nDens = h[3], nMix = h[4], nEnt = h[5];
    std::vector<float>    means, var;
    std::vector<uint32_t> dm, dc, off, dens;
    std::vector<double>   logw;
    if (!readVec(fm, means, size_t(nMeans) * D) || !readVec(fm, var, size_t(nCov) * D) || !readVec(fm, dm, nDens) ||
        !readVec(fm, dc, nDens) || !readVec(fm, off, nMix + 1) || !readVec(fm, dens, nEnt) || !readVec(fm, logw, nEnt))
        return nullptr;
    fclose(fm);
    std::unique_ptr<Mm::Gpu::MixtureSet> ms(new Mm::Gpu::MixtureSet(D));
    for (uint32_t i = 0; i < nMeans; ++i)
        ms->addMean(std::vector<float>(means.begin() + size_t(i) * D, means.begin() + size_t(i + 1) * D));
    for (uint32_t c = 0; c < nCov; ++c)
        ms->addCovariance(std::vector<float>(var.begin() + size_t(c) * D, var.begin() + size_t(c + 1) * D));
    for (uint32_t i = 0; i < nDens; ++i)
        ms->addDensity(dm[i], dc[i]);
    for (uint32_t m = 0; m < nMix; ++m)
        ms->addMixture(std::vector<uint32_t>(dens.begin() + off[m], dens.begin() + off[m + 1]),
                       std::vector<double>(logw.begin() + off[m], logw.begin() + off[m + 1]));
    return ms;
}

// ---------------------------------------------------------------------------------------------------------
// bench mode: the drop-in's throughput through the recognizer protocol, PCIe included
//   feature_scorer_driver bench <type> <bufferSizes> <frames> <mixtures> <densitiesPerMixture> <dim> <best 0|1>
//                               [readPermille]
// bufferSizes / frames: comma-separated lists of equal length (one scorer per buffer size, timed on that many
// frames).  Synthetic model of SURVEY 8(d) (means N(0,1), pooled variance 0.5 + |N(0,1)|, uniform weights;
// splitmix64 + Box-Muller) and N(0,1) frames.  Every frame's context is consumed as FeatureScorerNode dumps
// it: score(e) for every emission (and bestDensity(e) for every emission with best = 1, the dump's read; with
// best = 2 an aligner's read instead: bestDensity(e) of 1-10 emissions per frame, drawn per frame).
// readPermille < 1000: a search-like consumer instead, score(e) of that share of the emissions per frame, a
// scattered set that moves from frame to frame (the search's active states; SearchSpace.cc:1613-1659).
// One warm-up segment, then one timed segment per size; prints one JSON line per size.
// ---------------------------------------------------------------------------------------------------------
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

std::vector<uint32_t> parseList(const char* s) {
    std::vector<uint32_t> out;
    for (const char* p = s; *p;) {
        char* end = nullptr;
        out.push_back(static_cast<uint32_t>(strtoul(p, &end, 10)));
        p = *end == ',' ? end + 1 : end;
        if (end == p && *p)
            break;
    }
    return out;
}
}  // namespace

static int benchMain(int argc, char** argv) {
    if (argc != 9 && argc != 10) {
        fprintf(stderr, "usage: %s bench type bufferSizes frames mixtures densitiesPerMixture dim best [readPermille]\n",
                argv[0]);
        return 2;
    }
    const uint32_t permille = argc == 10 ? std::min<uint32_t>(1000, atoi(argv[9])) : 1000;
    const std::string           type  = argv[2];
    const std::vector<uint32_t> sizes = parseList(argv[3]), counts = parseList(argv[4]);
    const uint32_t              M = atoi(argv[5]), K = atoi(argv[6]), D = atoi(argv[7]);
    const uint32_t              bestMode = static_cast<uint32_t>(atoi(argv[8]));
    const bool                  readBest = bestMode != 0;
    if (sizes.empty() || sizes.size() != counts.size())
        return 2;
    Rng                 rng{12345};
    Mm::Gpu::MixtureSet ms(D);
    std::vector<float>  v(D);
    for (uint32_t k = 0; k < D; ++k)
        v[k] = 0.5f + std::fabs(rng.normal());
    ms.addCovariance(v);
    std::vector<uint32_t> dens(K);
    std::vector<double>   logw(K, std::log(1.0 / K));
    for (uint32_t m = 0; m < M; ++m) {
        for (uint32_t j = 0; j < K; ++j) {
            for (uint32_t k = 0; k < D; ++k)
                v[k] = rng.normal();
            dens[j] = ms.addDensity(ms.addMean(v), 0);
        }
        ms.addMixture(dens, logw);
    }
    uint32_t maxF = 0;
    for (uint32_t c : counts)
        maxF = std::max(maxF, c);
    std::vector<Mm::Gpu::FeatureVector> frames(maxF, Mm::Gpu::FeatureVector(D));
    for (auto& f : frames)
        for (auto& x : f)
            x = rng.normal();
    for (size_t i = 0; i < sizes.size(); ++i) {
        const uint32_t         B = sizes[i], F = counts[i];
        Mm::Gpu::Configuration cfg;
        cfg.type       = type;
        cfg.bufferSize = B;
        std::string err;
        auto        scorer = Mm::Gpu::createFeatureScorer(ms, cfg, &err);
        if (!scorer) {
            fprintf(stderr, "createFeatureScorer failed: %s\n", err.c_str());
            return 3;
        }
        double   sink  = 0;
        uint64_t sinkB = 0;
        // search-like consumer: 64 scattered active sets (ascending emission indices), one per frame in turn,
        // drawn before the timed segment so that the consumer's own cost is the reads alone
        std::vector<std::vector<uint32_t>> active;
        if (permille < 1000) {
            Rng sel{777};
            active.resize(64);
            for (auto& a : active)
                for (uint32_t e = 0; e < M; ++e)
                    if (sel.next() % 1000u < permille)
                        a.push_back(e);
        }
        uint32_t frameNo = 0;
        Rng      pick{999};
        auto     consume = [&](const Mm::Gpu::Scorer& s) {
            const uint32_t n   = s->nEmissions();
            float          acc = 0;
            if (permille >= 1000)
                for (uint32_t e = 0; e < n; ++e)
                    acc += s->score(e);
            else
                for (uint32_t e : active[frameNo++ & 63u])
                    acc += s->score(e);
            sink += acc;
            if (readBest && s->hasBestDensity()) {
                if (bestMode == 2)  // an aligner: the frame's 1-10 aligned / competing emissions
                    for (uint32_t k = 1 + static_cast<uint32_t>(pick.next() % 10u); k > 0; --k)
                        sinkB += s->bestDensity(static_cast<uint32_t>(pick.next() % n));
                else
                    for (uint32_t e = 0; e < n; ++e)
                        sinkB += s->bestDensity(e);
            }
        };
        auto segment = [&](uint32_t t0, uint32_t t1) {
            scorer->reset();
            for (uint32_t t = t0; t < t1; ++t) {
                if (scorer->isBuffered() && !scorer->bufferFilled())
                    scorer->addFeature(frames[t]);
                else
                    consume(scorer->getScorer(frames[t]));
            }
            if (scorer->isBuffered())
                while (!scorer->bufferEmpty())
                    consume(scorer->flush());
        };
        segment(0, std::min<uint32_t>(F, std::max<uint32_t>(2 * B, 64)));  // warm-up
        auto lc = [&]() -> uint32_t {
            if (auto* b = dynamic_cast<Mm::Gpu::GpuBatchFeatureScorer*>(scorer.get()))
                return b->nLaunches();
            if (auto* u = dynamic_cast<Mm::Gpu::GpuFeatureScorer*>(scorer.get()))
                return u->nLaunches();
            return 0;
        };
        const uint32_t l0 = lc();
        const auto     t0 = std::chrono::steady_clock::now();
        segment(0, F);
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"type\": \"%s\", \"buffer_size\": %u, \"frames\": %u, \"seconds\": %.6f, \"frames_per_s\": %.1f, "
               "\"launches\": %u, \"best\": %s, \"read_permille\": %u, \"mixtures\": %u, \"densities\": %u, "
               "\"dim\": %u, \"checksum\": %.6e}\n",
               type.c_str(), B, F, sec, F / sec, lc() - l0, bestMode == 2 ? "\"sparse 1-10 per frame\"" : readBest ? "true" : "false",
               permille, M, M * K, D,
               sink + double(sinkB));
        fflush(stdout);
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && std::string(argv[1]) == "bench")
        return benchMain(argc, argv);
    if (argc != 7 && argc != 8) {
        fprintf(stderr, "usage: %s model.bin frames.bin out.bin type bufferSize segments [recognizer|node|delayed|search|late|aligner|memo]\n",
                argv[0]);
        return 2;
    }
    const std::string protocol = argc == 8 ? argv[7] : "recognizer";
    if (protocol != "recognizer" && protocol != "node" && protocol != "delayed" && protocol != "search" &&
        protocol != "late" && protocol != "aligner" && protocol != "memo")
        return 2;
    // the reference memoizes bestDensity(e) per (frame, e) (AssigningFeatureScorer.hh:110-121): "memo" asks
    // bestDensity(0) first, then every other emission (past the drop-in's kSparseMax single-pair answers), then
    // bestDensity(0) again; output: the first answer of each emission; stderr: "memo mismatches: N" (second != first)
    const bool memo = protocol == "memo";
    uint32_t   memoMismatches = 0;
    const bool search = protocol == "search";  // the recognizer's sequence, score(e) only (no bestDensity)
    const bool late   = protocol == "late";    // score(e) only for the first half of the frames, then bestDensity too
    // an aligner's read (AbstractMixtureSetEstimator.cc:370-384): score(e) of every emission, bestDensity(e) of 1-10
    // emissions per frame drawn from the frame's number (the others' best densities stay 0xffffffff in the output)
    const bool aligner = protocol == "aligner";
    uint32_t   consumed = 0;
    const bool     delayed = protocol == "delayed";
    const uint32_t kDelay  = 3;
    std::deque<Mm::Gpu::Scorer> pending;
    const bool node = protocol == "node";
    if (delayed && atoi(argv[5]) > 1)
        return 2;  // a buffered context is valid only until the next getScorer() reuses its position
    const std::string modelPath(argv[1]);
    const std::string dump(".drvmodel");
    const bool        pms = !(modelPath.size() >= dump.size() &&
                              modelPath.compare(modelPath.size() - dump.size(), dump.size(), dump) == 0);
    FILE*             ff  = fopen(argv[2], "rb");
    if (!ff)
        return 2;
    std::unique_ptr<Mm::Gpu::MixtureSet> model;
    if (pms) {
        std::string err;
        model = Mm::Gpu::MixtureSet::read(modelPath, &err);
        if (!model) {
            fprintf(stderr, "MixtureSet::read failed: %s\n", err.c_str());
            return 3;
        }
    }
    else
        model = readBinaryModel(modelPath);
    if (!model)
        return 2;
    const uint32_t D = model->dimension();
    uint32_t fh[2];
    if (fread(fh, sizeof(uint32_t), 2, ff) != 2 || fh[1] != D)
        return 2;
    std::vector<float> frames;
    if (!readVec(ff, frames, size_t(fh[0]) * D))
        return 2;
    fclose(ff);
    const uint32_t F = fh[0];

    const Mm::Gpu::MixtureSet& ms = *model;
    Mm::Gpu::Configuration cfg;
    cfg.type       = argv[4];
    cfg.bufferSize = static_cast<uint32_t>(atoi(argv[5]));
    // RASR_DRIVER_SHARD_DEVICES="0,0,0": the density-sharded scorer ("density-shard-devices" of the adapter)
    if (const char* sd = std::getenv("RASR_DRIVER_SHARD_DEVICES"))
        for (uint32_t d : parseList(sd))
            cfg.shardDevices.push_back(static_cast<int>(d));
    // RASR_DRIVER_CACHE_ARCHIVE=path: the density clustering's cache archive (preselection types); the driver reports
    // where the clustering came from on stderr ("clustering: built|written|cached")
    if (const char* ca = std::getenv("RASR_DRIVER_CACHE_ARCHIVE"))
        cfg.cacheArchive = ca;
    std::string                             err;
    std::unique_ptr<Mm::Gpu::FeatureScorer> scorer = Mm::Gpu::createFeatureScorer(ms, cfg, &err);
    if (!scorer) {
        fprintf(stderr, "createFeatureScorer failed: %s\n", err.c_str());
        return 3;
    }
    if (const int src = scorer->densityClusteringSource(); src >= 0)
        fprintf(stderr, "clustering: %s\n", src == GMM_CLUSTERING_CACHED ? "cached" : src == GMM_CLUSTERING_WRITTEN ? "written" : "built");
    const uint32_t        M = scorer->nMixtures();
    std::vector<float>    outS;
    std::vector<uint32_t> outB;
    auto consume = [&](const Mm::Gpu::Scorer& s) {  // the search reads score(e) for active e
        const uint32_t n        = node ? s->nEmissions() : M;  // the node dumps nEmissions() values per frame
        const bool     readBest = !search && (!late || 2 * consumed >= F) && s->hasBestDensity();
        const size_t   row      = outB.size();
        for (uint32_t e = 0; e < n; ++e) {
            outS.push_back(node ? -s->score(e) : s->score(e));  // FeatureScorerNode::putData: +log space
            outB.push_back(readBest && !aligner && !memo ? s->bestDensity(e) : 0xffffffffu);
        }
        if (memo && readBest) {
            const Mm::Gpu::DensityInMixture first = s->bestDensity(0);
            outB[row]                    = first;
            for (uint32_t e = 1; e < n; ++e)
                outB[row + e] = s->bestDensity(e);
            if (s->bestDensity(0) != first)
                ++memoMismatches;
        }
        if (aligner && readBest) {
            Rng pick{0x5eedull + consumed};
            for (uint32_t k = 1 + static_cast<uint32_t>(pick.next() % 10u); k > 0; --k) {
                const uint32_t e = static_cast<uint32_t>(pick.next() % n);
                outB[row + e]    = s->bestDensity(e);
            }
        }
        ++consumed;
    };
    const uint32_t segments = static_cast<uint32_t>(atoi(argv[6]));
    for (uint32_t seg = 0; seg < segments; ++seg) {
        if (!node)
            scorer->reset();  // Recognizer.cc:186
        const uint32_t t0 = F * seg / segments, t1 = F * (seg + 1) / segments;
        auto take = [&](const Mm::Gpu::Scorer& s) {
            if (!delayed)
                return consume(s);
            pending.push_back(s);
            if (pending.size() > kDelay) {
                consume(pending.front());
                pending.pop_front();
            }
        };
        for (uint32_t t = t0; t < t1; ++t) {
            Mm::Gpu::FeatureVector f(frames.begin() + size_t(t) * D, frames.begin() + size_t(t + 1) * D);
            if (scorer->isBuffered() && !scorer->bufferFilled())  // Recognizer.cc:275-277, FeatureScorerNode.cc:131-134
                scorer->addFeature(f);
            else
                take(scorer->getScorer(f));
        }
        if (scorer->isBuffered())  // Recognizer.cc:200-204, FeatureScorerNode.cc:148-154
            while (!scorer->bufferEmpty())
                take(scorer->flush());
        while (!pending.empty()) {
            consume(pending.front());
            pending.pop_front();
        }
        if (node) {  // FeatureScorerNode.cc:157-159
            scorer->finalize();
            scorer->reset();
        }
    }
    if (memo)
        fprintf(stderr, "memo mismatches: %u\n", memoMismatches);
    uint32_t launches = 0;
    if (auto* b = dynamic_cast<Mm::Gpu::GpuBatchFeatureScorer*>(scorer.get()))
        launches = b->nLaunches();
    else if (auto* u = dynamic_cast<Mm::Gpu::GpuFeatureScorer*>(scorer.get()))
        launches = u->nLaunches();
    FILE* fo = fopen(argv[3], "wb");
    const uint32_t oh[3] = {static_cast<uint32_t>(outS.size() / (M ? M : 1)), M, launches};
    fwrite(oh, sizeof(uint32_t), 3, fo);
    fwrite(outS.data(), sizeof(float), outS.size(), fo);
    fwrite(outB.data(), sizeof(uint32_t), outB.size(), fo);
    fclose(fo);
    return 0;
}
