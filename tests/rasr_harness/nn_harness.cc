// nn_harness.cc -- TEST INFRASTRUCTURE ONLY: the RASR-side hybrid-DNN adapter (integration/rasr/Nn/
// GpuBatchFeatureScorer.cc + GpuBatchFeatureScorerNetwork.cc) linked and run inside test doubles of RASR's plugin
// machinery and of the Nn network classes (tests/rasr_harness/include, see its README), in two builds (Makefile):
//   rasr_nn_harness      (CPU)  over the f32 C-ABI stand-in (nn_standin.cc);
//   rasr_nn_harness_gpu  (GPU, -DHARNESS_PRODUCT) over the PRODUCT library librasr_gmm.so (nnGemm8p, bf16 MFMA).
//
// usage: rasr_nn_harness <case directory>
//   config.txt    resource lines "<path>.<parameter> = <value>" (the network, prior and class-label configuration
//                 of the scorer at "acoustic-model.mixture-set"), plus "harness.buffer-sizes = 1,8,64"
//   mixtures.bin  u32 M, then per mixture u32 K and K f64 log weights (the mixture set the class count and the
//                 prior come from)
//   frames.bin    u32 F, u32 D, F x D f32
// For every buffer size B it
//   1. registers the adapter at the Nn id range (Nn::registerGpuBatchFeatureScorer, as src/Nn/Module.cc:39-67
//      registers nn-batch-feature-scorer) and creates the scorer through Mm::FeatureScorerFactory;
//   2. runs Speech::OfflineRecognizer's sequence (src/Speech/Recognizer.cc:272-282 / :198-206) over 2 segments with
//      reset() between them: addFeature until bufferFilled(), then getScorer(f), flush() until bufferEmpty(); every
//      context is read for all emissions (score(e)) right away, as the search does;
//   3. writes scores_<B>.bin: F x M f32, row t = the scores of frame t (the caller compares them with
//      oracle/nn_oracle.py).  Exit 0 = the protocol delivered every frame exactly once.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include <Mm/FeatureScorerFactory.hh>
#include <Mm/Module.hh>

#include "../../integration/rasr/Nn/GpuBatchFeatureScorer.hh"

namespace {

template <class T>
bool readAll(FILE* f, T* p, size_t n) {
    return std::fread(p, sizeof(T), n, f) == n;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: %s <case directory>\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    Core::Configuration root;
    {
        std::ifstream in(dir + "/config.txt");
        std::string   line;
        while (std::getline(in, line)) {
            const size_t eq = line.find('=');
            if (line.empty() || line[0] == '#' || eq == std::string::npos)
                continue;
            auto trim = [](std::string s) {
                const size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t");
                return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
            };
            root.set(trim(line.substr(0, eq)), trim(line.substr(eq + 1)));
        }
    }
    // the mixture set: only its mixture count and weights matter to the NN scorer (Prior::setFromMixtureSet)
    Core::Ref<Mm::MixtureSet> ms;
    {
        FILE* f = std::fopen((dir + "/mixtures.bin").c_str(), "rb");
        u32   M = 0;
        verify(f && readAll(f, &M, 1));
        ms = Core::Ref<Mm::MixtureSet>(new Mm::MixtureSet(1));
        const Mm::MeanIndex mean = ms->addMean(std::vector<Mm::MeanType>(1, 0.0f));
        ms->addCovariance(std::vector<Mm::VarianceType>(1, 1.0f));
        for (u32 m = 0; m < M; ++m) {
            u32 K = 0;
            verify(readAll(f, &K, 1));
            std::vector<f64> w(K);
            verify(readAll(f, w.data(), K));
            Mm::Mixture x;
            for (u32 j = 0; j < K; ++j)
                x.addLogDensity(ms->addDensity(mean, 0), w[j]);
            ms->addMixture(x);
        }
        std::fclose(f);
    }
    std::vector<float> frames;
    u32                F = 0, D = 0;
    {
        FILE* f = std::fopen((dir + "/frames.bin").c_str(), "rb");
        verify(f && readAll(f, &F, 1) && readAll(f, &D, 1));
        frames.resize(static_cast<size_t>(F) * D);
        verify(readAll(f, frames.data(), frames.size()));
        std::fclose(f);
    }
    std::vector<u32> bufferSizes;
    {
        std::string v;
        verify(Core::Configuration(root, "harness").get("buffer-sizes", v));
        std::stringstream ss(v);
        for (std::string x; std::getline(ss, x, ',');)
            bufferSizes.push_back(static_cast<u32>(std::atoi(x.c_str())));
    }

    Nn::registerGpuBatchFeatureScorer();  // id 0x310, name gpu-nn-batch-feature-scorer
    u32 id = 0;
    verify(Mm::Module::instance().featureScorerFactory()->idOf("gpu-nn-batch-feature-scorer", id) && id == 0x310);
    int failures = 0;
    for (u32 B : bufferSizes) {
        root.set("acoustic-model.mixture-set.buffer-size", std::to_string(B));
        const Core::Configuration c(Core::Configuration(root, "acoustic-model"), "mixture-set");
        Core::Ref<Mm::FeatureScorer> scorer(Mm::Module::instance().featureScorerFactory()->createFeatureScorer(
                id, c, Core::Ref<const Mm::AbstractMixtureSet>(ms.get())));
        verify(scorer);
        const u32          M = scorer->nMixtures();
        std::vector<float> out;
        out.reserve(static_cast<size_t>(F) * M);
        auto feed = [&](const Mm::FeatureScorer::Scorer& s) {
            verify(s->nEmissions() == M);
            for (u32 e = 0; e < M; ++e)
                out.push_back(s->score(e));
        };
        const u32 segments = 2;
        for (u32 seg = 0; seg < segments; ++seg) {
            scorer->reset();
            for (u32 t = F * seg / segments; t < F * (seg + 1) / segments; ++t) {
                const Mm::FeatureVector v(frames.begin() + static_cast<size_t>(t) * D,
                                          frames.begin() + static_cast<size_t>(t + 1) * D);
                if (!scorer->bufferFilled())
                    scorer->addFeature(v);
                else
                    feed(scorer->getScorer(v));
            }
            while (!scorer->bufferEmpty())
                feed(scorer->flush());
        }
        const bool complete = out.size() == static_cast<size_t>(F) * M;
        failures += complete ? 0 : 1;
        FILE* f = std::fopen((dir + "/scores_" + std::to_string(B) + ".bin").c_str(), "wb");
        verify(f && std::fwrite(out.data(), sizeof(float), out.size(), f) == out.size());
        std::fclose(f);
        std::printf("nn recognizer buffer-size %4u: %u frames x %u classes %s\n", B, F, M,
                    complete ? "delivered" : "INCOMPLETE");
    }
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "PASSED", failures);
    return failures ? 1 : 0;
}
