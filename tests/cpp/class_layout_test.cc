// Host check of the score-only layouts against the arithmetic their kernels apply to them, without a GPU:
// the class layout (gmm_prepare.cc buildClassLayout, preselection-batch-int: gmm_kernels_i8.hip
// scoreI8Seg<..., SCORE_ONLY>) and the slot layout (buildSlotLayout, the other calls without best densities:
// scoreI8Cls -- every tile gives rows 4g + s and 4g + s + 2 the parity of bit 2g + s of the mixture word, the
// kernel's minimum is min over (g, s) of 2 min(dot + h) + p).  For the class layout:
//   * every entry of every mixture sits in exactly one row; padding rows carry the pad constant and zero operands;
//   * a class tile's rows in lane group g have the parity of bit g of the mixture word, a mixed tile's row
//     R = 16 i + 4g + r (i-th mixed tile) has parity (R >= er);
//   * for random quantized frames, the kernel's minimum -- class tiles: min over rows of v = dot + h, then
//     2 v + p_g; mixed tiles: min of 2 v + p; the stand-in tile of an odd count never wins -- equals the
//     direct min over the mixture's entries of 2 dot + Q (the key of BatchIntFeatureScorer / SimdFeatureScorer).
// Models: ragged, tiny, empty, all-even / all-odd-heavy and 160-density mixtures, D = 16 / 39 / 45 / 64.
// Prints "ok" and exits 0, or the first mismatch and exits 1.
#include "../../rasr_amd/csrc/gmm_prepare.hh"

#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace rasr_gmm;

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
        double s = 0;
        for (int i = 0; i < 12; ++i)
            s += uniform();
        return static_cast<float>(s - 6.0);
    }
};

int check(uint32_t nMix, const std::vector<uint32_t>& counts, uint32_t D, Flavor flavor, uint64_t seed, int kind) {
    Rng                   rng{seed};
    std::vector<uint32_t> off{0};
    for (uint32_t c : counts)
        off.push_back(off.back() + c);
    const uint32_t        N = off.back();
    std::vector<float>    means(static_cast<size_t>(N) * D), var(D);
    std::vector<uint32_t> dm(N), dc(N, 0), dens(N);
    std::vector<double>   logw(N);
    for (uint32_t k = 0; k < D; ++k)
        var[k] = 0.5f + std::fabs(rng.normal());
    for (uint32_t i = 0; i < N; ++i) {
        for (uint32_t k = 0; k < D; ++k)
            means[static_cast<size_t>(i) * D + k] = rng.normal();
        dm[i] = i;
        dens[i] = i;
        logw[i] = -0.1 - 3.0 * rng.uniform();
    }
    gmm_mixture_set ms{};
    ms.dimension           = D;
    ms.n_means             = N;
    ms.means               = means.data();
    ms.n_covariances       = 1;
    ms.variances           = var.data();
    ms.n_densities         = N;
    ms.density_mean        = dm.data();
    ms.density_covariance  = dc.data();
    ms.n_mixtures          = nMix;
    ms.mixture_offsets     = off.data();
    ms.mixture_densities   = dens.data();
    ms.mixture_log_weights = logw.data();
    PreparedQuantized p;
    const std::string err = prepareQuantized(ms, flavor, ShardRange{0, 0}, p, kind);
    if (!err.empty()) {
        std::printf("prepareQuantized: %s\n", err.c_str());
        return 1;
    }
    if (p.scoreOnly != kind) {
        std::printf("D=%u: the score-only layout %d was not used (%d)\n", D, kind, p.scoreOnly);
        return 1;
    }
    const Tiling& t  = p.tiling;
    const uint32_t Dp = p.paddedDimension;
    // Q and -a' per entry
    std::vector<int64_t> Q(N);
    std::vector<int32_t> an(static_cast<size_t>(N) * D);
    for (uint32_t x = 0; x < N; ++x) {
        int64_t ss = 0;
        for (uint32_t k = 0; k < D; ++k) {
            const int32_t v = 128 - static_cast<int32_t>(p.preparedMean[static_cast<size_t>(x) * Dp + k]);
            an[static_cast<size_t>(x) * D + k] = v;
            ss += static_cast<int64_t>(v) * v;
        }
        Q[x] = static_cast<int64_t>(p.constantWeight[x]) + ss;
    }
    // coverage and parity rules
    std::vector<int> seen(N, 0);
    const bool       slots = kind == kScoreOnlySlots;
    for (uint32_t m = 0; m < nMix; ++m) {
        const uint32_t w = p.mixOddMask[m], nc = slots ? t.mixTileOffset[m + 1] - t.mixTileOffset[m] : w >> 16,
                       er = slots ? 0u : (w >> 4) & 0xfffu;
        if (slots && (w >> 8) != 0) {
            std::printf("mixture %u: slot word %08x\n", m, w);
            return 1;
        }
        if (slots) {  // the tile count is the smallest that holds both parities (2 rows per class and tile)
            uint32_t nE = 0, nO = 0;
            for (uint32_t x = off[m]; x < off[m + 1]; ++x)
                (Q[x] & 1 ? nO : nE) += 1;
            const auto fits = [&](uint32_t T) {
                for (uint32_t e = 0; e <= 8; ++e)
                    if (2 * e * T >= nE && 2 * (8 - e) * T >= nO)
                        return true;
                return false;
            };
            const uint32_t T = nc, ev = static_cast<uint32_t>(__builtin_popcount(~w & 0xffu));
            if (!fits(T) || (T > 0 && fits(T - 1)) || 2 * ev * T < nE || 2 * (8 - ev) * T < nO) {
                std::printf("mixture %u: %u tiles for %u even / %u odd rows (%u even classes)\n", m, T, nE, nO, ev);
                return 1;
            }
        }
        const uint32_t t0 = t.mixTileOffset[m], t1 = t.mixTileOffset[m + 1];
        if (t0 + nc > t1) {
            std::printf("mixture %u: %u class tiles of %u\n", m, nc, t1 - t0);
            return 1;
        }
        for (uint32_t tile = t0; tile < t1; ++tile)
            for (uint32_t r = 0; r < kTileRows; ++r) {
                const uint32_t x = t.rowEntry[static_cast<size_t>(tile) * kTileRows + r];
                const int32_t  h = p.tileP[static_cast<size_t>(tile) * kTileRows + r];
                if (x == UINT32_MAX) {
                    if (h != 0x30000000) {
                        std::printf("mixture %u tile %u row %u: padding constant %d\n", m, tile, r, h);
                        return 1;
                    }
                    continue;
                }
                if (x < off[m] || x >= off[m + 1] || seen[x]++) {
                    std::printf("mixture %u: entry %u misplaced or repeated\n", m, x);
                    return 1;
                }
                const uint32_t par = static_cast<uint32_t>(Q[x] & 1);
                const uint32_t want = slots ? (w >> (2 * (r / 4) + (r & 1))) & 1u
                                            : tile < t0 + nc ? (w >> (r / 4)) & 1u
                                                             : ((tile - t0 - nc) * 16 + r >= er ? 1u : 0u);
                if (par != want || h != static_cast<int32_t>(Q[x] >> 1)) {
                    std::printf("mixture %u tile %u row %u: parity %u, expected %u (h %d)\n", m, tile, r, par, want, h);
                    return 1;
                }
            }
    }
    for (uint32_t x = 0; x < N; ++x)
        if (!seen[x]) {
            std::printf("entry %u not placed\n", x);
            return 1;
        }
    // the kernel's minimum against the direct one, on random frames b' in [-128, 127]
    std::vector<int32_t> b(Dp);
    for (int f = 0; f < 24; ++f) {
        for (uint32_t k = 0; k < Dp; ++k)
            b[k] = k < D ? static_cast<int32_t>(rng.next() % 256) - 128 : 0;
        if (f == 0)
            for (uint32_t k = 0; k < D; ++k)
                b[k] = 127;  // the extreme frame
        for (uint32_t m = 0; m < nMix; ++m) {
            int64_t direct = INT64_MAX;
            for (uint32_t x = off[m]; x < off[m + 1]; ++x) {
                int64_t dot = 0;
                for (uint32_t k = 0; k < D; ++k)
                    dot += static_cast<int64_t>(an[static_cast<size_t>(x) * D + k]) * b[k];
                direct = std::min(direct, 2 * dot + Q[x]);
            }
            const uint32_t w = p.mixOddMask[m], nc = w >> 16, er = (w >> 4) & 0xfffu;
            const uint32_t t0 = t.mixTileOffset[m], t1 = t.mixTileOffset[m + 1];
            int64_t        kern = INT64_MAX;
            if (slots) {  // scoreI8Cls: per register (g, s) the min of dot + h over rows 4g + s, 4g + s + 2 of every tile
                for (uint32_t c = 0; c < 8; ++c) {
                    int64_t vmin = 0x3fffffff;
                    for (uint32_t tile = t0; tile < t1; ++tile)
                        for (uint32_t r = 4 * (c / 2) + c % 2; r < 4 * (c / 2) + 4; r += 2) {
                            int64_t dot = 0;
                            for (uint32_t k = 0; k < D; ++k) {
                                const uint32_t lane = (k / 16) * 16 + r, j = k % 16;
                                dot += static_cast<int64_t>(p.tileA[(static_cast<size_t>(tile) * kLanes + lane) * 16 + j]) * b[k];
                            }
                            vmin = std::min(vmin, dot + p.tileP[static_cast<size_t>(tile) * kTileRows + r]);
                        }
                    kern = std::min(kern, 2 * vmin + ((w >> c) & 1u));
                }
                if (off[m] != off[m + 1] && kern != direct) {
                    std::printf("slots D=%u mixture %u (%u entries) frame %d: kernel %lld, direct %lld\n", D, m,
                                off[m + 1] - off[m], f, static_cast<long long>(kern), static_cast<long long>(direct));
                    return 1;
                }
                continue;
            }
            for (uint32_t g = 0; g < 4; ++g) {  // one lane group: its class minimum in the v domain
                int64_t vmin = 0x3fffffff;
                for (uint32_t tile = t0; tile < t0 + nc; ++tile)
                    for (uint32_t r = 4 * g; r < 4 * g + 4; ++r) {
                        int64_t dot = 0;
                        for (uint32_t k = 0; k < D; ++k) {
                            const uint32_t lane = (k / 16) * 16 + r, j = k % 16;
                            dot += static_cast<int64_t>(p.tileA[(static_cast<size_t>(tile) * kLanes + lane) * 16 + j]) * b[k];
                        }
                        vmin = std::min(vmin, dot + p.tileP[static_cast<size_t>(tile) * kTileRows + r]);
                    }
                kern = std::min(kern, 2 * vmin + ((w >> g) & 1u));
            }
            for (uint32_t tile = t0 + nc; tile < t1; ++tile)
                for (uint32_t r = 0; r < kTileRows; ++r) {
                    int64_t dot = 0;
                    for (uint32_t k = 0; k < D; ++k) {
                        const uint32_t lane = (k / 16) * 16 + r, j = k % 16;
                        dot += static_cast<int64_t>(p.tileA[(static_cast<size_t>(tile) * kLanes + lane) * 16 + j]) * b[k];
                    }
                    const uint32_t R = (tile - t0 - nc) * 16 + r;
                    kern = std::min(kern, 2 * (dot + p.tileP[static_cast<size_t>(tile) * kTileRows + r]) + (R >= er ? 1 : 0));
                }
            if (off[m] == off[m + 1])
                continue;  // empty mixture: the kernel's emit reports Core::Type<int>::max
            if (kern != direct) {
                std::printf("D=%u mixture %u (%u entries) frame %d: kernel %lld, direct %lld\n", D, m, off[m + 1] - off[m], f,
                            static_cast<long long>(kern), static_cast<long long>(direct));
                return 1;
            }
        }
    }
    return 0;
}
}  // namespace

int main() {
    Rng rng{99};
    for (uint32_t D : {16u, 39u, 45u, 64u}) {
        std::vector<uint32_t> ragged, tiny, big;
        for (int m = 0; m < 120; ++m)
            ragged.push_back(1 + static_cast<uint32_t>(rng.next() % 300));
        for (int m = 0; m < 200; ++m)
            tiny.push_back(static_cast<uint32_t>(rng.next() % 10));
        for (int m = 0; m < 60; ++m)
            big.push_back(160);
        for (int kind : {kScoreOnlyClass, kScoreOnlySlots})
            for (Flavor fl : {Flavor::Simd, Flavor::BatchInt})
                for (const auto* c : {&ragged, &tiny, &big})
                    if (check(static_cast<uint32_t>(c->size()), *c, D, fl, D * 7 + c->size(), kind) != 0)
                        return 1;
    }

    std::printf("ok\n");
    return 0;
}
