// gmm_prepare.cc -- host-side model preparation (see gmm_prepare.hh).
//
// Every scalar formula below restates the reference expression as the
// reference binary computes it: built with -O2 -ffast-math -msse3
// (config/cc-gcc.make, config/proc-x86_64.make), GCC turns some of them into
// specific instruction sequences (rsqrtss + Newton-Raphson for 1/sqrt, an
// add-0.49999997-and-truncate for round, a float division for the quantization
// scale).  They are written out explicitly here so this file gives the same
// bits whatever flags it is compiled with.
#include "gmm_prepare.hh"

#include <xmmintrin.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>

namespace rasr_gmm {

// ---------------------------------------------------------------------------
// scalar arithmetic
// ---------------------------------------------------------------------------

// inverseSquareRoot<f32> (src/Mm/Utilities.hh:87-91) compiled with -ffast-math:
//   y = rsqrtss(x); r = ((x*y)*y + -3) * (y * -0.5)
// rsqrtss is the host CPU's own approximation, exactly as in the reference binary.
float refInverseSqrt(float x) {
    __m128 vx = _mm_set_ss(x);
    __m128 y  = _mm_rsqrt_ss(vx);
    __m128 t  = _mm_mul_ss(_mm_mul_ss(vx, y), y);
    __m128 u  = _mm_mul_ss(y, _mm_set_ss(-0.5f));
    t         = _mm_add_ss(t, _mm_set_ss(-3.0f));
    return _mm_cvtss_f32(_mm_mul_ss(t, u));
}

// (s32)float with x86 cvttss2si semantics: truncation, 0x80000000 when out of range / NaN.
int32_t refTruncF32(float x) {
    if (!(std::fabs(x) < 2147483648.0f))
        return std::numeric_limits<int32_t>::min();
    return static_cast<int32_t>(x);
}

int32_t refTruncF64(double x) {
    if (!(x > -2147483649.0 && x < 2147483648.0))
        return std::numeric_limits<int32_t>::min();
    return static_cast<int32_t>(x);
}

// (int)round(x), src/Mm/Utilities.hh:189, as built: t = x + copysign(nextbelow(0.5), x); cvttss2si(t).
int32_t refRoundToInt(float x) {
    const float h = std::copysign(0x1.fffffep-2f, x);  // 0.49999997f
    return refTruncF32(x + h);
}

// quantize<f32,u8>::operator() (Utilities.hh:186-190): clip((int)round(x) + 128) to [0,255].
// The +128 is a 32-bit wrapping add in the reference binary.
uint8_t refQuantize(float x) {
    int32_t v = static_cast<int32_t>(static_cast<uint32_t>(refRoundToInt(x)) + 128u);
    if (v > 255)
        v = 255;
    if (v < 0)
        v = 0;
    return static_cast<uint8_t>(v);
}

// gaussLogNormFactor (Utilities.hh:55-76): D*log(2 pi) + sum log|v| in double, in order.
// log(2 pi) is the constant GCC folds at compile time.
double refGaussLogNorm(const float* var, uint32_t d) {
    double result = 0;
    for (uint32_t i = 0; i < d; ++i)
        result += std::log(static_cast<double>(std::fabs(var[i])));
    return static_cast<double>(d) * 0x1.d67f1c864beb4p+0 + result;
}

// quantizationScalingFactor (SimdFeatureScorer.cc:128-133), as built: 255/(1.25*2*m) folds to
// the single-precision division 102.0f / m.
float refQuantizationScalingFactor(float minv, float maxv) {
    float a = std::fabs(minv), b = std::fabs(maxv);
    float m = a < b ? b : a;
    return 102.0f / m;
}

// ---------------------------------------------------------------------------
// validation and tiling
// ---------------------------------------------------------------------------

std::string validate(const gmm_mixture_set& ms) {
    if (ms.dimension == 0)
        return "dimension must be > 0";
    if (!ms.means || !ms.variances || !ms.density_mean || !ms.density_covariance || !ms.mixture_offsets ||
        (!ms.mixture_densities && ms.n_mixtures && ms.mixture_offsets[ms.n_mixtures]) ||
        (!ms.mixture_log_weights && ms.n_mixtures && ms.mixture_offsets[ms.n_mixtures]))
        return "null table in mixture set";
    if (ms.n_covariances == 0)
        return "mixture set has no covariance";
    if (ms.mixture_offsets[0] != 0)
        return "mixture_offsets[0] must be 0";
    for (uint32_t m = 0; m < ms.n_mixtures; ++m)
        if (ms.mixture_offsets[m + 1] < ms.mixture_offsets[m])
            return "mixture_offsets must be non-decreasing";
    const uint32_t nEntries = ms.mixture_offsets[ms.n_mixtures];
    for (uint32_t e = 0; e < nEntries; ++e)
        if (ms.mixture_densities[e] >= ms.n_densities)
            return "mixture entry references a density out of range";
    for (uint32_t i = 0; i < ms.n_densities; ++i) {
        if (ms.density_mean[i] >= ms.n_means)
            return "density references a mean out of range";
        if (ms.density_covariance[i] >= ms.n_covariances)
            return "density references a covariance out of range";
    }
    // require(checkDiagonal(diagonal)) -- CovarianceFeatureScorerElement.cc:26,38-42
    for (size_t i = 0; i < static_cast<size_t>(ms.n_covariances) * ms.dimension; ++i)
        if (!(ms.variances[i] > 0))
            return "covariance diagonal must be > 0";
    return "";
}

static void buildTiling(const gmm_mixture_set& ms, ShardRange shard, Tiling& t, uint32_t rows = kTileRows,
                        bool groupByCovariance = true) {
    const uint32_t nMix = shard.end - shard.begin;
    t.mixTileOffset.assign(nMix + 1, 0);
    t.tileCovariance.clear();
    t.rowEntry.clear();
    t.rowDensityInMixture.clear();
    t.maxEntriesPerMixture = 0;
    t.rows                 = rows;
    std::vector<uint32_t> order;
    for (uint32_t mi = 0; mi < nMix; ++mi) {
        const uint32_t m = shard.begin + mi;
        const uint32_t b = ms.mixture_offsets[m], e = ms.mixture_offsets[m + 1];
        t.maxEntriesPerMixture = std::max(t.maxEntriesPerMixture, e - b);
        order.resize(e - b);
        std::iota(order.begin(), order.end(), b);
        // group rows by covariance (one frame-side operand per tile); stable keeps entry order.  Without grouping
        // (the covariance-free split layout) a tile takes 16 consecutive entries whatever their covariances
        if (groupByCovariance)
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
                return ms.density_covariance[ms.mixture_densities[x]] < ms.density_covariance[ms.mixture_densities[y]];
            });
        size_t i = 0;
        while (i < order.size()) {
            const uint32_t cov = ms.density_covariance[ms.mixture_densities[order[i]]];
            size_t         j   = i;
            while (j < order.size() && (!groupByCovariance || ms.density_covariance[ms.mixture_densities[order[j]]] == cov))
                ++j;
            for (size_t r0 = i; r0 < j; r0 += rows) {
                t.tileCovariance.push_back(cov);
                for (uint32_t r = 0; r < rows; ++r) {
                    if (r0 + r < j) {
                        t.rowEntry.push_back(order[r0 + r]);
                        t.rowDensityInMixture.push_back(order[r0 + r] - b);
                    }
                    else {
                        t.rowEntry.push_back(UINT32_MAX);
                        t.rowDensityInMixture.push_back(UINT32_MAX);
                    }
                }
            }
            i = j;
        }
        t.mixTileOffset[mi + 1] = static_cast<uint32_t>(t.tileCovariance.size());
    }
    t.nTiles = static_cast<uint32_t>(t.tileCovariance.size());
}

static ShardRange normalizeShard(const gmm_mixture_set& ms, ShardRange s) {
    if (s.begin == 0 && s.end == 0)
        return ShardRange{0, ms.n_mixtures};
    return s;
}

// ---------------------------------------------------------------------------
// quantized scorers: SIMD-diagonal-maximum, batch-diagonal-maximum-int
// ---------------------------------------------------------------------------

// Score-only class layout (PreparedQuantized::scoreOnly).  A mixture's tiles are `nc` class tiles followed by
// mixed tiles.  In a class tile the entries with even and odd Q = c + sum a'^2 sit in disjoint lane groups (k
// groups even, 4 - k odd, the same k for all class tiles of the mixture: lane group g's parity is bit g of the
// mixture's word), so the kernel keeps min(dot + h) there with one v_min3 per two candidates.  The entries the
// class tiles leave over go to the mixed tiles, evens first, in row order (row 4g + r of mixed tile i is entry
// 16 i + 4g + r of that remainder, odd from index `er` on), where the kernel forms 2 (dot + h) + p per candidate.
// (k, nc) minimise the cost of the mixture's pair steps (a pair step never mixes a class and a mixed tile; an
// odd count ends on the never-winning stand-in tile), a mixed step counted kMixedCost class steps.  Every row
// carries h = Q >> 1 (the MFMA's C input) and -a'.  Padding rows carry kClassPadC (never below a real row's
// value, and 2 v + 1 stays inside int32).  Word of mixture m: bits 0-3 the odd lane groups of its class
// tiles, bits 4-15 er, bits 16-31 nc.
static constexpr int32_t kClassPadC  = 0x30000000;
static constexpr int64_t kClassLimit = int64_t(1) << 29;  // |2 dot + Q| bound of a real row
static constexpr double  kMixedCost  = 1.25;               // a mixed pair step against a class pair step

// false: some row's |2 dot + Q| may reach kClassLimit; the key layout is used instead
static bool classLayoutFits(const gmm_mixture_set& ms, ShardRange shard, const PreparedQuantized& out) {
    const uint32_t D = out.dimension, Dp = out.paddedDimension;
    for (uint32_t m = shard.begin; m < shard.end; ++m)
        if (ms.mixture_offsets[m + 1] - ms.mixture_offsets[m] > 16u * 65535u)
            return false;  // the class tile count needs 16 bits of the mixture word
    for (uint32_t x = ms.mixture_offsets[shard.begin]; x < ms.mixture_offsets[shard.end]; ++x) {
        const uint8_t* pm    = out.preparedMean.data() + static_cast<size_t>(x) * Dp;
        int64_t        sumSq = 0, sumAbs = 0;
        for (uint32_t k = 0; k < D; ++k) {
            const int64_t an = 128 - static_cast<int32_t>(pm[k]);
            if (an > 127)
                return false;  // mean quantized to 0: not an s8 operand (the key layout reports it)
            sumSq += an * an;
            sumAbs += an < 0 ? -an : an;
        }
        const int64_t q = static_cast<int64_t>(out.constantWeight[x]) + sumSq;
        if ((q < 0 ? -q : q) + 2 * 128 * sumAbs >= kClassLimit)
            return false;
    }
    return true;
}

// the (k, nc) of a mixture with nE even and nO odd entries (ClassPlan::er: even entries left for mixed tiles)
struct ClassPlan {
    uint32_t k = 2, nc = 0, nm = 0, er = 0;
};

static ClassPlan planClassTiles(uint32_t nE, uint32_t nO) {
    ClassPlan best;
    double    bestCost = 1e300;
    for (uint32_t k = 0; k <= 4; ++k) {
        const uint32_t ce = 4 * k, co = 4 * (4 - k);
        // class tiles beyond the point where both classes are used up only add padding
        const uint32_t ncMax = std::max(ce ? (nE + ce - 1) / ce : 0u, co ? (nO + co - 1) / co : 0u);
        for (uint32_t nc = 0; nc <= ncMax; ++nc) {
            const uint32_t er = nE - std::min(nE, ce * nc), orr = nO - std::min(nO, co * nc);
            const uint32_t nm   = (er + orr + 15) / 16;
            const double   cost = (nc + 1) / 2 + kMixedCost * ((nm + 1) / 2) + 1e-3 * nm;  // ties: fewer mixed tiles
            if (cost < bestCost)
                bestCost = cost, best = ClassPlan{k, nc, nm, er};
        }
    }
    return best;
}

static std::string buildClassLayout(const gmm_mixture_set& ms, ShardRange shard, PreparedQuantized& out) {
    const uint32_t D = out.dimension, Dp = out.paddedDimension, nMix = shard.end - shard.begin;
    Tiling&        t = out.tiling;
    t                = Tiling();
    t.mixTileOffset.assign(nMix + 1, 0);
    out.mixOddMask.assign(nMix, 0);
    out.tileA.clear();
    out.tileP.clear();
    std::vector<uint32_t> cls[2], rest;
    for (uint32_t mi = 0; mi < nMix; ++mi) {
        const uint32_t m = shard.begin + mi;
        const uint32_t b = ms.mixture_offsets[m], e = ms.mixture_offsets[m + 1];
        t.maxEntriesPerMixture = std::max(t.maxEntriesPerMixture, e - b);
        cls[0].clear();
        cls[1].clear();
        std::vector<int64_t> qOf(e - b);
        for (uint32_t x = b; x < e; ++x) {
            const uint8_t* pm    = out.preparedMean.data() + static_cast<size_t>(x) * Dp;
            int64_t        sumSq = 0;
            for (uint32_t k = 0; k < D; ++k) {
                const int64_t an = 128 - static_cast<int32_t>(pm[k]);
                sumSq += an * an;
            }
            qOf[x - b] = static_cast<int64_t>(out.constantWeight[x]) + sumSq;
            cls[static_cast<uint64_t>(qOf[x - b]) & 1u].push_back(x);
        }
        const uint32_t  nE = static_cast<uint32_t>(cls[0].size()), nO = static_cast<uint32_t>(cls[1].size());
        const ClassPlan pl = nE + nO ? planClassTiles(nE, nO) : ClassPlan{2, 0, 0, 0};
        if (pl.er > 0xfffu || pl.nc > 0xffffu)
            return "class layout: mixture too large for the mixture word";
        const uint32_t k = pl.k, tiles = pl.nc + pl.nm;
        out.mixOddMask[mi] = ((0xfu << k) & 0xfu) | (pl.er << 4) | (pl.nc << 16);
        const uint32_t t0 = t.nTiles;
        t.nTiles += tiles;
        out.tileA.resize(static_cast<size_t>(t.nTiles) * kLanes * 16, 0);
        out.tileP.resize(static_cast<size_t>(t.nTiles) * kTileRows, kClassPadC);
        t.rowEntry.resize(static_cast<size_t>(t.nTiles) * kTileRows, UINT32_MAX);
        t.rowDensityInMixture.resize(static_cast<size_t>(t.nTiles) * kTileRows, UINT32_MAX);
        t.tileCovariance.resize(t.nTiles, 0);
        const auto place = [&](uint32_t x, uint32_t tile, uint32_t r) {  // row r (4g + j) of tile
            const uint8_t* pm = out.preparedMean.data() + static_cast<size_t>(x) * Dp;
            for (uint32_t kk = 0; kk < D; ++kk) {
                const int32_t  an   = 128 - static_cast<int32_t>(pm[kk]);
                const uint32_t lane = (kk / 16) * 16 + r, j = kk % 16;  // one K step: kk < 64
                out.tileA[(static_cast<size_t>(tile) * kLanes + lane) * 16 + j] = static_cast<int8_t>(an);
            }
            out.tileP[static_cast<size_t>(tile) * kTileRows + r] = static_cast<int32_t>(qOf[x - b] >> 1);  // floor
            t.rowEntry[static_cast<size_t>(tile) * kTileRows + r]            = x;
            t.rowDensityInMixture[static_cast<size_t>(tile) * kTileRows + r] = x - ms.mixture_offsets[shard.begin + mi];
        };
        rest.clear();
        for (int c = 0; c < 2; ++c) {
            const uint32_t g0 = c ? k : 0, ng = c ? 4 - k : k;  // lane groups of the class
            const size_t   cap = static_cast<size_t>(4) * ng * pl.nc;
            for (size_t i = 0; i < cls[c].size(); ++i) {
                if (i >= cap) {
                    rest.push_back(cls[c][i]);  // evens first: c = 0 is placed before c = 1
                    continue;
                }
                const uint32_t tile = t0 + static_cast<uint32_t>(i / (4 * ng));
                const uint32_t slot = static_cast<uint32_t>(i % (4 * ng));
                place(cls[c][i], tile, 4 * (g0 + slot / 4) + slot % 4);  // rows 4g..4g+3 belong to lane group g
            }
        }
        for (size_t i = 0; i < rest.size(); ++i)
            place(rest[i], t0 + pl.nc + static_cast<uint32_t>(i / 16), static_cast<uint32_t>(i % 16));
        t.mixTileOffset[mi + 1] = t.nTiles;
    }
    out.idxBits   = 0;
    out.scoreOnly = kScoreOnlyClass;
    return "";
}

// Slot layout (kScoreOnlySlots: calls without best densities, preselection aside).  The 16 rows of a tile form 8
// classes (g, s) -- rows 4g + s and 4g + s + 2, the rows that lane group g's running-minimum register s collects
// in scoreI8Cls.  Every tile of a mixture gives class (g, s) the same parity of Q = c + sum a'^2 (bit 2g + s of the
// mixture word: odd), so the kernel keeps min(v = dot + h) per register, one v_min3 per two candidates in every
// tile, and forms 2 v + p once, at the mixture end.  With e even classes (the classes 0 .. e-1 in the order 2g + s)
// a tile holds 2e even and 2(8 - e) odd rows; T is the smallest tile count that holds the mixture's nE even and nO
// odd rows, e an even number where one fits (both registers of a lane group then share the parity: the kernel's
// cheaper emit).  No mixed tiles: in exchange for their per-candidate 2 v + p, a mixture may need one tile more
// (11 instead of 10 at 160 densities).  Unused rows carry kClassPadC and zero operands.
static std::string buildSlotLayout(const gmm_mixture_set& ms, ShardRange shard, PreparedQuantized& out) {
    const uint32_t D = out.dimension, Dp = out.paddedDimension, nMix = shard.end - shard.begin;
    Tiling&        t = out.tiling;
    t                = Tiling();
    t.mixTileOffset.assign(nMix + 1, 0);
    out.mixOddMask.assign(nMix, 0);
    out.tileA.clear();
    out.tileP.clear();
    std::vector<uint32_t> cls[2];
    std::vector<int64_t>  qOf;
    for (uint32_t mi = 0; mi < nMix; ++mi) {
        const uint32_t m = shard.begin + mi;
        const uint32_t b = ms.mixture_offsets[m], e = ms.mixture_offsets[m + 1];
        t.maxEntriesPerMixture = std::max(t.maxEntriesPerMixture, e - b);
        cls[0].clear();
        cls[1].clear();
        qOf.assign(e - b, 0);
        for (uint32_t x = b; x < e; ++x) {
            const uint8_t* pm    = out.preparedMean.data() + static_cast<size_t>(x) * Dp;
            int64_t        sumSq = 0;
            for (uint32_t k = 0; k < D; ++k) {
                const int64_t an = 128 - static_cast<int32_t>(pm[k]);
                sumSq += an * an;
            }
            qOf[x - b] = static_cast<int64_t>(out.constantWeight[x]) + sumSq;
            cls[static_cast<uint64_t>(qOf[x - b]) & 1u].push_back(x);
        }
        const uint32_t nE = static_cast<uint32_t>(cls[0].size()), nO = static_cast<uint32_t>(cls[1].size());
        uint32_t       T = (nE + nO + 15) / 16, ev = 0;
        for (;; ++T) {  // smallest T, then an even e if one fits
            int pick = -1;
            for (uint32_t c = 0; c <= 8; ++c)
                if (2 * c * T >= nE && 2 * (8 - c) * T >= nO && (pick < 0 || (pick & 1)))
                    pick = static_cast<int>(c);
            if (pick >= 0 || nE + nO == 0) {
                ev = pick < 0 ? 8 : static_cast<uint32_t>(pick);
                break;
            }
        }
        out.mixOddMask[mi] = (0xffu << ev) & 0xffu;
        const uint32_t t0 = t.nTiles;
        t.nTiles += T;
        out.tileA.resize(static_cast<size_t>(t.nTiles) * kLanes * 16, 0);
        out.tileP.resize(static_cast<size_t>(t.nTiles) * kTileRows, kClassPadC);
        t.rowEntry.resize(static_cast<size_t>(t.nTiles) * kTileRows, UINT32_MAX);
        t.rowDensityInMixture.resize(static_cast<size_t>(t.nTiles) * kTileRows, UINT32_MAX);
        t.tileCovariance.resize(t.nTiles, 0);
        for (int p = 0; p < 2; ++p) {
            const uint32_t c0 = p ? ev : 0, nc = p ? 8 - ev : ev;  // the classes of this parity
            for (size_t i = 0; i < cls[p].size(); ++i) {
                const uint32_t x = cls[p][i];
                // tile by tile: the class's 2 rows, class after class
                const uint32_t tile = t0 + static_cast<uint32_t>(i / (2 * nc));
                const uint32_t c = c0 + static_cast<uint32_t>(i % (2 * nc)) / 2, j = static_cast<uint32_t>(i % 2);
                const uint32_t r = 4 * (c >> 1) + (c & 1) + 2 * j;  // row 4g + s + 2j
                const uint8_t* pm = out.preparedMean.data() + static_cast<size_t>(x) * Dp;
                for (uint32_t kk = 0; kk < D; ++kk) {
                    const int32_t  an   = 128 - static_cast<int32_t>(pm[kk]);
                    const uint32_t lane = (kk / 16) * 16 + r, jj = kk % 16;  // one K step: kk < 64
                    out.tileA[(static_cast<size_t>(tile) * kLanes + lane) * 16 + jj] = static_cast<int8_t>(an);
                }
                out.tileP[static_cast<size_t>(tile) * kTileRows + r]            = static_cast<int32_t>(qOf[x - b] >> 1);
                t.rowEntry[static_cast<size_t>(tile) * kTileRows + r]            = x;
                t.rowDensityInMixture[static_cast<size_t>(tile) * kTileRows + r] = x - b;
            }
        }
        t.mixTileOffset[mi + 1] = t.nTiles;
    }
    out.idxBits   = 0;
    out.scoreOnly = kScoreOnlySlots;
    return "";
}

std::string prepareQuantized(const gmm_mixture_set& ms, Flavor flavor, ShardRange shard, PreparedQuantized& out,
                             int scoreOnlyLayout) {
    std::string err = validate(ms);
    if (!err.empty())
        return err;
    shard = normalizeShard(ms, shard);
    if (shard.begin > shard.end || shard.end > ms.n_mixtures)
        return "invalid mixture shard";
    const uint32_t D = ms.dimension, C = ms.n_covariances;
    if (flavor == Flavor::BatchInt && C != 1)
        return "feature scorer supports only globally pooled variance";  // BatchFeatureScorer.cc:341-343
    if (D > 2 * kI8K)
        return "quantized scorer supports dimension <= 128";
    out            = PreparedQuantized();
    out.flavor     = flavor;
    out.dimension  = D;
    out.paddedDimension = (D + 15u) / 16u * 16u;  // IntelOptimization.hh:51-58 (BlockSize 16)
    out.nCovariances = C;
    out.nMixtures  = shard.end - shard.begin;
    out.kSteps     = (D + kI8K - 1) / kI8K;

    // CovarianceFeatureScorerElement::operator= (CovarianceFeatureScorerElement.cc:20-36)
    std::vector<float> isv(static_cast<size_t>(C) * D);
    std::vector<float> logNorm(C);
    for (uint32_t c = 0; c < C; ++c) {
        const float* var = ms.variances + static_cast<size_t>(c) * D;
        for (uint32_t k = 0; k < D; ++k)
            isv[static_cast<size_t>(c) * D + k] = refInverseSqrt(var[k]);
        logNorm[c] = static_cast<float>(refGaussLogNorm(var, D));
    }

    // getScaling (SimdFeatureScorer.cc:106-126) / quantizationScale (BatchFeatureScorer.cc:318-336):
    // bounds of mean * isv over ALL densities of the mixture set (shards share one scale).
    float minMean = FLT_MAX, maxMean = -FLT_MAX;
    for (uint32_t i = 0; i < ms.n_densities; ++i) {
        const float* mean = ms.means + static_cast<size_t>(ms.density_mean[i]) * D;
        const float* iv   = isv.data() + static_cast<size_t>(ms.density_covariance[i]) * D;
        for (uint32_t k = 0; k < D; ++k) {
            float dm = mean[k] * iv[k];
            minMean  = std::min(minMean, dm);
            maxMean  = std::max(maxMean, dm);
        }
    }
    const float s             = refQuantizationScalingFactor(minMean, maxMean);
    out.scaling               = s;
    out.scalingSquared        = s * s;                         // cc:72
    out.inverseQuantizationFactor = 0.5f / out.scalingSquared; // cc:73
    out.batchScale            = static_cast<float>(2.0 * static_cast<double>(out.scalingSquared));  // cc:356

    // scale(s): isv *= s; logNorm *= s*s  (CovarianceFeatureScorerElement.cc:45-51, BatchFeatureScorer.cc:357-359)
    out.isvScaled.resize(isv.size());
    out.logNormScaled.resize(C);
    for (uint32_t c = 0; c < C; ++c) {
        for (uint32_t k = 0; k < D; ++k)
            out.isvScaled[static_cast<size_t>(c) * D + k] = isv[static_cast<size_t>(c) * D + k] * s;
        out.logNormScaled[c] = logNorm[c] * (s * s);
    }

    // reference tables per mixture entry: prepared mean (u8, 0-padded to Dp) and constant weight
    const uint32_t nEntries = ms.mixture_offsets[ms.n_mixtures];
    const uint32_t Dp       = out.paddedDimension;
    out.preparedMean.assign(static_cast<size_t>(nEntries) * Dp, 0);
    out.constantWeight.assign(nEntries, 0);
    for (uint32_t m = 0; m < ms.n_mixtures; ++m) {
        for (uint32_t e = ms.mixture_offsets[m]; e < ms.mixture_offsets[m + 1]; ++e) {
            const uint32_t dns  = ms.mixture_densities[e];
            const uint32_t cov  = ms.density_covariance[dns];
            const float*   mean = ms.means + static_cast<size_t>(ms.density_mean[dns]) * D;
            const float*   iv   = out.isvScaled.data() + static_cast<size_t>(cov) * D;
            for (uint32_t k = 0; k < D; ++k)
                out.preparedMean[static_cast<size_t>(e) * Dp + k] = refQuantize(mean[k] * iv[k]);
            const double lw = ms.mixture_log_weights[e];
            if (flavor == Flavor::Simd) {
                // SimdFeatureScorer.cc:96 + IntelOptimization.cc:47
                float w = static_cast<float>(static_cast<double>(out.scalingSquared * -2.0f) * lw);
                out.constantWeight[e] = refTruncF32(w + out.logNormScaled[cov]);
            }
            else {
                // BatchFeatureScorer.cc:376 (logNormFactor = logNorm * scaleSquared, cc:359)
                out.constantWeight[e] = refTruncF64(static_cast<double>(out.logNormScaled[cov]) -
                                                    static_cast<double>(out.batchScale) * lw);
            }
        }
    }

    out.isvDevice.assign(static_cast<size_t>(C) * out.kSteps * kI8K, 0.0f);
    for (uint32_t c = 0; c < C; ++c)
        for (uint32_t k = 0; k < D; ++k)
            out.isvDevice[static_cast<size_t>(c) * out.kSteps * kI8K + k] = out.isvScaled[static_cast<size_t>(c) * D + k];
    // a mixture whose plan does not fit the mixture word keeps the whole model on the key layout
    if (scoreOnlyLayout != kScoreOnlyNone && C == 1 && out.kSteps == 1 && classLayoutFits(ms, shard, out) &&
        (scoreOnlyLayout == kScoreOnlySlots ? buildSlotLayout(ms, shard, out) : buildClassLayout(ms, shard, out)).empty())
        return "";
    out.scoreOnly = kScoreOnlyNone;
    out.mixOddMask.clear();

    // device tiles
    buildTiling(ms, shard, out.tiling);
    uint32_t ib = 1;
    while ((1u << ib) < std::max<uint32_t>(out.tiling.maxEntriesPerMixture, 2u))
        ++ib;
    out.idxBits = ib;
    // packed = value * 2^ib + density must stay below the padding-row value.  With several
    // covariances the kernel adds the frame's sum (q-128)^2 << ib (<= D * 128^2) to every row,
    // padding rows included, so their constant leaves that much headroom.
    const uint32_t T      = out.tiling.nTiles;
    const uint32_t KS     = out.kSteps;
    const bool     multiC = C > 1;
    const int64_t  ssMax  = multiC ? static_cast<int64_t>(D) * 128 * 128 : 0;
    const int64_t  packedLimit = (static_cast<int64_t>(1) << (31 - ib)) - 2 - ssMax;
    if (packedLimit <= 0)
        return "mixtures too large for the packed (score, density) int32 encoding";
    const int32_t padRow = static_cast<int32_t>(static_cast<int64_t>(kPadRowPacked) - (ssMax << ib));
    out.tileA.assign(static_cast<size_t>(T) * KS * kLanes * 16, 0);
    out.tileP.assign(static_cast<size_t>(T) * kTileRows, padRow);
    for (uint32_t t = 0; t < T; ++t) {
        for (uint32_t r = 0; r < kTileRows; ++r) {
            const uint32_t e = out.tiling.rowEntry[static_cast<size_t>(t) * kTileRows + r];
            if (e == UINT32_MAX)
                continue;
            const uint8_t* pm     = out.preparedMean.data() + static_cast<size_t>(e) * Dp;
            int64_t        sumSq  = 0;
            int64_t        sumAbs = 0;
            for (uint32_t k = 0; k < D; ++k) {
                const int32_t an = 128 - static_cast<int32_t>(pm[k]);  // -(a - 128)
                sumSq += static_cast<int64_t>(an) * an;
                sumAbs += an < 0 ? -an : an;
                if (an < -128 || an > 127)
                    return "prepared mean outside the s8 operand range (mean quantized to 0)";
                // fragment order: k = ks*64 + 16*(lane>>4) + j, row = lane & 15
                const uint32_t ks = k / kI8K, kk = k % kI8K;
                const uint32_t lane = (kk / 16) * 16 + r, j = kk % 16;
                out.tileA[((static_cast<size_t>(t) * KS + ks) * kLanes + lane) * 16 + j] = static_cast<int8_t>(an);
            }
            const int64_t biasv = static_cast<int64_t>(out.constantWeight[e]) + sumSq;
            const int64_t bound = (biasv < 0 ? -biasv : biasv) + 2 * 128 * sumAbs + ssMax;
            if (bound > packedLimit)
                return "model outside the packed (score, density) int32 range; use fewer densities per mixture";
            const uint32_t dnsIdx = out.tiling.rowDensityInMixture[static_cast<size_t>(t) * kTileRows + r];
            out.tileP[static_cast<size_t>(t) * kTileRows + r] =
                    static_cast<int32_t>(biasv * (static_cast<int64_t>(1) << ib) + dnsIdx);
        }
    }
    return "";
}

// ---------------------------------------------------------------------------
// float scorers: diagonal-maximum, batch-diagonal-maximum-float
// ---------------------------------------------------------------------------

std::string prepareFloat(const gmm_mixture_set& ms, Flavor flavor, float mixtureWeightScale, float gaussianScale,
                         ShardRange shard, PreparedFloat& out, bool wantSplit, uint32_t splitRowsWanted) {
    std::string err = validate(ms);
    if (!err.empty())
        return err;
    shard = normalizeShard(ms, shard);
    if (shard.begin > shard.end || shard.end > ms.n_mixtures)
        return "invalid mixture shard";
    const uint32_t D = ms.dimension, C = ms.n_covariances;
    if (flavor == Flavor::BatchFloat && C != 1)
        return "feature scorer supports only globally pooled covariance";  // BatchFeatureScorer.cc:146-148
    if (D > 126)
        return "float scorer supports dimension <= 126";
    out              = PreparedFloat();
    out.flavor       = flavor;
    out.dimension    = D;
    out.nCovariances = C;
    out.nMixtures    = shard.end - shard.begin;
    out.foldNorm     = C > 1;
    const uint32_t kUsed = D + 1 + (out.foldNorm ? 1 : 0);
    out.kSteps       = f32KStepsInstantiated((kUsed + 3) / 4);

    // diagonal-maximum: covariance.scale(gaussianScale_ = sqrt(gaussian-scale)) (GDMFS.cc:51,83-84);
    // batch-float: unscaled (BatchFeatureScorer.cc:155-160).
    // diagonal-sum inherits init() from diagonal-maximum (GaussDiagonalMaximumFeatureScorer.hh:96)
    const bool  dm = flavor == Flavor::DiagonalMaximum || flavor == Flavor::DiagonalSum;
    const float gs = dm ? static_cast<float>(std::sqrt(static_cast<double>(gaussianScale))) : 1.0f;
    out.isv.resize(static_cast<size_t>(C) * D);
    out.logNorm.resize(C);
    for (uint32_t c = 0; c < C; ++c) {
        const float* var = ms.variances + static_cast<size_t>(c) * D;
        for (uint32_t k = 0; k < D; ++k) {
            float iv = refInverseSqrt(var[k]);
            out.isv[static_cast<size_t>(c) * D + k] = dm ? iv * gs : iv;
        }
        float ln      = static_cast<float>(refGaussLogNorm(var, D));
        out.logNorm[c] = dm ? ln * (gs * gs) : ln;
    }

    // centre of the expansion: the mean over all means of the set (not only the shard's, so every
    // shard of a model takes the same one)
    out.centre.assign(D, 0.0f);
    if (ms.n_means > 0)
        for (uint32_t k = 0; k < D; ++k) {
            double sum = 0;
            for (uint32_t i = 0; i < ms.n_means; ++i)
                sum += ms.means[static_cast<size_t>(i) * D + k];
            const float c = static_cast<float>(sum / ms.n_means);
            out.centre[k] = std::isfinite(c) ? c : 0.0f;
        }

    buildTiling(ms, shard, out.tiling);
    const uint32_t T = out.tiling.nTiles, KS = out.kSteps;

    // row constant c_d (everything but the distance)
    const auto rowConstant = [&](uint32_t e) -> double {
        const uint32_t cov = ms.density_covariance[ms.mixture_densities[e]];
        if (dm) {
            // minus2LogWeights_ (MixtureFeatureScorerElement.cc:26,30-33) + logNorm (GDMFS.cc:126-129)
            const float m2lw = static_cast<float>(-2 * ms.mixture_log_weights[e]) * mixtureWeightScale;
            return static_cast<double>(m2lw) + static_cast<double>(out.logNorm[cov]);
        }
        // BatchFeatureScorer.cc:167: constants = logNormFactor - 2 * logWeight (f32)
        return static_cast<float>(static_cast<double>(out.logNorm[cov]) - 2 * ms.mixture_log_weights[e]);
    };
    // Single covariance: the kernel keeps (value, tile) in one float whose low tileBits mantissa
    // bits hold the tile number, which orders correctly only for positive values.  A row's value
    // is ||x'-m'||^2 + c_d >= c_d, so shift every constant by K0 when some c_d < 1.
    out.offsetK0 = 0.0f;
    out.tileBits = 1;
    if (!out.foldNorm) {
        double minC = 1.0;
        for (uint32_t e : out.tiling.rowEntry)
            if (e != UINT32_MAX)
                minC = std::min(minC, rowConstant(e));
        if (minC < 1.0)
            out.offsetK0 = static_cast<float>(std::ceil(1.0 - minC));
        uint32_t maxTiles = 1;
        for (uint32_t m = 0; m < out.nMixtures; ++m)
            maxTiles = std::max(maxTiles, out.tiling.mixTileOffset[m + 1] - out.tiling.mixTileOffset[m]);
        while ((1u << out.tileBits) < maxTiles)
            ++out.tileBits;
        if (out.tileBits > 8)
            return "float scorer supports at most 4096 densities per mixture";  // key precision 2^-15
    }

    // one row of the contraction for entry e: m2[k] = -2 m'_k (f32, as the native kernel's operand)
    // and the row constant ||m'||^2 + c_d + K0 (f64); false for a padding row (e == UINT32_MAX)
    const auto entryValues = [&](uint32_t e, float* m2, double& cst) -> bool {
        if (e == UINT32_MAX)
            return false;
        const uint32_t dns  = ms.mixture_densities[e];
        const uint32_t cov  = ms.density_covariance[dns];
        const float*   mean = ms.means + static_cast<size_t>(ms.density_mean[dns]) * D;
        const float*   iv   = out.isv.data() + static_cast<size_t>(cov) * D;
        double         mm   = 0;
        for (uint32_t k = 0; k < D; ++k) {
            // (mu - c) isv in f64, one rounding to the f32 operand; the reference's own difference is
            // (mu - x) isv in f32 (GaussDiagonalMaximumFeatureScorer.cc:144-218)
            const float mp = static_cast<float>((static_cast<double>(mean[k]) - out.centre[k]) * iv[k]);
            m2[k]          = -2.0f * mp;
            mm += static_cast<double>(mp) * mp;
        }
        cst = mm + rowConstant(e) + out.offsetK0;
        return true;
    };
    const auto rowValues = [&](uint32_t t, uint32_t r, float* m2, double& cst) -> bool {
        return entryValues(out.tiling.rowEntry[static_cast<size_t>(t) * kTileRows + r], m2, cst);
    };
    std::vector<float> m2(D);
    double             cst = 0;

    // ---- split-f16 layout ----
    // Tile height: 16 rows (v_mfma_f32_16x16x32_f16, tile pairs, keys (tile << 2 | slot)) or 32 rows
    // (v_mfma_f32_32x32x16_f16, keys (tile << 4 | accumulator register)); keys drop at most 8 mantissa
    // bits (the reported score within 2^-16 relative), else the f32 kernel.  32 rows by default only
    // where their 16-wide K steps save a step over the 32-wide ones (e.g. D = 45: K 144 vs 160): the
    // chip holds a lower clock on the 32x32 shape (D = 39, K 128 both: 1.44 vs 1.38 ms).
    const auto bitsFor = [](uint32_t n) {
        uint32_t b = 1;
        while ((1u << b) < n)
            ++b;
        return b;
    };
    uint32_t maxEntries = 1;
    for (uint32_t m = 0; m < out.nMixtures; ++m)
        maxEntries = std::max(maxEntries, ms.mixture_offsets[shard.begin + m + 1] - ms.mixture_offsets[shard.begin + m]);
    const uint32_t keyBits32 = bitsFor((maxEntries + 31) / 32) + 4;
    const uint32_t keyBits16 = bitsFor(((maxEntries + 15) / 16 + 1) & ~1u) + 2;
    const bool     fits32    = keyBits32 <= 8 && splitKSteps32(D) <= kSplit32MaxKSteps;
    // 32-row tiles only where they save more K than the clock they cost: the 32x32x16 loop holds a lower clock
    // than the 16x16x32 one on this power-bound kernel (MI355X_MICROARCH.md DVFS item 7).  With 64-frame waves that
    // was ~1.15x the time per K column (D = 45: 5.90 vs 5.70 ms, profiles/r02/ab/ab_d45_shape.txt); with 128-frame
    // waves (round 5) the 32-row kernel is the faster one at D = 45 (5.308 vs 5.368 ms, K 144 vs 160, ~1.05x per
    // K column, profiles/r05/s20)
    const bool     saves32   = splitKSteps32(D) * 16 * 105 < splitKSteps(D) * 32 * 100;
    const bool     want32    = splitRowsWanted == 32 || (splitRowsWanted == 0 && saves32);
    // diagonal-sum: 32-row tiles wherever they fit (scoreSplit32Sum: its VALU-bound epilogue gets 1.5x the issue
    // cycles per unit of matrix work on the 32x32x16 shape), unless 16 rows are asked for (scoreSplitSum)
    const bool     sum32     = flavor == Flavor::DiagonalSum && splitRowsWanted != 16;
    const uint32_t rows      = (fits32 && (want32 || sum32 || keyBits16 > 8)) ? 32 : (keyBits16 <= 8 ? 16 : 0);
    if (wantSplit && !out.foldNorm && splitKSteps(D) <= 8 && T > 0 && rows != 0) {
        std::vector<double> maxAbs(D, 0.0);
        double              maxConst = 0;
        for (uint32_t e : out.tiling.rowEntry)
            if (entryValues(e, m2.data(), cst)) {
                for (uint32_t k = 0; k < D; ++k)
                    maxAbs[k] = std::max(maxAbs[k], std::fabs(static_cast<double>(m2[k])));
                maxConst = std::max(maxConst, std::fabs(cst));
            }
        // diagonal-sum adds every row of a mixture to its sum: padding rows (copies of a real row, which
        // never win a minimum) must not add, so their constant is raised by 2^29 (2^(-0.72 * 2^29)
        // underflows to 0 in the sum; the key never wins)
        const double padBias = flavor == Flavor::DiagonalSum ? std::ldexp(1.0, 29) : 0.0;
        maxConst += padBias;
        bool finite = std::isfinite(maxConst);
        for (double v : maxAbs)
            finite = finite && std::isfinite(v);
        // limbs at 2^b0, 2^(b0-11), 2^(b0-22), 2^(b0-33): f16 frame-side multipliers need
        // b0 <= 15 and b0 - 33 >= -24; limb 0 must hold const / 2^b0 <= 2^15
        int b0 = 9;
        while (b0 < 15 && maxConst / std::ldexp(1.0, b0) > 32768.0)
            ++b0;
        if (finite && maxConst / std::ldexp(1.0, b0) <= 32768.0) {
            out.split        = true;
            out.splitRows    = rows;
            out.kSteps16     = rows == 32 ? splitKSteps32(D) : splitKSteps(D);
            out.splitKeyBits = rows == 32 ? keyBits32 : keyBits16;
            // the split tiling; 16-row tiles: an even tile count per mixture (the kernel walks tile
            // pairs), a pad tile repeating row 0 of the mixture's first tile in every row (an exact tie
            // with a lower density index never wins)
            Tiling st;
            buildTiling(ms, shard, st, rows);
            std::vector<uint32_t> fillEntry(st.nTiles, UINT32_MAX);  // [tile] entry a padding row repeats
            for (uint32_t t = 0; t < st.nTiles; ++t)
                fillEntry[t] = st.rowEntry[static_cast<size_t>(t) * rows];
            if (rows == 16) {
                Tiling                pt;
                std::vector<uint32_t> pf;
                pt.rows                 = rows;
                pt.maxEntriesPerMixture = st.maxEntriesPerMixture;
                pt.mixTileOffset.assign(out.nMixtures + 1, 0);
                for (uint32_t m = 0; m < out.nMixtures; ++m) {
                    const uint32_t b = st.mixTileOffset[m], e = st.mixTileOffset[m + 1];
                    for (uint32_t t = b; t < e; ++t) {
                        pt.tileCovariance.push_back(st.tileCovariance[t]);
                        pf.push_back(fillEntry[t]);
                        pt.rowEntry.insert(pt.rowEntry.end(), st.rowEntry.begin() + static_cast<size_t>(t) * rows,
                                           st.rowEntry.begin() + static_cast<size_t>(t + 1) * rows);
                        pt.rowDensityInMixture.insert(pt.rowDensityInMixture.end(),
                                                      st.rowDensityInMixture.begin() + static_cast<size_t>(t) * rows,
                                                      st.rowDensityInMixture.begin() + static_cast<size_t>(t + 1) * rows);
                    }
                    if ((e - b) & 1u) {
                        pt.tileCovariance.push_back(st.tileCovariance[b]);
                        pf.push_back(fillEntry[b]);
                        pt.rowEntry.insert(pt.rowEntry.end(), rows, UINT32_MAX);
                        pt.rowDensityInMixture.insert(pt.rowDensityInMixture.end(), rows, UINT32_MAX);
                    }
                    pt.mixTileOffset[m + 1] = static_cast<uint32_t>(pt.tileCovariance.size());
                }
                pt.nTiles = static_cast<uint32_t>(pt.tileCovariance.size());
                st        = std::move(pt);
                fillEntry = std::move(pf);
            }
            out.tiling         = std::move(st);
            out.splitFillEntry = fillEntry;
            const uint32_t TP  = out.tiling.nTiles;
            for (uint32_t s = 0; s < kSplitLimbs; ++s)
                out.limbExp[s] = b0 - 11 * static_cast<int32_t>(s);
            // per-dimension power of two that puts max|m''_d| in [2^7, 2^8): m'' and x'' then sit in
            // the middle of the f16 range for frames of the model's own scale
            out.dimScale.assign(D, 1.0f);
            std::vector<double> inv(D, 1.0);
            for (uint32_t k = 0; k < D; ++k)
                if (maxAbs[k] > 0) {
                    int ex;
                    std::frexp(maxAbs[k], &ex);  // maxAbs in [2^(ex-1), 2^ex)
                    const int a     = std::max(-60, std::min(60, ex - 1 - 7));
                    out.dimScale[k] = static_cast<float>(std::ldexp(1.0, a));
                    inv[k]          = std::ldexp(1.0, -a);
                }
            const auto h16 = [](double v) {
                const _Float16 h = static_cast<_Float16>(v);  // round to nearest even, one rounding
                uint16_t       b;
                std::memcpy(&b, &h, 2);
                return b;
            };
            const auto f16v = [](uint16_t b) {
                _Float16 h;
                std::memcpy(&h, &b, 2);
                return static_cast<double>(h);
            };
            // K per tile row: kSteps16 steps of 32 (16-row tiles) or of 16 (32-row tiles)
            const uint32_t KW = out.kSteps16 * (rows == 32 ? 16 : 32);
            out.tileH.assign(static_cast<size_t>(TP) * rows * KW, 0);
            std::vector<uint16_t> row(KW);
            for (uint32_t t = 0; t < TP; ++t) {
                for (uint32_t r = 0; r < rows; ++r) {
                    std::fill(row.begin(), row.end(), 0);
                    // a padding row repeats row 0 of its tile (a pad tile: of its mixture's first tile)
                    const bool real = entryValues(out.tiling.rowEntry[static_cast<size_t>(t) * rows + r], m2.data(), cst);
                    if (real || entryValues(fillEntry[t], m2.data(), cst)) {
                        if (!real)
                            cst += padBias;
                        for (uint32_t k = 0; k < D; ++k) {
                            const float    v  = static_cast<float>(m2[k] * inv[k]);  // exact: power of two
                            const uint16_t hi = h16(v);
                            const uint16_t lo = h16(static_cast<double>(v) - f16v(hi));
                            row[k]            = hi;
                            row[D + k]        = hi;
                            row[2 * D + k]    = lo;
                        }
                        double rem = cst;
                        for (uint32_t s = 0; s < kSplitLimbs; ++s) {
                            const uint16_t l = h16(std::ldexp(rem, -out.limbExp[s]));
                            row[3 * D + s]   = l;
                            rem -= std::ldexp(f16v(l), out.limbExp[s]);
                        }
                        for (uint32_t s = 0; s < kSplitXXLimbs; ++s)
                            row[3 * D + kSplitLimbs + s] = h16(std::ldexp(1.0, kSplitXXExp[s]));
                    }
                    // fragment order: v_mfma_f32_16x16x32_f16 lane = 16*((k>>3)&3) + row, step k>>5;
                    // v_mfma_f32_32x32x16_f16 lane = 32*((k>>3)&1) + row, step k>>4
                    for (uint32_t k = 0; k < KW; ++k) {
                        const uint32_t lane = rows == 32 ? 32 * ((k >> 3) & 1) + r : 16 * ((k >> 3) & 3) + r;
                        const uint32_t step = rows == 32 ? k >> 4 : k >> 5;
                        out.tileH[((static_cast<size_t>(t) * out.kSteps16 + step) * kLanes + lane) * 8 + (k & 7)] = row[k];
                    }
                }
            }
        }
    }

    // ---- split-f16 layout for several covariances (round 6): the covariance-free expansion ----
    // With y = x - c (the frame about the centre), mu' = mu - c and w = isv^2 of the row's covariance,
    //     ||(x - mu) isv||^2 = sum_d w_d y_d^2 - 2 sum_d w_d mu'_d y_d + sum_d w_d mu'_d^2,
    // so one frame operand [y^2, y] serves every covariance (no C x frames buffers, no tiles split by covariance):
    // K = [0,D) wh Yh, [D,2D) wh Yl, [2D,3D) wl Yh, [3D,4D) nh zh, [4D,5D) nh zl, [5D,6D) nl zh, [6D,6D+4) the row
    // constant's limbs, where Y = y^2 2^a_d, z = y 2^b_d (frame side), w'' = w 2^-a_d, n'' = -2 w mu' 2^-b_d (model
    // side), the powers of two putting the model's largest |w''| and |n''| of a dimension in [2^7, 2^8).  Twice
    // the pooled layout's K (6 D + 4: 238 -> 256 at D = 39), on the same kernels (they are K-agnostic), against the
    // native f32 kernel's 1/16-rate MFMAs and per-covariance frame operands.
    const uint32_t keyBitsCov = bitsFor(((maxEntries + 15) / 16 + 1) & ~1u) + 2;
    if (wantSplit && out.foldNorm && splitCovKSteps(D) <= 8 && T > 0 && keyBitsCov <= 8) {
        Tiling st;
        buildTiling(ms, shard, st, 16, false);
        double minC = 1.0;
        for (uint32_t e : st.rowEntry)
            if (e != UINT32_MAX)
                minC = std::min(minC, rowConstant(e));
        const float k0 = minC < 1.0 ? static_cast<float>(std::ceil(1.0 - minC)) : 0.0f;
        // per row: w_d, n_d = -2 w_d mu'_d (f64) and the constant sum w mu'^2 + c_row + K0
        const auto covValues = [&](uint32_t e, double* w, double* n, double& c) -> bool {
            if (e == UINT32_MAX)
                return false;
            const uint32_t dns  = ms.mixture_densities[e];
            const uint32_t cov  = ms.density_covariance[dns];
            const float*   mean = ms.means + static_cast<size_t>(ms.density_mean[dns]) * D;
            const float*   iv   = out.isv.data() + static_cast<size_t>(cov) * D;
            double         mm   = 0;
            for (uint32_t k = 0; k < D; ++k) {
                const double wk = static_cast<double>(iv[k]) * iv[k];
                const double mp = static_cast<double>(mean[k]) - out.centre[k];
                w[k]            = wk;
                n[k]            = -2.0 * wk * mp;
                mm += wk * mp * mp;
            }
            c = mm + rowConstant(e) + k0;
            return true;
        };
        std::vector<double> wv(D), nv(D), maxW(D, 0.0), maxN(D, 0.0);
        double              cv = 0, maxConst = 0;
        for (uint32_t e : st.rowEntry)
            if (covValues(e, wv.data(), nv.data(), cv)) {
                for (uint32_t k = 0; k < D; ++k) {
                    maxW[k] = std::max(maxW[k], std::fabs(wv[k]));
                    maxN[k] = std::max(maxN[k], std::fabs(nv[k]));
                }
                maxConst = std::max(maxConst, std::fabs(cv));
            }
        const double padBias = flavor == Flavor::DiagonalSum ? std::ldexp(1.0, 29) : 0.0;
        maxConst += padBias;
        bool finite = std::isfinite(maxConst);
        for (uint32_t k = 0; k < D; ++k)
            finite = finite && std::isfinite(maxW[k]) && std::isfinite(maxN[k]);
        int b0 = 9;
        while (b0 < 15 && maxConst / std::ldexp(1.0, b0) > 32768.0)
            ++b0;
        if (finite && maxConst / std::ldexp(1.0, b0) <= 32768.0) {
            out.split        = true;
            out.splitCov     = true;
            out.splitRows    = 16;
            out.kSteps16     = splitCovKSteps(D);
            out.splitKeyBits = keyBitsCov;
            out.offsetK0     = k0;
            // an even tile count per mixture (the pair kernel), the pad tile repeating the mixture's first row
            std::vector<uint32_t> fillEntry;
            Tiling                pt;
            pt.rows                 = 16;
            pt.maxEntriesPerMixture = st.maxEntriesPerMixture;
            pt.mixTileOffset.assign(out.nMixtures + 1, 0);
            for (uint32_t m = 0; m < out.nMixtures; ++m) {
                const uint32_t b = st.mixTileOffset[m], e = st.mixTileOffset[m + 1];
                for (uint32_t t = b; t < e; ++t) {
                    pt.tileCovariance.push_back(st.tileCovariance[t]);
                    fillEntry.push_back(st.rowEntry[static_cast<size_t>(t) * 16]);
                    pt.rowEntry.insert(pt.rowEntry.end(), st.rowEntry.begin() + static_cast<size_t>(t) * 16,
                                       st.rowEntry.begin() + static_cast<size_t>(t + 1) * 16);
                    pt.rowDensityInMixture.insert(pt.rowDensityInMixture.end(),
                                                  st.rowDensityInMixture.begin() + static_cast<size_t>(t) * 16,
                                                  st.rowDensityInMixture.begin() + static_cast<size_t>(t + 1) * 16);
                }
                if ((e - b) & 1u) {
                    pt.tileCovariance.push_back(st.tileCovariance[b]);
                    fillEntry.push_back(st.rowEntry[static_cast<size_t>(b) * 16]);
                    pt.rowEntry.insert(pt.rowEntry.end(), 16, UINT32_MAX);
                    pt.rowDensityInMixture.insert(pt.rowDensityInMixture.end(), 16, UINT32_MAX);
                }
                pt.mixTileOffset[m + 1] = static_cast<uint32_t>(pt.tileCovariance.size());
            }
            pt.nTiles          = static_cast<uint32_t>(pt.tileCovariance.size());
            out.tiling         = std::move(pt);
            out.splitFillEntry = fillEntry;
            for (uint32_t s2 = 0; s2 < kSplitLimbs; ++s2)
                out.limbExp[s2] = b0 - 11 * static_cast<int32_t>(s2);
            // frame-side multipliers: [0, D) 2^a_d for y^2, [D, 2D) 2^b_d for y
            out.dimScale.assign(2 * D, 1.0f);
            std::vector<double> inv(2 * D, 1.0);
            for (uint32_t k = 0; k < 2 * D; ++k) {
                const double mx = k < D ? maxW[k] : maxN[k - D];
                if (mx > 0) {
                    int ex;
                    std::frexp(mx, &ex);
                    const int a     = std::max(-60, std::min(60, ex - 1 - 7));
                    out.dimScale[k] = static_cast<float>(std::ldexp(1.0, a));
                    inv[k]          = std::ldexp(1.0, -a);
                }
            }
            const auto h16 = [](double v) {
                const _Float16 h = static_cast<_Float16>(v);
                uint16_t       b;
                std::memcpy(&b, &h, 2);
                return b;
            };
            const auto f16v = [](uint16_t b) {
                _Float16 h;
                std::memcpy(&h, &b, 2);
                return static_cast<double>(h);
            };
            const uint32_t TP = out.tiling.nTiles, KW = out.kSteps16 * 32;
            out.tileH.assign(static_cast<size_t>(TP) * 16 * KW, 0);
            std::vector<uint16_t> row(KW);
            for (uint32_t t = 0; t < TP; ++t)
                for (uint32_t r = 0; r < 16; ++r) {
                    std::fill(row.begin(), row.end(), 0);
                    const bool real = covValues(out.tiling.rowEntry[static_cast<size_t>(t) * 16 + r], wv.data(), nv.data(), cv);
                    if (real || covValues(fillEntry[t], wv.data(), nv.data(), cv)) {
                        if (!real)
                            cv += padBias;
                        for (uint32_t k = 0; k < D; ++k) {
                            const float    w2 = static_cast<float>(wv[k] * inv[k]);
                            const uint16_t wh = h16(w2);
                            const uint16_t wl = h16(static_cast<double>(w2) - f16v(wh));
                            row[k]            = wh;
                            row[D + k]        = wh;
                            row[2 * D + k]    = wl;
                            const float    n2 = static_cast<float>(nv[k] * inv[D + k]);
                            const uint16_t nh = h16(n2);
                            const uint16_t nl = h16(static_cast<double>(n2) - f16v(nh));
                            row[3 * D + k]    = nh;
                            row[4 * D + k]    = nh;
                            row[5 * D + k]    = nl;
                        }
                        double rem = cv;
                        for (uint32_t s2 = 0; s2 < kSplitLimbs; ++s2) {
                            const uint16_t l = h16(std::ldexp(rem, -out.limbExp[s2]));
                            row[6 * D + s2]  = l;
                            rem -= std::ldexp(f16v(l), out.limbExp[s2]);
                        }
                    }
                    for (uint32_t k = 0; k < KW; ++k)  // v_mfma_f32_16x16x32_f16: lane 16((k>>3)&3) + row, step k>>5
                        out.tileH[((static_cast<size_t>(t) * out.kSteps16 + (k >> 5)) * kLanes + 16 * ((k >> 3) & 3) + r) *
                                          8 + (k & 7)] = row[k];
                }
        }
    }

    if (flavor == Flavor::DiagonalSum && !out.split)
        return "diagonal-sum runs on the split-f16 kernel only: dimension <= 83 (one covariance) or <= 42 (several), "
               "<= 1024 densities per mixture";

    // ---- native f32 layout ----
    if (!out.split) {
        out.tileA.assign(static_cast<size_t>(T) * KS * kLanes, 0.0f);
        std::vector<float> row(KS * 4);
        for (uint32_t t = 0; t < T; ++t) {
            for (uint32_t r = 0; r < kTileRows; ++r) {
                std::fill(row.begin(), row.end(), 0.0f);
                if (!rowValues(t, r, m2.data(), cst)) {
                    row[D] = FLT_MAX;  // padding row: bias +FLT_MAX never wins a strict minimum
                }
                else {
                    for (uint32_t k = 0; k < D; ++k)
                        row[k] = m2[k];
                    row[D] = static_cast<float>(cst);
                    if (out.foldNorm)
                        row[D + 1] = 1.0f;
                }
                // fragment order of v_mfma_f32_16x16x4_f32: lane = 16*(k&3) + row, step s = k>>2
                for (uint32_t k = 0; k < KS * 4; ++k)
                    out.tileA[(static_cast<size_t>(t) * KS + k / 4) * kLanes + (k % 4) * 16 + r] = row[k];
            }
        }
    }
    out.isvDevice.assign(static_cast<size_t>(C) * KS * 4, 0.0f);
    for (uint32_t c = 0; c < C; ++c)
        for (uint32_t k = 0; k < D; ++k)
            out.isvDevice[static_cast<size_t>(c) * KS * 4 + k] = out.isv[static_cast<size_t>(c) * D + k];
    return "";
}

// ---------------------------------------------------------------------------
// reference-order float scorers
// ---------------------------------------------------------------------------

std::string prepareDirect(const gmm_mixture_set& ms, Flavor flavor, float mixtureWeightScale, float gaussianScale,
                          ShardRange shard, uint32_t nb, PreparedDirect& out) {
    std::string err = validate(ms);
    if (!err.empty())
        return err;
    shard = normalizeShard(ms, shard);
    if (shard.begin > shard.end || shard.end > ms.n_mixtures)
        return "invalid mixture shard";
    const uint32_t D = ms.dimension, C = ms.n_covariances;
    const bool     batch = flavor == Flavor::BatchFloat;
    if (batch && C != 1)
        return "feature scorer supports only globally pooled covariance";  // BatchFeatureScorer.cc:146-148
    if (D > 128 || nb == 0 || (batch ? 4 * nb < (D + 7) / 8 * 8 : nb < D / 4))
        return "reference-order scorer supports dimension <= 128";
    out     = PreparedDirect();
    out.nb  = nb;
    out.L   = 4 * nb + 4;
    const uint32_t L = out.L, nfb = D / 4;
    // slot of dimension k in the row layout (gmm_kernels_direct.hip)
    const auto slot = [&](uint32_t k) { return batch || k < 4 * nfb ? k : 4 * nb + (k - 4 * nfb); };

    // diagonal-maximum: GaussDiagonalMaximumFeatureScorer::init (GDMFS.cc:64-86): isv and logNorm scaled by
    // gaussianScale_ = sqrt(gaussian-scale), minus2LogWeights scaled by mixture-weight-scale; batch-float:
    // BatchFloatFeatureScorer::init (BatchFeatureScorer.cc:145-175), unscaled
    const float gs = batch ? 1.0f : static_cast<float>(std::sqrt(static_cast<double>(gaussianScale)));
    out.isv.assign(static_cast<size_t>(C) * L, 0.0f);
    out.logNorm.resize(C);
    for (uint32_t c = 0; c < C; ++c) {
        const float* var = ms.variances + static_cast<size_t>(c) * D;
        for (uint32_t k = 0; k < D; ++k) {
            const float iv = refInverseSqrt(var[k]);
            out.isv[static_cast<size_t>(c) * L + slot(k)] = batch ? iv : iv * gs;
        }
        const float ln = static_cast<float>(refGaussLogNorm(var, D));
        out.logNorm[c] = batch ? ln : ln * (gs * gs);
    }
    const uint32_t eb = ms.mixture_offsets[shard.begin], ee = ms.mixture_offsets[shard.end];
    out.nMixtures = shard.end - shard.begin;
    out.nEntries  = ee - eb;
    out.mixOff.resize(out.nMixtures + 1);
    for (uint32_t m = 0; m <= out.nMixtures; ++m)
        out.mixOff[m] = ms.mixture_offsets[shard.begin + m] - eb;
    out.mean.assign(static_cast<size_t>(out.nEntries) * L, 0.0f);
    out.entryCov.resize(out.nEntries);
    out.constant.resize(out.nEntries);
    for (uint32_t e = eb; e < ee; ++e) {
        const uint32_t dns  = ms.mixture_densities[e];
        const uint32_t cov  = ms.density_covariance[dns];
        const float*   mean = ms.means + static_cast<size_t>(ms.density_mean[dns]) * D;
        float*         row  = out.mean.data() + static_cast<size_t>(e - eb) * L;
        for (uint32_t k = 0; k < D; ++k)  // batch: means_ = mean * variance_ (std::multiplies<float>, cc:171)
            row[slot(k)] = batch ? mean[k] * out.isv[k] : mean[k];
        out.entryCov[e - eb] = cov;
        const double lw      = ms.mixture_log_weights[e];
        // MixtureFeatureScorerElement.cc:26,30-33: (f32)(-2 log w) * scale; BatchFeatureScorer.cc:173:
        // constants_ = logNormFactor - 2 * logWeight
        out.constant[e - eb] = batch ? static_cast<float>(static_cast<double>(out.logNorm[0]) - 2 * lw)
                                     : static_cast<float>(-2 * lw) * mixtureWeightScale;
    }
    return "";
}

}  // namespace rasr_gmm
