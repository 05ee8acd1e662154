// gmm_prepare.hh -- host-side model preparation for the MI355X GMM scorer.
//
// The reference scorers prepare their tables on the host once per model
// (SimdFeatureScorer.cc:64-104, GaussDiagonalMaximumFeatureScorer.cc:64-86,
// BatchFeatureScorer.cc:145-172,339-380).  This file reproduces that arithmetic
// bit for bit (independently of the compiler flags this file is built with) and
// lays the result out for the device kernels:
//
//   * densities of a mixture are grouped by covariance and cut into tiles of 16
//     rows (one MFMA row block); tiles of a mixture are contiguous (CSR
//     mixture -> tiles), the tail of every tile is padded with rows that can
//     never win the minimum;
//   * quantized mode (SIMD-diagonal-maximum, batch-int): per tile a 1 KiB s8
//     operand block in v_mfma_i32_16x16x64_i8 fragment order plus 16 packed
//     int32 row constants;
//   * float mode (diagonal-maximum, batch-float): per tile K/4 x 64 f32 operands
//     in v_mfma_f32_16x16x4_f32 fragment order, the row constant folded into
//     the K column `dimension`.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/rasr_gmm.h"
#include "gmm_kernels.hh"

namespace rasr_gmm {

constexpr uint32_t kTileRows     = 16;   // densities per MFMA tile
constexpr uint32_t kLanes        = 64;   // wavefront
constexpr uint32_t kI8K          = 64;   // K of v_mfma_i32_16x16x64_i8
constexpr int32_t  kPadRowPacked = 0x7fffffff;

// K/4 steps of the float kernel that are instantiated (gmm_kernels.hip); a model is padded up to one of these.
inline uint32_t f32KStepsInstantiated(uint32_t kSteps) {
    static const uint32_t ks[] = {2, 4, 6, 8, 10, 12, 14, 16, 20, 24, 28, 32};
    for (uint32_t k : ks)
        if (kSteps <= k)
            return k;
    return 0;
}

// ---- reference scalar arithmetic (flag-independent restatement) ----
float   refInverseSqrt(float x);               // Utilities.hh:87-91 as built (-ffast-math): rsqrtss + NR
int32_t refRoundToInt(float x);                // (int)round(x) as built: add 0.49999997 with sign, cvttss2si
uint8_t refQuantize(float x);                  // quantize<f32,u8>, Utilities.hh:179-191
double  refGaussLogNorm(const float* var, uint32_t d);   // Utilities.hh:55-76
float   refQuantizationScalingFactor(float minv, float maxv); // SimdFeatureScorer.cc:128-133 as built
int32_t refTruncF32(float x);                  // (s32)float, cvttss2si
int32_t refTruncF64(double x);                 // (s32)double, cvttsd2si

enum class Flavor : int { Simd = 0, BatchInt = 1, DiagonalMaximum = 2, BatchFloat = 3, DiagonalSum = 4 };

struct Tiling {
    uint32_t              nTiles = 0;
    std::vector<uint32_t> mixTileOffset;   // [nMixtures+1] (shard-relative mixtures)
    std::vector<uint32_t> tileCovariance;  // [nTiles]
    std::vector<uint32_t> rowEntry;        // [nTiles*16] entry index or UINT32_MAX for padding
    std::vector<uint32_t> rowDensityInMixture; // [nTiles*rows]
    uint32_t              rows = kTileRows;        // densities per tile
    uint32_t              maxEntriesPerMixture = 0;
};

// score-only layouts of the quantized scorers (PreparedQuantized::scoreOnly, I8Args::scoreOnly)
constexpr int kScoreOnlyNone = 0, kScoreOnlyClass = 1, kScoreOnlySlots = 2;

struct PreparedQuantized {
    Flavor   flavor = Flavor::Simd;
    uint32_t dimension = 0, paddedDimension = 0, nCovariances = 0, nMixtures = 0;
    uint32_t kSteps = 1;              // K blocks of 64
    uint32_t idxBits = 1;
    float    scaling = 0, scalingSquared = 0, inverseQuantizationFactor = 0;
    float    batchScale = 0;          // BatchIntFeatureScorer::scale_ = 2 s^2
    std::vector<float>   isvScaled;   // [C][dimension]
    std::vector<float>   logNormScaled; // [C]
    std::vector<uint8_t> preparedMean;  // [entries][paddedDimension]  (reference table, for inspection)
    std::vector<int32_t> constantWeight;// [entries]
    Tiling               tiling;
    std::vector<int8_t>  tileA;       // [nTiles][kSteps][64 lanes][16]
    std::vector<int32_t> tileP;       // [nTiles][16]
    std::vector<float>   isvDevice;   // [C][kSteps*64], zero padded
    // score-only class layout (calls without best densities; one covariance, one K step): tileP holds the
    // MFMA's C input h = Q >> 1 (Q = c + sum a'^2), so the accumulator is v = dot + h and the row value
    // 2 dot + Q = 2 v + p.  A mixture's class tiles split its rows by the parity p over the tile's 4 lane
    // groups (bit g of mixOddMask[m]: lane group g holds odd-Q rows); its mixed tiles that follow hold the
    // rest, evens first in row order (gmm_prepare.cc buildClassLayout, gmm_kernels_i8.hip SCORE_ONLY).
    // mixOddMask[m]: bits 0-3 the odd lane groups, bits 4-15 the first odd index of the mixed rows, bits
    // 16-31 the class tile count.  That is kScoreOnlyClass, the layout preselection-batch-int masks.
    // kScoreOnlySlots (the other calls without best densities; gmm_prepare.cc buildSlotLayout,
    // gmm_kernels_i8.hip scoreI8Cls): no mixed tiles; every tile gives the 8 classes (g, s) -- rows 4g + s and
    // 4g + s + 2 -- the parity of bit 2g + s of mixOddMask[m].
    int                  scoreOnly = 0;   // kScoreOnlyNone / kScoreOnlyClass / kScoreOnlySlots
    std::vector<uint32_t> mixOddMask;  // [nMixtures]
};

struct PreparedFloat {
    Flavor   flavor = Flavor::DiagonalMaximum;
    uint32_t dimension = 0, nCovariances = 0, nMixtures = 0;
    uint32_t kSteps = 0;              // K/4
    bool     foldNorm = false;        // multi-covariance: ||x'||^2 folded into K column dimension+1
    uint32_t tileBits = 1;            // single covariance: ceil(log2(max tiles per mixture))
    float    offsetK0 = 0;            // single covariance: added to every row constant (values > 0)
    std::vector<float> isv;           // [C][dimension] (after gaussian-scale)
    std::vector<float> logNorm;       // [C]
    Tiling             tiling;
    std::vector<float> tileA;         // [nTiles][kSteps][64 lanes]  (empty when split)
    std::vector<float> isvDevice;     // [C][kSteps*4] zero padded
    // per-dimension centre (input units, the mean of all the set's means): both sides of the
    // expanded quadratic form are taken about it, x' = (x - c) isv, m' = (mu - c) isv, so the
    // terms ||x'||^2, ||m'||^2, x'.m' stay of the order of the model's spread, not of |mu / sigma|
    std::vector<float> centre;        // [dimension]
    std::vector<uint32_t> splitFillEntry; // split tiling: [tile] the entry its padding rows repeat
    // split-f16 kernel (single covariance, gmm_kernels_split.hip): every f32 operand is a sum of
    // two f16 pieces, hi + lo; a row is  sum_d [mh*xh + mh*xl + ml*xh]  +  sum_s limb_s * 2^(b_s)
    bool                  split    = false;
    uint32_t              kSteps16 = 0;    // K/32 steps of v_mfma_f32_16x16x32_f16
    std::vector<uint16_t> tileH;           // [nTiles][kSteps16][64 lanes][8] f16 bits (kSteps16: K steps of the
                                           // tile's MFMA, 32 wide for 16-row tiles, 16 wide for 32-row tiles)
    std::vector<float>    dimScale;        // [dimension]: 2^a_d, x'' = x' * 2^a_d, m'' = -2 m' / 2^a_d
    int32_t               limbExp[4] = {0, 0, 0, 0};  // b_s: the frame side of limb s is 2^(b_s - e_frame)
    // split kernel keys: the low splitKeyBits mantissa bits hold (tile in mixture << 2 | row slot);
    // every mixture has an even number of tiles (pad tiles repeat the mixture's first row)
    uint32_t              splitKeyBits = 0;
    uint32_t              splitRows    = 16;  // tile height: 16 (16x16x32 MFMA, tile pairs) or 32 (32x32x16)
    // several covariances on the split kernels (gmm_prepare.cc, the covariance-free expansion): the frame operand
    // is [y^2, y] about the centre (prepareFramesSplitCov), dimScale has 2 D entries, K = 6 D + 4
    bool                  splitCov     = false;
};


struct ShardRange {
    uint32_t begin = 0, end = 0;
};

// Reference-order float scorers (GMM_FLAG_REFERENCE_ORDER, gmm_kernels_direct.hip): rows of L = 4 nb + 4
// floats per mixture entry (diagonal-maximum: the D / 4 whole 4-dimension blocks, zeros, the D % 4
// remaining dimensions in the last 4 slots; batch-float: mean * isv, zeros), the covariances' isv rows in
// the same layout, the per-entry constants and covariance, CSR entry offsets of the shard's mixtures.
struct PreparedDirect {
    uint32_t              nb = 0, L = 0, nMixtures = 0, nEntries = 0;
    std::vector<float>    mean;       // [nEntries][L]
    std::vector<float>    isv;        // [C][L]
    std::vector<uint32_t> entryCov;   // [nEntries]
    std::vector<float>    constant;   // [nEntries] minus2LogWeights / batch constants_
    std::vector<float>    logNorm;    // [C]
    std::vector<uint32_t> mixOff;     // [nMixtures + 1]
};

// Returns empty string on success, else an error message.
std::string validate(const gmm_mixture_set& ms);
// scoreOnlyLayout: lay out that score-only layout (kScoreOnlyClass / kScoreOnlySlots) when it applies (out.scoreOnly
// says whether it did)
std::string prepareQuantized(const gmm_mixture_set& ms, Flavor flavor, ShardRange shard, PreparedQuantized& out,
                             int scoreOnlyLayout = kScoreOnlyNone);
// wantSplit: lay the model out for the split-f16 kernel when it applies (one covariance,
// 3*dimension+7 <= 256, row constants below 2^30); out.split says whether it did.
std::string prepareFloat(const gmm_mixture_set& ms, Flavor flavor, float mixtureWeightScale, float gaussianScale,
                         ShardRange shard, PreparedFloat& out, bool wantSplit = false, uint32_t splitRowsWanted = 0);
// nb: 4-dimension blocks of the kernel instantiation (directBlocks)
std::string prepareDirect(const gmm_mixture_set& ms, Flavor flavor, float mixtureWeightScale, float gaussianScale,
                          ShardRange shard, uint32_t nb, PreparedDirect& out);

}  // namespace rasr_gmm
