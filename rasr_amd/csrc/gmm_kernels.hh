// gmm_kernels.hh -- launch interface of the MI355X GMM scorer kernels (gmm_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <set>
#include <utility>

namespace rasr_gmm {

// hipFuncAttributeMaxDynamicSharedMemorySize for `fn` on the current device, once per (kernel, device): a
// process may drive several GPUs (gmm_scorer_create_sharded, one handle per GPU), and the attribute belongs to
// the device's copy of the kernel
inline hipError_t allowDynamicLds(const void* fn, int bytes) {
    static std::mutex                        mu;
    static std::set<std::pair<const void*, int>> done;
    int                                      dev = 0;
    hipError_t                               e   = hipGetDevice(&dev);
    if (e != hipSuccess)
        return e;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({fn, dev}))
        return hipSuccess;
    if ((e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes)) == hipSuccess)
        done.insert({fn, dev});
    return e;
}

#ifndef GMM_I8_NF
#define GMM_I8_NF 8
#endif
#ifndef GMM_F32_NF
#define GMM_F32_NF 4
#endif
constexpr int      kI8NF          = GMM_I8_NF;   // column blocks of 16 frames per wave, quantized kernel
constexpr int      kF32NF         = GMM_F32_NF;  // column blocks of 16 frames per wave, float kernel
constexpr uint32_t kWavesPerBlock = 4;
constexpr uint32_t kI8FramesPerBlock  = kWavesPerBlock * kI8NF * 16;   // 512
#ifndef GMM_I8_CLS_NF
#define GMM_I8_CLS_NF 16  // scoreI8Cls (calls without best densities, slot layout): column blocks per wave (8 or 16)
#endif
constexpr int      kI8ClsNF           = GMM_I8_CLS_NF;
constexpr uint32_t kI8ClsFramesPerBlock = kWavesPerBlock * kI8ClsNF * 16;
constexpr uint32_t kI8SmallFrames     = kWavesPerBlock * 4 * 16;        // 256: the small-call tile (I8Args::smallTile)
constexpr uint32_t kI8TinyFrames      = 4 * 16;                         // 64: one 64-frame wave per workgroup
constexpr uint32_t kF32FramesPerBlock = kWavesPerBlock * kF32NF * 16;  // 256
constexpr uint32_t kFramePadQuantum   = 512;
constexpr uint32_t kTilePad           = 16;   // zero tiles after the last one (prefetch / LDS segments)

struct I8Args {
    const void*     tileA;        // i32x4 [T+1][KS][64]
    const void*     tileP;        // i32x4 [T+1][4]
    const uint32_t* tileCov;      // [T+1]
    const uint32_t* mixTileOff;   // [nMixtures+1]
    const uint32_t* chunkMixOff;  // [nChunks+1]
    const int8_t*   frameQ;       // [C][nFramesPad][KS*64]
    const int32_t*  frameSS;      // [C][nFramesPad]
    float*          scores;
    uint32_t*       best;
    uint32_t        nFrames, nFramesPad, scoreStride;
    uint32_t        nChunks, nFrameTiles, mixBase;
    uint32_t        idxBits;
    int             flavor;       // 0 SIMD-diagonal-maximum, 1 batch-int
    float           s2, batchScale, outScale;
    float           finB, finInv; // the finalize's divisor b = 2 s^2 and RN(1 / b) (gmm_kernels_i8.hip finalizeStoreI8)
    float           finInvLo;     // RN(1 / b - finInv): 1 / b as a sum of two floats
    int             finDivide;    // 1: scales outside the range of the multiply-and-correct finalize, divide
    // preselection-batch-int (gmm_kernels_presel.hip): per-(frame, cluster) mask, per-row cluster offsets
    const uint32_t* selT;         // [nFramesPad/64][nClusters][16] u32, byte (frame%64)/16 = 0xff: deselected
    const uint8_t*  selC;         // [nFramesPad/128][nClusters][16] u8: the wave tables (launchCompactSelection)
    const void*     tileClu;      // u32 [T+pad][16]: cluster * 16 * kI8PreselEntryBytes (byte offset into a wave's table)
    uint32_t        nClusters;
    int             presel;
    // score-only layouts (gmm_prepare.hh PreparedQuantized::scoreOnly): tileP is the MFMA's C input; 1 = the class
    // layout (preselection-batch-int: mixOddMask[m] bit g = lane group g holds odd-Q rows, then mixed tiles), 2 = the
    // slot layout (scoreI8Cls: mixOddMask[m] bit 2g + s = the rows of lane group g's register s hold odd-Q rows)
    const uint32_t* mixOddMask;
    int             scoreOnly;
    // small calls (no preselection): 1 = 64 frames per wave, 256 per workgroup (<= kI8SmallFrames frames: half
    // the padded frames of the 128-frame waves); 2 = one such wave per workgroup (<= kI8TinyFrames frames)
    int             smallTile;
};

struct F32Args {
    const float*    tileA;        // [T+1][KS][64]
    const uint32_t* tileCov;      // [T+1]
    const uint32_t* rowDns;       // [T+1][16]
    const uint32_t* mixTileOff;
    const uint32_t* chunkMixOff;
    const float*    frameX;       // [C][nFramesPad/16][KS][64]
    const float*    frameXX;      // [C][nFramesPad]
    float*          scores;
    uint32_t*       best;
    uint32_t        nFrames, nFramesPad, scoreStride;
    uint32_t        nChunks, nFrameTiles, mixBase;
    int             flavor;       // 2 diagonal-maximum, 3 batch-float
    uint32_t        tileBits;     // single covariance: low mantissa bits holding the tile number
    float           offsetK0;     // single covariance: constant added to every row so values are > 0
    float           outScale;
};

#ifndef GMM_SPLIT_NF
#define GMM_SPLIT_NF 8  // 4 or 8 (A/B builds)
#endif
// scoreSplit (diagonal-maximum, batch-float): column blocks of 16 frames per wave.  At 8 (128 frames per wave,
// one wave per SIMD, the frame operands in the accumulator file) every tile fragment a wave loads feeds twice
// the MFMAs of 4, and the pair step's VALU is the epilogue alone: 4.68 against 5.35 ms per 32768 frames, A/B.
constexpr int      kSplitNF             = GMM_SPLIT_NF;
#ifndef GMM_SPLIT_FPB
#define GMM_SPLIT_FPB 256
#endif
constexpr uint32_t kSplitFramesPerBlock = GMM_SPLIT_FPB;  // frames per workgroup of every split kernel (A/B: 512)
constexpr uint32_t kSplitWaves          = kSplitFramesPerBlock / 64;  // 64 frames per wave: scoreSplit32,
                                                                      // scoreSplitSum, preselection-batch-float
constexpr uint32_t kSplitMainWaves      = kSplitFramesPerBlock / (16 * kSplitNF);  // scoreSplit
#ifndef GMM_SPLIT_WIDE
#define GMM_SPLIT_WIDE 1  // scoreSplitWide for K steps <= 4 without preselection (0: the pair kernel, A/B)
#endif
#ifndef GMM_SPLIT_WIDE5
#define GMM_SPLIT_WIDE5 0  // 192-frame waves at K steps 5 (A/B: no faster than the pair kernel)
#endif
// scoreSplitWide (16-row tiles, diagonal-maximum / batch-float without preselection): frames of its one-wave
// workgroups at ks K steps -- 16 column blocks at K <= 128 (the frame operands fill the 256 AGPRs) -- or 0 where the
// pair kernel scoreSplit runs
constexpr uint32_t splitWideFrames(uint32_t ks) {
    return !GMM_SPLIT_WIDE ? 0u : ks <= 4 ? 256u : (GMM_SPLIT_WIDE5 && ks == 5) ? 192u : 0u;
}

constexpr uint32_t kSplitLimbs   = 4;
constexpr uint32_t kSplitXXLimbs = 3;
// the frame's ||x'||^2 rides in K as three f16 limbs against these powers of two on the model side
constexpr int kSplitXXExp[kSplitXXLimbs] = {15, 4, -7};
// K layout of the split kernel: [0,D) mh*xh, [D,2D) mh*xl, [2D,3D) ml*xh, [3D,3D+4) row-constant
// limbs, [3D+4,3D+7) ||x'||^2 limbs
inline uint32_t splitKSteps(uint32_t dimension) {  // K/32 steps of v_mfma_f32_16x16x32_f16
    return (3 * dimension + kSplitLimbs + kSplitXXLimbs + 31) / 32;
}
inline uint32_t splitKSteps32(uint32_t dimension) {  // K/16 steps of v_mfma_f32_32x32x16_f16
    return (3 * dimension + kSplitLimbs + kSplitXXLimbs + 15) / 16;
}
// several covariances (the covariance-free layout): K = [y^2 terms 3D][y terms 3D][row-constant limbs 4]
inline uint32_t splitCovKSteps(uint32_t dimension) {
    return (6 * dimension + kSplitLimbs + 31) / 32;
}

struct SplitArgs {
    const void*     tileH;        // f16 [T+pad][KS16][64][8]
    const uint32_t* mixTileOff;
    const uint32_t* chunkMixOff;
    const void*     frameH;       // f16 [nFramesPad/16][KS16][64][8]
    const float*    frameXX;      // [nFramesPad]  ||x'||^2 * 2^-e
    const int32_t*  frameExp;     // [nFramesPad]  e
    float*          scores;
    uint32_t*       best;
    uint32_t        nFrames, nFramesPad, scoreStride;
    uint32_t        nChunks, nFrameTiles, mixBase;
    int             flavor;       // 2 diagonal-maximum, 3 batch-float, 4 diagonal-sum
    uint32_t        tileBits;
    float           offsetK0;
    float           outScale;
    // preselection-batch-float: as I8Args; a mixture without a selected density scores backoff
    const uint32_t* selT;
    const void*     tileClu;
    uint32_t        nClusters;
    int             presel;
    float           backoff;
};

hipError_t launchPrepareFramesI8(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesPad,
                                 uint32_t nFramesRead, uint32_t D, uint32_t C, uint32_t KS, const float* isv, int8_t* frameQ,
                                 int32_t* frameSS, hipStream_t stream);
hipError_t launchPrepareFramesF32(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesPad,
                                  uint32_t nFramesRead, uint32_t D, uint32_t C, uint32_t KS, int foldNorm, const float* isv,
                                  const float* centre, float* frameX,
                                  float* frameXX, hipStream_t stream);
hipError_t launchPrepareFramesSplit(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesRead,
                                    uint32_t D, uint32_t rows, uint32_t kSteps, const float* isv, const float* centre,
                                    const float* dimScale,
                                    const int32_t* limbExp, void* frameH, float* frameXX, int32_t* frameExp,
                                    hipStream_t stream);
// several covariances: frameH [nFramesPad/16][KS16][64][8] with the K layout of splitCovKSteps, frameExp = e
hipError_t launchPrepareFramesSplitCov(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesRead,
                                       uint32_t D, uint32_t kSteps, const float* centre, const float* dimScale,
                                       const int32_t* limbExp, void* frameH, int32_t* frameExp, hipStream_t stream);
hipError_t launchScoreSplit(const SplitArgs& a, uint32_t rows, uint32_t kSteps, hipStream_t stream);
hipError_t launchScoreSplitSum(const SplitArgs& a, uint32_t rows, uint32_t kSteps, hipStream_t stream);  // diagonal-sum
constexpr uint32_t kSplit32MaxKSteps = 10;  // 32-row split kernel instantiated for K/16 <= 10 (D <= 51)
hipError_t launchScoreI8(const I8Args& a, uint32_t kSteps, bool multiCov, hipStream_t stream);

// reference-order float scorers (GMM_FLAG_REFERENCE_ORDER, gmm_kernels_direct.hip): one frame per lane, the
// reference's own f32 operation order per density, densities streamed through the scalar cache
constexpr uint32_t kDirectFramesPerBlock = 256;
struct DirectArgs {
    const float*    mean;         // [entries][Dp]: diagonal-maximum the means, batch-float mean * isv (f32)
    const float*    isv;          // [C][Dp]: 1/sqrt(var) (diagonal-maximum: times sqrt(gaussian-scale))
    const uint32_t* entryCov;     // [entries]
    const float*    constant;     // [entries]: minus2LogWeights (diagonal-maximum) / constants_ (batch-float)
    const float*    logNorm;      // [C] (diagonal-maximum)
    const uint32_t* mixOff;       // [nMixtures+1] entry offsets (shard-relative)
    const uint32_t* chunkMixOff;  // [nChunks+1]
    const float*    frames;
    float*          scores;
    uint32_t*       best;
    uint32_t        nFrames, frameStride, scoreStride;
    uint32_t        nChunks, nFrameTiles;
    uint32_t        D, Dp;        // Dp: row length L = 4 NB + 4 floats (directBlocks)
    int             batch;        // 0 diagonal-maximum, 1 batch-diagonal-maximum-float
    int             multiCov;     // several covariances (isv row per density)
    float           outScale;
};
hipError_t launchScoreDirect(const DirectArgs& a, hipStream_t stream);
uint32_t   directBlocks(uint32_t D, bool batch);  // 4-dimension blocks of the row layout, 0 = unsupported

// sparse best densities (gmm_best_density_pairs, gmm_kernels_pairs.hip): one wave per (frame, mixture) pair,
// the mixture's entries scored in the reference's own arithmetic and scanned in entry order
enum PairKind : int { kPairSimd = 0, kPairDiagonalMaximum = 1, kPairDiagonalSum = 2 };
struct PairArgs {
    const float*    frames;      // [nFrames][frameStride]
    const uint32_t* pairFrame;   // [nPairs] frame of the pair
    const uint32_t* pairMix;     // [nPairs] mixture of the pair (shard-relative)
    uint32_t*       best;        // [nPairs] density in mixture, 0xffffffff: none (empty mixture, no finite score)
    const uint32_t* mixOff;      // [nMixtures+1] entry offsets (shard-relative)
    const uint32_t* entryCov;    // [entries]
    // SIMD-diagonal-maximum: prepared means (u8, rows of Dp), constant weights, isv * s rows of isvStride
    const uint8_t*  qMean;
    const int32_t*  qConst;
    // diagonal-maximum / diagonal-sum: the reference-order row layout of the direct scorer (rows of L floats)
    const float*    fMean;
    const float*    fConst;      // minus2LogWeights
    const float*    fLogNorm;    // [C]
    const float*    isv;         // SIMD: [C][isvStride]; float: [C][L]
    uint32_t        nFrames, frameStride, nPairs, nMixtures;
    uint32_t        D, Dp, L, nb, isvStride;
    int             kind;        // PairKind
};
hipError_t launchBestPairs(const PairArgs& a, hipStream_t stream);
// quantized LDS kernel: the never-winning stand-in tile after the segment ring (operands, row constants,
// PRESEL cluster offsets)
constexpr uint32_t kI8DummyTileBytes(int ks, bool presel) { return static_cast<uint32_t>(ks) * 1024u + 64u + (presel ? 64u : 0u); }
#ifndef GMM_I8_PRESEL_NF
#define GMM_I8_PRESEL_NF 8
#endif
// preselection-batch-int: frames per wave / 16 (8: two 64-frame mask words per wave; 4 kept for A/B)
constexpr uint32_t kI8PreselNF           = GMM_I8_PRESEL_NF;
// bytes of a mask table entry (gmm_kernels_i8.hip): a row's cluster offset is cluster * 16 * this
constexpr uint32_t kI8PreselEntryBytes   = 1;
constexpr uint32_t kI8PreselFramesPerBlock = kWavesPerBlock * kI8PreselNF * 16;

// density-sharded exchange (gmm_kernels_shard.hip): (score, density) <-> order-preserving int64 keys
hipError_t launchPackShardKeys(const float* scores, const uint32_t* best, const uint32_t* bestOffset, uint32_t rows,
                               uint32_t nFrames, uint32_t stride, int64_t* keys, hipStream_t stream);
hipError_t launchUnpackShardKeys(const int64_t* keys, uint32_t rows, uint32_t nFrames, float* scores, uint32_t* best,
                                 uint32_t stride, hipStream_t stream);
hipError_t launchFillShardKeys(int64_t* keys, size_t n, hipStream_t stream);  // keys[i] = INT64_MAX
hipError_t launchMinShardKeys(const int64_t* slots, uint32_t nSlots, size_t n, int64_t* out, hipStream_t stream);
// dst[i] = min(dst[i], src[i]): the device-local fold of the RCCL exchange (parts that share a GPU)
hipError_t launchMinIntoShardKeys(int64_t* dst, const int64_t* src, size_t n, hipStream_t stream);

// frame-major host tables (gmm_kernels_layout.hip): dst[c * dstPitch + r] = src[r * srcPitch + c], 32-bit words
hipError_t launchCopyWords2D(const uint32_t* src, uint32_t srcPitch, uint32_t* dst, uint32_t dstPitch, uint32_t rows,
                             uint32_t cols, hipStream_t stream);
hipError_t launchTransposeWords(const uint32_t* src, uint32_t rows, uint32_t cols, uint32_t srcPitch, uint32_t* dst,
                                uint32_t dstPitch, hipStream_t stream);

// density preselection (gmm_kernels_presel.hip)
hipError_t launchAssignDensities(bool quantized, const void* means, uint32_t nDensities, uint32_t Dp,
                                 const void* clusterMeans, uint32_t nClusters, uint8_t* clusterOf, hipStream_t stream);
hipError_t launchSelectClusters(bool quantized, const float* frames, uint32_t nFrames, uint32_t frameStride,
                                uint32_t nFramesRead, uint32_t D, uint32_t Dp, const float* variance,
                                const void* clusterMeans, uint32_t nClusters, uint32_t nSelected, uint32_t* selT,
                                hipStream_t stream);
// the quantized scorer's mask table: [nFramesRead / 128][nClusters][16] u8 entries from the byte mask
hipError_t launchCompactSelection(const uint32_t* selT, uint32_t nFramesRead, uint32_t nClusters, uint8_t* selC,
                                  hipStream_t stream);
hipError_t launchScoreF32(const F32Args& a, uint32_t kSteps, bool multiCov, hipStream_t stream);

}  // namespace rasr_gmm
