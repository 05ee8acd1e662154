// gmm_kernels.hip -- MI355X (gfx950) kernels of the diagonal-GMM feature scorer.
//
// Hot path: for a batch of F frames and every mixture e of the model,
//   score(e,t) = min_{d in e} [ c_d + || A_d - x_t ||^2 ]   (+ argmin)
// RASR computes it per frame and density with a JIT'd SSE2 u8 SSD
// (src/Mm/SimdFeatureScorer.cc:158-176, src/Mm/SSE2CodeGenerator.cc:324-374)
// or SSE float code (src/Mm/GaussDiagonalMaximumFeatureScorer.cc:116-218).
// Here the cross term is a dense (densities x K) . (K x frames) contraction on
// the matrix cores and the per-mixture minimum is a running min in the MFMA
// accumulator registers, reduced across the wave once per mixture:
//
//   quantized (SIMD-diagonal-maximum, batch-int): v_mfma_i32_16x16x64_i8 on
//     s8 operands (q - 128); exact integer arithmetic; epilogue per element is
//     one v_lshl_add (constant + 2*dot, packed with the density index in the
//     low bits) and one v_min_i32 -> bit-identical scores and argmins;
//   float (diagonal-maximum, batch-float): v_mfma_f32_16x16x4_f32, the row
//     constant folded into one K column; epilogue v_cmp + 2 v_cndmask.
//
// Work decomposition: one 256-thread workgroup = 4 waves x NF column blocks of
// 16 frames; it walks a chunk of consecutive mixtures (all their tiles of 16
// densities).  Workgroups that share a chunk are placed on one XCD (blockIdx %
// 8) and run back to back, so each chunk's tiles are fetched from HBM/MALL into
// that XCD's L2 once and re-read from L2 by the other frame tiles.
//
// Every kernel is compiled with -ffp-contract=off; the quantizer additionally
// uses __fmul_rn / __fadd_rn so it can never be contracted into an FMA.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "gmm_kernels.hh"

namespace rasr_gmm {
namespace dev {

typedef int   i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// reference quantizer, device side (mirrors refRoundToInt / refQuantize in gmm_prepare.cc)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int refRoundToInt(float x) {
    const float t = __fadd_rn(x, copysignf(0x1.fffffep-2f, x));
    if (!(fabsf(t) < 2147483648.0f))
        return INT_MIN;  // cvttss2si "integer indefinite"
    return static_cast<int>(t);
}

// q(x) - 128 in [-128, 127]  (quantize<f32,u8>, src/Mm/Utilities.hh:186-190)
__device__ __forceinline__ int quantizeCentered(float x) {
    int v = static_cast<int>(static_cast<unsigned>(refRoundToInt(x)) + 128u);
    v     = v > 255 ? 255 : v;
    v     = v < 0 ? 0 : v;
    return v - 128;
}

// ---------------------------------------------------------------------------
// frame preparation (quantized): Context::Context, SimdFeatureScorer.cc:22-35
//   frameQ [C][nFramesPad][KS*64] s8 (q - 128, 0 in the padding), frameSS [C][nFramesPad] = sum (q-128)^2
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prepareFramesI8(const float* __restrict__ frames, uint32_t nFrames,
                                                        uint32_t frameStride, uint32_t nFramesPad,
                                                        uint32_t nFramesRead, uint32_t D,
                                                        uint32_t C, uint32_t KS, const float* __restrict__ isv,
                                                        int8_t* __restrict__ frameQ, int32_t* __restrict__ frameSS) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= C * nFramesRead)
        return;
    const uint32_t c = gid / nFramesRead, f = gid % nFramesRead;
    const float*   x  = frames + static_cast<size_t>(f) * frameStride;
    const float*   iv = isv + static_cast<size_t>(c) * KS * 64;
    i32x4*         out = reinterpret_cast<i32x4*>(frameQ + (static_cast<size_t>(c) * nFramesPad + f) * KS * 64);
    int            ss = 0;
    for (uint32_t blk = 0; blk < KS * 4; ++blk) {
        i32x4 w;
        for (int q4 = 0; q4 < 4; ++q4) {
            uint32_t word = 0;
            for (int b = 0; b < 4; ++b) {
                const uint32_t k = blk * 16 + q4 * 4 + b;
                int            v = 0;
                if (f < nFrames && k < D) {
                    v = quantizeCentered(__fmul_rn(x[k], iv[k]));  // multiplyAndQuantize, IntelOptimization.cc:63
                    ss += v * v;
                }
                word |= (static_cast<uint32_t>(v) & 0xffu) << (8 * b);
            }
            w[q4] = static_cast<int>(word);
        }
        out[blk] = w;
    }
    frameSS[static_cast<size_t>(c) * nFramesPad + f] = ss;
}

// ---------------------------------------------------------------------------
// frame preparation (float): x' = x * isv, fragment order of v_mfma_f32_16x16x4_f32
//   frameX [C][nFramesPad/16][KS][64]: lane l of step s holds x'[16 fb + (l&15)][4 s + (l>>4)]
//   column D is 1 (picks the row constant), column D+1 is ||x'||^2 when foldNorm
//   frameXX [C][nFramesPad] = ||x'||^2
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prepareFramesF32(const float* __restrict__ frames, uint32_t nFrames,
                                                         uint32_t frameStride, uint32_t nFramesPad,
                                                         uint32_t nFramesRead, uint32_t D,
                                                         uint32_t C, uint32_t KS, int foldNorm,
                                                         const float* __restrict__ isv, float* __restrict__ frameX,
                                                         float* __restrict__ frameXX) {
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= C * nFramesRead)
        return;
    const uint32_t c = gid / nFramesRead, f = gid % nFramesRead;
    const float*   x  = frames + static_cast<size_t>(f) * frameStride;
    const float*   iv = isv + static_cast<size_t>(c) * KS * 4;
    const bool     valid = f < nFrames;
    float          xx    = 0.0f;
    if (valid)
        for (uint32_t k = 0; k < D; ++k) {
            const float v = __fmul_rn(x[k], iv[k]);
            xx            = __fadd_rn(xx, __fmul_rn(v, v));
        }
    float* base = frameX + (static_cast<size_t>(c) * (nFramesPad / 16) + f / 16) * KS * 64;
    for (uint32_t k = 0; k < KS * 4; ++k) {
        float v = 0.0f;
        if (valid) {
            if (k < D)
                v = __fmul_rn(x[k], iv[k]);
            else if (k == D)
                v = 1.0f;
            else if (k == D + 1 && foldNorm)
                v = xx;
        }
        base[(k >> 2) * 64 + (k & 3) * 16 + (f & 15)] = v;
    }
    frameXX[static_cast<size_t>(c) * nFramesPad + f] = xx;
}

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------

// Workgroup -> (chunk, frame tile).  Blocks b and b+8 share an XCD (round-robin
// dispatch); give each XCD whole chunks and walk their frame tiles back to back.
__device__ __forceinline__ bool mapBlock(uint32_t nChunks, uint32_t nFrameTiles, uint32_t& chunk, uint32_t& ft) {
    const uint32_t b = blockIdx.x, xcd = b & 7u, j = b >> 3;
    chunk            = xcd + 8u * (j / nFrameTiles);
    ft               = j % nFrameTiles;
    return chunk < nChunks;
}

// ---------------------------------------------------------------------------
// quantized scorer
// ---------------------------------------------------------------------------
template <int NF, int KS, bool MULTI>
__global__ __launch_bounds__(256) void scoreI8(I8Args a) {
    static_assert(NF == 4 || NF == 8, "NF");
    constexpr int NPL = NF / 4;  // results per lane per mixture
    const int     lane = threadIdx.x & 63;
    const int     wave = threadIdx.x >> 6;
    const int     g    = lane >> 4;
    uint32_t      chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * (4u * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const int      ib = static_cast<int>(a.idxBits);
    const i32x4*   tA = static_cast<const i32x4*>(a.tileA);
    const i32x4*   tP = static_cast<const i32x4*>(a.tileP);

    // frame operands (B fragments) of covariance 0; per-lane frame = frame0 + 16 cb + (lane & 15)
    i32x4      B[NF][KS];
    int        ssCol[NF];  // MULTI: sum sq of the column's frame for the current covariance
    uint32_t   curCov = 0;
    const auto loadB  = [&](uint32_t cov) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            const uint32_t f = frame0 + cb * 16 + (lane & 15);
            const i32x4*   q = reinterpret_cast<const i32x4*>(
                    a.frameQ + (static_cast<size_t>(cov) * a.nFramesPad + f) * (KS * 64)) + g;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                B[cb][ks] = q[ks * 4];
            if constexpr (MULTI)
                ssCol[cb] = a.frameSS[static_cast<size_t>(cov) * a.nFramesPad + f];
        }
    };
    loadB(0);
    int ssOut[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i)
        ssOut[i] = MULTI ? 0 : a.frameSS[frame0 + 64 * i + lane];

    uint32_t t = a.mixTileOff[m0];
    i32x4    An[KS];
    i32x4    Pn;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
        An[ks] = tA[(static_cast<size_t>(t) * KS + ks) * 64 + lane];
    Pn = tP[static_cast<size_t>(t) * 4 + g];

    for (uint32_t m = m0; m < m1; ++m) {
        const uint32_t tEnd = a.mixTileOff[m + 1];
        int            best[NF][4];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                best[cb][r] = INT_MAX;

        for (; t < tEnd; ++t) {
            i32x4 A[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                A[ks] = An[ks];
            const i32x4 P = Pn;
            // prefetch the next tile (arrays carry one padding tile at the end)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                An[ks] = tA[(static_cast<size_t>(t + 1) * KS + ks) * 64 + lane];
            Pn = tP[static_cast<size_t>(t + 1) * 4 + g];
            if constexpr (MULTI) {
                const uint32_t cov = a.tileCov[t];
                if (cov != curCov) {
                    curCov = cov;
                    loadB(cov);
                }
            }
#pragma unroll
            for (int cb = 0; cb < NF; ++cb) {
                i32x4 acc = {0, 0, 0, 0};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[ks], B[cb][ks], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    // packed = (c + sum a'^2 + 2 dot(-a', b')) << ib | density   (see gmm_prepare.cc)
                    int v = static_cast<int>((static_cast<uint32_t>(acc[r]) << (ib + 1)) + static_cast<uint32_t>(P[r]));
                    if constexpr (MULTI)
                        v = static_cast<int>(static_cast<uint32_t>(v) + (static_cast<uint32_t>(ssCol[cb]) << ib));
                    best[cb][r] = min(best[cb][r], v);
                }
            }
        }

        // per-mixture reduction: 4 rows in-lane, then a reduce-scatter over the 4 lane groups
        int v[NF];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            v[cb] = min(min(best[cb][0], best[cb][1]), min(best[cb][2], best[cb][3]));
        const bool hi1 = (g >> 1) & 1, hi0 = g & 1;
        int        w[NF / 2];  // after the xor-32 step: column blocks cb with bit1 == hi1
#pragma unroll
        for (int p = 0; p < NF / 2; ++p) {
            const int c    = (p & 1) | ((p >> 1) << 2);  // 0,1,4,5: bit1 clear
            const int send = hi1 ? v[c] : v[c ^ 2];
            const int keep = hi1 ? v[c ^ 2] : v[c];
            w[p]           = min(keep, __shfl_xor(send, 32));
        }
        int res[NPL];  // result for column block cb = g + 4 i
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const int send = hi0 ? w[2 * i] : w[2 * i + 1];
            const int keep = hi0 ? w[2 * i + 1] : w[2 * i];
            res[i]         = min(keep, __shfl_xor(send, 16));
        }

        const uint32_t mo = m - a.mixBase;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const uint32_t f = frame0 + 64 * i + lane;
            if (f >= a.nFrames)
                continue;
            const int packed = res[i];
            int       q;
            uint32_t  dns;
            if (packed == INT_MAX) {  // mixture without densities: minScore stays Core::Type<int>::max
                q   = INT_MAX;
                dns = 0xffffffffu;
            }
            else {
                q   = (packed >> ib) + ssOut[i];
                dns = static_cast<uint32_t>(packed) & ((1u << ib) - 1u);
            }
            float score;
            if (a.flavor == 0)  // SimdFeatureScorer.cc:142: 0.5 * q / scalingSquared_ in double
                score = static_cast<float>(0.5 * static_cast<double>(q) / static_cast<double>(a.s2));
            else  // BatchFeatureScorer.cc:468: (f32)best / scale_
                score = __fdiv_rn(static_cast<float>(q), a.batchScale);
            if (a.outScale != 1.0f)
                score = __fmul_rn(a.outScale, score);  // ScaledContextScorer::score, ScaledFeatureScorer.hh:62-64
            const size_t o = static_cast<size_t>(mo) * a.scoreStride + f;
            a.scores[o]    = score;
            if (a.best)
                a.best[o] = dns;
        }
    }
}

// ---------------------------------------------------------------------------
// float scorer
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lexMin(float& v, uint32_t& i, float v2, uint32_t i2) {
    const bool take = (v2 < v) || (v2 == v && i2 < i);
    v               = take ? v2 : v;
    i               = take ? i2 : i;
}

template <int NF, int KS, bool MULTI>
__global__ __launch_bounds__(256) void scoreF32(F32Args a) {
    static_assert(NF == 4 || NF == 8, "NF");
    constexpr int NPL = NF / 4;
    const int     lane = threadIdx.x & 63;
    const int     wave = threadIdx.x >> 6;
    const int     g    = lane >> 4;
    uint32_t      chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * (4u * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t fb0    = frame0 / 16u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t nFB = a.nFramesPad / 16u;

    float      B[NF][KS];
    uint32_t   curCov = 0;
    const auto loadB  = [&](uint32_t cov) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            const float* x = a.frameX + ((static_cast<size_t>(cov) * nFB + fb0 + cb) * KS) * 64 + lane;
#pragma unroll
            for (int s = 0; s < KS; ++s)
                B[cb][s] = x[s * 64];
        }
    };
    loadB(0);
    float xxOut[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i)
        xxOut[i] = MULTI ? 0.0f : a.frameXX[frame0 + 64 * i + lane];

    uint32_t t = a.mixTileOff[m0];
    float    An[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
        An[s] = a.tileA[(static_cast<size_t>(t) * KS + s) * 64 + lane];

    for (uint32_t m = m0; m < m1; ++m) {
        const uint32_t tBeg = t, tEnd = a.mixTileOff[m + 1];
        float          best[NF][4];
        uint32_t       bt[NF][4];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                best[cb][r] = 3.40282347e+38f;
                bt[cb][r]   = 0;
            }

        for (; t < tEnd; ++t) {
            float A[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s)
                A[s] = An[s];
#pragma unroll
            for (int s = 0; s < KS; ++s)
                An[s] = a.tileA[(static_cast<size_t>(t + 1) * KS + s) * 64 + lane];
            if constexpr (MULTI) {
                const uint32_t cov = a.tileCov[t];
                if (cov != curCov) {
                    curCov = cov;
                    loadB(cov);
                }
            }
            f32x4 acc[NF];
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                acc[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
                    acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], B[cb][s], acc[cb], 0, 0, 0);
            const uint32_t tl = t - tBeg;
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool lt = acc[cb][r] < best[cb][r];  // strict: earliest tile wins ties
                    best[cb][r]   = lt ? acc[cb][r] : best[cb][r];
                    bt[cb][r]     = lt ? tl : bt[cb][r];
                }
        }

        // density index of each candidate, then lexicographic (score, density) reduction
        float    v[NF];
        uint32_t vi[NF];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            v[cb]  = 3.40282347e+38f;
            vi[cb] = 0xffffffffu;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (!(best[cb][r] < 3.40282347e+38f))
                    continue;
                const uint32_t row = 4u * g + r;
                uint32_t       dns;
                if constexpr (MULTI)
                    dns = a.rowDns[(static_cast<size_t>(tBeg) + bt[cb][r]) * 16 + row];
                else
                    dns = bt[cb][r] * 16u + row;
                lexMin(v[cb], vi[cb], best[cb][r], dns);
            }
        }
        const bool hi1 = (g >> 1) & 1, hi0 = g & 1;
        float      w[NF / 2];
        uint32_t   wi[NF / 2];
#pragma unroll
        for (int p = 0; p < NF / 2; ++p) {
            const int      c  = (p & 1) | ((p >> 1) << 2);
            const float    sv = hi1 ? v[c] : v[c ^ 2];
            const uint32_t si = hi1 ? vi[c] : vi[c ^ 2];
            float          kv = hi1 ? v[c ^ 2] : v[c];
            uint32_t       ki = hi1 ? vi[c ^ 2] : vi[c];
            lexMin(kv, ki, __shfl_xor(sv, 32), static_cast<uint32_t>(__shfl_xor(static_cast<int>(si), 32)));
            w[p]  = kv;
            wi[p] = ki;
        }
        const uint32_t mo = m - a.mixBase;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const float    sv = hi0 ? w[2 * i] : w[2 * i + 1];
            const uint32_t si = hi0 ? wi[2 * i] : wi[2 * i + 1];
            float          kv = hi0 ? w[2 * i + 1] : w[2 * i];
            uint32_t       ki = hi0 ? wi[2 * i + 1] : wi[2 * i];
            lexMin(kv, ki, __shfl_xor(sv, 16), static_cast<uint32_t>(__shfl_xor(static_cast<int>(si), 16)));
            const uint32_t f = frame0 + 64 * i + lane;
            if (f >= a.nFrames)
                continue;
            float score;
            if (ki == 0xffffffffu) {  // no density: bestScore stays Core::Type<Score>::max
                score = a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f;
            }
            else {
                const float total = MULTI ? kv : __fadd_rn(kv, xxOut[i]);
                score             = a.flavor == 2 ? 0.5f * total : (total < 3.40282347e+38f ? 0.5f * total : total);
            }
            if (a.outScale != 1.0f)
                score = __fmul_rn(a.outScale, score);
            const size_t o = static_cast<size_t>(mo) * a.scoreStride + f;
            a.scores[o]    = score;
            if (a.best)
                a.best[o] = ki;
        }
    }
}

}  // namespace dev

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
using dev::prepareFramesF32;
using dev::prepareFramesI8;

hipError_t launchPrepareFramesI8(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesPad,
                                 uint32_t nFramesRead, uint32_t D, uint32_t C, uint32_t KS, const float* isv,
                                 int8_t* frameQ, int32_t* frameSS, hipStream_t stream) {
    const uint32_t n = C * nFramesRead;
    hipLaunchKernelGGL(prepareFramesI8, dim3((n + 255) / 256), dim3(256), 0, stream, frames, nFrames, frameStride,
                       nFramesPad, nFramesRead, D, C, KS, isv, frameQ, frameSS);
    return hipGetLastError();
}

hipError_t launchPrepareFramesF32(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesPad,
                                  uint32_t nFramesRead, uint32_t D, uint32_t C, uint32_t KS, int foldNorm,
                                  const float* isv, float* frameX, float* frameXX, hipStream_t stream) {
    const uint32_t n = C * nFramesRead;
    hipLaunchKernelGGL(prepareFramesF32, dim3((n + 255) / 256), dim3(256), 0, stream, frames, nFrames, frameStride,
                       nFramesPad, nFramesRead, D, C, KS, foldNorm, isv, frameX, frameXX);
    return hipGetLastError();
}

template <int NF, int KS, bool MULTI>
static void launchI8T(const I8Args& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::scoreI8<NF, KS, MULTI>), dim3(grid), dim3(256), 0, s, a);
}

hipError_t launchScoreI8(const I8Args& a, uint32_t kSteps, bool multiCov, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    if (kSteps == 1)
        multiCov ? launchI8T<kI8NF, 1, true>(a, grid, stream) : launchI8T<kI8NF, 1, false>(a, grid, stream);
    else if (kSteps == 2)
        multiCov ? launchI8T<kI8NF, 2, true>(a, grid, stream) : launchI8T<kI8NF, 2, false>(a, grid, stream);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

template <int KS>
static void launchF32K(const F32Args& a, bool multi, uint32_t grid, hipStream_t s) {
    if (multi)
        hipLaunchKernelGGL((dev::scoreF32<kF32NF, KS, true>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dev::scoreF32<kF32NF, KS, false>), dim3(grid), dim3(256), 0, s, a);
}

hipError_t launchScoreF32(const F32Args& a, uint32_t kSteps, bool multiCov, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    switch (kSteps) {
        case 2: launchF32K<2>(a, multiCov, grid, stream); break;
        case 4: launchF32K<4>(a, multiCov, grid, stream); break;
        case 6: launchF32K<6>(a, multiCov, grid, stream); break;
        case 8: launchF32K<8>(a, multiCov, grid, stream); break;
        case 10: launchF32K<10>(a, multiCov, grid, stream); break;
        case 12: launchF32K<12>(a, multiCov, grid, stream); break;
        case 14: launchF32K<14>(a, multiCov, grid, stream); break;
        case 16: launchF32K<16>(a, multiCov, grid, stream); break;
        case 20: launchF32K<20>(a, multiCov, grid, stream); break;
        case 24: launchF32K<24>(a, multiCov, grid, stream); break;
        case 28: launchF32K<28>(a, multiCov, grid, stream); break;
        case 32: launchF32K<32>(a, multiCov, grid, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rasr_gmm
