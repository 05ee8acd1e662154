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
//
// This file: the float kernels (accumulators in AGPRs: measured faster for the f32 MFMA chains).
#include "gmm_device.hh"

namespace rasr_gmm {
namespace dev {

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
                                                         const float* __restrict__ isv,
                                                         const float* __restrict__ centre, float* __restrict__ frameX,
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
            const float v = __fmul_rn(__fsub_rn(x[k], centre[k]), iv[k]);
            xx            = __fadd_rn(xx, __fmul_rn(v, v));
        }
    float* base = frameX + (static_cast<size_t>(c) * (nFramesPad / 16) + f / 16) * KS * 64;
    for (uint32_t k = 0; k < KS * 4; ++k) {
        float v = 0.0f;
        if (valid) {
            if (k < D)
                v = __fmul_rn(__fsub_rn(x[k], centre[k]), iv[k]);
            else if (k == D)
                v = 1.0f;
            else if (k == D + 1 && foldNorm)
                v = xx;
        }
        base[(k >> 2) * 64 + (k & 3) * 16 + (f & 15)] = v;
    }
    frameXX[static_cast<size_t>(c) * nFramesPad + f] = xx;
}

template <int NF, int KS, bool MULTI>
#ifndef GMM_F32_MIN_WAVES
#define GMM_F32_MIN_WAVES 1  // __launch_bounds__ minimum waves per SIMD (register budget)
#endif
__global__ __launch_bounds__(256, GMM_F32_MIN_WAVES) void scoreF32(F32Args a) {
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
    // single covariance: ||x'||^2 of the lane's frame column is the MFMA chain's initial
    // accumulator, so a row's result is the whole (positive, see K0) distance + constant
    f32x4 XX[NF];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        const float xx = MULTI ? 0.0f : a.frameXX[frame0 + cb * 16 + (lane & 15)];
        XX[cb]         = f32x4{xx, xx, xx, xx};
    }

    uint32_t   t = a.mixTileOff[m0];
    float      A0[KS], A1[KS];
    const auto loadTile = [&](uint32_t tt, float(&A)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = a.tileA[(static_cast<size_t>(tt) * KS + s) * 64 + lane];
    };
    loadTile(t, A0);
    loadTile(t + 1, A1);
    const auto chain = [&](const float(&A)[KS], f32x4(&acc)[NF]) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            acc[cb] = MULTI ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} : XX[cb];
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s], B[cb][s], acc[cb], 0, 0, 0);
    };
    // key = value with its low tileBits mantissa bits replaced by the tile number (values are > 0):
    // one v_and_or per candidate and a float min keep (score, tile), lower tile on equal keys.
    const uint32_t tmask = (1u << a.tileBits) - 1u;
    const auto     key   = [&](float v, uint32_t tl) { return __uint_as_float((__float_as_uint(v) & ~tmask) | tl); };

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

        if constexpr (!MULTI) {
            // one tile per loop step (measured faster than two per step or a deferred epilogue,
            // DESIGN.md section 4)
            for (; t < tEnd;) {
                f32x4 accA[NF];
                chain(A0, accA);
                const uint32_t tl = t - tBeg;
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        best[cb][r] = fminf(best[cb][r], key(accA[cb][r], tl));
#pragma unroll
                for (int s = 0; s < KS; ++s)
                    A0[s] = A1[s];
                loadTile(t + 2, A1);
                ++t;
            }
        }
        else {
            for (; t < tEnd; ++t) {
                const uint32_t cov = a.tileCov[t];
                if (cov != curCov) {
                    curCov = cov;
                    loadB(cov);
                }
                f32x4 acc[NF];
                chain(A0, acc);
#pragma unroll
                for (int s = 0; s < KS; ++s)
                    A0[s] = A1[s];
                loadTile(t + 2, A1);
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
                const uint32_t row = 4u * g + r;
                float          val;
                uint32_t       dns;
                if constexpr (MULTI) {
                    val = best[cb][r];
                    if (!(val < 3.40282347e+38f))
                        continue;
                    dns = a.rowDns[(static_cast<size_t>(tBeg) + bt[cb][r]) * 16 + row];
                }
                else {
                    const uint32_t bits = __float_as_uint(best[cb][r]);
                    val                 = __uint_as_float(bits & ~tmask);
                    if (!(val < 1e37f))  // padding rows (constant FLT_MAX) or no tile
                        continue;
                    dns = (bits & tmask) * 16u + row;
                }
                lexMin(v[cb], vi[cb], val, dns);
            }
        }
        float    w[NF / 2];
        uint32_t wi[NF / 2];
#pragma unroll
        for (int p = 0; p < NF / 2; ++p) {
            const int c = (p & 1) | ((p >> 1) << 2);
            swapLexMin32(v[c], vi[c], v[c ^ 2], vi[c ^ 2], w[p], wi[p]);
        }
        const uint32_t mo = m - a.mixBase;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            float    kv;
            uint32_t ki;
            swapLexMin16(w[2 * i], wi[2 * i], w[2 * i + 1], wi[2 * i + 1], kv, ki);
            const uint32_t f = frame0 + 64 * i + lane;
            if (f >= a.nFrames)
                continue;
            float score;
            if (ki == 0xffffffffu) {  // no density: bestScore stays Core::Type<Score>::max
                score = a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f;
            }
            else {
                const float total = a.offsetK0 != 0.0f ? __fsub_rn(kv, a.offsetK0) : kv;
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

using dev::prepareFramesF32;

hipError_t launchPrepareFramesF32(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesPad,
                                  uint32_t nFramesRead, uint32_t D, uint32_t C, uint32_t KS, int foldNorm,
                                  const float* isv, const float* centre, float* frameX, float* frameXX,
                                  hipStream_t stream) {
    const uint32_t n = C * nFramesRead;
    hipLaunchKernelGGL(prepareFramesF32, dim3((n + 255) / 256), dim3(256), 0, stream, frames, nFrames, frameStride,
                       nFramesPad, nFramesRead, D, C, KS, foldNorm, isv, centre, frameX, frameXX);
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
