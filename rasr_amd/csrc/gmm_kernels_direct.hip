// gmm_kernels_direct.hip -- the float scorers in the reference's own operation order
// (GMM_FLAG_REFERENCE_ORDER): scores bit-identical to the CPU restatement of the reference binary
// (the CPU restatement under oracle/, compiled with the reference's -O2 -ffast-math -msse3), at VALU speed.
//
//   diagonal-maximum (GaussDiagonalMaximumFeatureScorer::calculateScoreAndDensity/distance,
//   GaussDiagonalMaximumFeatureScorer.cc:116-181): per density four lane sums over k = j (mod 4) of
//   ((mu - x) * isv)^2 for k < D & ~3 (subps, mulps, mulps, addps: every operation rounded), the lane
//   sums added pairwise (s0 + s1) + (s2 + s3) (_mm_hadd_ps), then the remaining D % 4 terms in order;
//   score = ((f64) dist + (f64) minus2LogWeight) + (f64) logNorm (the order -ffast-math gives the
//   reference's three-term sum, checked in the compiled oracle); best kept as f32, replaced when
//   (f64) best > score (strict: the lowest density on ties); result 0.5f * best.
//   batch-diagonal-maximum-float (BatchFloatFeatureScorer::fillScoreCacheTpl, BatchFeatureScorer.cc:
//   187-234): means and frames pre-multiplied by isv (f32); per 8-dimension block two 4-lane sums
//   s1 (constant in lane 0) and s2 of (m - x)^2; v = s1 + s2; (v3 + v1) + (v2 + v0); minimum in f32
//   (minss: the old score unless the new value is smaller); 0.5 * score unless FLT_MAX.
//
// One frame per lane, 64 frames per wave, 256 per workgroup; a workgroup walks a chunk of mixtures
// (chunks x frame tiles, XCD-aware as the other scorers).  Every density's mean, isv row and constants
// are wave-uniform and read through the scalar cache; the frame (Dp floats) stays in VGPRs, so the
// kernel is instantiated for the number of 4-dimension blocks it can hold.
#include "gmm_device.hh"

namespace rasr_gmm {
namespace dev {

// Read-only model tables through the scalar data cache: the constant address space makes the wave-uniform
// loads below s_load (the kernel's stores go elsewhere; nothing writes these tables).
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cst(const T* p) {
    return (const __attribute__((address_space(4))) T*)p;
}

// Row layout (host, gmm_api.cc prepareDirect), L = 4 NB + 4 floats per mean / isv row and per frame:
// diagonal-maximum: dims 0 .. 4 nfb - 1 in the first 4 nfb slots (zeros up to 4 NB), the D % 4 remaining
// dims in the last 4 slots (zeros after them); batch-float: dims 0 .. D - 1, zeros up to 4 NB.  Zero slots
// add exactly +0 to a non-negative sum, so every density runs the same branch-free code.
template <int NB, bool BATCH, bool MULTI>
__global__ __launch_bounds__(256) void scoreDirect(DirectArgs a) {
    constexpr int L    = 4 * NB + 4;
    const int     lane = threadIdx.x & 63;
    const int     wave = threadIdx.x >> 6;
    uint32_t      chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t f  = ft * kDirectFramesPerBlock + static_cast<uint32_t>(wave) * 64u + static_cast<uint32_t>(lane);
    const bool     in = f < a.nFrames;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t D = a.D, nfb = D / 4u;

    // the frame in the row layout: diagonal-maximum raw, batch-float times isv (setFeature,
    // BatchFeatureScorer.cc:138-143)
    float x[L];
#pragma unroll
    for (int k = 0; k < L; ++k) {
        // source dimension of slot k (or none)
        uint32_t src = 0xffffffffu;
        if constexpr (BATCH)
            src = k < 4 * NB && static_cast<uint32_t>(k) < D ? static_cast<uint32_t>(k) : 0xffffffffu;
        else if (k < 4 * NB)
            src = static_cast<uint32_t>(k) < 4u * nfb ? static_cast<uint32_t>(k) : 0xffffffffu;
        else
            src = 4u * nfb + static_cast<uint32_t>(k - 4 * NB) < D ? 4u * nfb + static_cast<uint32_t>(k - 4 * NB)
                                                                   : 0xffffffffu;
        float v = 0.0f;
        if (in && src != 0xffffffffu) {
            v = a.frames[static_cast<size_t>(f) * a.frameStride + src];
            if constexpr (BATCH)
                v = __fmul_rn(v, a.isv[k]);
        }
        x[k] = v;
    }
    // one covariance: its isv row in registers
    float ivr[MULTI ? 1 : L];
    if constexpr (!MULTI) {
#pragma unroll
        for (int k = 0; k < L; ++k)
            ivr[k] = a.isv[k];
    }
    const auto mixOff   = cst(a.mixOff);
    const auto meanT    = cst(a.mean);
    const auto isvT     = cst(a.isv);
    const auto entryCov = cst(a.entryCov);
    const auto constant = cst(a.constant);
    const auto logNorm  = cst(a.logNorm);

    for (uint32_t m = m0; m < m1; ++m) {
        const uint32_t e0 = mixOff[m], e1 = mixOff[m + 1];
        float          best    = 3.40282347e+38f;  // Core::Type<Score>::max
        uint32_t       bestIdx = 0xffffffffu;
        for (uint32_t i = e0; i < e1; ++i) {
            const auto mu = meanT + static_cast<size_t>(i) * L;
            if constexpr (!BATCH) {
                const uint32_t cov = MULTI ? entryCov[i] : 0u;
                const auto     iv  = isvT + static_cast<size_t>(cov) * L;
                float          s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    const int   k  = 4 * b;
                    const float d0 = __fmul_rn(__fsub_rn(mu[k], x[k]), MULTI ? iv[k] : ivr[k]);
                    const float d1 = __fmul_rn(__fsub_rn(mu[k + 1], x[k + 1]), MULTI ? iv[k + 1] : ivr[k + 1]);
                    const float d2 = __fmul_rn(__fsub_rn(mu[k + 2], x[k + 2]), MULTI ? iv[k + 2] : ivr[k + 2]);
                    const float d3 = __fmul_rn(__fsub_rn(mu[k + 3], x[k + 3]), MULTI ? iv[k + 3] : ivr[k + 3]);
                    s0 = __fadd_rn(s0, __fmul_rn(d0, d0));
                    s1 = __fadd_rn(s1, __fmul_rn(d1, d1));
                    s2 = __fadd_rn(s2, __fmul_rn(d2, d2));
                    s3 = __fadd_rn(s3, __fmul_rn(d3, d3));
                }
                float r = __fadd_rn(__fadd_rn(s0, s1), __fadd_rn(s2, s3));
#pragma unroll
                for (int j = 0; j < 3; ++j) {  // the D % 4 remaining terms, in order (zero slots add +0)
                    const int   k = 4 * NB + j;
                    const float d = __fmul_rn(__fsub_rn(mu[k], x[k]), MULTI ? iv[k] : ivr[k]);
                    r             = __fadd_rn(r, __fmul_rn(d, d));
                }
                const double score = __dadd_rn(__dadd_rn(static_cast<double>(r), static_cast<double>(constant[i])),
                                               static_cast<double>(logNorm[cov]));
                if (static_cast<double>(best) > score) {
                    best    = static_cast<float>(score);
                    bestIdx = i - e0;
                }
            }
            else {
                float p0 = constant[i], p1 = 0.0f, p2 = 0.0f, p3 = 0.0f;  // s1 = _mm_load_ss(constant)
                float q0 = 0.0f, q1 = 0.0f, q2 = 0.0f, q3 = 0.0f;         // s2
#pragma unroll
                for (int b = 0; b < NB / 2; ++b) {
                    const int   k  = 8 * b;
                    const float u0 = __fsub_rn(mu[k], x[k]), u1 = __fsub_rn(mu[k + 1], x[k + 1]);
                    const float u2 = __fsub_rn(mu[k + 2], x[k + 2]), u3 = __fsub_rn(mu[k + 3], x[k + 3]);
                    p0 = __fadd_rn(p0, __fmul_rn(u0, u0));
                    p1 = __fadd_rn(p1, __fmul_rn(u1, u1));
                    p2 = __fadd_rn(p2, __fmul_rn(u2, u2));
                    p3 = __fadd_rn(p3, __fmul_rn(u3, u3));
                    const float w0 = __fsub_rn(mu[k + 4], x[k + 4]), w1 = __fsub_rn(mu[k + 5], x[k + 5]);
                    const float w2 = __fsub_rn(mu[k + 6], x[k + 6]), w3 = __fsub_rn(mu[k + 7], x[k + 7]);
                    q0 = __fadd_rn(q0, __fmul_rn(w0, w0));
                    q1 = __fadd_rn(q1, __fmul_rn(w1, w1));
                    q2 = __fadd_rn(q2, __fmul_rn(w2, w2));
                    q3 = __fadd_rn(q3, __fmul_rn(w3, w3));
                }
                const float v0 = __fadd_rn(p0, q0), v1 = __fadd_rn(p1, q1), v2 = __fadd_rn(p2, q2),
                            v3 = __fadd_rn(p3, q3);
                const float val = __fadd_rn(__fadd_rn(v3, v1), __fadd_rn(v2, v0));
                best            = best < val ? best : val;  // minss
            }
        }
        if (in) {
            float score;
            if constexpr (BATCH)
                score = best < 3.40282347e+38f ? __fmul_rn(best, 0.5f) : best;
            else
                score = __fmul_rn(0.5f, best);
            if (a.outScale != 1.0f)
                score = __fmul_rn(a.outScale, score);  // ScaledContextScorer::score
            const size_t o = static_cast<size_t>(m) * a.scoreStride + f;
            a.scores[o]    = score;
            if (!BATCH && a.best)
                a.best[o] = bestIdx;
        }
    }
}

}  // namespace dev

template <int NB>
static void launchDirectNB(const DirectArgs& a, bool multi, uint32_t grid, hipStream_t s) {
    if (a.batch)
        hipLaunchKernelGGL((dev::scoreDirect<NB, true, false>), dim3(grid), dim3(256), 0, s, a);
    else if (multi)
        hipLaunchKernelGGL((dev::scoreDirect<NB, false, true>), dim3(grid), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((dev::scoreDirect<NB, false, false>), dim3(grid), dim3(256), 0, s, a);
}

// 4-dimension blocks of the row layout for dimension D (diagonal-maximum: D / 4 whole blocks, the rest in
// the tail slots; batch-float: the padded dimension, a multiple of 8, over 4)
uint32_t directBlocks(uint32_t D, bool batch) {
    const uint32_t need = batch ? (D + 7u) / 8u * 2u : D / 4u;
    for (uint32_t nb : {2u, 4u, 6u, 8u, 10u, 12u, 16u, 24u, 32u})
        if (need <= nb)
            return nb;
    return 0;  // D > 128
}

hipError_t launchScoreDirect(const DirectArgs& a, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    const uint32_t nb = directBlocks(a.D, a.batch != 0);
    if (nb == 0 || a.Dp != 4u * nb + 4u)  // the host laid the rows out for exactly this instantiation
        return hipErrorInvalidValue;
    const bool multi = a.multiCov != 0;
    switch (nb) {
        case 2: launchDirectNB<2>(a, multi, grid, stream); break;
        case 4: launchDirectNB<4>(a, multi, grid, stream); break;
        case 6: launchDirectNB<6>(a, multi, grid, stream); break;
        case 8: launchDirectNB<8>(a, multi, grid, stream); break;
        case 10: launchDirectNB<10>(a, multi, grid, stream); break;
        case 12: launchDirectNB<12>(a, multi, grid, stream); break;
        case 16: launchDirectNB<16>(a, multi, grid, stream); break;
        case 24: launchDirectNB<24>(a, multi, grid, stream); break;
        default: launchDirectNB<32>(a, multi, grid, stream); break;
    }
    return hipGetLastError();
}

}  // namespace rasr_gmm
