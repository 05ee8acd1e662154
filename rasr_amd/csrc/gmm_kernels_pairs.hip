// gmm_kernels_pairs.hip -- best densities of a list of (frame, mixture) pairs (gmm_best_density_pairs).
//
// An aligner reads bestDensity(e) for one to a few emissions per frame (AssigningFeatureScorer.hh:110-121,
// AbstractMixtureSetEstimator.cc:370-384), not the whole [mixture][frame] table the keyed scorers write.  This
// kernel answers such a list from frames that are still on the device: one wave per pair, its 64 lanes score 64
// of the mixture's entries at a time in the reference's own arithmetic, and every lane then walks the 64 values
// in entry order (v_readlane: the running best is wave-uniform), so the reference's scan order and tie rule hold
// as written, including its order-dependent float compare:
//   * SIMD-diagonal-maximum (SimdFeatureScorer.cc:135-176): the frame quantized per covariance as the scorer's
//     frame preparation does (quantize(x * isv * s)), the u8 sum of squared differences with the prepared means
//     plus the constant weight (int32), replaced when strictly smaller (lowest entry on ties) -- bit-exact;
//   * diagonal-maximum (GaussDiagonalMaximumFeatureScorer.cc:116-181): the reference-order f32 distance of the
//     direct scorer (gmm_kernels_direct.hip: four lane sums over 4-dimension blocks, pairwise, then the D % 4
//     tail), the f64 three-term score, the f32-stored best replaced when (f64) best > score;
//   * diagonal-sum (GaussDiagonalMaximumFeatureScorer.cc:238-286): the same distance, the f32 score
//     0.5 ((w + logNorm) + dist), the minimum by a strict f32 compare.
// The keyed table scorers compute the float types' best densities on the split-f16 MFMA path; on a near tie
// (scores within the float tolerance) the two may name different densities, as either may differ from the
// CPU restatement (tests/test_best_pairs.py).
// Sparse work by design: a pair costs one mixture's entries x D, so the kernel is latency-bound and unremarkable
// in throughput; the gain is the table it does not compute (an aligner's frame asks for ~1-10 of ~5000 mixtures).
#include "gmm_device.hh"

#include <cfloat>

namespace rasr_gmm {
namespace dev {

__device__ __forceinline__ uint32_t readLane(uint32_t v, uint32_t j) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(j)));
}

// reference-order f32 distance of entry i (gmm_kernels_direct.hip, MULTI): frame slot k of the row layout is
// dimension k for k < 4 nfb, dimension 4 nfb + j for the tail slot 4 nb + j, none otherwise (zero)
__device__ __forceinline__ float refDistance(const PairArgs& a, const float* x, uint32_t i, uint32_t cov) {
    const float*   mu  = a.fMean + static_cast<size_t>(i) * a.L;
    const float*   iv  = a.isv + static_cast<size_t>(cov) * a.L;
    const uint32_t nfb = a.D / 4u;
    float          s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
    for (uint32_t b = 0; b < a.nb; ++b) {
        const uint32_t k  = 4u * b;
        const bool     in = b < nfb;
        const float    x0 = in ? x[k] : 0.0f, x1 = in ? x[k + 1] : 0.0f, x2 = in ? x[k + 2] : 0.0f,
                    x3 = in ? x[k + 3] : 0.0f;
        const float d0 = __fmul_rn(__fsub_rn(mu[k], x0), iv[k]);
        const float d1 = __fmul_rn(__fsub_rn(mu[k + 1], x1), iv[k + 1]);
        const float d2 = __fmul_rn(__fsub_rn(mu[k + 2], x2), iv[k + 2]);
        const float d3 = __fmul_rn(__fsub_rn(mu[k + 3], x3), iv[k + 3]);
        s0             = __fadd_rn(s0, __fmul_rn(d0, d0));
        s1             = __fadd_rn(s1, __fmul_rn(d1, d1));
        s2             = __fadd_rn(s2, __fmul_rn(d2, d2));
        s3             = __fadd_rn(s3, __fmul_rn(d3, d3));
    }
    float r = __fadd_rn(__fadd_rn(s0, s1), __fadd_rn(s2, s3));
    for (uint32_t j = 0; j < 3u; ++j) {
        const uint32_t k  = 4u * a.nb + j, dim = 4u * nfb + j;
        const float    xv = dim < a.D ? x[dim] : 0.0f;
        const float    d  = __fmul_rn(__fsub_rn(mu[k], xv), iv[k]);
        r                 = __fadd_rn(r, __fmul_rn(d, d));
    }
    return r;
}

template <int KIND>
__global__ __launch_bounds__(256) void bestPairs(PairArgs a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t p    = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (p >= a.nPairs)
        return;
    const uint32_t f = a.pairFrame[p], m = a.pairMix[p];
    uint32_t       bestIdx = 0xffffffffu;  // Core::Type<size_t>::max as DensityInMixture: none
    if (f < a.nFrames && m < a.nMixtures) {
        const float*   x  = a.frames + static_cast<size_t>(f) * a.frameStride;
        const uint32_t e0 = a.mixOff[m], e1 = a.mixOff[m + 1];
        int32_t        bestI = INT_MAX;  // Core::Type<int>::max (SimdFeatureScorer.cc:160)
        float          bestF = FLT_MAX;  // Core::Type<Score>::max
        for (uint32_t base = e0; base < e1; base += 64u) {
            const uint32_t i = base + lane;
            uint32_t       v0 = 0, v1 = 0;  // this lane's entry value (f64: two words)
            if (i < e1) {
                const uint32_t cov = a.entryCov[i];
                if constexpr (KIND == kPairSimd) {
                    const uint8_t* mu = a.qMean + static_cast<size_t>(i) * a.Dp;
                    const float*   iv = a.isv + static_cast<size_t>(cov) * a.isvStride;
                    uint32_t       ss = 0;
                    for (uint32_t k = 0; k < a.D; ++k) {
                        const int d = static_cast<int>(mu[k]) - (quantizeCentered(__fmul_rn(x[k], iv[k])) + 128);
                        ss += static_cast<uint32_t>(d * d);
                    }
                    v0 = static_cast<uint32_t>(a.qConst[i]) + ss;  // int score = constant + l2norm (wraps as int)
                }
                else if constexpr (KIND == kPairDiagonalMaximum) {
                    const float  r = refDistance(a, x, i, cov);
                    // GDMFS.cc:129-132: ((f64) w + (f64) logNorm) + (f64) distance
                    const double s = __dadd_rn(__dadd_rn(static_cast<double>(a.fConst[i]),
                                                         static_cast<double>(a.fLogNorm[cov])),
                                               static_cast<double>(r));
                    const uint64_t b = static_cast<uint64_t>(__double_as_longlong(s));
                    v0               = static_cast<uint32_t>(b);
                    v1               = static_cast<uint32_t>(b >> 32);
                }
                else {
                    const float r = refDistance(a, x, i, cov);
                    // GDMFS.cc:255-257: (w + logNorm) + distance in f32
                    const float s = __fadd_rn(__fadd_rn(a.fConst[i], a.fLogNorm[cov]), r);
                    v0            = __float_as_uint(__fmul_rn(0.5f, s));
                }
            }
            // the reference's scan, in entry order, over this block's values (wave-uniform)
            const uint32_t n = min(64u, e1 - base);
            for (uint32_t j = 0; j < n; ++j) {
                if constexpr (KIND == kPairSimd) {
                    const int32_t s = static_cast<int32_t>(readLane(v0, j));
                    if (s < bestI) {
                        bestI   = s;
                        bestIdx = base + j - e0;
                    }
                }
                else if constexpr (KIND == kPairDiagonalMaximum) {
                    const double s = __longlong_as_double(static_cast<long long>(
                            (static_cast<uint64_t>(readLane(v1, j)) << 32) | readLane(v0, j)));
                    if (static_cast<double>(bestF) > s) {  // GDMFS.cc:133-136: the f32-stored best against f64
                        bestF   = static_cast<float>(s);
                        bestIdx = base + j - e0;
                    }
                }
                else {
                    const float s = __uint_as_float(readLane(v0, j));
                    if (bestF > s) {
                        bestF   = s;
                        bestIdx = base + j - e0;
                    }
                }
            }
        }
    }
    if (lane == 0)
        a.best[p] = bestIdx;
}

}  // namespace dev

hipError_t launchBestPairs(const PairArgs& a, hipStream_t stream) {
    if (a.nPairs == 0)
        return hipSuccess;
    const dim3 grid((a.nPairs + 3u) / 4u);
    switch (a.kind) {
        case kPairSimd: hipLaunchKernelGGL(dev::bestPairs<kPairSimd>, grid, dim3(256), 0, stream, a); break;
        case kPairDiagonalMaximum:
            hipLaunchKernelGGL(dev::bestPairs<kPairDiagonalMaximum>, grid, dim3(256), 0, stream, a);
            break;
        case kPairDiagonalSum: hipLaunchKernelGGL(dev::bestPairs<kPairDiagonalSum>, grid, dim3(256), 0, stream, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rasr_gmm
