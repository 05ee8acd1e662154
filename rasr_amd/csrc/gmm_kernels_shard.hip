// gmm_kernels_shard.hip -- exchange format of the density-sharded layout (BASELINE config 4).
//
// When a mixture's densities are split over GPUs, each GPU's score for it is a partial minimum over
// its part.  The partial (score, best density) pairs are packed into one int64 key per (mixture,
// frame) whose signed order is the reference's order of candidates -- lower score first, then the
// lower density index (the strict < of SimdFeatureScorer.cc:158-176) -- so an RCCL all-reduce with
// MIN over the keys is the per-frame reduce, and unpacking restores (score, density).
//
//   key = (s32(score) << 32) | density,   s32(score) = float bits as a signed int whose order is the
//                                          float order (negative floats: bits ^ 0x7fffffff; -0 as +0)
//
// Scores are monotone transforms of the kernels' minima (0.5 q / s^2, 0.5 (v - K0), scale > 0), so the
// minimum of partial scores is the score of the minimum.
#include "gmm_device.hh"

namespace rasr_gmm {
namespace dev {

__device__ __forceinline__ int32_t orderedBits(float s) {
    const uint32_t u = __float_as_uint(s) == 0x80000000u ? 0u : __float_as_uint(s);  // -0 == +0 (strict < ties)
    return static_cast<int32_t>(u >= 0x80000000u ? u ^ 0x7fffffffu : u);
}

__device__ __forceinline__ float unorderedBits(int32_t v) {
    const uint32_t u = static_cast<uint32_t>(v);
    return __uint_as_float(u >= 0x80000000u ? u ^ 0x7fffffffu : u);
}

__global__ __launch_bounds__(256) void packShardKeys(const float* __restrict__ scores, const uint32_t* __restrict__ best,
                                                     const uint32_t* __restrict__ bestOffset, uint32_t rows,
                                                     uint32_t nFrames, uint32_t stride, int64_t* __restrict__ keys) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= static_cast<size_t>(rows) * nFrames)
        return;
    const uint32_t r = static_cast<uint32_t>(i / nFrames), t = static_cast<uint32_t>(i % nFrames);
    const size_t   o = static_cast<size_t>(r) * stride + t;
    uint32_t       d = 0;
    if (best) {
        d = best[o];
        if (d != 0xffffffffu && bestOffset)
            d += bestOffset[r];
    }
    const uint64_t k = (static_cast<uint64_t>(static_cast<uint32_t>(orderedBits(scores[o]))) << 32) | d;
    keys[i]          = static_cast<int64_t>(k);
}

__global__ __launch_bounds__(256) void unpackShardKeys(const int64_t* __restrict__ keys, uint32_t rows, uint32_t nFrames,
                                                       float* __restrict__ scores, uint32_t* __restrict__ best,
                                                       uint32_t stride) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= static_cast<size_t>(rows) * nFrames)
        return;
    const uint32_t r = static_cast<uint32_t>(i / nFrames), t = static_cast<uint32_t>(i % nFrames);
    const size_t   o = static_cast<size_t>(r) * stride + t;
    const uint64_t k = static_cast<uint64_t>(keys[i]);
    scores[o]        = unorderedBits(static_cast<int32_t>(static_cast<uint32_t>(k >> 32)));
    if (best)
        best[o] = static_cast<uint32_t>(k);
}

// identity of the per-frame reduce: the keys of split mixtures a GPU holds no part of
__global__ __launch_bounds__(256) void fillShardKeys(int64_t* __restrict__ keys, size_t n) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n)
        keys[i] = INT64_MAX;
}

// the per-frame reduce of the copy exchange: out[i] = min over the slots' keys (slot j at slots + j * n)
__global__ __launch_bounds__(256) void minShardKeys(const int64_t* __restrict__ slots, uint32_t nSlots, size_t n,
                                                    int64_t* __restrict__ out) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    int64_t k = slots[i];
    for (uint32_t j = 1; j < nSlots; ++j)
        k = min(k, slots[j * n + i]);
    out[i] = k;
}

// the device-local fold of the RCCL exchange: another part's keys on the same GPU into the GPU's first part's
__global__ __launch_bounds__(256) void minIntoShardKeys(int64_t* __restrict__ dst, const int64_t* __restrict__ src,
                                                        size_t n) {
    const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n)
        dst[i] = min(dst[i], src[i]);
}

}  // namespace dev

hipError_t launchPackShardKeys(const float* scores, const uint32_t* best, const uint32_t* bestOffset, uint32_t rows,
                               uint32_t nFrames, uint32_t stride, int64_t* keys, hipStream_t stream) {
    const size_t n = static_cast<size_t>(rows) * nFrames;
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::packShardKeys, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, stream, scores,
                       best, bestOffset, rows, nFrames, stride, keys);
    return hipGetLastError();
}

hipError_t launchUnpackShardKeys(const int64_t* keys, uint32_t rows, uint32_t nFrames, float* scores, uint32_t* best,
                                 uint32_t stride, hipStream_t stream) {
    const size_t n = static_cast<size_t>(rows) * nFrames;
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::unpackShardKeys, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, stream, keys,
                       rows, nFrames, scores, best, stride);
    return hipGetLastError();
}

hipError_t launchFillShardKeys(int64_t* keys, size_t n, hipStream_t stream) {
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::fillShardKeys, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, stream, keys, n);
    return hipGetLastError();
}

hipError_t launchMinShardKeys(const int64_t* slots, uint32_t nSlots, size_t n, int64_t* out, hipStream_t stream) {
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::minShardKeys, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, stream, slots,
                       nSlots, n, out);
    return hipGetLastError();
}

hipError_t launchMinIntoShardKeys(int64_t* dst, const int64_t* src, size_t n, hipStream_t stream) {
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::minIntoShardKeys, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, stream, dst, src,
                       n);
    return hipGetLastError();
}

}  // namespace rasr_gmm
