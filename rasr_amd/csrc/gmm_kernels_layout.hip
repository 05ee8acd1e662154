// gmm_kernels_layout.hip -- frame-major copies of the score tables for host callers.
//
// The scorer kernels write mixture-major tables ([mixture][frame], BatchFeatureScorerBase::scores_,
// src/Mm/BatchFeatureScorer.hh:177-186): lane l stores frame frame0 + l, 256 contiguous bytes per wave.
// A host caller that reads a frame's scores for all (or the active) mixtures -- the search through
// ContextScorer::score(e), FeatureScorerNode's dump -- walks a mixture-major table with a stride of the
// whole buffer per emission, one cache miss per score on the host.  gmm_score_host_ring with
// GMM_HOST_FRAME_MAJOR therefore transposes each chunk on the device (this kernel, an HBM-bound pass of
// 2 x 4 B per (frame, mixture) at a few TB/s) and copies contiguous frame rows over PCIe.
#include "gmm_device.hh"

#include <algorithm>

namespace rasr_gmm {
namespace dev {

// dst[c * dstPitch + r] = src[r * srcPitch + c] for r < rows, c < cols (32-bit words); 64 x 64 tiles through
// LDS (row pitch 65 words: the column reads of the store phase hit 64 different banks), 256 threads
__global__ __launch_bounds__(256) void transposeWords(const uint32_t* __restrict__ src, uint32_t rows, uint32_t cols,
                                                      uint32_t srcPitch, uint32_t* __restrict__ dst, uint32_t dstPitch) {
    __shared__ uint32_t tile[64][65];
    const uint32_t tx = threadIdx.x & 63u, ty = threadIdx.x >> 6;
    const uint32_t r0 = blockIdx.y * 64u, c0 = blockIdx.x * 64u;
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t r = r0 + ty + 4u * i, c = c0 + tx;
        if (r < rows && c < cols)
            tile[ty + 4u * i][tx] = src[static_cast<size_t>(r) * srcPitch + c];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t c = c0 + ty + 4u * i, r = r0 + tx;
        if (r < rows && c < cols)
            dst[static_cast<size_t>(c) * dstPitch + r] = tile[tx][ty + 4u * i];
    }
}

// dst[r * dstPitch + c] = src[r * srcPitch + c] for r < rows, c < cols (32-bit words): the small host calls' frame
// gather from a page-locked ring and table stores into page-locked caller tables (either side may be host memory
// mapped for the device; one row per 64-lane group, so a row's words go out as whole 256-byte bursts)
__global__ __launch_bounds__(256) void copyWords2D(const uint32_t* __restrict__ src, uint32_t srcPitch,
                                                   uint32_t* __restrict__ dst, uint32_t dstPitch, uint32_t rows,
                                                   uint32_t cols) {
    if (srcPitch == cols && dstPitch == cols) {  // one contiguous run (e.g. one frame's mixture-major column)
        const size_t n = static_cast<size_t>(rows) * cols;
        for (size_t i = static_cast<size_t>(blockIdx.x) * 256u + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256u)
            dst[i] = src[i];
        return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t r = blockIdx.x * 4u + (threadIdx.x >> 6); r < rows; r += gridDim.x * 4u)
        for (uint32_t c = lane; c < cols; c += 64u)
            dst[static_cast<size_t>(r) * dstPitch + c] = src[static_cast<size_t>(r) * srcPitch + c];
}

}  // namespace dev

hipError_t launchCopyWords2D(const uint32_t* src, uint32_t srcPitch, uint32_t* dst, uint32_t dstPitch, uint32_t rows,
                             uint32_t cols, hipStream_t stream) {
    if (rows == 0 || cols == 0)
        return hipSuccess;
    const uint32_t blocks = std::min<uint32_t>((rows + 3u) / 4u, 1024u);
    hipLaunchKernelGGL(dev::copyWords2D, dim3(blocks), dim3(256), 0, stream, src, srcPitch, dst, dstPitch, rows, cols);
    return hipGetLastError();
}

hipError_t launchTransposeWords(const uint32_t* src, uint32_t rows, uint32_t cols, uint32_t srcPitch, uint32_t* dst,
                                uint32_t dstPitch, hipStream_t stream) {
    if (rows == 0 || cols == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::transposeWords, dim3((cols + 63u) / 64u, (rows + 63u) / 64u), dim3(256), 0, stream, src, rows,
                       cols, srcPitch, dst, dstPitch);
    return hipGetLastError();
}

}  // namespace rasr_gmm
