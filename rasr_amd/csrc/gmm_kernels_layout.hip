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

}  // namespace dev

hipError_t launchTransposeWords(const uint32_t* src, uint32_t rows, uint32_t cols, uint32_t srcPitch, uint32_t* dst,
                                uint32_t dstPitch, hipStream_t stream) {
    if (rows == 0 || cols == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::transposeWords, dim3((cols + 63u) / 64u, (rows + 63u) / 64u), dim3(256), 0, stream, src, rows,
                       cols, srcPitch, dst, dstPitch);
    return hipGetLastError();
}

}  // namespace rasr_gmm
