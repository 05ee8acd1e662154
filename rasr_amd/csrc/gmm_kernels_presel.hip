// gmm_kernels_presel.hip -- density preselection of "preselection-batch-float" / "preselection-batch-int"
// (src/Mm/BatchFeatureScorer.cc:238-289, 478-533; src/Mm/DensityClustering.{hh,tcc}).
//
// The reference scores, per frame, only the densities whose cluster is among the frame's
// select-clusters nearest density clusters (a CPU saving).  On the matrix cores every density of a tile
// is computed anyway, so here the preselection is a per-(frame, cluster) mask applied in the scoring
// kernels' epilogue (gmm_kernels_split.hip, gmm_kernels_i8.hip); this file builds the mask:
//
//   assignDensities  k-means assignment step of DensityClustering::build (one thread per density,
//                    distances summed in the reference order, strict < keeps the first nearest);
//   selectClusters   selectClusters per frame: the distance to every cluster, the rank of each
//                    distance by counting, and -- only for a frame with a tie across the selection
//                    boundary -- a replay of the reference's std::sort along the partition path that
//                    holds the boundary (gmm_refsort.hh), so the selection equals the reference's also
//                    on ties.
//
// Mask layout (read by the scorers' lanes straight from LDS): for every block of 64 frames, every
// cluster c and t = frame % 16 one u32 whose byte cb = (frame % 64) / 16 is 0x00 (c selected) or 0xff
// (not selected): OR-ed, sign-extended, into a scorer's (value | tag) key it turns a deselected density
// into the all-ones key, which never wins the minimum.
#include "gmm_device.hh"
#include "gmm_refsort.hh"

namespace rasr_gmm {
namespace dev {

template <bool INT>
struct PreselTypes;
template <>
struct PreselTypes<false> {
    typedef float Feature;
    typedef float Distance;
};
template <>
struct PreselTypes<true> {
    typedef uint8_t Feature;
    typedef int32_t Distance;
};

// unrolledVectorDistance (src/Mm/Utilities.hh:244-284), one component: score += (a - b)^2 in the
// element type's arithmetic (f32 without contraction: the reference is an SSE build without FMA)
__device__ __forceinline__ float addSq(float s, float a, float b) {
    const float d = __fsub_rn(a, b);
    return __fadd_rn(s, __fmul_rn(d, d));
}
__device__ __forceinline__ int32_t addSq(int32_t s, int32_t a, int32_t b) {
    const int32_t d = a - b;
    return s + d * d;
}

// ---------------------------------------------------------------------------
// DensityClustering::assignDensities (DensityClustering.tcc:80-99)
// ---------------------------------------------------------------------------
template <bool INT, int DPMAX>
__global__ __launch_bounds__(256) void assignDensities(const void* __restrict__ meansV, uint32_t nDensities, uint32_t Dp,
                                                       const void* __restrict__ clusterMeansV, uint32_t nClusters,
                                                       uint8_t* __restrict__ clusterOf) {
    typedef typename PreselTypes<INT>::Feature  F;
    typedef typename PreselTypes<INT>::Distance Dist;
    const F*       means = static_cast<const F*>(meansV);
    const F*       cm    = static_cast<const F*>(clusterMeansV);
    const uint32_t e     = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nDensities)
        return;
    Dist row[DPMAX];
#pragma unroll
    for (int k = 0; k < DPMAX; ++k)
        row[k] = k < static_cast<int>(Dp) ? static_cast<Dist>(means[static_cast<size_t>(e) * Dp + k]) : Dist(0);
    Dist     best = 0;
    uint32_t bc   = 0;
    for (uint32_t c = 0; c < nClusters; ++c) {
        Dist s = 0;
#pragma unroll
        for (int k = 0; k < DPMAX; ++k)
            if (k < static_cast<int>(Dp))
                s = addSq(s, static_cast<Dist>(cm[static_cast<size_t>(c) * Dp + k]), row[k]);
        if (c == 0 || s < best) {
            best = s;
            bc   = c;
        }
    }
    clusterOf[e] = static_cast<uint8_t>(bc);
}

// ---------------------------------------------------------------------------
// DensityClustering::selectClusters (DensityClustering.tcc:151-176) for kSelFrames frames per workgroup
// ---------------------------------------------------------------------------
constexpr int kSelFrames = 16;
constexpr int kSelMaxDp  = 128;

template <bool INT>
__global__ __launch_bounds__(256) void selectClusters(const float* __restrict__ frames, uint32_t nFrames,
                                                      uint32_t frameStride, uint32_t D, uint32_t Dp,
                                                      const float* __restrict__ variance,
                                                      const void* __restrict__ clusterMeansV, uint32_t nClusters,
                                                      uint32_t nSelected, uint32_t* __restrict__ selT) {
    typedef typename PreselTypes<INT>::Feature  F;
    typedef typename PreselTypes<INT>::Distance Dist;
    __shared__ Dist    feat[kSelFrames][kSelMaxDp];
    __shared__ Dist    dist[kSelFrames][256];
    __shared__ uint8_t idx[kSelFrames][256];
    __shared__ uint8_t sel[kSelFrames][256];
    __shared__ int     ambiguous[kSelFrames];
    const F*           cm  = static_cast<const F*>(clusterMeansV);
    const uint32_t     f0  = blockIdx.x * kSelFrames;
    const uint32_t     tid = threadIdx.x;
    if (tid < kSelFrames)
        ambiguous[tid] = 0;
    // setFeature (BatchFeatureScorer.cc:137-142 float: x * isv; 382-388 int: quantize(x * isv * s)),
    // zero-padded to the padded dimension
    for (uint32_t i = tid; i < kSelFrames * Dp; i += blockDim.x) {
        const uint32_t f = i / Dp, k = i % Dp, frame = f0 + f;
        Dist           v = 0;
        if (frame < nFrames && k < D) {
            const float x = __fmul_rn(frames[static_cast<size_t>(frame) * frameStride + k], variance[k]);
            if constexpr (INT)
                v = quantizeCentered(x) + 128;  // quantize<f32, u8>
            else
                v = x;
        }
        feat[f][k] = v;
    }
    __syncthreads();
    const uint32_t c = tid;
    if (c < nClusters) {
        Dist acc[kSelFrames];
#pragma unroll
        for (int f = 0; f < kSelFrames; ++f)
            acc[f] = 0;
        for (uint32_t k = 0; k < Dp; ++k) {
            const Dist m = static_cast<Dist>(cm[static_cast<size_t>(c) * Dp + k]);
#pragma unroll
            for (int f = 0; f < kSelFrames; ++f)
                acc[f] = addSq(acc[f], feat[f][k], m);  // unrolledVectorDistance(feature, clusterMean)
        }
#pragma unroll
        for (int f = 0; f < kSelFrames; ++f)
            dist[f][c] = acc[f];
    }
    __syncthreads();
    // rank by counting: less = #{d_j < d_c}, equal = #{d_j == d_c}.  Selected when less + equal <=
    // select-clusters, deselected when less >= select-clusters, otherwise the order std::sort gives
    // the tied clusters decides (and a NaN distance leaves the order to the replay as well)
    if (c < nClusters) {
        for (int f = 0; f < kSelFrames; ++f) {
            const Dist d    = dist[f][c];
            uint32_t   less = 0, equal = 0;
            for (uint32_t j = 0; j < nClusters; ++j) {
                const Dist v = dist[f][j];
                less += v < d ? 1u : 0u;
                equal += v == d ? 1u : 0u;
            }
            sel[f][c] = less + equal <= nSelected ? 1 : 0;
            if (!(d == d) || (less < nSelected && less + equal > nSelected))
                ambiguous[f] = 1;
        }
    }
    __syncthreads();
    if (tid < kSelFrames && ambiguous[tid]) {
        const int f = static_cast<int>(tid);
        for (uint32_t j = 0; j < nClusters; ++j)
            idx[f][j] = static_cast<uint8_t>(j);
        RefSortRange<Dist, uint8_t> s{dist[f], idx[f]};
        s.selectFirst(static_cast<int>(nClusters), static_cast<int>(nSelected));  // the set sort leaves in [0, k)
        for (uint32_t j = 0; j < nClusters; ++j)
            sel[f][j] = 0;
        for (uint32_t i = 0; i < nSelected; ++i)
            sel[f][idx[f][i]] = 1;
    }
    __syncthreads();
    // mask bytes: the workgroup's 16 frames share the 64-frame block and the byte cb, t = f
    if (c < nClusters) {
        uint8_t* out = reinterpret_cast<uint8_t*>(selT) + (static_cast<size_t>(f0 / 64) * nClusters + c) * 64 +
                       (f0 % 64) / 16;
#pragma unroll
        for (int f = 0; f < kSelFrames; ++f)
            out[4 * f] = sel[f][c] ? 0x00 : 0xff;
    }
}

// ---------------------------------------------------------------------------
// the quantized scorer's per-wave mask table (gmm_kernels_i8.hip scoreI8Seg<PRESEL>, 128 frames per wave), built
// once per call from the byte mask: for every group of 128 frames, cluster c and t = frame % 16 one byte, bit j:
// frame 16 j + t of the group did not select c (j = 0..7) -- the index of the u64 in the scorer's LDS look-up table
// that expands the 8 bits into one 0x00 / 0xff byte per column block.  4 KiB per 128 frames at 256 clusters (an
// eighth of the byte mask, which every chunk's workgroups would otherwise re-read and compress): with the frame
// operands, a 32768-frame call's 3 MiB stay in an XCD's L2 while its workgroups walk their chunks.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void compactSelection(const uint32_t* __restrict__ selT, uint32_t nGroups,
                                                        uint32_t nClusters, uint8_t* __restrict__ selC) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;  // (group, cluster, t)
    if (i >= nGroups * nClusters * 16u)
        return;
    const uint32_t t = i % 16u, c = (i / 16u) % nClusters, grp = i / (16u * nClusters);
    const uint32_t w0 = selT[(static_cast<size_t>(2 * grp) * nClusters + c) * 16u + t];
    const uint32_t w1 = selT[(static_cast<size_t>(2 * grp + 1) * nClusters + c) * 16u + t];
    const auto     nib = [](uint32_t w) { return ((w & 0x01010101u) * 0x01020408u) >> 24 & 0xfu; };  // bit q = byte q
    selC[i]            = static_cast<uint8_t>(nib(w0) | nib(w1) << 4);
}

}  // namespace dev

hipError_t launchCompactSelection(const uint32_t* selT, uint32_t nFramesRead, uint32_t nClusters, uint8_t* selC,
                                  hipStream_t stream) {
    if (nFramesRead % 128 || nClusters > 256)
        return hipErrorInvalidValue;
    const uint32_t n = nFramesRead / 128 * nClusters * 16;
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::compactSelection, dim3((n + 255) / 256), dim3(256), 0, stream, selT, nFramesRead / 128,
                       nClusters, selC);
    return hipGetLastError();
}

hipError_t launchAssignDensities(bool quantized, const void* means, uint32_t nDensities, uint32_t Dp,
                                 const void* clusterMeans, uint32_t nClusters, uint8_t* clusterOf, hipStream_t stream) {
    if (nDensities == 0)
        return hipSuccess;
    const dim3 grid((nDensities + 255) / 256), block(256);
    if (Dp <= 64) {
        if (quantized)
            hipLaunchKernelGGL((dev::assignDensities<true, 64>), grid, block, 0, stream, means, nDensities, Dp,
                               clusterMeans, nClusters, clusterOf);
        else
            hipLaunchKernelGGL((dev::assignDensities<false, 64>), grid, block, 0, stream, means, nDensities, Dp,
                               clusterMeans, nClusters, clusterOf);
    }
    else if (Dp <= 128) {
        if (quantized)
            hipLaunchKernelGGL((dev::assignDensities<true, 128>), grid, block, 0, stream, means, nDensities, Dp,
                               clusterMeans, nClusters, clusterOf);
        else
            hipLaunchKernelGGL((dev::assignDensities<false, 128>), grid, block, 0, stream, means, nDensities, Dp,
                               clusterMeans, nClusters, clusterOf);
    }
    else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launchSelectClusters(bool quantized, const float* frames, uint32_t nFrames, uint32_t frameStride,
                                uint32_t nFramesRead, uint32_t D, uint32_t Dp, const float* variance,
                                const void* clusterMeans, uint32_t nClusters, uint32_t nSelected, uint32_t* selT,
                                hipStream_t stream) {
    if (Dp > static_cast<uint32_t>(dev::kSelMaxDp) || nClusters > 256 || nFramesRead % 64)
        return hipErrorInvalidValue;  // the kernel's LDS arrays and the mask's 64-frame blocks
    const uint32_t nBlocks = nFramesRead / dev::kSelFrames;
    if (nBlocks == 0)
        return hipSuccess;
    if (quantized)
        hipLaunchKernelGGL(dev::selectClusters<true>, dim3(nBlocks), dim3(256), 0, stream, frames, nFrames, frameStride,
                           D, Dp, variance, clusterMeans, nClusters, nSelected, selT);
    else
        hipLaunchKernelGGL(dev::selectClusters<false>, dim3(nBlocks), dim3(256), 0, stream, frames, nFrames,
                           frameStride, D, Dp, variance, clusterMeans, nClusters, nSelected, selT);
    return hipGetLastError();
}

}  // namespace rasr_gmm
