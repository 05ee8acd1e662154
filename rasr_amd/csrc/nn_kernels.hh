// nn_kernels.hh -- launch interface of the hybrid-DNN scorer kernels (nn_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rasr_nn {

constexpr uint32_t kNnTileM = 256;  // output units per workgroup tile (nnGemm8p: 8 waves, 128 KiB LDS)
constexpr uint32_t kNnTileN = 256;  // frames per workgroup tile
constexpr uint32_t kNnTileK = 64;            // K per pipeline stage

// One layer: Out = act(A . B^T + bias) with A = W^T [Mpad][Kpad] (bf16 bits), B = layer input
// [Npad][Kpad] (bf16 bits, frame-major).  Hidden layers store Y [Npad][Mpad] bf16 (the next
// layer's B); the top layer stores scores[m * scoreStride + n] = -(A . B^T + bias)[m][n] for
// m < M, n < nFrames.
struct NnGemmArgs {
    const uint16_t* A;
    const uint16_t* B;
    const float*    bias;      // [Mpad]
    uint16_t*       Y;         // hidden layers
    float*          scores;    // top layer
    uint32_t        Mpad, Kpad, Npad, M, nFrames, scoreStride;
    int             act;       // nn_activation
    float           gamma;
    int             top;
    int             swapped;   // top layer computed as C^T (A = activations, B = W^T): set by launchNnGemm
    // nnGemm128 split-K (hidden layers of calls that leave most CUs idle): kSplit workgroups per tile sum K
    // ranges into part [kSplit][Npad][Mpad] f32, nnSplitReduce adds them in split order + bias + activation
    uint32_t        kSplit;    // 0 / 1: no split
    float*          part;
};

hipError_t launchNnPrepareInput(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t D,
                                uint32_t Kpad, uint16_t* X, hipStream_t stream);
hipError_t launchNnGemm(const NnGemmArgs& a, hipStream_t stream);
// calls of up to kNnSmallFrames frames (Npad = the frames rounded up to 16, beyond 64 to 64): one 16-unit row block
// x <= 64 frames per workgroup (nnGemmSmall)
#ifndef NN_SMALL_FRAMES
#define NN_SMALL_FRAMES 128  // split-K nnGemm128 beyond (profiles/r04/s32: 102 vs 117 us at 128, 155 vs 117 at 160)
#endif
constexpr uint32_t kNnSmallFrames = NN_SMALL_FRAMES;
hipError_t launchNnGemmSmall(const NnGemmArgs& a, hipStream_t stream);
// layers whose nnGemm8p grid would have fewer than kNnTile128Wgs workgroups (Npad a multiple of 256): 128 x 128
// tiles (nnGemm128), 4x the workgroups
#ifndef NN_TILE128_WGS
#define NN_TILE128_WGS 192  // profiles/r04/s30: 2048-unit layers on nnGemm128 up to 5888 frames
#endif
constexpr uint32_t kNnTile128Wgs = NN_TILE128_WGS;
hipError_t launchNnGemm128(const NnGemmArgs& a, hipStream_t stream);
// split-K workspace of a scorer: kSplit x Npad x Mpad f32 of a hidden layer split when its 128-tile grid is below
// kNnSplitWgs, kSplit = min(kNnMaxSplit, 2 kNnSplitWgs / grid): <= 2 x kNnSplitWgs x 128 x 128 floats
constexpr uint32_t kNnSplitWgs = 192, kNnMaxSplit = 8;
constexpr size_t   kNnSplitFloats = static_cast<size_t>(2u * kNnSplitWgs) * 128u * 128u;

}  // namespace rasr_nn
