// gmm_device.hh -- device helpers shared by the MI355X scorer kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "gmm_kernels.hh"

namespace rasr_gmm {
namespace dev {

typedef int   i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef GMM_STORE_CPOL
// cache policy of the score-table stores: 2 = non-temporal (nt).  The table is written once and never
// re-read by the kernel; streaming it leaves the L2 to the model tiles every frame tile of a chunk
// re-reads (A/B, profiles/r02/ab/ab_store_nt.txt: -1.4 % fp32, -0.35 % SIMD)
#define GMM_STORE_CPOL 2
#endif
#ifndef GMM_I8_LDS
#define GMM_I8_LDS 1  // quantized kernel, one covariance: tiles staged through LDS (scoreI8Seg)
#endif

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

__device__ __forceinline__ void lexMin(float& v, uint32_t& i, float v2, uint32_t i2) {
    const bool take = (v2 < v) || (v2 == v && i2 < i);
    v               = take ? v2 : v;
    i               = take ? i2 : i;
}

// Cross-lane exchanges of the per-mixture reduce-scatter, as VALU permutes (no LDS round trip).
// v_permlane32_swap(x, y) swaps x's lanes 32..63 with y's lanes 0..31; v_permlane16_swap(x, y)
// swaps x's odd 16-lane rows with y's even rows.  Taking min(x', y') afterwards leaves, in every
// lane, the minimum over the lane and its partner (lane ^ 32, resp. lane ^ 16) of x in the lanes
// that keep x and of y in the lanes that keep y: one swap + one min per exchanged pair.
// Read-only per-launch tables (mixture tile offsets, mixture words) through the constant address space: a uniform
// load from it is an s_load wherever it sits.  Through a generic pointer, a load after the kernel's own buffer stores
// (the emit) cannot be proven unclobbered, so the compiler makes it a vector load plus v_readfirstlane and waits
// s_waitcnt vmcnt(0) for it -- draining every tile load (or LDS-DMA) in flight at each mixture boundary.
#ifndef GMM_CONST_TABLES
#define GMM_CONST_TABLES 1
#endif
#if GMM_CONST_TABLES
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* constTable(const T* p) {
    return (const __attribute__((address_space(4))) T*)p;
}
#else
template <class T>
__device__ __forceinline__ const T* constTable(const T* p) {
    return p;
}
#endif
__device__ __forceinline__ int swapMin32(int x, int y) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
    return min(static_cast<int>(r[0]), static_cast<int>(r[1]));
}
__device__ __forceinline__ int swapMin16(int x, int y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    return min(static_cast<int>(r[0]), static_cast<int>(r[1]));
}
__device__ __forceinline__ void swapLexMin32(float xv, uint32_t xi, float yv, uint32_t yi, float& v, uint32_t& i) {
    const auto rv = __builtin_amdgcn_permlane32_swap(__float_as_uint(xv), __float_as_uint(yv), false, false);
    const auto ri = __builtin_amdgcn_permlane32_swap(xi, yi, false, false);
    v             = __uint_as_float(rv[0]);
    i             = ri[0];
    lexMin(v, i, __uint_as_float(rv[1]), ri[1]);
}
__device__ __forceinline__ void swapLexMin16(float xv, uint32_t xi, float yv, uint32_t yi, float& v, uint32_t& i) {
    const auto rv = __builtin_amdgcn_permlane16_swap(__float_as_uint(xv), __float_as_uint(yv), false, false);
    const auto ri = __builtin_amdgcn_permlane16_swap(xi, yi, false, false);
    v             = __uint_as_float(rv[0]);
    i             = ri[0];
    lexMin(v, i, __uint_as_float(rv[1]), ri[1]);
}

}  // namespace dev
}  // namespace rasr_gmm
