// nn_kernels.hip -- the hybrid-DNN scorer's layers on gfx950: one bf16 GEMM per layer with the bias,
// the activation (or, on the top layer, the negation into the class-major score table) fused into
// the epilogue.
//
// GEMM: C[M x N] = A[M x K] . B[N x K]^T, A = W^T (output units x inputs), B = activations (frames x
// inputs), both K-contiguous, so both MFMA operands are 16-byte row pieces.  A 256-thread workgroup
// computes a 128 x 128 tile as 2 x 2 waves of 64 x 64 (4 x 4 v_mfma_f32_16x16x32_bf16 accumulators);
// K advances in 64-wide stages staged global -> LDS by global_load_lds_dwordx4 (each wave issues 4 x
// 1 KiB for A and for B), double-buffered: the next stage's DMA is in flight while the current one is
// read, with a counted s_waitcnt vmcnt and raw s_barriers (a __syncthreads would drain the DMA).
// LDS rows are 128 B (64 bf16); the 16-byte piece c of row r sits at piece c ^ (r & 7), so the 16
// lanes of a ds_read_b128 that read one piece of 16 consecutive rows spread over the banks; the
// swizzle is applied on the per-lane global source address (the LDS side of global_load_lds is
// lane-linear).  Workgroups are mapped so that the ones sharing an XCD sweep the output-unit tiles of
// one frame tile (its activations stay in that XCD's L2).
#include "nn_kernels.hh"

namespace rasr_nn {
namespace dev {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float  f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float activate(float x, int act, float gamma) {
    switch (act) {
        case 1: return 1.0f / (1.0f + __expf(-gamma * x));  // SigmoidLayer
        case 2: return tanhf(x);                           // TanhLayer
        case 3: return x > 0.0f ? x : 0.0f;                // RectifiedLayer
        case 4: return x > 0.0f ? x : __expf(x) - 1.0f;    // ExponentialLinearLayer (alpha 1)
        default: return x;                                 // IdentityLayer
    }
}

__device__ __forceinline__ uint16_t toBf16(float x) {
    return __builtin_bit_cast(uint16_t, static_cast<__bf16>(x));  // v_cvt_pk_bf16_f32, RNE, NaN kept
}

__global__ __launch_bounds__(256) void nnPrepareInput(const float* __restrict__ frames, uint32_t nFrames,
                                                      uint32_t frameStride, uint32_t D, uint32_t Kpad,
                                                      uint16_t* __restrict__ X) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nFrames * D)
        return;
    const uint32_t t = i / D, k = i % D;
    X[static_cast<size_t>(t) * Kpad + k] = toBf16(frames[static_cast<size_t>(t) * frameStride + k]);
}

__global__ __launch_bounds__(256, 2) void nnGemm(NnGemmArgs a) {
    __shared__ __attribute__((aligned(16))) uint16_t lds[2][2][kNnTileM * kNnTileK];  // [stage][A|B], one array

    const int      lane = threadIdx.x & 63;
    const int      wave = threadIdx.x >> 6;
    const uint32_t nMT = a.Mpad / kNnTileM, nNT = a.Npad / kNnTileN, nwg = nMT * nNT;
    // bijective XCD remap: blocks b, b+8, ... (one XCD) get consecutive tile ids
    const uint32_t b = blockIdx.x, xcd = b & 7u, q = nwg / 8u, r = nwg % 8u;
    const uint32_t id = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (b >> 3);
    const uint32_t m0 = (id % nMT) * kNnTileM, n0 = (id / nMT) * kNnTileN;
    const uint32_t wr = static_cast<uint32_t>(wave) >> 1, wc = static_cast<uint32_t>(wave) & 1u;

    // stage s <- K columns [k0, k0 + 64): 16 pieces of 8 rows x 128 B per operand, 4 per wave
    const uint32_t prow = static_cast<uint32_t>(lane) >> 3, ppos = static_cast<uint32_t>(lane) & 7u;
    const auto     issue = [&](int s, uint32_t k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t piece = static_cast<uint32_t>(wave) * 4u + i;
            const uint32_t row   = piece * 8u + prow;
            const uint32_t c     = ppos ^ (row & 7u);
            __builtin_amdgcn_global_load_lds(a.A + static_cast<size_t>(m0 + row) * a.Kpad + k0 + 8u * c,
                                             &lds[s][0][piece * 512u], 16, 0, 0);
            __builtin_amdgcn_global_load_lds(a.B + static_cast<size_t>(n0 + row) * a.Kpad + k0 + 8u * c,
                                             &lds[s][1][piece * 512u], 16, 0, 0);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    const uint32_t nK = a.Kpad / kNnTileK;
    issue(0, 0);
    for (uint32_t kt = 0; kt < nK; ++kt) {
        const int s = static_cast<int>(kt & 1u);
        if (kt + 1 < nK) {
            issue(s ^ 1, (kt + 1) * kNnTileK);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this stage's 8 DMAs landed, the next 8 fly
        }
        else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // every wave's pieces of stage s are in LDS
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8         fa[4], fb[4];
            const uint32_t c = static_cast<uint32_t>(ks) * 4u + (static_cast<uint32_t>(lane) >> 4);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t ra = wr * 64u + 16u * i + (static_cast<uint32_t>(lane) & 15u);
                const uint32_t rb = wc * 64u + 16u * i + (static_cast<uint32_t>(lane) & 15u);
                fa[i] = *reinterpret_cast<const bf16x8*>(&lds[s][0][ra * 64u + ((c ^ (ra & 7u)) * 8u)]);
                fb[i] = *reinterpret_cast<const bf16x8*>(&lds[s][1][rb * 64u + ((c ^ (rb & 7u)) * 8u)]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage s is free for the DMA of stage kt + 2
    }

    // epilogue: rows m = m0 + 64 wr + 16 i + 4 (lane >> 4) + rr, frame n = n0 + 64 wc + 16 j + (lane & 15)
    const uint32_t g = static_cast<uint32_t>(lane) >> 4, col = static_cast<uint32_t>(lane) & 15u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t mb = m0 + wr * 64u + 16u * i + 4u * g;
        const f32x4    bs = *reinterpret_cast<const f32x4*>(a.bias + mb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t n = n0 + wc * 64u + 16u * j + col;
            if (a.top) {
                if (n < a.nFrames)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        if (mb + rr < a.M)
                            a.scores[static_cast<size_t>(mb + rr) * a.scoreStride + n] = -(acc[i][j][rr] + bs[rr]);
            }
            else {
                u16x4 v;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    v[rr] = toBf16(activate(acc[i][j][rr] + bs[rr], a.act, a.gamma));
                *reinterpret_cast<u16x4*>(a.Y + static_cast<size_t>(n) * a.Mpad + mb) = v;
            }
        }
    }
}

}  // namespace dev

hipError_t launchNnPrepareInput(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t D,
                                uint32_t Kpad, uint16_t* X, hipStream_t stream) {
    const uint32_t n = nFrames * D;
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::nnPrepareInput, dim3((n + 255) / 256), dim3(256), 0, stream, frames, nFrames, frameStride,
                       D, Kpad, X);
    return hipGetLastError();
}

hipError_t launchNnGemm(const NnGemmArgs& a, hipStream_t stream) {
    if (a.Mpad % kNnTileM || a.Npad % kNnTileN || a.Kpad % kNnTileK || a.Kpad == 0)
        return hipErrorInvalidValue;  // the kernel reads whole tiles without bounds checks
    const uint32_t nwg = (a.Mpad / kNnTileM) * (a.Npad / kNnTileN);
    if (nwg == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::nnGemm, dim3(nwg), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace rasr_nn
