// nn_kernels.hip -- the hybrid-DNN scorer's layers on gfx950: one bf16 GEMM per layer with the bias,
// the activation (or, on the top layer, the negation into the class-major score table) fused into
// the epilogue.
//
// GEMM: C[M x N] = A[M x K] . B[N x K]^T, A = W^T (output units x inputs), B = activations (frames x
// inputs), both K-contiguous, so both MFMA operands are 16-byte row pieces.  Production kernel:
// nnGemm8p below (NN_GEMM_TILE 256, NN_GEMM_VARIANT 8); nnGemm256 (the two-half schedule) is kept for A/B.  nnGemm (NN_GEMM_TILE 128, kept for A/B): a 256-thread workgroup
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

#include <algorithm>

namespace rasr_nn {
namespace dev {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float  f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float  f32x16 __attribute__((ext_vector_type(16)));

#ifndef NN_SIGMOID_FMA
#define NN_SIGMOID_FMA 1  // hidden-layer sigmoid epilogue: bias and gamma folded into one FMA feeding v_exp_f32
#endif
#ifndef NN_FAST_TANH
#define NN_FAST_TANH 1
#endif
#ifndef NN_FAST_SIGMOID
#define NN_FAST_SIGMOID 1
#endif
__device__ __forceinline__ float activate(float x, int act, float gamma) {
    switch (act) {
#if NN_FAST_SIGMOID
        // SigmoidLayer; v_rcp_f32 (1 ulp) instead of the IEEE division sequence (~10 VALU per value in an
        // epilogue the matrix cores wait for): far below the bf16 rounding of the layer output
        case 1: return __builtin_amdgcn_rcpf(1.0f + __expf(-gamma * x));
#else
        case 1: return 1.0f / (1.0f + __expf(-gamma * x));  // SigmoidLayer
#endif
#if NN_FAST_TANH
        // TanhLayer as 1 - 2 / (2^(2 log2(e) x) + 1): v_exp_f32 + v_rcp_f32 instead of libm's tanhf.  That form
        // has an absolute error of ~1e-7, which near 0 is a large RELATIVE error (bf16 keeps small outputs to
        // 2^-9 relative), so |x| < 2^-4 takes x (1 - x^2 / 3) (the next term, 2 x^5 / 15, is < 2.1e-6 relative);
        // +-1 and NaN kept
        case 2: {
            const float x2 = x * x;
            return fabsf(x) < 0.0625f ? x * fmaf(x2, -0.333333343f, 1.0f)
                                      : 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(2.88539008177792681f * x));
        }
#else
        case 2: return tanhf(x);                           // TanhLayer
#endif
        case 3: return x > 0.0f ? x : 0.0f;                // RectifiedLayer
        // ExponentialLinearLayer (alpha 1): the reference's own form, alpha (exp(x) - 1) in T
        // (Math::FastMatrix::elu, src/Math/FastMatrix.hh:1656-1665), cancellation near 0- included
        case 4: return x > 0.0f ? x : __expf(x) - 1.0f;
        default: return x;                                 // IdentityLayer
    }
}

__device__ __forceinline__ uint16_t toBf16(float x) {
    return __builtin_bit_cast(uint16_t, static_cast<__bf16>(x));  // v_cvt_pk_bf16_f32, RNE, NaN kept
}

// one workgroup per frame, two features per thread, one 4-byte store of the bf16 pair (Kpad is a multiple of
// 64, so the pair never leaves the row; the feature after an odd D is written as 0, the padding's value)
__global__ __launch_bounds__(256) void nnPrepareInput(const float* __restrict__ frames, uint32_t nFrames,
                                                      uint32_t frameStride, uint32_t D, uint32_t Kpad,
                                                      uint16_t* __restrict__ X) {
    const uint32_t t = blockIdx.x;
    const float*   f = frames + static_cast<size_t>(t) * frameStride;
    uint32_t*      x = reinterpret_cast<uint32_t*>(X + static_cast<size_t>(t) * Kpad);
    for (uint32_t k = 2u * threadIdx.x; k < D; k += 512u) {
        const uint32_t lo = toBf16(f[k]);
        const uint32_t hi = k + 1u < D ? toBf16(f[k + 1u]) : 0u;
        x[k / 2u]         = lo | (hi << 16);
    }
}

__global__ __launch_bounds__(256) void nnGemm(NnGemmArgs a) {
    constexpr uint32_t kNnTileM = 128, kNnTileN = 128, kNnTileK = 64;  // this kernel's tile (NN_GEMM_TILE 128)
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

// ---------------------------------------------------------------------------
// nnGemm256: 256 x 256 output tile per 512-thread workgroup, 8 waves as 2 (units) x 4 (frames), each
// wave 128 x 64 (8 x 4 accumulators of v_mfma_f32_16x16x32_bf16).  K advances in 64-wide tiles, two
// LDS buffers of 64 KiB (A 256 rows | B 256 rows, 128-B rows) filled by global_load_lds_dwordx4 in
// half-tiles of 128 rows (16 KiB: two 1-KiB wave-instructions per wave).  Per K-tile u (buffer u & 1):
//   H0: stage A of tile u+1 (other buffer); s_waitcnt vmcnt(8) retires tile u (8 = the B of u+1 and
//       A of u+1 issued after it); barrier; read the wave's A rows 0..63 and all its B rows; 32 MFMAs;
//       barrier (B of buffer u & 1 free);
//   H1: stage B of tile u+2 (this buffer); read A rows 64..127; 32 MFMAs; barrier (A free).
// So B is prefetched ~3 half-steps and A ~2 ahead, one counted vmcnt per K-tile, never 0 in the loop
// (0 only when no later tile exists).  LDS rows: the 16-B piece c of row r sits at c ^ ((r >> 1) & 7):
// the 16 lanes of a ds_read_b128 group (16 consecutive rows, one piece) then hit 16 different 16-B
// bank slots (two 128-B rows share a 256-B bank row), conflict-free.
// ---------------------------------------------------------------------------
extern __shared__ __attribute__((aligned(16))) uint16_t nnLds[];  // [2 buffers][A | B][256 * 64]

#ifndef NN_GEMM_VARIANT
#define NN_GEMM_VARIANT 8  // 8: nnGemm8p (production); 0: nnGemm256 three barriers per K-tile (H0 | H1); 1: reads front-loaded, two barriers
#endif
#ifndef NN_GEMM_SETPRIO
#define NN_GEMM_SETPRIO 0  // s_setprio(1) around the MFMA clusters
#endif
#if NN_GEMM_SETPRIO
#define NN_SETPRIO(x) __builtin_amdgcn_s_setprio(x)
#else
#define NN_SETPRIO(x) ((void)0)
#endif

__device__ __forceinline__ uint32_t nnSwz(uint32_t r) {
    return (r >> 1) & 7u;
}

__global__ __launch_bounds__(512) void nnGemm256(NnGemmArgs a) {
    constexpr uint32_t T = 256, BK = 64, kOp = T * BK;  // elements per operand image
    const int          lane = threadIdx.x & 63;
    const int          wave = threadIdx.x >> 6;
    const uint32_t     nMT = a.Mpad / T, nNT = a.Npad / T, nwg = nMT * nNT;
    const uint32_t     b = blockIdx.x, xcd = b & 7u, q = nwg / 8u, r = nwg % 8u;
    const uint32_t     id = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (b >> 3);
    const uint32_t     m0 = (id % nMT) * T, n0 = (id / nMT) * T;
    const uint32_t     wr = static_cast<uint32_t>(wave) >> 2, wc = static_cast<uint32_t>(wave) & 3u;
    const uint32_t     nK = a.Kpad / BK;

    // half h (rows 128 h .. 128 h + 127) of operand op (0 = A, 1 = B) of K-tile u into buffer buf
    const auto stage = [&](int op, uint32_t h, uint32_t u, uint32_t buf) {
        const uint16_t* src  = op == 0 ? a.A : a.B;
        const uint32_t  base = op == 0 ? m0 : n0;
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i) {
            const uint32_t p   = static_cast<uint32_t>(wave) * 128u + i * 64u + static_cast<uint32_t>(lane);
            const uint32_t row = h * 128u + p / 8u;
            const uint32_t c   = (p % 8u) ^ nnSwz(row);
            __builtin_amdgcn_global_load_lds(src + static_cast<size_t>(base + row) * a.Kpad + u * BK + 8u * c,
                                             nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + h * (kOp / 2) +
                                                     (static_cast<uint32_t>(wave) * 128u + i * 64u) * 8u,
                                             16, 0, 0);
        }
    };
    const auto stageA = [&](uint32_t u, uint32_t buf) {
        stage(0, 0, u, buf);
        stage(0, 1, u, buf);
    };
    const auto stageB = [&](uint32_t u, uint32_t buf) {
        stage(1, 0, u, buf);
        stage(1, 1, u, buf);
    };
    const auto frag = [&](uint32_t buf, int op, uint32_t row, uint32_t ks) {
        const uint32_t c = ks * 4u + (static_cast<uint32_t>(lane) >> 4);
        return *reinterpret_cast<const bf16x8*>(nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + row * BK +
                                                (c ^ nnSwz(row)) * 8u);
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};

    const uint32_t rl = static_cast<uint32_t>(lane) & 15u;
    stageB(0, 0);
    stageA(0, 0);
    if (nK > 1)
        stageB(1, 1);
    for (uint32_t u = 0; u < nK; ++u) {
        const uint32_t buf = u & 1u;
        // H0
        if (u + 1 < nK) {
            stageA(u + 1, buf ^ 1u);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        }
        else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // every wave's pieces of tile u are in LDS
        bf16x8 fa[4][2], fb[4][2], fa2[4][2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                fb[j][ks] = frag(buf, 1, wc * 64u + 16u * j + rl, ks);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa[i][ks] = frag(buf, 0, wr * 128u + 16u * i + rl, ks);
        }
#if NN_GEMM_VARIANT == 1
        // all of the tile's reads up front (A rows 64..127 too), 64 MFMAs, one closing barrier
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa2[i][ks] = frag(buf, 0, wr * 128u + 64u + 16u * i + rl, ks);
#endif
        NN_SETPRIO(1);
#if NN_GEMM_VARIANT == 2
        // A rows 64..127 read in the middle of the first half's MFMAs (latency hidden behind 16 MFMAs)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa2[i][ks] = frag(buf, 0, wr * 128u + 64u + 16u * i + rl, ks);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], acc[i][j], 0, 0, 0);
        NN_SETPRIO(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // B of this buffer read by every wave
        if (u + 2 < nK)
            stageB(u + 2, buf);
        NN_SETPRIO(1);
#else
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[j][ks], acc[i][j], 0, 0, 0);
#endif
#if NN_GEMM_VARIANT == 0 || NN_GEMM_VARIANT == 3
        NN_SETPRIO(0);
#if NN_GEMM_VARIANT == 3
        // A rows 64..127 read behind the first half's MFMAs, before the barrier
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa2[i][ks] = frag(buf, 0, wr * 128u + 64u + 16u * i + rl, ks);
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // B of this buffer read by every wave
        // H1
        if (u + 2 < nK)
            stageB(u + 2, buf);
#if NN_GEMM_VARIANT == 0
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa2[i][ks] = frag(buf, 0, wr * 128u + 64u + 16u * i + rl, ks);
#endif
        NN_SETPRIO(1);
#endif
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa2[i][ks], fb[j][ks], acc[4 + i][j], 0, 0, 0);
        NN_SETPRIO(0);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // A (and B) of this buffer read by every wave
#if NN_GEMM_VARIANT == 1
        if (u + 2 < nK)
            stageB(u + 2, buf);
#endif
    }

    // epilogue: rows m = m0 + 128 wr + 16 i + 4 (lane >> 4) + rr, frame n = n0 + 64 wc + 16 j + (lane & 15)
    const uint32_t g = static_cast<uint32_t>(lane) >> 4, col = rl;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t mb = m0 + wr * 128u + 16u * i + 4u * g;
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

// ---------------------------------------------------------------------------
// nnGemm8p: the same 256 x 256 tile, 8 waves, 128 KiB LDS and swizzle as nnGemm256, with the K-tile
// cut into four phases (the HIP guide's phase-interleaved schedule).  A wave owns rows {64 wr + 0..63}
// of both A halves (rows 0..127 | 128..255) and columns {32 wc + 0..31} of both B halves, so its
// output is four 64 x 32 quadrants (Ah, Bh') and a phase computes one quadrant over K = 64 (16 MFMAs):
//   p1 (A0, B0): read A0 sub-tile + B0 sub-tile; stage B1 of tile v+1 (other buffer)
//   p2 (A0, B1): read B1;                         stage A1 of tile v+1 (other buffer)
//   p3 (A1, B1): read A1;                         stage A0 of tile v+2 (this buffer: A0 last read in p1)
//   p4 (A1, B0): no reads;                        stage B0 of tile v+2 (this buffer: B0 last read in p1);
//                s_waitcnt vmcnt(4) retires tile v+1 (A0/B0 of v+2 stay in flight across the barrier)
// Each phase: reads, stage, [wait], barrier, lgkmcnt(0), 16 MFMAs, barrier.  The wave group wr = 1 runs
// one barrier behind group 0 (an extra barrier before the loop; group 0 takes it after), so on every
// SIMD (one wave of each group) one wave issues MFMAs while the other reads LDS.  With that stagger a
// half-tile is restaged at least two phases after its last read in either group, and a staged tile is
// read one phase after the wait that retires it.
// ---------------------------------------------------------------------------
#ifndef NN8_STAGGER
#define NN8_STAGGER 1  // wave group 1 one barrier behind group 0
#endif
#ifndef NN8_EARLY
#define NN8_EARLY 0  // 1: both halves of tile v+1 still missing are staged in p1 (3 phases before the wait)
#endif
#ifndef NN8_MFMA32
#define NN8_MFMA32 0  // 1: each quadrant on v_mfma_f32_32x32x16_bf16 (2 blocks of 32 x 32, 8 MFMAs) instead of 16x16x32
#endif
#ifndef NN8_STORE16
#define NN8_STORE16 1  // hidden-layer epilogue: 16-byte stores (permlane16 exchange) instead of 8-byte (A/B: -3.4 %)
#endif
#ifndef NN8_TOP_COLS_FIRST
#define NN8_TOP_COLS_FIRST 1  // the C^T top layer's tile order: columns (classes) of one frame tile first
#endif
#ifndef NN8_TOP_SWAP
#define NN8_TOP_SWAP 1  // top layer as C^T (frames x classes): 16-byte stores into the class-major score table
#endif
#ifndef NN8_PRIO_MODE
#define NN8_PRIO_MODE 2  // 0: s_setprio(1) around each MFMA cluster; 1: once for group 1; 2: none (fastest, A/B)
#endif
#if NN8_PRIO_MODE == 0
#define NN8_PRIO(x) __builtin_amdgcn_s_setprio(x)
#else
#define NN8_PRIO(x) ((void)0)
#endif
__global__ __launch_bounds__(512) void nnGemm8p(NnGemmArgs a) {
    constexpr uint32_t T = 256, BK = 64, kOp = T * BK;
    const int          lane = threadIdx.x & 63;
    const uint32_t     wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t     nMT = a.Mpad / T, nNT = a.Npad / T, nwg = nMT * nNT;
    const uint32_t     b = blockIdx.x, xcd = b & 7u, q = nwg / 8u, r = nwg % 8u;
    const uint32_t     id = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (b >> 3);
    // workgroups sharing an XCD take consecutive ids: they sweep the tile rows of one column tile (the
    // activations of one frame tile stay in that XCD's L2); the top layer run as C^T (frames as rows) sweeps
    // the columns of one row tile instead, so that its frame tile's activations are the shared operand again
    const bool         colsFirst = NN8_TOP_COLS_FIRST && a.swapped;
    const uint32_t     m0 = (colsFirst ? id / nNT : id % nMT) * T, n0 = (colsFirst ? id % nNT : id / nMT) * T;
    const uint32_t     wr = wave >> 2, wc = wave & 3u;
    const uint32_t     nK = a.Kpad / BK;

    const auto stage = [&](int op, uint32_t h, uint32_t u, uint32_t buf) {
        const uint16_t* src  = op == 0 ? a.A : a.B;
        const uint32_t  base = op == 0 ? m0 : n0;
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i) {
            const uint32_t p   = wave * 128u + i * 64u + static_cast<uint32_t>(lane);
            const uint32_t row = h * 128u + p / 8u;
            const uint32_t c   = (p % 8u) ^ nnSwz(row);
            __builtin_amdgcn_global_load_lds(src + static_cast<size_t>(base + row) * a.Kpad + u * BK + 8u * c,
                                             nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + h * (kOp / 2) +
                                                     (wave * 128u + i * 64u) * 8u,
                                             16, 0, 0);
        }
    };
    const auto frag = [&](uint32_t buf, int op, uint32_t row, uint32_t ks) {
        const uint32_t c = ks * 4u + (static_cast<uint32_t>(lane) >> 4);
        return *reinterpret_cast<const bf16x8*>(nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + row * BK +
                                                (c ^ nnSwz(row)) * 8u);
    };
    const uint32_t rl = static_cast<uint32_t>(lane) & 15u;
#if NN8_MFMA32
    // 32 x 32 blocks: lane l holds row (l & 31), k = 16 s + 8 (l >> 5) + 0..7 of A and B (16-byte piece
    // 2 s + (l >> 5)); accumulator register i = row (i & 3) + 8 (i >> 2) + 4 (l >> 5), column l & 31
    const uint32_t r32 = static_cast<uint32_t>(lane) & 31u, h32 = static_cast<uint32_t>(lane) >> 5;
    const auto     frag32 = [&](uint32_t buf, int op, uint32_t row, uint32_t s) {
        const uint32_t c = 2u * s + h32;
        return *reinterpret_cast<const bf16x8*>(nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + row * BK +
                                                (c ^ nnSwz(row)) * 8u);
    };
    typedef bf16x8 FragA[2][4];
    typedef bf16x8 FragB[4];
    const auto readA = [&](uint32_t buf, uint32_t h, FragA& fa) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ib = 0; ib < 2; ++ib)
                fa[ib][s] = frag32(buf, 0, h * 128u + wr * 64u + 32u * ib + r32, s);
    };
    const auto readB = [&](uint32_t buf, uint32_t h, FragB& fb) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            fb[s] = frag32(buf, 1, h * 128u + wc * 32u + r32, s);
    };
    f32x16 acc[4][2];  // [2 ha + ib][hb]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            acc[i][j] = f32x16{};
    const auto quadrant = [&](int ha, int hb, const FragA& fa, const FragB& fb) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        NN8_PRIO(1);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ib = 0; ib < 2; ++ib)
                acc[2 * ha + ib][hb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[ib][s], fb[s], acc[2 * ha + ib][hb], 0, 0, 0);
        NN8_PRIO(0);
        __builtin_amdgcn_sched_barrier(0);
    };
#else
    // sub-tile reads: A half h -> rows 128 h + 64 wr + 16 i + rl; B half h -> rows 128 h + 32 wc + 16 j + rl
    typedef bf16x8 FragA[4][2];
    typedef bf16x8 FragB[2][2];
    const auto readA = [&](uint32_t buf, uint32_t h, FragA& fa) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa[i][ks] = frag(buf, 0, h * 128u + wr * 64u + 16u * i + rl, ks);
    };
    const auto readB = [&](uint32_t buf, uint32_t h, FragB& fb) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                fb[j][ks] = frag(buf, 1, h * 128u + wc * 32u + 16u * j + rl, ks);
    };

    f32x4 acc[8][4];  // [4 ha + i][2 hb + j]
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const auto quadrant = [&](int ha, int hb, const FragA& fa, const FragB& fb) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        NN8_PRIO(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[4 * ha + i][2 * hb + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[j][ks], acc[4 * ha + i][2 * hb + j], 0, 0, 0);
        NN8_PRIO(0);
        __builtin_amdgcn_sched_barrier(0);
    };

#endif

    // prologue: tile 0 whole, A0 / B0 of tile 1; tile 0 retired
    stage(0, 0, 0, 0);
    stage(0, 1, 0, 0);
    stage(1, 0, 0, 0);
    stage(1, 1, 0, 0);
    if (nK > 1) {
        stage(0, 0, 1, 1);
        stage(1, 0, 1, 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (NN8_STAGGER && wr == 1)
        __builtin_amdgcn_s_barrier();  // the stagger
#if NN8_PRIO_MODE == 1
    if (wr == 1)
        __builtin_amdgcn_s_setprio(1);  // static form: the younger half keeps priority
#endif

    FragA fa;
    FragB fb0, fb1;
    for (uint32_t v = 0; v < nK; ++v) {
        const uint32_t buf = v & 1u;
        const bool     n1 = v + 1 < nK, n2 = v + 2 < nK;
        // p1
        readA(buf, 0, fa);
        readB(buf, 0, fb0);
        if (n1) {
            stage(1, 1, v + 1, buf ^ 1u);
            if (NN8_EARLY)
                stage(0, 1, v + 1, buf ^ 1u);
        }
        __builtin_amdgcn_s_barrier();
        quadrant(0, 0, fa, fb0);
        __builtin_amdgcn_s_barrier();
        // p2
        readB(buf, 1, fb1);
        if (!NN8_EARLY && n1)
            stage(0, 1, v + 1, buf ^ 1u);
        __builtin_amdgcn_s_barrier();
        quadrant(0, 1, fa, fb1);
        __builtin_amdgcn_s_barrier();
        // p3
        readA(buf, 1, fa);
        if (n2)
            stage(0, 0, v + 2, buf);
        __builtin_amdgcn_s_barrier();
        quadrant(1, 1, fa, fb1);
        __builtin_amdgcn_s_barrier();
        // p4
        if (n2) {
            stage(1, 0, v + 2, buf);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        }
        else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        quadrant(1, 0, fa, fb0);
        __builtin_amdgcn_s_barrier();
    }
    if (NN8_STAGGER && wr == 0)
        __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier

#if NN8_MFMA32
    // epilogue: block (ha, ib, hb) register 4 q + rr -> row m0 + 128 ha + 64 wr + 32 ib + 8 q + 4 h32 + rr,
    //           frame n0 + 128 hb + 32 wc + r32
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t n = n0 + 128u * j + wc * 32u + r32;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t mb = m0 + 128u * (i >> 1) + wr * 64u + 32u * (i & 1) + 8u * q + 4u * h32;
                const f32x4    bs = *reinterpret_cast<const f32x4*>(a.bias + mb);
                if (a.top) {
                    if (n < a.nFrames)
#pragma unroll
                        for (int rr = 0; rr < 4; ++rr)
                            if (mb + rr < a.M)
                                a.scores[static_cast<size_t>(mb + rr) * a.scoreStride + n] = -(acc[i][j][4 * q + rr] + bs[rr]);
                }
                else {
                    u16x4 v;
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        v[rr] = toBf16(activate(acc[i][j][4 * q + rr] + bs[rr], a.act, a.gamma));
                    *reinterpret_cast<u16x4*>(a.Y + static_cast<size_t>(n) * a.Mpad + mb) = v;
                }
            }
        }
    }
#else
    // epilogue: rows m = m0 + 128 (i >> 2) + 64 wr + 16 (i & 3) + 4 (lane >> 4) + rr,
    //           frame n = n0 + 128 (j >> 1) + 32 wc + 16 (j & 1) + (lane & 15)
    const uint32_t g = static_cast<uint32_t>(lane) >> 4, col = rl;
#if NN8_STORE16
    if (!a.top) {
        // 16-byte stores: accumulators i, i + 1 (rows 16 apart) packed to bf16 and exchanged between lane
        // groups by one v_permlane16_swap per dword, so lane group g holds 8 consecutive rows (units) of its
        // frame: rows 16 i + 16 (g & 1) + 8 (g >> 1) + 0..7 -- half the store instructions, 64-byte runs
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            const uint32_t mb0 = m0 + 128u * (i >> 2) + wr * 64u + 16u * (i & 3);
            const f32x4    b0  = *reinterpret_cast<const f32x4*>(a.bias + mb0 + 4u * g);
            const f32x4    b1  = *reinterpret_cast<const f32x4*>(a.bias + mb0 + 16u + 4u * g);
#if NN_SIGMOID_FMA
            const float sk  = -a.gamma * 1.44269504088896341f;
            const f32x4 bk0 = b0 * sk, bk1 = b1 * sk;
#endif
            const uint32_t mst = mb0 + 16u * (g & 1u) + 8u * (g >> 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t n = n0 + 128u * (j >> 1) + wc * 32u + 16u * (j & 1) + col;
                u16x4          v0, v1;
#if NN_SIGMOID_FMA
                if (a.act == 1) {
                    // sigmoid(x + b) = 1 / (1 + 2^((x + b) k)), k = -gamma log2(e): one FMA into the exponent
                    // (x k + b k) instead of the add, the gamma multiply and __expf's log2(e) multiply
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        v0[rr] = toBf16(__builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][j][rr], sk, bk0[rr]))));
                        v1[rr] = toBf16(__builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i + 1][j][rr], sk, bk1[rr]))));
                    }
                }
                else
#endif
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    v0[rr] = toBf16(activate(acc[i][j][rr] + b0[rr], a.act, a.gamma));
                    v1[rr] = toBf16(activate(acc[i + 1][j][rr] + b1[rr], a.act, a.gamma));
                }
                const uint2 x = __builtin_bit_cast(uint2, v0), y = __builtin_bit_cast(uint2, v1);
                const auto  s0 = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
                const auto  s1 = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
                const uint4 w  = {static_cast<uint32_t>(s0[0]), static_cast<uint32_t>(s1[0]),
                                  static_cast<uint32_t>(s0[1]), static_cast<uint32_t>(s1[1])};
                *reinterpret_cast<uint4*>(a.Y + static_cast<size_t>(n) * a.Mpad + mst) = w;
            }
        }
        return;
    }
#endif
#if NN8_TOP_SWAP
    if (a.swapped) {
        // top layer as C^T: rows are frames, columns classes, so a lane holds 4 consecutive frames of one
        // class -- one 16-byte store into the class-major score table instead of four 4-byte ones
        const bool vec = (a.scoreStride & 3u) == 0u && (reinterpret_cast<uintptr_t>(a.scores) & 15u) == 0u;
        float      bc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t c = n0 + 128u * (j >> 1) + wc * 32u + 16u * (j & 1) + col;
            bc[j]            = a.bias[c];  // bias has Npad (= padded classes) entries
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t fr = m0 + 128u * (i >> 2) + wr * 64u + 16u * (i & 3) + 4u * g;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t c = n0 + 128u * (j >> 1) + wc * 32u + 16u * (j & 1) + col;
                if (c >= a.M)
                    continue;
                float* const dst = a.scores + static_cast<size_t>(c) * a.scoreStride + fr;
                const f32x4  v   = {-(acc[i][j][0] + bc[j]), -(acc[i][j][1] + bc[j]), -(acc[i][j][2] + bc[j]),
                                    -(acc[i][j][3] + bc[j])};
                if (vec && fr + 3u < a.nFrames)
                    *reinterpret_cast<f32x4*>(dst) = v;
                else
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        if (fr + rr < a.nFrames)
                            dst[rr] = v[rr];
            }
        }
        return;
    }
#endif
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t mb = m0 + 128u * (i >> 2) + wr * 64u + 16u * (i & 3) + 4u * g;
        const f32x4    bs = *reinterpret_cast<const f32x4*>(a.bias + mb);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t n = n0 + 128u * (j >> 1) + wc * 32u + 16u * (j & 1) + col;
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
#endif
}


// ---------------------------------------------------------------------------
// nnGemm8pp: nnGemm8p as a persistent kernel (NN_GEMM_VARIANT 9).  With one 128 KiB workgroup per CU,
// nnGemm8p pays every output tile's prologue (the first K-tiles from L2/HBM with nothing to overlap)
// and epilogue (bias, activation, stores with the matrix cores idle) in the open: 4 tile rounds per
// 2048-wide layer.  Here one workgroup per CU walks its output tiles (ids b = w, w + G, ... under the
// same bijective XCD remap) as ONE continuous stream of K-tiles: the phase schedule, the staging two
// K-tiles ahead and the counted waits run across tile seams unchanged, so the next tile's first K-tiles
// land while the current tile's last ones are multiplied, and the epilogue of a tile is issued between
// its last phase and the next tile's first.  The tile's bias (1 KiB, rows m0 .. m0+255) is staged into
// LDS by wave 0 with the first K-tile's p1 half (double-buffered by tile parity) and is retired by that
// step's p4 wait, before the epilogue that reads it.  The epilogue's stores are counted by vmcnt like the
// loads: the next tile's first p4 wait also retires them.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(512) void nnGemm8pp(NnGemmArgs a) {
    constexpr uint32_t T = 256, BK = 64, kOp = T * BK;
    const int          lane = threadIdx.x & 63;
    const uint32_t     wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t     nMT = a.Mpad / T, nNT = a.Npad / T, nwg = nMT * nNT;
    const uint32_t     G = gridDim.x, w = blockIdx.x;
    const uint32_t     q = nwg / 8u, r = nwg % 8u;
    const uint32_t     wr = wave >> 2, wc = wave & 3u;
    const uint32_t     nK = a.Kpad / BK;
    const uint32_t     nTiles = w < nwg ? (nwg - w + G - 1u) / G : 0u;
    const uint32_t     nSteps = nTiles * nK;
    float* const       biasLds = reinterpret_cast<float*>(nnLds + 4u * kOp);  // [2][256] after the operand buffers

    // output tile of this workgroup's k-th tile (bijective XCD remap of b = w + G k, as nnGemm8p)
    const auto tileOf = [&](uint32_t k, uint32_t& m0, uint32_t& n0) {
        const uint32_t b = w + G * k, xcd = b & 7u;
        const uint32_t id = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (b >> 3);
        m0                = (id % nMT) * T;
        n0                = (id / nMT) * T;
    };
    // position of a step in the stream: tile k (output tile m0, n0), K-tile u; advanced step by step
    // (no division per stage)
    struct Pos {
        uint32_t k, u, m0, n0;
    };
    const auto advance = [&](Pos& p) {
        if (++p.u == nK) {
            p.u = 0;
            ++p.k;
            tileOf(p.k, p.m0, p.n0);
        }
    };
    // stage operand op, half h of the step at p into buffer buf
    const auto stage = [&](int op, uint32_t h, const Pos& p, uint32_t buf) {
        const uint16_t* src  = op == 0 ? a.A : a.B;
        const uint32_t  base = op == 0 ? p.m0 : p.n0;
#pragma unroll
        for (uint32_t i = 0; i < 2; ++i) {
            const uint32_t pc  = wave * 128u + i * 64u + static_cast<uint32_t>(lane);
            const uint32_t row = h * 128u + pc / 8u;
            const uint32_t c   = (pc % 8u) ^ nnSwz(row);
            __builtin_amdgcn_global_load_lds(src + static_cast<size_t>(base + row) * a.Kpad + p.u * BK + 8u * c,
                                             nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + h * (kOp / 2) +
                                                     (wave * 128u + i * 64u) * 8u,
                                             16, 0, 0);
        }
    };
    const auto frag = [&](uint32_t buf, int op, uint32_t row, uint32_t ks) {
        const uint32_t c = ks * 4u + (static_cast<uint32_t>(lane) >> 4);
        return *reinterpret_cast<const bf16x8*>(nnLds + (buf * 2u + static_cast<uint32_t>(op)) * kOp + row * BK +
                                                (c ^ nnSwz(row)) * 8u);
    };
    const uint32_t rl = static_cast<uint32_t>(lane) & 15u;
    typedef bf16x8 FragA[4][2];
    typedef bf16x8 FragB[2][2];
    const auto     readA = [&](uint32_t buf, uint32_t h, FragA& fa) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                fa[i][ks] = frag(buf, 0, h * 128u + wr * 64u + 16u * i + rl, ks);
    };
    const auto readB = [&](uint32_t buf, uint32_t h, FragB& fb) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                fb[j][ks] = frag(buf, 1, h * 128u + wc * 32u + 16u * j + rl, ks);
    };
    f32x4      acc[8][4];  // [4 ha + i][2 hb + j]
    const auto zeroAcc = [&]() {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    };
    const auto quadrant = [&](int ha, int hb, const FragA& fa, const FragB& fb) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[4 * ha + i][2 * hb + j] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][ks], fb[j][ks], acc[4 * ha + i][2 * hb + j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
    };
    // the tile's bias into LDS slot k & 1 (wave 0: 64 lanes x 16 B = rows m0 .. m0 + 255)
    const auto stageBias = [&](uint32_t k) {
        if (wave == 0u) {
            uint32_t m0, n0;
            tileOf(k, m0, n0);
            __builtin_amdgcn_global_load_lds(a.bias + m0 + 4u * static_cast<uint32_t>(lane), biasLds + (k & 1u) * 256u,
                                             16, 0, 0);
        }
    };
    // epilogue of tile k: rows m = m0 + 128 (i >> 2) + 64 wr + 16 (i & 3) + 4 (lane >> 4) + rr,
    //                     frame n = n0 + 128 (j >> 1) + 32 wc + 16 (j & 1) + (lane & 15)
    const auto epilogue = [&](uint32_t k) {
        uint32_t m0, n0;
        tileOf(k, m0, n0);
        const uint32_t g = static_cast<uint32_t>(lane) >> 4, col = rl;
        const float*   bl = biasLds + (k & 1u) * 256u;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t mr = 128u * (i >> 2) + wr * 64u + 16u * (i & 3) + 4u * g;
            const uint32_t mb = m0 + mr;
            const f32x4    bs = *reinterpret_cast<const f32x4*>(bl + mr);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t n = n0 + 128u * (j >> 1) + wc * 32u + 16u * (j & 1) + col;
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
    };
    if (nSteps == 0)
        return;  // uniform over the workgroup, before any barrier

    // prologue: step 0 whole, A0 / B0 of step 1, the first tile's bias; step 0 retired
    Pos p0{0, 0, 0, 0};
    tileOf(0, p0.m0, p0.n0);
    Pos p1 = p0, p2;
    advance(p1);
    p2 = p1;
    advance(p2);
    stageBias(0);
    stage(0, 0, p0, 0);
    stage(0, 1, p0, 0);
    stage(1, 0, p0, 0);
    stage(1, 1, p0, 0);
    if (nSteps > 1) {
        stage(0, 0, p1, 1);
        stage(1, 0, p1, 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (NN8_STAGGER && wr == 1)
        __builtin_amdgcn_s_barrier();  // the stagger

    zeroAcc();
    FragA    fa;
    FragB    fb0, fb1;
    uint32_t u = 0, k = 0;  // K-tile and tile of step v; p1, p2: steps v + 1, v + 2
    for (uint32_t v = 0; v < nSteps; ++v) {
        const uint32_t buf = v & 1u;
        const bool     n1 = v + 1 < nSteps, n2 = v + 2 < nSteps;
        // p1 (a tile's first step also stages its bias: retired by this step's p4 wait)
        readA(buf, 0, fa);
        readB(buf, 0, fb0);
        if (u == 0u && v > 0u)
            stageBias(k);
        if (n1)
            stage(1, 1, p1, buf ^ 1u);
        __builtin_amdgcn_s_barrier();
        quadrant(0, 0, fa, fb0);
        __builtin_amdgcn_s_barrier();
        // p2
        readB(buf, 1, fb1);
        if (n1)
            stage(0, 1, p1, buf ^ 1u);
        __builtin_amdgcn_s_barrier();
        quadrant(0, 1, fa, fb1);
        __builtin_amdgcn_s_barrier();
        // p3
        readA(buf, 1, fa);
        if (n2)
            stage(0, 0, p2, buf);
        __builtin_amdgcn_s_barrier();
        quadrant(1, 1, fa, fb1);
        __builtin_amdgcn_s_barrier();
        // p4
        if (n2) {
            stage(1, 0, p2, buf);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        }
        else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        quadrant(1, 0, fa, fb0);
        __builtin_amdgcn_s_barrier();
        if (++u == nK) {  // uniform: the tile's last K-tile
            epilogue(k);
            zeroAcc();
            u = 0;
            ++k;
        }
        p1 = p2;
        advance(p2);
    }
    if (NN8_STAGGER && wr == 0)
        __builtin_amdgcn_s_barrier();  // matches group 1's extra barrier
}

}  // namespace dev

hipError_t launchNnPrepareInput(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t D,
                                uint32_t Kpad, uint16_t* X, hipStream_t stream) {
    const uint32_t n = nFrames * D;
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::nnPrepareInput, dim3(nFrames), dim3(256), 0, stream, frames, nFrames, frameStride, D, Kpad,
                       X);
    return hipGetLastError();
}

hipError_t launchNnGemm(const NnGemmArgs& a, hipStream_t stream) {
    if (a.Mpad % kNnTileM || a.Npad % kNnTileN || a.Kpad % kNnTileK || a.Kpad == 0)
        return hipErrorInvalidValue;  // the kernel reads whole tiles without bounds checks
#if NN_GEMM_VARIANT == 8 && !NN8_MFMA32 && NN8_TOP_SWAP
    if (kNnTileM == 256 && a.top && !a.swapped) {
        // the top layer as C^T = activations . W: the tile rows are frames, so the class-major score table
        // gets 16-byte stores (nnGemm8p epilogue); bias stays indexed by class (now the column)
        NnGemmArgs t = a;
        t.A          = a.B;
        t.B          = a.A;
        t.Mpad       = a.Npad;
        t.Npad       = a.Mpad;
        t.swapped    = 1;
        return launchNnGemm(t, stream);
    }
#endif
    const uint32_t nwg = (a.Mpad / kNnTileM) * (a.Npad / kNnTileN);
    if (nwg == 0)
        return hipSuccess;
    if constexpr (kNnTileM == 256) {
        constexpr uint32_t kLds = 2u * 2u * 256u * 64u * 2u + (NN_GEMM_VARIANT == 9 ? 2048u : 0u);  // 128 KiB (+ bias)
#if NN_GEMM_VARIANT == 9
        const auto kernel = dev::nnGemm8pp;
#elif NN_GEMM_VARIANT == 8
        const auto kernel = dev::nnGemm8p;
#else
        const auto kernel = dev::nnGemm256;
#endif
        static bool attr = false;
        if (!attr) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLds));
            if (e != hipSuccess)
                return e;
            attr = true;
        }
#if NN_GEMM_VARIANT == 9
        // persistent: one workgroup per CU (128 KiB of LDS each), each walking its tiles
        static int nCu = 0;
        if (nCu == 0) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&nCu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || nCu <= 0)
                nCu = 256;
        }
        const uint32_t grid = std::min<uint32_t>(nwg, static_cast<uint32_t>(nCu));
        hipLaunchKernelGGL(kernel, dim3(grid), dim3(512), kLds, stream, a);
#else
        hipLaunchKernelGGL(kernel, dim3(nwg), dim3(512), kLds, stream, a);
#endif
    }
    else {
        hipLaunchKernelGGL(dev::nnGemm, dim3(nwg), dim3(256), 0, stream, a);
    }
    return hipGetLastError();
}

}  // namespace rasr_nn
