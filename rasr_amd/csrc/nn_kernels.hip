// nn_kernels.hip -- the hybrid-DNN scorer's layers on gfx950: one bf16 GEMM per layer with the bias,
// the activation (or, on the top layer, the negation into the class-major score table) fused into
// the epilogue.
//
// GEMM: C[M x N] = A[M x K] . B[N x K]^T, A = W^T (output units x inputs), B = activations (frames x
// inputs), both K-contiguous, so both MFMA operands are 16-byte row pieces: nnGemm8p below, a 256 x 256
// output tile per 512-thread workgroup on v_mfma_f32_16x16x32_bf16, K in 64-wide tiles staged global -> LDS
// by global_load_lds_dwordx4, double-buffered, with counted s_waitcnt vmcnt and raw s_barriers (a
// __syncthreads would drain the DMA).  Workgroups are mapped so that the ones sharing an XCD sweep the
// output-unit tiles of one frame tile (its activations stay in that XCD's L2).  Calls too small to fill the
// chip with those tiles run nnGemm128 (128 x 128 tiles) or, up to 128 frames, nnGemmSmall.  The variants
// measured against nnGemm8p (the two-half schedule, a persistent form, 32x32x16 quadrants, s_setprio modes;
// DESIGN.md section 11) are kept out of this file: scripts/variants/.
#include "gmm_kernels.hh"  // rasr_gmm::allowDynamicLds
#include "nn_kernels.hh"

#include <algorithm>

namespace rasr_nn {
namespace dev {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float  f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float  f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float activate(float x, int act, float gamma) {
    switch (act) {
        // SigmoidLayer; v_rcp_f32 (1 ulp) instead of the IEEE division sequence (~10 VALU per value in an
        // epilogue the matrix cores wait for): far below the bf16 rounding of the layer output
        case 1: return __builtin_amdgcn_rcpf(1.0f + __expf(-gamma * x));
        // TanhLayer as 1 - 2 / (2^(2 log2(e) x) + 1): v_exp_f32 + v_rcp_f32 instead of libm's tanhf.  That form
        // has an absolute error of ~1e-7, which near 0 is a large RELATIVE error (bf16 keeps small outputs to
        // 2^-9 relative), so |x| < 2^-4 takes x (1 - x^2 / 3) (the next term, 2 x^5 / 15, is < 2.1e-6 relative);
        // +-1 and NaN kept
        case 2: {
            const float x2 = x * x;
            return fabsf(x) < 0.0625f ? x * fmaf(x2, -0.333333343f, 1.0f)
                                      : 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(2.88539008177792681f * x));
        }
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

// ---------------------------------------------------------------------------
// LDS: two buffers of 64 KiB (A 256 rows | B 256 rows, 128-B rows of 64 bf16).  The 16-B piece c of row r
// sits at c ^ ((r >> 1) & 7): the 16 lanes of a ds_read_b128 group (16 consecutive rows, one piece) then
// hit 16 different 16-B bank slots (two 128-B rows share a 256-B bank row), conflict-free.  The swizzle is
// applied on the per-lane global source address (the LDS side of global_load_lds is lane-linear).
// ---------------------------------------------------------------------------
extern __shared__ __attribute__((aligned(16))) uint16_t nnLds[];  // [2 buffers][A | B][256 * 64]

__device__ __forceinline__ uint32_t nnSwz(uint32_t r) {
    return (r >> 1) & 7u;
}

// ---------------------------------------------------------------------------
// nnGemm8p: 256 x 256 output tile, 8 waves as 2 (units) x 4 (frames), 128 KiB LDS, with the K-tile
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
#ifndef NN8_TOP_COLS_FIRST
#define NN8_TOP_COLS_FIRST 1  // the C^T top layer's tile order: columns (classes) of one frame tile first
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

    // epilogue: rows m = m0 + 128 (i >> 2) + 64 wr + 16 (i & 3) + 4 (lane >> 4) + rr,
    //           frame n = n0 + 128 (j >> 1) + 32 wc + 16 (j & 1) + (lane & 15)
    const uint32_t g = static_cast<uint32_t>(lane) >> 4, col = rl;
    if (!a.top) {
        // 16-byte stores: accumulators i, i + 1 (rows 16 apart) packed to bf16 and exchanged between lane
        // groups by one v_permlane16_swap per dword, so lane group g holds 8 consecutive rows (units) of its
        // frame: rows 16 i + 16 (g & 1) + 8 (g >> 1) + 0..7 -- half the store instructions, 64-byte runs
#pragma unroll
        for (int i = 0; i < 8; i += 2) {
            const uint32_t mb0 = m0 + 128u * (i >> 2) + wr * 64u + 16u * (i & 3);
            const f32x4    b0  = *reinterpret_cast<const f32x4*>(a.bias + mb0 + 4u * g);
            const f32x4    b1  = *reinterpret_cast<const f32x4*>(a.bias + mb0 + 16u + 4u * g);
            const float sk  = -a.gamma * 1.44269504088896341f;
            const f32x4 bk0 = b0 * sk, bk1 = b1 * sk;
            const uint32_t mst = mb0 + 16u * (g & 1u) + 8u * (g >> 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t n = n0 + 128u * (j >> 1) + wc * 32u + 16u * (j & 1) + col;
                u16x4          v0, v1;
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
}

// ---------------------------------------------------------------------------
// nnGemm128: calls between nnGemmSmall's range and a full chip of nnGemm8p tiles (~300 .. 4000 frames).
// There nnGemm8p's 256 x 256 tiles leave a 2048-unit layer Mpad / 256 x Npad / 256 workgroups (64 at 2048
// frames): each sweeps all of K on one CU, so the layer takes one tile's time (~40 us) with most CUs idle.
// A 128 x 128 tile gives 4x the workgroups for 1/4 of the work each.  256 threads as 2 x 2 waves of 64 x 64
// (4 x 4 accumulators of v_mfma_f32_16x16x32_bf16); K in 64-wide stages staged global -> LDS by
// global_load_lds_dwordx4 (4 x 1 KiB per wave and operand), double-buffered with a counted s_waitcnt vmcnt
// and raw s_barriers; nnGemm8p's LDS swizzle and XCD mapping.  The K order of every accumulator chain and the
// epilogue arithmetic are nnGemm8p's, so WITHOUT a K split a frame's scores are bit-identical between the two
// kernels (the top layer is not run as C^T here: 4-byte stores of 16 consecutive frames per class); a split layer
// (nnSplitReduce) and nnGemmSmall (K over 8 waves) add partial sums in another order and round differently,
// within the bf16 contract (tests/test_nn_scorer.py::test_nn_kernel_boundaries_within_contract).  A hidden layer whose
// 128-tile grid still leaves CUs idle (kSplit > 1) splits K: workgroup idS covers tile idS % tiles over the
// K-tiles of split idS / tiles and writes its f32 partial sums; nnSplitReduce finishes the layer.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void nnGemm128(NnGemmArgs a) {
    constexpr uint32_t T = 128, BK = 64, kOp = T * BK;
    __shared__ __attribute__((aligned(16))) uint16_t lds[2][2][kOp];  // [stage][A | B], 64 KiB
    const int      lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t nMT = a.Mpad / T, nNT = a.Npad / T, nTiles = nMT * nNT;
    const uint32_t S = a.kSplit > 1u ? a.kSplit : 1u, nwg = nTiles * S;
    const uint32_t b = blockIdx.x, xcd = b & 7u, q = nwg / 8u, r = nwg % 8u;
    const uint32_t idS = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (b >> 3);
    const uint32_t id = idS % nTiles, split = idS / nTiles;  // an XCD's workgroups: the tiles of one K range
    const uint32_t m0 = (id % nMT) * T, n0 = (id / nMT) * T;
    const uint32_t wr = wave >> 1, wc = wave & 1u;
    const uint32_t rl = static_cast<uint32_t>(lane) & 15u;

    // stage s <- K columns [k0, k0 + 64): 16 pieces of 8 rows x 128 B per operand, 4 per wave
    const auto issue = [&](uint32_t s, uint32_t k0) {
#pragma unroll
        for (uint32_t i = 0; i < 4; ++i) {
            const uint32_t piece = wave * 4u + i;
            const uint32_t row   = piece * 8u + (static_cast<uint32_t>(lane) >> 3);
            const uint32_t c     = (static_cast<uint32_t>(lane) & 7u) ^ nnSwz(row);
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

    // this workgroup's K-tiles [kt0, nK): all of K, or its split's share
    const uint32_t nKall = a.Kpad / BK, per = (nKall + S - 1u) / S;
    const uint32_t kt0 = min(nKall, split * per), nK = min(nKall, kt0 + per);
    if (kt0 < nK)
        issue(0, kt0 * BK);
    for (uint32_t kt = kt0; kt < nK; ++kt) {
        const uint32_t s = (kt - kt0) & 1u;
        if (kt + 1 < nK) {
            issue(s ^ 1u, (kt + 1) * BK);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this stage's 8 DMAs landed, the next 8 fly
        }
        else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // every wave's pieces of stage s are in LDS
#pragma unroll
        for (uint32_t ks = 0; ks < 2; ++ks) {
            bf16x8         fa[4], fb[4];
            const uint32_t c = ks * 4u + (static_cast<uint32_t>(lane) >> 4);
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                const uint32_t ra = wr * 64u + 16u * i + rl, rb = wc * 64u + 16u * i + rl;
                fa[i] = *reinterpret_cast<const bf16x8*>(&lds[s][0][ra * BK + (c ^ nnSwz(ra)) * 8u]);
                fb[i] = *reinterpret_cast<const bf16x8*>(&lds[s][1][rb * BK + (c ^ nnSwz(rb)) * 8u]);
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
    const uint32_t g  = static_cast<uint32_t>(lane) >> 4;
    if (S > 1u) {  // split K: the partial sums, 16 bytes of 4 units per frame; nnSplitReduce finishes the layer
        float* const p = a.part + static_cast<size_t>(split) * a.Npad * a.Mpad;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *reinterpret_cast<f32x4*>(p + static_cast<size_t>(n0 + wc * 64u + 16u * j + rl) * a.Mpad + m0 + wr * 64u +
                                          16u * i + 4u * g) = acc[i][j];
        return;
    }
    const float    sk = -a.gamma * 1.44269504088896341f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t mb = m0 + wr * 64u + 16u * i + 4u * g;
        const f32x4    bs = *reinterpret_cast<const f32x4*>(a.bias + mb);
        const f32x4    bk = bs * sk;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t n = n0 + wc * 64u + 16u * j + rl;
            if (a.top) {
                if (n < a.nFrames)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                        if (mb + rr < a.M)
                            a.scores[static_cast<size_t>(mb + rr) * a.scoreStride + n] = -(acc[i][j][rr] + bs[rr]);
                continue;
            }
            u16x4 v;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                v[rr] = a.act == 1  // nnGemm8p's sigmoid: bias and gamma folded into the exponent's FMA
                            ? toBf16(__builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][j][rr], sk, bk[rr]))))
                            : toBf16(activate(acc[i][j][rr] + bs[rr], a.act, a.gamma));
            *reinterpret_cast<u16x4*>(a.Y + static_cast<size_t>(n) * a.Mpad + mb) = v;
        }
    }
}

// nnGemm128's split-K finish for a hidden layer: per frame n and 4 units m, the kSplit partial sums added in split
// order (deterministic), then nnGemm8p's bias + activation epilogue into the next layer's bf16 rows
__global__ __launch_bounds__(256) void nnSplitReduce(NnGemmArgs a) {
    const uint32_t quads = a.Mpad / 4u;
    const uint32_t t = blockIdx.x * 256u + threadIdx.x;
    if (t >= a.Npad * quads)
        return;
    const uint32_t n = t / quads, m = (t % quads) * 4u;
    const size_t   off = static_cast<size_t>(n) * a.Mpad + m, plane = static_cast<size_t>(a.Npad) * a.Mpad;
    f32x4          acc = *reinterpret_cast<const f32x4*>(a.part + off);
    for (uint32_t s = 1; s < a.kSplit; ++s)
        acc += *reinterpret_cast<const f32x4*>(a.part + s * plane + off);
    const f32x4 bs = *reinterpret_cast<const f32x4*>(a.bias + m);
    const float sk = -a.gamma * 1.44269504088896341f;
    u16x4       v;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
        v[rr] = a.act == 1 ? toBf16(__builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(acc[rr], sk, bs[rr] * sk))))
                           : toBf16(activate(acc[rr] + bs[rr], a.act, a.gamma));
    *reinterpret_cast<u16x4*>(a.Y + off) = v;
}

// ---------------------------------------------------------------------------
// nnGemmSmall: calls of up to 64 frames (RASR's Nn::BatchFeatureScorer buffer-size defaults to 8,
// src/Nn/BatchFeatureScorer.cc:21-22).  nnGemm8p's 256 x 256 tiles leave such a layer to Mpad / 256
// workgroups (8 for 2048 units) that each sweep all of K: the call is latency-bound (~40 us per layer).
// Here a workgroup owns 16 output units (one MFMA row block) x NB column blocks of 16 frames, its WS waves
// split the K steps (Mpad / 16 workgroups per layer, 128 for 2048 units; 8 waves each: one round of KU = 8
// K steps of loads per wave at K = 2048), every weight read once straight from HBM into the MFMA A fragment
// (16 rows x 64 contiguous bytes per K step), the few frames' activations (<= 64 x Kpad bf16) from L2.  The
// partial sums are added in wave order through LDS (deterministic; the K order differs from nnGemm8p's, so the
// rounding does too), then nnGemm8p's epilogue arithmetic (the folded sigmoid included): bias + activation into
// the next layer's bf16 rows, or the negated scores of the top layer.
// ---------------------------------------------------------------------------
template <int NB, int WS>
__global__ __launch_bounds__(64 * WS) void nnGemmSmall(NnGemmArgs a) {
    constexpr int KU = 8;  // K steps of 32 whose fragments are loaded ahead
    __shared__ f32x4 part[WS][NB][64];
    const int      lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t m0   = blockIdx.x * 16u, n0 = blockIdx.y * 64u;  // 16 units x a group of <= 64 frames
    const uint32_t rl = static_cast<uint32_t>(lane) & 15u, kq = 8u * (static_cast<uint32_t>(lane) >> 4);
    // this wave's share of the K steps (Kpad / 32 of them, Kpad a multiple of 64)
    const uint32_t nK = a.Kpad / 32u, per = (nK + WS - 1u) / WS;
    const uint32_t k0 = min(nK, per * static_cast<uint32_t>(w)), k1 = min(nK, k0 + per);
    const bf16x8*  wa = reinterpret_cast<const bf16x8*>(a.A + static_cast<size_t>(m0 + rl) * a.Kpad + kq);
    const bf16x8*  xb[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
        xb[cb] = reinterpret_cast<const bf16x8*>(a.B + static_cast<size_t>(n0 + 16u * cb + rl) * a.Kpad + kq);
    f32x4 acc[NB];
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
        acc[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    uint32_t k = k0;
    for (; k + KU <= k1; k += KU) {
        bf16x8 fa[KU], fb[KU][NB];
#pragma unroll
        for (int u = 0; u < KU; ++u) {
            fa[u] = wa[(k + u) * 4u];  // 32 bf16 = four 16-byte pieces per K step
#pragma unroll
            for (int cb = 0; cb < NB; ++cb)
                fb[u][cb] = xb[cb][(k + u) * 4u];
        }
#pragma unroll
        for (int u = 0; u < KU; ++u)
#pragma unroll
            for (int cb = 0; cb < NB; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[u], fb[u][cb], acc[cb], 0, 0, 0);
    }
    for (; k < k1; ++k) {
        const bf16x8 fa = wa[k * 4u];
#pragma unroll
        for (int cb = 0; cb < NB; ++cb)
            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, xb[cb][k * 4u], acc[cb], 0, 0, 0);
    }
    // the WS partial sums, added in wave order (deterministic) by wave 0
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
        part[w][cb][lane] = acc[cb];
    __syncthreads();
    if (w != 0)
        return;
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
        acc[cb] = part[0][cb][lane];
#pragma unroll
        for (int v = 1; v < WS; ++v)
            acc[cb] += part[v][cb][lane];
    }
    // accumulator r of lane l: unit m0 + 4 (l >> 4) + r, frame 16 cb + (l & 15)
    const uint32_t mb = m0 + 4u * (static_cast<uint32_t>(lane) >> 4);
    const f32x4    bs = *reinterpret_cast<const f32x4*>(a.bias + mb);
    const float    sk = -a.gamma * 1.44269504088896341f;
    const f32x4    bk = bs * sk;
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
        const uint32_t n = n0 + 16u * cb + rl;
        if (a.top) {
            if (n < a.nFrames)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    if (mb + rr < a.M)
                        a.scores[static_cast<size_t>(mb + rr) * a.scoreStride + n] = -(acc[cb][rr] + bs[rr]);
        }
        else {
            u16x4 v;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                v[rr] = a.act == 1  // nnGemm8p's sigmoid: bias and gamma folded into the exponent's FMA
                            ? toBf16(__builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(__builtin_fmaf(acc[cb][rr], sk, bk[rr]))))
                            : toBf16(activate(acc[cb][rr] + bs[rr], a.act, a.gamma));
            *reinterpret_cast<u16x4*>(a.Y + static_cast<size_t>(n) * a.Mpad + mb) = v;
        }
    }
}

}  // namespace dev

hipError_t launchNnGemmSmall(const NnGemmArgs& a, hipStream_t stream) {
    // Npad: the frames rounded up to 16 (<= 64), or to 64 (groups of 64 frames, grid.y)
    if (a.Mpad % 16u || a.Kpad % 64u || a.Kpad == 0 || a.Npad == 0 || a.Npad % 16u || (a.Npad > 64 && a.Npad % 64u))
        return hipErrorInvalidValue;
    // one 16-unit row block x frame group per workgroup, its K steps split over kWs waves
    constexpr int kWs = 8;
    const dim3    grid(a.Mpad / 16u, (a.Npad + 63u) / 64u), block(64 * kWs);
    switch (a.Npad > 64 ? 4u : a.Npad / 16u) {
        case 1: hipLaunchKernelGGL((dev::nnGemmSmall<1, kWs>), grid, block, 0, stream, a); break;
        case 2: hipLaunchKernelGGL((dev::nnGemmSmall<2, kWs>), grid, block, 0, stream, a); break;
        case 3: hipLaunchKernelGGL((dev::nnGemmSmall<3, kWs>), grid, block, 0, stream, a); break;
        default: hipLaunchKernelGGL((dev::nnGemmSmall<4, kWs>), grid, block, 0, stream, a); break;
    }
    return hipGetLastError();
}

hipError_t launchNnGemm128(const NnGemmArgs& a, hipStream_t stream) {
    if (a.Mpad % 128u || a.Npad % 128u || a.Kpad % kNnTileK || a.Kpad == 0 || a.swapped)
        return hipErrorInvalidValue;  // whole tiles, no bounds checks
    const bool split = a.kSplit > 1u;
    if (split && (a.top || !a.part || a.kSplit > kNnMaxSplit ||
                  static_cast<size_t>(a.kSplit) * a.Npad * a.Mpad > kNnSplitFloats))
        return hipErrorInvalidValue;  // hidden layers only, within the workspace
    const uint32_t nwg = (a.Mpad / 128u) * (a.Npad / 128u) * (split ? a.kSplit : 1u);
    if (nwg == 0)
        return hipSuccess;
    hipLaunchKernelGGL(dev::nnGemm128, dim3(nwg), dim3(256), 0, stream, a);
    if (split) {
        const uint32_t n = a.Npad * (a.Mpad / 4u);
        hipLaunchKernelGGL(dev::nnSplitReduce, dim3((n + 255u) / 256u), dim3(256), 0, stream, a);
    }
    return hipGetLastError();
}

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
    if (a.top && !a.swapped) {
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
    const uint32_t nwg = (a.Mpad / kNnTileM) * (a.Npad / kNnTileN);
    if (nwg == 0)
        return hipSuccess;
    constexpr uint32_t kLds = 2u * 2u * 256u * 64u * 2u;  // 128 KiB
    const hipError_t e = rasr_gmm::allowDynamicLds(reinterpret_cast<const void*>(&dev::nnGemm8p), static_cast<int>(kLds));
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(dev::nnGemm8p, dim3(nwg), dim3(512), kLds, stream, a);
    return hipGetLastError();
}

}  // namespace rasr_nn
