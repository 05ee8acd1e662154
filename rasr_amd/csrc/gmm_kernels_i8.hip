// gmm_kernels_i8.hip -- MI355X (gfx950) kernels of the diagonal-GMM feature scorer: the quantized ones.
//
// Hot path: for a batch of F frames and every mixture e of the model,
//   score(e,t) = min_{d in e} [ c_d + || A_d - x_t ||^2 ]   (+ argmin)
// RASR computes it per frame and density with a JIT'd SSE2 u8 SSD
// (src/Mm/SimdFeatureScorer.cc:158-176, src/Mm/SSE2CodeGenerator.cc:324-374)
// or SSE float code (src/Mm/GaussDiagonalMaximumFeatureScorer.cc:116-218).
// Here the cross term is a dense (densities x K) . (K x frames) contraction on
// the matrix cores and the per-mixture minimum is a running min in the MFMA
// accumulator registers, reduced across the wave once per mixture:
//
//   quantized (SIMD-diagonal-maximum, batch-int; this file): v_mfma_i32_16x16x64_i8
//     on s8 operands (q - 128); exact integer arithmetic; epilogue per element is
//     one v_lshl_add (constant + 2*dot, packed with the density index in the
//     low bits) and half a v_min3_i32 -> bit-identical scores and argmins;
//   float (diagonal-maximum, batch-float, diagonal-sum): gmm_kernels_split.hip
//     (f32 operands as two f16 pieces on the f16 matrix cores) and
//     gmm_kernels_f32.hip (v_mfma_f32_16x16x4_f32).
//
// Work decomposition: one 256-thread workgroup = 4 waves x NF column blocks of
// 16 frames; it walks a chunk of consecutive mixtures (all their tiles of 16
// densities).  Workgroups that share a chunk are placed on one XCD (blockIdx %
// 8) and run back to back, so each chunk's tiles are fetched from HBM/MALL into
// that XCD's L2 once and re-read from L2 by the other frame tiles.
//
// Every kernel is compiled with -ffp-contract=off; the quantizer additionally
// uses __fmul_rn / __fadd_rn so it can never be contracted into an FMA.
//
// This file: the quantized kernels (built with -mllvm -amdgpu-mfma-vgpr-form, see Makefile).
#include <type_traits>

#include "gmm_device.hh"

#ifndef GMM_I8_SLOTS
#define GMM_I8_SLOTS 1  // scoreI8Seg: running-minimum registers per column block (1, 2 or 4; 1: -0.7 %)
#endif

namespace rasr_gmm {
namespace dev {

// ---------------------------------------------------------------------------
// frame preparation (quantized): Context::Context, SimdFeatureScorer.cc:22-35
//   frameQ [C][nFramesPad][KS*64] s8 (q - 128, 0 in the padding), frameSS [C][nFramesPad] = sum (q-128)^2
// ---------------------------------------------------------------------------
// 32 threads per (covariance, frame), 8 per 256-thread block: thread t quantizes the 16-byte block t of the
// frame's KS x 64 bytes (KS <= 8) and the frame's sum of squares is a shuffle sum (integer: any order).  One
// thread per frame walking the bytes serially took most of a small host call's preparation time.
__global__ __launch_bounds__(256) void prepareFramesI8(const float* __restrict__ frames, uint32_t nFrames,
                                                        uint32_t frameStride, uint32_t nFramesPad,
                                                        uint32_t nFramesRead, uint32_t D,
                                                        uint32_t C, uint32_t KS, const float* __restrict__ isv,
                                                        int8_t* __restrict__ frameQ, int32_t* __restrict__ frameSS) {
    const uint32_t g = blockIdx.x * 8u + (threadIdx.x >> 5), blk = threadIdx.x & 31u;
    if (g >= C * nFramesRead)
        return;  // whole 32-thread groups leave together
    const uint32_t c = g / nFramesRead, f = g % nFramesRead;
    const float*   x  = frames + static_cast<size_t>(f) * frameStride;
    const float*   iv = isv + static_cast<size_t>(c) * KS * 64;
    i32x4*         out = reinterpret_cast<i32x4*>(frameQ + (static_cast<size_t>(c) * nFramesPad + f) * KS * 64);
    int            ss = 0;
    if (blk < KS * 4) {
        i32x4 w;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
            uint32_t word = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint32_t k = blk * 16 + q4 * 4 + b;
                int            v = 0;
                if (f < nFrames && k < D) {
                    v = quantizeCentered(__fmul_rn(x[k], iv[k]));  // multiplyAndQuantize, IntelOptimization.cc:63
                    ss += v * v;
                }
                word |= (static_cast<uint32_t>(v) & 0xffu) << (8 * b);
            }
            w[q4] = static_cast<int>(word);
        }
        out[blk] = w;
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)
        ss += __shfl_xor(ss, o, 32);
    if (blk == 0)
        frameSS[static_cast<size_t>(c) * nFramesPad + f] = ss;
}

// ---------------------------------------------------------------------------
// quantized scorer
// ---------------------------------------------------------------------------
// Finalize and store the per-mixture minima: lane `lane` holds, in res[i], the packed (score, density) minimum
// of frame frame0 + 64 i + lane (both quantized kernels leave their reduce-scatter in this order).
template <int NPL, bool MAYBE_NONE, int NONE_FROM = INT_MAX>
__device__ __forceinline__ void finalizeStoreI8(const I8Args& a, float* __restrict__ scores,
                                                uint32_t* __restrict__ bestOut, const int (&res)[NPL], uint32_t m,
                                                uint32_t frame0, int lane, int ib, const int (&ssOut)[NPL]) {
    const uint32_t mo = m;
    // frames >= nFrames fall outside num_records: the buffer stores drop them (no per-lane branch; -0.75 %
    // against a per-lane frame test, profiles/r02)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(scores + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                     static_cast<int>(a.nFrames * 4u), 0x00020000);
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(bestOut ? bestOut + static_cast<size_t>(mo) * a.scoreStride
                                                              : nullptr,
                                                     (short)0, static_cast<int>(a.nFrames * 4u), 0x00020000);
    // Both reference finalizes divide by b = 2 s^2: SimdFeatureScorer.cc:142 (f32)(0.5 * q / (f64)s2) and
    // BatchFeatureScorer.cc:468 (f32)best / scale_ (scale_ = 2 s^2).  y = RN(x / b) from x (rh + rl) (1/b as two
    // floats: within 2^-47 of x / b after one rounding, so a faithful quotient) and one Markstein correction
    // (no special operands here: x a float integer, b a normal positive float).  batch: exactly the reference
    // (x = (f32) best).  SIMD, |q| < 2^24: x = q; a quotient of two floats is never an f32 midpoint, and q / b
    // is >= 2^-49 relative away from one, so the reference's double quotient (2^-53) rounds to the same f32.
    // Larger |q| (never from a real mixture), and scales outside the range where this applies (finDivide),
    // divide as the reference (tests/test_fastdiv_finalize.py: both in exact arithmetic).
    // All NPL values take the multiply-and-correct path first, then ONE test decides the rare exact division (a
    // test per value cost a branch and scalar mask juggling per value in the emit; -0.6 % batch-int, s24).
    // ScaledContextScorer::score (ScaledFeatureScorer.hh:62-64): a finite score times 1.0f is itself, so the
    // multiply is unconditional.
    float sc[NPL];
    int   qv[NPL];
    bool  far = false;  // this lane holds a SIMD q outside +-2^24 (never from a real mixture)
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const int  packed = res[i];
        const bool none   = MAYBE_NONE && packed >= NONE_FROM;  // no densities: Core::Type<int>::max
        qv[i]             = none ? INT_MAX : (packed >> ib) + ssOut[i];
        const float x = static_cast<float>(qv[i]), b = a.finB, r = a.finInv;
        const float y = __fmaf_rn(x, r, __fmul_rn(x, a.finInvLo));
        sc[i]         = __fmaf_rn(__fmaf_rn(-b, y, x), r, y);
        far           = far || static_cast<uint32_t>(qv[i] + (1 << 24)) >= (2u << 24);
    }
    if (a.finDivide != 0 || (a.flavor == 0 && far)) {
#pragma unroll
        for (int i = 0; i < NPL; ++i)
            if (a.finDivide != 0 || static_cast<uint32_t>(qv[i] + (1 << 24)) >= (2u << 24))
                sc[i] = a.flavor == 0 ? static_cast<float>(0.5 * static_cast<double>(qv[i]) / static_cast<double>(a.s2))
                                      : __fdiv_rn(static_cast<float>(qv[i]), a.batchScale);
    }
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        const uint32_t f   = frame0 + 64 * i + lane;
        const bool     none = MAYBE_NONE && res[i] >= NONE_FROM;
        const uint32_t dns  = none ? 0xffffffffu : static_cast<uint32_t>(res[i]) & ((1u << ib) - 1u);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(__fmul_rn(a.outScale, sc[i])), rs, f * 4u, 0,
                                              GMM_STORE_CPOL);
        if (bestOut)
            __builtin_amdgcn_raw_buffer_store_b32(dns, rb, f * 4u, 0, GMM_STORE_CPOL);
    }
}

// Per-mixture end: 4 rows in-lane, reduce-scatter over the 4 lane groups, finalize and store the
// scores (and best densities) of the wave's NF*16 frames for mixture m.  MAYBE_NONE: the minimum may
// still be INT_MAX (a mixture without densities; preselection: none selected).  A mixture with tiles
// never reaches INT_MAX otherwise (the host bounds every real row's packed value below 2^31 - 2^(ib+1),
// gmm_prepare.cc), so the scorer's per-mixture emit skips those selects (v_cndmask issues at a
// quarter of the rate of the other VALU ops).
template <int NF, bool MAYBE_NONE = true, int S = 4, int NONE_FROM = INT_MAX>
__device__ __forceinline__ void emitMixtureI8(const I8Args& a, float* __restrict__ scores, uint32_t* __restrict__ bestOut,
                                              const int (&best)[NF][S], uint32_t m, uint32_t frame0, int lane, int g,
                                              int ib, const int (&ssOut)[NF / 4]) {
    constexpr int NPL = NF / 4;
    // per-mixture reduction: the S running minima of a column block in-lane, then a reduce-scatter over
    // the 4 lane groups
    int v[NF];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        if constexpr (S == 4)
            v[cb] = min(min(best[cb][0], best[cb][1]), min(best[cb][2], best[cb][3]));
        else {
            int x = best[cb][0];
#pragma unroll
            for (int r = 1; r < S; ++r)
                x = min(x, best[cb][r]);
            v[cb] = x;
        }
    }
    int w[NF / 2];  // after the lane^32 step: column blocks cb with bit1 == (g >> 1)
    int res[NPL];   // after the lane^16 step: column block cb = g + 4 i
#pragma unroll
    for (int p = 0; p < NF / 2; ++p) {
        const int c = (p & 1) | ((p >> 1) << 2);  // 0,1,4,5: bit1 clear
        w[p]        = swapMin32(v[c], v[c ^ 2]);
    }
#pragma unroll
    for (int i = 0; i < NPL; ++i)
        res[i] = swapMin16(w[2 * i], w[2 * i + 1]);

    finalizeStoreI8<NPL, MAYBE_NONE, NONE_FROM>(a, scores, bestOut, res, m, frame0, lane, ib, ssOut);
}

template <int NF, int KS, bool MULTI>
__global__ __launch_bounds__(256) void scoreI8(I8Args a) {
    static_assert(NF == 4 || NF == 8, "NF");
    constexpr int NPL = NF / 4;  // results per lane per mixture
    const int     lane = threadIdx.x & 63;
    const int     wave = threadIdx.x >> 6;
    const int     g    = lane >> 4;
    uint32_t      chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * (4u * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const int      ib = static_cast<int>(a.idxBits);
    const i32x4*   tA = static_cast<const i32x4*>(a.tileA);
    const i32x4*   tP = static_cast<const i32x4*>(a.tileP);

    // frame operands (B fragments) of covariance 0; per-lane frame = frame0 + 16 cb + (lane & 15)
    i32x4      B[NF][KS];
    int        ssCol[NF];  // MULTI: sum sq of the column's frame for the current covariance
    uint32_t   curCov = 0;
    const auto loadB  = [&](uint32_t cov) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            const uint32_t f = frame0 + cb * 16 + (lane & 15);
            const i32x4*   q = reinterpret_cast<const i32x4*>(
                    a.frameQ + (static_cast<size_t>(cov) * a.nFramesPad + f) * (KS * 64)) + g;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
                B[cb][ks] = q[ks * 4];
            if constexpr (MULTI)
                ssCol[cb] = a.frameSS[static_cast<size_t>(cov) * a.nFramesPad + f];
        }
    };
    loadB(0);
    int ssOut[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i)
        ssOut[i] = MULTI ? 0 : a.frameSS[frame0 + 64 * i + lane];

    // Tile operands in flight: (A0, P0) = tile t, (A1, P1) = tile t+1.  The tile arrays carry
    // kTilePad zero tiles at the end, so the two-ahead prefetch never needs a bound check.
    uint32_t   t = a.mixTileOff[m0];
    i32x4      A0[KS], A1[KS];
    i32x4      P0, P1;
    const auto loadTile = [&](uint32_t tt, i32x4(&A)[KS], i32x4& P) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            A[ks] = tA[(static_cast<size_t>(tt) * KS + ks) * 64 + lane];
        P = tP[static_cast<size_t>(tt) * 4 + g];
    };
    loadTile(t, A0, P0);
    loadTile(t + 1, A1, P1);
    const uint32_t sh = static_cast<uint32_t>(ib + 1);
    // packed = (c + sum a'^2 + 2 dot(-a', b')) << ib | density   (see gmm_prepare.cc): one v_lshl_add
    const auto pack = [&](int acc, int p) {
        return static_cast<int>((static_cast<uint32_t>(acc) << sh) + static_cast<uint32_t>(p));
    };

    for (uint32_t m = m0; m < m1; ++m) {
        const uint32_t tEnd = a.mixTileOff[m + 1];
        int            best[NF][4];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                best[cb][r] = INT_MAX;

        if constexpr (!MULTI) {
            // two tiles per step: 2 NF independent MFMAs, the operands of tiles t+2, t+3 loaded
            // behind them, one v_min3 per pair of candidates
            for (; t + 1 < tEnd; t += 2) {
                i32x4 accA[NF], accB[NF];
#pragma unroll
                for (int cb = 0; cb < NF; ++cb) {
                    accA[cb] = i32x4{0, 0, 0, 0};
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks)
                        accA[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0[ks], B[cb][ks], accA[cb], 0, 0, 0);
                }
                const i32x4 PA = P0;
                loadTile(t + 2, A0, P0);
#pragma unroll
                for (int cb = 0; cb < NF; ++cb) {
                    accB[cb] = i32x4{0, 0, 0, 0};
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks)
                        accB[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1[ks], B[cb][ks], accB[cb], 0, 0, 0);
                }
                const i32x4 PB = P1;
                loadTile(t + 3, A1, P1);
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        best[cb][r] = min(best[cb][r], min(pack(accA[cb][r], PA[r]), pack(accB[cb][r], PB[r])));
            }
            if (t < tEnd) {  // odd tile count: last tile alone
                i32x4 accA[NF];
#pragma unroll
                for (int cb = 0; cb < NF; ++cb) {
                    accA[cb] = i32x4{0, 0, 0, 0};
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks)
                        accA[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0[ks], B[cb][ks], accA[cb], 0, 0, 0);
                }
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        best[cb][r] = min(best[cb][r], pack(accA[cb][r], P0[r]));
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    A0[ks] = A1[ks];
                P0 = P1;
                loadTile(t + 2, A1, P1);
                ++t;
            }
        }
        else {
            // several covariances: the frame operand follows the tile's covariance
            for (; t < tEnd; ++t) {
                const uint32_t cov = a.tileCov[t];
                if (cov != curCov) {
                    curCov = cov;
                    loadB(cov);
                }
#pragma unroll
                for (int cb = 0; cb < NF; ++cb) {
                    i32x4 acc = {0, 0, 0, 0};
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks)
                        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0[ks], B[cb][ks], acc, 0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int v = static_cast<int>(static_cast<uint32_t>(pack(acc[r], P0[r])) +
                                                       (static_cast<uint32_t>(ssCol[cb]) << ib));
                        best[cb][r] = min(best[cb][r], v);
                    }
                }
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    A0[ks] = A1[ks];
                P0 = P1;
                loadTile(t + 2, A1, P1);
            }
        }

        emitMixtureI8<NF>(a, a.scores, a.best, best, m, frame0, lane, g, ib, ssOut);
    }
}

// ---------------------------------------------------------------------------
// quantized scorer, single covariance, tile operands staged through LDS
//
// The four waves of a workgroup read the same tiles (they differ only in
// frames), so the tiles are fetched once per workgroup into an LDS ring of two
// segments of kSegTiles tiles by LDS-DMA (global_load_lds_dwordx4: one 1 KiB
// wave-instruction per 1 KiB operand block), a whole segment ahead of use.
// Per segment: wait for its DMA (counted vmcnt: every wave issues the same
// number of pieces), barrier, compute from LDS, barrier, refill the buffer with
// the segment after next.  Mixture boundaries are independent of segment
// boundaries.
// ---------------------------------------------------------------------------
#ifndef GMM_I8_SEG
#define GMM_I8_SEG 16  // tiles per LDS segment (A/B at 32768 frames: 16 -1.2 % vs 8, 4 +1.6 %; kTilePad >= SEG)
#endif
constexpr int kSegTiles = GMM_I8_SEG;

// preselection-batch-int: the segment ring and the waves' mask tables share one dynamic LDS array
extern __shared__ __attribute__((aligned(16))) int8_t i8DynLds[];

// The mixture boundaries and words are read through the constant address space (constTable, gmm_device.hh), so
// they stay scalar loads after the emit's stores (a vector load would need an s_waitcnt vmcnt(0) that drains the
// LDS-DMA queue).
//
// PRESEL (preselection-batch-int, NF = kI8PreselNF: 8, a wave's 128 frames are two 64-frame mask words; 4 kept
// for A/B): keys are biased by 2^31
// (the packed row constant XOR 2^31) and compared unsigned, so OR-ing the sign-extended mask byte of a
// (frame, density cluster) that the frame did not select makes the all-ones key, which never wins; the
// segment carries each tile's 16 row byte offsets into the wave's mask table (gmm_kernels_presel.hip).  The
// table has one entry past the clusters, "never selected", for padding rows and the stand-in tile.
// PRESEL with SCORE_ONLY (the default for preselection-batch-int, a batch type without best densities): the
// class layout below with the biased h as the MFMA's C input, so a class candidate is the accumulator u = v + 2^31
// and the mask is one v_or per candidate (no pack); a mixed candidate is 2 u + (p | 2^31) = 2 v + p + 2^31.
#ifndef GMM_I8_WAVES
#define GMM_I8_WAVES 4  // scoreI8Seg, one K step: waves per SIMD the register allocation must allow (0 = free)
#endif
//
// SCORE_ONLY (calls without best densities on the class layout, gmm_prepare.cc buildClassLayout): the row
// constant h = Q >> 1 is the MFMA's C input, so the accumulator holds v = dot + h (no pack: there is no density
// index to carry).  A mixture's class tiles come first: all their rows in lane group g have the parity p_g of Q
// (bit g of the mixture word mixOddMask[m]), so the running minimum there is one v_min3 per two candidates
// straight on the accumulators, and the lane's minimum of 2 dot + Q is 2 min(v) + p_g.  Its mixed tiles follow
// (word bits 16-31: the class tile count; bits 4-15: er): row 4g + r of mixed tile i has parity
// (16 i + 4g + r >= er), and their candidates 2 v + p go to a second running minimum, merged at the mixture end.
// A pair step holds two tiles of one kind.
template <int NF, int KS, bool PRESEL = false, int SEG = kSegTiles, bool SCORE_ONLY = false, int W = 4>
__global__ __launch_bounds__(64 * W, (KS == 1 && !PRESEL && GMM_I8_WAVES && W == 4) ? GMM_I8_WAVES : 1) void scoreI8Seg(I8Args a, const uint32_t* __restrict__ mixTileOffArg,
                                                   float* __restrict__ scores, uint32_t* __restrict__ bestOut,
                                                   const uint32_t* __restrict__ mixOddMaskArg = nullptr) {
    const auto mixTileOff = constTable(mixTileOffArg);
    const auto mixOddMask = constTable(mixOddMaskArg);
    static_assert(NF == 4 || NF == 8, "NF");
    static_assert(W == 4 || (W == 1 && !PRESEL), "waves per workgroup: 4, or 1 for small calls (no preselection)");
    static_assert(!PRESEL || NF == 4 || NF == 8, "preselection masks: one or two 64-frame words per wave");
    // PRESEL mask table entries: NF 4 a byte (4 deselection bits x 4: the byte offset of a u32 in maskLut), NF 8 a
    // u16 (8 bits x 8: the byte offset of a u64 in maskLut)
    constexpr uint32_t kEntryBytes = 1u;
    typedef typename std::conditional<NF == 8, uint64_t, uint32_t>::type LutW;  // a maskLut entry
    typedef uint2 MaskW;  // a row's mask bytes as registers: x blocks 0-3, y blocks 4-7 (NF 8)
    static_assert(!SCORE_ONLY || KS == 1, "score-only layout: one K step");
    constexpr int      kSegTiles = SEG;
    constexpr int      NPL       = NF / 4;
    constexpr uint32_t kTileA    = KS * 1024;                   // operand bytes per tile
    constexpr uint32_t kSegA     = kSegTiles * kTileA;
    constexpr uint32_t kSegP     = kSegA + kSegTiles * 64;      // + packed row constants
    constexpr uint32_t kSegBytes = kSegP + (PRESEL ? kSegTiles * 64 : 0);  // + row cluster offsets (u32)
    constexpr int      kPieces   = kSegTiles * KS / W;          // 1 KiB pieces per wave per segment
    constexpr uint32_t kRowLanes = 4 * kSegTiles / W;           // lanes loading 16 B of row constants per wave
    constexpr int      kIssued   = kPieces + 1 + (PRESEL ? 1 : 0);  // vector memory ops per wave per segment
    static_assert(kSegTiles * KS % W == 0 && kRowLanes <= 64, "segment pieces must split evenly over the waves");
    // after the ring: the stand-in second tile of a step that has one tile left (odd tile count, segment
    // end): zero operands (dot = 0), rows that never win, cluster offsets 0.  Every step is then a pair
    // step: one loop body, whose running minima stay in their registers (a second, single-tile body made
    // the compiler copy all NF*4 minima back at every step that did not end a mixture)
    constexpr uint32_t kDummyBytes = kI8DummyTileBytes(KS, PRESEL);
    // one __shared__ array per instantiation: PRESEL the dynamic one only (its size depends on the cluster count)
    // PRESEL: the 16-entry mask LUT is a static array (its address folds into the ds_read offset; the dynamic
    // array's base is a relocation the compiler adds per read), ring and tables the dynamic one
    int8_t* lds;
    LutW*   maskLut = nullptr;
    if constexpr (PRESEL) {
        __shared__ LutW lutStatic[NF == 8 ? 256 : 16];
        lds     = i8DynLds;
        maskLut = lutStatic;
    }
    else {
        __shared__ __attribute__((aligned(16))) int8_t ldsStatic[2 * kSegBytes + kDummyBytes];
        lds = ldsStatic;
    }

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g    = lane >> 4;
    uint32_t  chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;  // uniform over the workgroup, before any barrier
    const uint32_t frame0 = ft * (W * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const int      ib = static_cast<int>(a.idxBits);
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];
    const uint32_t nSeg = (T1 - T0 + kSegTiles - 1) / kSegTiles;
    const int8_t*  gA   = static_cast<const int8_t*>(a.tileA);
    const int8_t*  gP   = static_cast<const int8_t*>(a.tileP);
    const int8_t*  gClu = static_cast<const int8_t*>(a.tileClu);
    (void)gClu;

    // issue segment s into buffer (s & 1); tile arrays are padded by kTilePad >= kSegTiles tiles
    const auto issueSeg = [&](uint32_t s) {
        const uint32_t t0   = T0 + s * kSegTiles;
        int8_t*        base = lds + (s & 1u) * kSegBytes;
#pragma unroll
        for (int i = 0; i < kPieces; ++i) {
            const uint32_t piece = static_cast<uint32_t>(wave * kPieces + i);
            __builtin_amdgcn_global_load_lds(gA + static_cast<size_t>(t0) * kTileA + piece * 1024u + lane * 16,
                                             base + piece * 1024u, 16, 0, 0);
        }
        if (lane < kRowLanes)  // kSegTiles tiles x 64 B of row constants: 16 kRowLanes B per wave
            __builtin_amdgcn_global_load_lds(gP + static_cast<size_t>(t0) * 64 + wave * (kRowLanes * 16) + lane * 16,
                                             base + kSegA + wave * (kRowLanes * 16), 16, 0, 0);
        if constexpr (PRESEL) {  // kSegTiles tiles x 64 B of row cluster offsets: 16 kSegTiles B per wave
            if (lane < kSegTiles)
                __builtin_amdgcn_global_load_lds(gClu + static_cast<size_t>(t0) * 64 + wave * (kSegTiles * 16) + lane * 16,
                                                 base + kSegP + wave * (kSegTiles * 16), 16, 0, 0);
        }
    };
    {
        int8_t* const dummy = lds + 2 * kSegBytes;
        // non-PRESEL rows compare signed (INT_MAX never wins), PRESEL rows unsigned (biased: all ones, and their
        // rows sit in the never-selected cluster, so every kind of step masks them to all ones);
        // SCORE_ONLY: the class layout's padding value (2 v + 1 of a mixed step stays inside int32)
        const uint32_t never    = PRESEL ? 0xffffffffu : (SCORE_ONLY ? 0x30000000u : 0x7fffffffu);
        const uint32_t neverClu = PRESEL ? a.nClusters * 16u * kEntryBytes : 0u;  // u32 row offsets
        for (uint32_t i = threadIdx.x; i < kDummyBytes / 4; i += 64u * W)
            reinterpret_cast<uint32_t*>(dummy)[i] = (i >= kTileA / 4 && i < kTileA / 4 + 16)
                                                            ? never
                                                            : (i >= kTileA / 4 + 16 ? neverClu : 0u);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ordered before use by the first segment's barrier
    }
    // preselection: this wave's mask table [cluster][16] after the segment ring
    const uint32_t tabBase = 2 * kSegBytes + kDummyBytes;
    const uint32_t words   = PRESEL ? a.nClusters * 16u : 0u;  // entries of a table (u32 words of a 64-frame block)
    const uint32_t tabOff  = tabBase + static_cast<uint32_t>(wave) * (words + 16u) * kEntryBytes;
    if constexpr (PRESEL && NF == 8) {
        // the wave's 128 frames' table, built once per call (launchCompactSelection), by LDS-DMA ahead of the ring
        // (the oldest vector-memory operations: the first segment's counted wait covers them)
        const int8_t*  src   = reinterpret_cast<const int8_t*>(a.selC + static_cast<size_t>(frame0 / 128u) * words);
        const uint32_t bytes = words;
        for (uint32_t off = 0; off < bytes; off += 1024u)
            if (off + static_cast<uint32_t>(lane) * 16u < bytes)
                __builtin_amdgcn_global_load_lds(src + off + lane * 16, lds + tabOff + off, 16, 0, 0);
    }
    if (nSeg > 0)
        issueSeg(0);
    if (nSeg > 1)
        issueSeg(1);

    i32x4 B[NF][KS];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        const uint32_t f = frame0 + cb * 16 + (lane & 15);
        const i32x4*   q = reinterpret_cast<const i32x4*>(a.frameQ + static_cast<size_t>(f) * (KS * 64)) + g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            B[cb][ks] = q[ks * 4];
    }
    int ssOut[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i)
        ssOut[i] = a.frameSS[frame0 + 64 * i + lane];

    // preselection: this wave's mask table [cluster][16] after the segment ring
    uint32_t laneSel = 0;  // byte offset of (wave table, column t = lane & 15)
    // compressed: per (cluster, t) the bits "frame 16 cb + t did not select the cluster" (bit cb), stored as the byte
    // offset of the entry of maskLut that expands them to one 0x00 / 0xff mask byte per column block (NF 4: 4 KiB
    // per wave instead of 16, 5 workgroups per CU instead of 2).  NF 8: the table came by LDS-DMA (above)
    if constexpr (PRESEL) {
        for (uint32_t n = threadIdx.x; n < (NF == 8 ? 256u : 16u); n += 256u) {
            LutW v = 0;
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                v |= ((n >> cb) & 1u) ? LutW(0xff) << (8 * cb) : LutW(0);
            maskLut[n] = v;
        }
        if constexpr (NF == 4) {
            // the selection words of this wave's frames: one 64-frame block; bit 0 of byte q (0x00 / 0xff) of a
            // word says frame 16 q + t of the block did not select the cluster
            const i32x4* src0 = reinterpret_cast<const i32x4*>(a.selT + static_cast<size_t>(frame0 / 64u) * words);
            const auto   nib  = [](uint32_t w) { return ((w & 0x01010101u) * 0x01020408u) >> 24 & 0xfu; };  // bit q = byte q
            for (uint32_t i = static_cast<uint32_t>(lane); i < words / 4u; i += 64u) {
                const i32x4 w0     = src0[i];
                uint32_t    packed = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j)  // entry: 4 * the 4 bits
                    packed |= (nib(static_cast<uint32_t>(w0[j])) * 4u) << (8 * j);
                reinterpret_cast<uint32_t*>(lds + tabOff)[i] = packed;
            }
        }
        // the never-selected cluster: every frame deselected, in all 16 columns (NF 8: LUT index 255; NF 4: byte
        // offset 4 * 15)
        if (lane < 4)
            reinterpret_cast<uint32_t*>(lds + tabOff + words * kEntryBytes)[lane] = NF == 8 ? 0xffffffffu : 0x3c3c3c3cu;
        laneSel = tabOff + (static_cast<uint32_t>(lane) & 15u) * kEntryBytes;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LUT and entries before the first segment's barrier
    }
    // a tile's row constants (the host biases them by 2^31 for PRESEL) and mask words of this lane's 4 rows,
    // from the tile's 64-byte row-constant block pRow and 64-byte cluster-offset block cRow
    const auto tileRows = [&](const int8_t* pRow, const int8_t* cRow, i32x4& P, MaskW(&T)[4]) {
        P = *reinterpret_cast<const i32x4*>(pRow + g * 16);
        (void)cRow;
        if constexpr (PRESEL) {
            // the lane group's 4 row offsets (u32 cluster * 16 * entry bytes: byte offsets into the wave's table) as
            // one aligned 16-byte read (a 64-bit read of the DMA-filled ring made the waitcnt pass drain the DMA
            // queue, s_waitcnt vmcnt(0), at every pair step); table entries are LUT byte offsets
            const i32x4   c4 = *reinterpret_cast<const i32x4*>(cRow + g * 16);
            const int8_t* tb = lds + laneSel;
            const int8_t* lu = reinterpret_cast<const int8_t*>(maskLut);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t e = *reinterpret_cast<const uint8_t*>(tb + c4[j]);
                if constexpr (NF == 8)  // e: the LUT index (the 8 deselection bits)
                    T[j] = *reinterpret_cast<const uint2*>(lu + e * 8u);
                else
                    T[j] = uint2{*reinterpret_cast<const uint32_t*>(lu + e), 0u};
            }
        }
    };

    const uint32_t sh   = static_cast<uint32_t>(ib + 1);
    const auto     pack = [&](int acc, int p) {
        return static_cast<int>((static_cast<uint32_t>(acc) << sh) + static_cast<uint32_t>(p));
    };
    // PRESEL: x OR the sign-extended mask byte of column block cb (0xff: the frame did not select the row's
    // cluster), one v_or_b32_sdwa
    const auto maskOr = [](int x, MaskW T, int cb) -> int {
        // the 32-bit half holding block cb's byte (NF 8: the high half for blocks 4-7), then its byte
        const uint32_t h = (NF == 8 && cb >= 4) ? T.y : T.x;
        return static_cast<int>(static_cast<uint32_t>(x) |
                                static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(h >> (8 * (cb & 3))))));
    };
    (void)maskOr;
    // candidate key: the packed value; PRESEL: biased, OR the mask byte of column block cb
    const auto cand = [&](int acc, int p, MaskW T, int cb) -> int {
        if constexpr (PRESEL)
            return maskOr(pack(acc, p), T, cb);
        else
            return pack(acc, p);
    };
    const auto min2 = [](int x, int y) {
        if constexpr (PRESEL)
            return static_cast<int>(min(static_cast<uint32_t>(x), static_cast<uint32_t>(y)));
        else
            return min(x, y);
    };
    // running minima per column block: every key carries its density index, so the 4 row slots of a
    // lane can share kSlots registers (fewer to reduce and reset at each mixture end)
    // two K steps: 4 (fewer live values to schedule around); SCORE_ONLY: 2 (a chain of dependent v_min3 on one
    // register costs a wait state per link)
    constexpr int kSlots = SCORE_ONLY ? 2 : (KS == 1 ? GMM_I8_SLOTS : 4);
    static_assert(kSlots == 1 || kSlots == 2 || kSlots == 4, "slots");
    // SCORE_ONLY: minima of v = dot + h over a mixture's class tiles; at its first mixed tile they become 2 v + p_g
    // in place, and the mixed tiles' 2 v + p join them
    int best[NF][kSlots];
    const auto resetBest = [&]() {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < kSlots; ++r)  // PRESEL: 0xffffffff = biased INT_MAX; SCORE_ONLY: 2 v + 1 fits
                best[cb][r] = PRESEL ? -1 : (SCORE_ONLY ? 0x3fffffff : INT_MAX);
    };
    // SCORE_ONLY: the class tiles' minima of mixture mm as 2 v + p_g (this lane group's parity there)
    // PRESEL: biased, u = v + 2^31 -> 2 v + p + 2^31 = 2 u + (p | 2^31), all ones (nothing selected) kept
    const auto toMixed = [&](uint32_t mm) {
        const uint32_t p = ((mixOddMask[mm] >> g) & 1u) | (PRESEL ? 0x80000000u : 0u);
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < kSlots; ++r) {
                const uint32_t u = static_cast<uint32_t>(best[cb][r]);
                best[cb][r]      = static_cast<int>((PRESEL && u == 0xffffffffu) ? u : (u << 1) + p);
            }
    };
    uint32_t m    = m0;
    uint32_t tEnd = mixTileOff[m0 + 1];
    // SCORE_ONLY: the end of mixture m's class tiles, and its mixed rows' first odd index
    uint32_t tCls = 0, er = 0;
    // hot: the end of a mixture with tiles (its minimum is a real row: no INT_MAX case, unless PRESEL)
    const auto emit = [&](uint32_t mm, auto hot) {
        constexpr bool kMaybeNone = PRESEL || !decltype(hot)::value;
        if constexpr (SCORE_ONLY) {
            if constexpr (decltype(hot)::value) {
                // a mixture without mixed tiles still holds its class minima v: 2 v + p_g (uniform test)
                if (tCls >= tEnd)
                    toMixed(mm);
                if constexpr (PRESEL) {  // unbiased: 2 v + p, INT_MAX where the frame selected none of its rows
                    int unb[NF][kSlots];
#pragma unroll
                    for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                        for (int r = 0; r < kSlots; ++r)
                            unb[cb][r] = static_cast<int>(static_cast<uint32_t>(best[cb][r]) ^ 0x80000000u);
                    emitMixtureI8<NF, kMaybeNone, kSlots>(a, scores, bestOut, unb, mm, frame0, lane, g, 0, ssOut);
                }
                else
                    emitMixtureI8<NF, kMaybeNone, kSlots>(a, scores, bestOut, best, mm, frame0, lane, g, 0, ssOut);
            }
            else {
                int none[NF][1];  // a mixture without tiles: Core::Type<int>::max
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
                    none[cb][0] = INT_MAX;
                emitMixtureI8<NF, kMaybeNone, 1>(a, scores, bestOut, none, mm, frame0, lane, g, 0, ssOut);
            }
        }
        else if constexpr (PRESEL) {
            int unb[NF][kSlots];
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                for (int r = 0; r < kSlots; ++r)
                    unb[cb][r] = static_cast<int>(static_cast<uint32_t>(best[cb][r]) ^ 0x80000000u);
            emitMixtureI8<NF, kMaybeNone, kSlots>(a, scores, bestOut, unb, mm, frame0, lane, g, ib, ssOut);
        }
        else {
            emitMixtureI8<NF, kMaybeNone, kSlots>(a, scores, bestOut, best, mm, frame0, lane, g, ib, ssOut);
        }
    };
    const std::true_type  kHot{};
    const std::false_type kEmpty{};
    resetBest();
    // mixture m starts at tile tBeg (the previous mixture's end: no second load of its offset)
    const auto mixWord = [&](uint32_t tBeg) {
        if constexpr (SCORE_ONLY) {
            if (m < m1) {
                const uint32_t w = mixOddMask[m];
                tCls             = tBeg + (w >> 16);
                er               = (w >> 4) & 0xfffu;
            }
        }
    };
    // mixtures without tiles at the start of the chunk
    while (m < m1 && tEnd == T0) {
        emit(m, kEmpty);
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T1;
    }
    mixWord(T0);

    for (uint32_t s = 0; s < nSeg; ++s) {
        // this segment's pieces (issued one segment ago) have landed; the next segment's stay in flight
        if (s + 1 < nSeg)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kIssued) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const int8_t*  base   = lds + (s & 1u) * kSegBytes;
        const uint32_t segT0  = T0 + s * kSegTiles;
        const uint32_t segEnd = min(segT0 + kSegTiles, T1);
        // one pair step at tile t: two tiles of the same mixture (SCORE_ONLY: of the same kind), or the last one
        // beside the never-winning stand-in: 2 NF independent MFMAs, one v_min3 per candidate pair.  kind: 0 key
        // layout, 1 class tiles, 2 mixed tiles
        const auto step = [&](const uint32_t t, const bool two, auto kindC) {
            constexpr int       kKind = decltype(kindC)::value;
            const uint32_t      lt    = t - segT0;
            const int8_t* const dummy = lds + 2 * kSegBytes;
            const int8_t* const a0    = base + lt * kTileA;
            const int8_t* const a1    = two ? a0 + kTileA : dummy;
            const int8_t* const p0    = base + kSegA + lt * 64;
            const int8_t* const p1    = two ? p0 + 64 : dummy + kTileA;
            const int8_t* const c0    = base + kSegP + lt * 64;
            const int8_t* const c1    = two ? c0 + 64 : dummy + kTileA + 64;
            i32x4               A0[KS], A1[KS];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                A0[ks] = *reinterpret_cast<const i32x4*>(a0 + ks * 1024 + lane * 16);
                A1[ks] = *reinterpret_cast<const i32x4*>(a1 + ks * 1024 + lane * 16);
            }
            i32x4 P0, P1;
            MaskW T0w[4] = {}, T1w[4] = {};
            tileRows(p0, c0, P0, T0w);
            tileRows(p1, c1, P1, T1w);
            i32x4      accA[NF], accB[NF];
            const auto mfmas = [&](int cb) {
                if constexpr (kKind != 0) {  // the row constants enter as the accumulator input
                    accA[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0[0], B[cb][0], P0, 0, 0, 0);
                    accB[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1[0], B[cb][0], P1, 0, 0, 0);
                    return;
                }
                accA[cb] = i32x4{0, 0, 0, 0};
                accB[cb] = i32x4{0, 0, 0, 0};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    accA[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A0[ks], B[cb][ks], accA[cb], 0, 0, 0);
                    accB[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A1[ks], B[cb][ks], accB[cb], 0, 0, 0);
                }
            };
            // SCORE_ONLY mixed step: the parity of this lane's row r in each tile (row 4g + r of mixed tile i is
            // remainder entry 16 i + 4g + r, odd from er on; the stand-in's rows never win either way)
            int        pA[4] = {}, pB[4] = {};
            // p = (row index >= er) as the sign bit of thr - r: a shift the compiler may not turn into a compare
            // and a v_cndmask (11.5 cycles per wave64 against 2.9)
            const auto parities = [&]() {
                const int thr = static_cast<int>(er) - 16 * static_cast<int>(t - tCls) - 4 * g - 1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    asm("v_lshrrev_b32 %0, 31, %1" : "=v"(pA[r]) : "v"(thr - r));
                    asm("v_lshrrev_b32 %0, 31, %1" : "=v"(pB[r]) : "v"(thr - 16 - r));
                    if constexpr (PRESEL) {  // the bias of the unsigned comparison: p | 2^31
                        pA[r] |= static_cast<int>(0x80000000u);
                        pB[r] |= static_cast<int>(0x80000000u);
                    }
                }
            };
            const auto epilogueMixed = [&](int cb) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ua = static_cast<int>((static_cast<uint32_t>(accA[cb][r]) << 1) + static_cast<uint32_t>(pA[r]));
                    const int ub = static_cast<int>((static_cast<uint32_t>(accB[cb][r]) << 1) + static_cast<uint32_t>(pB[r]));
                    int&      bs = best[cb][r % kSlots];
                    if constexpr (PRESEL) {  // masked: all ones; biased keys compare unsigned
                        const int ma = maskOr(ua, T0w[r], cb), mb = maskOr(ub, T1w[r], cb);
                        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(bs) : "v"(bs), "v"(ma), "v"(mb));
                        continue;
                    }
                    bs           = min(bs, min(ua, ub));
                    asm volatile("" : "+v"(bs));
                }
            };
            const auto epilogue = [&](int cb) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (kKind == 1 && PRESEL) {
                        // the accumulators (biased v) OR the mask: compiler-visible reads (hazard wait states)
                        int&      bs = best[cb][r % kSlots];
                        const int ma = maskOr(accA[cb][r], T0w[r], cb), mb = maskOr(accB[cb][r], T1w[r], cb);
                        asm("v_min3_u32 %0, %1, %2, %3" : "=v"(bs) : "v"(bs), "v"(ma), "v"(mb));
                        continue;
                    }
                    if constexpr (kKind == 1) {
                        // a compiler-visible min (not inline asm): the accumulators are read soon after their
                        // MFMAs, and only compiler-visible reads get the hazard wait states.  The empty asm keeps
                        // each update one v_min3 (the compiler would reassociate the chain into v_min pairs)
                        int& bs = best[cb][r % kSlots];
                        bs      = min(bs, min(accA[cb][r], accB[cb][r]));
                        asm volatile("" : "+v"(bs));
                        continue;
                    }
                    const int ca = cand(accA[cb][r], P0[r], T0w[r], cb), cc = cand(accB[cb][r], P1[r], T1w[r], cb);
                    if constexpr (kSlots < 4) {
                        // several keys into one register: keep each update one v_min3 (the compiler would
                        // otherwise reassociate the chain into a tree of two-operand v_min); PRESEL compares
                        // the biased keys unsigned
                        int& bs = best[cb][r % kSlots];
                        if constexpr (PRESEL)
                            asm("v_min3_u32 %0, %1, %2, %3" : "=v"(bs) : "v"(bs), "v"(ca), "v"(cc));
                        else
                            asm("v_min3_i32 %0, %1, %2, %3" : "=v"(bs) : "v"(bs), "v"(ca), "v"(cc));
                    }
                    else
                        best[cb][r % kSlots] = min2(best[cb][r % kSlots], min2(ca, cc));
                }
            };
            // software pipeline over the column blocks: chunks {MFMAs of block cb, epilogue of block cb - 1}
            // fenced by sched_barrier, so every epilogue reads results whose MFMA latency has passed (no
            // hazard s_nop in the stream: 3 wait states per pair step instead of 99; -2.6 % at 32768 frames)
            // SCORE_ONLY: the epilogue is 4 v_min3 per block, too short to cover the MFMA latency at lag 1; lag 3
            // leaves the compiler the fewest hazard waits (A/B, 32768 frames: lag 3 1.338 ms, lag 2 1.341, a
            // separate single-tile step for odd tile counts 1.362)
            const auto pipeline = [&](auto lagC, auto epi) {
                constexpr int kLag = decltype(lagC)::value;
#pragma unroll
                for (int cb = 0; cb < kLag; ++cb)
                    mfmas(cb);
#pragma unroll
                for (int cb = kLag; cb < NF; ++cb) {
                    __builtin_amdgcn_sched_barrier(0);
                    mfmas(cb);
                    epi(cb - kLag);
                    // inside the chunk: the MFMAs first, then the epilogue (the scheduler would lead with the VALU)
                    __builtin_amdgcn_sched_group_barrier(0x008, 2 * KS, 0);
                    __builtin_amdgcn_sched_group_barrier(0x002, 64, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int cb = NF - kLag; cb < NF; ++cb)
                    epi(cb);
            };
            if constexpr (kKind == 2) {  // lag 1: 1, 2, 3 measured within noise
                parities();
                pipeline(std::integral_constant<int, 1>{}, epilogueMixed);
            }
            else
                pipeline(std::integral_constant<int, kKind == 1 ? 3 : 1>{}, epilogue);
        };
        const std::integral_constant<int, 0> kKeyed{};
        const std::integral_constant<int, 1> kClass{};
        const std::integral_constant<int, 2> kMixed{};
        uint32_t t = segT0;
        while (t < segEnd) {
            if constexpr (SCORE_ONLY) {
                // this mixture's class tiles in this segment (a loop with no kind or mixture test per step), then
                // its mixed ones
                const uint32_t cEnd = min(segEnd, tCls);
                while (t < cEnd) {
                    const bool two = t + 1 < cEnd;
                    step(t, two, kClass);
                    t += two ? 2u : 1u;
                }
                const uint32_t mEnd = min(segEnd, tEnd);
                if (t < mEnd) {
                    if (t == tCls)  // the mixture's first mixed tile: its class minima become 2 v + p_g
                        toMixed(m);
                    do {
                        const bool two = t + 1 < mEnd;
                        step(t, two, kMixed);
                        t += two ? 2u : 1u;
                    } while (t < mEnd);
                }
            }
            else {
                const bool two = t + 1 < segEnd && t + 1 < tEnd;
                step(t, two, kKeyed);
                t += two ? 2u : 1u;
            }
            // the mixture ending here, and further ones without tiles ending at the same point (rare)
            if (t == tEnd && m < m1) {
                emit(m, kHot);
                resetBest();
                ++m;
                tEnd = m < m1 ? mixTileOff[m + 1] : T1;
                while (t == tEnd && m < m1) {
                    emit(m, kEmpty);
                    ++m;
                    tEnd = m < m1 ? mixTileOff[m + 1] : T1;
                }
                mixWord(t);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // every wave is done reading buffer (s & 1)
        if (s + 2 < nSeg)
            issueSeg(s + 2);
    }
}

// ---------------------------------------------------------------------------
// quantized scorer without best densities on the slot layout (gmm_prepare.cc buildSlotLayout): the SIMD
// scorer's score-only twin, batch-diagonal-maximum-int / -fast.
//
// One tile per step: NF MFMAs with the tile's row constants h as the C input, so the accumulator holds
// v = dot + h, and two v_min3 per MFMA into the lane's two running minima per column block (register s takes
// rows s and s + 2 of the lane's four: one parity class of the mixture, bit 2g + s of its word).  Two v_min3 per
// MFMA are exactly the vector-issue cycles an MFMA leaves free, so the step is otherwise bare: no mixed tiles, no
// stand-in tile, no pack.  The epilogue of a step's last LAG column blocks runs in the next step under its first
// MFMAs (no hazard wait at a step end); the first step of the next mixture completes the previous one that way and
// emits it -- 2 min(v) + p per register, the reduce, finalize, stores -- under its own MFMAs, then its candidates
// set the minima (no resets).  Tiles come through scoreI8Seg's LDS ring (LDS-DMA one segment ahead); each step reads
// the next tile's operands from LDS.
// ---------------------------------------------------------------------------
#ifndef GMM_I8_CLS_LAG
#define GMM_I8_CLS_LAG 3  // column blocks whose epilogue runs one step late
#endif
#ifndef GMM_I8_PRESEL_CPF
#define GMM_I8_PRESEL_CPF 1  // preselection: the rows' cluster offsets read one tile ahead with the operands
#endif
#ifndef GMM_I8_PRESEL_SEG
// preselection-batch-int: tiles per LDS segment, one workgroup barrier per segment (8: -3.9 % against 4; 16 +4.4 %, the
// LDS then allows two waves per SIMD; profiles/r06/s6).  A lagged masked epilogue (the score-only step's pipeline, lag
// 1 / 2 / 3) measured +6 / +17 / +17 % (profiles/r06/s7)
#define GMM_I8_PRESEL_SEG 8
#endif
#ifndef GMM_I8_PRESEL_WAVES
#define GMM_I8_PRESEL_WAVES 3  // preselection: waves per SIMD the register allocation must allow
#endif
#ifndef GMM_I8_CLS_EARLYB
#define GMM_I8_CLS_EARLYB 1  // score-only: every prologue load waited for before the loop (see scoreI8Cls)
#endif
#ifndef GMM_I8_CLS_DIAG
#define GMM_I8_CLS_DIAG 0  // timing diagnostics only (wrong results): 1 = no per-mixture emit (the last one aside)
#endif
// PRESEL (preselection-batch-int, NF 8): the row constants are biased by 2^31 (the accumulator u = v + 2^31 is
// compared unsigned) and every candidate is OR-ed with the sign-extended mask byte of its (frame, row cluster), so a
// density whose cluster the frame did not select becomes all ones and never wins; padding rows sit in an extra
// never-selected cluster.  Per tile the lane reads its 4 rows' table entries (the wave's [cluster][t] table of
// launchCompactSelection, copied to LDS by LDS-DMA at the start) and their LUT expansions to 8 mask bytes, one per
// column block; the tile's epilogues follow its MFMAs in the same step (no pending tail).  A frame that selected
// none of a mixture's densities keeps all ones: Core::Type<int>::max, as the reference.
template <int NF, int SEG, int W, bool PRESEL = false>
__global__ __launch_bounds__(64 * W, W == 4 ? (PRESEL ? GMM_I8_PRESEL_WAVES : (NF == 16 ? 2 : 4)) : 1) void scoreI8Cls(I8Args a, const uint32_t* __restrict__ mixTileOffArg,
                                                                                   float* __restrict__ scores,
                                                                                   const uint32_t* __restrict__ mixWordArg) {
    const auto mixTileOff = constTable(mixTileOffArg);
    const auto mixWord = constTable(mixWordArg);
    static_assert(NF == 4 || NF == 8 || (NF == 16 && !PRESEL), "NF");
    static_assert(!PRESEL || (NF == 8 && W == 4), "preselection: 128-frame waves (two 64-frame mask words)");
    constexpr int      LAG       = PRESEL ? 0 : GMM_I8_CLS_LAG;
    constexpr int      NPL       = NF / 4;
    constexpr uint32_t kSegA     = SEG * 1024u;
    constexpr uint32_t kSegP     = kSegA + SEG * 64u;
    constexpr uint32_t kSegBytes = kSegP + (PRESEL ? SEG * 64u : 0u);  // + the rows' cluster offsets (u32)
    constexpr int      kPieces   = SEG / W;          // 1 KiB operand pieces per wave per segment
    constexpr uint32_t kRowLanes = 4u * SEG / W;     // lanes loading 16 B of row constants per wave
    constexpr int      kIssued   = kPieces + 1 + (PRESEL ? 1 : 0);
    constexpr int      kNeutral  = PRESEL ? -1 : 0x3fffffff;  // above every row (padding rows: 0x30000000)
    static_assert(SEG % W == 0 && kRowLanes <= 64 && (PRESEL || (LAG >= 1 && LAG < NF)), "segment / lag");
    // + 64: the look-ahead read past the last tile of buffer 1 stays inside the array.  PRESEL: ring and the waves'
    // mask tables in the dynamic array, the 256-entry LUT static (its address folds into the reads)
    int8_t* lds;
    int8_t* lut = nullptr;
    if constexpr (PRESEL) {
        __shared__ uint64_t lutStatic[256];
        lds = i8DynLds;
        lut = reinterpret_cast<int8_t*>(lutStatic);
    }
    else {
        __shared__ __attribute__((aligned(16))) int8_t ldsStatic[2 * kSegBytes + 64];
        lds = ldsStatic;
    }

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g    = lane >> 4;
    uint32_t  chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;  // uniform over the workgroup, before any barrier
    const uint32_t frame0 = ft * (W * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];
    const uint32_t nSeg = (T1 - T0 + SEG - 1) / SEG;
    const int8_t*  gA   = static_cast<const int8_t*>(a.tileA);
    const int8_t*  gP   = static_cast<const int8_t*>(a.tileP);

    const auto issueSeg = [&](uint32_t s) {  // tile arrays are padded by kTilePad >= SEG tiles
        const uint32_t t0   = T0 + s * SEG;
        int8_t*        base = lds + (s & 1u) * kSegBytes;
#pragma unroll
        for (int i = 0; i < kPieces; ++i) {
            const uint32_t piece = static_cast<uint32_t>(wave * kPieces + i);
            __builtin_amdgcn_global_load_lds(gA + static_cast<size_t>(t0) * 1024u + piece * 1024u + lane * 16,
                                             base + piece * 1024u, 16, 0, 0);
        }
        if (lane < kRowLanes)
            __builtin_amdgcn_global_load_lds(gP + static_cast<size_t>(t0) * 64 + wave * (kRowLanes * 16) + lane * 16,
                                             base + kSegA + wave * (kRowLanes * 16), 16, 0, 0);
        if constexpr (PRESEL) {
            if (lane < kRowLanes)
                __builtin_amdgcn_global_load_lds(static_cast<const int8_t*>(a.tileClu) + static_cast<size_t>(t0) * 64 +
                                                         wave * (kRowLanes * 16) + lane * 16,
                                                 base + kSegP + wave * (kRowLanes * 16), 16, 0, 0);
        }
    };
    // PRESEL: this wave's mask table [cluster][16] (+ the never-selected cluster) after the ring, by LDS-DMA ahead
    // of the ring (the oldest vector-memory operations: the first segment's counted wait covers them)
    // In LDS a table entry is the u16 byte offset 8 e of the LUT entry (no scaling per read); in global memory the
    // per-call table holds e itself (one byte: what every chunk's workgroups re-read stays in L2), so each wave
    // loads its 4 KiB (256 clusters) once into registers and expands it
    const uint32_t words  = PRESEL ? a.nClusters * 16u : 0u;  // entries (cluster, t)
    const uint32_t tabOff = 2 * kSegBytes + 64u + static_cast<uint32_t>(wave) * (words + 16u) * 2u;
    constexpr int  kTabV  = PRESEL ? 4 : 1;  // 16-byte pieces of the table per lane (<= 256 clusters)
    i32x4          tabV[kTabV];
    if constexpr (PRESEL) {
        const i32x4* src = reinterpret_cast<const i32x4*>(a.selC + static_cast<size_t>(frame0 / 128u) * words);
#pragma unroll
        for (int i = 0; i < kTabV; ++i)
            if ((i * 64u + static_cast<uint32_t>(lane)) * 16u < words)
                tabV[i] = src[i * 64 + lane];
    }
    i32x4      B[NF];
    int        ssOut[NPL];
    const auto loadFrames = [&] {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            B[cb] = reinterpret_cast<const i32x4*>(a.frameQ + static_cast<size_t>(frame0 + cb * 16 + (lane & 15)) * 64)[g];
#pragma unroll
        for (int i = 0; i < NPL; ++i)
            ssOut[i] = a.frameSS[frame0 + 64 * i + lane];
    };
    if (nSeg > 0)
        issueSeg(0);
    if (nSeg > 1)
        issueSeg(1);
    uint32_t laneSel = 0;  // PRESEL: byte offset of (wave table, column t = lane & 15)
    if constexpr (PRESEL) {
        for (uint32_t n = threadIdx.x; n < 256u; n += 64u * W) {  // entry n (8 deselection bits) -> 8 mask bytes
            uint64_t v = 0;
#pragma unroll
            for (int cb = 0; cb < 8; ++cb)
                v |= ((n >> cb) & 1u) ? uint64_t(0xff) << (8 * cb) : uint64_t(0);
            reinterpret_cast<uint64_t*>(lut)[n] = v;
        }
        // expand: bytes b0 b1 b2 b3 of a word -> u16 pairs (8 b0, 8 b1), (8 b2, 8 b3): LUT byte offsets
#pragma unroll
        for (int i = 0; i < kTabV; ++i) {
            const uint32_t q = i * 64u + static_cast<uint32_t>(lane);
            if (q * 16u >= words)
                continue;
            uint32_t o[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t w = static_cast<uint32_t>(tabV[i][j]);
                o[2 * j]         = ((w & 0xffu) | ((w & 0xff00u) << 8)) << 3;
                o[2 * j + 1]     = (((w >> 16) & 0xffu) | ((w >> 8) & 0xff0000u)) << 3;
            }
            uint4* dst = reinterpret_cast<uint4*>(lds + tabOff + q * 32u);
            dst[0]     = uint4{o[0], o[1], o[2], o[3]};
            dst[1]     = uint4{o[4], o[5], o[6], o[7]};
        }
        if (lane < 8)  // the never-selected cluster: every frame deselected (LUT entry 255: byte offset 2040)
            reinterpret_cast<uint32_t*>(lds + tabOff + words * 2u)[lane] = 0x07f807f8u;
        laneSel = tabOff + (static_cast<uint32_t>(lane) & 15u) * 2u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LUT and entries before the first segment's barrier
    }

    loadFrames();
    // Every load before the ring (frame operands, PRESEL's table, the first two segments) complete, by a real
    // s_waitcnt vmcnt(0) the waitcnt pass sees: otherwise the frame operands and ssOut stay "pending" for it into the
    // loops (it treats the counter as out of order while LDS-DMA is in flight, so no vmcnt(N) clears them), and it puts
    // an s_waitcnt vmcnt(0) before every 2-tile iteration's first MFMA and in every emit -- each draining the DMA queue,
    // i.e. waiting for the segment issued one segment ahead.  Here the wait costs the second segment's landing once.
    if constexpr (PRESEL || GMM_I8_CLS_EARLYB)
        __builtin_amdgcn_s_waitcnt(0x0f70);

    // mixture m ends at tile tEnd; its word wCur and the next mixture's end tNext are loaded one mixture ahead
    // (scalar loads whose latency the mixture's steps cover)
    uint32_t m = m0, tEnd = mixTileOff[m0 + 1], tNext = m0 + 1 < m1 ? mixTileOff[m0 + 2] : T1, wCur = mixWord[m0];
    typedef int i32x2 __attribute__((ext_vector_type(2)));
    i32x2 best[NF];  // the lane's two running minima per column block (a register pair: 64-bit resets)
    i32x4 acc[NF];   // acc[NF - LAG ..]: the previous step's blocks whose epilogue is pending
    const uint64_t kNeutral2 = (static_cast<uint64_t>(kNeutral) << 32) | static_cast<uint32_t>(kNeutral);
    // one v_min3 per two candidates; the empty asm keeps each update one v_min3 (the compiler would reassociate
    // the chain into two-operand v_min), the min itself stays compiler-visible (hazard wait states)
    const auto epiMin = [&](int cb) {
        int b0 = min(best[cb][0], min(acc[cb][0], acc[cb][2]));
        int b1 = min(best[cb][1], min(acc[cb][1], acc[cb][3]));
        asm volatile("" : "+v"(b0));
        asm volatile("" : "+v"(b1));
        best[cb] = i32x2{b0, b1};
    };
    const auto epiSet = [&](int cb) {  // a mixture's first tile: the minima start from its candidates
        best[cb] = i32x2{min(acc[cb][0], acc[cb][2]), min(acc[cb][1], acc[cb][3])};
    };
    // PRESEL: candidate (block cb, row r) OR the sign-extended mask byte cb of the row (one v_or_b32_sdwa), the
    // biased keys compared unsigned
    typedef uint2 MaskW;  // a row's 8 mask bytes: x blocks 0-3, y blocks 4-7
    const auto cand = [&](int cb, int r, const MaskW (&T)[4]) -> uint32_t {
        const uint32_t h = cb >= 4 ? T[r].y : T[r].x;
        return static_cast<uint32_t>(acc[cb][r]) |
               static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(h >> (8 * (cb & 3)))));
    };
    const auto epiMask = [&](int cb, const MaskW (&T)[4], bool set) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            uint32_t b = min(cand(cb, s2, T), cand(cb, s2 + 2, T));
            if (!set)
                b = min(static_cast<uint32_t>(best[cb][s2]), b);
            asm volatile("" : "+v"(b));
            best[cb][s2] = static_cast<int>(b);
        }
    };
    // per-mixture emit: 2 min(v) + p per register (p = bit 2g + s of the word), the lane's two registers merged,
    // the reduce-scatter over the lane groups, finalize and store
    const auto emit = [&](uint32_t mm) {
        const uint32_t w = wCur;
        int            v[NF][1];
        if constexpr (PRESEL) {
            // biased u = v + 2^31, clamped at 2^31 + 2^29 (all ones: nothing selected); 2 u + p = 2 v + p modulo 2^32
            // (the bias shifts out), and a clamped register gives 2^30 + p, reported as none
            constexpr uint32_t kClamp = 0x80000000u + (1u << 29);
            if (((w ^ (w >> 1)) & 0x55u) == 0u) {  // both registers of every lane group share the parity (uniform)
                const uint32_t p = (w >> (2 * g)) & 1u;
#pragma unroll
                for (int cb = 0; cb < NF; ++cb) {
                    const uint32_t u = min(min(static_cast<uint32_t>(best[cb][0]), static_cast<uint32_t>(best[cb][1])), kClamp);
                    v[cb][0]         = static_cast<int>((u << 1) + p);
                }
            }
            else {
                const uint32_t p0 = (w >> (2 * g)) & 1u, p1 = (w >> (2 * g + 1)) & 1u;
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
                    v[cb][0] = min(static_cast<int>((min(static_cast<uint32_t>(best[cb][0]), kClamp) << 1) + p0),
                                   static_cast<int>((min(static_cast<uint32_t>(best[cb][1]), kClamp) << 1) + p1));
            }
            emitMixtureI8<NF, true, 1, (1 << 30)>(a, scores, nullptr, v, mm, frame0, lane, g, 0, ssOut);
            return;
        }
        if (((w ^ (w >> 1)) & 0x55u) == 0u) {  // both registers of every lane group share the parity (uniform)
            const int p = static_cast<int>((w >> (2 * g)) & 1u);
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                v[cb][0] = static_cast<int>((static_cast<uint32_t>(min(best[cb][0], best[cb][1])) << 1) + p);
        }
        else {
            const int p0 = static_cast<int>((w >> (2 * g)) & 1u), p1 = static_cast<int>((w >> (2 * g + 1)) & 1u);
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                v[cb][0] = min(static_cast<int>((static_cast<uint32_t>(best[cb][0]) << 1) + p0),
                               static_cast<int>((static_cast<uint32_t>(best[cb][1]) << 1) + p1));
        }
        emitMixtureI8<NF, false, 1>(a, scores, nullptr, v, mm, frame0, lane, g, 0, ssOut);
    };
    const auto emitNone = [&](uint32_t mm) {  // a mixture without densities: Core::Type<int>::max
        int none[NF][1];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            none[cb][0] = INT_MAX;
        emitMixtureI8<NF, true, 1>(a, scores, nullptr, none, mm, frame0, lane, g, 0, ssOut);
    };
    const auto advance = [&]() {  // m -> m + 1
        ++m;
        tEnd = tNext;
        if (m < m1) {
            wCur  = mixWord[m];
            tNext = m + 1 < m1 ? mixTileOff[m + 2] : T1;
        }
    };
    // mixture m ended at tile t: emit it (and the mixtures without tiles that end at t too)
    const auto finish = [&](uint32_t t) {
        if (!(GMM_I8_CLS_DIAG & 1) || m + 1 == m1)
            emit(m);
        advance();
        while (t == tEnd && m < m1) {
            emitNone(m);
            advance();
        }
    };
    // the step of one tile: MFMA of block cb beside the epilogue of block cb - LAG (of the previous step for cb <
    // LAG), fenced so the scheduler keeps that pairing.  FIRST: the first tile of a mixture (after boundary()): no
    // pending tail; its candidates set the minima of its first NF - LAG blocks (no reset of those)
    const auto step = [&](const i32x4& A, const i32x4& P, const i32x4& Cpf, const int8_t* cptr, uint32_t t,
                          auto firstC, auto prefetch) {
        constexpr bool kFirst = decltype(firstC)::value;
        (void)cptr;
        if constexpr (!PRESEL)
            prefetch();
        if constexpr (PRESEL) {
            // the tile's mask rows: the lane's table entries (LUT indices), then their 8 mask bytes; the rows'
            // cluster offsets prefetched with the operands (GMM_I8_PRESEL_CPF) or read here
            i32x4 C = Cpf;
            if constexpr (!GMM_I8_PRESEL_CPF)
                C = *reinterpret_cast<const i32x4*>(cptr);
            // The 64-bit LUT read at a loaded address makes the waitcnt pass drain the LDS-DMA queue (s_waitcnt
            // vmcnt(0)) at every step, since it cannot tell the read from the ring the DMA fills; by then the next
            // segment, issued a segment ahead, has landed.  Two 32-bit reads from split tables avoid the wait but
            // measured 11 % slower (profiles/r05/s9), a conflict-free 16-entry nibble LUT 3.5 % slower
            // (profiles/r06/s24), these reads one step ahead flat (profiles/r06/s22)
            prefetch();
            MaskW T[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t e = *reinterpret_cast<const uint16_t*>(lds + laneSel + static_cast<uint32_t>(C[r]));
                T[r]             = *reinterpret_cast<const MaskW*>(lut + e);
            }
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B[cb], P, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                epiMask(cb, T, kFirst);
            __builtin_amdgcn_sched_barrier(0);
            return;
        }
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            __builtin_amdgcn_sched_barrier(0);
            acc[cb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B[cb], P, 0, 0, 0);
            if (cb >= LAG) {
                if (kFirst)
                    epiSet(cb - LAG);
                else
                    epiMin(cb - LAG);
            }
            else if (!kFirst)
                epiMin(NF - LAG + cb);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 64, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    // mixture m ends at tile t and another with tiles follows: the pending tail completes m, which is emitted; the
    // tail's minima restart above every row (the next mixture's first step sets the others)
    const auto boundary = [&](uint32_t t) {
        if constexpr (!PRESEL) {
#pragma unroll
            for (int cb = NF - LAG; cb < NF; ++cb)
                epiMin(cb);
        }
        finish(t);
        if constexpr (!PRESEL) {
#pragma unroll
            for (int cb = NF - LAG; cb < NF; ++cb)
                asm volatile("v_mov_b64 %0, %1" : "=v"(best[cb]) : "s"(kNeutral2));
        }
    };
    const std::true_type  kFirstTile{};
    const std::false_type kInner{};
    // before the chunk's first tile: minima above every row, and a pending tail that changes nothing
#pragma unroll
    for (int cb = 0; cb < NF; ++cb)
        asm volatile("v_mov_b64 %0, %1" : "=v"(best[cb]) : "s"(kNeutral2));
#pragma unroll
    for (int cb = NF - LAG; cb < NF; ++cb)
        acc[cb] = i32x4{kNeutral, kNeutral, kNeutral, kNeutral};
    while (m < m1 && tEnd == T0) {  // mixtures without tiles at the start of the chunk
        emitNone(m);
        advance();
    }
    bool fresh = false;  // the next step is the first of a mixture (its minima not yet started)

    for (uint32_t s = 0; s < nSeg; ++s) {
        // this segment's pieces (issued one segment ago) have landed; the next segment's stay in flight
        if (s + 1 < nSeg)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kIssued) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const int8_t*  base   = lds + (s & 1u) * kSegBytes;
        const uint32_t segT0  = T0 + s * SEG;
        const uint32_t segEnd = min(segT0 + SEG, T1);
        // this lane's operand addresses of the current tile t; tile t + i is i KiB (A) and i * 64 B (P) further
        const int8_t* pa = base + lane * 16;
        const int8_t* pp = base + kSegA + g * 16;
        // PRESEL: the lane group's 4 row cluster offsets, as one aligned 16-byte read
        const auto rd = [&](int i, i32x4& A, i32x4& P, i32x4& C) {  // (past the segment: read, never used)
            A = *reinterpret_cast<const i32x4*>(pa + i * 1024);
            P = *reinterpret_cast<const i32x4*>(pp + i * 64);
            if constexpr (PRESEL && GMM_I8_PRESEL_CPF)
                C = *reinterpret_cast<const i32x4*>(pp + (kSegP - kSegA) + i * 64);
        };
        const auto cp = [&](int i) { return pp + (kSegP - kSegA) + i * 64; };  // the tile's cluster offsets
        i32x4    A0, P0, C0, A1, P1, C1;  // tile t, and the next one in flight
        uint32_t t = segT0;
        rd(0, A0, P0, C0);
        while (t < segEnd) {
            if (fresh) {  // the first tile of a mixture
                step(A0, P0, C0, cp(0), t, kFirstTile, [&] { rd(1, A1, P1, C1); });
                A0 = A1;
                P0 = P1;
                C0 = C1;
                pa += 1024;
                pp += 64;
                ++t;
                fresh = false;
            }
            const uint32_t mEnd = min(segEnd, tEnd);
            // two tiles per iteration on alternating registers (no copies of the operands in flight)
            for (; t + 2 <= mEnd; t += 2) {
                step(A0, P0, C0, cp(0), t, kInner, [&] { rd(1, A1, P1, C1); });
                step(A1, P1, C1, cp(1), t + 1, kInner, [&] { rd(2, A0, P0, C0); });
                pa += 2048;
                pp += 128;
            }
            if (t < mEnd) {
                step(A0, P0, C0, cp(0), t, kInner, [&] { rd(1, A1, P1, C1); });
                A0 = A1;
                P0 = P1;
                C0 = C1;
                pa += 1024;
                pp += 64;
                ++t;
            }
            if (t == tEnd && t < T1) {  // mixture m ends here and another with tiles follows
                boundary(t);
                fresh = true;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // every wave is done reading buffer (s & 1)
        if (s + 2 < nSeg)
            issueSeg(s + 2);
    }
    // the chunk's last mixture with tiles (its pending tail first), then trailing mixtures without tiles
    if (m < m1) {
#pragma unroll
        for (int cb = NF - LAG; cb < NF; ++cb)
            epiMin(cb);  // (PRESEL: LAG 0, none)
        emit(m);
        advance();
        while (m < m1) {
            emitNone(m);
            advance();
        }
    }
}

}  // namespace dev

using dev::prepareFramesI8;

hipError_t launchPrepareFramesI8(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesPad,
                                 uint32_t nFramesRead, uint32_t D, uint32_t C, uint32_t KS, const float* isv,
                                 int8_t* frameQ, int32_t* frameSS, hipStream_t stream) {
    const uint32_t n = C * nFramesRead;  // (covariance, frame) pairs, 8 per block
    hipLaunchKernelGGL(prepareFramesI8, dim3((n + 7) / 8), dim3(256), 0, stream, frames, nFrames, frameStride,
                       nFramesPad, nFramesRead, D, C, KS, isv, frameQ, frameSS);
    return hipGetLastError();
}

template <int NF, int KS, bool MULTI, int W = 4>
static void launchI8T(const I8Args& a, uint32_t grid, hipStream_t s) {
#if GMM_I8_LDS
    if constexpr (!MULTI) {
        if (a.presel && a.scoreOnly == 2) {  // preselection-batch-int on the slot layout (3 waves per SIMD: registers)
            if constexpr (KS == 1 && kI8PreselNF == 8) {
                constexpr int      kSeg = GMM_I8_PRESEL_SEG;
                constexpr uint32_t kRing = 2 * kSeg * (1024 + 64 + 64) + 64;
                const uint32_t     lds   = kRing + 4u * (a.nClusters * 16u + 16u) * 2u;
                constexpr int      kMax  = static_cast<int>(kRing + 4u * (256u * 16u + 16u) * 2u);
                (void)allowDynamicLds(reinterpret_cast<const void*>(&dev::scoreI8Cls<8, kSeg, 4, true>), kMax);
                hipLaunchKernelGGL((dev::scoreI8Cls<8, kSeg, 4, true>), dim3(grid), dim3(256), lds, s, a, a.mixTileOff,
                                   a.scores, a.mixOddMask);
            }
            return;
        }
        if (a.presel) {  // preselection-batch-int: NF 4, 4-tile segments (ring + 4 mask tables < 80 KiB)
            constexpr int      kSeg  = 4;
            constexpr uint32_t kRing = 2 * (kSeg * (KS * 1024 + 64 + 64)) + kI8DummyTileBytes(KS, true);
            // after the ring, per wave the table of the clusters and the never-selected entry
            const uint32_t     lds   = kRing + 4u * (a.nClusters + 1u) * 16u * kI8PreselEntryBytes;
            constexpr int      kMax  = static_cast<int>(kRing + 4u * 257u * 16u * kI8PreselEntryBytes);
            if constexpr (KS == 1) {
                if (a.scoreOnly) {  // the class layout (the default)
                    (void)allowDynamicLds(
                            reinterpret_cast<const void*>(&dev::scoreI8Seg<kI8PreselNF, 1, true, kSeg, true>), kMax);
                    hipLaunchKernelGGL((dev::scoreI8Seg<kI8PreselNF, 1, true, kSeg, true>), dim3(grid), dim3(256), lds,
                                       s, a, a.mixTileOff, a.scores, nullptr, a.mixOddMask);
                    return;
                }
            }
            (void)allowDynamicLds(reinterpret_cast<const void*>(&dev::scoreI8Seg<kI8PreselNF, KS, true, kSeg>), kMax);
            hipLaunchKernelGGL((dev::scoreI8Seg<kI8PreselNF, KS, true, kSeg>), dim3(grid), dim3(256), lds, s, a,
                               a.mixTileOff, a.scores, a.best, nullptr);
            return;
        }
        // 16-tile segments for one K step (34 KiB per workgroup, 4 per CU); 8 for two (also 34 KiB); one-wave
        // workgroups take half of that (more of them per CU)
        constexpr int kSeg = (KS == 1 ? dev::kSegTiles : 8) / (W == 1 ? 2 : 1);
        if constexpr (KS == 1) {
            if (a.scoreOnly == 2) {  // calls without best densities on the slot layout (kI8ClsNF blocks per wave)
                constexpr int NFC = (W == 4 && NF == kI8NF) ? kI8ClsNF : NF;
                hipLaunchKernelGGL((dev::scoreI8Cls<NFC, kSeg, W>), dim3(grid), dim3(64 * W), 0, s, a, a.mixTileOff,
                                   a.scores, a.mixOddMask);
                return;
            }
            if (a.scoreOnly) {  // the class layout
                hipLaunchKernelGGL((dev::scoreI8Seg<NF, 1, false, kSeg, true, W>), dim3(grid), dim3(64 * W), 0, s, a,
                                   a.mixTileOff, a.scores, nullptr, a.mixOddMask);
                return;
            }
        }
        hipLaunchKernelGGL((dev::scoreI8Seg<NF, KS, false, kSeg, false, W>), dim3(grid), dim3(64 * W), 0, s, a,
                           a.mixTileOff, a.scores, a.best, nullptr);
        return;
    }
#endif
    hipLaunchKernelGGL((dev::scoreI8<NF, KS, MULTI>), dim3(grid), dim3(256), 0, s, a);
}

hipError_t launchScoreI8(const I8Args& a, uint32_t kSteps, bool multiCov, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    if (a.presel && (multiCov || !GMM_I8_LDS || a.nClusters == 0 || a.nClusters > 256 || !a.selT || !a.tileClu ||
                     (kI8PreselNF == 8 && !a.selC)))
        return hipErrorInvalidValue;
    if (a.scoreOnly && (multiCov || kSteps != 1 || !GMM_I8_LDS || !a.mixOddMask))
        return hipErrorInvalidValue;
    if (a.smallTile && a.presel)
        return hipErrorInvalidValue;  // the preselection kernels keep their frame tile
    // small calls: 64-frame waves (I8Args::smallTile), one wave per workgroup for the smallest (2)
    if (kSteps == 1 && a.smallTile == 2 && !multiCov)
        launchI8T<4, 1, false, 1>(a, grid, stream);
    else if (kSteps == 2 && a.smallTile == 2 && !multiCov)
        launchI8T<4, 2, false, 1>(a, grid, stream);
    else if (kSteps == 1 && a.smallTile)
        multiCov ? launchI8T<4, 1, true>(a, grid, stream) : launchI8T<4, 1, false>(a, grid, stream);
    else if (kSteps == 2 && a.smallTile)
        multiCov ? launchI8T<4, 2, true>(a, grid, stream) : launchI8T<4, 2, false>(a, grid, stream);
    else if (kSteps == 1)
        multiCov ? launchI8T<kI8NF, 1, true>(a, grid, stream) : launchI8T<kI8NF, 1, false>(a, grid, stream);
    else if (kSteps == 2)
        multiCov ? launchI8T<kI8NF, 2, true>(a, grid, stream) : launchI8T<kI8NF, 2, false>(a, grid, stream);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace rasr_gmm
