// gmm_kernels_split.hip -- float scorers (diagonal-maximum, batch-float) on the f16 matrix cores.
//
// gfx950 has no reduced-precision f32 matrix format (no xf32/TF32), and the f32 MFMA
// (v_mfma_f32_16x16x4_f32, 32 cycles per 16x16x4) runs at 1/16 of the f16 rate.  The float
// scorers therefore split every f32 operand into two f16 pieces, v = hi + lo with
// |v - hi - lo| <= 2^-22 |v|, and contract
//     x'.m'  ~  xh.mh + xl.mh + xh.ml          (the dropped xl.ml term is <= 2^-22 |x'||m'|)
// with v_mfma_f32_16x16x32_f16 (16 cycles per 16x16x32, f32 accumulation; f16 x f16 products
// are exact in f32).  Per 16 densities x 16 frames at D = 39: K = 3*39 + 4 = 121 -> 4 MFMAs =
// 64 cycles, against 10 f32 MFMAs = 320 cycles.  The result has the accuracy class of the f32
// kernel (whose (score, tile) key already truncates the low tileBits mantissa bits):
// tests/test_gpu_parity.py checks both against the f64-accumulating oracle at 1e-4 relative.
//
// Exponent range (f16 covers 2^-24 .. 65504):
//   * model side, per dimension d: m''_d = -2 m'_d / 2^a_d with max|m''_d| in [2^7, 2^8)
//     (host, gmm_prepare.cc); frame side x''_d = x'_d * 2^a_d, so x''.m'' = -2 x'.m' exactly;
//   * per frame: e = the power of two that brings max|x''| below 2^15 (0 for ordinary frames);
//     the whole column of that frame is computed scaled by 2^-e (operands, the ||x'||^2
//     initial accumulator, the constant limbs), which is exact, leaves the per-frame minimum
//     and argmin unchanged, and is undone on the final score;
//   * the row constant c (||m'||^2 + weight + norm + K0, f64 on the host) is carried by four f16
//     limbs at 2^b0, 2^(b0-11), 2^(b0-22), 2^(b0-33) against frame-side multipliers
//     2^(b_s - e): 44 bits of the constant.
// Padding rows (tail of a mixture's last tile) repeat row 0 of their tile: an exact tie with a
// lower density index, so they never win and no +inf enters the (value | tile) keys (+inf with
// tile bits would be a signalling NaN, which v_min_f32 turns into a quiet NaN result).
//
// K layout (host and frame preparation agree): [0,D) mh.xh, [D,2D) mh.xl, [2D,3D) ml.xh,
// [3D,3D+4) limbs, rest zero.  Fragment order of v_mfma_f32_16x16x32_f16: lane l holds
// A[row l&15][k = 8(l>>4) + j] and B[k = 8(l>>4) + j][col l&15], j = 0..7; C/D hold
// col l&15, rows 4(l>>4) + r.
//
// Work decomposition and epilogue are the f32 kernel's (gmm_kernels_f32.hip): a workgroup is
// 4 waves x NF column blocks of 16 frames walking a chunk of mixtures on one XCD; the running
// minimum is a float key whose low tileBits mantissa bits hold the tile number.
#include "gmm_device.hh"

#ifndef GMM_SPLIT_PAIR
#define GMM_SPLIT_PAIR 1  // two tiles per loop step, v_min3 over both
#endif
#ifndef GMM_SPLIT_EMIT_OLD
#define GMM_SPLIT_EMIT_OLD 0  // A/B only: per-candidate lexMin with validity branches at mixture end
#endif
#ifndef GMM_SPLIT_MIN_WAVES
#define GMM_SPLIT_MIN_WAVES 1
#endif

namespace rasr_gmm {
namespace dev {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint16_t h16bits(float v) {
    const _Float16 h = static_cast<_Float16>(v);
    return __builtin_bit_cast(uint16_t, h);
}

// ---------------------------------------------------------------------------
// frame preparation: one thread per frame
//   frameH  [nFramesPad/16][KS16][64][8] f16 (B fragments), frameXX = ||x'||^2 * 2^-e,
//   frameExp = e.  Rows >= nFrames are zero.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prepareFramesSplit(const float* __restrict__ frames, uint32_t nFrames,
                                                           uint32_t frameStride, uint32_t nFramesRead, uint32_t D,
                                                           uint32_t KS16, const float* __restrict__ isv,
                                                           const float* __restrict__ dimScale,
                                                           const int32_t* __restrict__ limbExp,
                                                           u32x4* __restrict__ frameH, float* __restrict__ frameXX,
                                                           int32_t* __restrict__ frameExp) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nFramesRead)
        return;
    const bool   valid = f < nFrames;
    const float* x     = frames + static_cast<size_t>(f) * frameStride;
    float        xx = 0.0f, ymax = 0.0f;
    bool         finite = true;
    if (valid)
        for (uint32_t k = 0; k < D; ++k) {
            const float v = __fmul_rn(x[k], isv[k]);  // x' exactly as the f32 kernel forms it
            xx            = __fadd_rn(xx, __fmul_rn(v, v));
            const float y = fabsf(v * dimScale[k]);
            finite        = finite && y <= 3.40282347e+38f;
            ymax          = fmaxf(ymax, y);
        }
    int e = 0;
    if (finite && ymax > 32768.0f) {
        int ex;
        frexpf(ymax, &ex);  // ymax in [2^(ex-1), 2^ex)
        e = ex - 15;
    }
    frameXX[f]  = ldexpf(xx, -e);
    frameExp[f] = e;
    const uint32_t fb = f >> 4, col = f & 15;
    for (uint32_t q = 0; q < KS16 * 4; ++q) {  // groups of 8 consecutive k
        uint32_t w[4] = {0, 0, 0, 0};
        if (valid)
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t k = 8 * q + j;
                uint16_t       h = 0;
                if (k < 3 * D) {
                    const uint32_t d  = k < D ? k : (k < 2 * D ? k - D : k - 2 * D);
                    const float    y  = ldexpf(__fmul_rn(x[d], isv[d]) * dimScale[d], -e);
                    const uint16_t hi = h16bits(y);
                    h = (k >= D && k < 2 * D) ? h16bits(y - static_cast<float>(__builtin_bit_cast(_Float16, hi))) : hi;
                }
                else if (k < 3 * D + kSplitLimbs) {
                    const int be = limbExp[k - 3 * D] - e;
                    h            = be < -24 ? 0 : h16bits(ldexpf(1.0f, be));
                }
                w[j >> 1] |= static_cast<uint32_t>(h) << (16 * (j & 1));
            }
        // step q>>2, lane group q&3
        frameH[(static_cast<size_t>(fb) * KS16 + (q >> 2)) * 64 + 16 * (q & 3) + col] = u32x4{w[0], w[1], w[2], w[3]};
    }
}

// ---------------------------------------------------------------------------
// end of a mixture: the (value | tile) keys of the 4 row slots -> (score, density) per frame,
// reduced across the four 16-lane groups by permlane swaps; lane l stores frame frame0 + 64 i + l
// ---------------------------------------------------------------------------
template <int NF>
__device__ __forceinline__ void emitMixtureSplit(const SplitArgs& a, float* __restrict__ scores,
                                                 uint32_t* __restrict__ bestOut, const float (&best)[NF][4],
                                                 uint32_t m, uint32_t frame0, int lane, int g, uint32_t tmask,
                                                 const int (&eOut)[NF / 4]) {
    constexpr int NPL = NF / 4;
    float         v[NF];   // key (value | tile) of the lane's best row slot
    uint32_t      vi[NF];  // its density in the mixture: tile * 16 + 4 g + r
#if GMM_SPLIT_EMIT_OLD
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        v[cb]  = 3.40282347e+38f;
        vi[cb] = 0xffffffffu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t bits = __float_as_uint(best[cb][r]);
            if (!(__uint_as_float(bits & ~tmask) < 1e37f))  // no finite candidate in this row slot
                continue;
            lexMin(v[cb], vi[cb], best[cb][r], (bits & tmask) * 16u + 4u * g + r);
        }
    }
#else
    // branch-free: within a lane the keys order by (value, tile), so the minimum key and the first
    // row slot holding it give the lexicographic (value, density) minimum; an empty slot keeps
    // FLT_MAX, which loses to every finite key and is caught after the lane reduction
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        const float k0 = best[cb][0], k1 = best[cb][1], k2 = best[cb][2], k3 = best[cb][3];
        const float mn = fminf(fminf(k0, k1), fminf(k2, k3));
        uint32_t    r  = k2 == mn ? 2u : 3u;
        r              = k1 == mn ? 1u : r;
        r              = k0 == mn ? 0u : r;
        v[cb]          = mn;
        vi[cb]         = ((__float_as_uint(mn) & tmask) << 4) | (4u * g + r);
    }
#endif
    float    w[NF / 2];
    uint32_t wi[NF / 2];
#pragma unroll
    for (int p = 0; p < NF / 2; ++p) {
        const int c = (p & 1) | ((p >> 1) << 2);
        swapLexMin32(v[c], vi[c], v[c ^ 2], vi[c ^ 2], w[p], wi[p]);
    }
    const uint32_t mo = m - a.mixBase;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        float    kv;
        uint32_t ki;
        swapLexMin16(w[2 * i], wi[2 * i], w[2 * i + 1], wi[2 * i + 1], kv, ki);
        const uint32_t f = frame0 + 64 * i + lane;
        if (f >= a.nFrames)
            continue;
        kv = __uint_as_float(__float_as_uint(kv) & ~tmask);
        if (!(kv < 1e37f))  // no finite candidate at all (empty mixture, or non-finite frame)
            ki = 0xffffffffu;
        float score;
        if (ki == 0xffffffffu) {  // no density: bestScore stays Core::Type<Score>::max
            score = a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f;
        }
        else {
            const float scaled = ldexpf(kv, eOut[i]);
            const float total  = a.offsetK0 != 0.0f ? __fsub_rn(scaled, a.offsetK0) : scaled;
            score              = a.flavor == 2 ? 0.5f * total : (total < 3.40282347e+38f ? 0.5f * total : total);
        }
        if (a.outScale != 1.0f)
            score = __fmul_rn(a.outScale, score);
        const size_t o = static_cast<size_t>(mo) * a.scoreStride + f;
        scores[o]      = score;
        if (bestOut)
            bestOut[o] = ki;
    }
}

// ---------------------------------------------------------------------------
// scorer
// ---------------------------------------------------------------------------
template <int NF, int KS>
__global__ __launch_bounds__(256, GMM_SPLIT_MIN_WAVES) void scoreSplit(SplitArgs a) {
    static_assert(NF == 4 || NF == 8, "NF");
    const int     lane = threadIdx.x & 63;
    const int     wave = threadIdx.x >> 6;
    const int     g    = lane >> 4;
    uint32_t      chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * (4u * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t fb0    = frame0 / 16u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];

    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NF][KS];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[cb][s] = fh[(static_cast<size_t>(fb0 + cb) * KS + s) * 64 + lane];
    f32x4 XX[NF];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        const float xx = a.frameXX[frame0 + cb * 16 + (lane & 15)];
        XX[cb]         = f32x4{xx, xx, xx, xx};
    }
    int eOut[NF / 4];  // frame exponents of the frames this lane stores (no vector load inside the loop)
#pragma unroll
    for (int i = 0; i < NF / 4; ++i)
        eOut[i] = a.frameExp[frame0 + 64 * i + lane];

    const f16x8* th = static_cast<const f16x8*>(a.tileH);
    uint32_t     t  = a.mixTileOff[m0];
    f16x8        A0[KS], A1[KS];
    const auto   loadTile = [&](uint32_t tt, f16x8(&A)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = th[(static_cast<size_t>(tt) * KS + s) * 64 + lane];
    };
    loadTile(t, A0);
    loadTile(t + 1, A1);
    const auto chain = [&](const f16x8(&A)[KS], f32x4(&acc)[NF]) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            acc[cb] = XX[cb];
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s], B[cb][s], acc[cb], 0, 0, 0);
    };
    const uint32_t tmask = (1u << a.tileBits) - 1u;
    // the value mask lives in a VGPR so that (bits & mask) | tile is ONE v_and_or_b32 (gfx950 VOP3 reads
    // at most one SGPR; mask and tile number both in SGPRs would split it into v_and + v_or)
    uint32_t vmask = ~tmask;
    asm volatile("" : "+v"(vmask));
    const auto key = [&](float v, uint32_t tl) { return __uint_as_float((__float_as_uint(v) & vmask) | tl); };

    for (uint32_t m = m0; m < m1; ++m) {
        const uint32_t tBeg = t, tEnd = a.mixTileOff[m + 1];
        float          best[NF][4];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                best[cb][r] = 3.40282347e+38f;

        for (; GMM_SPLIT_PAIR && t + 1 < tEnd; t += 2) {
            f32x4 accA[NF], accB[NF];
            chain(A0, accA);
            loadTile(t + 2, A0);
            chain(A1, accB);
            loadTile(t + 3, A1);
            const uint32_t tl = t - tBeg;
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    best[cb][r] = fminf(best[cb][r], fminf(key(accA[cb][r], tl), key(accB[cb][r], tl + 1)));
        }
        for (; t < tEnd; ++t) {
            f32x4 acc[NF];
            chain(A0, acc);
            const uint32_t tl = t - tBeg;
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    best[cb][r] = fminf(best[cb][r], key(acc[cb][r], tl));
#pragma unroll
            for (int s = 0; s < KS; ++s)
                A0[s] = A1[s];
            loadTile(t + 2, A1);
        }

        emitMixtureSplit<NF>(a, a.scores, a.best, best, m, frame0, lane, g, tmask, eOut);
    }
}

// ---------------------------------------------------------------------------
// scorer, tiles staged through LDS (the i8 kernel's segment ring, gmm_kernels_i8.hip): the four
// waves of a workgroup walk the same tiles, so each 8-tile segment (8 x KS KiB) is brought into
// LDS once by global_load_lds_dwordx4 (each wave issues a quarter of it) one segment ahead, and
// every wave reads its A fragments with ds_read_b128; one global request per tile and workgroup
// instead of one per wave, and eight tiles of latency hiding instead of two
// ---------------------------------------------------------------------------
constexpr int kSplitSegTiles = 8;

template <int NF, int KS>
__global__ __launch_bounds__(256, GMM_SPLIT_MIN_WAVES) void scoreSplitSeg(SplitArgs a,
                                                                         const uint32_t* __restrict__ mixTileOff,
                                                                         float* __restrict__ scores,
                                                                         uint32_t* __restrict__ bestOut) {
    static_assert(NF == 4 || NF == 8, "NF");
    constexpr uint32_t kTileA    = KS * 1024;  // operand bytes per tile
    constexpr uint32_t kSegBytes = kSplitSegTiles * kTileA;
    constexpr int      kPieces   = kSplitSegTiles * KS / 4;  // 1 KiB pieces per wave per segment
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kSegBytes];

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g    = lane >> 4;
    uint32_t  chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;  // uniform over the workgroup, before any barrier
    const uint32_t frame0 = ft * (4u * NF * 16u) + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t fb0    = frame0 / 16u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];
    const uint32_t nSeg = (T1 - T0 + kSplitSegTiles - 1) / kSplitSegTiles;
    const uint8_t* gA   = static_cast<const uint8_t*>(a.tileH);

    // segment s -> buffer (s & 1); the tile array is padded by kTilePad >= kSplitSegTiles tiles
    const auto issueSeg = [&](uint32_t s) {
        const uint32_t t0   = T0 + s * kSplitSegTiles;
        uint8_t*       base = lds + (s & 1u) * kSegBytes;
#pragma unroll
        for (int i = 0; i < kPieces; ++i) {
            const uint32_t piece = static_cast<uint32_t>(wave * kPieces + i);
            __builtin_amdgcn_global_load_lds(gA + static_cast<size_t>(t0) * kTileA + piece * 1024u + lane * 16,
                                             base + piece * 1024u, 16, 0, 0);
        }
    };
    if (nSeg > 0)
        issueSeg(0);
    if (nSeg > 1)
        issueSeg(1);

    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NF][KS];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[cb][s] = fh[(static_cast<size_t>(fb0 + cb) * KS + s) * 64 + lane];
    f32x4 XX[NF];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
        const float xx = a.frameXX[frame0 + cb * 16 + (lane & 15)];
        XX[cb]         = f32x4{xx, xx, xx, xx};
    }
    int eOut[NF / 4];  // frame exponents of the frames this lane stores (no vector load inside the loop)
#pragma unroll
    for (int i = 0; i < NF / 4; ++i)
        eOut[i] = a.frameExp[frame0 + 64 * i + lane];
    const uint32_t tmask = (1u << a.tileBits) - 1u;
    // the value mask lives in a VGPR so that (bits & mask) | tile is ONE v_and_or_b32 (gfx950 VOP3 reads
    // at most one SGPR; mask and tile number both in SGPRs would split it into v_and + v_or)
    uint32_t vmask = ~tmask;
    asm volatile("" : "+v"(vmask));
    const auto key = [&](float v, uint32_t tl) { return __uint_as_float((__float_as_uint(v) & vmask) | tl); };

    float      best[NF][4];
    const auto resetBest = [&]() {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                best[cb][r] = 3.40282347e+38f;
    };
    resetBest();
    uint32_t m = m0, tBeg = T0, tEnd = mixTileOff[m0 + 1];
    while (m < m1 && tEnd == T0) {  // mixtures without tiles at the start of the chunk
        emitMixtureSplit<NF>(a, scores, bestOut, best, m, frame0, lane, g, tmask, eOut);
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T1;
    }

    for (uint32_t s = 0; s < nSeg; ++s) {
        // this segment's pieces (issued one segment ago) have landed; the next segment's stay in flight
        if (s + 1 < nSeg)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPieces) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* base   = lds + (s & 1u) * kSegBytes;
        const uint32_t segT0  = T0 + s * kSplitSegTiles;
        const uint32_t segEnd = min(segT0 + kSplitSegTiles, T1);
        uint32_t       t      = segT0;
        while (t < segEnd) {
            const uint32_t lt = t - segT0;
            const uint32_t tl = t - tBeg;
            if (GMM_SPLIT_PAIR && t + 1 < segEnd && t + 1 < tEnd) {
                f16x8 A0[KS], A1[KS];
#pragma unroll
                for (int k = 0; k < KS; ++k) {
                    A0[k] = *reinterpret_cast<const f16x8*>(base + lt * kTileA + k * 1024 + lane * 16);
                    A1[k] = *reinterpret_cast<const f16x8*>(base + (lt + 1) * kTileA + k * 1024 + lane * 16);
                }
                f32x4 accA[NF], accB[NF];
#pragma unroll
                for (int cb = 0; cb < NF; ++cb) {
                    accA[cb] = XX[cb];
                    accB[cb] = XX[cb];
                }
#pragma unroll
                for (int k = 0; k < KS; ++k)
#pragma unroll
                    for (int cb = 0; cb < NF; ++cb) {
                        accA[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0[k], B[cb][k], accA[cb], 0, 0, 0);
                        accB[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A1[k], B[cb][k], accB[cb], 0, 0, 0);
                    }
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        best[cb][r] = fminf(best[cb][r], fminf(key(accA[cb][r], tl), key(accB[cb][r], tl + 1)));
                t += 2;
            }
            else {
                f16x8 A0[KS];
#pragma unroll
                for (int k = 0; k < KS; ++k)
                    A0[k] = *reinterpret_cast<const f16x8*>(base + lt * kTileA + k * 1024 + lane * 16);
                f32x4 acc[NF];
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
                    acc[cb] = XX[cb];
#pragma unroll
                for (int k = 0; k < KS; ++k)
#pragma unroll
                    for (int cb = 0; cb < NF; ++cb)
                        acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A0[k], B[cb][k], acc[cb], 0, 0, 0);
#pragma unroll
                for (int cb = 0; cb < NF; ++cb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        best[cb][r] = fminf(best[cb][r], key(acc[cb][r], tl));
                t += 1;
            }
            // mixture(s) ending here (further ones without tiles end at the same point)
            while (t == tEnd && m < m1) {
                emitMixtureSplit<NF>(a, scores, bestOut, best, m, frame0, lane, g, tmask, eOut);
                resetBest();
                ++m;
                tBeg = tEnd;
                tEnd = m < m1 ? mixTileOff[m + 1] : T1;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // every wave is done reading buffer (s & 1)
        if (s + 2 < nSeg)
            issueSeg(s + 2);
    }
}

}  // namespace dev

hipError_t launchPrepareFramesSplit(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesRead,
                                    uint32_t D, uint32_t KS16, const float* isv, const float* dimScale,
                                    const int32_t* limbExp, void* frameH, float* frameXX, int32_t* frameExp,
                                    hipStream_t stream) {
    hipLaunchKernelGGL(dev::prepareFramesSplit, dim3((nFramesRead + 255) / 256), dim3(256), 0, stream, frames, nFrames,
                       frameStride, nFramesRead, D, KS16, isv, dimScale, limbExp,
                       static_cast<dev::u32x4*>(frameH), frameXX, frameExp);
    return hipGetLastError();
}

#ifndef GMM_SPLIT_LDS
#define GMM_SPLIT_LDS 0  // tiles staged through LDS (scoreSplitSeg): measured slower, off
#endif

template <int KS>
static void launchSplitK(const SplitArgs& a, uint32_t grid, hipStream_t s) {
#if GMM_SPLIT_LDS
    hipLaunchKernelGGL((dev::scoreSplitSeg<kSplitNF, KS>), dim3(grid), dim3(256), 0, s, a, a.mixTileOff, a.scores,
                       a.best);
#else
    hipLaunchKernelGGL((dev::scoreSplit<kSplitNF, KS>), dim3(grid), dim3(256), 0, s, a);
#endif
}

hipError_t launchScoreSplit(const SplitArgs& a, uint32_t kSteps16, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    switch (kSteps16) {
        case 1: launchSplitK<1>(a, grid, stream); break;
        case 2: launchSplitK<2>(a, grid, stream); break;
        case 3: launchSplitK<3>(a, grid, stream); break;
        case 4: launchSplitK<4>(a, grid, stream); break;
        case 5: launchSplitK<5>(a, grid, stream); break;
        case 6: launchSplitK<6>(a, grid, stream); break;
        case 7: launchSplitK<7>(a, grid, stream); break;
        case 8: launchSplitK<8>(a, grid, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rasr_gmm
