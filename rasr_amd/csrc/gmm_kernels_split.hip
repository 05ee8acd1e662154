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
// [3D,3D+4) row-constant limbs, [3D+4,3D+7) limbs of the frame's ||x'||^2 2^-e (against 2^15,
// 2^4, 2^-7 on the model side), rest zero.  Fragment order of v_mfma_f32_16x16x32_f16: lane l holds
// A[row l&15][k = 8(l>>4) + j] and B[k = 8(l>>4) + j][col l&15], j = 0..7; C/D hold
// col l&15, rows 4(l>>4) + r.
//
// Work decomposition and epilogue follow the f32 kernel's (gmm_kernels_f32.hip): a workgroup's waves
// hold NF column blocks of 16 frames each and walk a chunk of mixtures on one XCD; the running
// minimum is a float key whose low tileBits mantissa bits hold the tile number.
#include "gmm_device.hh"

#include <type_traits>
#include <utility>

#ifndef GMM_SPLIT_MIN_WAVES
#define GMM_SPLIT_MIN_WAVES 1
#endif
#ifndef GMM_SPLIT_IL
#define GMM_SPLIT_IL 24  // MFMAs of a pipeline step interleaved with kIlV VALU each (sched_group_barrier)
#endif
#ifndef GMM_SPLIT_PRESEL_NF
#define GMM_SPLIT_PRESEL_NF 8  // preselection-batch-float: column blocks per wave (8: -6.7 % at D = 39, -9.6 % at 45, profiles/r04/s21)
#endif
// preselection-batch-float's column blocks per wave at K steps KS (8 spills beyond 5 K steps)
constexpr int splitPreselNF(int ks) { return GMM_SPLIT_PRESEL_NF == 8 && ks <= 5 ? 8 : 4; }
#ifndef GMM_SPLIT_PF
#define GMM_SPLIT_PF 2  // tile pairs in flight per wave (scoreSplit without preselection; 3: +2.6 % at D = 39, profiles/r04/s18)
#endif
#ifndef GMM_SPLIT_DIAG_HOT
#define GMM_SPLIT_DIAG_HOT 0  // diagnostic (wrong results): every tile load reads the chunk's first two tiles (L1-hot)
#endif
#ifndef GMM_SPLIT_DIAG_NOEMIT
#define GMM_SPLIT_DIAG_NOEMIT 0
#endif
#ifndef GMM_SPLIT_SUM_NF
#define GMM_SPLIT_SUM_NF 4  // diagonal-sum: column blocks of 16 frames per wave (4 or 8)
#endif
#ifndef GMM_SPLIT_TAG_EMIT
#define GMM_SPLIT_TAG_EMIT 0  // 1: a tile's keys carry (tile << 2) only; the slot r is OR-ed in at the mixture's end
#endif
#ifndef GMM_SPLIT_EMIT_FLAT
#define GMM_SPLIT_EMIT_FLAT 1  // the emit finalize without the exec-mask branch (A/B at 128 frames per wave: -0.25..-0.5 %)
#endif

namespace rasr_gmm {
namespace dev {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int... I, class F>
__device__ __forceinline__ void staticForImpl(std::integer_sequence<int, I...>, F&& f) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void staticFor(F&& f) {  // f(integral_constant<int, i>) for i = 0 .. N-1, in order
    staticForImpl(std::make_integer_sequence<int, N>{}, f);
}

__device__ __forceinline__ uint32_t umin3(uint32_t x, uint32_t y, uint32_t z) {
    return min(min(x, y), z);  // v_min3_u32
}

__device__ __forceinline__ uint16_t h16bits(float v) {
    const _Float16 h = static_cast<_Float16>(v);
    return __builtin_bit_cast(uint16_t, h);
}

// ---------------------------------------------------------------------------
// frame preparation: 32 threads per frame, 8 frames per 256-thread block
//   frameH  [nFramesPad/16][KS16][64][8] f16 (B fragments), frameXX = ||x'||^2 * 2^-e,
//   frameExp = e.  Rows >= nFrames are zero.
// The frame's x' go to LDS once (lane t of the frame's 32 takes d = t, t + 32, ...), the exponent from a
// shuffle max, ||x'||^2 in the reference's sequential order by the frame's first thread, then every thread
// builds its 8-value groups of K.  (One thread per frame walking K serially took 22 us for a 1-frame call,
// most of a small host call's device time: profiles/r04/s14.)
// ---------------------------------------------------------------------------
template <int ROWS>
__global__ __launch_bounds__(256) void prepareFramesSplit(const float* __restrict__ frames, uint32_t nFrames,
                                                           uint32_t frameStride, uint32_t nFramesRead, uint32_t D,
                                                           uint32_t KS16, const float* __restrict__ isv,
                                                           const float* __restrict__ centre,
                                                           const float* __restrict__ dimScale,
                                                           const int32_t* __restrict__ limbExp,
                                                           u32x4* __restrict__ frameH, float* __restrict__ frameXX,
                                                           int32_t* __restrict__ frameExp) {
    __shared__ float xs[8][128];  // x' of the block's frames (D <= 126)
    __shared__ float shXX[8];
    __shared__ int   shE[8];
    const uint32_t   fl = threadIdx.x >> 5, t = threadIdx.x & 31u;
    const uint32_t   f       = blockIdx.x * 8u + fl;
    const bool       inRange = f < nFramesRead, valid = f < nFrames;
    const float*     x       = frames + static_cast<size_t>(f) * frameStride;
    float            ymax    = 0.0f;
    int              finite  = 1;
    if (valid)
        for (uint32_t k = t; k < D; k += 32u) {
            const float v = __fmul_rn(__fsub_rn(x[k], centre[k]), isv[k]);  // x' as the f32 kernel forms it
            xs[fl][k]     = v;
            const float y = fabsf(v * dimScale[k]);
            finite        = finite && y <= 3.40282347e+38f;
            ymax          = fmaxf(ymax, y);
        }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        ymax   = fmaxf(ymax, __shfl_xor(ymax, o, 32));
        finite = finite & __shfl_xor(finite, o, 32);
    }
    __syncthreads();
    if (t == 0 && inRange) {
        float xx = 0.0f;
        if (valid)
            for (uint32_t k = 0; k < D; ++k)
                xx = __fadd_rn(xx, __fmul_rn(xs[fl][k], xs[fl][k]));
        int e = 0;
        if (finite && ymax > 32768.0f) {
            int ex;
            frexpf(ymax, &ex);  // ymax in [2^(ex-1), 2^ex)
            e = ex - 15;
        }
        if (finite && xx < 3.40282347e+38f && ldexpf(xx, -e) >= 1073741824.0f) {  // ||x'||^2 2^-e < 2^30 (its top limb)
            int ex;
            frexpf(xx, &ex);
            e = ex - 30;
        }
        const float xxs = ldexpf(xx, -e);
        frameXX[f]      = xxs;
        frameExp[f]     = e;
        shXX[fl]        = xxs;
        shE[fl]         = e;
    }
    __syncthreads();
    if (!inRange)
        return;
    const int   e   = shE[fl];
    const float xxs = shXX[fl];
    // ||x'||^2 2^-e as three f16 limbs against 2^15, 2^4, 2^-7 on the model side
    uint16_t xxl[kSplitXXLimbs];
    {
        float rem = xxs;
#pragma unroll
        for (uint32_t s = 0; s < kSplitXXLimbs; ++s) {
            xxl[s]         = h16bits(ldexpf(rem, -kSplitXXExp[s]));
            const float lv = ldexpf(static_cast<float>(__builtin_bit_cast(_Float16, xxl[s])), kSplitXXExp[s]);
            rem            = __fsub_rn(rem, lv);
        }
    }
    // B fragments: 16 rows: frame block f/16, lane 16*((k>>3)&3) + f%16, step k>>5;
    //              32 rows: frame block f/32, lane 32*((k>>3)&1) + f%32, step k>>4
    const uint32_t fb = f / ROWS, col = f % ROWS;
    for (uint32_t q = t; q < KS16 * (ROWS == 32 ? 2 : 4); q += 32u) {  // groups of 8 consecutive k
        uint32_t w[4] = {0, 0, 0, 0};
        if (valid)
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t k = 8 * q + j;
                uint16_t       h = 0;
                if (k < 3 * D) {
                    const uint32_t d  = k < D ? k : (k < 2 * D ? k - D : k - 2 * D);
                    const float    y  = ldexpf(xs[fl][d] * dimScale[d], -e);
                    const uint16_t hi = h16bits(y);
                    h = (k >= D && k < 2 * D) ? h16bits(y - static_cast<float>(__builtin_bit_cast(_Float16, hi))) : hi;
                }
                else if (k < 3 * D + kSplitLimbs) {
                    const int be = limbExp[k - 3 * D] - e;
                    h            = be < -24 ? 0 : h16bits(ldexpf(1.0f, be));
                }
                else if (k < 3 * D + kSplitLimbs + kSplitXXLimbs) {
                    const uint32_t s = k - 3 * D - kSplitLimbs;
                    h                = s == 0 ? xxl[0] : (s == 1 ? xxl[1] : xxl[2]);
                }
                w[j >> 1] |= static_cast<uint32_t>(h) << (16 * (j & 1));
            }
        const uint32_t step = ROWS == 32 ? q >> 1 : q >> 2;
        const uint32_t ln   = ROWS == 32 ? 32 * (q & 1) + col : 16 * (q & 3) + col;
        frameH[(static_cast<size_t>(fb) * KS16 + step) * 64 + ln] = u32x4{w[0], w[1], w[2], w[3]};
    }
}

// ---------------------------------------------------------------------------
// frame preparation for several covariances (the covariance-free layout, gmm_prepare.cc): y = x - c in f32,
// Y = y^2 2^a_d and z = y 2^b_d (dimScale [0, D) and [D, 2D)), the frame exponent e keeping max(|Y|, |z|) 2^-e
// below 2^15, K = [Yh, Yl, Yh][zh, zl, zh][2^(b_s - e) limbs].  32 threads per frame, 8 frames per block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prepareFramesSplitCov(const float* __restrict__ frames, uint32_t nFrames,
                                                              uint32_t frameStride, uint32_t nFramesRead, uint32_t D,
                                                              uint32_t KS16, const float* __restrict__ centre,
                                                              const float* __restrict__ dimScale,
                                                              const int32_t* __restrict__ limbExp,
                                                              u32x4* __restrict__ frameH, int32_t* __restrict__ frameExp) {
    __shared__ float ys[8][128];  // y of the block's frames (D <= 126)
    __shared__ int   shE[8];
    const uint32_t   fl = threadIdx.x >> 5, t = threadIdx.x & 31u;
    const uint32_t   f       = blockIdx.x * 8u + fl;
    const bool       inRange = f < nFramesRead, valid = f < nFrames;
    const float*     x       = frames + static_cast<size_t>(f) * frameStride;
    float            ymax    = 0.0f;
    int              finite  = 1;
    if (valid)
        for (uint32_t k = t; k < D; k += 32u) {
            const float y = __fsub_rn(x[k], centre[k]);
            ys[fl][k]     = y;
            const float a = fabsf(__fmul_rn(__fmul_rn(y, y), dimScale[k]));
            const float b = fabsf(__fmul_rn(y, dimScale[D + k]));
            finite        = finite && a <= 3.40282347e+38f && b <= 3.40282347e+38f;
            ymax          = fmaxf(ymax, fmaxf(a, b));
        }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        ymax   = fmaxf(ymax, __shfl_xor(ymax, o, 32));
        finite = finite & __shfl_xor(finite, o, 32);
    }
    if (t == 0 && inRange) {
        int e = 0;
        if (valid && finite && ymax > 32768.0f) {
            int ex;
            frexpf(ymax, &ex);  // ymax in [2^(ex-1), 2^ex)
            e = ex - 15;
        }
        frameExp[f] = e;
        shE[fl]     = e;
    }
    __syncthreads();
    if (!inRange)
        return;
    const int e = shE[fl];
    // B fragments (16-row tiles): frame block f/16, lane 16*((k>>3)&3) + f%16, step k>>5
    const uint32_t fb = f / 16u, col = f % 16u;
    for (uint32_t q = t; q < KS16 * 4; q += 32u) {  // groups of 8 consecutive k
        uint32_t w[4] = {0, 0, 0, 0};
        if (valid)
            for (uint32_t j = 0; j < 8; ++j) {
                const uint32_t k = 8 * q + j;
                uint16_t       h = 0;
                if (k < 6 * D) {
                    const uint32_t part = k / D, d = k - part * D;
                    const float    y    = ys[fl][d];
                    const float    v    = part < 3 ? ldexpf(__fmul_rn(__fmul_rn(y, y), dimScale[d]), -e)
                                                   : ldexpf(__fmul_rn(y, dimScale[D + d]), -e);
                    const uint16_t hi = h16bits(v);
                    h = (part == 1 || part == 4) ? h16bits(v - static_cast<float>(__builtin_bit_cast(_Float16, hi))) : hi;
                }
                else if (k < 6 * D + kSplitLimbs) {
                    const int be = limbExp[k - 6 * D] - e;
                    h            = be < -24 ? 0 : h16bits(ldexpf(1.0f, be));
                }
                w[j >> 1] |= static_cast<uint32_t>(h) << (16 * (j & 1));
            }
        frameH[(static_cast<size_t>(fb) * KS16 + (q >> 2)) * 64 + 16 * (q & 3) + col] = u32x4{w[0], w[1], w[2], w[3]};
    }
}

// ---------------------------------------------------------------------------
// keys: a row's value v > 0 (row constants shifted by K0, ||x'||^2 the initial accumulator) is kept
// as the u32 bits of the float with the low keyBits mantissa bits replaced by (tile << 2 | r), r the
// accumulator slot (row 4g + r of the tile in lane group g).  Positive floats order like their bits,
// so one v_and_or_b32 per value and one v_min3_u32 per two values keep, per lane and slot, the
// minimum by (value, tile); the lane group g is resolved at the end of the mixture, where keys
// equal in value and tag prefer the lower group (lower density index).
// ---------------------------------------------------------------------------
// end of a mixture: the 4 slot keys of each column block -> (score, density) per frame, reduced
// across the four 16-lane groups by permlane swaps (r0 of a swap always comes from the lower group);
// lane l stores frame frame0 + l.  Straight-line code (no branch splits the basic block it is
// scheduled into): uniform options are arithmetic, the frame bound is the buffer's num_records.
// ---------------------------------------------------------------------------
template <bool BEST>
__device__ __forceinline__ void emitKeysSplit(const SplitArgs& a, const uint32_t (&k)[4], uint32_t m, uint32_t frame0,
                                              int lane, uint32_t g, uint32_t kmask, int eOut, float noneScore);

template <bool BEST>
__device__ __forceinline__ void emitMixtureSplit(const SplitArgs& a, const uint32_t (&best)[4][4], uint32_t m,
                                                 uint32_t frame0, int lane, uint32_t g, uint32_t kmask, int eOut,
                                                 float noneScore) {
#if GMM_SPLIT_DIAG_NOEMIT  // diagnostic (wrong results): the emit's cost, the minima kept live by one XOR chain
    {
        uint32_t x = 0;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                x ^= best[cb][r];
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.scores + static_cast<size_t>(m - a.mixBase) * a.scoreStride,
                                                         (short)0, static_cast<int>(a.nFrames * 4u), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(x, rs, static_cast<uint32_t>(frame0 + lane) * 4u, 0, GMM_STORE_CPOL);
        return;
    }
#endif
    uint32_t k[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        if (GMM_SPLIT_TAG_EMIT && kmask)  // slot r's keys carry tile << 2 only: r joins here (all ones stay)
            k[cb] = min(umin3(best[cb][0], best[cb][1] | 1u, best[cb][2] | 2u), best[cb][3] | 3u);
        else
            k[cb] = min(umin3(best[cb][0], best[cb][1], best[cb][2]), best[cb][3]);
    }
    emitKeysSplit<BEST>(a, k, m, frame0, lane, g, kmask, eOut, noneScore);
}

// the per-block minima k[cb] (over the block's slots, lane group g of the tile rows in every lane) -> (score,
// density) of frame frame0 + lane
template <bool BEST>
__device__ __forceinline__ void emitKeysSplit(const SplitArgs& a, const uint32_t (&k)[4], uint32_t m, uint32_t frame0,
                                              int lane, uint32_t g, uint32_t kmask, int eOut, float noneScore) {
    // groups {g&1, g&1|2} of blocks (0,2) and (1,3): lanes < 32 keep blocks 0, 1, lanes >= 32 blocks 2, 3
    uint32_t w[2], wg[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const auto r    = __builtin_amdgcn_permlane32_swap(k[p], k[p + 2], false, false);
        const bool take = r[1] < r[0];
        w[p]            = take ? r[1] : r[0];
        wg[p]           = (g & 1u) | (take ? 2u : 0u);
    }
    // groups {even, odd} rows: lane l keeps block l >> 4
    const auto     rk   = __builtin_amdgcn_permlane16_swap(w[0], w[1], false, false);
    const auto     rg   = __builtin_amdgcn_permlane16_swap(wg[0], wg[1], false, false);
    const bool     take = rk[1] < rk[0];
    const uint32_t key  = take ? rk[1] : rk[0];
    const uint32_t grp  = take ? rg[1] : rg[0];

    // midpoint of the masked bits: within 2^-(24 - keyBits) of the minimum's value
    const float kv    = __uint_as_float((key & ~kmask) | ((kmask + 1u) >> 1));
    const bool  none  = !(kv < 1e37f);  // no finite candidate (empty mixture, non-finite frame)
    float       total = __fsub_rn(ldexpf(kv, eOut), a.offsetK0);
    if (GMM_SPLIT_EMIT_FLAT)
        asm volatile("" : "+v"(total));  // computed for every lane: the select below stays a v_cndmask
    // diagonal-maximum: 0.5 total; batch-float keeps an overflowed total (BatchFeatureScorer.cc:468)
    const float score = none ? noneScore
                             : __fmul_rn(a.outScale, (a.flavor == 3 && !(total < 3.40282347e+38f)) ? total : 0.5f * total);
    const uint32_t idx = none ? 0xffffffffu : ((((key & kmask) >> 2) << 4) | (grp << 2) | (key & 3u));
    const uint32_t mo  = m - a.mixBase;
    const uint32_t off = static_cast<uint32_t>(frame0 + lane) * 4u;
    // frames >= nFrames fall outside num_records: the buffer store drops them
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.scores + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                     static_cast<int>(a.nFrames * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(score), rs, off, 0, GMM_STORE_CPOL);
    if constexpr (BEST) {
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(a.best + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                         static_cast<int>(a.nFrames * 4u), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(idx, rb, off, 0, GMM_STORE_CPOL);
    }
}

// ---------------------------------------------------------------------------
// scorer.  A workgroup of 256 frames = 2 waves x 128 frames (8 column blocks of 16; preselection and
// K steps > 5 as noted below) walks a chunk of mixtures on one XCD.  The 128 frames' f16 fragments are
// loop-invariant MFMA B operands and live in the accumulator file (an "a"-constrained asm pins them),
// the accumulators in VGPRs, one wave per SIMD.  Every mixture has an even number of tiles (host), so the
// chunk is a flat sequence of tile pairs.  Operands of PF consecutive pairs rotate through PF register
// sets loaded PF pairs ahead, and the pipeline is software-staged: step p issues the 64 MFMAs of pair p
// beside the epilogue (tag + min) of pair p-1, interleaved MFMA : VALU by sched_group_barrier, then emits
// the mixture that pair p-1 ended, if any.  Mixture bounds are scalar
// loads (mixTileOff is a restrict kernel argument): a vector load there would come with an
// s_waitcnt vmcnt(0) draining the prefetch.
// ---------------------------------------------------------------------------
// PRESEL (preselection-batch-float): every key is OR-ed with the sign-extended mask byte of its
// (frame, density cluster), so a density whose cluster the frame did not select becomes the all-ones
// key and never wins; the wave's mask tables (one per 64 frames, gmm_kernels_presel.hip) sit in LDS, a
// tile carries the 16 rows' table offsets, and a pair's mask words are read in the step that issues its
// MFMAs.
extern __shared__ __attribute__((aligned(16))) uint32_t splitSelLds[];

template <int KS, bool BEST, bool PRESEL>
__global__ __launch_bounds__(PRESEL ? kSplitFramesPerBlock / splitPreselNF(KS) * 4 : 64 * kSplitMainWaves, GMM_SPLIT_MIN_WAVES) void scoreSplit(SplitArgs a,
                                                                      const uint32_t* __restrict__ mixTileOff) {
    constexpr int  NF   = PRESEL ? splitPreselNF(KS) : kSplitNF;  // 4 or 8 column blocks; the emit works on halves of 4
    constexpr int  NH   = NF / 4;
    static_assert(NF == 4 || NF == 8, "64 or 128 frames per wave");
    const int      lane = threadIdx.x & 63;
    const int      wave = threadIdx.x >> 6;
    const uint32_t g    = static_cast<uint32_t>(lane) >> 4;
    uint32_t       chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * kSplitFramesPerBlock + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t fb0    = frame0 / 16u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];

    // preselection: this wave's NH 64-frame mask tables [cluster][16] into LDS (each wave reads only its own)
    uint32_t laneSel = 0, selWords = 0;  // byte address of (wave's first table, column t = lane & 15); table words
    if constexpr (PRESEL) {
        selWords = a.nClusters * 16u;
        const u32x4* src = reinterpret_cast<const u32x4*>(a.selT + static_cast<size_t>(frame0 / 64u) * selWords);
        u32x4*       dst = reinterpret_cast<u32x4*>(splitSelLds + static_cast<uint32_t>(wave) * NH * selWords);
        for (uint32_t i = static_cast<uint32_t>(lane); i < NH * selWords / 4u; i += 64u)
            dst[i] = src[i];
        laneSel = (static_cast<uint32_t>(wave) * NH * selWords + (static_cast<uint32_t>(lane) & 15u)) * 4u;
    }
    const uint2* tclu = static_cast<const uint2*>(a.tileClu);

    const f16x8* th       = static_cast<const f16x8*>(a.tileH);
    const auto   loadTile = [&](uint32_t tt, f16x8(&A)[KS], uint2& Cw) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = th[(static_cast<size_t>(GMM_SPLIT_DIAG_HOT ? T0 + (tt & 1u) : tt) * KS + s) * 64 + lane];
        if constexpr (PRESEL)
            Cw = tclu[static_cast<size_t>(tt) * 4 + g];  // rows 4g .. 4g+3: cluster * 64, u16 each
    };
    // the mask words of a tile's 4 rows in this lane: T[h][r] of row 4g + r, column frame0 + 64 h + 16 cb +
    // (lane & 15) in byte cb
    const auto readSel = [&](const uint2& Cw, uint32_t(&T)[NH][4]) __attribute__((always_inline)) {
        if constexpr (PRESEL) {
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const char* base = reinterpret_cast<const char*>(splitSelLds) + laneSel + h * selWords * 4u;
                T[h][0]          = *reinterpret_cast<const uint32_t*>(base + (Cw.x & 0xffffu));
                T[h][1]          = *reinterpret_cast<const uint32_t*>(base + (Cw.x >> 16));
                T[h][2]          = *reinterpret_cast<const uint32_t*>(base + (Cw.y & 0xffffu));
                T[h][3]          = *reinterpret_cast<const uint32_t*>(base + (Cw.y >> 16));
            }
        }
    };

    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NF][KS];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[cb][s] = fh[(static_cast<size_t>(fb0 + cb) * KS + s) * 64 + lane];
    int eOut[NH];  // exponents of the frames this lane stores (frame0 + 64 h + lane)
#pragma unroll
    for (int h = 0; h < NH; ++h)
        eOut[h] = a.frameExp[frame0 + 64u * h + lane];
    // wait for the frame operands here, before the tile prefetch is issued: otherwise the waitcnt pass
    // sees them possibly pending at the loop header and drains the whole queue there every iteration
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            if constexpr (NF == 8)  // loop-invariant MFMA operands: to the accumulator file (VGPRs: the epilogue)
                asm volatile("" : "+a"(B[cb][s]));
            else
                asm volatile("" ::"v"(B[cb][s]));
    }
#pragma unroll
    for (int h = 0; h < NH; ++h)
        asm volatile("" ::"v"(eOut[h]));

    // operand registers of PF pairs in flight: pair j (counted from T0) in set j % PF, loaded when pair j - PF has
    // been issued (the tile array is padded by kTilePad >= 2 PF tiles: prefetching past T1 stays in bounds).
    // PF = 2; 3 measured 2.6 % slower at 128 frames per wave (GMM_SPLIT_PF)
    constexpr int PF = (PRESEL || KS > 5) ? 2 : GMM_SPLIT_PF;  // K steps 6-8: registers
    f16x8         R[PF][2][KS];
    uint2         C[PF][2];
#pragma unroll
    for (int j = 0; j < PF; ++j) {
        C[j][0] = C[j][1] = uint2{0, 0};
        loadTile(T0 + 2 * j, R[j][0], C[j][0]);
        loadTile(T0 + 2 * j + 1, R[j][1], C[j][1]);
    }

    // scores only (no best density; preselection-batch-float is a batch type): keys are the values' own bits
    const uint32_t kmask = BEST ? (1u << a.tileBits) - 1u : 0u;
    // the value mask lives in a VGPR so that (bits & mask) | tag is ONE v_and_or_b32 with the tag in an
    // SGPR (gfx950 VOP3 reads at most one SGPR)
    uint32_t vmask = ~kmask;
    asm volatile("" : "+v"(vmask));
    // score of a mixture without a finite candidate: Core::Type<Score>::max, halved by diagonal-maximum;
    // preselection: the backoff score (BatchFeatureScorer.cc:282-288)
    const float noneScore = __fmul_rn(a.outScale, PRESEL ? a.backoff
                                                         : (a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f));

    // running minima per column block and accumulator slot (one register per slot measured fastest: 4.81 ms
    // against 4.88 / 4.89 with the slots sharing 1 or 2 registers, profiles/r02/ab/ab_split_slots.txt)
    constexpr int kSlots = 4;
    uint32_t      best[NF][kSlots];
    const auto    resetBest = [&]() {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < kSlots; ++r)
                best[cb][r] = 0xffffffffu;
    };
    const auto chain = [&](const f16x8(&A)[KS], f32x4(&acc)[NF]) __attribute__((always_inline)) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            acc[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};  // ||x'||^2 is in K: the chain starts from an inline 0
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s], B[cb][s], acc[cb], 0, 0, 0);
    };
    // epilogue of one pair of tiles (tile numbers tl, tl + 1 in the mixture); TT: their mask words
    const auto pairEpilogue = [&](const f32x4(&acc)[2][NF], uint32_t tl, const uint32_t(&TT)[2][NH][4]) __attribute__((always_inline)) {
        // per-slot tags as opaque SGPRs: with a visible constant the compiler splits the tag OR off the
        // v_and_or_b32 into a v_and + v_or3 pair (non-volatile asm: no scheduling barrier)
        uint32_t tagA[4], tagB[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t rr = GMM_SPLIT_TAG_EMIT ? 0u : static_cast<uint32_t>(r);
            tagA[r] = (tl << 2) | rr;
            tagB[r] = ((tl + 1u) << 2) | rr;
            asm("" : "+s"(tagA[r]), "+s"(tagB[r]));
        }
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t ka = (__float_as_uint(acc[0][cb][r]) & vmask) | tagA[r];
                const uint32_t kb = (__float_as_uint(acc[1][cb][r]) & vmask) | tagB[r];
                if constexpr (PRESEL) {
                    // preselection-batch-float has no best density: the key is the value's own bits OR the
                    // sign-extended mask byte (one v_or_b32_sdwa per value; a deselected density becomes all ones,
                    // above every value; round 5 carried the tile tag too: 2 VALU per value)
                    const uint32_t ca = static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(TT[0][cb / 4][r] >> (8 * (cb % 4)))));
                    const uint32_t cc = static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(TT[1][cb / 4][r] >> (8 * (cb % 4)))));
                    best[cb][r] = umin3(best[cb][r], __float_as_uint(acc[0][cb][r]) | ca, __float_as_uint(acc[1][cb][r]) | cc);
                }
                else if constexpr (BEST) {
                    best[cb][r] = umin3(best[cb][r], ka, kb);
                }
                else {  // scores only: the full f32 value, no tag (one v_min3_u32 per two values)
                    (void)ka, (void)kb;
                    best[cb][r] = umin3(best[cb][r], __float_as_uint(acc[0][cb][r]), __float_as_uint(acc[1][cb][r]));
                }
            }
    };

    uint32_t m = m0, tBeg = T0, tEnd = m0 < m1 ? mixTileOff[m0 + 1] : T0;
    resetBest();
    const auto emit = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < NH; ++h)
            emitMixtureSplit<BEST>(a, *reinterpret_cast<const uint32_t(*)[4][4]>(&best[4 * h]), m, frame0 + 64u * h,
                                   lane, g, kmask, eOut[h], noneScore);
    };
    // after an emit at tile tNext: next mixture, and the empty ones that also end there (rare path)
    const auto advance = [&](uint32_t tNext) __attribute__((always_inline)) {
        ++m;
        tBeg = tNext;
        tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        while (m < m1 && tEnd == tNext) {
            emit();
            ++m;
            tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        }
    };
    // one pipeline step: the MFMAs of the pair in (A0, A1) into cur beside the epilogue of the pair in
    // prev, interleaved 1 MFMA : 2 VALU (the operand loads for PF pairs ahead follow, then finish())
    // (PRESEL: the mask words of the pair in (C0w, C1w) are read into TTcur; TTprev are prev's)
    constexpr int kIl = PRESEL ? 28 * NH : GMM_SPLIT_IL * NH, kIlV = PRESEL ? 3 : 2;
    const auto step = [&](const f16x8(&A0)[KS], const f16x8(&A1)[KS], f32x4(&cur)[2][NF],
                          const f32x4(&prev)[2][NF], uint32_t tPrev, const uint2& C0w, const uint2& C1w,
                          uint32_t(&TTcur)[2][NH][4], const uint32_t(&TTprev)[2][NH][4]) __attribute__((always_inline)) {
        chain(A0, cur[0]);
        chain(A1, cur[1]);
        readSel(C0w, TTcur[0]);
        readSel(C1w, TTcur[1]);
        pairEpilogue(prev, tPrev - tBeg, TTprev);
#pragma unroll
        for (int i = 0; i < kIl; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);     // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, kIlV, 0);  // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * NF * KS - kIl, 0);
    };
    // the emit of the mixture that ended at tile tNext, if any, in a block of its own (inside the interleaved
    // step it measured 9-11 % slower at 128 frames per wave)
    const auto finish = [&](uint32_t tNext) __attribute__((always_inline)) {
        if (tNext == tEnd) {
            emit();
            resetBest();
            advance(tNext);
        }
    };
    // the last pair's epilogue (nothing left to overlap it with)
    const auto drain = [&](const f32x4(&prev)[2][NF], uint32_t tPrev, const uint32_t(&TTprev)[2][NH][4]) __attribute__((always_inline)) {
        pairEpilogue(prev, tPrev - tBeg, TTprev);
        finish(tPrev + 2);
    };

    // mixtures without tiles at the start of the chunk
    while (m < m1 && tEnd == T0) {
        emit();
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T0;
    }
    if (T0 < T1) {
        // pair j: accumulators acc[j % 2] (step j reads pair j - 1's from the other set), operands R[j % PF];
        // the loop body is lcm(2, PF) pairs so that every index is a compile-time constant
        constexpr int U = PF % 2 == 0 ? PF : 2 * PF;
        f32x4         acc[2][2][NF];
        uint32_t      TT[2][2][NH][4] = {};
        chain(R[0][0], acc[0][0]);  // pair 0: nothing to finish beside it
        chain(R[0][1], acc[0][1]);
        readSel(C[0][0], TT[0][0]);
        readSel(C[0][1], TT[0][1]);
        loadTile(T0 + 2 * PF, R[0][0], C[0][0]);
        loadTile(T0 + 2 * PF + 1, R[0][1], C[0][1]);
        uint32_t t = T0 + 2;  // first tile of pair 1
        // sub-step i of a loop iteration: pair j = 1 + i (mod U) at tile tt
        const auto sub = [&](auto ic, uint32_t tt) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value, set = (1 + i) % PF, cur = (1 + i) % 2, prv = i % 2;
            step(R[set][0], R[set][1], acc[cur], acc[prv], tt - 2, C[set][0], C[set][1], TT[cur], TT[prv]);
            loadTile(tt + 2 * PF, R[set][0], C[set][0]);  // the tile array is padded by kTilePad >= 2 PF tiles
            loadTile(tt + 2 * PF + 1, R[set][1], C[set][1]);
            finish(tt);
        };
        for (; t + 2 * U <= T1; t += 2 * U)
            staticFor<U>([&](auto ic) __attribute__((always_inline)) { sub(ic, t + 2u * decltype(ic)::value); });
        // fewer than U pairs left, then the last pair's epilogue
        bool live = true;
        staticFor<U>([&](auto ic) __attribute__((always_inline)) {
            constexpr int  i  = decltype(ic)::value;
            const uint32_t tt = t + 2u * i;
            if (live) {
                if (tt < T1) {
                    sub(ic, tt);
                }
                else {
                    drain(acc[i % 2], tt - 2, TT[i % 2]);
                    live = false;
                }
            }
        });
    }
}

// ---------------------------------------------------------------------------
// scoreSplitWide (GMM_SPLIT_WIDE; no preselection): one wave per workgroup holds NF column blocks of 16 frames --
// 16 (256 frames) at K steps <= 4 (D <= 40), 12 (192 frames) at 5 (D <= 51), whose f16 fragments fill the
// accumulator file (256 / 240 AGPRs) -- and walks its chunk ONE tile per pipeline step: the tile's NF x KS MFMAs
// beside the epilogue of the previous tile.  Against scoreSplit's 128-frame waves every tile fragment a wave loads
// feeds 2x (1.5x) the MFMAs (less L2-to-CU traffic and per-tile address and loop work per MFMA), and the frame tiles
// of a chunk run at once on one XCD (4 one-wave workgroups per CU), so the chunk streams through its L2 about once.
// The min3 takes two slots of the same tile (rows 4g + r: the key's tag carries r), two running minima per block.
// ---------------------------------------------------------------------------
#ifndef GMM_SPLIT_WIDE_PF
#define GMM_SPLIT_WIDE_PF 3  // tiles in flight
#endif
#ifndef GMM_SPLIT_WIDE_IL
#define GMM_SPLIT_WIDE_IL 64  // MFMAs of a step interleaved 1 : 2 with the epilogue VALU (at 16 blocks; 64 with one slot: -0.5 %, profiles/r06/s5)
#endif
#ifndef GMM_SPLIT_WIDE_SLOTS
#define GMM_SPLIT_WIDE_SLOTS 1  // running minima per column block (1: the two min3 of a block chained; -1.3 %, profiles/r06/s5)
#endif

template <int KS, bool BEST>
__global__ __launch_bounds__(64, 1) void scoreSplitWide(SplitArgs a, const uint32_t* __restrict__ mixTileOff) {
    constexpr uint32_t FPB = splitWideFrames(KS);  // frames of the workgroup's one wave
    constexpr int      NF = FPB / 16, NH = NF / 4, PF = GMM_SPLIT_WIDE_PF, U = PF % 2 == 0 ? PF : 2 * PF;
    static_assert(FPB != 0 && NF * KS * 4 <= 256, "the frame operands fill at most the accumulator file");
    const int      lane = threadIdx.x & 63;
    const uint32_t g    = static_cast<uint32_t>(lane) >> 4;
    uint32_t       chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * FPB, fb0 = frame0 / 16u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];

    const f16x8* th       = static_cast<const f16x8*>(a.tileH);
    const auto   loadTile = [&](uint32_t tt, f16x8(&A)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = th[(static_cast<size_t>(tt) * KS + s) * 64 + lane];
    };
    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NF][KS];
#pragma unroll
    for (int cb = 0; cb < NF; ++cb)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[cb][s] = fh[(static_cast<size_t>(fb0 + cb) * KS + s) * 64 + lane];
    int eOut[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h)
        eOut[h] = a.frameExp[frame0 + 64u * h + lane];
    // the frame operands complete before the tile prefetch, then pinned to the accumulator file
#pragma unroll
    for (int cb = 0; cb < NF; ++cb)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            asm volatile("" : "+a"(B[cb][s]));
#pragma unroll
    for (int h = 0; h < NH; ++h)
        asm volatile("" ::"v"(eOut[h]));

    f16x8 R[PF][KS];  // tile j (from T0) in set j % PF; the tile array's kTilePad tiles keep prefetches in bounds
#pragma unroll
    for (int j = 0; j < PF; ++j)
        loadTile(T0 + j, R[j]);

    const uint32_t kmask = BEST ? (1u << a.tileBits) - 1u : 0u;
    uint32_t       vmask = ~kmask;
    asm volatile("" : "+v"(vmask));
    const float noneScore = __fmul_rn(a.outScale, a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f);

    // slot 0: rows 4g, 4g + 1; slot 1: rows 4g + 2, 4g + 3 (GMM_SPLIT_WIDE_SLOTS 1: one slot, the min3 chained)
    uint32_t   best[NF][2];
    const auto resetBest = [&]() {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            best[cb][0] = best[cb][1] = 0xffffffffu;
    };
    const auto chain = [&](const f16x8(&A)[KS], f32x4(&acc)[NF]) __attribute__((always_inline)) {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            acc[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                acc[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s], B[cb][s], acc[cb], 0, 0, 0);
    };
    const auto epilogue = [&](const f32x4(&acc)[NF], uint32_t tl) __attribute__((always_inline)) {
        uint32_t tag[4];  // opaque SGPRs: one v_and_or_b32 per value
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            tag[r] = (tl << 2) | static_cast<uint32_t>(r);
            asm("" : "+s"(tag[r]));
        }
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            uint32_t v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                v[r] = BEST ? (__float_as_uint(acc[cb][r]) & vmask) | tag[r] : __float_as_uint(acc[cb][r]);
#if GMM_SPLIT_WIDE_SLOTS == 1
            best[cb][0] = umin3(umin3(best[cb][0], v[0], v[1]), v[2], v[3]);
#else
            best[cb][0] = umin3(best[cb][0], v[0], v[1]);
            best[cb][1] = umin3(best[cb][1], v[2], v[3]);
#endif
        }
    };

    uint32_t   m = m0, tBeg = T0, tEnd = m0 < m1 ? mixTileOff[m0 + 1] : T0;
    const auto emit = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
            uint32_t k[4];
#pragma unroll
            for (int cb = 0; cb < 4; ++cb)
                k[cb] = min(best[4 * h + cb][0], best[4 * h + cb][1]);
            emitKeysSplit<BEST>(a, k, m, frame0 + 64u * h, lane, g, kmask, eOut[h], noneScore);
        }
    };
    const auto advance = [&](uint32_t tNext) __attribute__((always_inline)) {
        ++m;
        tBeg = tNext;
        tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        while (m < m1 && tEnd == tNext) {
            emit();
            ++m;
            tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        }
    };
    const auto finish = [&](uint32_t tNext) __attribute__((always_inline)) {
        if (tNext == tEnd) {
            emit();
            resetBest();
            advance(tNext);
        }
    };
    constexpr int kIl = GMM_SPLIT_WIDE_IL * NF / 16;  // MFMAs with 2 VALU each: the 6 NF epilogue VALU
    const auto    step = [&](const f16x8(&A)[KS], f32x4(&cur)[NF], const f32x4(&prev)[NF], uint32_t tPrev)
            __attribute__((always_inline)) {
        chain(A, cur);
        epilogue(prev, tPrev - tBeg);
#pragma unroll
        for (int i = 0; i < kIl; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NF * KS - kIl, 0);
    };

    resetBest();
    while (m < m1 && tEnd == T0) {  // mixtures without tiles at the start of the chunk
        emit();
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T0;
    }
    if (T0 < T1) {
        f32x4 acc[2][NF];
        chain(R[0], acc[0]);  // tile T0: nothing to finish beside it
        loadTile(T0 + PF, R[0]);
        uint32_t t = T0 + 1;
        // tile tt = T0 + j with j = 1 + i (mod U): operands R[j % PF], accumulators acc[j % 2]
        const auto sub = [&](auto ic, uint32_t tt) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value, set = (1 + i) % PF, cur = (1 + i) % 2, prv = i % 2;
            step(R[set], acc[cur], acc[prv], tt - 1);
            loadTile(tt + PF, R[set]);
            finish(tt);
        };
        for (; t + U <= T1; t += U)
            staticFor<U>([&](auto ic) __attribute__((always_inline)) { sub(ic, t + decltype(ic)::value); });
        bool live = true;
        staticFor<U>([&](auto ic) __attribute__((always_inline)) {
            constexpr int  i  = decltype(ic)::value;
            const uint32_t tt = t + i;
            if (live) {
                if (tt < T1) {
                    sub(ic, tt);
                }
                else {  // the last tile's epilogue
                    epilogue(acc[i % 2], tt - 1 - tBeg);
                    finish(tt);
                    live = false;
                }
            }
        });
    }
}

// ---------------------------------------------------------------------------
// 32-density tiles on v_mfma_f32_32x32x16_f16 (mixtures of <= 512 densities).  Per 16x16x32-equivalent
// of work the 32x32x16 MFMA holds the SIMD's vector issue half as long (8 of 32 cycles), which leaves
// the issue slots to the epilogue VALU.  Lane l (r = l & 31, h = l >> 5) holds A[row r][k = 16s+8h+j],
// B[k = 16s+8h+j][frame r] and accumulator register i = row (i & 3) + 8 (i >> 2) + 4 h of frame r.
// A wave owns 64 frames (two 32-frame blocks); one pipeline step = one tile = 2 x KS MFMAs beside
// the epilogue of the previous tile.  Keys: value bits with the low keyBits replaced by
// (tile << 4 | i); four slots per block keep the minimum over registers {q, q+4, q+8, q+12}.
// ---------------------------------------------------------------------------
template <bool BEST>
__device__ __forceinline__ void emitMixtureSplit32(const SplitArgs& a, const uint32_t (&best)[2][4], uint32_t m,
                                                   uint32_t frame0, int lane, uint32_t kmask, int eOut,
                                                   float noneScore) {
    uint32_t k[2];
#pragma unroll
    for (int b = 0; b < 2; ++b)
        k[b] = min(umin3(best[b][0], best[b][1], best[b][2]), best[b][3]);
    // lanes < 32 keep block 0, lanes >= 32 block 1; r[0] from lane half h = 0, r[1] from h = 1
    const auto     r    = __builtin_amdgcn_permlane32_swap(k[0], k[1], false, false);
    // (value, tile) first, then the row in the tile: row(i, h) = (i & 3) + 8 (i >> 2) + 4 h
    const uint32_t hi0  = r[0] & ~15u, hi1 = r[1] & ~15u;
    const uint32_t row0 = (r[0] & 3u) | ((r[0] & 12u) << 1), row1 = ((r[1] & 3u) | ((r[1] & 12u) << 1)) + 4u;
    // scores only: untagged values, the plain minimum
    const bool     take = BEST ? (hi1 < hi0 || (hi1 == hi0 && row1 < row0)) : r[1] < r[0];
    const uint32_t key  = take ? r[1] : r[0];
    const uint32_t row  = take ? row1 : row0;

    const float kv    = __uint_as_float((key & ~kmask) | ((kmask + 1u) >> 1));
    const bool  none  = !(kv < 1e37f);
    const float total = __fsub_rn(ldexpf(kv, eOut), a.offsetK0);
    const float score = none ? noneScore
                             : __fmul_rn(a.outScale, (a.flavor == 3 && !(total < 3.40282347e+38f)) ? total : 0.5f * total);
    const uint32_t idx = none ? 0xffffffffu : ((((key & kmask) >> 4) << 5) | row);
    const uint32_t mo  = m - a.mixBase;
    const uint32_t off = static_cast<uint32_t>(frame0 + lane) * 4u;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.scores + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                     static_cast<int>(a.nFrames * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(score), rs, off, 0, GMM_STORE_CPOL);
    if constexpr (BEST) {
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(a.best + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                         static_cast<int>(a.nFrames * 4u), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(idx, rb, off, 0, GMM_STORE_CPOL);
    }
}

#ifndef GMM_SPLIT32_IL
#define GMM_SPLIT32_IL 3  // scoreSplit32: VALU per MFMA in a step's interleave
#endif
#ifndef GMM_SPLIT32_NB
#define GMM_SPLIT32_NB 4  // 32-frame column blocks per wave of scoreSplit32 (4: 128 frames, B in the AGPRs; 2: 64)
#endif

template <int KS, bool BEST>
__global__ __launch_bounds__(64 * (kSplitFramesPerBlock / (32 * GMM_SPLIT32_NB)), GMM_SPLIT_MIN_WAVES) void scoreSplit32(
        SplitArgs a, const uint32_t* __restrict__ mixTileOff) {
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    constexpr int NB = GMM_SPLIT32_NB, NH = NB / 2;  // blocks of 32 frames; halves of 64 frames (one emit each)
    static_assert(NB == 2 || NB == 4, "64 or 128 frames per wave");
    const int      lane = threadIdx.x & 63;
    const int      wave = threadIdx.x >> 6;
    uint32_t       chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * kSplitFramesPerBlock + static_cast<uint32_t>(wave) * (32u * NB);
    const uint32_t fb0    = frame0 / 32u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];

    const f16x8* th       = static_cast<const f16x8*>(a.tileH);
    const auto   loadTile = [&](uint32_t tt, f16x8(&A)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = th[(static_cast<size_t>(tt) * KS + s) * 64 + lane];
    };
    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NB][KS];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[b][s] = fh[(static_cast<size_t>(fb0 + b) * KS + s) * 64 + lane];
    int eOut[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h)
        eOut[h] = a.frameExp[frame0 + 64u * h + lane];
    // frame operands complete before the tile prefetch (see scoreSplit); 128-frame waves keep them in the AGPRs
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int s = 0; s < KS; ++s)
            if constexpr (NB == 4)
                asm volatile("" : "+a"(B[b][s]));
            else
                asm volatile("" ::"v"(B[b][s]));
#pragma unroll
    for (int h = 0; h < NH; ++h)
        asm volatile("" ::"v"(eOut[h]));

    f16x8 R0[KS], R1[KS];  // tiles t (even steps) and t + 1; padded tile array: loads past T1 stay in bounds
    loadTile(T0, R0);
    loadTile(T0 + 1, R1);

    const uint32_t kmask = BEST ? (1u << a.tileBits) - 1u : 0u;  // scores only: untagged values
    uint32_t       vmask = ~kmask;
    asm volatile("" : "+v"(vmask));
    const float noneScore = __fmul_rn(a.outScale, a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f);

    uint32_t   best[NB][4];
    const auto resetBest = [&]() {
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                best[b][q] = 0xffffffffu;
    };
    const auto chain = [&](const f16x8(&A)[KS], f32x16(&acc)[NB]) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
            acc[b] = f32x16{};  // ||x'||^2 is in K: the chain starts from an inline 0
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int b = 0; b < NB; ++b)
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], B[b][s], acc[b], 0, 0, 0);
    };
    const auto epilogue = [&](const f32x16(&acc)[NB], uint32_t tl) {
        uint32_t tag[16];  // opaque SGPRs (one v_and_or_b32 per value)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            tag[i] = (tl << 4) | static_cast<uint32_t>(i);
            asm("" : "+s"(tag[i]));
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if constexpr (!BEST) {  // scores only: the values' own bits
                    best[b][q] = umin3(umin3(best[b][q], __float_as_uint(acc[b][q]), __float_as_uint(acc[b][q + 4])),
                                       __float_as_uint(acc[b][q + 8]), __float_as_uint(acc[b][q + 12]));
                    continue;
                }
                const uint32_t k0 = (__float_as_uint(acc[b][q]) & vmask) | tag[q];
                const uint32_t k1 = (__float_as_uint(acc[b][q + 4]) & vmask) | tag[q + 4];
                const uint32_t k2 = (__float_as_uint(acc[b][q + 8]) & vmask) | tag[q + 8];
                const uint32_t k3 = (__float_as_uint(acc[b][q + 12]) & vmask) | tag[q + 12];
                best[b][q]        = umin3(umin3(best[b][q], k0, k1), k2, k3);
            }
    };

    uint32_t m = m0, tBeg = T0, tEnd = m0 < m1 ? mixTileOff[m0 + 1] : T0;
    resetBest();
    const auto emit = [&]() {
#pragma unroll
        for (int h = 0; h < NH; ++h)
            emitMixtureSplit32<BEST>(a, *reinterpret_cast<const uint32_t(*)[2][4]>(&best[2 * h]), m, frame0 + 64u * h,
                                     lane, kmask, eOut[h], noneScore);
    };
    const auto advance = [&](uint32_t tNext) {
        ++m;
        tBeg = tNext;
        tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        while (m < m1 && tEnd == tNext) {
            emit();
            ++m;
            tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        }
    };
    const auto finish = [&](uint32_t tNext) {
        if (tNext == tEnd) {
            emit();
            resetBest();
            advance(tNext);
        }
    };
    // MFMAs of the tile in A into cur beside the epilogue of tile tPrev (in prev), 1 MFMA : GMM_SPLIT32_IL VALU
    const auto step = [&](const f16x8(&A)[KS], f32x16(&cur)[NB], const f32x16(&prev)[NB], uint32_t tPrev) {
        chain(A, cur);
        epilogue(prev, tPrev - tBeg);
#pragma unroll
        for (int i = 0; i < NB * KS; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);              // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, GMM_SPLIT32_IL, 0);  // VALU
        }
    };

    while (m < m1 && tEnd == T0) {  // mixtures without tiles at the start of the chunk
        emit();
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T0;
    }
    if (T0 < T1) {
        f32x16   accX[NB], accY[NB];
        uint32_t t = T0;
        chain(R0, accX);  // tile T0: nothing to finish beside it
        loadTile(t + 2, R0);
        t += 1;
        for (; t + 2 <= T1; t += 2) {
            step(R1, accY, accX, t - 1);
            loadTile(t + 2, R1);
            finish(t);
            step(R0, accX, accY, t);
            loadTile(t + 3, R0);
            finish(t + 1);
        }
        if (t < T1) {  // one more tile (in R1)
            step(R1, accY, accX, t - 1);
            finish(t);
            epilogue(accY, t - tBeg);
            finish(t + 1);
        }
        else {
            epilogue(accX, t - 1 - tBeg);
            finish(t);
        }
    }
}

// ---------------------------------------------------------------------------
// diagonal-sum (GaussDiagonalSumFeatureScorer, GaussDiagonalMaximumFeatureScorer.cc:221-298):
// score = best - log sum_d exp(best - s_d) = -log sum_d exp(-s_d), best density as diagonal-maximum.
// With u the MFMA value (2 s + K0, times 2^-e) and kap = 0.5 log2(e) 2^e of the frame,
// exp(-s_d) = exp(K0/2) 2^(-kap u_d), so every lane keeps, per column block, a reference R (on the
// kap u scale) and per slot S = sum 2^(R - kap u): one v_fma + v_exp + v_add per value beside the
// (tag, min) key of diagonal-maximum.  R is re-based (a uniform branch, taken at the first tile of a
// mixture and rarely after) whenever the smallest value so far would put an exponent above 64; the
// final score is R ln2 - K0/2 - ln(S) after the (R, S) pairs of the four lane groups are merged on a
// common R.
//
// Software pipeline per 16-row tile: step t issues the KS x NF MFMAs of tile t beside the epilogue of
// tile t-1, in two halves around the re-base branch -- keys + min and the re-base test beside the first
// KS/2 k-steps, the exponentials and sums beside the rest -- then emits the mixture tile t-1 ended, if
// any.  Two slots per column block (a key carries its row, so any slot may hold any row).  Operands of
// four consecutive tiles in flight (R0..R3), accumulators alternate between two sets.
// ---------------------------------------------------------------------------
template <bool BEST>
__device__ __forceinline__ void emitMixtureSplitSum(const SplitArgs& a, const uint32_t (&best)[4][2],
                                                    const float (&S)[4][2], const float (&R)[4], uint32_t m,
                                                    uint32_t frame0, int lane, uint32_t g, uint32_t kmask) {
    uint32_t k[4];
    float    sum[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
        k[cb]   = min(best[cb][0], best[cb][1]);
        sum[cb] = S[cb][0] + S[cb][1];
    }
    // merge (R, S) of two lane groups on the smaller R
    const auto merge = [](float ra, float sa, float rb, float sb, float& r, float& sm) {
        const float d = ra - rb;
        r             = fminf(ra, rb);
        sm            = d <= 0.0f ? __builtin_fmaf(sb, __builtin_amdgcn_exp2f(d), sa)
                                  : __builtin_fmaf(sa, __builtin_amdgcn_exp2f(-d), sb);
    };
    uint32_t w[2], wg[2];
    float    wr[2], ws[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const auto     r    = __builtin_amdgcn_permlane32_swap(k[p], k[p + 2], false, false);
        const auto     rr   = __builtin_amdgcn_permlane32_swap(__float_as_uint(R[p]), __float_as_uint(R[p + 2]), false, false);
        const auto     rs   = __builtin_amdgcn_permlane32_swap(__float_as_uint(sum[p]), __float_as_uint(sum[p + 2]), false, false);
        const bool     take = r[1] < r[0];
        w[p]                = take ? r[1] : r[0];
        wg[p]               = (g & 1u) | (take ? 2u : 0u);
        merge(__uint_as_float(rr[0]), __uint_as_float(rs[0]), __uint_as_float(rr[1]), __uint_as_float(rs[1]), wr[p], ws[p]);
    }
    const auto     rk   = __builtin_amdgcn_permlane16_swap(w[0], w[1], false, false);
    const auto     rg   = __builtin_amdgcn_permlane16_swap(wg[0], wg[1], false, false);
    const auto     rr   = __builtin_amdgcn_permlane16_swap(__float_as_uint(wr[0]), __float_as_uint(wr[1]), false, false);
    const auto     rs   = __builtin_amdgcn_permlane16_swap(__float_as_uint(ws[0]), __float_as_uint(ws[1]), false, false);
    const bool     take = rk[1] < rk[0];
    const uint32_t key  = take ? rk[1] : rk[0];
    const uint32_t grp  = take ? rg[1] : rg[0];
    float          rf, sf;
    merge(__uint_as_float(rr[0]), __uint_as_float(rs[0]), __uint_as_float(rr[1]), __uint_as_float(rs[1]), rf, sf);

    const float kv   = __uint_as_float((key & ~kmask) | ((kmask + 1u) >> 1));
    const bool  none = !(kv < 1e37f);  // empty mixture: R stays 1e30, S = 0 -> +inf, as the reference
    // -log sum exp(-s_d) = R ln2 - K0/2 - ln S  (ln S = log2 S * ln2)
    const float score = __fmul_rn(a.outScale, (rf - __builtin_amdgcn_logf(sf)) * 0.693147181f - 0.5f * a.offsetK0);
    const uint32_t idx = none ? 0xffffffffu : ((((key & kmask) >> 2) << 4) | (grp << 2) | (key & 3u));
    const uint32_t mo  = m - a.mixBase;
    const uint32_t off = static_cast<uint32_t>(frame0 + lane) * 4u;
    const auto rs_ = __builtin_amdgcn_make_buffer_rsrc(a.scores + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                      static_cast<int>(a.nFrames * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(score), rs_, off, 0, GMM_STORE_CPOL);
    if constexpr (BEST) {
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(a.best + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                         static_cast<int>(a.nFrames * 4u), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(idx, rb, off, 0, GMM_STORE_CPOL);
    }
}

template <int KS, bool BEST>
__global__ __launch_bounds__(kSplitFramesPerBlock / GMM_SPLIT_SUM_NF * 4, GMM_SPLIT_MIN_WAVES) void scoreSplitSum(
        SplitArgs a, const uint32_t* __restrict__ mixTileOffArg) {
    // mixture bounds through the constant address space (constTable): -2.1 % here (profiles/r05/s26); the other
    // split kernels keep the generic pointer (the wide kernel neutral, scoreSplit32 +0.6 %, s27)
    const auto mixTileOff = constTable(mixTileOffArg);
    constexpr int  NF   = GMM_SPLIT_SUM_NF;  // 4 or 8 column blocks; the emit works on halves of 4
    constexpr int  NH   = NF / 4;
    constexpr int  KH   = KS / 2;  // k-steps issued beside the first half of the epilogue
    const int      lane = threadIdx.x & 63;
    const int      wave = threadIdx.x >> 6;
    const uint32_t g    = static_cast<uint32_t>(lane) >> 4;
    uint32_t       chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * kSplitFramesPerBlock + static_cast<uint32_t>(wave) * (NF * 16u);
    const uint32_t fb0    = frame0 / 16u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];

    const f16x8* th       = static_cast<const f16x8*>(a.tileH);
    const auto   loadTile = [&](uint32_t tt, f16x8(&A)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = th[(static_cast<size_t>(tt) * KS + s) * 64 + lane];
    };
    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NF][KS];
    float        kap[NF];  // 0.5 log2(e) 2^e of the frame in column lane & 15 of block cb
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[cb][s] = fh[(static_cast<size_t>(fb0 + cb) * KS + s) * 64 + lane];
        kap[cb] = ldexpf(0.721347520f, a.frameExp[frame0 + 16 * cb + (lane & 15)]);
    }
#pragma unroll
    for (int cb = 0; cb < NF; ++cb) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if constexpr (NF == 8)
                asm volatile("" : "+a"(B[cb][s]));
            else
                asm volatile("" ::"v"(B[cb][s]));
        }
        asm volatile("" ::"v"(kap[cb]));
    }
    // the tile array is padded by kTilePad >= 4 tiles: prefetching past T1 stays in bounds
    f16x8 R0[KS], R1[KS], R2[KS], R3[KS];
    loadTile(T0, R0);
    loadTile(T0 + 1, R1);
    loadTile(T0 + 2, R2);
    loadTile(T0 + 3, R3);

    const uint32_t kmask = BEST ? (1u << a.tileBits) - 1u : 0u;  // scores only: untagged values
    uint32_t       vmask = ~kmask;
    asm volatile("" : "+v"(vmask));

    uint32_t   best[NF][2];
    float      S[NF][2], Rf[NF];
    const auto resetBest = [&]() {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            Rf[cb] = 1e30f;  // no reference yet: the first tile re-bases it
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                best[cb][h] = 0xffffffffu;
                S[cb][h]    = 0.0f;
            }
        }
    };
    uint32_t m = m0, tBeg = T0, tEnd = m0 < m1 ? mixTileOff[m0 + 1] : T0;
    resetBest();
    const auto emit = [&]() {
#pragma unroll
        for (int h = 0; h < NH; ++h)
            emitMixtureSplitSum<BEST>(a, *reinterpret_cast<const uint32_t(*)[4][2]>(&best[4 * h]),
                                      *reinterpret_cast<const float(*)[4][2]>(&S[4 * h]),
                                      *reinterpret_cast<const float(*)[4]>(&Rf[4 * h]), m, frame0 + 64u * h, lane, g,
                                      kmask);
    };
    const auto advance = [&](uint32_t tNext) {
        ++m;
        tBeg = tNext;
        tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        while (m < m1 && tEnd == tNext) {
            emit();
            ++m;
            tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        }
    };
    // after the epilogue of the tile that ends at tNext
    const auto finish = [&](uint32_t tNext) {
        if (tNext == tEnd) {
            emit();
            resetBest();
            advance(tNext);
        }
    };

    // keys + min of tile tPrev (values prev) and the re-base test, beside MFMA k-steps [0, KH) into cur
    const auto firstHalf = [&](const f16x8(&A)[KS], f32x4(&cur)[NF], const f32x4(&prev)[NF], uint32_t tPrev) -> bool {
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
            cur[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < KH; ++s)
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                cur[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s], B[cb][s], cur[cb], 0, 0, 0);
        const uint32_t tl = tPrev - tBeg;
        uint32_t       tag[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            tag[r] = (tl << 2) | static_cast<uint32_t>(r);
            asm("" : "+s"(tag[r]));  // opaque: one v_and_or_b32 per key
        }
        bool reb = false;
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            // scores only: the minimum serves the re-base test alone, on the values' own bits (no tag)
            const uint32_t k0 = BEST ? (__float_as_uint(prev[cb][0]) & vmask) | tag[0] : __float_as_uint(prev[cb][0]);
            const uint32_t k1 = BEST ? (__float_as_uint(prev[cb][1]) & vmask) | tag[1] : __float_as_uint(prev[cb][1]);
            const uint32_t k2 = BEST ? (__float_as_uint(prev[cb][2]) & vmask) | tag[2] : __float_as_uint(prev[cb][2]);
            const uint32_t k3 = BEST ? (__float_as_uint(prev[cb][3]) & vmask) | tag[3] : __float_as_uint(prev[cb][3]);
            best[cb][0]       = umin3(best[cb][0], k0, k1);
            best[cb][1]       = umin3(best[cb][1], k2, k3);
            const float vmin  = __uint_as_float(BEST ? min(best[cb][0], best[cb][1]) & vmask : min(best[cb][0], best[cb][1]));
            reb               = reb || __builtin_fmaf(vmin, -kap[cb], Rf[cb]) > 64.0f;
        }
        constexpr int kM1 = KH * NF;
        if constexpr (kM1 > 0) {
#pragma unroll
            for (int i = 0; i < kM1; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);  // VALU
            }
        }
        return reb;
    };
    // the exponentials and sums of tile tPrev, beside MFMA k-steps [KH, KS) into cur
    const auto secondHalf = [&](const f16x8(&A)[KS], f32x4(&cur)[NF], const f32x4(&prev)[NF]) {
#pragma unroll
        for (int s = KH; s < KS; ++s)
#pragma unroll
            for (int cb = 0; cb < NF; ++cb)
                cur[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s], B[cb][s], cur[cb], 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                S[cb][h] += __builtin_amdgcn_exp2f(__builtin_fmaf(prev[cb][2 * h], -kap[cb], Rf[cb])) +
                            __builtin_amdgcn_exp2f(__builtin_fmaf(prev[cb][2 * h + 1], -kap[cb], Rf[cb]));
#pragma unroll
        for (int i = 0; i < (KS - KH) * NF; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // VALU
        }
    };
    const auto rebase = [&]() {  // uniform: new reference R = kap * (best value so far)
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            const float nr = kap[cb] * __uint_as_float(min(best[cb][0], best[cb][1]) & vmask);
            const float f  = __builtin_amdgcn_exp2f(nr - Rf[cb]);
            Rf[cb]         = nr;
            S[cb][0] *= f;
            S[cb][1] *= f;
        }
    };
    // step: MFMAs of the tile in A into cur beside the epilogue of tile tPrev (prev); then its emit
    const auto step = [&](const f16x8(&A)[KS], f32x4(&cur)[NF], const f32x4(&prev)[NF], uint32_t tPrev) {
        if (__builtin_amdgcn_ballot_w64(firstHalf(A, cur, prev, tPrev)) != 0)
            rebase();
        secondHalf(A, cur, prev);
    };
    // the last tile's epilogue (no MFMAs left to issue beside it)
    const auto drain = [&](const f32x4(&prev)[NF], uint32_t tPrev) {
        const uint32_t tl = tPrev - tBeg;
        bool           reb = false;
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            uint32_t k[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                k[r] = BEST ? (__float_as_uint(prev[cb][r]) & vmask) | ((tl << 2) | static_cast<uint32_t>(r))
                            : __float_as_uint(prev[cb][r]);
            best[cb][0]      = umin3(best[cb][0], k[0], k[1]);
            best[cb][1]      = umin3(best[cb][1], k[2], k[3]);
            const float vmin = __uint_as_float(min(best[cb][0], best[cb][1]) & vmask);
            reb              = reb || __builtin_fmaf(vmin, -kap[cb], Rf[cb]) > 64.0f;
        }
        if (__builtin_amdgcn_ballot_w64(reb) != 0)
            rebase();
#pragma unroll
        for (int cb = 0; cb < NF; ++cb)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                S[cb][h] += __builtin_amdgcn_exp2f(__builtin_fmaf(prev[cb][2 * h], -kap[cb], Rf[cb])) +
                            __builtin_amdgcn_exp2f(__builtin_fmaf(prev[cb][2 * h + 1], -kap[cb], Rf[cb]));
        finish(tPrev + 1);
    };

    while (m < m1 && tEnd == T0) {  // mixtures without tiles at the start of the chunk
        emit();
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T0;
    }
    if (T0 < T1) {
        // T1 - T0 is even: after the first tile, whole groups of four steps, then one or three more
        f32x4 accX[NF], accY[NF];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            accX[cb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < KS; ++s)
                accX[cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(R0[s], B[cb][s], accX[cb], 0, 0, 0);
        }
        loadTile(T0 + 4, R0);
        uint32_t t = T0;  // tile whose values are in accX
        for (; t + 4 < T1; t += 4) {
            step(R1, accY, accX, t);
            loadTile(t + 5, R1);
            finish(t + 1);
            step(R2, accX, accY, t + 1);
            loadTile(t + 6, R2);
            finish(t + 2);
            step(R3, accY, accX, t + 2);
            loadTile(t + 7, R3);
            finish(t + 3);
            step(R0, accX, accY, t + 3);
            loadTile(t + 8, R0);
            finish(t + 4);
        }
        // T1 - 1 - t is 1 or 3
        step(R1, accY, accX, t);
        finish(t + 1);
        if (t + 2 < T1) {
            step(R2, accX, accY, t + 1);
            finish(t + 2);
            step(R3, accY, accX, t + 2);
            finish(t + 3);
            drain(accY, t + 3);
        }
        else {
            drain(accY, t + 1);
        }
    }
}

// ---------------------------------------------------------------------------
// diagonal-sum on 32-row tiles (v_mfma_f32_32x32x16_f16; round 6).  The sum's epilogue is VALU-bound: per
// value a key (v_and_or_b32), half a v_min3, and v_fma + v_exp_f32 + v_add_f32 for the exponential sum, about 23
// issue cycles, where diagonal-maximum needs 6.  A 16x16x32 MFMA holds the SIMD's vector issue for 8 of its 16
// cycles, a 32x32x16 one for 8 of its 32, so per unit of matrix work the 32-row shape leaves 1.5x the issue
// cycles to that epilogue (MI355X_MICROARCH.md, the issue-cost row).  Layout and keys are scoreSplit32's: a
// wave holds 4 column blocks of 32 frames (128 frames, f16 fragments in the AGPRs), lane l owns frame l & 31 of a
// block and rows (i & 3) + 8 (i >> 2) + 4 (l >> 5) in its accumulator registers i; keys carry (tile << 4 | i).
// Exponential sum (as scoreSplitSum): exp(-s_d) = exp(K0/2) 2^(-kap u_d) with kap = 0.5 log2(e) 2^e of the frame;
// per lane and block a reference R and S = sum 2^(R - kap u).  R follows the running minimum every tile without a
// branch (online rescale: R' = min(R, kap min u), S *= 2^(R' - R)), so every exponent is <= 0.  Padding rows carry
// a 2^29 constant bias (gmm_prepare.cc): their exponentials underflow to 0 and their keys never win.
// ---------------------------------------------------------------------------
template <bool BEST>
__device__ __forceinline__ void emitMixtureSplit32Sum(const SplitArgs& a, const uint32_t (&best)[2][2],
                                                      const float (&S)[2][2], const float (&R)[2], uint32_t m,
                                                      uint32_t frame0, int lane, uint32_t kmask) {
    uint32_t k[2];
    float    sum[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        k[b]   = min(best[b][0], best[b][1]);
        sum[b] = S[b][0] + S[b][1];
    }
    // lanes < 32 keep block 0, lanes >= 32 block 1; [0] from lane half h = 0 (rows 4h ..), [1] from h = 1
    const auto r  = __builtin_amdgcn_permlane32_swap(k[0], k[1], false, false);
    const auto rr = __builtin_amdgcn_permlane32_swap(__float_as_uint(R[0]), __float_as_uint(R[1]), false, false);
    const auto rs = __builtin_amdgcn_permlane32_swap(__float_as_uint(sum[0]), __float_as_uint(sum[1]), false, false);
    const uint32_t hi0 = r[0] & ~15u, hi1 = r[1] & ~15u;
    const uint32_t row0 = (r[0] & 3u) | ((r[0] & 12u) << 1), row1 = ((r[1] & 3u) | ((r[1] & 12u) << 1)) + 4u;
    const bool     take = BEST ? (hi1 < hi0 || (hi1 == hi0 && row1 < row0)) : r[1] < r[0];
    const uint32_t key  = take ? r[1] : r[0];
    const uint32_t row  = take ? row1 : row0;
    // merge the two halves' (R, S) on the smaller R
    const float ra = __uint_as_float(rr[0]), rb = __uint_as_float(rr[1]);
    const float sa = __uint_as_float(rs[0]), sb = __uint_as_float(rs[1]);
    const float d  = ra - rb;
    const float rf = fminf(ra, rb);
    const float sf = d <= 0.0f ? __builtin_fmaf(sb, __builtin_amdgcn_exp2f(d), sa)
                               : __builtin_fmaf(sa, __builtin_amdgcn_exp2f(-d), sb);

    const float kv   = __uint_as_float((key & ~kmask) | ((kmask + 1u) >> 1));
    const bool  none = !(kv < 1e37f);  // empty mixture: R stays 1e30, S = 0 -> +inf, as the reference
    // -log sum exp(-s_d) = R ln2 - K0/2 - ln S
    const float score = __fmul_rn(a.outScale, (rf - __builtin_amdgcn_logf(sf)) * 0.693147181f - 0.5f * a.offsetK0);
    const uint32_t idx = none ? 0xffffffffu : ((((key & kmask) >> 4) << 5) | row);
    const uint32_t mo  = m - a.mixBase;
    const uint32_t off = static_cast<uint32_t>(frame0 + lane) * 4u;
    const auto rsS = __builtin_amdgcn_make_buffer_rsrc(a.scores + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                      static_cast<int>(a.nFrames * 4u), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(score), rsS, off, 0, GMM_STORE_CPOL);
    if constexpr (BEST) {
        const auto rb_ = __builtin_amdgcn_make_buffer_rsrc(a.best + static_cast<size_t>(mo) * a.scoreStride, (short)0,
                                                          static_cast<int>(a.nFrames * 4u), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(idx, rb_, off, 0, GMM_STORE_CPOL);
    }
}

#ifndef GMM_SPLIT32_SUM_IL
#define GMM_SPLIT32_SUM_IL 6  // VALU per MFMA in the interleave of a step (6: -1.8 % against 10, 13 +2 %; profiles/r06/s14, s15)
#endif

template <int KS, bool BEST>
__global__ __launch_bounds__(64 * (kSplitFramesPerBlock / 128), 1) void scoreSplit32Sum(
        SplitArgs a, const uint32_t* __restrict__ mixTileOffArg) {
    typedef float f32x16 __attribute__((ext_vector_type(16)));
    const auto    mixTileOff = constTable(mixTileOffArg);
    constexpr int NB = 4, NH = 2;  // blocks of 32 frames; halves of 64 frames (one emit each)
    const int     lane = threadIdx.x & 63;
    const int     wave = threadIdx.x >> 6;
    uint32_t      chunk, ft;
    if (!mapBlock(a.nChunks, a.nFrameTiles, chunk, ft))
        return;
    const uint32_t frame0 = ft * kSplitFramesPerBlock + static_cast<uint32_t>(wave) * (32u * NB);
    const uint32_t fb0    = frame0 / 32u;
    const uint32_t m0 = a.chunkMixOff[chunk], m1 = a.chunkMixOff[chunk + 1];
    const uint32_t T0 = mixTileOff[m0], T1 = mixTileOff[m1];

    const f16x8* th       = static_cast<const f16x8*>(a.tileH);
    const auto   loadTile = [&](uint32_t tt, f16x8(&A)[KS]) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            A[s] = th[(static_cast<size_t>(tt) * KS + s) * 64 + lane];
    };
    const f16x8* fh = static_cast<const f16x8*>(a.frameH);
    f16x8        B[NB][KS];
    float        kap[NB];  // 0.5 log2(e) 2^e of this lane's frame in block b
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            B[b][s] = fh[(static_cast<size_t>(fb0 + b) * KS + s) * 64 + lane];
        kap[b] = ldexpf(0.721347520f, a.frameExp[frame0 + 32u * b + (static_cast<uint32_t>(lane) & 31u)]);
    }
    // frame operands complete before the tile prefetch, then pinned to the accumulator file
#pragma unroll
    for (int b = 0; b < NB; ++b) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
            asm volatile("" : "+a"(B[b][s]));
        asm volatile("" ::"v"(kap[b]));
    }
    f16x8 R0[KS], R1[KS];  // tiles t (even steps) and t + 1; the padded tile array keeps loads past T1 in bounds
    loadTile(T0, R0);
    loadTile(T0 + 1, R1);

    const uint32_t kmask = BEST ? (1u << a.tileBits) - 1u : 0u;  // scores only: untagged values
    uint32_t       vmask = ~kmask;
    asm volatile("" : "+v"(vmask));

    uint32_t   best[NB][2];  // slot 0: registers 0..7, slot 1: 8..15 (the key carries the register)
    float      S[NB][2], Rf[NB];
    const auto resetBest = [&]() {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            Rf[b]      = 1e30f;  // no reference yet: the first tile sets it (S = 0 * 2^-huge = 0)
            best[b][0] = best[b][1] = 0xffffffffu;
            S[b][0] = S[b][1] = 0.0f;
        }
    };
    const auto chain = [&](const f16x8(&A)[KS], f32x16(&acc)[NB]) __attribute__((always_inline)) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
            acc[b] = f32x16{};  // ||x'||^2 is in K: the chain starts from an inline 0
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int b = 0; b < NB; ++b)
                acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[s], B[b][s], acc[b], 0, 0, 0);
    };
    const auto epilogue = [&](const f32x16(&acc)[NB], uint32_t tl) __attribute__((always_inline)) {
        uint32_t tag[16];  // opaque SGPRs (one v_and_or_b32 per key)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            tag[i] = (tl << 4) | static_cast<uint32_t>(i);
            asm("" : "+s"(tag[i]));
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            uint32_t k[16];
#pragma unroll
            for (int i = 0; i < 16; ++i)
                k[i] = BEST ? (__float_as_uint(acc[b][i]) & vmask) | tag[i] : __float_as_uint(acc[b][i]);
#pragma unroll
            for (int h = 0; h < 2; ++h)
                best[b][h] = umin3(umin3(umin3(umin3(best[b][h], k[8 * h], k[8 * h + 1]), k[8 * h + 2], k[8 * h + 3]),
                                         k[8 * h + 4], k[8 * h + 5]),
                                   k[8 * h + 6], k[8 * h + 7]);
            // online rescale to the running minimum: every exponent below stays <= 0
            const float vmin = __uint_as_float(min(best[b][0], best[b][1]) & vmask);
            const float nr   = fminf(Rf[b], kap[b] * vmin);
            const float f    = __builtin_amdgcn_exp2f(nr - Rf[b]);
            Rf[b]            = nr;
            S[b][0] *= f;
            S[b][1] *= f;
#pragma unroll
            for (int i = 0; i < 16; ++i)
                S[b][i & 1] += __builtin_amdgcn_exp2f(__builtin_fmaf(acc[b][i], -kap[b], nr));
        }
    };

    uint32_t m = m0, tBeg = T0, tEnd = m0 < m1 ? mixTileOff[m0 + 1] : T0;
    resetBest();
    const auto emit = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int h = 0; h < NH; ++h)
            emitMixtureSplit32Sum<BEST>(a, *reinterpret_cast<const uint32_t(*)[2][2]>(&best[2 * h]),
                                        *reinterpret_cast<const float(*)[2][2]>(&S[2 * h]),
                                        *reinterpret_cast<const float(*)[2]>(&Rf[2 * h]), m, frame0 + 64u * h, lane,
                                        kmask);
    };
    const auto advance = [&](uint32_t tNext) __attribute__((always_inline)) {
        ++m;
        tBeg = tNext;
        tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        while (m < m1 && tEnd == tNext) {
            emit();
            ++m;
            tEnd = m < m1 ? mixTileOff[m + 1] : tNext;
        }
    };
    const auto finish = [&](uint32_t tNext) __attribute__((always_inline)) {
        if (tNext == tEnd) {
            emit();
            resetBest();
            advance(tNext);
        }
    };
    // MFMAs of the tile in A into cur beside the epilogue of tile tPrev (in prev)
    const auto step = [&](const f16x8(&A)[KS], f32x16(&cur)[NB], const f32x16(&prev)[NB], uint32_t tPrev)
            __attribute__((always_inline)) {
        chain(A, cur);
        epilogue(prev, tPrev - tBeg);
#pragma unroll
        for (int i = 0; i < NB * KS; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, GMM_SPLIT32_SUM_IL, 0);  // VALU
        }
    };

    while (m < m1 && tEnd == T0) {  // mixtures without tiles at the start of the chunk
        emit();
        ++m;
        tEnd = m < m1 ? mixTileOff[m + 1] : T0;
    }
    if (T0 < T1) {
        f32x16   accX[NB], accY[NB];
        uint32_t t = T0;
        chain(R0, accX);  // tile T0: nothing to finish beside it
        loadTile(t + 2, R0);
        t += 1;
        for (; t + 2 <= T1; t += 2) {
            step(R1, accY, accX, t - 1);
            loadTile(t + 2, R1);
            finish(t);
            step(R0, accX, accY, t);
            loadTile(t + 3, R0);
            finish(t + 1);
        }
        if (t < T1) {  // one more tile (in R1)
            step(R1, accY, accX, t - 1);
            finish(t);
            epilogue(accY, t - tBeg);
            finish(t + 1);
        }
        else {
            epilogue(accX, t - 1 - tBeg);
            finish(t);
        }
    }
}

}  // namespace dev

hipError_t launchPrepareFramesSplit(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesRead,
                                    uint32_t D, uint32_t rows, uint32_t kSteps, const float* isv, const float* centre,
                                    const float* dimScale,
                                    const int32_t* limbExp, void* frameH, float* frameXX, int32_t* frameExp,
                                    hipStream_t stream) {
    if (rows == 32)
        hipLaunchKernelGGL(dev::prepareFramesSplit<32>, dim3((nFramesRead + 7) / 8), dim3(256), 0, stream, frames,
                           nFrames, frameStride, nFramesRead, D, kSteps, isv, centre, dimScale, limbExp,
                           static_cast<dev::u32x4*>(frameH), frameXX, frameExp);
    else
        hipLaunchKernelGGL(dev::prepareFramesSplit<16>, dim3((nFramesRead + 7) / 8), dim3(256), 0, stream, frames,
                           nFrames, frameStride, nFramesRead, D, kSteps, isv, centre, dimScale, limbExp,
                           static_cast<dev::u32x4*>(frameH), frameXX, frameExp);
    return hipGetLastError();
}

hipError_t launchPrepareFramesSplitCov(const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nFramesRead,
                                       uint32_t D, uint32_t kSteps, const float* centre, const float* dimScale,
                                       const int32_t* limbExp, void* frameH, int32_t* frameExp, hipStream_t stream) {
    hipLaunchKernelGGL(dev::prepareFramesSplitCov, dim3((nFramesRead + 7) / 8), dim3(256), 0, stream, frames, nFrames,
                       frameStride, nFramesRead, D, kSteps, centre, dimScale, limbExp, static_cast<dev::u32x4*>(frameH),
                       frameExp);
    return hipGetLastError();
}

template <int KS>
static void launchSplitK(const SplitArgs& a, uint32_t grid, hipStream_t s) {
    if constexpr (splitWideFrames(KS) != 0) {
        if (!a.presel) {
            if (a.best)
                hipLaunchKernelGGL((dev::scoreSplitWide<KS, true>), dim3(grid), dim3(64), 0, s, a, a.mixTileOff);
            else
                hipLaunchKernelGGL((dev::scoreSplitWide<KS, false>), dim3(grid), dim3(64), 0, s, a, a.mixTileOff);
            return;
        }
    }
    if (a.presel) {  // preselection-batch-float: no best density; the waves' mask tables in dynamic LDS
        // the block's 256 frames = 4 tables of [clusters][16] words, whatever the waves
        const uint32_t lds = kSplitFramesPerBlock / 64u * a.nClusters * 64u;
        (void)allowDynamicLds(reinterpret_cast<const void*>(&dev::scoreSplit<KS, false, true>),
                              static_cast<int>(kSplitFramesPerBlock / 64u * 256u * 64u));
        hipLaunchKernelGGL((dev::scoreSplit<KS, false, true>), dim3(grid), dim3(kSplitFramesPerBlock / splitPreselNF(KS) * 4),
                           lds, s, a, a.mixTileOff);
    }
    else if (a.best)
        hipLaunchKernelGGL((dev::scoreSplit<KS, true, false>), dim3(grid), dim3(64 * kSplitMainWaves), 0, s, a,
                           a.mixTileOff);
    else
        hipLaunchKernelGGL((dev::scoreSplit<KS, false, false>), dim3(grid), dim3(64 * kSplitMainWaves), 0, s, a,
                           a.mixTileOff);
}

template <int KS>
static void launchSplit32K(const SplitArgs& a, uint32_t grid, hipStream_t s) {
    if (a.best)
        hipLaunchKernelGGL((dev::scoreSplit32<KS, true>), dim3(grid), dim3(64 * (kSplitFramesPerBlock / (32 * GMM_SPLIT32_NB))),
                           0, s, a, a.mixTileOff);
    else
        hipLaunchKernelGGL((dev::scoreSplit32<KS, false>), dim3(grid), dim3(64 * (kSplitFramesPerBlock / (32 * GMM_SPLIT32_NB))),
                           0, s, a, a.mixTileOff);
}

hipError_t launchScoreSplit(const SplitArgs& a, uint32_t rows, uint32_t kSteps16, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    if (a.presel && (rows != 16 || a.nClusters == 0 || a.nClusters > 256 || !a.selT || !a.tileClu))
        return hipErrorInvalidValue;  // the mask tables are laid out for 16-row tiles and <= 256 clusters
    if (rows == 32) {
        switch (kSteps16) {
            case 1: launchSplit32K<1>(a, grid, stream); break;
            case 2: launchSplit32K<2>(a, grid, stream); break;
            case 3: launchSplit32K<3>(a, grid, stream); break;
            case 4: launchSplit32K<4>(a, grid, stream); break;
            case 5: launchSplit32K<5>(a, grid, stream); break;
            case 6: launchSplit32K<6>(a, grid, stream); break;
            case 7: launchSplit32K<7>(a, grid, stream); break;
            case 8: launchSplit32K<8>(a, grid, stream); break;
            case 9: launchSplit32K<9>(a, grid, stream); break;
            case 10: launchSplit32K<10>(a, grid, stream); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
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

template <int KS>
static void launchSplitSumK(const SplitArgs& a, uint32_t grid, hipStream_t s) {
    if (a.best)
        hipLaunchKernelGGL((dev::scoreSplitSum<KS, true>), dim3(grid), dim3(kSplitFramesPerBlock / GMM_SPLIT_SUM_NF * 4), 0,
                           s, a, a.mixTileOff);
    else
        hipLaunchKernelGGL((dev::scoreSplitSum<KS, false>), dim3(grid), dim3(kSplitFramesPerBlock / GMM_SPLIT_SUM_NF * 4),
                           0, s, a, a.mixTileOff);
}

template <int KS>
static void launchSplit32SumK(const SplitArgs& a, uint32_t grid, hipStream_t s) {
    if (a.best)
        hipLaunchKernelGGL((dev::scoreSplit32Sum<KS, true>), dim3(grid), dim3(64 * (kSplitFramesPerBlock / 128)), 0, s, a,
                           a.mixTileOff);
    else
        hipLaunchKernelGGL((dev::scoreSplit32Sum<KS, false>), dim3(grid), dim3(64 * (kSplitFramesPerBlock / 128)), 0, s,
                           a, a.mixTileOff);
}

hipError_t launchScoreSplitSum(const SplitArgs& a, uint32_t rows, uint32_t kSteps16, hipStream_t stream) {
    const uint32_t grid = 8u * ((a.nChunks + 7u) / 8u) * a.nFrameTiles;
    if (grid == 0)
        return hipSuccess;
    if (rows == 32) {
        switch (kSteps16) {
            case 1: launchSplit32SumK<1>(a, grid, stream); break;
            case 2: launchSplit32SumK<2>(a, grid, stream); break;
            case 3: launchSplit32SumK<3>(a, grid, stream); break;
            case 4: launchSplit32SumK<4>(a, grid, stream); break;
            case 5: launchSplit32SumK<5>(a, grid, stream); break;
            case 6: launchSplit32SumK<6>(a, grid, stream); break;
            case 7: launchSplit32SumK<7>(a, grid, stream); break;
            case 8: launchSplit32SumK<8>(a, grid, stream); break;
            case 9: launchSplit32SumK<9>(a, grid, stream); break;
            case 10: launchSplit32SumK<10>(a, grid, stream); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    switch (kSteps16) {
        case 1: launchSplitSumK<1>(a, grid, stream); break;
        case 2: launchSplitSumK<2>(a, grid, stream); break;
        case 3: launchSplitSumK<3>(a, grid, stream); break;
        case 4: launchSplitSumK<4>(a, grid, stream); break;
        case 5: launchSplitSumK<5>(a, grid, stream); break;
        case 6: launchSplitSumK<6>(a, grid, stream); break;
        case 7: launchSplitSumK<7>(a, grid, stream); break;
        case 8: launchSplitSumK<8>(a, grid, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rasr_gmm
