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
// scorer
// ---------------------------------------------------------------------------
template <int NF, int KS>
__global__ __launch_bounds__(256, GMM_SPLIT_MIN_WAVES) void scoreSplit(SplitArgs a) {
    static_assert(NF == 4 || NF == 8, "NF");
    constexpr int NPL  = NF / 4;
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
    const auto     key   = [&](float v, uint32_t tl) { return __uint_as_float((__float_as_uint(v) & ~tmask) | tl); };

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

        float    v[NF];
        uint32_t vi[NF];
#pragma unroll
        for (int cb = 0; cb < NF; ++cb) {
            v[cb]  = 3.40282347e+38f;
            vi[cb] = 0xffffffffu;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t bits = __float_as_uint(best[cb][r]);
                const float    val  = __uint_as_float(bits & ~tmask);
                if (!(val < 1e37f))  // no finite candidate in this row slot
                    continue;
                lexMin(v[cb], vi[cb], val, (bits & tmask) * 16u + 4u * g + r);
            }
        }
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
            float score;
            if (ki == 0xffffffffu) {  // no density: bestScore stays Core::Type<Score>::max
                score = a.flavor == 2 ? 0.5f * 3.40282347e+38f : 3.40282347e+38f;
            }
            else {
                const float scaled = ldexpf(kv, a.frameExp[f]);
                const float total  = a.offsetK0 != 0.0f ? __fsub_rn(scaled, a.offsetK0) : scaled;
                score              = a.flavor == 2 ? 0.5f * total : (total < 3.40282347e+38f ? 0.5f * total : total);
            }
            if (a.outScale != 1.0f)
                score = __fmul_rn(a.outScale, score);
            const size_t o = static_cast<size_t>(mo) * a.scoreStride + f;
            a.scores[o]    = score;
            if (a.best)
                a.best[o] = ki;
        }
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

template <int KS>
static void launchSplitK(const SplitArgs& a, uint32_t grid, hipStream_t s) {
    hipLaunchKernelGGL((dev::scoreSplit<kSplitNF, KS>), dim3(grid), dim3(256), 0, s, a);
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
