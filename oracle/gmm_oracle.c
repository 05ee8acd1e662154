/*
 * gmm_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port").
 * See gmm_oracle.h for scope and the PARITY UNPINNED status.
 *
 * Build (oracle/Makefile): gcc -std=gnu99 -O2 -ffast-math -msse3 -funsigned-char
 * i.e. the reference's own flags (config/cc-gcc.make:26-29, config/proc-x86_64.make:13-20,31),
 * so every floating-point expression below is compiled under the same
 * transformations as the reference expression it restates.  Expressions are
 * written in the reference's operand order and types on purpose.
 */
#define _GNU_SOURCE
#include "gmm_oracle.h"

#include <emmintrin.h>
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* scalar building blocks                                                     */
/* ------------------------------------------------------------------------- */

/* inverseSquareRoot<VarianceType>::operator() -- src/Mm/Utilities.hh:87-91:
 *   return (T)1 / (T)sqrt(x);
 * `sqrt` resolves to ::sqrt(double) (only /usr/include/math.h is reachable from
 * src/Mm/CovarianceFeatureScorerElement.cc); GCC narrows (float)sqrt((double)x)
 * to sqrtf and, under -ffast-math, expands 1.0f/sqrtf(x) to rsqrtss + one
 * Newton-Raphson step.  Same source expression, same flags => same instructions. */
float orc_inverse_sqrt(float x) {
    return (float)1 / (float)sqrt(x);
}

/* quantize<f32,u8>::operator() -- src/Mm/Utilities.hh:179-191:
 *   offset = (int)round((255 + 0 + 1) / 2) = 128;  clip((int)round(x) + offset) to [0,255] */
uint8_t orc_quantize(float x) {
    static const int offset = 128;
    int              v      = (int)round(x) + offset;
    if (v < 0)
        v = 0;
    if (v > 255)
        v = 255;
    return (uint8_t)v;
}

/* gaussLogNormFactor(begin,end) -- src/Mm/Utilities.hh:55-76:
 *   (double)n * log((double)2*M_PI) + sum_i log(Core::abs(v_i))   [double accumulation]
 * Core::abs(float) returns float (src/Core/Utility.hh:119-121); log is ::log(double). */
double orc_gauss_log_norm(const float* v, uint32_t d) {
    double   result = 0;
    uint32_t i;
    for (i = 0; i < d; ++i)
        result += log(fabsf(v[i]));
    return (double)d * log((double)2 * M_PI) + result;
}

/* SimdGaussDiagonalMaximumFeatureScorer::quantizationScalingFactor -- SimdFeatureScorer.cc:128-133 */
float orc_quantization_scaling_factor(float min_value, float max_value) {
    int   quantizedIntervalSize = (int)255 - (int)0; /* Core::Type<u8>::max - min (Core/Types.hh:78-79) */
    float a                     = fabsf(min_value);
    float b                     = fabsf(max_value);
    float intervalSize          = 2 * (a < b ? b : a);
    return (float)quantizedIntervalSize / (1.25 * intervalSize);
}

/* SimdFeatureScorer.cc:96  scaledMinus2LogWeight = scalingSquared_ * -2 * logWeight  (Weight = f64)
 * passed as `Score` (f32) to createDensityElement, IntelOptimization.cc:47:
 *   constantWeight_ = (s32)(scaledMinus2LogWeight + logNormalizationFactor())          */
static float orc_scaled_minus2_log_weight(float scaling_squared, double log_weight) {
    double w = scaling_squared * -2 * log_weight;
    return (float)w;
}
int32_t orc_constant_weight(float scaling_squared, double log_weight, float log_norm_scaled) {
    float w = orc_scaled_minus2_log_weight(scaling_squared, log_weight);
    return (int32_t)(w + log_norm_scaled);
}

/* SimdFeatureScorer.cc:142   result.score = 0.5 * quantizedResult.first / scalingSquared_; (Score = f32) */
float orc_simd_final_score(int32_t q, float scaling_squared) {
    return (float)(0.5 * q / scaling_squared);
}

/* BatchFeatureScorer.cc:376   *c = static_cast<s32>(logNormFactor - scale_ * mixture.logWeight(dns)); */
int32_t orc_batch_int_constant(float log_norm_scaled, float scale, double log_weight) {
    return (int32_t)(log_norm_scaled - scale * log_weight);
}

/* BatchFeatureScorer.cc:468   *result = static_cast<f32>(best) / scale_; */
float orc_batch_int_final_score(int32_t best, float scale) {
    return (float)best / scale;
}

/* GaussDiagonalMaximumFeatureScorer::distance, SSE3 branch -- GDMFS.cc:144-181
 * (the reference is built with -msse3, so __SSE3__ is defined). */
typedef float v4sf __attribute__((vector_size(16)));
float orc_float_distance(const float* feature, const float* mean, const float* isv, uint32_t d) {
    uint32_t cmp     = 0;
    float    result  = 0;
    float    df;
    v4sf     sum     = {0, 0, 0, 0};
    uint32_t eff_dim = d & (~3u);
    while (cmp < eff_dim) {
        v4sf m, f, s, t;
        memcpy(&m, mean + cmp, 16);
        memcpy(&f, feature + cmp, 16);
        memcpy(&s, isv + cmp, 16);
        t = (m - f) * s;
        sum += t * t;
        cmp += 4u;
    }
    /* _mm_hadd_ps(sum,sum) lanes 0,1 = (s0+s1), (s2+s3); result += buffer[0] + buffer[1] */
    {
        float h0 = sum[0] + sum[1];
        float h1 = sum[2] + sum[3];
        result += h0 + h1;
    }
    switch (d - eff_dim) {
        case 3:
            df = (mean[cmp] - feature[cmp]) * isv[cmp];
            result += df * df;
            ++cmp;
            /* fall through */
        case 2:
            df = (mean[cmp] - feature[cmp]) * isv[cmp];
            result += df * df;
            ++cmp;
            /* fall through */
        case 1:
            df = (mean[cmp] - feature[cmp]) * isv[cmp];
            result += df * df;
    }
    return result;
}

/* ------------------------------------------------------------------------- */
/* threading helper: frames are independent (no cross-frame scorer state)      */
/* ------------------------------------------------------------------------- */
typedef void (*orc_frame_fn)(void* ctx, uint32_t t0, uint32_t t1);
typedef struct {
    orc_frame_fn fn;
    void*        ctx;
    uint32_t     t0, t1;
} orc_job;

static void* orc_job_main(void* p) {
    orc_job* j = (orc_job*)p;
    j->fn(j->ctx, j->t0, j->t1);
    return NULL;
}

static void orc_parallel_frames(orc_frame_fn fn, void* ctx, uint32_t n_frames, int n_threads) {
    if (n_threads <= 1 || n_frames < 2) {
        fn(ctx, 0, n_frames);
        return;
    }
    if ((uint32_t)n_threads > n_frames)
        n_threads = (int)n_frames;
    pthread_t* th   = (pthread_t*)malloc(sizeof(pthread_t) * n_threads);
    orc_job*   jobs = (orc_job*)malloc(sizeof(orc_job) * n_threads);
    int        i;
    for (i = 0; i < n_threads; ++i) {
        jobs[i].fn  = fn;
        jobs[i].ctx = ctx;
        jobs[i].t0  = (uint32_t)((uint64_t)n_frames * i / n_threads);
        jobs[i].t1  = (uint32_t)((uint64_t)n_frames * (i + 1) / n_threads);
        pthread_create(&th[i], NULL, orc_job_main, &jobs[i]);
    }
    for (i = 0; i < n_threads; ++i)
        pthread_join(th[i], NULL);
    free(th);
    free(jobs);
}

/* ------------------------------------------------------------------------- */
/* SIMD-diagonal-maximum                                                       */
/* ------------------------------------------------------------------------- */

/* FeatureScorerIntelOptimization::multiplyAndQuantize -- IntelOptimization.cc:50-67
 * r[k] = quantize(x[k] * y[k]), zero padded to optimalVectorSize (BlockSize 16, IntelOptimization.hh:51-58) */
static void orc_multiply_and_quantize(const float* x, const float* y, uint32_t d, uint32_t dp, uint8_t* r) {
    uint32_t k;
    for (k = 0; k < d; ++k)
        r[k] = orc_quantize(x[k] * y[k]);
    for (; k < dp; ++k)
        r[k] = 0;
}

int orc_simd_prepare(const orc_mixture_set* ms, orc_simd_model* out) {
    const uint32_t D  = ms->dimension;
    const uint32_t Dp = (D + 15u) / 16u * 16u;
    const uint32_t C  = ms->n_covariances;
    uint32_t       c, k, i, m;
    memset(out, 0, sizeof(*out));
    out->dimension        = D;
    out->padded_dimension = Dp;
    out->n_covariances    = C;
    out->n_entries        = ms->mixture_offsets[ms->n_mixtures];
    out->isv              = (float*)malloc(sizeof(float) * C * D);
    out->log_norm         = (float*)malloc(sizeof(float) * C);

    /* init(): covarianceTable_[i] = *covariance(i)  -- SimdFeatureScorer.cc:64-67,
     * CovarianceFeatureScorerElement.cc:20-38 */
    for (c = 0; c < C; ++c) {
        const float* var = ms->variances + (size_t)c * D;
        for (k = 0; k < D; ++k) {
            if (!(var[k] > 0))
                return -1; /* require(checkDiagonal(diagonal)) */
            out->isv[(size_t)c * D + k] = orc_inverse_sqrt(var[k]);
        }
        out->log_norm[c] = (float)orc_gauss_log_norm(var, D);
    }

    /* getScaling -- SimdFeatureScorer.cc:106-126: bounds of mean*isv over all densities */
    {
        float minMean = -(-FLT_MAX); /* Core::Type<MeanType>::max */
        float maxMean = -FLT_MAX;    /* Core::Type<MeanType>::min (Core/Types.hh:146-147) */
        for (i = 0; i < ms->n_densities; ++i) {
            const float* mean = ms->means + (size_t)ms->density_mean[i] * D;
            const float* isv  = out->isv + (size_t)ms->density_covariance[i] * D;
            for (k = 0; k < D; ++k) {
                float dividedMean = mean[k] * isv[k];
                minMean           = minMean < dividedMean ? minMean : dividedMean;
                maxMean           = maxMean < dividedMean ? dividedMean : maxMean;
            }
        }
        out->scaling = orc_quantization_scaling_factor(minMean, maxMean);
    }
    out->scaling_squared             = out->scaling * out->scaling;
    out->inverse_quantization_factor = 0.5 / out->scaling_squared;

    /* covarianceTable_[i].scale(scaling) -- CovarianceFeatureScorerElement.cc:45-51 */
    for (c = 0; c < C; ++c) {
        for (k = 0; k < D; ++k)
            out->isv[(size_t)c * D + k] = out->isv[(size_t)c * D + k] * out->scaling;
        out->log_norm[c] *= out->scaling * out->scaling;
    }

    /* buildMixtureTable -- SimdFeatureScorer.cc:81-104 */
    out->prepared_mean    = (uint8_t*)malloc((size_t)out->n_entries * Dp);
    out->constant_weight  = (int32_t*)malloc(sizeof(int32_t) * out->n_entries);
    out->entry_covariance = (uint32_t*)malloc(sizeof(uint32_t) * out->n_entries);
    for (m = 0; m < ms->n_mixtures; ++m) {
        uint32_t e;
        for (e = ms->mixture_offsets[m]; e < ms->mixture_offsets[m + 1]; ++e) {
            uint32_t     dns  = ms->mixture_densities[e];
            uint32_t     cov  = ms->density_covariance[dns];
            const float* mean = ms->means + (size_t)ms->density_mean[dns] * D;
            out->entry_covariance[e] = cov;
            orc_multiply_and_quantize(mean, out->isv + (size_t)cov * D, D, Dp,
                                      out->prepared_mean + (size_t)e * Dp);
            out->constant_weight[e] =
                    orc_constant_weight(out->scaling_squared, ms->mixture_log_weights[e], out->log_norm[cov]);
        }
    }
    return 0;
}

void orc_simd_free(orc_simd_model* m) {
    free(m->isv);
    free(m->log_norm);
    free(m->prepared_mean);
    free(m->constant_weight);
    free(m->entry_covariance);
    memset(m, 0, sizeof(*m));
}

void orc_simd_quantize_frame(const orc_simd_model* m, const float* x, uint8_t* out) {
    uint32_t c;
    for (c = 0; c < m->n_covariances; ++c)
        orc_multiply_and_quantize(x, m->isv + (size_t)c * m->dimension, m->dimension, m->padded_dimension,
                                  out + (size_t)c * m->padded_dimension);
}

/* SSE2L2NormCodeGenerator::run -- SSE2CodeGenerator.cc:324-374 (JIT): per 16-byte block
 * |a-b| = psubusb(a,b) | psubusb(b,a); punpck{l,h}bw with zero; pmaddwd; paddd; horizontal add. */
static inline int orc_l2norm_u8(const uint8_t* a, const uint8_t* b, uint32_t dp) {
    __m128i  sum  = _mm_setzero_si128();
    __m128i  zero = _mm_setzero_si128();
    uint32_t o;
    for (o = 0; o < dp; o += 16) {
        __m128i x  = _mm_loadu_si128((const __m128i*)(a + o));
        __m128i y  = _mm_loadu_si128((const __m128i*)(b + o));
        __m128i d  = _mm_or_si128(_mm_subs_epu8(x, y), _mm_subs_epu8(y, x));
        __m128i lo = _mm_unpacklo_epi8(d, zero);
        __m128i hi = _mm_unpackhi_epi8(d, zero);
        sum        = _mm_add_epi32(sum, _mm_madd_epi16(lo, lo));
        sum        = _mm_add_epi32(sum, _mm_madd_epi16(hi, hi));
    }
    sum = _mm_add_epi32(sum, _mm_shuffle_epi32(sum, _MM_SHUFFLE(1, 0, 3, 2)));
    sum = _mm_add_epi32(sum, _mm_shuffle_epi32(sum, _MM_SHUFFLE(2, 3, 0, 1)));
    return _mm_cvtsi128_si32(sum);
}

typedef struct {
    const orc_simd_model*  m;
    const orc_mixture_set* ms;
    const float*           frames;
    uint32_t               n_frames, frame_stride;
    float*                 scores;
    uint32_t*              best;
    int32_t*               raw;
} orc_simd_ctx;

static void orc_simd_frames(void* p, uint32_t t0, uint32_t t1) {
    const orc_simd_ctx*   x  = (const orc_simd_ctx*)p;
    const orc_simd_model* m  = x->m;
    const uint32_t        Dp = m->padded_dimension;
    uint8_t* q = (uint8_t*)malloc((size_t)m->n_covariances * Dp);
    uint32_t t, e;
    for (t = t0; t < t1; ++t) {
        /* Context::Context -- SimdFeatureScorer.cc:22-35 */
        orc_simd_quantize_frame(m, x->frames + (size_t)t * x->frame_stride, q);
        for (e = 0; e < x->ms->n_mixtures; ++e) {
            /* quantizedScore -- SimdFeatureScorer.cc:158-176 */
            int      minScore    = 2147483647;  /* Core::Type<int>::max */
            uint64_t bestDensity = UINT64_MAX;  /* Core::Type<size_t>::max */
            uint32_t b = x->ms->mixture_offsets[e], en = x->ms->mixture_offsets[e + 1], i;
            for (i = b; i < en; ++i) {
                int score = m->constant_weight[i] +
                            orc_l2norm_u8(m->prepared_mean + (size_t)i * Dp,
                                          q + (size_t)m->entry_covariance[i] * Dp, Dp);
                if (score < minScore) {
                    minScore    = score;
                    bestDensity = i - b;
                }
            }
            /* calculateScoreAndDensity -- SimdFeatureScorer.cc:135-145 */
            {
                size_t o = (size_t)e * x->n_frames + t;
                if (x->scores)
                    x->scores[o] = orc_simd_final_score(minScore, m->scaling_squared);
                if (x->best)
                    x->best[o] = (uint32_t)bestDensity; /* DensityInMixture (u32) */
                if (x->raw)
                    x->raw[o] = minScore;
            }
        }
    }
    free(q);
}

int orc_simd_score(const orc_simd_model* m, const orc_mixture_set* ms, const float* frames,
                   uint32_t n_frames, uint32_t frame_stride, float* scores, uint32_t* best_density,
                   int32_t* raw_min, int n_threads) {
    orc_simd_ctx x;
    x.m = m;
    x.ms = ms;
    x.frames = frames;
    x.n_frames = n_frames;
    x.frame_stride = frame_stride;
    x.scores = scores;
    x.best = best_density;
    x.raw = raw_min;
    orc_parallel_frames(orc_simd_frames, &x, n_frames, n_threads);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* diagonal-maximum (float)                                                    */
/* ------------------------------------------------------------------------- */

int orc_float_prepare(const orc_mixture_set* ms, float mixture_weight_scale, float gaussian_scale,
                      orc_float_model* out) {
    const uint32_t D = ms->dimension, C = ms->n_covariances;
    uint32_t       c, k, e;
    /* GaussDiagonalMaximumFeatureScorer ctor: gaussianScale_(std::sqrt(paramGaussianScale(c))) -- cc:51 */
    /* gaussianScale_ is a member set in the constructor and scale() squares the value it is passed, so
     * neither sees sqrt(g) * sqrt(g) (which gcc -ffast-math would fold to g): both go through memory */
    volatile float gsv  = (float)sqrt((double)gaussian_scale);
    const float    gs   = gsv;
    volatile float gs2v = gs * gs;
    const float    gs2  = gs2v;
    memset(out, 0, sizeof(*out));
    out->dimension     = D;
    out->n_covariances = C;
    out->n_entries     = ms->mixture_offsets[ms->n_mixtures];
    out->isv           = (float*)malloc(sizeof(float) * C * D);
    out->log_norm      = (float*)malloc(sizeof(float) * C);
    /* init -- cc:64-86 */
    for (c = 0; c < C; ++c) {
        const float* var = ms->variances + (size_t)c * D;
        for (k = 0; k < D; ++k) {
            if (!(var[k] > 0))
                return -1;
            out->isv[(size_t)c * D + k] = orc_inverse_sqrt(var[k]);
        }
        out->log_norm[c] = (float)orc_gauss_log_norm(var, D);
        /* covarianceTable_[i].scale(gaussianScale_): logNormalizationFactor_ *= factor * factor
         * (CovarianceFeatureScorerElement.cc:45-51).  Compiled by itself, with the reference's flags, that
         * function squares the factor first (x * (f * f)); written inline here, gcc -ffast-math would
         * reassociate it into (x * f) * f, so the square is formed separately. */
        for (k = 0; k < D; ++k)
            out->isv[(size_t)c * D + k] = out->isv[(size_t)c * D + k] * gs;
        out->log_norm[c] = out->log_norm[c] * gs2;
    }
    /* mixtureTable_[i] = *mixture(i); scale(mixtureWeightScale_) -- MixtureFeatureScorerElement.cc:21-33 */
    out->minus2_log_weight = (float*)malloc(sizeof(float) * out->n_entries);
    for (e = 0; e < out->n_entries; ++e) {
        float w                   = -2 * ms->mixture_log_weights[e];
        out->minus2_log_weight[e] = w * mixture_weight_scale;
    }
    return 0;
}

void orc_float_free(orc_float_model* m) {
    free(m->isv);
    free(m->log_norm);
    free(m->minus2_log_weight);
    memset(m, 0, sizeof(*m));
}

typedef struct {
    const orc_float_model* m;
    const orc_mixture_set* ms;
    const float*           frames;
    uint32_t               n_frames, frame_stride;
    float*                 scores;
    uint32_t*              best;
} orc_float_ctx;

static void orc_float_frames(void* p, uint32_t t0, uint32_t t1) {
    const orc_float_ctx*   x  = (const orc_float_ctx*)p;
    const orc_float_model* m  = x->m;
    const orc_mixture_set* ms = x->ms;
    const uint32_t         D  = m->dimension;
    uint32_t               t, e, i;
    for (t = t0; t < t1; ++t) {
        const float* f = x->frames + (size_t)t * x->frame_stride;
        for (e = 0; e < ms->n_mixtures; ++e) {
            /* calculateScoreAndDensity -- GaussDiagonalMaximumFeatureScorer.cc:116-142 */
            float    bestScore   = FLT_MAX;
            uint64_t bestDensity = UINT64_MAX;
            uint32_t b = ms->mixture_offsets[e], en = ms->mixture_offsets[e + 1];
            for (i = b; i < en; ++i) {
                uint32_t dns   = ms->mixture_densities[i];
                uint32_t cov   = ms->density_covariance[dns];
                double   score = (double)m->minus2_log_weight[i] + (double)m->log_norm[cov] +
                               (double)orc_float_distance(f, ms->means + (size_t)ms->density_mean[dns] * D,
                                                          m->isv + (size_t)cov * D, D);
                if (bestScore > score) {
                    bestScore   = score;
                    bestDensity = i - b;
                }
            }
            {
                size_t o = (size_t)e * x->n_frames + t;
                if (x->scores)
                    x->scores[o] = 0.5 * bestScore;
                if (x->best)
                    x->best[o] = (uint32_t)bestDensity;
            }
        }
    }
}

int orc_float_score(const orc_float_model* m, const orc_mixture_set* ms, const float* frames,
                    uint32_t n_frames, uint32_t frame_stride, float* scores, uint32_t* best_density,
                    int n_threads) {
    orc_float_ctx x;
    x.m = m;
    x.ms = ms;
    x.frames = frames;
    x.n_frames = n_frames;
    x.frame_stride = frame_stride;
    x.scores = scores;
    x.best = best_density;
    orc_parallel_frames(orc_float_frames, &x, n_frames, n_threads);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* diagonal-sum: GaussDiagonalSumFeatureScorer (GaussDiagonalMaximumFeatureScorer.cc:221-298)   */
/* ------------------------------------------------------------------------- */
static void orc_float_sum_frames(void* p, uint32_t t0, uint32_t t1) {
    const orc_float_ctx*   x  = (const orc_float_ctx*)p;
    const orc_float_model* m  = x->m;
    const orc_mixture_set* ms = x->ms;
    const uint32_t         D  = m->dimension;
    uint32_t               t, e, i, maxn = 1;
    float*                 sc;
    for (e = 0; e < ms->n_mixtures; ++e)
        if (ms->mixture_offsets[e + 1] - ms->mixture_offsets[e] > maxn)
            maxn = ms->mixture_offsets[e + 1] - ms->mixture_offsets[e];
    sc = (float*)malloc(sizeof(float) * maxn);  /* scores_ (cc:224, maximumNumberOfDensities) */
    for (t = t0; t < t1; ++t) {
        const float* f = x->frames + (size_t)t * x->frame_stride;
        for (e = 0; e < ms->n_mixtures; ++e) {
            uint32_t b = ms->mixture_offsets[e], n = ms->mixture_offsets[e + 1] - b;
            float    bestScore   = FLT_MAX;  /* Core::Type<Score>::max */
            uint64_t bestDensity = UINT64_MAX;
            float    sumExp      = 0;
            /* calculateScoresAndNumberOfDensities -- cc:238-261: Score (f32) arithmetic */
            for (i = 0; i < n; ++i) {
                uint32_t dns   = ms->mixture_densities[b + i];
                uint32_t cov   = ms->density_covariance[dns];
                float    score = m->minus2_log_weight[b + i] + m->log_norm[cov] +
                              orc_float_distance(f, ms->means + (size_t)ms->density_mean[dns] * D,
                                                 m->isv + (size_t)cov * D, D);
                sc[i] = (float)(0.5 * score);
            }
            /* calculateScoreAndDensity -- cc:263-286 */
            for (i = 0; i < n; ++i)
                if (bestScore > sc[i]) {
                    bestScore   = sc[i];
                    bestDensity = i;
                }
            for (i = 0; i < n; ++i)
                sumExp += expf(bestScore - sc[i]);
            {
                size_t o = (size_t)e * x->n_frames + t;
                if (x->scores)
                    x->scores[o] = bestScore - logf(sumExp);
                if (x->best)
                    x->best[o] = (uint32_t)bestDensity;
            }
        }
    }
    free(sc);
}

int orc_float_sum_score(const orc_float_model* m, const orc_mixture_set* ms, const float* frames,
                        uint32_t n_frames, uint32_t frame_stride, float* scores, uint32_t* best_density,
                        int n_threads) {
    orc_float_ctx x;
    x.m = m;
    x.ms = ms;
    x.frames = frames;
    x.n_frames = n_frames;
    x.frame_stride = frame_stride;
    x.scores = scores;
    x.best = best_density;
    orc_parallel_frames(orc_float_sum_frames, &x, n_frames, n_threads);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* batch-diagonal-maximum-int                                                  */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint32_t       D, Dp;
    float          scale_;       /* 2 * s^2 (BatchFeatureScorer.cc:356)        */
    float*         variance;     /* isv * s, padded                           */
    uint8_t*       means;        /* entries x Dp                               */
    int32_t*       constants;
    const orc_mixture_set* ms;
    const float*   frames;
    uint32_t       n_frames, frame_stride;
    float*         scores;
    /* preselection-batch-int (ClusterIterator, BatchFeatureScorer.cc:500-529): NULL = every density */
    const uint8_t* entry_cluster;  /* clusterIndexForDensity_ [entries]              */
    const uint8_t* selection;      /* activeClusters_ [n_frames][n_clusters]          */
    uint32_t       n_clusters;
} orc_bint_ctx;

static void orc_bint_frames(void* p, uint32_t t0, uint32_t t1) {
    const orc_bint_ctx* x = (const orc_bint_ctx*)p;
    uint8_t* feature = (uint8_t*)malloc(x->Dp);
    uint32_t t, e, i, k;
    for (t = t0; t < t1; ++t) {
        /* setFeature -- cc:384-390: memset 0, transform MultiplyAndQuantize */
        const float* f = x->frames + (size_t)t * x->frame_stride;
        memset(feature, 0, x->Dp);
        for (k = 0; k < x->D; ++k)
            feature[k] = orc_quantize(f[k] * x->variance[k]);
        for (e = 0; e < x->ms->n_mixtures; ++e) {
            /* fillScoreCacheTpl -- cc:423-470 */
            int32_t best = 2147483647;
            for (i = x->ms->mixture_offsets[e]; i < x->ms->mixture_offsets[e + 1]; ++i) {
                if (x->selection && !x->selection[(size_t)t * x->n_clusters + x->entry_cluster[i]])
                    continue; /* selector.value() false -- cc:439 */
                int32_t tmp = orc_l2norm_u8(x->means + (size_t)i * x->Dp, feature, x->Dp);
                tmp += x->constants[i];
                if (tmp < best)
                    best = tmp;
            }
            x->scores[(size_t)e * x->n_frames + t] = orc_batch_int_final_score(best, x->scale_);
        }
    }
    free(feature);
}

int orc_batch_int_score(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                        uint32_t frame_stride, float* scores, int n_threads) {
    return orc_batch_int_score_sel(ms, frames, n_frames, frame_stride, scores, n_threads, NULL, NULL, 0);
}

int orc_batch_int_score_sel(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                            uint32_t frame_stride, float* scores, int n_threads, const uint8_t* entry_cluster,
                            const uint8_t* selection, uint32_t n_clusters) {
    orc_bint_ctx x;
    uint32_t     k, i, m, D = ms->dimension;
    float        isv0[4096];
    float        logNorm;
    if (ms->n_covariances != 1 || D > 4096)
        return -1; /* criticalError("... only globally pooled variance") cc:341-343 */
    memset(&x, 0, sizeof(x));
    x.D  = D;
    x.Dp = (D + 15u) / 16u * 16u;
    x.variance = (float*)calloc(x.Dp, sizeof(float));
    for (k = 0; k < D; ++k) {
        if (!(ms->variances[k] > 0))
            return -1;
        isv0[k] = orc_inverse_sqrt(ms->variances[k]);
        x.variance[k] = isv0[k];
    }
    logNorm = (float)orc_gauss_log_norm(ms->variances, D);
    {
        /* quantizationScale -- cc:318-336 */
        float minMean = FLT_MAX, maxMean = -FLT_MAX;
        float scale, scaleSquared, logNormFactor;
        for (i = 0; i < ms->n_densities; ++i) {
            const float* mean = ms->means + (size_t)ms->density_mean[i] * D;
            for (k = 0; k < D; ++k) {
                float dividedMean = mean[k] * x.variance[k];
                minMean           = minMean < dividedMean ? minMean : dividedMean;
                maxMean           = maxMean < dividedMean ? dividedMean : maxMean;
            }
        }
        scale        = orc_quantization_scaling_factor(minMean, maxMean);
        scaleSquared = scale * scale;
        x.scale_     = 2.0 * scaleSquared;
        for (k = 0; k < x.Dp; ++k)
            x.variance[k] = x.variance[k] * scale;
        logNormFactor = logNorm * scaleSquared;
        x.means       = (uint8_t*)calloc((size_t)ms->mixture_offsets[ms->n_mixtures] * x.Dp, 1);
        x.constants   = (int32_t*)malloc(sizeof(int32_t) * ms->mixture_offsets[ms->n_mixtures]);
        for (m = 0; m < ms->n_mixtures; ++m) {
            uint32_t e;
            for (e = ms->mixture_offsets[m]; e < ms->mixture_offsets[m + 1]; ++e) {
                const float* mean = ms->means + (size_t)ms->density_mean[ms->mixture_densities[e]] * D;
                for (k = 0; k < D; ++k)
                    x.means[(size_t)e * x.Dp + k] = orc_quantize(mean[k] * x.variance[k]);
                x.constants[e] = orc_batch_int_constant(logNormFactor, x.scale_, ms->mixture_log_weights[e]);
            }
        }
    }
    x.ms = ms;
    x.frames = frames;
    x.n_frames = n_frames;
    x.frame_stride = frame_stride;
    x.scores = scores;
    x.entry_cluster = entry_cluster;
    x.selection = selection;
    x.n_clusters = n_clusters;
    orc_parallel_frames(orc_bint_frames, &x, n_frames, n_threads);
    free(x.variance);
    free(x.means);
    free(x.constants);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* batch-diagonal-maximum-float                                                */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint32_t D, Dp;
    float*   variance;   /* isv, padded with 0 */
    float*   means;      /* entries x Dp       */
    float*   constants;
    const orc_mixture_set* ms;
    const float* frames;
    uint32_t n_frames, frame_stride;
    float*   scores;
    /* preselection-batch-float (ClusterDensitySelection, BatchFeatureScorer.cc:265-289): NULL = all */
    const uint8_t* entry_cluster;
    const uint8_t* selection;
    uint32_t n_clusters;
    float    backoff;
} orc_bflt_ctx;

static void orc_bflt_frames(void* p, uint32_t t0, uint32_t t1) {
    const orc_bflt_ctx* x = (const orc_bflt_ctx*)p;
    float*   feature = (float*)malloc(sizeof(float) * x->Dp);
    uint32_t t, e, i, k;
    for (t = t0; t < t1; ++t) {
        const float* f = x->frames + (size_t)t * x->frame_stride;
        /* setFeature -- cc:137-142 */
        memset(feature, 0, sizeof(float) * x->Dp);
        for (k = 0; k < x->D; ++k)
            feature[k] = f[k] * x->variance[k];
        for (e = 0; e < x->ms->n_mixtures; ++e) {
            /* fillScoreCacheTpl -- cc:187-234 */
            float score = FLT_MAX;
            for (i = x->ms->mixture_offsets[e]; i < x->ms->mixture_offsets[e + 1]; ++i) {
                if (x->selection && !x->selection[(size_t)t * x->n_clusters + x->entry_cluster[i]])
                    continue; /* if (!selector(rp, dns)) continue; -- cc:206-207 */
                const float* mean = x->means + (size_t)i * x->Dp;
                v4sf s1 = {x->constants[i], 0, 0, 0}, s2 = {0, 0, 0, 0}, a, b, x1, x2, r;
                uint32_t d;
                for (d = 0; d < x->Dp; d += 8) {
                    memcpy(&a, mean + d, 16);
                    memcpy(&b, feature + d, 16);
                    x1 = a - b;
                    s1 = s1 + x1 * x1;
                    memcpy(&a, mean + d + 4, 16);
                    memcpy(&b, feature + d + 4, 16);
                    x2 = a - b;
                    s2 = s2 + x2 * x2;
                }
                s1 = s1 + s2;
                /* shuffle(1,0,3,2) + add, shuffle(2,3,0,1) + add -> lane 0 */
                r = (v4sf){s1[2], s1[3], s1[0], s1[1]};
                s1 = r + s1;
                r = (v4sf){s1[1], s1[0], s1[3], s1[2]};
                s1 = r + s1;
                score = score < s1[0] ? score : s1[0]; /* _mm_min_ps(load_ss(score), s1) lane 0 */
            }
            if (score < FLT_MAX)
                score *= 0.5;
            if (x->selection && score == FLT_MAX)
                score = x->backoff; /* BatchPreselectionFloatFeatureScorer::fillScoreCache, cc:282-288 */
            x->scores[(size_t)e * x->n_frames + t] = score;
        }
    }
    free(feature);
}

int orc_batch_float_score(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                          uint32_t frame_stride, float* scores, int n_threads) {
    return orc_batch_float_score_sel(ms, frames, n_frames, frame_stride, scores, n_threads, NULL, NULL, 0, 0.0f);
}

int orc_batch_float_score_sel(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                              uint32_t frame_stride, float* scores, int n_threads, const uint8_t* entry_cluster,
                              const uint8_t* selection, uint32_t n_clusters, float backoff) {
    orc_bflt_ctx x;
    uint32_t     k, m, D = ms->dimension;
    float        logNormFactor;
    if (ms->n_covariances != 1)
        return -1;
    memset(&x, 0, sizeof(x));
    x.D  = D;
    x.Dp = (D + 7u) / 8u * 8u; /* BlockSize 8 (cc:120) */
    x.variance = (float*)calloc(x.Dp, sizeof(float));
    for (k = 0; k < D; ++k) {
        if (!(ms->variances[k] > 0))
            return -1;
        x.variance[k] = orc_inverse_sqrt(ms->variances[k]);
    }
    logNormFactor = (float)orc_gauss_log_norm(ms->variances, D);
    x.means     = (float*)calloc((size_t)ms->mixture_offsets[ms->n_mixtures] * x.Dp, sizeof(float));
    x.constants = (float*)malloc(sizeof(float) * ms->mixture_offsets[ms->n_mixtures]);
    for (m = 0; m < ms->n_mixtures; ++m) {
        uint32_t e;
        for (e = ms->mixture_offsets[m]; e < ms->mixture_offsets[m + 1]; ++e) {
            const float* mean = ms->means + (size_t)ms->density_mean[ms->mixture_densities[e]] * D;
            for (k = 0; k < D; ++k)
                x.means[(size_t)e * x.Dp + k] = mean[k] * x.variance[k];
            /* cc:167  *c = logNormFactor - 2 * mixture.logWeight(dns); */
            x.constants[e] = logNormFactor - 2 * ms->mixture_log_weights[e];
        }
    }
    x.ms = ms;
    x.frames = frames;
    x.n_frames = n_frames;
    x.frame_stride = frame_stride;
    x.scores = scores;
    x.entry_cluster = entry_cluster;
    x.selection = selection;
    x.n_clusters = n_clusters;
    x.backoff = backoff;
    orc_parallel_frames(orc_bflt_frames, &x, n_frames, n_threads);
    free(x.variance);
    free(x.means);
    free(x.constants);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* helpers for known-answer tests                                              */
/* ------------------------------------------------------------------------- */
void orc_quantize_array(const float* x, uint32_t n, uint8_t* out) {
    uint32_t i;
    for (i = 0; i < n; ++i)
        out[i] = orc_quantize(x[i]);
}

/* BatchIntFeatureScorer::init tables (BatchFeatureScorer.cc:339-380): scale_, variance_, constants_ */
int orc_batch_int_prepare(const orc_mixture_set* ms, float* scale_out, float* variance_out, int32_t* constants_out) {
    uint32_t k, i, m, D = ms->dimension;
    float    minMean = FLT_MAX, maxMean = -FLT_MAX, scale, scaleSquared, scale_, logNormFactor;
    float*   variance;
    if (ms->n_covariances != 1)
        return -1;
    variance = (float*)malloc(sizeof(float) * D);
    for (k = 0; k < D; ++k)
        variance[k] = orc_inverse_sqrt(ms->variances[k]);
    for (i = 0; i < ms->n_densities; ++i) {
        const float* mean = ms->means + (size_t)ms->density_mean[i] * D;
        for (k = 0; k < D; ++k) {
            float dividedMean = mean[k] * variance[k];
            minMean           = minMean < dividedMean ? minMean : dividedMean;
            maxMean           = maxMean < dividedMean ? dividedMean : maxMean;
        }
    }
    scale        = orc_quantization_scaling_factor(minMean, maxMean);
    scaleSquared = scale * scale;
    scale_       = 2.0 * scaleSquared;
    for (k = 0; k < D; ++k)
        variance[k] = variance[k] * scale;
    logNormFactor = (float)orc_gauss_log_norm(ms->variances, D) * scaleSquared;
    for (m = 0; m < ms->n_mixtures; ++m) {
        uint32_t e;
        for (e = ms->mixture_offsets[m]; e < ms->mixture_offsets[m + 1]; ++e)
            constants_out[e] = orc_batch_int_constant(logNormFactor, scale_, ms->mixture_log_weights[e]);
    }
    *scale_out = scale_;
    memcpy(variance_out, variance, sizeof(float) * D);
    free(variance);
    return 0;
}

/* BatchFloatFeatureScorer::init / setFeature tables (BatchFeatureScorer.cc:144-170, 137-142):
 *   variance [Dp] (isv, 0-padded), means [entries][Dp] = mean * variance (f32), constants [entries] */
int orc_batch_float_tables(const orc_mixture_set* ms, float* variance_out, float* means_out, float* constants_out) {
    uint32_t k, m, D = ms->dimension, Dp = (ms->dimension + 7u) / 8u * 8u;
    float    logNormFactor;
    if (ms->n_covariances != 1)
        return -1;
    memset(variance_out, 0, sizeof(float) * Dp);
    for (k = 0; k < D; ++k)
        variance_out[k] = orc_inverse_sqrt(ms->variances[k]);
    logNormFactor = (float)orc_gauss_log_norm(ms->variances, D);
    memset(means_out, 0, sizeof(float) * (size_t)ms->mixture_offsets[ms->n_mixtures] * Dp);
    for (m = 0; m < ms->n_mixtures; ++m) {
        uint32_t e;
        for (e = ms->mixture_offsets[m]; e < ms->mixture_offsets[m + 1]; ++e) {
            const float* mean = ms->means + (size_t)ms->density_mean[ms->mixture_densities[e]] * D;
            for (k = 0; k < D; ++k)
                means_out[(size_t)e * Dp + k] = mean[k] * variance_out[k];
            constants_out[e] = logNormFactor - 2 * ms->mixture_log_weights[e];
        }
    }
    return 0;
}

/* BatchIntFeatureScorer::init / setFeature tables (BatchFeatureScorer.cc:339-390):
 *   variance [Dp] (isv * scale, 0-padded), means [entries][Dp] u8 (quantize(mean * variance)) */
int orc_batch_int_tables(const orc_mixture_set* ms, float* variance_out, uint8_t* means_out) {
    uint32_t k, m, D = ms->dimension, Dp = (ms->dimension + 15u) / 16u * 16u;
    float    scale_;
    int32_t* constants = (int32_t*)malloc(sizeof(int32_t) * (ms->mixture_offsets[ms->n_mixtures] + 1));
    memset(variance_out, 0, sizeof(float) * Dp);
    if (orc_batch_int_prepare(ms, &scale_, variance_out, constants) != 0) {
        free(constants);
        return -1;
    }
    free(constants);
    memset(means_out, 0, (size_t)ms->mixture_offsets[ms->n_mixtures] * Dp);
    for (m = 0; m < ms->n_mixtures; ++m) {
        uint32_t e;
        for (e = ms->mixture_offsets[m]; e < ms->mixture_offsets[m + 1]; ++e) {
            const float* mean = ms->means + (size_t)ms->density_mean[ms->mixture_densities[e]] * D;
            for (k = 0; k < D; ++k)
                means_out[(size_t)e * Dp + k] = orc_quantize(mean[k] * variance_out[k]);
        }
    }
    return 0;
}
