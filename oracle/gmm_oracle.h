/*
 * gmm_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of RASR's diagonal-covariance GMM feature scorers, used as the
 * parity checker for the MI355X scorer and as the CPU baseline ("port") in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * Nothing in rasr_amd/ links or calls it.
 *
 * PARITY STATUS: UNPINNED.  The reference hot path cannot be built in this
 * image without stand-ins for generated code (src/Core/Utility.hh:18 needs the
 * make-generated Modules.hh, src/Core/Configuration.cc:26 the bison-generated
 * ArithmeticExpressionParser.hh; bison is absent), and the reference holds no
 * tests, golden vectors or fixtures for src/Mm scorers.
 * The restatement follows the reference source line by line (citations below)
 * and is compiled with the reference's own flags (config/cc-gcc.make,
 * config/proc-x86_64.make: -O2 -ffast-math -msse3 -funsigned-char) so that
 * GCC applies the same floating-point transformations to the same expressions.
 *
 * Scorers restated (reference feature-scorer-type names, src/Mm/Module.cc:84-107):
 *   "SIMD-diagonal-maximum"          src/Mm/SimdFeatureScorer.cc
 *   "diagonal-maximum"               src/Mm/GaussDiagonalMaximumFeatureScorer.cc
 *   "batch-diagonal-maximum-int"     src/Mm/BatchFeatureScorer.cc:293-474
 *   "batch-diagonal-maximum-float"   src/Mm/BatchFeatureScorer.cc:120-234
 *
 * All score tables are mixture-major: scores[e * n_frames + t], the layout of
 * BatchFeatureScorerBase::scores_ (src/Mm/BatchFeatureScorer.hh:177-186).
 */
#ifndef GMM_ORACLE_H
#define GMM_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* In-memory Mm::MixtureSet (src/Mm/MixtureSet.hh:140-212). */
typedef struct {
    uint32_t        dimension;
    uint32_t        n_means;
    const float*    means;               /* n_means x dimension              */
    uint32_t        n_covariances;
    const float*    variances;           /* n_covariances x dimension, diag  */
    uint32_t        n_densities;
    const uint32_t* density_mean;        /* GaussDensity::meanIndex()        */
    const uint32_t* density_covariance;  /* GaussDensity::covarianceIndex()  */
    uint32_t        n_mixtures;
    const uint32_t* mixture_offsets;     /* n_mixtures + 1 (CSR)             */
    const uint32_t* mixture_densities;   /* Mixture::densityIndex(dns)       */
    const double*   mixture_log_weights; /* Mixture::logWeight(dns), f64     */
} orc_mixture_set;

/* ---- scalar building blocks (exported for known-answer tests) ---- */
float   orc_inverse_sqrt(float x);          /* Utilities.hh:87-91 under -ffast-math */
uint8_t orc_quantize(float x);              /* Utilities.hh:179-191 quantize<f32,u8> */
double  orc_gauss_log_norm(const float* v, uint32_t d); /* Utilities.hh:55-76 */
float   orc_quantization_scaling_factor(float min_value, float max_value); /* SimdFeatureScorer.cc:128-133 */
int32_t orc_constant_weight(float scaling_squared, double log_weight, float log_norm_scaled); /* cc:96 + IntelOptimization.cc:47 */
float   orc_simd_final_score(int32_t q, float scaling_squared);  /* SimdFeatureScorer.cc:142 */
int32_t orc_batch_int_constant(float log_norm_scaled, float scale, double log_weight);  /* BatchFeatureScorer.cc:376 */
float   orc_batch_int_final_score(int32_t best, float scale); /* BatchFeatureScorer.cc:468 */
float   orc_float_distance(const float* feature, const float* mean, const float* isv, uint32_t d); /* GDMFS.cc:144-218 */

/* ---- SIMD-diagonal-maximum (src/Mm/SimdFeatureScorer.cc) ---- */
typedef struct {
    uint32_t dimension, padded_dimension, n_covariances, n_entries;
    float    scaling;                      /* getScaling, cc:106-126           */
    float    scaling_squared;              /* cc:72                           */
    float    inverse_quantization_factor;  /* cc:73                           */
    float*   isv;                          /* C x D, after scale(s) cc:75-76  */
    float*   log_norm;                     /* C, after scale(s)               */
    uint8_t* prepared_mean;                /* n_entries x Dp (cc:81-104)       */
    int32_t* constant_weight;              /* n_entries                       */
    uint32_t* entry_covariance;            /* n_entries                       */
} orc_simd_model;

int  orc_simd_prepare(const orc_mixture_set* ms, orc_simd_model* out);
void orc_simd_free(orc_simd_model* m);
/* Context ctor: quantized feature per covariance, out is C x Dp (cc:22-35). */
void orc_simd_quantize_frame(const orc_simd_model* m, const float* x, uint8_t* out);
/* scores / best_density / raw_min: mixture-major [n_mixtures][n_frames]; any may be NULL. */
int  orc_simd_score(const orc_simd_model* m, const orc_mixture_set* ms,
                    const float* frames, uint32_t n_frames, uint32_t frame_stride,
                    float* scores, uint32_t* best_density, int32_t* raw_min, int n_threads);

/* ---- diagonal-maximum (src/Mm/GaussDiagonalMaximumFeatureScorer.cc) ---- */
typedef struct {
    uint32_t dimension, n_covariances, n_entries;
    float*   isv;              /* C x D after scale(sqrt(gaussian-scale)) */
    float*   log_norm;         /* C                                       */
    float*   minus2_log_weight;/* n_entries, after scale(mixture-weight-scale) */
} orc_float_model;

int  orc_float_prepare(const orc_mixture_set* ms, float mixture_weight_scale, float gaussian_scale,
                       orc_float_model* out);
void orc_float_free(orc_float_model* m);
int  orc_float_score(const orc_float_model* m, const orc_mixture_set* ms,
                     const float* frames, uint32_t n_frames, uint32_t frame_stride,
                     float* scores, uint32_t* best_density, int n_threads);
/* diagonal-sum (GaussDiagonalSumFeatureScorer): same model as diagonal-maximum (inherited init) */
int  orc_float_sum_score(const orc_float_model* m, const orc_mixture_set* ms,
                         const float* frames, uint32_t n_frames, uint32_t frame_stride,
                         float* scores, uint32_t* best_density, int n_threads);

/* ---- batch-diagonal-maximum-int / -float (src/Mm/BatchFeatureScorer.cc) ---- */
int orc_batch_int_score(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                        uint32_t frame_stride, float* scores, int n_threads);
int orc_batch_float_score(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                          uint32_t frame_stride, float* scores, int n_threads);

/* ---- preselection-batch-int / -float (BatchFeatureScorer.cc:238-289, 478-533): the batch scorers
 * restricted to the densities whose cluster the frame selected; entry_cluster [entries] is
 * clusterIndexForDensity_, selection [n_frames][n_clusters] activeClusters_ (presel_oracle.cc) ---- */
int orc_batch_int_score_sel(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                            uint32_t frame_stride, float* scores, int n_threads, const uint8_t* entry_cluster,
                            const uint8_t* selection, uint32_t n_clusters);
int orc_batch_float_score_sel(const orc_mixture_set* ms, const float* frames, uint32_t n_frames,
                              uint32_t frame_stride, float* scores, int n_threads, const uint8_t* entry_cluster,
                              const uint8_t* selection, uint32_t n_clusters, float backoff);
/* the prepared tables the clustering runs on: Dp = dimension padded to 8 (float) / 16 (int) */
int orc_batch_float_tables(const orc_mixture_set* ms, float* variance_out, float* means_out, float* constants_out);
int orc_batch_int_tables(const orc_mixture_set* ms, float* variance_out, uint8_t* means_out);

/* ---- helpers for known-answer tests ---- */
void orc_quantize_array(const float* x, uint32_t n, uint8_t* out);
int  orc_batch_int_prepare(const orc_mixture_set* ms, float* scale_out, float* variance_out, int32_t* constants_out);

#ifdef __cplusplus
}
#endif
#endif
