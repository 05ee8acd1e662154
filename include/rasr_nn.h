/*
 * rasr_nn.h -- C-ABI of the MI355X hybrid-DNN acoustic scorer (SURVEY.md 8(f) row 3,
 * BASELINE.json config 5): the drop-in for Nn::BatchFeatureScorer
 * (src/Nn/BatchFeatureScorer.cc:25-171), which registers as an Mm::FeatureScorer
 * (src/Nn/Module.cc:39-67) and scores a buffer of feature vectors with a feed-forward
 * network whose top layer is "linear+softmax" evaluated WITHOUT the softmax, after the
 * scaled log prior was removed from its bias (BatchFeatureScorer.cc:52-79,
 * BiasLayer::removeLogPriorFromBias, src/Nn/LinearLayer.cc:499-518):
 *
 *     h_0 = x,   h_l = act_l(W_l^T h_{l-1} + b_l)            (LinearLayer::_forward, LinearLayer.cc:297-321)
 *     score(e, t) = -(W_L^T h_{L-1} + b_L - prior_scale * log_prior)[e]   (getScore, cc:148-171)
 *
 * Weights are given as Nn::LinearLayer keeps them: W_l is [input_dim][output_dim]
 * row-major (output = W^T input).  The GPU computes on bf16 MFMA (v_mfma_f32_16x16x32_bf16)
 * with f32 accumulation: weights and hidden activations are rounded to bf16, bias,
 * activation functions and scores are f32.  Status codes as rasr_gmm.h (GMM_OK, ...).
 * Score tables are class-major: scores[e * score_stride + t], as the GMM scorer's.
 */
#ifndef RASR_NN_H
#define RASR_NN_H

#include <stddef.h>
#include <stdint.h>

#include "rasr_gmm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Activation layers of src/Nn/ActivationLayer.hh (Nn::Module layer types). */
typedef enum {
    NN_ACT_IDENTITY = 0, /* IdentityLayer (ActivationLayer.hh:31)                          */
    NN_ACT_SIGMOID  = 1, /* SigmoidLayer: 1 / (1 + exp(-gamma x)) ("gamma", ActivationLayer.cc:103-131) */
    NN_ACT_TANH     = 2, /* TanhLayer (ActivationLayer.hh:49)                              */
    NN_ACT_RELU     = 3, /* RectifiedLayer: max(0, x) (ActivationLayer.hh:193)             */
    NN_ACT_ELU      = 4  /* ExponentialLinearLayer, alpha 1 (ActivationLayer.cc:333-348)  */
} nn_activation;

typedef struct {
    uint32_t      input_dim, output_dim;
    const float*  weights;    /* [input_dim][output_dim], output = weights^T input + bias */
    const float*  bias;       /* [output_dim] (NULL: no bias, LinearLayer hasBias_ false)  */
    nn_activation activation; /* ignored for the top layer (softmax not evaluated)        */
    float         gamma;      /* sigmoid scale ("gamma", default 1)                      */
} nn_layer_desc;

typedef struct {
    uint32_t             n_layers; /* >= 1; the last one is the top (linear+softmax) layer   */
    const nn_layer_desc* layers;
    const float*         log_prior;   /* [top output_dim] Prior::logPrior_ or NULL (no prior)  */
    float                prior_scale; /* "priori-scale" (Prior.cc:28-29, default 1)           */
} nn_network_desc;

typedef struct nn_scorer nn_scorer;

/* Prior::setFromMixtureSet (src/Nn/Prior.cc:159-190) with a one-to-one class label mapping:
 * log_prior[m] = log(sum_d exp(logw_md) / sum_m' sum_d exp(logw_m'd)).  n_mixtures floats. */
int nn_prior_from_mixture_set(const gmm_mixture_set* mixture_set, float* log_prior);

/* Network upload (bias minus prior_scale * log_prior on the top layer, done once in f64,
 * as BatchFeatureScorer::init does, cc:67-79) for up to max_frames frames per call. */
int nn_scorer_create(const nn_network_desc* network, uint32_t max_frames, int device, nn_scorer** out);
int nn_scorer_destroy(nn_scorer* scorer);
uint32_t nn_scorer_n_classes(const nn_scorer* scorer);
uint32_t nn_scorer_input_dim(const nn_scorer* scorer);

/* Score n_frames feature vectors (DEVICE pointers, row t at frames + t * frame_stride),
 * scores [n_classes][score_stride] f32, enqueued on `stream` (hipStream_t, NULL = default).
 * Replaces BatchFeatureScorer::getScore's network_.forward(buffer_) (cc:148-171). */
int nn_score_device(nn_scorer* scorer, const float* frames, uint32_t n_frames, uint32_t frame_stride,
                    float* scores, uint32_t score_stride, void* stream);
/* Same with HOST buffers (copies in and out, synchronizes; n_frames <= max_frames). */
int nn_score_host(nn_scorer* scorer, const float* frames, uint32_t n_frames, uint32_t frame_stride,
                  float* scores, uint32_t score_stride);
/* nn_score_host with flags.  NN_HOST_FRAME_MAJOR: scores are frame-major, scores[t * score_stride + e]
 * (score_stride >= n_classes) -- the layout of the reference's output matrix, whose column t holds frame
 * t's classes (Math::FastMatrix is column-major; BatchFeatureScorer::getScore reads at(e, position),
 * BatchFeatureScorer.cc:148-171), so a context's score(e) calls read one contiguous row. */
#define NN_HOST_FRAME_MAJOR 2u
int nn_score_host_ex(nn_scorer* scorer, const float* frames, uint32_t n_frames, uint32_t frame_stride,
                     float* scores, uint32_t score_stride, uint32_t flags);

/* bench.py instrumentation, as gmm_scorer_set_timing / gmm_scorer_kernel_time: HIP events
 * around the layer GEMMs of every call; total GEMM time (ms) and call count since the last reset. */
int nn_scorer_set_timing(nn_scorer* scorer, int enable);
int nn_scorer_kernel_time(nn_scorer* scorer, double* total_ms, uint32_t* n_calls, int reset);

const char* nn_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* RASR_NN_H */
