// nn_api.cc -- C-ABI of the MI355X hybrid-DNN acoustic scorer (include/rasr_nn.h).
//
// One handle = the network resident on one GPU: per layer W^T as bf16 [Mpad][Kpad] (zero padded to
// the 128 x 64 GEMM tiles) and the f32 bias (the top layer's with the scaled log prior removed),
// plus activation buffers for config max_frames.  nn_score_device enqueues one input conversion
// and one fused GEMM per layer on the caller's stream; no host synchronisation, no allocation.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rasr_nn.h"
#include "gmm_hostio.hh"
#include "gmm_kernels.hh"  // launchTransposeWords (gmm_kernels_layout.hip)
#include "nn_kernels.hh"

using namespace rasr_nn;

namespace {

thread_local std::string gNnError;

int fail(int code, const std::string& msg) {
    gNnError = msg;
    return code;
}

#define NN_HIP_CHECK(expr)                                                                          \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail(GMM_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));        \
    } while (0)

uint32_t roundUp(uint32_t x, uint32_t q) {
    return (x + q - 1) / q * q;
}

// f32 -> bf16 bits, round to nearest even (NaN kept a NaN)
uint16_t bf16Bits(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u)
        return static_cast<uint16_t>((u >> 16) | 0x40u);
    return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

struct Layer {
    uint32_t  K = 0, M = 0, Kpad = 0, Mpad = 0;
    int       act   = 0;
    float     gamma = 1.0f;
    uint16_t* dW    = nullptr;  // W^T [Mpad][Kpad]
    float*    dBias = nullptr;  // [Mpad]
};

}  // namespace

struct nn_scorer {
    int                device = 0;
    std::vector<Layer> layers;
    uint32_t           maxFrames = 0, maxFramesPad = 0;
    uint16_t*          dX0 = nullptr;             // [maxFramesPad][layers[0].Kpad]
    std::vector<uint16_t*> dH;                    // hidden outputs [maxFramesPad][Mpad]
    bool               timing = false;
    hipEvent_t         ev0 = nullptr, ev1 = nullptr;
    bool               pending = false;
    double             totalMs = 0;
    uint32_t           nCalls  = 0;
    // nn_score_host staging (lazily, for max_frames)
    hipStream_t        hostStream = nullptr;
    float*             dHostF = nullptr;  // [maxFrames][K]
    float*             dHostS = nullptr;  // [M][maxFrames]
    float*             dHostT = nullptr;  // [maxFrames][M] (frame-major)
    float*             dPart  = nullptr;  // nnGemm128 split-K partial sums [kNnSplitFloats]

    ~nn_scorer() {
        (void)hipSetDevice(device);
        for (auto& l : layers) {
            (void)hipFree(l.dW);
            (void)hipFree(l.dBias);
        }
        (void)hipFree(dX0);
        for (float* p : {dHostF, dHostS, dHostT, dPart})
            (void)hipFree(p);
        if (hostStream)
            (void)hipStreamDestroy(hostStream);
        for (auto* h : dH)
            (void)hipFree(h);
        if (ev0)
            (void)hipEventDestroy(ev0);
        if (ev1)
            (void)hipEventDestroy(ev1);
    }
};

namespace {

int collectTiming(nn_scorer* s) {
    if (!s->pending)
        return GMM_OK;
    NN_HIP_CHECK(hipEventSynchronize(s->ev1));
    float ms = 0;
    NN_HIP_CHECK(hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->totalMs += ms;
    s->nCalls += 1;
    s->pending = false;
    return GMM_OK;
}

}  // namespace

namespace {

// calls of up to this many frames run nnGemmSmall (RASR_NN_SMALL_FRAMES overrides, 0 = never: A/B)
uint32_t smallGemmFrames() {
    static const uint32_t n = [] {
        const char* e = std::getenv("RASR_NN_SMALL_FRAMES");
        return e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : kNnSmallFrames;
    }();
    return n;
}

// layers whose nnGemm8p grid is smaller than this run nnGemm128 (RASR_NN_TILE128_WGS overrides, 0 = never: A/B)
uint32_t tile128Wgs() {
    static const uint32_t n = [] {
        const char* e = std::getenv("RASR_NN_TILE128_WGS");
        return e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : kNnTile128Wgs;
    }();
    return n;
}

// nnGemm128 splits the K range of hidden layers whose 128-tile grid is below kNnSplitWgs (RASR_NN_SPLIT_K=0: never)
bool splitK() {
    static const bool on = [] {
        const char* e = std::getenv("RASR_NN_SPLIT_K");
        return !e || std::strtoul(e, nullptr, 10) != 0;
    }();
    return on;
}

// the most workgroups a tile's K range is split over (RASR_NN_MAX_SPLIT overrides, 2..kNnMaxSplit: A/B)
uint32_t maxSplit() {
    static const uint32_t n = [] {
        const char* e = std::getenv("RASR_NN_MAX_SPLIT");
        const uint32_t v = e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : 4u;
        return std::max(2u, std::min(kNnMaxSplit, v));
    }();
    return n;
}

}  // namespace

extern "C" {

const char* nn_last_error(void) {
    return gNnError.c_str();
}

int nn_prior_from_mixture_set(const gmm_mixture_set* ms, float* logPrior) {
    if (!ms || !logPrior || !ms->mixture_offsets || !ms->mixture_log_weights)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    // Prior::setFromMixtureSet (src/Nn/Prior.cc:159-190): f32 sums of mixture->weight(dns) = exp(logw), an f64
    // (Mm::Weight, src/Mm/Types.hh:30): `f32 += f64` adds in f64 and rounds the sum to f32 once per density;
    // normalized by their (double-accumulated, std::accumulate with 0.0) total, then std::log
    std::vector<float> p(ms->n_mixtures, 0.0f);
    for (uint32_t m = 0; m < ms->n_mixtures; ++m)
        for (uint32_t i = ms->mixture_offsets[m]; i < ms->mixture_offsets[m + 1]; ++i)
            p[m] = static_cast<float>(static_cast<double>(p[m]) + std::exp(ms->mixture_log_weights[i]));
    double total = 0.0;
    for (float v : p)
        total += v;
    const float w = static_cast<float>(total);
    for (uint32_t m = 0; m < ms->n_mixtures; ++m)
        logPrior[m] = std::log(p[m] / w);
    return GMM_OK;
}

int nn_scorer_create(const nn_network_desc* net, uint32_t maxFrames, int device, nn_scorer** out) {
    if (!net || !out || !net->layers || net->n_layers == 0 || maxFrames == 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid network description");
    *out = nullptr;
    for (uint32_t l = 0; l < net->n_layers; ++l) {
        const nn_layer_desc& d = net->layers[l];
        if (!d.weights || d.input_dim == 0 || d.output_dim == 0)
            return fail(GMM_ERR_INVALID_ARGUMENT, "layer " + std::to_string(l) + ": empty weights");
        if (l > 0 && d.input_dim != net->layers[l - 1].output_dim)
            return fail(GMM_ERR_INVALID_ARGUMENT, "layer " + std::to_string(l) + ": input dimension " +
                                                      std::to_string(d.input_dim) + " != previous output " +
                                                      std::to_string(net->layers[l - 1].output_dim));
        if (d.activation < NN_ACT_IDENTITY || d.activation > NN_ACT_ELU)
            return fail(GMM_ERR_UNSUPPORTED, "layer " + std::to_string(l) + ": unknown activation");
    }
    auto s          = std::make_unique<nn_scorer>();
    s->device       = device;
    s->maxFrames    = maxFrames;
    s->maxFramesPad = roundUp(maxFrames, kNnTileN);
    NN_HIP_CHECK(hipSetDevice(device));
    for (uint32_t l = 0; l < net->n_layers; ++l) {
        const nn_layer_desc& d   = net->layers[l];
        const bool           top = l + 1 == net->n_layers;
        Layer                L;
        L.K     = d.input_dim;
        L.M     = d.output_dim;
        L.Kpad  = l == 0 ? roundUp(L.K, kNnTileK) : s->layers[l - 1].Mpad;
        L.Mpad  = roundUp(L.M, kNnTileM);
        L.act   = d.activation;
        L.gamma = d.gamma;
        // W^T [Mpad][Kpad] bf16, zero padding (padded inputs meet zero weights)
        std::vector<uint16_t> wt(static_cast<size_t>(L.Mpad) * L.Kpad, 0);
        for (uint32_t k = 0; k < L.K; ++k)
            for (uint32_t m = 0; m < L.M; ++m)
                wt[static_cast<size_t>(m) * L.Kpad + k] = bf16Bits(d.weights[static_cast<size_t>(k) * L.M + m]);
        // bias; top layer: bias - prior_scale * log_prior (BiasLayer::removeLogPriorFromBias, LinearLayer.cc:499-518)
        std::vector<float> bias(L.Mpad, 0.0f);
        for (uint32_t m = 0; m < L.M; ++m) {
            float b = d.bias ? d.bias[m] : 0.0f;
            if (top && net->log_prior && net->prior_scale != 0.0f)
                b -= net->prior_scale * net->log_prior[m];
            bias[m] = b;
        }
        s->layers.push_back(L);  // owned by s from here on (freed by ~nn_scorer on any failure below)
        Layer& D = s->layers.back();
        NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&D.dW), wt.size() * sizeof(uint16_t)));
        NN_HIP_CHECK(hipMemcpy(D.dW, wt.data(), wt.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
        NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&D.dBias), bias.size() * sizeof(float)));
        NN_HIP_CHECK(hipMemcpy(D.dBias, bias.data(), bias.size() * sizeof(float), hipMemcpyHostToDevice));
        if (!top) {
            const size_t bytes = static_cast<size_t>(s->maxFramesPad) * L.Mpad * sizeof(uint16_t);
            s->dH.push_back(nullptr);
            NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dH.back()), bytes));
            NN_HIP_CHECK(hipMemset(s->dH.back(), 0, bytes));
        }
    }
    // padded input columns stay zero: the conversion writes columns < input_dim only
    const size_t xBytes = static_cast<size_t>(s->maxFramesPad) * s->layers[0].Kpad * sizeof(uint16_t);
    NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dX0), xBytes));
    NN_HIP_CHECK(hipMemset(s->dX0, 0, xBytes));
    if (splitK() && maxFrames > smallGemmFrames())  // only calls beyond the small-call range split K
        NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dPart), kNnSplitFloats * sizeof(float)));
    NN_HIP_CHECK(hipEventCreate(&s->ev0));
    NN_HIP_CHECK(hipEventCreate(&s->ev1));
    NN_HIP_CHECK(hipDeviceSynchronize());
    *out = s.release();
    return GMM_OK;
}

int nn_scorer_destroy(nn_scorer* s) {
    delete s;
    return GMM_OK;
}

uint32_t nn_scorer_n_classes(const nn_scorer* s) {
    return s ? s->layers.back().M : 0;
}

uint32_t nn_scorer_input_dim(const nn_scorer* s) {
    return s ? s->layers.front().K : 0;
}

int nn_score_device(nn_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
                    uint32_t scoreStride, void* stream) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    if (nFrames == 0)
        return GMM_OK;
    if (nFrames > s->maxFrames)
        return fail(GMM_ERR_CAPACITY, "n_frames exceeds max_frames");
    if (!frames || !scores || frameStride < s->layers[0].K || scoreStride < nFrames)
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid frames/scores/stride");
    NN_HIP_CHECK(hipSetDevice(s->device));
    hipStream_t    st   = static_cast<hipStream_t>(stream);
    const bool     small = nFrames <= smallGemmFrames();
    const uint32_t Npad  = small ? roundUp(nFrames, nFrames <= 64 ? 16u : 64u) : roundUp(nFrames, kNnTileN);
    NN_HIP_CHECK(launchNnPrepareInput(frames, nFrames, frameStride, s->layers[0].K, s->layers[0].Kpad, s->dX0, st));
    if (s->timing) {
        int rc = collectTiming(s);
        if (rc != GMM_OK)
            return rc;
        NN_HIP_CHECK(hipEventRecord(s->ev0, st));
    }
    const uint16_t* in = s->dX0;
    for (size_t l = 0; l < s->layers.size(); ++l) {
        const Layer& L   = s->layers[l];
        const bool   top = l + 1 == s->layers.size();
        NnGemmArgs   a{};
        a.A           = L.dW;
        a.B           = in;
        a.bias        = L.dBias;
        a.Y           = top ? nullptr : s->dH[l];
        a.scores      = top ? scores : nullptr;
        a.Mpad        = L.Mpad;
        a.Kpad        = L.Kpad;
        a.Npad        = Npad;
        a.M           = L.M;
        a.nFrames     = nFrames;
        a.scoreStride = scoreStride;
        a.act         = L.act;
        a.gamma       = L.gamma;
        a.top         = top ? 1 : 0;
        // the top layer keeps nnGemm8p from 2/3 of the limit on (its C^T form's 16-byte score stores; 2048 frames
        // x 5000 classes, 160 tiles of 256: 194 vs 208 us for the whole network, profiles/r04/s30)
        const uint32_t lim = top ? tile128Wgs() * 2u / 3u : tile128Wgs();
        const bool     mid = !small && (L.Mpad / kNnTileM) * (Npad / kNnTileN) < lim;
        // hidden layers whose 128-tile grid leaves most CUs idle: K split over up to 4 workgroups per tile
        const uint32_t wg128 = (L.Mpad / 128u) * (Npad / 128u);
        if (mid && !top && s->dPart && wg128 < kNnSplitWgs) {
            a.kSplit = std::min(maxSplit(), 2u * kNnSplitWgs / wg128);
            a.part   = s->dPart;
        }
        NN_HIP_CHECK(small ? launchNnGemmSmall(a, st) : mid ? launchNnGemm128(a, st) : launchNnGemm(a, st));
        in = a.Y;
    }
    if (s->timing) {
        NN_HIP_CHECK(hipEventRecord(s->ev1, st));
        s->pending = true;
    }
    return GMM_OK;
}

int nn_score_host(nn_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
                  uint32_t scoreStride) {
    return nn_score_host_ex(s, frames, nFrames, frameStride, scores, scoreStride, 0);
}

int nn_score_host_ex(nn_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
                     uint32_t scoreStride, uint32_t flags) {
    if (!s || !frames || !scores)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if ((flags & ~NN_HOST_FRAME_MAJOR) != 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "unknown flags");
    if (nFrames == 0)
        return GMM_OK;
    if (nFrames > s->maxFrames)
        return fail(GMM_ERR_CAPACITY, "n_frames exceeds max_frames");
    const bool     frameMajor = (flags & NN_HOST_FRAME_MAJOR) != 0;
    const uint32_t K = s->layers[0].K, M = s->layers.back().M;
    if (frameStride < K || scoreStride < (frameMajor ? M : nFrames))
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid frame/score stride");
    NN_HIP_CHECK(hipSetDevice(s->device));
    // persistent staging (allocated once for max_frames) on the scorer's own stream: dense [F][K] frames,
    // [M][F] scores and, frame-major, their transpose [F][M]
    if (!s->hostStream) {
        NN_HIP_CHECK(hipStreamCreateWithFlags(&s->hostStream, hipStreamNonBlocking));
        NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostF), static_cast<size_t>(s->maxFrames) * K * sizeof(float)));
        NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostS), static_cast<size_t>(s->maxFrames) * M * sizeof(float)));
    }
    if (frameMajor && !s->dHostT)
        NN_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostT), static_cast<size_t>(s->maxFrames) * M * sizeof(float)));
    // only the caller's K used floats per frame row are read; only the call's rows / columns of a strided caller
    // table are written (the rest stays untouched, as with gmm_score_host)
    // small calls (<= 64 frames) with page-locked buffers the device addresses at the same pointer: no copy engine,
    // a kernel gathers the frame rows and the transpose / a strided copy kernel writes the caller's table over PCIe
    // (as gmm_score_host_ring's small calls, gmm_api.cc scoreHostSmall)
    static const bool smallOn = [] {  // RASR_GMM_SMALL_HOST=0: the copy-engine path (A/B)
        const char* e = std::getenv("RASR_GMM_SMALL_HOST");
        return !(e && e[0] == '0');
    }();
    const bool small =
            smallOn && nFrames <= 64 && rasr_gmm::isDeviceMappedHost(frames) && rasr_gmm::isDeviceMappedHost(scores);
    int rc = GMM_OK;
    auto run = [&]() -> int {
        if (small)
            NN_HIP_CHECK(rasr_gmm::launchCopyWords2D(reinterpret_cast<const uint32_t*>(frames), frameStride,
                                                     reinterpret_cast<uint32_t*>(s->dHostF), K, nFrames, K, s->hostStream));
        else
            NN_HIP_CHECK(hipMemcpy2DAsync(s->dHostF, static_cast<size_t>(K) * sizeof(float), frames,
                                          static_cast<size_t>(frameStride) * sizeof(float),
                                          static_cast<size_t>(K) * sizeof(float), nFrames, hipMemcpyHostToDevice,
                                          s->hostStream));
        int r = nn_score_device(s, s->dHostF, nFrames, K, s->dHostS, nFrames, s->hostStream);
        if (r != GMM_OK)
            return r;
        if (small) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(s->dHostS);
            uint32_t*       dst = reinterpret_cast<uint32_t*>(scores);
            if (frameMajor)
                NN_HIP_CHECK(rasr_gmm::launchTransposeWords(src, M, nFrames, nFrames, dst, scoreStride, s->hostStream));
            else
                NN_HIP_CHECK(rasr_gmm::launchCopyWords2D(src, nFrames, dst, scoreStride, M, nFrames, s->hostStream));
        }
        else if (frameMajor) {
            NN_HIP_CHECK(rasr_gmm::launchTransposeWords(reinterpret_cast<const uint32_t*>(s->dHostS), M, nFrames, nFrames,
                                                        reinterpret_cast<uint32_t*>(s->dHostT), M, s->hostStream));
            NN_HIP_CHECK(hipMemcpy2DAsync(scores, static_cast<size_t>(scoreStride) * sizeof(float), s->dHostT,
                                          static_cast<size_t>(M) * sizeof(float), static_cast<size_t>(M) * sizeof(float),
                                          nFrames, hipMemcpyDeviceToHost, s->hostStream));
        }
        else
            NN_HIP_CHECK(hipMemcpy2DAsync(scores, static_cast<size_t>(scoreStride) * sizeof(float), s->dHostS,
                                          static_cast<size_t>(nFrames) * sizeof(float),
                                          static_cast<size_t>(nFrames) * sizeof(float), M, hipMemcpyDeviceToHost,
                                          s->hostStream));
        NN_HIP_CHECK(hipStreamSynchronize(s->hostStream));
        return GMM_OK;
    };
    rc = run();
    if (rc != GMM_OK)
        (void)hipStreamSynchronize(s->hostStream);  // nothing of this call may still run into the caller's buffers
    return rc;
}

int nn_scorer_set_timing(nn_scorer* s, int enable) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    int rc = collectTiming(s);
    s->timing = enable != 0;
    return rc;
}

int nn_scorer_kernel_time(nn_scorer* s, double* totalMs, uint32_t* nCalls, int reset) {
    if (!s || !totalMs || !nCalls)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    int rc = collectTiming(s);
    if (rc != GMM_OK)
        return rc;
    *totalMs = s->totalMs;
    *nCalls  = s->nCalls;
    if (reset) {
        s->totalMs = 0;
        s->nCalls  = 0;
    }
    return GMM_OK;
}

}  // extern "C"
