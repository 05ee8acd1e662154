// nn_standin.cc -- TEST INFRASTRUCTURE ONLY: a CPU stand-in for the parts of the NN C-ABI (include/rasr_nn.h) and the
// page-locked allocator of include/rasr_gmm.h that the RASR-side NN adapter (integration/rasr/Nn/) calls, so the
// adapter can be linked and run on the CPU by tests/rasr_harness/nn_harness.cc.  The forward pass is the
// reference's f32 arithmetic (LinearLayer::_forward, src/Nn/LinearLayer.cc:297-321: out = W^T in + bias; the
// activation layers of src/Nn/ActivationLayer.cc), the same restatement as oracle/nn_oracle.py forward_f32; the top
// layer's output is written negated (BatchFeatureScorer::getScore, cc:148-171).  Never part of librasr_gmm.so.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rasr_gmm.h"
#include "../../include/rasr_nn.h"

namespace {
thread_local std::string gError;
int fail(int code, const std::string& m) {
    gError = m;
    return code;
}
struct Layer {
    uint32_t           in, out;
    std::vector<float> w, b;  // w [in][out]
    nn_activation      act;
    float              gamma;
};
}  // namespace

struct nn_scorer {
    std::vector<Layer> layers;
    uint32_t           maxFrames;
};

extern "C" {

const char* nn_last_error(void) { return gError.c_str(); }
const char* gmm_last_error(void) { return gError.c_str(); }

int gmm_host_alloc(size_t bytes, void** p) {
    if (!p)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null ptr");
    *p = bytes ? std::malloc(bytes) : nullptr;
    return (*p || !bytes) ? GMM_OK : fail(GMM_ERR_OUT_OF_MEMORY, "malloc");
}
int gmm_host_free(void* p) {
    std::free(p);
    return GMM_OK;
}

int nn_scorer_create(const nn_network_desc* net, uint32_t maxFrames, int device, nn_scorer** out) {
    (void)device;
    if (!net || !out || !net->layers || net->n_layers == 0 || maxFrames == 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid network description");
    nn_scorer* s = new nn_scorer();
    s->maxFrames = maxFrames;
    for (uint32_t l = 0; l < net->n_layers; ++l) {
        const nn_layer_desc& d = net->layers[l];
        if (l && d.input_dim != s->layers.back().out) {
            delete s;
            return fail(GMM_ERR_INVALID_ARGUMENT, "layer dimensions do not chain");
        }
        Layer x{d.input_dim, d.output_dim, std::vector<float>(d.weights, d.weights + size_t(d.input_dim) * d.output_dim),
                d.bias ? std::vector<float>(d.bias, d.bias + d.output_dim) : std::vector<float>(d.output_dim, 0.0f),
                d.activation, d.gamma};
        if (l + 1 == net->n_layers && net->log_prior && net->prior_scale != 0.0f)
            for (uint32_t o = 0; o < d.output_dim; ++o)
                x.b[o] -= net->prior_scale * net->log_prior[o];
        s->layers.push_back(x);
    }
    *out = s;
    return GMM_OK;
}

int nn_scorer_destroy(nn_scorer* s) {
    delete s;
    return GMM_OK;
}
uint32_t nn_scorer_n_classes(const nn_scorer* s) { return s ? s->layers.back().out : 0; }
uint32_t nn_scorer_input_dim(const nn_scorer* s) { return s ? s->layers.front().in : 0; }

int nn_score_host_ex(nn_scorer* s, const float* frames, uint32_t n, uint32_t fstride, float* scores, uint32_t stride,
                     uint32_t flags) {
    if (!s || (n && (!frames || !scores)))
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if (n > s->maxFrames)
        return fail(GMM_ERR_CAPACITY, "n_frames exceeds max_frames");
    const bool fm = (flags & NN_HOST_FRAME_MAJOR) != 0;
    for (uint32_t t = 0; t < n; ++t) {
        std::vector<float> h(frames + size_t(t) * fstride, frames + size_t(t) * fstride + s->layers.front().in);
        for (size_t l = 0; l < s->layers.size(); ++l) {
            const Layer&       L = s->layers[l];
            std::vector<float> z(L.out);
            for (uint32_t o = 0; o < L.out; ++o) {
                float acc = 0.0f;
                for (uint32_t i = 0; i < L.in; ++i)
                    acc += L.w[size_t(i) * L.out + o] * h[i];
                z[o] = acc + L.b[o];
                if (l + 1 == s->layers.size())
                    continue;
                switch (L.act) {
                    case NN_ACT_SIGMOID: z[o] = 1.0f / (1.0f + std::exp(-L.gamma * z[o])); break;
                    case NN_ACT_TANH: z[o] = std::tanh(z[o]); break;
                    case NN_ACT_RELU: z[o] = z[o] > 0.0f ? z[o] : 0.0f; break;
                    case NN_ACT_ELU: z[o] = z[o] > 0.0f ? z[o] : std::exp(z[o]) - 1.0f; break;
                    default: break;
                }
            }
            h.swap(z);
        }
        for (uint32_t e = 0; e < h.size(); ++e)
            scores[fm ? size_t(t) * stride + e : size_t(e) * stride + t] = -h[e];
    }
    return GMM_OK;
}

}  // extern "C"
