// gmm_standin.cc -- TEST INFRASTRUCTURE ONLY: a CPU stand-in for the parts of the C-ABI (include/rasr_gmm.h)
// that the host-side scorer classes (rasr_amd/csrc/host/GpuFeatureScorer.cc) call, backed by the oracle
// restatement (oracle/gmm_oracle.c).  It reproduces the ABI's semantics -- ring positions, mixture- or
// frame-major tables, best densities kept until fetched and invalidated by the next host call, status codes
// -- so that the RASR-side adapter can be linked and run on the CPU by tests/rasr_harness/harness.cc.
// Never linked into librasr_gmm.so; the product path is the HIP library.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rasr_gmm.h"
#include "../../include/rasr_gmm_io.h"
#include "../../oracle/gmm_oracle.h"

namespace {
thread_local std::string gError;
int fail(int code, const std::string& m) {
    gError = m;
    return code;
}
}  // namespace

struct gmm_scorer {
    gmm_scorer_type       type;
    gmm_scorer_config     cfg;
    uint32_t              D = 0, C = 0, M = 0;
    std::vector<float>    means, vars;
    std::vector<uint32_t> dMean, dCov, off, dens;
    std::vector<double>   logw;
    orc_mixture_set       ms{};
    orc_simd_model        simd{};
    orc_float_model       flt{};
    bool                  hasSimd = false, hasFloat = false;
    uint64_t              call = 0, keptCall = 0;
    std::vector<uint32_t> kept;       // [M][n] best densities of the kept call
    std::vector<uint32_t> keptPos;    // ring position of each of its frames
    bool                  keptFrameMajor = false;
    ~gmm_scorer() {
        if (hasSimd)
            orc_simd_free(&simd);
        if (hasFloat)
            orc_float_free(&flt);
    }
};

extern "C" {

void gmm_default_config(gmm_scorer_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->mixture_weight_scale = 1.0f;
    c->gaussian_scale       = 1.0f;
    c->score_scale          = 1.0f;
    c->max_frames           = 4096;
    c->clusters             = 256;
    c->select_clusters      = 32;
    c->clustering_iterations = 5;
    c->backoff_score        = 40000.0f;
}

const char* gmm_last_error(void) { return gError.c_str(); }

// the cache archive and flags of the last create (the harness checks the adapter's "cache-archive" resolution)
std::string gStandinCacheArchive;
uint32_t    gStandinFlags = 0;

int gmm_scorer_create(const gmm_mixture_set* m, gmm_scorer_type type, const gmm_scorer_config* cfg, int device,
                      gmm_scorer** out) {
    (void)device;
    if (!m || !out || !cfg)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if (type != GMM_SIMD_DIAGONAL_MAXIMUM && type != GMM_DIAGONAL_MAXIMUM && type != GMM_BATCH_DIAGONAL_MAXIMUM_INT &&
        type != GMM_BATCH_DIAGONAL_MAXIMUM_FLOAT)
        return fail(GMM_ERR_UNSUPPORTED, "stand-in: type not restated");
    gmm_scorer* s = new gmm_scorer();
    s->type       = type;
    s->cfg        = *cfg;
    gStandinCacheArchive = cfg->cache_archive ? cfg->cache_archive : "";
    gStandinFlags        = cfg->flags;
    s->D = m->dimension, s->C = m->n_covariances, s->M = m->n_mixtures;
    const uint32_t nE = m->mixture_offsets[m->n_mixtures];
    s->means.assign(m->means, m->means + static_cast<size_t>(m->n_means) * m->dimension);
    s->vars.assign(m->variances, m->variances + static_cast<size_t>(m->n_covariances) * m->dimension);
    s->dMean.assign(m->density_mean, m->density_mean + m->n_densities);
    s->dCov.assign(m->density_covariance, m->density_covariance + m->n_densities);
    s->off.assign(m->mixture_offsets, m->mixture_offsets + m->n_mixtures + 1);
    s->dens.assign(m->mixture_densities, m->mixture_densities + nE);
    s->logw.assign(m->mixture_log_weights, m->mixture_log_weights + nE);
    s->ms = orc_mixture_set{m->dimension, m->n_means, s->means.data(), m->n_covariances, s->vars.data(),
                            m->n_densities, s->dMean.data(), s->dCov.data(), m->n_mixtures, s->off.data(),
                            s->dens.data(), s->logw.data()};
    if (type == GMM_SIMD_DIAGONAL_MAXIMUM) {
        if (orc_simd_prepare(&s->ms, &s->simd) != 0) {
            delete s;
            return fail(GMM_ERR_INVALID_ARGUMENT, "orc_simd_prepare");
        }
        s->hasSimd = true;
    }
    if (type == GMM_DIAGONAL_MAXIMUM) {
        if (orc_float_prepare(&s->ms, cfg->mixture_weight_scale, cfg->gaussian_scale, &s->flt) != 0) {
            delete s;
            return fail(GMM_ERR_INVALID_ARGUMENT, "orc_float_prepare");
        }
        s->hasFloat = true;
    }
    *out = s;
    return GMM_OK;
}

// the sharded handle: the stand-in records the device list it was asked for (the harness checks that the
// adapter's "density-shard-devices" reaches it) and scores the whole model (sharding does not change results)
std::vector<int> gStandinShardDevices;

int gmm_scorer_create_sharded(const gmm_mixture_set* m, gmm_scorer_type type, const gmm_scorer_config* cfg,
                              const int* devices, uint32_t n, int exchange, gmm_scorer** out) {
    if (!devices || n == 0 || exchange != GMM_EXCHANGE_AUTO)
        return fail(GMM_ERR_INVALID_ARGUMENT, "stand-in: devices / exchange");
    gStandinShardDevices.assign(devices, devices + n);
    return gmm_scorer_create(m, type, cfg, devices[0], out);
}

int gmm_scorer_clustering_source(const gmm_scorer* s, int* source) {
    (void)s;
    (void)source;
    return fail(GMM_ERR_UNSUPPORTED, "stand-in: no preselection types");
}

int gmm_scorer_destroy(gmm_scorer* s) {
    delete s;
    return GMM_OK;
}
uint32_t gmm_scorer_n_mixtures(const gmm_scorer* s) { return s ? s->M : 0; }
uint32_t gmm_scorer_dimension(const gmm_scorer* s) { return s ? s->D : 0; }
uint32_t gmm_scorer_n_covariances(const gmm_scorer* s) { return s ? s->C : 0; }

int gmm_scorer_quantization(const gmm_scorer* s, float* scaling, float* invQ) {
    if (!s || !s->hasSimd)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type is not quantized");
    if (scaling)
        *scaling = s->simd.scaling;
    if (invQ)
        *invQ = s->simd.inverse_quantization_factor;
    return GMM_OK;
}

int gmm_scorer_multiply_and_quantize(const gmm_scorer* s, const float* f, uint8_t* out) {
    if (!s || !s->hasSimd)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type is not quantized");
    orc_simd_quantize_frame(&s->simd, f, out);
    return GMM_OK;
}

int gmm_score_host_ring(gmm_scorer* s, const float* ring, uint32_t R, uint32_t first, uint32_t n, uint32_t fstride,
                        float* scores, uint32_t* best, uint32_t stride, uint32_t flags, uint64_t* callId) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    if ((flags & GMM_HOST_KEEP_BEST) && (flags & GMM_HOST_LAZY_BEST))
        return fail(GMM_ERR_INVALID_ARGUMENT, "GMM_HOST_KEEP_BEST and GMM_HOST_LAZY_BEST together");
    if ((flags & (GMM_HOST_KEEP_BEST | GMM_HOST_LAZY_BEST)) && best)
        return fail(GMM_ERR_INVALID_ARGUMENT, "GMM_HOST_KEEP_BEST / GMM_HOST_LAZY_BEST with a best_density table");
    const bool fm       = (flags & GMM_HOST_FRAME_MAJOR) != 0;
    const bool assign   = s->type == GMM_SIMD_DIAGONAL_MAXIMUM || s->type == GMM_DIAGONAL_MAXIMUM;
    // the stand-in computes the best densities with the scores either way (the oracle has no score-only mode)
    const bool keepBest = (flags & (GMM_HOST_KEEP_BEST | GMM_HOST_LAZY_BEST)) && assign;
    s->keptCall         = 0;
    const uint64_t id   = ++s->call;
    if (callId)
        *callId = id;
    if (n == 0)
        return GMM_OK;
    if (n > s->cfg.max_frames)
        return fail(GMM_ERR_CAPACITY, "n_frames exceeds config.max_frames");
    if (!ring || !scores || fstride < s->D || first >= R || n > R || stride < (fm ? s->M : R))
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid frames/scores/stride/ring");
    std::vector<float>    x(static_cast<size_t>(n) * s->D), sc(static_cast<size_t>(s->M) * n);
    std::vector<uint32_t> bd(static_cast<size_t>(s->M) * n, 0xffffffffu), pos(n);
    for (uint32_t i = 0; i < n; ++i) {
        pos[i] = (first + i) % R;
        std::memcpy(&x[static_cast<size_t>(i) * s->D], ring + static_cast<size_t>(pos[i]) * fstride, s->D * sizeof(float));
    }
    int rc = 0;
    switch (s->type) {
        case GMM_SIMD_DIAGONAL_MAXIMUM: rc = orc_simd_score(&s->simd, &s->ms, x.data(), n, s->D, sc.data(), bd.data(), 0, 1); break;
        case GMM_DIAGONAL_MAXIMUM: rc = orc_float_score(&s->flt, &s->ms, x.data(), n, s->D, sc.data(), bd.data(), 1); break;
        case GMM_BATCH_DIAGONAL_MAXIMUM_INT: rc = orc_batch_int_score(&s->ms, x.data(), n, s->D, sc.data(), 1); break;
        default: rc = orc_batch_float_score(&s->ms, x.data(), n, s->D, sc.data(), 1); break;
    }
    if (rc != 0)
        return fail(GMM_ERR_DEVICE, "oracle scoring failed");
    for (uint32_t e = 0; e < s->M; ++e)
        for (uint32_t i = 0; i < n; ++i) {
            const size_t o = fm ? static_cast<size_t>(pos[i]) * stride + e : static_cast<size_t>(e) * stride + pos[i];
            float        v = sc[static_cast<size_t>(e) * n + i];
            if (s->cfg.score_scale != 1.0f)
                v = s->cfg.score_scale * v;
            scores[o] = v;
            if (best)
                best[o] = assign ? bd[static_cast<size_t>(e) * n + i] : 0xffffffffu;
        }
    if (keepBest) {
        s->keptCall       = id;
        s->kept           = bd;
        s->keptPos        = pos;
        s->keptFrameMajor = fm;
    }
    return GMM_OK;
}

// GMM_HOST_ASYNC: the stand-in scores synchronously, so the wait has nothing to wait for
int gmm_host_call_wait(gmm_scorer* s, uint64_t callId) {
    (void)callId;
    return s ? GMM_OK : fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
}

int gmm_score_host(gmm_scorer* s, const float* frames, uint32_t n, uint32_t fstride, float* scores, uint32_t* best,
                   uint32_t stride) {
    return gmm_score_host_ring(s, frames, n ? n : 1, 0, n, fstride, scores, best, stride, 0, nullptr);
}

int gmm_fetch_best_density(gmm_scorer* s, uint64_t callId, uint32_t* best, uint32_t stride) {
    if (!s || !best)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if (callId == 0 || callId != s->keptCall)
        return fail(GMM_ERR_INVALID_ARGUMENT, "no best densities kept for this call");
    const uint32_t n = static_cast<uint32_t>(s->keptPos.size());
    for (uint32_t e = 0; e < s->M; ++e)
        for (uint32_t i = 0; i < n; ++i) {
            const size_t o = s->keptFrameMajor ? static_cast<size_t>(s->keptPos[i]) * stride + e
                                               : static_cast<size_t>(e) * stride + s->keptPos[i];
            best[o] = s->kept[static_cast<size_t>(e) * n + i];
        }
    return GMM_OK;
}

int gmm_best_density_pairs(gmm_scorer* s, uint64_t callId, const uint32_t* positions, const uint32_t* mixtures,
                           uint32_t nPairs, uint32_t* best) {
    if (!s || (nPairs && (!positions || !mixtures || !best)))
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if (callId == 0 || callId != s->keptCall)
        return fail(GMM_ERR_INVALID_ARGUMENT, "no frames kept for this call");
    const uint32_t n = static_cast<uint32_t>(s->keptPos.size());
    for (uint32_t j = 0; j < nPairs; ++j) {
        uint32_t i = 0;
        while (i < n && s->keptPos[i] != positions[j])
            ++i;
        if (i == n || mixtures[j] >= s->M)
            return fail(GMM_ERR_INVALID_ARGUMENT, "position not scored by this call or mixture out of range");
        best[j] = s->kept[static_cast<size_t>(mixtures[j]) * n + i];
    }
    return GMM_OK;
}

int gmm_best_density_pairs_device(gmm_scorer*, const float*, uint32_t, uint32_t, const uint32_t*, const uint32_t*,
                                  uint32_t, uint32_t*, void*) {
    return fail(GMM_ERR_UNSUPPORTED, "stand-in: no device memory");
}

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

// mixture-set files are not part of this harness
int gmm_mixture_set_read(const char*, uint32_t, uint32_t, gmm_mixture_set*) {
    return fail(GMM_ERR_UNSUPPORTED, "stand-in: no file reader");
}
int gmm_mixture_set_free(gmm_mixture_set*) { return GMM_OK; }

}  // extern "C"
