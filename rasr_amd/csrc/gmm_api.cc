// gmm_api.cc -- C-ABI of the MI355X GMM feature scorer (include/rasr_gmm.h).
//
// One handle = one prepared model resident on one GPU (tiles, row constants,
// scaled inverse deviations) plus frame staging buffers sized for
// config.max_frames.  gmm_score_device enqueues two kernels on the caller's
// stream: the frame preparation (quantize / scale the feature vectors, the
// per-frame Context of the reference, SimdFeatureScorer.cc:22-35) and the
// scorer.  No host synchronisation, no allocation on that path.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: the library is opened at run time (Rccl below)

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rasr_gmm.h"
#include "gmm_hostio.hh"
#include "gmm_kernels.hh"
#include "gmm_prepare.hh"
#include "gmm_presel.hh"
#include "gmm_shard.hh"
#include "kernel_id.h"  // build/kernel_id.h (Makefile): GMM_KERNEL_ID

using namespace rasr_gmm;

namespace {

thread_local std::string gLastError;

int fail(int code, const std::string& msg) {
    gLastError = msg;
    return code;
}

#define GMM_HIP_CHECK(expr)                                                                         \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess)                                                                       \
            return fail(GMM_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));        \
    } while (0)

// RCCL, opened on first use by a density-sharded handle with the RCCL exchange: single-GPU users of the library
// need no RCCL installation, and the library has no link-time dependency on it
struct Rccl {
    ncclResult_t (*commInitAll)(ncclComm_t*, int, const int*)                                           = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t)                                                             = nullptr;
    ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*groupStart)()                                                                        = nullptr;
    ncclResult_t (*groupEnd)()                                                                          = nullptr;
    const char* (*errorString)(ncclResult_t)                                                            = nullptr;
    std::string error;  // empty: loaded
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void*                    h = nullptr;
        std::vector<std::string> names{"librccl.so.1", "librccl.so"};
        if (const char* rocm = std::getenv("ROCM_PATH"))
            names.push_back(std::string(rocm) + "/lib/librccl.so.1");
        names.push_back("/opt/rocm/lib/librccl.so.1");
        for (const std::string& name : names)
            if ((h = dlopen(name.c_str(), RTLD_NOW | RTLD_GLOBAL)))
                break;
        if (!h) {
            const char* e = dlerror();
            x.error = std::string("cannot open librccl.so.1: ") + (e ? e : "?");
            return x;
        }
        x.commInitAll = reinterpret_cast<decltype(x.commInitAll)>(dlsym(h, "ncclCommInitAll"));
        x.commDestroy = reinterpret_cast<decltype(x.commDestroy)>(dlsym(h, "ncclCommDestroy"));
        x.allReduce   = reinterpret_cast<decltype(x.allReduce)>(dlsym(h, "ncclAllReduce"));
        x.groupStart  = reinterpret_cast<decltype(x.groupStart)>(dlsym(h, "ncclGroupStart"));
        x.groupEnd    = reinterpret_cast<decltype(x.groupEnd)>(dlsym(h, "ncclGroupEnd"));
        x.errorString = reinterpret_cast<decltype(x.errorString)>(dlsym(h, "ncclGetErrorString"));
        if (!x.commInitAll || !x.commDestroy || !x.allReduce || !x.groupStart || !x.groupEnd || !x.errorString)
            x.error = "librccl.so lacks an nccl* entry point";
        return x;
    }();
    return r;
}

template <class T>
int upload(T** dst, const std::vector<T>& src, size_t padElems = 0) {
    const size_t n = src.size() + padElems;
    if (n == 0) {
        *dst = nullptr;
        return GMM_OK;
    }
    GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dst), n * sizeof(T)));
    GMM_HIP_CHECK(hipMemset(*dst, 0, n * sizeof(T)));
    if (!src.empty())
        GMM_HIP_CHECK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return GMM_OK;
}

// gmm_score_host_ring: the caller's frames are the rows ring[(first + i) % ringSize], i < nFrames
struct HostRing {
    const float* frames;
    uint32_t     ringSize, first, nFrames, frameStride;
};

// [t0, t0 + n) of a call, copied to destination columns [col, col + n)
struct HostSegment {
    uint32_t chunk, t0, n, col;
};

struct ChunkTable {
    uint32_t  nChunks = 0;
    uint32_t* dMixOff = nullptr;
};

}  // namespace

namespace rasr_gmm {
// shared with the other C-ABI translation units (host/MixtureSetFile.cc)
void setLastError(const std::string& msg) {
    gLastError = msg;
}
}  // namespace rasr_gmm

// gmm_scorer_create_sharded: the parts of a density-sharded handle (defined below)
struct DensityGroup;
struct DensityGroupDelete {
    void operator()(DensityGroup* g) const;
};

struct gmm_scorer {
    gmm_scorer_type   type;
    Flavor            flavor;
    bool              quantized = false;
    int               device    = 0;
    gmm_scorer_config cfg{};
    uint32_t          D = 0, C = 0, nMix = 0, mixBase = 0, nTiles = 0, kSteps = 0;
    uint32_t          nFramesPad = 0;
    bool              multiCov   = false;
    bool              foldNorm   = false;
    bool              split      = false;  // float types on the split-f16 kernel
    bool              direct     = false;  // float types in the reference's operation order (scoreDirect)
    uint32_t          directL    = 0;      // row length of the direct layout
    uint32_t          kSteps16   = 0;      // split kernel: K steps (32 wide for 16-row tiles, 16 wide for 32-row)
    uint32_t          splitRows  = 16;     // split kernel tile height
    bool              splitCov   = false;  // split kernels, several covariances (covariance-free frame operand)
    uint32_t          tileBits   = 1;
    float             offsetK0   = 0;
    // density preselection (preselection-batch-*)
    bool                    presel = false;
    DensityClustering       clustering;
    void*                   dClusterMeans = nullptr;
    uint32_t*               dSelT         = nullptr;  // [nFramesPad/64][clusters][16]
    uint8_t*                dSelC         = nullptr;  // quantized: [nFramesPad/128][clusters][16] wave-table entries
    void*                   dTileClu      = nullptr;  // [tiles + pad][16]: u16 cluster * 64 (float), u32 cluster * 16 (int)
    uint32_t                lastFrames    = 0;
    // quantized scalars
    uint32_t idxBits = 1, paddedDimension = 0;
    int      scoreOnly   = kScoreOnlyNone;  // score-only layout (no best densities, cheaper epilogue): kScoreOnly*
    uint32_t* dMixOddMask = nullptr;
    float    scaling = 0, scalingSquared = 0, invQ = 0, batchScale = 0;
    std::vector<float>    isvScaled;     // [C][D] (quantized types)
    std::vector<uint32_t> mixTileOff;    // host copy
    // device model
    void*     dTileA     = nullptr;
    void*     dTileP     = nullptr;
    uint32_t* dTileCov   = nullptr;
    uint32_t* dRowDns    = nullptr;
    uint32_t* dMixTileOff = nullptr;
    float*    dIsv       = nullptr;
    float*    dCentre    = nullptr;  // float types: centre of the expanded quadratic form [D]
    float*    dDirMean   = nullptr;  // reference-order layout (PreparedDirect)
    float*    dDirConst  = nullptr;
    float*    dDirLogNorm = nullptr;
    uint32_t* dDirCov    = nullptr;
    // device frame staging
    int8_t*  dFrameQ  = nullptr;
    int32_t* dFrameSS = nullptr;
    float*   dFrameX  = nullptr;
    float*   dFrameXX = nullptr;
    void*    dFrameH  = nullptr;   // split kernel
    int32_t* dFrameExp = nullptr;
    float*   dDimScale = nullptr;
    int32_t* dLimbExp  = nullptr;
    // host-API staging
    float*    dHostFrames = nullptr;
    float*    dHostScores = nullptr;
    uint32_t* dHostBest   = nullptr;
    // gmm_score_host pipeline (large calls): scoring and copy-out streams, one event per frame chunk,
    // a double-buffered pinned staging ring for pageable destinations and its copy threads
    hipStream_t                   hostCompute = nullptr, hostCopy = nullptr;
    hipEvent_t                    hostStart   = nullptr;
    std::vector<hipEvent_t>       chunkDone;
    hipEvent_t                    stageDone[2] = {nullptr, nullptr};
    void*                         hStage       = nullptr;  // 2 x hStageBytes, hipHostMalloc
    size_t                        hStageBytes  = 0;
    std::unique_ptr<HostCopyPool> copyPool;
    std::map<uint32_t, ChunkTable> chunks;  // keyed by frame tiles per call
    // host calls (gmm_score_host*): id of the last one; the one whose best densities dHostBest keeps
    // (GMM_HOST_KEEP_BEST) with its ring mapping and copy segments, for gmm_fetch_best_density
    uint64_t                 hostCall = 0, keptBestCall = 0;
    // GMM_HOST_ASYNC: the host call in flight (0: none) and its completion, recorded on hostCopy
    uint64_t                 asyncCall = 0;
    hipEvent_t               asyncDone = nullptr;
    HostRing                 keptRing{};
    std::vector<HostSegment> keptSegs;
    bool                     keptFrameMajor = false;
    bool                     keptLazy = false, keptComputed = false;  // GMM_HOST_LAZY_BEST: computed on fetch
    float*                   dHostScoresT   = nullptr;  // frame-major copies (GMM_HOST_FRAME_MAJOR)
    uint32_t*                dHostBestT     = nullptr;
    // kernel timing (gmm_scorer_set_timing)
    bool                                        timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    size_t                                      eventsUsed = 0;
    // density-sharded handle (gmm_scorer_create_sharded): no model of its own; the parts score, this handle
    // holds the full-table host staging on devices[0]
    std::unique_ptr<DensityGroup, DensityGroupDelete> group;
    // SIMD-diagonal-maximum: the same model on the score-only class layout, which every call without a best
    // density table runs (gmm_score_device with best_density NULL, GMM_HOST_LAZY_BEST host calls): the
    // reference's score(e) without the index-carrying pack, bit-identical scores
    std::unique_ptr<gmm_scorer> scoresOnly;
    int clusteringSource = GMM_CLUSTERING_BUILT;  // preselection: built, built and written, or read from the archive
    // the caller's cache_archive string is only valid during create: keep a copy, and cfg.cache_archive stays null
    std::string cacheArchive;
    // sparse best densities (gmm_best_density_pairs, gmm_kernels_pairs.hip): entry-major tables of the assigning
    // types in the reference's arithmetic; pairKind -1 where the model has none (e.g. float D > 128)
    int       pairKind = -1;
    uint32_t  pairL = 0, pairNb = 0, pairIsvStride = 0;
    uint32_t* dPairMixOff = nullptr;
    uint32_t* dPairCov    = nullptr;
    uint8_t*  dPairQMean  = nullptr;
    int32_t*  dPairQConst = nullptr;
    float*    dPairFMean  = nullptr;
    float*    dPairFConst = nullptr;
    float*    dPairLogNorm = nullptr;
    float*    dPairIsv    = nullptr;
    // host pair lists: a page-locked staging buffer the kernel reads and writes in place (frame, mixture, best)
    uint32_t* hPairStage   = nullptr;
    size_t    pairStageCap = 0;  // pairs

    ~gmm_scorer() {
        void* ptrs[] = {dTileA,   dTileP,   dTileCov, dRowDns,     dMixTileOff, dIsv,      dFrameQ,
                        dFrameSS, dFrameX,  dFrameXX, dHostFrames, dHostScores, dHostBest, dFrameH,
                        dFrameExp, dDimScale, dLimbExp, dClusterMeans, dSelT, dSelC, dTileClu, dCentre,
                        dDirMean, dDirConst, dDirLogNorm, dDirCov, dHostScoresT, dHostBestT, dMixOddMask,
                        dPairMixOff, dPairCov, dPairQMean, dPairQConst, dPairFMean, dPairFConst, dPairLogNorm,
                        dPairIsv};
        for (void* p : ptrs)
            if (p)
                (void)hipFree(p);
        if (hPairStage)
            (void)hipHostFree(hPairStage);
        for (auto& kv : chunks)
            if (kv.second.dMixOff)
                (void)hipFree(kv.second.dMixOff);
        for (auto& ev : events) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
        for (hipEvent_t ev : chunkDone)
            (void)hipEventDestroy(ev);
        if (asyncCall && asyncDone)
            (void)hipEventSynchronize(asyncDone);  // no DMA into a caller's table may outlive the scorer
        for (hipEvent_t ev : {hostStart, stageDone[0], stageDone[1], asyncDone})
            if (ev)
                (void)hipEventDestroy(ev);
        for (hipStream_t st : {hostCompute, hostCopy})
            if (st)
                (void)hipStreamDestroy(st);
        if (hStage)
            (void)hipHostFree(hStage);
    }
};

namespace {

// the split scorer runs scoreSplitWide (gmm_kernels_split.hip launchSplitK: 16-row tiles, no preselection, not
// diagonal-sum, K steps with a wide instantiation)
bool splitWideOf(const gmm_scorer* s) {
    return s->split && s->splitRows == 16 && !s->presel && s->flavor != Flavor::DiagonalSum &&
           splitWideFrames(s->kSteps16) != 0;
}

uint32_t framesPerBlock(const gmm_scorer* s) {
    if (s->quantized)
        return s->presel ? kI8PreselFramesPerBlock
                         : (s->scoreOnly == kScoreOnlySlots ? kI8ClsFramesPerBlock : kI8FramesPerBlock);
    if (s->direct)
        return kDirectFramesPerBlock;
    if (!s->split)
        return kF32FramesPerBlock;
    return splitWideOf(s) ? splitWideFrames(s->kSteps16) : kSplitFramesPerBlock;
}

// the frame tile of one call: the quantized kernels take 256-frame tiles for calls of up to 256 frames and
// 64-frame ones (one wave per workgroup, one covariance) for calls of up to 64 (I8Args::smallTile)
int i8SmallTile(const gmm_scorer* s, uint32_t nFrames) {
    if (!s->quantized || s->presel || nFrames > kI8SmallFrames)
        return 0;
    return nFrames <= kI8TinyFrames && !s->multiCov ? 2 : 1;
}

uint32_t framesPerBlock(const gmm_scorer* s, uint32_t nFrames) {
    switch (i8SmallTile(s, nFrames)) {
        case 2: return kI8TinyFrames;
        case 1: return kI8SmallFrames;
        default: return framesPerBlock(s);
    }
}

// the selection of every frame of the call: mask words for whole 64-frame blocks (padding frames too)
int selectClustersFor(gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, uint32_t nPadCall,
                      hipStream_t stream) {
    GMM_HIP_CHECK(launchSelectClusters(s->quantized, frames, nFrames, frameStride, nPadCall, s->D,
                                       s->clustering.paddedDimension, s->dIsv, s->dClusterMeans,
                                       s->clustering.nClusters, s->clustering.nSelected, s->dSelT, stream));
    if (s->dSelC)  // the quantized kernel's per-wave tables
        GMM_HIP_CHECK(launchCompactSelection(s->dSelT, nPadCall, s->clustering.nClusters, s->dSelC, stream));
    s->lastFrames = nFrames;
    return GMM_OK;
}

// Cut the shard's mixtures into chunks of about equal tile count so that
// chunks x frame-tiles gives enough workgroups to fill 256 CUs several times.
int chunkTableFor(gmm_scorer* s, uint32_t nFrameTiles, const ChunkTable** out) {
    auto it = s->chunks.find(nFrameTiles);
    if (it != s->chunks.end()) {
        *out = &it->second;
        return GMM_OK;
    }
#ifndef GMM_TARGET_BLOCKS
#define GMM_TARGET_BLOCKS 8192
#endif
#ifndef GMM_SPLIT_TARGET_BLOCKS
// the split kernels' cap: fewer, longer chunks reload a wave's 128 frame operands less often (A/B at 32768 frames:
// 2048 -> 4.653 ms, 4096 -> 4.700, 8192 -> 4.753; at 8192 frames 1.299 / 1.309 / 1.318, profiles/r04/s13)
#define GMM_SPLIT_TARGET_BLOCKS 2048
#endif
    // RASR_GMM_TARGET_BLOCKS: tuning override (scripts/sweep_chunks.sh, scripts/sweep_small_batches.sh)
    static const uint32_t kOverride = [] {
        const char* e = std::getenv("RASR_GMM_TARGET_BLOCKS");
        const long  v = e ? std::strtol(e, nullptr, 10) : 0;
        return v > 0 ? static_cast<uint32_t>(v) : 0u;
    }();
    // Small calls (few frame tiles) with many one-mixture chunks reload the frame operands once per mixture:
    // fewer, larger chunks there (measured, profiles/r03/sweep_small_batches.txt: split kernel at 256 frames
    // 0.048 ms with 1024 blocks vs 0.063 with 8192, at 1024 frames 0.160 vs 0.175; quantized kernel at 1024
    // frames 0.0695 with 2048 vs 0.0729); large calls keep GMM_TARGET_BLOCKS
    const uint32_t kTargetBlocks =
            kOverride ? kOverride
            : s->split ? std::clamp<uint32_t>(nFrameTiles * 256u, 1024u,
                                              s->flavor == Flavor::DiagonalSum && s->splitRows == 16
                                                      ? uint32_t(GMM_TARGET_BLOCKS)  // 64-frame waves:
                                                                               : uint32_t(GMM_SPLIT_TARGET_BLOCKS))  // 8192 (A/B)
            : s->quantized && !s->presel ? std::clamp<uint32_t>(nFrameTiles * 1024u, 2048u, uint32_t(GMM_TARGET_BLOCKS))
                                         : uint32_t(GMM_TARGET_BLOCKS);
    uint32_t       target        = std::max<uint32_t>(1, (kTargetBlocks + nFrameTiles - 1) / nFrameTiles);
    // whole rounds of the 8 XCDs: mapBlock gives XCD x the chunks x, x + 8, ..., so a count just past a multiple of 8
    // leaves most XCDs idle for the last chunk (12 chunks of 171 192-frame tiles: 7.59 ms against 5.51 for 16 chunks
    // of 128 256-frame tiles at D = 45, profiles/r05/s15)
    if (target > 8)
        target = (target + 7u) / 8u * 8u;
    target                       = std::min<uint32_t>(target, std::max<uint32_t>(1, s->nMix));
    const uint32_t T             = s->nTiles;
    const uint32_t perChunk      = std::max<uint32_t>(1, (T + target - 1) / target);
    std::vector<uint32_t> off{0};
    uint32_t              acc = 0;
    for (uint32_t m = 0; m < s->nMix; ++m) {
        acc += s->mixTileOff[m + 1] - s->mixTileOff[m];
        if (acc >= perChunk && m + 1 < s->nMix) {
            off.push_back(m + 1);
            acc = 0;
        }
    }
    off.push_back(s->nMix);
    ChunkTable ct;
    ct.nChunks = static_cast<uint32_t>(off.size() - 1);
    int rc     = upload(&ct.dMixOff, off);
    if (rc != GMM_OK)
        return rc;
    auto ins = s->chunks.emplace(nFrameTiles, ct);
    *out     = &ins.first->second;
    return GMM_OK;
}

// HIP events around the scorer kernel, on the kernel's own stream (bench.py roofline timing).
struct TimedSpan {
    gmm_scorer* s;
    hipStream_t stream;
    hipEvent_t  b = nullptr, e = nullptr;
    TimedSpan(gmm_scorer* sc, hipStream_t st) : s(sc), stream(st) {}
    hipError_t begin() {
        if (!s->timing)
            return hipSuccess;
        if (s->eventsUsed == s->events.size()) {
            hipEvent_t x, y;
            hipError_t err = hipEventCreate(&x);
            if (err != hipSuccess)
                return err;
            if ((err = hipEventCreate(&y)) != hipSuccess)
                return err;
            s->events.emplace_back(x, y);
        }
        b = s->events[s->eventsUsed].first;
        e = s->events[s->eventsUsed].second;
        ++s->eventsUsed;
        return hipEventRecord(b, stream);
    }
    hipError_t end() { return s->timing ? hipEventRecord(e, stream) : hipSuccess; }
};

int groupScore(gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
               uint32_t* best, uint32_t scoreStride, hipStream_t stream);

// the GMM_HOST_ASYNC call in flight, if any, is complete on return: its staging (frames, prepared frames,
// device tables) is free for the next call of any kind
int waitAsync(gmm_scorer* s) {
    if (!s->asyncCall)
        return GMM_OK;
    s->asyncCall       = 0;
    const hipError_t e = hipEventSynchronize(s->asyncDone);
    if (e != hipSuccess)
        return fail(GMM_ERR_DEVICE, std::string("hipEventSynchronize (GMM_HOST_ASYNC call): ") + hipGetErrorString(e));
    return GMM_OK;
}

int scoreImpl(gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
              uint32_t* best, uint32_t scoreStride, hipStream_t stream) {
    if (nFrames == 0 || s->nMix == 0)
        return GMM_OK;
    if (nFrames > s->cfg.max_frames)
        return fail(GMM_ERR_CAPACITY, "n_frames exceeds config.max_frames");
    if (!frames || !scores || frameStride < s->D || scoreStride < nFrames)
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid frames/scores/stride");
    GMM_HIP_CHECK(hipSetDevice(s->device));
    if (s->group)
        return groupScore(s, frames, nFrames, frameStride, scores, best, scoreStride, stream);
    if (!best && s->scoresOnly)
        return scoreImpl(s->scoresOnly.get(), frames, nFrames, frameStride, scores, nullptr, scoreStride, stream);
    const uint32_t fpb         = framesPerBlock(s, nFrames);
    const uint32_t nFrameTiles = (nFrames + fpb - 1) / fpb;
    const uint32_t nPadCall    = nFrameTiles * fpb;  // rows the scorer reads
    const ChunkTable* ct       = nullptr;
    int               rc       = chunkTableFor(s, nFrameTiles, &ct);
    if (rc != GMM_OK)
        return rc;
    if (s->presel && (rc = selectClustersFor(s, frames, nFrames, frameStride, nPadCall, stream)) != GMM_OK)
        return rc;
    if (s->quantized) {
        GMM_HIP_CHECK(launchPrepareFramesI8(frames, nFrames, frameStride, s->nFramesPad, nPadCall, s->D, s->C,
                                            s->kSteps, s->dIsv, s->dFrameQ, s->dFrameSS, stream));
        I8Args a{};
        a.tileA       = s->dTileA;
        a.tileP       = s->dTileP;
        a.tileCov     = s->dTileCov;
        a.mixTileOff  = s->dMixTileOff;
        a.chunkMixOff = ct->dMixOff;
        a.frameQ      = s->dFrameQ;
        a.frameSS     = s->dFrameSS;
        a.scores      = scores;
        a.best        = s->flavor == Flavor::Simd ? best : nullptr;
        a.nFrames     = nFrames;
        a.nFramesPad  = s->nFramesPad;
        a.scoreStride = scoreStride;
        a.nChunks     = ct->nChunks;
        a.nFrameTiles = nFrameTiles;
        a.mixBase     = 0;
        a.idxBits     = s->idxBits;
        a.flavor      = s->flavor == Flavor::Simd ? 0 : 1;
        a.s2          = s->scalingSquared;
        // finalize by multiplication and two corrections (gmm_kernels_i8.hip finalizeStoreI8): b = 2 s^2 (the SIMD
        // scorer's 0.5 / s2, the batch scorers' scale_, both exactly 2 s2 in f32) and RN(1 / b) by IEEE division;
        // scales far outside a real model's range keep the division
        a.finB        = s->flavor == Flavor::Simd ? 2.0f * s->scalingSquared : s->batchScale;
        a.finInv      = 1.0f / a.finB;
        a.finInvLo    = static_cast<float>(1.0 / static_cast<double>(a.finB) - static_cast<double>(a.finInv));
        a.finDivide   = (a.finB >= 1e-30f && a.finB <= 1e30f) ? 0 : 1;
        a.batchScale  = s->batchScale;
        a.outScale    = s->cfg.score_scale;
        a.presel      = s->presel ? 1 : 0;
        a.selT        = s->dSelT;
        a.selC        = s->dSelC;
        a.tileClu     = s->dTileClu;
        a.nClusters   = s->clustering.nClusters;
        a.mixOddMask  = s->dMixOddMask;
        a.scoreOnly   = s->scoreOnly;
        a.smallTile   = i8SmallTile(s, nFrames);
        TimedSpan span(s, stream);
        GMM_HIP_CHECK(span.begin());
        GMM_HIP_CHECK(launchScoreI8(a, s->kSteps, s->multiCov, stream));
        GMM_HIP_CHECK(span.end());
    }
    else if (s->direct) {
        DirectArgs a{};
        a.mean        = s->dDirMean;
        a.isv         = s->dIsv;
        a.entryCov    = s->dDirCov;
        a.constant    = s->dDirConst;
        a.logNorm     = s->dDirLogNorm;
        a.mixOff      = s->dMixTileOff;
        a.chunkMixOff = ct->dMixOff;
        a.frames      = frames;
        a.scores      = scores;
        a.best        = s->flavor == Flavor::DiagonalMaximum ? best : nullptr;
        a.nFrames     = nFrames;
        a.frameStride = frameStride;
        a.scoreStride = scoreStride;
        a.nChunks     = ct->nChunks;
        a.nFrameTiles = nFrameTiles;
        a.D           = s->D;
        a.Dp          = s->directL;
        a.batch       = s->flavor == Flavor::BatchFloat ? 1 : 0;
        a.multiCov    = s->C > 1 ? 1 : 0;
        a.outScale    = s->cfg.score_scale;
        TimedSpan span(s, stream);
        GMM_HIP_CHECK(span.begin());
        GMM_HIP_CHECK(launchScoreDirect(a, stream));
        GMM_HIP_CHECK(span.end());
    }
    else if (s->split) {
        if (s->splitCov)
            GMM_HIP_CHECK(launchPrepareFramesSplitCov(frames, nFrames, frameStride, nPadCall, s->D, s->kSteps16, s->dCentre,
                                                      s->dDimScale, s->dLimbExp, s->dFrameH, s->dFrameExp, stream));
        else
            GMM_HIP_CHECK(launchPrepareFramesSplit(frames, nFrames, frameStride, nPadCall, s->D, s->splitRows, s->kSteps16,
                                                   s->dIsv, s->dCentre, s->dDimScale, s->dLimbExp, s->dFrameH, s->dFrameXX,
                                                   s->dFrameExp, stream));
        SplitArgs a{};
        a.tileH       = s->dTileA;
        a.mixTileOff  = s->dMixTileOff;
        a.chunkMixOff = ct->dMixOff;
        a.frameH      = s->dFrameH;
        a.frameXX     = s->dFrameXX;
        a.frameExp    = s->dFrameExp;
        a.scores      = scores;
        a.best        = s->flavor != Flavor::BatchFloat ? best : nullptr;
        a.nFrames     = nFrames;
        a.nFramesPad  = s->nFramesPad;
        a.scoreStride = scoreStride;
        a.nChunks     = ct->nChunks;
        a.nFrameTiles = nFrameTiles;
        a.mixBase     = 0;
        a.flavor      = s->flavor == Flavor::DiagonalMaximum ? 2 : (s->flavor == Flavor::DiagonalSum ? 4 : 3);
        a.tileBits    = s->tileBits;
        a.offsetK0    = s->offsetK0;
        a.outScale    = s->cfg.score_scale;
        a.presel      = s->presel ? 1 : 0;
        a.selT        = s->dSelT;
        a.tileClu     = s->dTileClu;
        a.nClusters   = s->clustering.nClusters;
        a.backoff     = s->cfg.backoff_score;
        TimedSpan span(s, stream);
        GMM_HIP_CHECK(span.begin());
        if (s->flavor == Flavor::DiagonalSum)
            GMM_HIP_CHECK(launchScoreSplitSum(a, s->splitRows, s->kSteps16, stream));
        else
            GMM_HIP_CHECK(launchScoreSplit(a, s->splitRows, s->kSteps16, stream));
        GMM_HIP_CHECK(span.end());
    }
    else {
        GMM_HIP_CHECK(launchPrepareFramesF32(frames, nFrames, frameStride, s->nFramesPad, nPadCall, s->D, s->C, s->kSteps,
                                             s->foldNorm ? 1 : 0, s->dIsv, s->dCentre, s->dFrameX, s->dFrameXX,
                                             stream));
        F32Args a{};
        a.tileA       = static_cast<const float*>(s->dTileA);
        a.tileCov     = s->dTileCov;
        a.rowDns      = s->dRowDns;
        a.mixTileOff  = s->dMixTileOff;
        a.chunkMixOff = ct->dMixOff;
        a.frameX      = s->dFrameX;
        a.frameXX     = s->dFrameXX;
        a.scores      = scores;
        a.best        = s->flavor == Flavor::DiagonalMaximum ? best : nullptr;
        a.nFrames     = nFrames;
        a.nFramesPad  = s->nFramesPad;
        a.scoreStride = scoreStride;
        a.nChunks     = ct->nChunks;
        a.nFrameTiles = nFrameTiles;
        a.mixBase     = 0;
        a.flavor      = s->flavor == Flavor::DiagonalMaximum ? 2 : 3;
        a.tileBits    = s->tileBits;
        a.offsetK0    = s->offsetK0;
        a.outScale    = s->cfg.score_scale;
        TimedSpan span(s, stream);
        GMM_HIP_CHECK(span.begin());
        GMM_HIP_CHECK(launchScoreF32(a, s->kSteps, s->multiCov, stream));
        GMM_HIP_CHECK(span.end());
    }
    return GMM_OK;
}

Flavor flavorOf(gmm_scorer_type t, bool* quantized, bool* ok) {
    *ok = true;
    switch (t) {
        case GMM_SIMD_DIAGONAL_MAXIMUM: *quantized = true; return Flavor::Simd;
        case GMM_BATCH_DIAGONAL_MAXIMUM_INT:
        case GMM_BATCH_DIAGONAL_MAXIMUM_FAST: *quantized = true; return Flavor::BatchInt;
        case GMM_DIAGONAL_MAXIMUM: *quantized = false; return Flavor::DiagonalMaximum;
        case GMM_BATCH_DIAGONAL_MAXIMUM_FLOAT: *quantized = false; return Flavor::BatchFloat;
        case GMM_BATCH_PRESELECTION_FLOAT: *quantized = false; return Flavor::BatchFloat;
        case GMM_BATCH_PRESELECTION_INT: *quantized = true; return Flavor::BatchInt;
        case GMM_DIAGONAL_SUM: *quantized = false; return Flavor::DiagonalSum;
    }
    *ok = false;
    return Flavor::Simd;
}

}  // namespace

extern "C" {

void gmm_default_config(gmm_scorer_config* cfg) {
    if (!cfg)
        return;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->mixture_weight_scale = 1.0f;
    cfg->gaussian_scale       = 1.0f;
    cfg->score_scale          = 1.0f;
    cfg->max_frames           = 4;  // "buffer-size" default, BatchFeatureScorer.cc:28-29
    cfg->clusters              = 256;  // DensityClustering.cc:19-32
    cfg->select_clusters       = 32;
    cfg->clustering_iterations = 5;
    cfg->backoff_score         = 40000.0f;
}

}  // extern "C"

namespace {

// The quantized scorer with several covariances (and the native f32 kernel) prepares the frames once per
// covariance, as the reference's Context does (SimdFeatureScorer.cc:22-35): a C x frames table.  A table past three
// quarters of the device's free memory is refused with its size (an untied 800k model at 32768 frames would need
// terabytes); the float types on the covariance-free split layout need no such table.
int checkCovarianceTable(size_t bytes, uint32_t C, uint32_t maxFrames) {
    if (C <= 1)
        return GMM_OK;
    size_t freeB = 0, totalB = 0;
    if (hipMemGetInfo(&freeB, &totalB) != hipSuccess)
        freeB = 0;
    if (bytes <= freeB / 4 * 3)
        return GMM_OK;
    char msg[320];
    std::snprintf(msg, sizeof(msg),
                  "%u covariances x %u frames need %.1f GiB of per-covariance frame operands (%.1f GiB free): lower "
                  "max_frames / buffer-size, or use a float scorer type (covariance-free layout, no such table)",
                  C, maxFrames, static_cast<double>(bytes) / (1u << 30), static_cast<double>(freeB) / (1u << 30));
    return fail(GMM_ERR_UNSUPPORTED, msg);
}

// preselection: the clustering over all entries' prepared means, the tiles' row cluster offsets and the
// per-call mask table.  rowEntry / fill: the scorer tiling (16 rows) and, for the split layout, the
// entry a padding row repeats (a padding row must be deselected with the row it copies).
int setupPreselection(gmm_scorer* s, const gmm_mixture_set& ms, const void* entryMeans, uint32_t Dp,
                      const std::vector<uint32_t>& rowEntry, const std::vector<uint32_t>* fill) {
    const uint32_t nEntries = ms.mixture_offsets[ms.n_mixtures];
    // DensityClustering::build (DensityClustering.tcc:122-155): the cached clustering if the archive holds a matching
    // one, else build it and cache it
    const std::string& archive = s->cacheArchive;
    std::vector<char> item;
    const uint32_t    nClusters = std::min(s->cfg.clusters, nEntries);  // "reducing number of clusters", cc:51-54
    const bool        cached    = !archive.empty() && nEntries > 0 && s->cfg.select_clusters >= 1 &&
                         s->cfg.select_clusters <= nClusters && readArchiveItem(archive, "density-clustering", item) &&
                         decodeClusteringItem(item, s->quantized, Dp, nClusters, nEntries, s->cfg.select_clusters,
                                              s->clustering);
    if (!cached) {
        std::string err = buildDensityClustering(s->quantized, entryMeans, nEntries, Dp, s->cfg.clusters,
                                                 s->cfg.select_clusters, s->cfg.clustering_iterations, s->clustering);
        if (!err.empty())
            return fail(GMM_ERR_INVALID_ARGUMENT, err);
        // a write failure leaves the scorer as it is (the reference logs it and goes on)
        if (!archive.empty() && !(s->cfg.flags & GMM_FLAG_CACHE_ARCHIVE_READ_ONLY) &&
            writeArchiveItem(archive, "density-clustering", encodeClusteringItem(s->clustering, nEntries)))
            s->clusteringSource = GMM_CLUSTERING_WRITTEN;
    }
    else
        s->clusteringSource = GMM_CLUSTERING_CACHED;
    const DensityClustering& dc = s->clustering;
    const uint32_t           T  = static_cast<uint32_t>(rowEntry.size() / kTileRows);
    // per tile row: the byte offset of its cluster in a wave's mask table -- the float kernel's word table
    // (u16, 64 B per cluster), the quantized kernel's byte table (u32, 16 B per cluster, whose entry nClusters is
    // "never selected": the padding rows' cluster, so a frame that selected none of a mixture's rows keeps all
    // ones; one u32 per row so a lane group's 4 rows are one aligned 16-byte word)
    const auto clusterOf = [&](uint32_t t, uint32_t r) -> uint32_t {
        uint32_t e = rowEntry[static_cast<size_t>(t) * kTileRows + r];
        if (e == UINT32_MAX && fill)
            e = (*fill)[t];
        return e == UINT32_MAX ? (s->quantized ? dc.nClusters : 0u) : dc.clusterOfEntry[e];
    };
    int rc;
    if (s->quantized) {
        // the slot kernel's LDS entries are u16 (the LUT byte offset), the key-layout kernel's u8
        const uint32_t        per = 16u * (s->scoreOnly == kScoreOnlySlots ? 2u : kI8PreselEntryBytes);
        std::vector<uint32_t> clu(static_cast<size_t>(T + kTilePad) * kTileRows, dc.nClusters * per);
        for (uint32_t t = 0; t < T; ++t)
            for (uint32_t r = 0; r < kTileRows; ++r)
                clu[static_cast<size_t>(t) * kTileRows + r] = clusterOf(t, r) * per;
        uint32_t* d = nullptr;
        rc          = upload(&d, clu);
        s->dTileClu = d;
    }
    else {
        std::vector<uint16_t> clu(static_cast<size_t>(T + kTilePad) * kTileRows, 0);
        for (uint32_t t = 0; t < T; ++t)
            for (uint32_t r = 0; r < kTileRows; ++r)
                clu[static_cast<size_t>(t) * kTileRows + r] = static_cast<uint16_t>(clusterOf(t, r) * 64u);
        uint16_t* d = nullptr;
        rc          = upload(&d, clu);
        s->dTileClu = d;
    }
    if (rc != GMM_OK)
        return rc;
    if (s->quantized)
        rc = upload(reinterpret_cast<uint8_t**>(&s->dClusterMeans), dc.meansQ);
    else
        rc = upload(reinterpret_cast<float**>(&s->dClusterMeans), dc.meansF);
    if (rc != GMM_OK)
        return rc;
    const size_t selBytes = static_cast<size_t>(s->nFramesPad / 64) * dc.nClusters * 64;
    GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dSelT), selBytes));
    GMM_HIP_CHECK(hipMemset(s->dSelT, 0xff, selBytes));
    if (s->quantized && kI8PreselNF == 8) {
        const size_t cBytes = static_cast<size_t>(s->nFramesPad / 128) * dc.nClusters * 16;
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dSelC), cBytes));
        GMM_HIP_CHECK(hipMemset(s->dSelC, 0, cBytes));
    }
    return GMM_OK;
}

// gmm_score_host / gmm_score_host_ring.  The caller's frames are the rows ring[(first + i) % ringSize],
// i < nFrames, and the scores of call frame i go to column (first + i) % ringSize of the caller's
// [nMix][scoreStride] tables (gmm_score_host: ringSize = nFrames, first = 0).  The frames are scored on
// hostCompute in frame chunks (one chunk for small tables); the copy-out of chunk k on hostCopy overlaps
// the scoring of chunk k+1.  A chunk that straddles the ring's wrap is copied out as two segments, so every
// copy has contiguous destination columns.  A pinned destination is written by the DMA engines directly;
// a pageable one goes through a pinned double-buffered staging ring: the D2H of piece j+1 is in flight
// while the copy threads move piece j into the caller's rows (the runtime's own pageable path is one
// thread, ~10 GB/s).  With GMM_HOST_KEEP_BEST the best densities stay in dHostBest (no copy) for
// gmm_fetch_best_density.
constexpr size_t   kHostPipelineBytes = size_t(8) << 20;
constexpr uint32_t kHostChunkFrames   = 8192;
constexpr uint32_t kHostMaxChunks     = 8;
constexpr size_t   kHostStageBytes    = size_t(16) << 20;

int ensureHostPipeline(gmm_scorer* s, uint32_t nChunks) {
    if (!s->hostCompute) {
        GMM_HIP_CHECK(hipStreamCreateWithFlags(&s->hostCompute, hipStreamNonBlocking));
        GMM_HIP_CHECK(hipStreamCreateWithFlags(&s->hostCopy, hipStreamNonBlocking));
        GMM_HIP_CHECK(hipEventCreateWithFlags(&s->hostStart, hipEventDisableTiming));
        for (hipEvent_t& ev : s->stageDone)
            GMM_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    while (s->chunkDone.size() < nChunks) {
        hipEvent_t ev = nullptr;
        GMM_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        s->chunkDone.push_back(ev);
    }
    return GMM_OK;
}

int ensureHostStage(gmm_scorer* s, size_t rowBytes) {
    const size_t want = std::max(kHostStageBytes, rowBytes);
    if (s->hStageBytes >= want)
        return GMM_OK;
    if (s->hStage)
        GMM_HIP_CHECK(hipHostFree(s->hStage));
    s->hStage      = nullptr;
    s->hStageBytes = 0;
    GMM_HIP_CHECK(hipHostMalloc(&s->hStage, 2 * want, hipHostMallocDefault));
    s->hStageBytes = want;
    if (!s->copyPool)
        s->copyPool.reset(new HostCopyPool(hostCopyThreads()));
    return GMM_OK;
}

// the call's frame range [t0, t0 + n) of chunk k, cut at the ring's wrap
void appendSegments(const HostRing& r, uint32_t k, uint32_t t0, uint32_t n, std::vector<HostSegment>& out) {
    const uint32_t wrap = r.ringSize - r.first;  // call frame that lands in column 0
    if (t0 < wrap && t0 + n > wrap) {
        out.push_back(HostSegment{k, t0, wrap - t0, r.first + t0});
        out.push_back(HostSegment{k, wrap, t0 + n - wrap, 0});
    }
    else
        out.push_back(HostSegment{k, t0, n, t0 < wrap ? r.first + t0 : t0 - wrap});
}

// device tables -> caller tables at the segments' ring positions, on hostCopy after each segment's chunk;
// synchronizes hostCopy.  Mixture-major: the device tables [nMix][nFrames] (dHostScores, dHostBest) into
// columns of [nMix][scoreStride]; frame-major: their transposes [nFrames][nMix] (dHostScoresT, dHostBestT)
// into rows of [ringSize][scoreStride].
int copyOutTables(gmm_scorer* s, const std::vector<HostSegment>& segs, uint32_t nFrames, bool frameMajor, float* scores,
                  uint32_t* best, uint32_t scoreStride, bool async = false) {
    struct Table {
        char*       dst;
        const char* src;
    };
    struct Copy {  // one 2D copy: `height` rows of `width` bytes
        uint32_t    chunk;
        const char* src;
        size_t      sPitch;
        char*       dst;
        size_t      dPitch, width, height;
    };
    const char* srcS = reinterpret_cast<const char*>(frameMajor ? s->dHostScoresT : s->dHostScores);
    const char* srcB = reinterpret_cast<const char*>(frameMajor ? s->dHostBestT : s->dHostBest);
    std::vector<Copy> direct, staged;
    const size_t      M = s->nMix, dPitch = static_cast<size_t>(scoreStride) * 4;
    for (Table t : {Table{reinterpret_cast<char*>(scores), srcS}, Table{reinterpret_cast<char*>(best), srcB}}) {
        if (!t.dst)
            continue;
        const bool pinned = isPinnedHost(t.dst);
        for (const HostSegment& g : segs) {
            const Copy c = frameMajor ? Copy{g.chunk, t.src + static_cast<size_t>(g.t0) * M * 4, M * 4,
                                             t.dst + static_cast<size_t>(g.col) * dPitch, dPitch, M * 4, g.n}
                                      : Copy{g.chunk, t.src + static_cast<size_t>(g.t0) * 4, static_cast<size_t>(nFrames) * 4,
                                             t.dst + static_cast<size_t>(g.col) * 4, dPitch, static_cast<size_t>(g.n) * 4, M};
            if (c.width && c.height)
                (pinned ? direct : staged).push_back(c);
        }
    }
    for (size_t i = 0; i < direct.size(); ++i) {
        const Copy& c = direct[i];
        if (i == 0 || direct[i - 1].chunk != c.chunk)
            GMM_HIP_CHECK(hipStreamWaitEvent(s->hostCopy, s->chunkDone[c.chunk], 0));
        GMM_HIP_CHECK(hipMemcpy2DAsync(c.dst, c.dPitch, c.src, c.sPitch, c.width, c.height, hipMemcpyDeviceToHost, s->hostCopy));
    }
    if (!staged.empty()) {
        size_t maxW = 4;
        for (const Copy& c : staged)
            maxW = std::max(maxW, c.width);
        int rc;
        if ((rc = ensureHostStage(s, maxW)) != GMM_OK)
            return rc;
        struct Piece {
            Copy   c;
            size_t r0, r1;
        };
        std::vector<Piece> pieces;
        for (const Copy& c : staged) {
            const size_t rows = std::max<size_t>(1, s->hStageBytes / c.width);
            for (size_t r0 = 0; r0 < c.height; r0 += rows)
                pieces.push_back(Piece{c, r0, std::min(c.height, r0 + rows)});
        }
        char* stage[2] = {static_cast<char*>(s->hStage), static_cast<char*>(s->hStage) + s->hStageBytes};
        auto  issue    = [&](size_t j) -> int {
            const Piece& p = pieces[j];
            if (j == 0 || pieces[j - 1].c.chunk != p.c.chunk)
                GMM_HIP_CHECK(hipStreamWaitEvent(s->hostCopy, s->chunkDone[p.c.chunk], 0));
            GMM_HIP_CHECK(hipMemcpy2DAsync(stage[j & 1], p.c.width, p.c.src + p.r0 * p.c.sPitch, p.c.sPitch, p.c.width,
                                           p.r1 - p.r0, hipMemcpyDeviceToHost, s->hostCopy));
            GMM_HIP_CHECK(hipEventRecord(s->stageDone[j & 1], s->hostCopy));
            return GMM_OK;
        };
        if ((rc = issue(0)) != GMM_OK)
            return rc;
        for (size_t j = 0; j < pieces.size(); ++j) {
            // stage[(j+1)&1] was drained by the host copy of piece j-1 (synchronous, below)
            if (j + 1 < pieces.size() && (rc = issue(j + 1)) != GMM_OK)
                return rc;
            GMM_HIP_CHECK(hipEventSynchronize(s->stageDone[j & 1]));
            const Piece& p   = pieces[j];
            const char*  src = stage[j & 1];
            s->copyPool->parallelFor(p.r1 - p.r0, [&](size_t b, size_t e) {
                for (size_t r = b; r < e; ++r)
                    std::memcpy(p.c.dst + (p.r0 + r) * p.c.dPitch, src + r * p.c.width, p.c.width);
            });
        }
    }
    if (async)  // page-locked destinations only (checked by the caller): nothing was staged
        return GMM_OK;
    GMM_HIP_CHECK(hipStreamSynchronize(s->hostCopy));
    return GMM_OK;
}

// frame-major copies of the device tables' columns [t0, t0 + n) (gmm_kernels_layout.hip)
int transposeChunk(gmm_scorer* s, bool scores, bool best, uint32_t t0, uint32_t n, uint32_t nFrames) {
    const uint32_t M = s->nMix;
    if (scores)
        GMM_HIP_CHECK(launchTransposeWords(reinterpret_cast<const uint32_t*>(s->dHostScores) + t0, M, n, nFrames,
                                           reinterpret_cast<uint32_t*>(s->dHostScoresT) + static_cast<size_t>(t0) * M, M,
                                           s->hostCompute));
    if (best)
        GMM_HIP_CHECK(launchTransposeWords(s->dHostBest + t0, M, n, nFrames, s->dHostBestT + static_cast<size_t>(t0) * M, M,
                                           s->hostCompute));
    return GMM_OK;
}

// Small calls (up to kSmallHostFrames frames: the drop-in's buffer sizes 1..64, RASR's default is 4) are bound by
// their fixed cost, not by PCIe bandwidth: the pipeline below spends two copy-engine transfers, two cross-stream
// events and two synchronizations on a few kilobytes.  With a page-locked ring and page-locked tables mapped at
// the same address on the device (gmm_host_alloc, hipHostMalloc), such a call runs on one stream with no copy
// engine: a kernel gathers the frame rows from the ring, the scorer runs as for any call, and the transpose (frame
// major) or a strided copy kernel (mixture major) stores the tables straight into the caller's rows over PCIe;
// one synchronization.  RASR_GMM_SMALL_HOST=0 turns it off (A/B).
constexpr uint32_t kSmallHostFrames = 64;

bool smallHostPathEnabled() {
    static const bool on = [] {
        const char* e = std::getenv("RASR_GMM_SMALL_HOST");
        return !(e && e[0] == '0');
    }();
    return on;
}

void keepBestOf(gmm_scorer* s, const HostRing& r, const std::vector<HostSegment>& segs, bool frameMajor, bool lazyBest) {
    s->keptBestCall   = s->hostCall;
    s->keptRing       = r;
    s->keptSegs       = segs;
    s->keptFrameMajor = frameMajor;
    s->keptLazy       = lazyBest;
    s->keptComputed   = !lazyBest;
}

int scoreHostSmall(gmm_scorer* s, const HostRing& r, float* scores, uint32_t* best, uint32_t scoreStride, bool keepBest,
                   bool lazyBest, bool frameMajor, bool async) {
    const uint32_t nFrames = r.nFrames, M = s->nMix;
    int            rc      = ensureHostPipeline(s, 1);
    if (rc != GMM_OK)
        return rc;
    std::vector<HostSegment> segs;
    appendSegments(r, 0, 0, nFrames, segs);
    const uint32_t D = s->D;
    GMM_HIP_CHECK(hipEventRecord(s->hostStart, nullptr));
    GMM_HIP_CHECK(hipStreamWaitEvent(s->hostCompute, s->hostStart, 0));
    for (const HostSegment& g : segs)
        GMM_HIP_CHECK(launchCopyWords2D(reinterpret_cast<const uint32_t*>(r.frames + static_cast<size_t>(g.col) * r.frameStride),
                                        r.frameStride, reinterpret_cast<uint32_t*>(s->dHostFrames + static_cast<size_t>(g.t0) * D),
                                        D, g.n, D, s->hostCompute));
    const bool withBest = best || (keepBest && !lazyBest);
    if ((rc = scoreImpl(s, s->dHostFrames, nFrames, D, s->dHostScores, withBest ? s->dHostBest : nullptr, nFrames,
                        s->hostCompute)) != GMM_OK)
        return rc;
    struct Table {
        uint32_t*       dst;
        const uint32_t* src;
    };
    for (Table t : {Table{reinterpret_cast<uint32_t*>(scores), reinterpret_cast<const uint32_t*>(s->dHostScores)},
                    Table{best, s->dHostBest}}) {
        if (!t.dst)
            continue;
        for (const HostSegment& g : segs) {
            if (frameMajor)
                GMM_HIP_CHECK(launchTransposeWords(t.src + g.t0, M, g.n, nFrames, t.dst + static_cast<size_t>(g.col) * scoreStride,
                                                   scoreStride, s->hostCompute));
            else
                GMM_HIP_CHECK(launchCopyWords2D(t.src + g.t0, nFrames, t.dst + g.col, scoreStride, M, g.n, s->hostCompute));
        }
    }
    if (keepBest)  // gmm_fetch_best_density's copies wait for this call's scorer
        GMM_HIP_CHECK(hipEventRecord(s->chunkDone[0], s->hostCompute));
    if (async) {
        if (!s->asyncDone)
            GMM_HIP_CHECK(hipEventCreateWithFlags(&s->asyncDone, hipEventDisableTiming));
        GMM_HIP_CHECK(hipEventRecord(s->asyncDone, s->hostCompute));
        s->asyncCall = s->hostCall;
    }
    else
        GMM_HIP_CHECK(hipStreamSynchronize(s->hostCompute));
    if (keepBest)
        keepBestOf(s, r, segs, frameMajor, lazyBest);
    return GMM_OK;
}

int scoreHostImpl(gmm_scorer* s, const HostRing& r, float* scores, uint32_t* best, uint32_t scoreStride, bool keepBest,
                  bool lazyBest, bool frameMajor, bool async) {
    if (r.nFrames <= kSmallHostFrames && !s->presel && !s->group && smallHostPathEnabled() && isDeviceMappedHost(r.frames) &&
        isDeviceMappedHost(scores) && (!best || isDeviceMappedHost(best)))
        return scoreHostSmall(s, r, scores, best, scoreStride, keepBest, lazyBest, frameMajor, async);
    const uint32_t fpb = framesPerBlock(s), nFrames = r.nFrames;
    // frame chunks for large tables; one chunk for preselection (gmm_scorer_cluster_selection reports the
    // last call's whole batch)
    const bool large   = static_cast<size_t>(nFrames) * std::max<uint32_t>(s->nMix, 1) * sizeof(float) >= kHostPipelineBytes;
    uint32_t   nChunks = s->presel || !large ? 1u : std::clamp<uint32_t>(nFrames / kHostChunkFrames, 1u, kHostMaxChunks);
    const uint32_t per = ((nFrames + nChunks - 1) / nChunks + fpb - 1) / fpb * fpb;
    nChunks            = (nFrames + per - 1) / per;
    int rc             = ensureHostPipeline(s, nChunks);
    if (rc != GMM_OK)
        return rc;
    std::vector<HostSegment> segs, rows;
    appendSegments(r, 0, 0, nFrames, rows);  // the frame rows: at most two contiguous runs of the ring
    for (uint32_t k = 0; k < nChunks; ++k)
        appendSegments(r, k, k * per, std::min(per, nFrames - k * per), segs);
    const size_t D = s->D;
    // after the legacy stream's earlier work (gmm_score_device callers on stream 0 share the staging)
    GMM_HIP_CHECK(hipEventRecord(s->hostStart, nullptr));
    GMM_HIP_CHECK(hipStreamWaitEvent(s->hostCompute, s->hostStart, 0));
    for (const HostSegment& g : rows)
        GMM_HIP_CHECK(hipMemcpy2DAsync(s->dHostFrames + g.t0 * D, D * sizeof(float),
                                       r.frames + static_cast<size_t>(g.col) * r.frameStride,
                                       static_cast<size_t>(r.frameStride) * sizeof(float), D * sizeof(float), g.n,
                                       hipMemcpyHostToDevice, s->hostCompute));
    const bool withBest = best || (keepBest && !lazyBest);
    for (uint32_t k = 0; k < nChunks; ++k) {
        const uint32_t t0 = k * per, n = std::min(per, nFrames - t0);
        rc = scoreImpl(s, s->dHostFrames + t0 * D, n, s->D, s->dHostScores + t0, withBest ? s->dHostBest + t0 : nullptr,
                       nFrames, s->hostCompute);
        if (rc == GMM_OK && frameMajor)
            rc = transposeChunk(s, true, best != nullptr, t0, n, nFrames);
        if (rc != GMM_OK)
            return rc;
        GMM_HIP_CHECK(hipEventRecord(s->chunkDone[k], s->hostCompute));
    }
    if ((rc = copyOutTables(s, segs, nFrames, frameMajor, scores, best, scoreStride, async)) != GMM_OK)
        return rc;
    if (async) {  // the copies wait for every chunk: their end is the call's end
        if (!s->asyncDone)
            GMM_HIP_CHECK(hipEventCreateWithFlags(&s->asyncDone, hipEventDisableTiming));
        GMM_HIP_CHECK(hipEventRecord(s->asyncDone, s->hostCopy));
        s->asyncCall = s->hostCall;
    }
    else
        GMM_HIP_CHECK(hipStreamSynchronize(s->hostCompute));
    if (keepBest)
        keepBestOf(s, r, segs, frameMajor, lazyBest);
    return GMM_OK;
}

// On an error after work was queued, wait for both pipeline streams before returning: no DMA into the
// caller's buffers and no kernel reading dHostFrames may outlive the call (later calls order only against
// the null stream).
// types with an assignment (AssigningFeatureScorer: SIMD-diagonal-maximum, diagonal-maximum, diagonal-sum)
bool hasAssignment(const gmm_scorer* s) {
    return s->flavor == Flavor::Simd || s->flavor == Flavor::DiagonalMaximum || s->flavor == Flavor::DiagonalSum;
}

int scoreHost(gmm_scorer* s, const HostRing& r, float* scores, uint32_t* best, uint32_t scoreStride, uint32_t flags,
              uint64_t* callId) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    if ((flags & ~(GMM_HOST_KEEP_BEST | GMM_HOST_FRAME_MAJOR | GMM_HOST_LAZY_BEST | GMM_HOST_ASYNC)) != 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "unknown flags");
    const bool async = (flags & GMM_HOST_ASYNC) != 0;
    if (async && ((scores && !isPinnedHost(scores)) || (best && !isPinnedHost(best))))
        return fail(GMM_ERR_INVALID_ARGUMENT, "GMM_HOST_ASYNC needs page-locked score / best tables (gmm_host_alloc)");
    int wrc = waitAsync(s);  // the previous asynchronous call's staging and tables
    if (wrc != GMM_OK)
        return wrc;
    const bool frameMajor = (flags & GMM_HOST_FRAME_MAJOR) != 0;
    if ((flags & GMM_HOST_KEEP_BEST) && (flags & GMM_HOST_LAZY_BEST))
        return fail(GMM_ERR_INVALID_ARGUMENT, "GMM_HOST_KEEP_BEST and GMM_HOST_LAZY_BEST together");
    if ((flags & (GMM_HOST_KEEP_BEST | GMM_HOST_LAZY_BEST)) && best)
        return fail(GMM_ERR_INVALID_ARGUMENT, "GMM_HOST_KEEP_BEST / GMM_HOST_LAZY_BEST with a best_density table");
    // batch types: nothing to keep
    const bool keepBest = (flags & (GMM_HOST_KEEP_BEST | GMM_HOST_LAZY_BEST)) && hasAssignment(s);
    const bool lazyBest = keepBest && (flags & GMM_HOST_LAZY_BEST);
    // a new host call replaces the best densities a previous one kept
    s->keptBestCall = 0;
    const uint64_t id = ++s->hostCall;
    if (callId)
        *callId = id;
    if (r.nFrames == 0)
        return GMM_OK;
    if (r.nFrames > s->cfg.max_frames)
        return fail(GMM_ERR_CAPACITY, "n_frames exceeds config.max_frames");
    if (!r.frames || !scores || r.frameStride < s->D || r.first >= r.ringSize || r.nFrames > r.ringSize ||
        scoreStride < (frameMajor ? s->nMix : r.ringSize))
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid frames/scores/stride/ring");
    GMM_HIP_CHECK(hipSetDevice(s->device));
    const size_t maxF = s->cfg.max_frames;
    if (!s->dHostFrames) {
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostFrames), maxF * s->D * sizeof(float)));
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostScores), maxF * std::max<uint32_t>(s->nMix, 1) * sizeof(float)));
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostBest), maxF * std::max<uint32_t>(s->nMix, 1) * sizeof(uint32_t)));
    }
    if (frameMajor && !s->dHostScoresT) {
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostScoresT), maxF * std::max<uint32_t>(s->nMix, 1) * sizeof(float)));
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dHostBestT), maxF * std::max<uint32_t>(s->nMix, 1) * sizeof(uint32_t)));
    }
    const int rc = scoreHostImpl(s, r, scores, best, scoreStride, keepBest, lazyBest, frameMajor, async);
    if (rc != GMM_OK)
        for (hipStream_t st : {s->hostCompute, s->hostCopy})
            if (st)
                (void)hipStreamSynchronize(st);
    return rc;
}


// ---------------------------------------------------------------------------------------------------------
// Density-sharded handles (gmm_scorer_create_sharded, BASELINE config 4 for a C / C++ caller): one process,
// part r of the density shard plan (gmm_shard.hh) on devices[r].  A call, on the caller's stream S of
// devices[0]:
//   every part, on its own stream after S's start event: frames -> its device (peer copy; none on devices[0]),
//     its sub-model scored into [nLocal][n], the split mixtures it holds packed into keys [nSplit][n]
//     (INT64_MAX for the ones it does not hold), then
//   the per-frame reduce of the keys, either
//     RCCL: on every GPU the keys of its other parts folded into its first part's (minIntoShardKeys), then an
//       all-reduce(MIN) over those first parts, one rank per distinct GPU (ncclGroupStart/End, one comm per GPU);
//       with every part on one GPU that is a one-rank all-reduce, which is how a one-GPU box runs this path, or
//     COPY: peer copies of every part's keys to devices[0] and minShardKeys there;
//   every part copies its whole mixtures (local rows [rowLo, rowHi)) into the full table's rows;
//   S waits for every part, unpacks the split mixtures' keys into their rows.
// The full table's other rows come straight from the parts: no all-gather (the caller reads one table).
}  // namespace

struct DensityPart {
    gmm_scorer*  scorer = nullptr;  // sub-model (null: the part holds no mixture)
    int          device = 0;
    DensityShard shard;
    uint32_t     nLocal = 0, rowLo = 0, rowHi = 0;             // rows [rowLo, rowHi): whole mixtures
    std::vector<std::pair<uint32_t, uint32_t>> held;           // (split slot, local row)
    uint32_t*    dHeldOffset = nullptr;                        // [held] in-mixture index of the row's first entry
    hipStream_t  stream      = nullptr;
    hipEvent_t   done        = nullptr;
    hipEvent_t   keysReady   = nullptr;  // RCCL: this part's keys packed (parts other than their GPU's first)
    std::vector<uint32_t> fold;          // RCCL: the other parts on this part's GPU (this part is their first)
    float*       dFrames     = nullptr;  // [maxF][D] (parts not on devices[0])
    float*       dScores     = nullptr;  // [nLocal][maxF]
    uint32_t*    dBest       = nullptr;
    int64_t*     dKeys       = nullptr;  // [nSplit][maxF]
};

struct DensityGroup {
    std::vector<DensityPart> parts;
    std::vector<uint32_t>    split;  // mixtures held by more than one part
    int                      exchange = GMM_EXCHANGE_AUTO;
    std::vector<uint32_t>    ranks;  // RCCL: the first part on each distinct GPU, in device-list order
    std::vector<ncclComm_t>  comms;  // RCCL: one per entry of ranks
    int                      lead     = 0;        // devices[0]
    int64_t*                 dGather  = nullptr;  // COPY: [parts][nSplit][maxF] on the lead
    int64_t*                 dReduced = nullptr;  // COPY: [nSplit][maxF]
    hipEvent_t               start = nullptr, finish = nullptr;  // on the caller's stream (lead)
    bool                     timing = false;

    ~DensityGroup() {
        for (DensityPart& p : parts) {
            (void)hipSetDevice(p.device);
            if (p.stream)
                (void)hipStreamSynchronize(p.stream);
        }
        for (ncclComm_t c : comms)
            if (c)
                (void)rccl().commDestroy(c);
        for (DensityPart& p : parts) {
            (void)hipSetDevice(p.device);
            for (void* q : {static_cast<void*>(p.dHeldOffset), static_cast<void*>(p.dFrames), static_cast<void*>(p.dScores),
                            static_cast<void*>(p.dBest), static_cast<void*>(p.dKeys)})
                if (q)
                    (void)hipFree(q);
            for (hipEvent_t ev : {p.done, p.keysReady})
                if (ev)
                    (void)hipEventDestroy(ev);
            if (p.stream)
                (void)hipStreamDestroy(p.stream);
            if (p.scorer)
                delete p.scorer;
        }
        (void)hipSetDevice(lead);
        for (void* q : {static_cast<void*>(dGather), static_cast<void*>(dReduced)})
            if (q)
                (void)hipFree(q);
        for (hipEvent_t ev : {start, finish})
            if (ev)
                (void)hipEventDestroy(ev);
    }
};

namespace {

#define GMM_NCCL_CHECK(expr)                                                                        \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess)                                                                      \
            return fail(GMM_ERR_DEVICE, std::string(#expr) + ": " + rccl().errorString(r_));      \
    } while (0)

int groupScore(gmm_scorer* s, const float* frames, uint32_t n, uint32_t frameStride, float* scores, uint32_t* best,
               uint32_t scoreStride, hipStream_t stream) {
    DensityGroup&  g        = *s->group;
    const size_t   nS       = g.split.size(), keyN = nS * n, D = s->D;
    const bool     withBest = best && hasAssignment(s);
    const uint32_t P        = static_cast<uint32_t>(g.parts.size());
    // the parts' buffers are free once the previous call's reads of them (on its stream) are done
    GMM_HIP_CHECK(hipStreamWaitEvent(stream, g.finish, 0));
    GMM_HIP_CHECK(hipEventRecord(g.start, stream));
    for (DensityPart& p : g.parts) {
        GMM_HIP_CHECK(hipSetDevice(p.device));
        GMM_HIP_CHECK(hipStreamWaitEvent(p.stream, g.start, 0));
        const float* f  = frames;
        uint32_t     fs = frameStride;
        if (p.dFrames) {
            GMM_HIP_CHECK(hipMemcpy2DAsync(p.dFrames, D * sizeof(float), frames, static_cast<size_t>(frameStride) * sizeof(float),
                                           D * sizeof(float), n, hipMemcpyDefault, p.stream));
            f = p.dFrames, fs = s->D;
        }
        int rc;
        if (p.scorer && (rc = scoreImpl(p.scorer, f, n, fs, p.dScores, withBest ? p.dBest : nullptr, n, p.stream)) != GMM_OK)
            return rc;
        if (nS) {
            GMM_HIP_CHECK(launchFillShardKeys(p.dKeys, keyN, p.stream));
            for (size_t h = 0; h < p.held.size(); ++h) {
                const uint32_t slot = p.held[h].first, row = p.held[h].second;
                GMM_HIP_CHECK(launchPackShardKeys(p.dScores + static_cast<size_t>(row) * n,
                                                  withBest ? p.dBest + static_cast<size_t>(row) * n : nullptr,
                                                  p.dHeldOffset + h, 1, n, n, p.dKeys + static_cast<size_t>(slot) * n,
                                                  p.stream));
            }
            if (p.keysReady)
                GMM_HIP_CHECK(hipEventRecord(p.keysReady, p.stream));
        }
    }
    // the per-frame reduce of the split mixtures
    const int64_t* reduced = nullptr;
    if (nS && g.exchange == GMM_EXCHANGE_RCCL) {
        // on every GPU: its other parts' keys folded into its first part's, on that part's stream
        for (uint32_t r : g.ranks) {
            DensityPart& lead = g.parts[r];
            GMM_HIP_CHECK(hipSetDevice(lead.device));
            for (uint32_t f : lead.fold) {
                GMM_HIP_CHECK(hipStreamWaitEvent(lead.stream, g.parts[f].keysReady, 0));
                GMM_HIP_CHECK(launchMinIntoShardKeys(lead.dKeys, g.parts[f].dKeys, keyN, lead.stream));
            }
        }
        // across GPUs: all-reduce(MIN) in place, one rank per GPU
        const Rccl& x = rccl();
        GMM_NCCL_CHECK(x.groupStart());
        ncclResult_t nr = ncclSuccess;
        hipError_t   hr = hipSuccess;
        for (size_t i = 0; i < g.ranks.size() && nr == ncclSuccess && hr == hipSuccess; ++i) {
            DensityPart& p = g.parts[g.ranks[i]];
            if ((hr = hipSetDevice(p.device)) == hipSuccess)
                nr = x.allReduce(p.dKeys, p.dKeys, keyN, ncclInt64, ncclMin, g.comms[i], p.stream);
        }
        const ncclResult_t ne = x.groupEnd();  // always closes the group, also after a failed enqueue
        if (hr != hipSuccess)
            return fail(GMM_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(hr));
        GMM_NCCL_CHECK(nr);
        GMM_NCCL_CHECK(ne);
        reduced = g.parts[0].dKeys;  // part 0 is the first part on the lead device
    }
    else if (nS) {
        for (uint32_t i = 0; i < P; ++i) {
            DensityPart& p = g.parts[i];
            GMM_HIP_CHECK(hipSetDevice(p.device));
            GMM_HIP_CHECK(hipMemcpyPeerAsync(g.dGather + i * keyN, g.lead, p.dKeys, p.device, keyN * sizeof(int64_t), p.stream));
        }
        reduced = g.dReduced;
    }
    // whole mixtures straight into the full table
    for (DensityPart& p : g.parts) {
        GMM_HIP_CHECK(hipSetDevice(p.device));
        const size_t rows = p.rowHi - p.rowLo;
        if (rows) {
            const size_t dst = static_cast<size_t>(p.shard.mixBegin + p.rowLo) * scoreStride, src = static_cast<size_t>(p.rowLo) * n;
            GMM_HIP_CHECK(hipMemcpy2DAsync(scores + dst, static_cast<size_t>(scoreStride) * 4, p.dScores + src, static_cast<size_t>(n) * 4,
                                           static_cast<size_t>(n) * 4, rows, hipMemcpyDefault, p.stream));
            if (withBest)
                GMM_HIP_CHECK(hipMemcpy2DAsync(best + dst, static_cast<size_t>(scoreStride) * 4, p.dBest + src,
                                               static_cast<size_t>(n) * 4, static_cast<size_t>(n) * 4, rows, hipMemcpyDefault,
                                               p.stream));
        }
        GMM_HIP_CHECK(hipEventRecord(p.done, p.stream));
    }
    GMM_HIP_CHECK(hipSetDevice(g.lead));
    for (DensityPart& p : g.parts)
        GMM_HIP_CHECK(hipStreamWaitEvent(stream, p.done, 0));
    if (nS && g.exchange != GMM_EXCHANGE_RCCL)
        GMM_HIP_CHECK(launchMinShardKeys(g.dGather, P, keyN, g.dReduced, stream));
    for (size_t i = 0; i < nS; ++i) {
        const size_t row = static_cast<size_t>(g.split[i]) * scoreStride;
        GMM_HIP_CHECK(launchUnpackShardKeys(reduced + i * n, 1, n, scores + row, withBest ? best + row : nullptr, scoreStride,
                                            stream));
    }
    GMM_HIP_CHECK(hipEventRecord(g.finish, stream));
    return GMM_OK;
}

// the handle whose prepared model answers model queries (quantization, launch info): a part's
const gmm_scorer* modelOf(const gmm_scorer* s) {
    if (s && s->group)
        for (const DensityPart& p : s->group->parts)
            if (p.scorer)
                return p.scorer;
    return s;
}

bool minReducible(gmm_scorer_type t) {
    return t == GMM_SIMD_DIAGONAL_MAXIMUM || t == GMM_DIAGONAL_MAXIMUM || t == GMM_BATCH_DIAGONAL_MAXIMUM_FLOAT ||
           t == GMM_BATCH_DIAGONAL_MAXIMUM_INT || t == GMM_BATCH_DIAGONAL_MAXIMUM_FAST;
}

}  // namespace

void DensityGroupDelete::operator()(DensityGroup* g) const {
    delete g;
}

namespace {
}  // namespace

namespace {

// gmm_best_density_pairs' entry-major tables (the assigning types): SIMD-diagonal-maximum the reference's prepared
// u8 means and constant weights of the shard's entries (q: the scorer's own preparation, dIsv its isv * s rows);
// diagonal-maximum / diagonal-sum the direct scorer's reference-order rows (prepareDirect).  A model the direct
// layout does not take (D > 128) has no sparse path: gmm_best_density_pairs reports it, the caller refills.
int setupPairs(gmm_scorer* s, const gmm_mixture_set& ms, ShardRange shard, const PreparedQuantized* q) {
    if (shard.begin == 0 && shard.end == 0)
        shard.end = ms.n_mixtures;
    const uint32_t eb = ms.mixture_offsets[shard.begin], ee = ms.mixture_offsets[shard.end];
    std::vector<uint32_t> mixOff(shard.end - shard.begin + 1), cov(ee - eb);
    for (uint32_t m = shard.begin; m <= shard.end; ++m)
        mixOff[m - shard.begin] = ms.mixture_offsets[m] - eb;
    for (uint32_t e = eb; e < ee; ++e)
        cov[e - eb] = ms.density_covariance[ms.mixture_densities[e]];
    int rc = GMM_OK;
    if (s->flavor == Flavor::Simd) {
        if (!q)
            return GMM_OK;
        const size_t         Dp = q->paddedDimension;
        std::vector<uint8_t> mean(q->preparedMean.begin() + eb * Dp, q->preparedMean.begin() + ee * Dp);
        std::vector<int32_t> cst(q->constantWeight.begin() + eb, q->constantWeight.begin() + ee);
        if ((rc = upload(&s->dPairQMean, mean)) || (rc = upload(&s->dPairQConst, cst)))
            return rc;
        s->pairIsvStride = q->kSteps * kI8K;  // dIsv: [C][kSteps * 64]
        s->pairKind      = kPairSimd;
    }
    else if (s->flavor == Flavor::DiagonalMaximum || s->flavor == Flavor::DiagonalSum) {
        PreparedDirect p;
        const uint32_t nb = directBlocks(ms.dimension, false);
        if (nb == 0 || !prepareDirect(ms, Flavor::DiagonalMaximum, s->cfg.mixture_weight_scale, s->cfg.gaussian_scale,
                                      shard, nb, p).empty())
            return GMM_OK;
        if ((rc = upload(&s->dPairFMean, p.mean)) || (rc = upload(&s->dPairFConst, p.constant)) ||
            (rc = upload(&s->dPairLogNorm, p.logNorm)) || (rc = upload(&s->dPairIsv, p.isv)))
            return rc;
        s->pairL    = p.L;
        s->pairNb   = p.nb;
        s->pairKind = s->flavor == Flavor::DiagonalSum ? kPairDiagonalSum : kPairDiagonalMaximum;
    }
    else
        return GMM_OK;
    if ((rc = upload(&s->dPairMixOff, mixOff)) || (rc = upload(&s->dPairCov, cov)))
        s->pairKind = -1;
    return rc;
}

// classLayout: lay the quantized model out for the score-only kernel (gmm_prepare.cc buildClassLayout) whatever
// the type (the SIMD scorer's scoresOnly twin); batch-int/-fast use it by default
int createScorer(const gmm_mixture_set* ms, gmm_scorer_type type, const gmm_scorer_config* config, int device,
                 bool classLayout, gmm_scorer** out) {
    if (!ms || !out)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    bool   quantized = false, ok = false;
    Flavor flavor    = flavorOf(type, &quantized, &ok);
    if (!ok)
        return fail(GMM_ERR_UNSUPPORTED, "unknown feature scorer type");
    gmm_scorer_config cfg;
    gmm_default_config(&cfg);
    if (config)
        cfg = *config;
    if (cfg.max_frames == 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "max_frames must be > 0");
    // BatchUnrolledIntFeatureScorer (BatchFeatureScorer.cc:550-604): padded dimension > 48 is refused by the
    // reference itself (cc:552-555); below 48 its unrolled loop still loads 3 x 16 bytes per row and steps the
    // means by 48 bytes (cc:591) across rows laid out at the padded dimension (cc:367-375), reading other rows
    // and past its allocation -- undefined, so refused here; at exactly 48 it is batch-int's arithmetic.
    if (type == GMM_BATCH_DIAGONAL_MAXIMUM_FAST && (ms->dimension + 15) / 16 * 16 > 48)
        return fail(GMM_ERR_UNSUPPORTED, "This feature scorer supports only features with max. 48 components");
    if (type == GMM_BATCH_DIAGONAL_MAXIMUM_FAST && (ms->dimension + 15) / 16 * 16 < 48)
        return fail(GMM_ERR_UNSUPPORTED, "batch-diagonal-maximum-fast needs 33..48 components (padded dimension 48): "
                                         "the reference's fixed 48-byte loads are undefined for smaller dimensions; "
                                         "use batch-diagonal-maximum-int");
    const bool presel = type == GMM_BATCH_PRESELECTION_FLOAT || type == GMM_BATCH_PRESELECTION_INT;
    const bool direct = (cfg.flags & GMM_FLAG_REFERENCE_ORDER) != 0;
    if (direct && type != GMM_DIAGONAL_MAXIMUM && type != GMM_BATCH_DIAGONAL_MAXIMUM_FLOAT)
        return fail(GMM_ERR_UNSUPPORTED, "the reference-order flag applies to diagonal-maximum and "
                                         "batch-diagonal-maximum-float only");
    if (presel && (cfg.clusters == 0 || cfg.clusters > 256))
        return fail(GMM_ERR_INVALID_ARGUMENT, "clusters must be in [1, 256]");
    if (presel && (cfg.flags & (GMM_FLAG_NATIVE_F32 | GMM_FLAG_SPLIT_TILE32)))
        return fail(GMM_ERR_UNSUPPORTED, "preselection runs on the 16-row split-f16 / quantized kernels only");
    ShardRange shard{cfg.mixture_begin, cfg.mixture_end};

    auto s      = std::make_unique<gmm_scorer>();
    s->type     = type;
    s->flavor   = flavor;
    s->quantized = quantized;
    s->device   = device;
    s->cfg      = cfg;
    s->cacheArchive      = cfg.cache_archive ? cfg.cache_archive : "";
    s->cfg.cache_archive = nullptr;
    s->D        = ms->dimension;
    s->C        = ms->n_covariances;
    s->nFramesPad = (cfg.max_frames + kFramePadQuantum - 1) / kFramePadQuantum * kFramePadQuantum;
    s->presel     = presel;

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(GMM_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= ndev)
        return fail(GMM_ERR_INVALID_ARGUMENT, "device index out of range");
    GMM_HIP_CHECK(hipSetDevice(device));

    const Tiling* tiling = nullptr;
    int           rc     = GMM_OK;
    if (quantized) {
        PreparedQuantized p;
        // batch types have no best densities: the score-only class layout where it applies
        // (preselection-batch-int included: the kernel masks the class layout's candidates)
        // (preselection-batch-int included: the kernel masks the slot layout's candidates)
        const bool        scoreOnlyLayout =
                classLayout || (flavor == Flavor::BatchInt && !(cfg.flags & GMM_FLAG_FULL_KEYS));
        std::string       err = prepareQuantized(*ms, flavor, shard, p,
                                                 scoreOnlyLayout ? kScoreOnlySlots : kScoreOnlyNone);
        if (!err.empty())
            return fail(GMM_ERR_INVALID_ARGUMENT, err);
        s->scoreOnly = p.scoreOnly;
        // scoreI8Cls workgroups of kI8ClsFramesPerBlock frames: the frame tables hold whole workgroups
        if (s->scoreOnly == kScoreOnlySlots && !presel && kI8ClsFramesPerBlock > kFramePadQuantum)
            s->nFramesPad = (cfg.max_frames + kI8ClsFramesPerBlock - 1) / kI8ClsFramesPerBlock * kI8ClsFramesPerBlock;
        if (p.scoreOnly && (rc = upload(&s->dMixOddMask, p.mixOddMask)) != GMM_OK)
            return rc;
        s->nMix            = p.nMixtures;
        s->kSteps          = p.kSteps;
        s->idxBits         = p.idxBits;
        s->paddedDimension = p.paddedDimension;
        s->scaling         = p.scaling;
        s->scalingSquared  = p.scalingSquared;
        s->invQ            = p.inverseQuantizationFactor;
        s->batchScale      = p.batchScale;
        s->isvScaled       = p.isvScaled;
        s->multiCov        = s->C > 1;
        s->nTiles          = p.tiling.nTiles;
        s->mixTileOff      = p.tiling.mixTileOffset;
        // preselection-batch-int compares keys biased by 2^31 as unsigned (gmm_kernels_i8.hip, PRESEL)
        if (presel)
            for (int32_t& v : p.tileP)
                v = static_cast<int32_t>(static_cast<uint32_t>(v) ^ 0x80000000u);
        // one zero padding tile so the kernels may prefetch tile t+1 unconditionally
        // kTilePad zero tiles at the end: the kernels prefetch two tiles ahead without bound checks
        if ((rc = upload(reinterpret_cast<int8_t**>(&s->dTileA), p.tileA, kTilePad * kLanes * 16 * p.kSteps)) ||
            (rc = upload(reinterpret_cast<int32_t**>(&s->dTileP), p.tileP, kTilePad * kTileRows)) ||
            (rc = upload(&s->dTileCov, p.tiling.tileCovariance, kTilePad)) ||
            (rc = upload(&s->dMixTileOff, s->mixTileOff)) ||
            (rc = upload(&s->dIsv, p.isvDevice)))
            return rc;
        const size_t nQ = static_cast<size_t>(s->C) * s->nFramesPad;
        if ((rc = checkCovarianceTable(nQ * (s->kSteps * kI8K + sizeof(int32_t)), s->C, cfg.max_frames)) != GMM_OK)
            return rc;
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dFrameQ), nQ * s->kSteps * kI8K));
        GMM_HIP_CHECK(hipMemset(s->dFrameQ, 0, nQ * s->kSteps * kI8K));
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dFrameSS), nQ * sizeof(int32_t)));
        GMM_HIP_CHECK(hipMemset(s->dFrameSS, 0, nQ * sizeof(int32_t)));
        (void)tiling;
        // BatchPreselectionIntFeatureScorer::init: clustering_->build(means_) over the u8 means
        if (presel && (rc = setupPreselection(s.get(), *ms, p.preparedMean.data(), p.paddedDimension,
                                              p.tiling.rowEntry, nullptr)) != GMM_OK)
            return rc;
        if (!classLayout && (rc = setupPairs(s.get(), *ms, shard, &p)) != GMM_OK)
            return rc;
    }
    else if (direct) {
        PreparedDirect p;
        std::string    err = prepareDirect(*ms, flavor, cfg.mixture_weight_scale, cfg.gaussian_scale, shard,
                                           directBlocks(ms->dimension, flavor == Flavor::BatchFloat), p);
        if (!err.empty())
            return fail(GMM_ERR_INVALID_ARGUMENT, err);
        s->direct     = true;
        s->directL    = p.L;
        s->nMix       = p.nMixtures;
        s->multiCov   = s->C > 1;
        s->nTiles     = p.nEntries;  // chunks are cut by entries (chunkTableFor)
        s->mixTileOff = p.mixOff;
        if ((rc = upload(&s->dDirMean, p.mean)) || (rc = upload(&s->dIsv, p.isv)) || (rc = upload(&s->dDirCov, p.entryCov)) ||
            (rc = upload(&s->dDirConst, p.constant)) || (rc = upload(&s->dDirLogNorm, p.logNorm)) ||
            (rc = upload(&s->dMixTileOff, s->mixTileOff)) || (rc = setupPairs(s.get(), *ms, shard, nullptr)))
            return rc;
    }
    else {
        PreparedFloat p;
        std::string   err = prepareFloat(*ms, flavor, cfg.mixture_weight_scale, cfg.gaussian_scale, shard, p,
                                         (cfg.flags & GMM_FLAG_NATIVE_F32) == 0,
                                         (presel || (cfg.flags & GMM_FLAG_SPLIT_TILE16))
                                                 ? 16u
                                                 : ((cfg.flags & GMM_FLAG_SPLIT_TILE32) ? 32u : 0u));
        if (!err.empty())
            return fail(GMM_ERR_INVALID_ARGUMENT, err);
        if (presel && (!p.split || p.splitRows != 16))
            return fail(GMM_ERR_UNSUPPORTED, "preselection-batch-float needs the 16-row split-f16 layout (one "
                                             "covariance, dimension <= 83, <= 1024 densities per mixture)");
        s->split    = p.split;
        s->splitCov = p.splitCov;
        s->kSteps16 = p.kSteps16;
        s->splitRows = p.splitRows;
        // wide workgroups of 192 frames (K steps 5) read up to 191 rows past the call: room for them in the frame
        // tables, which are laid out in 512-frame quanta
        if (splitWideOf(s.get()) && kSplitFramesPerBlock % splitWideFrames(s->kSteps16) != 0)
            s->nFramesPad = (cfg.max_frames + splitWideFrames(s->kSteps16) + kFramePadQuantum - 1) / kFramePadQuantum *
                            kFramePadQuantum;
        s->nMix       = p.nMixtures;
        s->kSteps     = p.kSteps;
        s->multiCov   = s->C > 1;
        s->foldNorm   = p.foldNorm;
        s->tileBits   = p.split ? p.splitKeyBits : p.tileBits;  // split kernel: key bits
        s->offsetK0   = p.offsetK0;
        s->nTiles     = p.tiling.nTiles;
        s->mixTileOff = p.tiling.mixTileOffset;
        if (s->split) {
            const std::vector<int32_t> limbs(p.limbExp, p.limbExp + kSplitLimbs);
            const size_t nH = static_cast<size_t>(s->nFramesPad) * p.kSteps16 * (p.splitRows == 32 ? 16 : 32);
            if ((rc = upload(reinterpret_cast<uint16_t**>(&s->dTileA), p.tileH, kTilePad * kLanes * 8 * p.kSteps16)) ||
                (rc = upload(&s->dDimScale, p.dimScale)) || (rc = upload(&s->dLimbExp, limbs)) ||
                (rc = upload(&s->dMixTileOff, s->mixTileOff)) || (rc = upload(&s->dIsv, p.isvDevice)) ||
                (rc = upload(&s->dCentre, p.centre)))
                return rc;
            GMM_HIP_CHECK(hipMalloc(&s->dFrameH, nH * sizeof(uint16_t)));
            GMM_HIP_CHECK(hipMemset(s->dFrameH, 0, nH * sizeof(uint16_t)));
            GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dFrameXX), s->nFramesPad * sizeof(float)));
            GMM_HIP_CHECK(hipMemset(s->dFrameXX, 0, s->nFramesPad * sizeof(float)));
            GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dFrameExp), s->nFramesPad * sizeof(int32_t)));
            GMM_HIP_CHECK(hipMemset(s->dFrameExp, 0, s->nFramesPad * sizeof(int32_t)));
            if (presel) {
                // BatchPreselectionFloatFeatureScorer::init: clustering over means_ = mean * isv (f32),
                // 0-padded to the batch-float padded dimension (BlockSize 8, BatchFeatureScorer.cc:145-170)
                const uint32_t     D = ms->dimension, Dp = (D + 7u) / 8u * 8u;
                const uint32_t     nEntries = ms->mixture_offsets[ms->n_mixtures];
                std::vector<float> em(static_cast<size_t>(nEntries) * Dp, 0.0f);
                for (uint32_t e = 0; e < nEntries; ++e) {
                    const float* mean = ms->means + static_cast<size_t>(ms->density_mean[ms->mixture_densities[e]]) * D;
                    for (uint32_t k = 0; k < D; ++k)
                        em[static_cast<size_t>(e) * Dp + k] = mean[k] * p.isv[k];
                }
                if ((rc = setupPreselection(s.get(), *ms, em.data(), Dp, p.tiling.rowEntry, &p.splitFillEntry)) != GMM_OK)
                    return rc;
            }
            if ((rc = setupPairs(s.get(), *ms, shard, nullptr)) != GMM_OK)
                return rc;
            s->mixBase = shard.begin == 0 && shard.end == 0 ? 0 : shard.begin;
            GMM_HIP_CHECK(hipDeviceSynchronize());
            *out = s.release();
            return GMM_OK;
        }
        if ((rc = upload(reinterpret_cast<float**>(&s->dTileA), p.tileA, kTilePad * kLanes * p.kSteps)) ||
            (rc = upload(&s->dTileCov, p.tiling.tileCovariance, kTilePad)) ||
            (rc = upload(&s->dRowDns, p.tiling.rowDensityInMixture, kTilePad * kTileRows)) ||
            (rc = upload(&s->dMixTileOff, s->mixTileOff)) || (rc = upload(&s->dIsv, p.isvDevice)) ||
            (rc = upload(&s->dCentre, p.centre)))
            return rc;
        const size_t nX = static_cast<size_t>(s->C) * s->nFramesPad;
        if ((rc = checkCovarianceTable(nX * (s->kSteps * 4 + 1) * sizeof(float), s->C, cfg.max_frames)) != GMM_OK)
            return rc;
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dFrameX), nX * s->kSteps * 4 * sizeof(float)));
        GMM_HIP_CHECK(hipMemset(s->dFrameX, 0, nX * s->kSteps * 4 * sizeof(float)));
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&s->dFrameXX), nX * sizeof(float)));
        GMM_HIP_CHECK(hipMemset(s->dFrameXX, 0, nX * sizeof(float)));
        if ((rc = setupPairs(s.get(), *ms, shard, nullptr)) != GMM_OK)
            return rc;
    }
    s->mixBase = shard.begin == 0 && shard.end == 0 ? 0 : shard.begin;
    GMM_HIP_CHECK(hipDeviceSynchronize());
    *out = s.release();
    return GMM_OK;
}

}  // namespace

extern "C" {

int gmm_scorer_create(const gmm_mixture_set* ms, gmm_scorer_type type, const gmm_scorer_config* config,
                      int device, gmm_scorer** out) {
    int rc = createScorer(ms, type, config, device, false, out);
    if (rc != GMM_OK || type != GMM_SIMD_DIAGONAL_MAXIMUM || ((*out)->cfg.flags & GMM_FLAG_FULL_KEYS))
        return rc;
    gmm_scorer* s = *out;
    if (s->multiCov || s->kSteps != 1)
        return GMM_OK;  // the class layout covers one covariance and D <= 64 (the key layout serves the rest)
    if (s->cfg.flags & GMM_FLAG_NO_SCORE_ONLY_TWIN)
        return GMM_OK;  // callers that always ask for best densities (aligners): no second copy of the model
    // best effort: the twin only speeds up calls without best densities, so a twin that cannot be built (e.g. the
    // device has no room for a second copy of the model) leaves a valid scorer on the key layout
    gmm_scorer* twin = nullptr;
    if (createScorer(ms, type, &s->cfg, device, true, &twin) != GMM_OK) {
        (void)hipGetLastError();
        (void)hipSetDevice(device);
        gLastError.clear();
        return GMM_OK;
    }
    if (twin->scoreOnly)
        s->scoresOnly.reset(twin);
    else  // some row's |2 dot + Q| may leave the class layout's range
        gmm_scorer_destroy(twin);
    return GMM_OK;
}

int gmm_scorer_create_sharded(const gmm_mixture_set* ms, gmm_scorer_type type, const gmm_scorer_config* config,
                              const int* devices, uint32_t nDevices, int exchange, gmm_scorer** out) {
    if (!ms || !out || !devices || nDevices == 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument or no devices");
    *out = nullptr;
    if (exchange != GMM_EXCHANGE_AUTO && exchange != GMM_EXCHANGE_RCCL && exchange != GMM_EXCHANGE_COPY)
        return fail(GMM_ERR_INVALID_ARGUMENT, "unknown exchange");
    gmm_scorer_config cfg;
    gmm_default_config(&cfg);
    if (config)
        cfg = *config;
    if (!minReducible(type))
        return fail(GMM_ERR_UNSUPPORTED, "density sharding combines split mixtures by a minimum: SIMD-diagonal-maximum, "
                                         "diagonal-maximum and batch-diagonal-maximum-* only");
    if (cfg.mixture_begin != 0 || cfg.mixture_end != 0)
        return fail(GMM_ERR_UNSUPPORTED, "a density-sharded handle shards the whole mixture set (mixture_begin/end 0)");
    if (!(cfg.score_scale > 0.0f))
        return fail(GMM_ERR_UNSUPPORTED, "density sharding needs a positive score scale (the minimum commutes with it)");
    if (cfg.max_frames == 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "max_frames must be > 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(GMM_ERR_DEVICE, "no HIP device available");
    for (uint32_t i = 0; i < nDevices; ++i)
        if (devices[i] < 0 || devices[i] >= ndev)
            return fail(GMM_ERR_INVALID_ARGUMENT, "device index out of range");
    if (nDevices == 1)  // the unsharded scorer itself
        return gmm_scorer_create(ms, type, &cfg, devices[0], out);

    std::vector<DensityShard> plan;
    std::string               err = planDensityShards(ms->mixture_offsets, ms->n_mixtures, nDevices, plan);
    if (!err.empty())
        return fail(GMM_ERR_INVALID_ARGUMENT, err);
    std::unique_ptr<DensityGroup> g(new DensityGroup);
    g->split = splitMixtures(plan);
    g->lead  = devices[0];
    // AUTO: RCCL when the parts span several GPUs and librccl opens, else the copy exchange (it needs no library);
    // only an explicit GMM_EXCHANGE_RCCL turns a missing RCCL into an error
    std::vector<int> gpus;
    for (uint32_t i = 0; i < nDevices; ++i)
        if (std::find(gpus.begin(), gpus.end(), devices[i]) == gpus.end())
            gpus.push_back(devices[i]);
    if (g->split.empty())
        g->exchange = GMM_EXCHANGE_AUTO;
    else if (exchange == GMM_EXCHANGE_AUTO)
        g->exchange = (gpus.size() > 1 && rccl().error.empty()) ? GMM_EXCHANGE_RCCL : GMM_EXCHANGE_COPY;
    else
        g->exchange = exchange;
    if (g->exchange == GMM_EXCHANGE_RCCL && !rccl().error.empty())
        return fail(GMM_ERR_UNSUPPORTED, "the RCCL exchange: " + rccl().error);
    const size_t maxF = cfg.max_frames, nS = g->split.size();
    const auto   isSplit = [&](uint32_t m) { return std::binary_search(g->split.begin(), g->split.end(), m); };
    g->parts.resize(nDevices);
    for (uint32_t r = 0; r < nDevices; ++r) {
        DensityPart& p = g->parts[r];
        p.device       = devices[r];
        p.shard        = plan[r];
        p.nLocal       = p.shard.mixEnd - p.shard.mixBegin;
        GMM_HIP_CHECK(hipSetDevice(p.device));
        GMM_HIP_CHECK(hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking));
        GMM_HIP_CHECK(hipEventCreateWithFlags(&p.done, hipEventDisableTiming));
        if (p.nLocal) {
            // the part's sub-model: mixtures [mixBegin, mixEnd) cut to the entry range, the same densities, means
            // and covariances (so model-global preparation -- the quantization scale -- is the unsharded one)
            const uint32_t        mb = p.shard.mixBegin, eb = p.shard.entryBegin, ee = p.shard.entryEnd;
            std::vector<uint32_t> lo(p.nLocal + 1);
            for (uint32_t j = 0; j <= p.nLocal; ++j)
                lo[j] = std::min(std::max(ms->mixture_offsets[mb + j], eb), ee);
            lo[0] = std::max(eb, ms->mixture_offsets[mb]);
            const uint32_t base = lo[0];
            for (uint32_t& v : lo)
                v -= base;
            gmm_mixture_set sub     = *ms;
            sub.n_mixtures          = p.nLocal;
            sub.mixture_offsets     = lo.data();
            sub.mixture_densities   = ms->mixture_densities + base;
            sub.mixture_log_weights = ms->mixture_log_weights + base;
            int rc = gmm_scorer_create(&sub, type, &cfg, p.device, &p.scorer);
            if (rc != GMM_OK)
                return rc;
            GMM_HIP_CHECK(hipSetDevice(p.device));
            GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p.dScores), p.nLocal * maxF * sizeof(float)));
            GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p.dBest), p.nLocal * maxF * sizeof(uint32_t)));
            p.rowLo = isSplit(mb) ? 1 : 0;
            p.rowHi = isSplit(p.shard.mixEnd - 1) ? p.nLocal - 1 : p.nLocal;
            p.rowHi = std::max(p.rowHi, p.rowLo);
            std::vector<uint32_t> offsets;
            for (uint32_t i = 0; i < nS; ++i)
                if (g->split[i] >= mb && g->split[i] < p.shard.mixEnd) {
                    p.held.emplace_back(i, g->split[i] - mb);
                    offsets.push_back(g->split[i] == mb ? p.shard.firstOffset : 0);
                }
            if ((rc = upload(&p.dHeldOffset, offsets)) != GMM_OK)
                return rc;
        }
        if (nS)
            GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p.dKeys), nS * maxF * sizeof(int64_t)));
        if (p.device != g->lead) {
            GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&p.dFrames), maxF * ms->dimension * sizeof(float)));
            // xGMI peer access both ways: frames out of the lead, tables and keys into it
            int can = 0;
            GMM_HIP_CHECK(hipDeviceCanAccessPeer(&can, g->lead, p.device));
            if (!can)
                return fail(GMM_ERR_UNSUPPORTED, "devices without peer access");
            for (int a : {g->lead, p.device}) {
                GMM_HIP_CHECK(hipSetDevice(a));
                const hipError_t e = hipDeviceEnablePeerAccess(a == g->lead ? p.device : g->lead, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return fail(GMM_ERR_DEVICE, std::string("hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
                (void)hipGetLastError();
            }
        }
    }
    if (g->exchange == GMM_EXCHANGE_RCCL) {
        // one rank per GPU: the first part on each GPU; the others fold their keys into it first
        for (int d : gpus)
            for (uint32_t r = 0; r < nDevices; ++r)
                if (devices[r] == d) {
                    g->ranks.push_back(r);
                    for (uint32_t f = r + 1; f < nDevices; ++f)
                        if (devices[f] == d) {
                            g->parts[r].fold.push_back(f);
                            GMM_HIP_CHECK(hipSetDevice(d));
                            GMM_HIP_CHECK(hipEventCreateWithFlags(&g->parts[f].keysReady, hipEventDisableTiming));
                        }
                    break;
                }
        g->comms.assign(gpus.size(), nullptr);
        GMM_NCCL_CHECK(rccl().commInitAll(g->comms.data(), static_cast<int>(gpus.size()), gpus.data()));
    }
    GMM_HIP_CHECK(hipSetDevice(g->lead));
    if (g->exchange == GMM_EXCHANGE_COPY) {
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&g->dGather), nDevices * nS * maxF * sizeof(int64_t)));
        GMM_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&g->dReduced), nS * maxF * sizeof(int64_t)));
    }
    GMM_HIP_CHECK(hipEventCreateWithFlags(&g->start, hipEventDisableTiming));
    GMM_HIP_CHECK(hipEventCreateWithFlags(&g->finish, hipEventDisableTiming));

    // the handle: no model of its own; the kernel layout of the parts (frame chunking) and the full table's size
    const gmm_scorer* m = nullptr;
    for (const DensityPart& p : g->parts)
        if (p.scorer && !m)
            m = p.scorer;
    auto s        = std::make_unique<gmm_scorer>();
    s->type       = type;
    s->flavor     = m ? m->flavor : Flavor::Simd;
    s->quantized  = m ? m->quantized : false;
    s->split      = m ? m->split : false;
    s->splitCov   = m ? m->splitCov : false;
    s->direct     = m ? m->direct : false;
    s->splitRows  = m ? m->splitRows : 16;
    s->kSteps16   = m ? m->kSteps16 : 0;
    s->device     = g->lead;
    s->cfg        = cfg;
    s->cfg.cache_archive = nullptr;  // valid only during create (the parts took their copies)
    s->D          = ms->dimension;
    s->C          = ms->n_covariances;
    s->nMix       = ms->n_mixtures;
    s->nFramesPad = (cfg.max_frames + kFramePadQuantum - 1) / kFramePadQuantum * kFramePadQuantum;
    if (!m) {
        bool q = false, ok = false;
        s->flavor    = flavorOf(type, &q, &ok);
        s->quantized = q;
    }
    s->group.reset(g.release());
    *out = s.release();
    return GMM_OK;
}

int gmm_scorer_shard_info(const gmm_scorer* s, uint32_t* nParts, int* exchange) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    if (nParts)
        *nParts = s->group ? static_cast<uint32_t>(s->group->parts.size()) : 1u;
    if (exchange)
        *exchange = s->group ? s->group->exchange : GMM_EXCHANGE_AUTO;
    return GMM_OK;
}

int gmm_scorer_destroy(gmm_scorer* s) {
    if (!s)
        return GMM_OK;
    (void)hipSetDevice(s->device);
    delete s;
    return GMM_OK;
}

uint32_t gmm_scorer_n_mixtures(const gmm_scorer* s) {
    return s ? s->nMix : 0;
}

uint32_t gmm_scorer_dimension(const gmm_scorer* s) {
    return s ? s->D : 0;
}

uint32_t gmm_scorer_n_covariances(const gmm_scorer* s) {
    return s ? s->C : 0;
}

int gmm_scorer_type_of(const gmm_scorer* s) {
    return s ? static_cast<int>(s->type) : -1;
}

int gmm_score_device(gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
                     uint32_t* best, uint32_t scoreStride, void* stream) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    const int wrc = waitAsync(s);  // a GMM_HOST_ASYNC call still uses the frame staging
    if (wrc != GMM_OK)
        return wrc;
    return scoreImpl(s, frames, nFrames, frameStride, scores, best, scoreStride, static_cast<hipStream_t>(stream));
}

int gmm_score_host(gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride, float* scores,
                   uint32_t* best, uint32_t scoreStride) {
    return scoreHost(s, HostRing{frames, std::max<uint32_t>(nFrames, 1), 0, nFrames, frameStride}, scores, best,
                     scoreStride, 0, nullptr);
}

int gmm_score_host_ring(gmm_scorer* s, const float* ring, uint32_t ringSize, uint32_t first, uint32_t nFrames,
                        uint32_t frameStride, float* scores, uint32_t* best, uint32_t scoreStride, uint32_t flags,
                        uint64_t* callId) {
    return scoreHost(s, HostRing{ring, ringSize, first, nFrames, frameStride}, scores, best, scoreStride, flags, callId);
}

int gmm_host_call_wait(gmm_scorer* s, uint64_t callId) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    return callId != 0 && callId == s->asyncCall ? waitAsync(s) : GMM_OK;
}

int gmm_fetch_best_density(gmm_scorer* s, uint64_t callId, uint32_t* best, uint32_t scoreStride) {
    if (!s || !best)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    const int wrc = waitAsync(s);
    if (wrc != GMM_OK)
        return wrc;
    if (!hasAssignment(s))
        return fail(GMM_ERR_UNSUPPORTED, "scorer type has no best densities (batch types)");
    if (callId == 0 || callId != s->keptBestCall)
        return fail(GMM_ERR_INVALID_ARGUMENT, "no best densities kept for this call (a later host call replaced them)");
    if (scoreStride < (s->keptFrameMajor ? s->nMix : s->keptRing.ringSize))
        return fail(GMM_ERR_INVALID_ARGUMENT, "score_stride below the call's table layout");
    GMM_HIP_CHECK(hipSetDevice(s->device));
    int rc = GMM_OK;
    if (!s->keptComputed) {
        // GMM_HOST_LAZY_BEST: score the call's frames (still in dHostFrames) again, with best densities, in one
        // launch; its scores land in the device table only (the caller's copy stays the score-only one)
        const uint32_t n = s->keptRing.nFrames;
        rc = scoreImpl(s, s->dHostFrames, n, s->D, s->dHostScores, s->dHostBest, n, s->hostCompute);
        if (rc != GMM_OK) {
            (void)hipStreamSynchronize(s->hostCompute);
            return rc;
        }
        if (!s->keptFrameMajor)
            for (const HostSegment& g : s->keptSegs)
                GMM_HIP_CHECK(hipEventRecord(s->chunkDone[g.chunk], s->hostCompute));
        s->keptComputed = true;
    }
    if (s->keptFrameMajor) {  // transpose the kept best densities now; every chunk's copy waits for it
        if ((rc = transposeChunk(s, false, true, 0, s->keptRing.nFrames, s->keptRing.nFrames)) != GMM_OK)
            return rc;
        for (const HostSegment& g : s->keptSegs)
            GMM_HIP_CHECK(hipEventRecord(s->chunkDone[g.chunk], s->hostCompute));
    }
    // (mixture-major: the call's chunks were complete when it returned, the copies wait on events reached)
    rc = copyOutTables(s, s->keptSegs, s->keptRing.nFrames, s->keptFrameMajor, nullptr, best, scoreStride);
    if (rc != GMM_OK)
        (void)hipStreamSynchronize(s->hostCopy);
    return rc;
}

namespace {
PairArgs pairArgsOf(const gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride) {
    PairArgs a{};
    a.frames      = frames;
    a.nFrames     = nFrames;
    a.frameStride = frameStride;
    a.mixOff      = s->dPairMixOff;
    a.entryCov    = s->dPairCov;
    a.qMean       = s->dPairQMean;
    a.qConst      = s->dPairQConst;
    a.fMean       = s->dPairFMean;
    a.fConst      = s->dPairFConst;
    a.fLogNorm    = s->dPairLogNorm;
    a.isv         = s->pairKind == kPairSimd ? s->dIsv : s->dPairIsv;
    a.nMixtures   = s->nMix;
    a.D           = s->D;
    a.Dp          = s->paddedDimension;
    a.L           = s->pairL;
    a.nb          = s->pairNb;
    a.isvStride   = s->pairIsvStride;
    a.kind        = s->pairKind;
    return a;
}

int checkPairs(const gmm_scorer* s) {
    if (!hasAssignment(s))
        return fail(GMM_ERR_UNSUPPORTED, "scorer type has no best densities (batch types)");
    if (s->group || s->pairKind < 0)
        return fail(GMM_ERR_UNSUPPORTED, "no sparse best-density path for this scorer (density-sharded handle, or a "
                                         "float model of dimension > 128): use gmm_fetch_best_density");
    return GMM_OK;
}
}  // namespace

int gmm_best_density_pairs(gmm_scorer* s, uint64_t callId, const uint32_t* positions, const uint32_t* mixtures,
                           uint32_t nPairs, uint32_t* best) {
    if (!s || (nPairs && (!positions || !mixtures || !best)))
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    const int wrc = waitAsync(s);
    if (wrc != GMM_OK)
        return wrc;
    int rc = checkPairs(s);
    if (rc != GMM_OK)
        return rc;
    if (callId == 0 || callId != s->keptBestCall)
        return fail(GMM_ERR_INVALID_ARGUMENT, "no frames kept for this call (a later host call replaced them)");
    if (nPairs == 0)
        return GMM_OK;
    const HostRing& r = s->keptRing;
    GMM_HIP_CHECK(hipSetDevice(s->device));
    if (s->pairStageCap < nPairs) {
        if (s->hPairStage)
            GMM_HIP_CHECK(hipHostFree(s->hPairStage));
        s->hPairStage   = nullptr;
        s->pairStageCap = 0;
        const size_t cap = std::max<size_t>(nPairs, 256);
        GMM_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&s->hPairStage), 3 * cap * sizeof(uint32_t),
                                    hipHostMallocMapped));
        s->pairStageCap = cap;
    }
    uint32_t* st = s->hPairStage;
    for (uint32_t i = 0; i < nPairs; ++i) {
        // ring position -> frame of the call (the call's frame t sits at ring position (first + t) % ringSize)
        const uint32_t pos = positions[i];
        const uint32_t t   = pos < r.ringSize ? (pos + r.ringSize - r.first) % r.ringSize : 0xffffffffu;
        if (t >= r.nFrames)
            return fail(GMM_ERR_INVALID_ARGUMENT, "position not scored by this call");
        if (mixtures[i] >= s->nMix)
            return fail(GMM_ERR_INVALID_ARGUMENT, "mixture index out of range");
        st[i]          = t;
        st[nPairs + i] = mixtures[i];
    }
    uint32_t* dst = nullptr;
    GMM_HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dst), st, 0));
    PairArgs a  = pairArgsOf(s, s->dHostFrames, r.nFrames, s->D);
    a.pairFrame = dst;
    a.pairMix   = dst + nPairs;
    a.best      = dst + 2 * static_cast<size_t>(nPairs);
    a.nPairs    = nPairs;
    // after the call's own frame staging on hostCompute (the kernel reads dHostFrames)
    GMM_HIP_CHECK(launchBestPairs(a, s->hostCompute));
    GMM_HIP_CHECK(hipStreamSynchronize(s->hostCompute));
    std::memcpy(best, st + 2 * static_cast<size_t>(nPairs), nPairs * sizeof(uint32_t));
    return GMM_OK;
}

int gmm_best_density_pairs_device(gmm_scorer* s, const float* frames, uint32_t nFrames, uint32_t frameStride,
                                  const uint32_t* pairFrame, const uint32_t* pairMixture, uint32_t nPairs,
                                  uint32_t* best, void* stream) {
    if (!s || (nPairs && (!frames || !pairFrame || !pairMixture || !best)))
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    int rc = checkPairs(s);
    if (rc != GMM_OK)
        return rc;
    if (frameStride < s->D)
        return fail(GMM_ERR_INVALID_ARGUMENT, "frame_stride below the dimension");
    if (nPairs == 0)
        return GMM_OK;
    GMM_HIP_CHECK(hipSetDevice(s->device));
    PairArgs a  = pairArgsOf(s, frames, nFrames, frameStride);
    a.pairFrame = pairFrame;
    a.pairMix   = pairMixture;
    a.best      = best;
    a.nPairs    = nPairs;
    GMM_HIP_CHECK(launchBestPairs(a, static_cast<hipStream_t>(stream)));
    return GMM_OK;
}

int gmm_host_alloc(size_t bytes, void** ptr) {
    if (!ptr)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null ptr");
    *ptr = nullptr;
    if (bytes == 0)
        return GMM_OK;
    GMM_HIP_CHECK(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
    return GMM_OK;
}

int gmm_host_free(void* ptr) {
    if (ptr)
        GMM_HIP_CHECK(hipHostFree(ptr));
    return GMM_OK;
}

int gmm_scorer_quantization(const gmm_scorer* s, float* scaling, float* invQ) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    s = modelOf(s);  // a sharded handle: its parts share the model-global quantization scale
    if (!s->quantized)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type is not quantized");
    if (scaling)
        *scaling = s->scaling;
    if (invQ)
        *invQ = s->invQ;
    return GMM_OK;
}

int gmm_scorer_multiply_and_quantize(const gmm_scorer* s, const float* feature, uint8_t* out) {
    if (!s || !feature || !out)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    s = modelOf(s);
    if (!s->quantized)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type is not quantized");
    const uint32_t Dp = s->paddedDimension;
    for (uint32_t c = 0; c < s->C; ++c) {
        uint8_t* r = out + static_cast<size_t>(c) * Dp;
        for (uint32_t k = 0; k < s->D; ++k)
            r[k] = refQuantize(feature[k] * s->isvScaled[static_cast<size_t>(c) * s->D + k]);
        for (uint32_t k = s->D; k < Dp; ++k)
            r[k] = 0;
    }
    return GMM_OK;
}

int gmm_prepare_quantized_host(const gmm_mixture_set* ms, gmm_scorer_type type, float* scaling, float* isv,
                               float* logNorm, uint8_t* preparedMean, int32_t* constantWeight) {
    if (!ms)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null mixture set");
    bool   quantized = false, ok = false;
    Flavor flavor    = flavorOf(type, &quantized, &ok);
    if (!ok || !quantized)
        return fail(GMM_ERR_UNSUPPORTED, "type is not a quantized scorer");
    PreparedQuantized p;
    std::string       err = prepareQuantized(*ms, flavor, ShardRange{}, p);
    if (!err.empty())
        return fail(GMM_ERR_INVALID_ARGUMENT, err);
    if (scaling)
        *scaling = p.scaling;
    if (isv)
        std::copy(p.isvScaled.begin(), p.isvScaled.end(), isv);
    if (logNorm)
        std::copy(p.logNormScaled.begin(), p.logNormScaled.end(), logNorm);
    if (preparedMean)
        std::copy(p.preparedMean.begin(), p.preparedMean.end(), preparedMean);
    if (constantWeight)
        std::copy(p.constantWeight.begin(), p.constantWeight.end(), constantWeight);
    return GMM_OK;
}

int gmm_scorer_launch_info(const gmm_scorer* s, uint32_t nFrames, uint32_t* nLaunches, const char** name) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    s = modelOf(s);  // a sharded handle: per part
    (void)nFrames;
    if (nLaunches)
        *nLaunches = s->presel ? 3 : 2;
    if (name)
        *name = s->quantized ? "scoreI8" : s->direct ? "scoreDirect" : (s->split ? (s->flavor == Flavor::DiagonalSum ? (s->splitRows == 32 ? "scoreSplit32Sum" : "scoreSplitSum")
                                                                         : (s->splitRows == 32 ? "scoreSplit32" : (splitWideOf(s) ? "scoreSplitWide" : "scoreSplit")))
                                                       : "scoreF32");
    return GMM_OK;
}

int gmm_scorer_set_timing(gmm_scorer* s, int enable) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    s->timing     = enable != 0;
    s->eventsUsed = 0;
    if (s->scoresOnly)
        gmm_scorer_set_timing(s->scoresOnly.get(), enable);
    if (s->group)  // sharded: every part times its own kernels
        for (DensityPart& p : s->group->parts)
            if (p.scorer)
                gmm_scorer_set_timing(p.scorer, enable);
    return GMM_OK;
}

int gmm_scorer_kernel_time(gmm_scorer* s, double* totalMs, uint32_t* nLaunches, int reset) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    if (s->group) {  // sharded: the parts run concurrently -- the slowest part's total, its launch count
        double   worst = 0;
        uint32_t n     = 0;
        for (DensityPart& p : s->group->parts) {
            double   t = 0;
            uint32_t k = 0;
            int      rc;
            if (p.scorer && (rc = gmm_scorer_kernel_time(p.scorer, &t, &k, reset)) != GMM_OK)
                return rc;
            if (p.scorer && (t > worst || n == 0))
                worst = t, n = k;
        }
        if (totalMs)
            *totalMs = worst;
        if (nLaunches)
            *nLaunches = n;
        return GMM_OK;
    }
    GMM_HIP_CHECK(hipSetDevice(s->device));
    double total = 0;
    for (size_t i = 0; i < s->eventsUsed; ++i) {
        GMM_HIP_CHECK(hipEventSynchronize(s->events[i].second));
        float ms = 0;
        GMM_HIP_CHECK(hipEventElapsedTime(&ms, s->events[i].first, s->events[i].second));
        total += ms;
    }
    uint32_t launches = static_cast<uint32_t>(s->eventsUsed);
    if (s->scoresOnly) {  // calls without best densities ran on the twin
        double   t = 0;
        uint32_t k = 0;
        int      rc;
        if ((rc = gmm_scorer_kernel_time(s->scoresOnly.get(), &t, &k, reset)) != GMM_OK)
            return rc;
        total += t;
        launches += k;
    }
    if (totalMs)
        *totalMs = total;
    if (nLaunches)
        *nLaunches = launches;
    if (reset)
        s->eventsUsed = 0;
    return GMM_OK;
}

int gmm_scorer_density_clustering(const gmm_scorer* s, uint32_t* nClusters, uint32_t* paddedDimension,
                                  uint8_t* clusterOfEntry, void* clusterMeans) {
    if (!s)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null scorer");
    if (!s->presel)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type has no density preselection");
    const DensityClustering& dc = s->clustering;
    if (nClusters)
        *nClusters = dc.nClusters;
    if (paddedDimension)
        *paddedDimension = dc.paddedDimension;
    if (clusterOfEntry)
        std::copy(dc.clusterOfEntry.begin(), dc.clusterOfEntry.end(), clusterOfEntry);
    if (clusterMeans) {
        if (dc.quantized)
            std::copy(dc.meansQ.begin(), dc.meansQ.end(), static_cast<uint8_t*>(clusterMeans));
        else
            std::copy(dc.meansF.begin(), dc.meansF.end(), static_cast<float*>(clusterMeans));
    }
    return GMM_OK;
}

int gmm_scorer_clustering_source(const gmm_scorer* s, int* source) {
    if (!s || !source)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if (!s->presel)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type has no density preselection");
    *source = s->clusteringSource;
    return GMM_OK;
}

int gmm_cache_archive_read_item(const char* path, const char* name, void* data, uint64_t capacity, uint64_t* size) {
    if (!path || !name || !size)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    std::vector<char> item;
    if (!readArchiveItem(path, name, item))
        return fail(GMM_ERR_INVALID_ARGUMENT, std::string("no item ") + name + " in cache archive " + path);
    *size = item.size();
    if (data)
        std::memcpy(data, item.data(), std::min<uint64_t>(capacity, item.size()));
    return GMM_OK;
}

int gmm_cache_archive_write_item(const char* path, const char* name, const void* data, uint64_t size) {
    if (!path || !name || !name[0] || (size && !data))
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument or empty item name");
    const char* p = static_cast<const char*>(data);
    if (!writeArchiveItem(path, name, std::vector<char>(p, p + size)))
        return fail(GMM_ERR_INVALID_ARGUMENT, std::string("cannot write cache archive ") + path);
    return GMM_OK;
}

int gmm_scorer_cluster_selection(gmm_scorer* s, uint32_t nFrames, uint8_t* selection) {
    if (!s || !selection)
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    if (!s->presel)
        return fail(GMM_ERR_UNSUPPORTED, "scorer type has no density preselection");
    if (nFrames > s->lastFrames)
        return fail(GMM_ERR_INVALID_ARGUMENT, "n_frames exceeds the frames of the last score call");
    GMM_HIP_CHECK(hipSetDevice(s->device));
    GMM_HIP_CHECK(hipDeviceSynchronize());
    const uint32_t        nC     = s->clustering.nClusters;
    const uint32_t        blocks = (nFrames + 63) / 64;
    std::vector<uint32_t> words(static_cast<size_t>(blocks) * nC * 16);
    if (!words.empty())
        GMM_HIP_CHECK(hipMemcpy(words.data(), s->dSelT, words.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t t = 0; t < nFrames; ++t)
        for (uint32_t c = 0; c < nC; ++c) {
            const uint32_t w = words[(static_cast<size_t>(t / 64) * nC + c) * 16 + t % 16];
            selection[static_cast<size_t>(t) * nC + c] = ((w >> (8 * ((t % 64) / 16))) & 0xffu) == 0 ? 1 : 0;
        }
    return GMM_OK;
}

int gmm_density_clustering_seeds(uint32_t nEntries, uint32_t nClusters, uint32_t* seeds) {
    if (!seeds || nClusters == 0 || nClusters > nEntries)
        return fail(GMM_ERR_INVALID_ARGUMENT, "need 0 < n_clusters <= n_entries and an output array");
    const std::vector<uint32_t> v = clusteringSeeds(nEntries, nClusters);
    std::copy(v.begin(), v.end(), seeds);
    return GMM_OK;
}

int gmm_shard_pack_keys(const float* scores, const uint32_t* best, const uint32_t* bestOffset, uint32_t rows,
                        uint32_t nFrames, uint32_t stride, int64_t* keys, void* stream) {
    if (rows == 0 || nFrames == 0)
        return GMM_OK;
    if (!scores || !keys || stride < nFrames)
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid scores/keys/stride");
    GMM_HIP_CHECK(launchPackShardKeys(scores, best, bestOffset, rows, nFrames, stride, keys, static_cast<hipStream_t>(stream)));
    return GMM_OK;
}

int gmm_shard_unpack_keys(const int64_t* keys, uint32_t rows, uint32_t nFrames, float* scores, uint32_t* best,
                          uint32_t stride, void* stream) {
    if (rows == 0 || nFrames == 0)
        return GMM_OK;
    if (!scores || !keys || stride < nFrames)
        return fail(GMM_ERR_INVALID_ARGUMENT, "invalid scores/keys/stride");
    GMM_HIP_CHECK(launchUnpackShardKeys(keys, rows, nFrames, scores, best, stride, static_cast<hipStream_t>(stream)));
    return GMM_OK;
}

const char* gmm_last_error(void) {
    return gLastError.c_str();
}

const char* gmm_version(void) {
    return "rasr_amd-gmm 0.2 (gfx950)";
}

const char* gmm_kernel_id(void) {
    return GMM_KERNEL_ID;
}

}  // extern "C"
