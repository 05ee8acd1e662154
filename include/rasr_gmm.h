/*
 * rasr_gmm.h -- C-ABI of the MI355X diagonal-covariance GMM feature scorer.
 *
 * This is the drop-in boundary for RASR's acoustic scoring hot path
 * (Mm::FeatureScorer plugin surface, src/Mm/FeatureScorer.hh:28-164).  Plain
 * pointers and sizes only; no HIP or torch types.  Every entry point returns
 * an int status (GMM_OK == 0, negative on error, message via gmm_last_error());
 * nothing throws across the ABI (the reference is built -fno-exceptions,
 * config/cc-gcc.make:27).  One handle per GPU; a handle is not thread-safe
 * (RASR scorers are single-thread objects, src/Core/ReferenceCounting.hh:43-77).
 *
 * Score tables are mixture-major: score(e, t) = scores[e * score_stride + t],
 * the layout of BatchFeatureScorerBase::scores_ (src/Mm/BatchFeatureScorer.hh:177-186).
 */
#ifndef RASR_GMM_H
#define RASR_GMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GMM_OK 0
#define GMM_ERR_INVALID_ARGUMENT -1
#define GMM_ERR_UNSUPPORTED -2
#define GMM_ERR_DEVICE -3
#define GMM_ERR_OUT_OF_MEMORY -4
#define GMM_ERR_CAPACITY -5

/* Feature-scorer types; numeric values are Mm::Module_::FeatureScorerType
 * (src/Mm/Module.hh:48-70), names are the reference's registration strings
 * (src/Mm/Module.cc:84-107). */
typedef enum {
    GMM_BATCH_DIAGONAL_MAXIMUM_FLOAT = 0, /* "batch-diagonal-maximum-float" BatchFeatureScorer.cc:120-234 */
    GMM_BATCH_PRESELECTION_FLOAT     = 1, /* "preselection-batch-float"     BatchFeatureScorer.cc:238-289 */
    GMM_BATCH_PRESELECTION_INT       = 2, /* "preselection-batch-int"       BatchFeatureScorer.cc:478-533 */
    GMM_BATCH_DIAGONAL_MAXIMUM_INT   = 3, /* "batch-diagonal-maximum-int"   BatchFeatureScorer.cc:293-474 */
    GMM_BATCH_DIAGONAL_MAXIMUM_FAST  = 4, /* "batch-diagonal-maximum-fast"  BatchFeatureScorer.cc:537-604 */
    GMM_DIAGONAL_MAXIMUM             = 5, /* "diagonal-maximum"   GaussDiagonalMaximumFeatureScorer.cc */
    GMM_SIMD_DIAGONAL_MAXIMUM        = 9, /* "SIMD-diagonal-maximum" SimdFeatureScorer.cc            */
    GMM_DIAGONAL_SUM                 = 12 /* diagonalSum: GaussDiagonalSumFeatureScorer
                                             (GaussDiagonalMaximumFeatureScorer.cc:221-298), no
                                             registration string in the reference factory; here
                                             "diagonal-sum".  Split-f16 kernels only: one covariance
                                             (dimension <= 83) or several (dimension <= 42). */
} gmm_scorer_type;

/* In-memory Mm::MixtureSet (src/Mm/MixtureSet.hh:140-212).  Replaces what the
 * reference scorers read in init() (SimdFeatureScorer.cc:64-104,
 * GaussDiagonalMaximumFeatureScorer.cc:64-86, BatchFeatureScorer.cc:59-75).
 * Densities may be shared between mixtures (CSR over mixture entries). */
typedef struct {
    uint32_t        dimension;           /* MixtureSet::dimension()                        */
    uint32_t        n_means;
    const float*    means;               /* n_means x dimension (Mean, GaussDensity.hh)     */
    uint32_t        n_covariances;
    const float*    variances;           /* n_covariances x dimension: Covariance::diagonal() */
    uint32_t        n_densities;
    const uint32_t* density_mean;        /* GaussDensity::meanIndex()       [n_densities]    */
    const uint32_t* density_covariance;  /* GaussDensity::covarianceIndex() [n_densities]    */
    uint32_t        n_mixtures;
    const uint32_t* mixture_offsets;     /* [n_mixtures + 1], entries of mixture m are [o[m], o[m+1]) */
    const uint32_t* mixture_densities;   /* Mixture::densityIndex(dns)      [n_entries]      */
    const double*   mixture_log_weights; /* Mixture::logWeight(dns) (Mm::Weight = f64) [n_entries] */
} gmm_mixture_set;

/* Scorer configuration (Core::Configuration parameters of the replaced scorers). */
typedef struct {
    float    mixture_weight_scale; /* "mixture-weight-scale" GaussDiagonalMaximumFeatureScorer.cc:38-40 (default 1) */
    float    gaussian_scale;       /* "gaussian-scale" GaussDiagonalMaximumFeatureScorer.cc:42-44 (default 1)       */
    float    score_scale;          /* FeatureScorerScaling scale, ScaledFeatureScorer.hh:62-64 (default 1)         */
    uint32_t max_frames;           /* largest n_frames of one gmm_score_* call ("buffer-size", cc:28-29)         */
    uint32_t mixture_begin;        /* mixture shard [begin, end) scored by this handle; 0,0 = all mixtures        */
    uint32_t mixture_end;
    uint32_t flags;                /* GMM_FLAG_* bits, 0 = defaults                                               */
    /* density preselection (preselection-batch-*): the "density-clustering" parameters,
     * DensityClustering.cc:19-32.  The clustering is built (or read from cache_archive) at create time. */
    uint32_t clusters;              /* "clusters" (256, range 1..256), reduced to the density count      */
    uint32_t select_clusters;       /* "select-clusters" (32)                                           */
    uint32_t clustering_iterations; /* "iterations" (5)                                                 */
    float    backoff_score;         /* "backoff-score" (40000): float type, mixture with no selected density */
    /* "cache-archive" (DensityClustering.cc:27-28, 59-95; DensityClustering.tcc:122-155): path of a RASR cache archive
     * file (Core::MappedArchive).  The preselection types read the clustering from its item "density-clustering" when
     * magic, version, types, padded dimension, cluster and density counts match, else build it and write the item
     * there (other items of the archive are kept).  NULL or "": no cache (always built). */
    const char* cache_archive;
} gmm_scorer_config;

/* Float types (diagonal-maximum, batch-float, diagonal-sum) run on the f16 matrix cores with every f32 operand
 * split into two f16 pieces (f32 accuracy class).  Several covariances (covariance-tying none or
 * mixture-specific, diagonal-maximum / diagonal-sum) take the covariance-free layout: one frame operand
 * [(x - c)^2, (x - c)] for every covariance, K = 6 dimension + 4, dimension <= 42; beyond that the f32-MFMA kernel
 * with per-covariance frame operands.  This flag selects the f32-MFMA kernel always. */
#define GMM_FLAG_NATIVE_F32 1u
/* Tile height of the split-f16 kernel.  By default 32-density tiles (v_mfma_f32_32x32x16_f16, K in
 * steps of 16) are used where they save more than 5 % of K over 16-density tiles (v_mfma_f32_16x16x32_f16,
 * K in steps of 32; the 32x32 loop holds a lower clock) -- e.g. dimension 9 or 45, not 39 -- and the mixtures
 * have <= 512 densities, or where a mixture is too large for 16-density tiles; these flags force one
 * height (tests, A/B timing; TILE32 applies only within those limits). */
#define GMM_FLAG_SPLIT_TILE16 2u
#define GMM_FLAG_SPLIT_TILE32 4u
/* diagonal-maximum, batch-diagonal-maximum-float: evaluate every density in the reference's own f32
 * operation order (GaussDiagonalMaximumFeatureScorer::distance, GDMFS.cc:144-181;
 * BatchFloatFeatureScorer::fillScoreCacheTpl, BatchFeatureScorer.cc:187-234) on the vector ALUs: scores
 * and best densities bit-identical to the reference's arithmetic, at a fraction of the matrix-core
 * kernels' rate.  Dimension <= 128; other types refuse the flag. */
#define GMM_FLAG_REFERENCE_ORDER 8u
/* batch-diagonal-maximum-int / -fast (one covariance, dimension <= 64) run a score-only layout by default:
 * a mixture's rows grouped by the parity of their constant, the constant in the matrix core's accumulator
 * input, one v_min3 per two candidates (no density index to pack).  Same scores, bit for bit.  This flag
 * keeps the (score, density) key layout of SIMD-diagonal-maximum instead (A/B timing, tests). */
#define GMM_FLAG_FULL_KEYS 16u
/* SIMD-diagonal-maximum keeps, besides its key layout, a second copy of the quantized model on the score-only
 * layout for calls without best densities (the search's score(e)); ~64 B per density more device memory.  The
 * twin is best effort: if it cannot be built the scorer serves every call from the key layout.  This flag skips
 * it (callers that always ask for best densities, e.g. aligners). */
#define GMM_FLAG_NO_SCORE_ONLY_TWIN 32u
/* cache_archive is read-only ("read-only" of the archive, Core/Application.cc:43, 399-400): a clustering that is not
 * found there is built but not written. */
#define GMM_FLAG_CACHE_ARCHIVE_READ_ONLY 64u

typedef struct gmm_scorer gmm_scorer;

/* Fill *cfg with the reference defaults. */
void gmm_default_config(gmm_scorer_config* cfg);

/* Prepare the model on the host exactly as the reference scorer's init() does
 * (quantization scale, 1/sqrt(var), prepared means, constant weights) and
 * upload it to `device`.  Replaces the FeatureScorerFactory::createInstance
 * call (src/Mm/FeatureScorerFactory.hh:114-122) for the selected type.
 * SIMD-diagonal-maximum with several covariances quantizes each frame per covariance (SimdFeatureScorer.cc:22-35)
 * into a covariances x max_frames x 64 B table: GMM_ERR_UNSUPPORTED, the size in gmm_last_error(), when that table
 * exceeds three quarters of the device's free memory. */
int gmm_scorer_create(const gmm_mixture_set* mixture_set, gmm_scorer_type type,
                      const gmm_scorer_config* config, int device, gmm_scorer** out);
int gmm_scorer_destroy(gmm_scorer* scorer);

/* FeatureScorer::nMixtures() (FeatureScorer.hh:49), AssigningFeatureScorer::dimension(). */
uint32_t gmm_scorer_n_mixtures(const gmm_scorer* scorer);
uint32_t gmm_scorer_dimension(const gmm_scorer* scorer);
uint32_t gmm_scorer_n_covariances(const gmm_scorer* scorer);  /* MixtureSet::nCovariances() */
int      gmm_scorer_type_of(const gmm_scorer* scorer);

/* Score n_frames feature vectors (row t at frames + t * frame_stride floats)
 * against every mixture of the handle's shard.  DEVICE pointers, enqueued on
 * `stream` (a hipStream_t; NULL = default stream), asynchronous.
 *   scores       [n_mixtures][score_stride] f32: ContextScorer::score(e) per frame
 *   best_density [n_mixtures][score_stride] u32 or NULL: AssigningContextScorer::bestDensity(e)
 *                (batch types have no assignment and ignore it).
 *                Quantized types: bit-exact (lowest index on equal scores, the reference's strict `<`).
 *                Float types: the kernel orders candidates by the f32 score with its low 6-8 mantissa bits
 *                replaced by a (tile, row) tag, so two densities whose scores agree within ~2^-16
 *                relative may be reported in either order (the lower index wins exact ties); the score
 *                itself stays within the 1e-4 contract.
 * Replaces per-frame Context construction + calculateScoreAndDensity
 * (SimdFeatureScorer.cc:22-35,135-176) and BatchFeatureScorerBase::fillScoreCache
 * (BatchFeatureScorer.cc:98-105). */
int gmm_score_device(gmm_scorer* scorer, const float* frames, uint32_t n_frames, uint32_t frame_stride,
                     float* scores, uint32_t* best_density, uint32_t score_stride, void* stream);

/* Same with HOST buffers (copies in, scores, copies out, synchronizes).  Large batches are scored in
 * frame chunks with the copy-out of one chunk overlapped with the scoring of the next; a score/best
 * buffer from gmm_host_alloc (or otherwise page-locked) is written by DMA directly, a pageable one
 * through a pinned staging ring and RASR_GMM_HOST_THREADS copy threads (default 8). */
int gmm_score_host(gmm_scorer* scorer, const float* frames, uint32_t n_frames, uint32_t frame_stride,
                   float* scores, uint32_t* best_density, uint32_t score_stride);

/* The ring buffer of BatchFeatureScorerBase (features_ / scores_, src/Mm/BatchFeatureScorer.hh:164-198,
 * fillScoreCache over `length` buffered positions from `featureIndex`, BatchFeatureScorer.cc:98-105) in ONE
 * call, wrapped or not: the frames are the host rows ring[((first + i) % ring_size) * frame_stride],
 * i < n_frames (n_frames <= ring_size, first < ring_size), and the results of ring position p go to column p
 * of the [n_mixtures][score_stride] tables (score_stride >= ring_size).  HOST buffers, synchronous, as
 * gmm_score_host (which is this call with ring_size = n_frames, first = 0).
 * flags: GMM_HOST_KEEP_BEST (best_density must be NULL): the best densities are computed but not copied;
 *   the scorer keeps them on the device until its next host call, and gmm_fetch_best_density copies them
 *   into the caller's table on demand -- a caller that reads only score(e) (the search) moves 4 instead of
 *   8 bytes per (frame, mixture) over PCIe, while bestDensity(e) (the aligners) still works.
 * flags: GMM_HOST_FRAME_MAJOR: the tables are frame-major instead, results of ring position p in ROW p of
 *   [ring_size][score_stride] (score_stride >= n_mixtures): a caller reading one frame's scores for many
 *   mixtures (ContextScorer::score(e) of the search, FeatureScorerNode's dump) reads contiguous memory
 *   instead of one cache line per emission.  The device transposes each chunk before the copy.
 * *call_id (may be NULL) receives the call's id. */
#define GMM_HOST_KEEP_BEST 1u
#define GMM_HOST_FRAME_MAJOR 2u
/* flags: GMM_HOST_LAZY_BEST (best_density must be NULL; not with GMM_HOST_KEEP_BEST): the call computes scores
 *   only -- SIMD-diagonal-maximum on its score-only kernel, the float types without the index tag, so their
 *   scores are plain f32 -- and keeps its frames on the device until the scorer's next host call;
 *   gmm_fetch_best_density then computes the best densities from them (one more scoring pass over the call's
 *   frames, whose scores are not copied again).  The reference likewise evaluates bestDensity(e) only when
 *   asked (AssigningFeatureScorer.hh:110-121): a search that reads only score(e) never pays for the
 *   assignment.
 * Small calls (n_frames <= 64, e.g. a recognizer's buffer of 1..64 frames) whose ring and tables all come from
 *   gmm_host_alloc run on one stream without the copy engine: a kernel reads the ring rows and the tables are
 *   written by kernels over PCIe (about 80 us instead of 125 us for one frame at 800k densities, DESIGN.md
 *   section 4).  Other buffers take the copy-engine path; the results are bit-identical either way. */
#define GMM_HOST_LAZY_BEST 4u
/* flags: GMM_HOST_ASYNC: the call returns once its copies and kernels are enqueued; its tables are written when
 *   gmm_host_call_wait(scorer, call_id) returns (or any later host call of the scorer, which waits for it
 *   first).  The score (and best) tables must be page-locked (gmm_host_alloc); the ring rows of the call are read
 *   asynchronously and must not change until the wait.  The drop-in's ring buffer uses it to score the newest
 *   frames on the GPU while the caller consumes the older ones. */
#define GMM_HOST_ASYNC 8u
int gmm_score_host_ring(gmm_scorer* scorer, const float* ring, uint32_t ring_size, uint32_t first,
                        uint32_t n_frames, uint32_t frame_stride, float* scores, uint32_t* best_density,
                        uint32_t score_stride, uint32_t flags, uint64_t* call_id);

/* Waits for host call `call_id` (made with GMM_HOST_ASYNC; any other call id returns at once).  Status of the
 * call's device work. */
int gmm_host_call_wait(gmm_scorer* scorer, uint64_t call_id);

/* Best densities of host call `call_id` (made with GMM_HOST_KEEP_BEST or GMM_HOST_LAZY_BEST) into the same ring positions of
 * best_density, in the same layout, that its scores went to.  GMM_ERR_INVALID_ARGUMENT once a later
 * host call of this scorer has replaced them (the caller scores those frames again). */
int gmm_fetch_best_density(gmm_scorer* scorer, uint64_t call_id, uint32_t* best_density, uint32_t score_stride);

/* Sparse best densities: AssigningContextScorer::bestDensity(e) for a LIST of (ring position, mixture) pairs of host
 * call `call_id` (made with GMM_HOST_KEEP_BEST or GMM_HOST_LAZY_BEST, its frames still on the device), instead of
 * the whole table gmm_fetch_best_density computes and copies.  best_density[i] receives the density-in-mixture
 * index for frame positions[i] (a ring position that call scored) and mixture mixtures[i]; 0xffffffff for a
 * mixture without a finite candidate.  HOST arrays, synchronous (one small kernel; about the latency of one
 * launch).  The mixture's densities are scored in the reference's own arithmetic and scanned in its order
 * (AssigningFeatureScorer.hh:110-121, SimdFeatureScorer.cc:135-176, GaussDiagonalMaximumFeatureScorer.cc:116-142,
 * 263-286): SIMD-diagonal-maximum bit-exact; the float types as the CPU restatement computes them (a near tie may
 * name another density than the keyed table scorers, within their float contract).  Errors: GMM_ERR_INVALID_ARGUMENT
 * once a later host call replaced the frames, for a position the call did not score or a mixture out of range;
 * GMM_ERR_UNSUPPORTED for batch types, density-sharded handles and float models of dimension > 128 (the caller
 * uses gmm_fetch_best_density).  Replaces the per-emission bestDensity(e) of the reference's context scorers for
 * callers that ask a few emissions per frame (aligners, AbstractMixtureSetEstimator.cc:370-384). */
int gmm_best_density_pairs(gmm_scorer* scorer, uint64_t call_id, const uint32_t* positions, const uint32_t* mixtures,
                           uint32_t n_pairs, uint32_t* best_density);

/* The same for frames in DEVICE memory (row t at frames + t * frame_stride floats, t < n_frames) and DEVICE pair
 * arrays (pair_frame[i] < n_frames, pair_mixture[i] < the handle's mixtures; an out-of-range pair yields
 * 0xffffffff), enqueued on `stream` (a hipStream_t; NULL = default stream), asynchronous. */
int gmm_best_density_pairs_device(gmm_scorer* scorer, const float* frames, uint32_t n_frames, uint32_t frame_stride,
                                  const uint32_t* pair_frame, const uint32_t* pair_mixture, uint32_t n_pairs,
                                  uint32_t* best_density, void* stream);

/* Page-locked host memory for gmm_score_host's outputs (the buffer a batched caller keeps, e.g.
 * BatchFeatureScorerBase::scores_, BatchFeatureScorer.hh:177-186), so that callers need no HIP
 * headers.  gmm_host_free(NULL) is a no-op. */
int gmm_host_alloc(size_t bytes, void** ptr);
int gmm_host_free(void* ptr);

/* SimdGaussDiagonalMaximumFeatureScorer accessors used by AcousticLookAhead
 * (src/Search/AdvancedTreeSearch/AcousticLookAhead.cc:156,447):
 * inverseQuantizationFactor() (SimdFeatureScorer.hh:128-130) and the
 * quantization scale s (SimdFeatureScorer.cc:69).  Quantized types only. */
int gmm_scorer_quantization(const gmm_scorer* scorer, float* scaling, float* inverse_quantization_factor);

/* multiplyAndQuantize(featureVector) (SimdFeatureScorer.cc:37-52): out receives
 * n_covariances x padded_dimension u8, padded_dimension = dimension rounded up to 16. */
int gmm_scorer_multiply_and_quantize(const gmm_scorer* scorer, const float* feature, uint8_t* out);

/* Host-side model preparation only (no device needed): the prepared tables
 * of the SIMD / batch-int scorers, for CPU-side verification.
 *   isv [n_covariances * dimension] scaled 1/sqrt(var); log_norm [n_covariances];
 *   prepared_mean [n_entries * padded_dimension] u8; constant_weight [n_entries].
 * Any output pointer may be NULL. */
int gmm_prepare_quantized_host(const gmm_mixture_set* mixture_set, gmm_scorer_type type, float* scaling,
                               float* isv, float* log_norm, uint8_t* prepared_mean, int32_t* constant_weight);

/* Number of kernel launches one gmm_score_device call enqueues, and the name
 * of the dominant kernel (for profiling scripts). */
int gmm_scorer_launch_info(const gmm_scorer* scorer, uint32_t n_frames, uint32_t* n_launches,
                           const char** main_kernel_name);

/* Instrumentation for bench.py: when enabled, every gmm_score_* call records a
 * pair of HIP events on its stream around the scorer kernel (the dominant
 * launch); gmm_scorer_kernel_time synchronizes on the last event and returns
 * the summed kernel time and launch count since the last reset. */
int gmm_scorer_set_timing(gmm_scorer* scorer, int enable);
int gmm_scorer_kernel_time(gmm_scorer* scorer, double* total_ms, uint32_t* n_launches, int reset);

/* RASR cache archives (Core::MappedArchive, src/Core/MappedArchive.{hh,cc}; the file behind a "cache-archive"
 * parameter): read item `name` of the archive at `path` -- *size receives its byte count; up to `capacity` bytes are
 * copied into `data` (may be NULL to ask the size) -- or write it (the archive is created, or rewritten with its other
 * items kept).  GMM_ERR_INVALID_ARGUMENT if the file is not an archive of that format or has no such item.  Host
 * only; the preselection scorers use them for the item "density-clustering" (gmm_scorer_config.cache_archive). */
/* Where a preselection scorer's density clustering came from (DensityClustering<F, D>::build,
 * DensityClustering.tcc:122-155, which logs "using cached density clustering" / "density clustering written"):
 * GMM_CLUSTERING_BUILT (built, not written: no or a read-only cache archive, or the write failed),
 * GMM_CLUSTERING_WRITTEN (built and written to the cache archive), GMM_CLUSTERING_CACHED (read from it).
 * GMM_ERR_UNSUPPORTED for a type without preselection. */
#define GMM_CLUSTERING_BUILT 0
#define GMM_CLUSTERING_WRITTEN 1
#define GMM_CLUSTERING_CACHED 2
int gmm_scorer_clustering_source(const gmm_scorer* scorer, int* source);
int gmm_cache_archive_read_item(const char* path, const char* name, void* data, uint64_t capacity, uint64_t* size);
int gmm_cache_archive_write_item(const char* path, const char* name, const void* data, uint64_t size);

/* Density preselection (preselection-batch-float / -int).
 * gmm_scorer_density_clustering: the clustering the handle was built with, over ALL mixture entries of
 * the mixture set (entry = CSR position in mixture_densities, the reference's density index):
 *   cluster_of_entry [n_entries] (clusterIndexForDensity_), cluster_means [clusters][padded_dimension]
 *   (f32 for the float type, u8 for the int type; padded dimension = dimension rounded up to 8 / 16).
 * gmm_scorer_cluster_selection: the selection the last gmm_score_* call used, [n_frames][clusters]
 *   0/1 (activeClusters_); synchronizes the device.
 * gmm_density_clustering_seeds: host-only, the entry each cluster is initialized from
 *   (initializeClusters: srand(1), rand() % n_entries without repetition, DensityClustering.tcc:60-74). */
int gmm_scorer_density_clustering(const gmm_scorer* scorer, uint32_t* n_clusters, uint32_t* padded_dimension,
                                  uint8_t* cluster_of_entry, void* cluster_means);
int gmm_scorer_cluster_selection(gmm_scorer* scorer, uint32_t n_frames, uint8_t* selection);
int gmm_density_clustering_seeds(uint32_t n_entries, uint32_t n_clusters, uint32_t* seed_entries);

/* Density-sharded layout (BASELINE config 4: a mixture's densities split over GPUs, per-frame reduce over
 * RCCL).  The reference is single-process (no counterpart); these define the exchange format.
 * gmm_shard_pack_keys: [rows][n_frames] int64 keys = (order-preserving score bits << 32) | (best density
 *   + best_offset[row]), whose signed minimum is the reference's winner (lower score, then lower density
 *   index); best / best_offset may be NULL (density 0 / offset 0).  An all-reduce(MIN) over the keys of
 *   the GPUs holding parts of a mixture is the per-frame reduce.
 * gmm_shard_unpack_keys: keys -> scores (and best densities if best != NULL).
 * DEVICE pointers, row stride `stride` for scores/best, keys dense; asynchronous on `stream`. */
int gmm_shard_pack_keys(const float* scores, const uint32_t* best, const uint32_t* best_offset, uint32_t rows,
                        uint32_t n_frames, uint32_t stride, int64_t* keys, void* stream);
int gmm_shard_unpack_keys(const int64_t* keys, uint32_t rows, uint32_t n_frames, float* scores, uint32_t* best,
                          uint32_t stride, void* stream);

/* The density shard plan over `world` GPUs (host-only): part r holds the mixture entries [E r / P, E (r+1) / P)
 * of the CSR order.  shard_table (may be NULL) receives [world][5] = {entry_begin, entry_end, mixture_begin,
 * mixture_end, first_offset} (first_offset: in-mixture index of the part's first entry of mixture_begin);
 * split (may be NULL, room for world - 1) the mixtures held by more than one part, ascending; *n_split their
 * number. */
int gmm_density_shard_plan(const uint32_t* mixture_offsets, uint32_t n_mixtures, uint32_t world,
                           uint32_t* shard_table, uint32_t* split, uint32_t* n_split);

/* Density-sharded scorer for one process driving several GPUs (an RASR process whose model is split over
 * the GPUs of a node): part r of the plan above is an ordinary scorer on devices[r]; a call scores every
 * part on its own stream, combines the mixtures split between parts by a per-frame minimum over
 * gmm_shard_pack_keys keys, and assembles the full [n_mixtures] table on devices[0].  The handle is a
 * gmm_scorer: gmm_score_device (DEVICE pointers on devices[0]), gmm_score_host, gmm_score_host_ring (all
 * flags), gmm_fetch_best_density and the accessors work on it.  Scorer types whose mixture score is the
 * minimum over its densities only (SIMD-diagonal-maximum, diagonal-maximum, batch-diagonal-maximum-*):
 * GMM_ERR_UNSUPPORTED otherwise.  Quantized types give the unsharded scorer's results bit for bit; the
 * float types stay within their f32 contract (a part's split-f16 scaling follows its own densities).
 * n_devices == 1 creates the unsharded scorer itself.  exchange: the per-frame reduce --
 *   GMM_EXCHANGE_RCCL: an RCCL all-reduce(MIN) over the parts' keys (ncclCommInitAll over devices, one
 *     stream per GPU; the devices must be distinct),
 *   GMM_EXCHANGE_COPY: peer copies of the keys to devices[0] and a minimum kernel there (any devices,
 *     repeats allowed: N parts on one GPU),
 *   GMM_EXCHANGE_AUTO: RCCL when the devices are distinct, else COPY.
 * config->mixture_begin / mixture_end must be 0 (the whole set is sharded). */
#define GMM_EXCHANGE_AUTO 0
#define GMM_EXCHANGE_RCCL 1
#define GMM_EXCHANGE_COPY 2
int gmm_scorer_create_sharded(const gmm_mixture_set* mixture_set, gmm_scorer_type type,
                              const gmm_scorer_config* config, const int* devices, uint32_t n_devices,
                              int exchange, gmm_scorer** out);
/* Parts of a handle (1 for an unsharded one) and the exchange it resolved to (GMM_EXCHANGE_RCCL / _COPY;
 * GMM_EXCHANGE_AUTO for an unsharded handle or a plan without split mixtures). */
int gmm_scorer_shard_info(const gmm_scorer* scorer, uint32_t* n_parts, int* exchange);

const char* gmm_last_error(void);
const char* gmm_version(void);
/* Identity of this build's device code (a hash of the kernel sources and compile flags); profiling
 * summaries record it, so a counter measurement is matched to the kernels it was taken on. */
const char* gmm_kernel_id(void);

#ifdef __cplusplus
}
#endif
#endif /* RASR_GMM_H */
