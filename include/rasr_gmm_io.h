/*
 * rasr_gmm_io.h -- mixture-set files for the MI355X GMM scorer (C-ABI).
 *
 * Reads and writes RASR's plain-text mixture-set format ("#Version: 2.0",
 * ".pms", optionally gzip-compressed ".pms.gz") into the gmm_mixture_set
 * tables that gmm_scorer_create() takes.  Replaces the reference's loading
 * chain for this format:
 *   Mm::Module_::readMixtureSet        src/Mm/Module.cc:152-182
 *   MixtureSetReader::FormatReader     src/Mm/MixtureSetReader.cc:28-47
 *   MixtureSetEstimatorReader          src/Mm/MixtureSetReader.cc:52-74 (binary estimator files, below)
 *   Core::CompressedPlainTextFormat    src/Core/FormatSet.hh:302-320 (gzip detected from the data)
 *   MixtureSet::read / ::write         src/Mm/MixtureSet.cc:142-214
 *   Mixture::read / ::write            src/Mm/Mixture.cc:81-107
 *   GaussDensityTopology::read/write   src/Mm/MixtureSetTopology.cc:19-30
 *   Mean / DiagonalCovariance r/w      src/Mm/GaussDensity.cc:25-69
 * Numbers are parsed with the grammar and rounding of the reference's
 * std::istream extraction (f32 means/variances, f64 weights), so the tables
 * are bit-identical to the reference's MixtureSet after reading.
 *
 * Errors (negative status, message via gmm_last_error()):
 *   GMM_ERR_INVALID_ARGUMENT  unreadable file, malformed or truncated text -- the cases in
 *                             which the reference's read() returns !stream.good(), including a
 *                             file whose last number is not followed by a line break (std::istream
 *                             sets eofbit, MixtureSet.cc:213);
 *                             indices out of range, or a mean/covariance whose length differs
 *                             from dimension() (undefined behaviour in the reference's scorers)
 *   GMM_ERR_UNSUPPORTED       "#Version:" above 2.0 (criticalError, MixtureSet.cc:181-183);
 *                             a covariance type other than DiagonalCovariance (MixtureSet.cc:185-187)
 */
#ifndef RASR_GMM_IO_H
#define RASR_GMM_IO_H

#include <stdint.h>

#include "rasr_gmm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Parameters of the maximum-likelihood estimation that turns an estimator (accumulator) file into a
 * mixture set (AbstractMixtureSetEstimator, src/Mm/AbstractMixtureSetEstimator.cc:25-58; the reader takes
 * them from the mixture-set configuration). */
typedef struct {
    double   minimum_observation_weight; /* "minimum-observation-weight" (5): densities of a mixture with less
                                            accumulated weight are removed (except the heaviest one)        */
    double   minimum_relative_weight;    /* "minimum-relative-weight" (0), relative to the mixture's weight   */
    double   minimum_variance;           /* "minimum-variance" (0): variances below are raised to it          */
    uint32_t allow_zero_weights;         /* "allow-zero-weights" (false): else a zero-weight mixture fails    */
    uint32_t normalize_mixture_weights;  /* "normalize-mixture-weights" (true)                               */
} gmm_estimator_config;

void gmm_default_estimator_config(gmm_estimator_config* config);

/* Estimate a mixture set from the bytes of a binary maximum-likelihood estimator file ("MIXSET" magic,
 * written by RASR's trainers, AbstractMixtureSetEstimator::write, cc:481-509): the reference's
 * MixtureSetReader::MixtureSetEstimatorReader (src/Mm/MixtureSetReader.cc:52-74) = estimator->read
 * (AbstractMixtureSetEstimator.cc:433-479) then estimate() (:299-337): densities below the minimum weights
 * removed, means = sums / weight, pooled variances = (sum of squares - sum over the covariance's means of
 * mean sum^2 / mean weight) / weight, raised to minimum_variance, mixture log weights normalized.  Errors:
 * GMM_ERR_INVALID_ARGUMENT for a wrong magic, a truncated file, out-of-range indices, accumulators whose size
 * differs from the dimension, a zero-weight mixture (unless allowed) or a mixture without densities,
 * a covariance whose weight differs from its means' (the reference's criticalError / verify). */
int gmm_mixture_set_estimate(const void* data, uint64_t size, const gmm_estimator_config* config,
                             gmm_mixture_set* out);

/* gmm_mixture_set_read with explicit estimator parameters (NULL = defaults). */
int gmm_mixture_set_read_config(const char* filename, const gmm_estimator_config* config, uint32_t dimension_offset,
                                uint32_t reduced_dimension, gmm_mixture_set* out);

/* Read a mixture-set file into *out (arrays allocated by the library; release
 * them with gmm_mixture_set_free).  The format follows the reference's reader dispatch on the file name
 * extension (MixtureSetReader.cc:28-35, MixtureSetReader.hh:105-117, Core::filenameExtension): ".pms" and
 * ".gz" are the text format below, every other name a binary estimator file (gmm_mixture_set_estimate with
 * the default parameters).  dimension_offset / reduced_dimension are the
 * "reduced-mixture-set-dimension-offset" / "reduced-mixture-set-dimension"
 * parameters (Module.cc:42-49, applied at :165-175): the first
 * dimension_offset components of every mean and covariance are dropped, then,
 * if reduced_dimension > 0, every mean is cut or zero-padded and every
 * covariance cut or one-padded to reduced_dimension (MixtureSet.cc:109-126,
 * GaussDensity.hh:191-194).  0, 0 = the file as written.  A version below 2.0
 * holds linear mixture weights, stored as log(w), or -DBL_MAX for w <= 0
 * (Mixture.cc:63-66). */
int gmm_mixture_set_read(const char* filename, uint32_t dimension_offset, uint32_t reduced_dimension,
                         gmm_mixture_set* out);

/* Same from a memory buffer (plain or gzip bytes). */
int gmm_mixture_set_parse(const void* data, uint64_t size, uint32_t dimension_offset, uint32_t reduced_dimension,
                          gmm_mixture_set* out);

/* Release the arrays of a set filled by gmm_mixture_set_read/_parse and zero *ms. */
int gmm_mixture_set_free(gmm_mixture_set* ms);

/* Write *ms in the text format of MixtureSet::write (MixtureSet.cc:142-168) with
 * `precision` significant digits (Module_::writeMixtureSet, default 6,
 * Module.hh:145); gzip-compressed when filename ends in ".gz" or ".Z"
 * (CompressedOutputStream::open, src/Core/CompressedStream.cc:77-102).
 * Covariance feature weights are written as 1 (they are folded into the
 * variances on read, GaussDensity.cc:62-64). */
int gmm_mixture_set_write(const char* filename, const gmm_mixture_set* ms, uint32_t precision);

#ifdef __cplusplus
}
#endif

#endif /* RASR_GMM_IO_H */
