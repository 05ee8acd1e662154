/*
 * rasr_gmm_io.h -- mixture-set files for the MI355X GMM scorer (C-ABI).
 *
 * Reads and writes RASR's plain-text mixture-set format ("#Version: 2.0",
 * ".pms", optionally gzip-compressed ".pms.gz") into the gmm_mixture_set
 * tables that gmm_scorer_create() takes.  Replaces the reference's loading
 * chain for this format:
 *   Mm::Module_::readMixtureSet        src/Mm/Module.cc:152-182
 *   MixtureSetReader::FormatReader     src/Mm/MixtureSetReader.cc:28-47
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

/* Read a mixture-set file into *out (arrays allocated by the library; release
 * them with gmm_mixture_set_free).  dimension_offset / reduced_dimension are the
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
