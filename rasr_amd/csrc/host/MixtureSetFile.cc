// MixtureSetFile.cc -- RASR plain-text mixture-set files <-> gmm_mixture_set (include/rasr_gmm_io.h).
//
// The reference reads a ".pms"/".pms.gz" file through std::istream extraction
// (MixtureSet::read, src/Mm/MixtureSet.cc:170-214) on top of a zstr stream that
// inflates gzip/zlib data when it sees the magic bytes and passes anything else
// through (src/Core/CompressedStream.cc:37-54).  Here the whole file is loaded
// (inflated in one pass when compressed) and scanned by a cursor that implements
// the same extraction rules as libstdc++'s num_get:
//   * leading white space skipped (C-locale isspace); hitting the end while skipping
//     fails the extraction;
//   * unsigned: optional sign, decimal digits; "-n" wraps modulo 2^32; overflow fails;
//   * float/double: [sign] digits [. digits] [(e|E) [sign] digits] (the exponent only
//     after mantissa digits), converted by strtof/strtod in the "C" locale; a token the
//     conversion does not consume entirely fails, and so does overflow to +-inf;
//   * an extraction that runs into the end of the data sets eofbit, and the reference
//     returns stream.good() (MixtureSet.cc:213), so a file whose last number is not
//     followed by white space is rejected as the reference rejects it.
// Values are stored exactly as the reference stores them: means as f32 (MeanType,
// src/Mm/Types.hh:28), mixture weights as f64 (Weight), variances as
// f32(f64(f32 v) * f64 w) (GaussDensity.cc:54-69).
#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cfloat>
#include <clocale>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <locale.h>
#include <string>
#include <vector>

#include "../../../include/rasr_gmm_io.h"

namespace rasr_gmm {
void setLastError(const std::string& msg);  // gmm_api.cc
}

namespace {

using rasr_gmm::setLastError;

locale_t cLocale() {
    static locale_t loc = newlocale(LC_NUMERIC_MASK, "C", (locale_t)0);
    return loc;
}

bool isSpace(char c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
}
bool isDigit(char c) {
    return c >= '0' && c <= '9';
}

// ---------------------------------------------------------------------------
// bytes -> text (Core::CompressedInputStream: zstr auto-detection of gzip / zlib headers)
// ---------------------------------------------------------------------------
bool isCompressed(const unsigned char* p, size_t n) {
    if (n < 2)
        return false;
    if (p[0] == 0x1f && p[1] == 0x8b)
        return true;  // gzip
    return p[0] == 0x78 && (p[1] == 0x01 || p[1] == 0x9c || p[1] == 0xda);  // zlib
}

bool inflateAll(const unsigned char* in, size_t n, std::string& out, std::string& err) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 15 + 32) != Z_OK) {  // +32: gzip or zlib header, detected
        err = "zlib: inflateInit2 failed";
        return false;
    }
    out.clear();
    size_t consumed = 0;
    std::vector<char> buf(1 << 20);
    for (;;) {
        if (zs.avail_in == 0 && consumed < n) {
            const size_t take = std::min<size_t>(n - consumed, 1u << 30);
            zs.next_in        = const_cast<Bytef*>(in + consumed);
            zs.avail_in       = static_cast<uInt>(take);
            consumed += take;
        }
        zs.next_out  = reinterpret_cast<Bytef*>(buf.data());
        zs.avail_out = static_cast<uInt>(buf.size());
        const int rc = inflate(&zs, Z_NO_FLUSH);
        out.append(buf.data(), buf.size() - zs.avail_out);
        if (rc == Z_STREAM_END) {
            // concatenated gzip members (as written by `cat a.gz b.gz`) continue the text
            const size_t pos = consumed - zs.avail_in;
            if (pos + 2 <= n && isCompressed(in + pos, n - pos)) {
                inflateReset(&zs);
                continue;
            }
            break;
        }
        if (rc != Z_OK && rc != Z_BUF_ERROR) {
            err = std::string("zlib: ") + (zs.msg ? zs.msg : "corrupt compressed data");
            inflateEnd(&zs);
            return false;
        }
        if (rc == Z_BUF_ERROR && zs.avail_in == 0 && consumed == n) {
            err = "zlib: truncated compressed data";
            inflateEnd(&zs);
            return false;
        }
    }
    inflateEnd(&zs);
    return true;
}

// ---------------------------------------------------------------------------
// std::istream extraction rules over an in-memory text
// ---------------------------------------------------------------------------
class Cursor {
public:
    Cursor(const char* begin, const char* end) : p_(begin), end_(end) {}

    bool atEof() const { return eof_; }
    size_t offset(const char* begin) const { return static_cast<size_t>(p_ - begin); }

    // std::getline(istream, string): up to '\n' (consumed, not stored)
    bool getline(std::string& line) {
        line.clear();
        if (eof_)
            return false;
        const char* q = p_;
        while (q < end_ && *q != '\n')
            ++q;
        line.assign(p_, q);
        if (q == end_) {
            eof_ = true;
            p_   = q;
            return !line.empty();
        }
        p_ = q + 1;
        return true;
    }

    bool u32(uint32_t& v) {
        if (!skipSpace())
            return false;
        bool neg = false;
        if (*p_ == '+' || *p_ == '-') {
            neg = *p_ == '-';
            if (++p_ == end_) {
                eof_ = true;
                return false;
            }
        }
        uint64_t acc    = 0;
        bool     digits = false, overflow = false;
        while (p_ < end_ && isDigit(*p_)) {
            acc      = acc * 10 + static_cast<uint64_t>(*p_ - '0');
            overflow = overflow || acc > 0xffffffffull;
            digits   = true;
            ++p_;
        }
        if (p_ == end_)
            eof_ = true;
        if (!digits || overflow)
            return false;
        v = neg ? static_cast<uint32_t>(0u - static_cast<uint32_t>(acc)) : static_cast<uint32_t>(acc);
        return true;
    }

    bool f32(float& v) {
        if (!scanFloat())
            return false;
        char* stop = nullptr;
        v          = strtof_l(tok_.c_str(), &stop, cLocale());
        return stop != tok_.c_str() && *stop == '\0' && !std::isinf(v);
    }

    bool f64(double& v) {
        if (!scanFloat())
            return false;
        char* stop = nullptr;
        v          = strtod_l(tok_.c_str(), &stop, cLocale());
        return stop != tok_.c_str() && *stop == '\0' && !std::isinf(v);
    }

private:
    bool skipSpace() {
        if (eof_)
            return false;  // a previous extraction set eofbit: the sentry fails
        while (p_ < end_ && isSpace(*p_))
            ++p_;
        if (p_ == end_) {
            eof_ = true;
            return false;
        }
        return true;
    }

    // the characters libstdc++'s num_get::_M_extract_float accumulates
    bool scanFloat() {
        tok_.clear();
        if (!skipSpace())
            return false;
        if (*p_ == '+' || *p_ == '-')
            tok_.push_back(*p_++);
        bool mantissa = false, dot = false, sci = false;
        while (p_ < end_) {
            const char c = *p_;
            if (isDigit(c)) {
                mantissa = true;
            }
            else if (c == '.' && !dot && !sci) {
                dot = true;
            }
            else if ((c == 'e' || c == 'E') && !sci && mantissa) {
                sci = true;
                tok_.push_back(c);
                ++p_;
                if (p_ < end_ && (*p_ == '+' || *p_ == '-'))
                    tok_.push_back(*p_++);
                continue;
            }
            else {
                break;
            }
            tok_.push_back(c);
            ++p_;
        }
        if (p_ == end_)
            eof_ = true;
        return true;
    }

    const char* p_;
    const char* end_;
    bool        eof_ = false;
    std::string tok_;
};

// ---------------------------------------------------------------------------
// text -> tables
// ---------------------------------------------------------------------------
struct Tables {
    uint32_t              dimension = 0;
    std::vector<float>    meanData, varData;
    std::vector<uint64_t> meanOff{0}, varOff{0};
    std::vector<uint32_t> dnsMean, dnsCov, mixOff{0}, mixDns;
    std::vector<double>   mixLogW;
};

struct Status {
    int         code = GMM_OK;
    std::string msg;
    bool        fail(int c, const std::string& m) {
        code = c;
        msg  = m;
        return false;
    }
};

// don't let a corrupt count allocate more than the text could hold
size_t boundedReserve(uint64_t count, size_t textBytes, size_t bytesPerItem) {
    return static_cast<size_t>(std::min<uint64_t>(count, textBytes / bytesPerItem + 1));
}

bool parseText(const char* begin, const char* end, Tables& t, Status& st) {
    Cursor      in(begin, end);
    std::string line;
    const auto  malformed = [&](const char* what) {
        return st.fail(GMM_ERR_INVALID_ARGUMENT, std::string("mixture set: malformed or truncated ") + what +
                                                         " (byte " + std::to_string(in.offset(begin)) + ")");
    };
    // header lines (MixtureSet.cc:178-188)
    if (!in.getline(line) || line.size() < 10)
        return malformed("\"#Version:\" line");
    const float version = static_cast<float>(strtod_l(line.c_str() + 10, nullptr, cLocale()));  // atof
    if (version > 2.0)
        return st.fail(GMM_ERR_UNSUPPORTED, "mixture set: version \"" + line.substr(10) + "\" not supported");
    if (!in.getline(line) || line.size() < 17)
        return malformed("\"#CovarianceType:\" line");
    if (line.compare(17, std::string::npos, "DiagonalCovariance") != 0)
        return st.fail(GMM_ERR_UNSUPPORTED, "mixture set: covariance type \"" + line.substr(17) +
                                                    "\" (only DiagonalCovariance is supported)");
    uint32_t nMix, nDns, nMean, nCov;
    if (!in.u32(t.dimension) || !in.u32(nMix) || !in.u32(nDns) || !in.u32(nMean) || !in.u32(nCov))
        return malformed("header");
    const size_t bytes = static_cast<size_t>(end - begin);

    // mixtures (Mixture::read, Mixture.cc:90-107)
    t.mixOff.reserve(boundedReserve(nMix + 1ull, bytes, 2));
    for (uint32_t m = 0; m < nMix; ++m) {
        uint32_t n;
        if (!in.u32(n))
            return malformed("mixture");
        if (t.mixDns.size() + n > 0xffffffffull)
            return st.fail(GMM_ERR_INVALID_ARGUMENT, "mixture set: more than 2^32 mixture entries");
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t dns;
            double   w;
            if (!in.u32(dns) || !in.f64(w))
                return malformed("mixture");
            if (version < 2.0)  // Mixture::addDensity: linear weight (Mixture.cc:63-66)
                w = w > 0 ? std::log(w) : -DBL_MAX;
            t.mixDns.push_back(dns);
            t.mixLogW.push_back(w);
        }
        t.mixOff.push_back(static_cast<uint32_t>(t.mixDns.size()));
    }
    // densities (GaussDensityTopology::read, MixtureSetTopology.cc:23-30)
    t.dnsMean.reserve(boundedReserve(nDns, bytes, 4));
    t.dnsCov.reserve(boundedReserve(nDns, bytes, 4));
    for (uint32_t d = 0; d < nDns; ++d) {
        uint32_t mi, ci;
        if (!in.u32(mi) || !in.u32(ci))
            return malformed("density");
        t.dnsMean.push_back(mi);
        t.dnsCov.push_back(ci);
    }
    // means (Mean::read, GaussDensity.cc:32-43)
    t.meanOff.reserve(boundedReserve(nMean + 1ull, bytes, 2));
    t.meanData.reserve(boundedReserve(uint64_t(nMean) * t.dimension, bytes, 2));
    for (uint32_t i = 0; i < nMean; ++i) {
        uint32_t n;
        if (!in.u32(n))
            return malformed("mean");
        for (uint32_t k = 0; k < n; ++k) {
            float v;
            if (!in.f32(v))
                return malformed("mean");
            t.meanData.push_back(v);
        }
        t.meanOff.push_back(t.meanData.size());
    }
    // covariances (DiagonalCovariance::read, GaussDensity.cc:54-69): variance x feature weight
    t.varOff.reserve(boundedReserve(nCov + 1ull, bytes, 2));
    for (uint32_t i = 0; i < nCov; ++i) {
        uint32_t n;
        if (!in.u32(n))
            return malformed("covariance");
        for (uint32_t k = 0; k < n; ++k) {
            float  v;
            double w;
            if (!in.f32(v) || !in.f64(w))
                return malformed("covariance");
            t.varData.push_back(static_cast<float>(static_cast<double>(v) * w));
        }
        t.varOff.push_back(t.varData.size());
    }
    if (in.atEof())  // stream.good() is false: eofbit (MixtureSet.cc:213)
        return st.fail(GMM_ERR_INVALID_ARGUMENT,
                       "mixture set: end of data inside the last number (the reference's read() fails without "
                       "a trailing line break)");
    return true;
}

// MixtureSet::setOffset then ::setDimension (Module.cc:165-175, MixtureSet.cc:109-126) on one
// table of rows; returns the rows as a dense [rows][dim] array
bool reshapeRows(const std::vector<float>& data, const std::vector<uint64_t>& off, uint32_t offset, uint32_t reduced,
                 uint32_t dim, float pad, const char* what, std::vector<float>& outRows, Status& st) {
    const size_t rows = off.size() - 1;
    outRows.assign(rows * size_t(dim), 0.0f);
    for (size_t r = 0; r < rows; ++r) {
        const uint64_t n = off[r + 1] - off[r];
        if (offset > n)
            return st.fail(GMM_ERR_INVALID_ARGUMENT, std::string("mixture set: ") + what + " " + std::to_string(r) +
                                                             " is shorter than the dimension offset");
        uint64_t len = n - offset;
        if (reduced > 0) {
            len = reduced;  // resize: cut or pad
        }
        if (len != dim)
            return st.fail(GMM_ERR_INVALID_ARGUMENT,
                           std::string("mixture set: ") + what + " " + std::to_string(r) + " has " +
                                   std::to_string(n - offset) + " components, dimension() is " + std::to_string(dim));
        float*         dst  = outRows.data() + r * size_t(dim);
        const float*   src  = data.data() + off[r] + offset;
        const uint64_t have = n - offset;
        for (uint32_t k = 0; k < dim; ++k)
            dst[k] = k < have ? src[k] : pad;
    }
    return true;
}

template <class T>
T* copyOut(const std::vector<T>& v);

// Module_::readMixtureSet's offset / reduced dimension (Module.cc:165-175) on a set already in tables
int offsetAndReduce(gmm_mixture_set* ms, uint32_t offset, uint32_t reduced) {
    if (offset == 0 && reduced == 0)
        return GMM_OK;
    Status                st;
    const uint32_t        D = ms->dimension, dim = reduced > 0 ? reduced : (offset <= D ? D - offset : 0);
    std::vector<float>    m(ms->means, ms->means + size_t(ms->n_means) * D), v(ms->variances, ms->variances + size_t(ms->n_covariances) * D);
    std::vector<uint64_t> mo(ms->n_means + 1), vo(ms->n_covariances + 1);
    for (size_t i = 0; i < mo.size(); ++i)
        mo[i] = i * D;
    for (size_t i = 0; i < vo.size(); ++i)
        vo[i] = i * D;
    std::vector<float> means, vars;
    if (!reshapeRows(m, mo, offset, reduced, dim, 0.0f, "mean", means, st) ||
        !reshapeRows(v, vo, offset, reduced, dim, 1.0f, "covariance", vars, st)) {
        gmm_mixture_set_free(ms);
        setLastError(st.msg);
        return st.code;
    }
    float* nm = copyOut(means);
    float* nv = copyOut(vars);
    if (!nm || !nv) {
        std::free(nm);
        std::free(nv);
        gmm_mixture_set_free(ms);
        setLastError("mixture set: out of host memory");
        return GMM_ERR_OUT_OF_MEMORY;
    }
    std::free(const_cast<float*>(ms->means));
    std::free(const_cast<float*>(ms->variances));
    ms->means     = nm;
    ms->variances = nv;
    ms->dimension = dim;
    return GMM_OK;
}

template <class T>
T* copyOut(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc(std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (p && !v.empty())
        std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

int parseBytes(const unsigned char* data, size_t size, uint32_t offset, uint32_t reduced, gmm_mixture_set* out) {
    if (!out) {
        setLastError("gmm_mixture_set: null output");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    std::memset(out, 0, sizeof(*out));
    std::string inflated;
    const char* begin = reinterpret_cast<const char*>(data);
    const char* end   = begin + size;
    if (isCompressed(data, size)) {
        std::string err;
        if (!inflateAll(data, size, inflated, err)) {
            setLastError("mixture set: " + err);
            return GMM_ERR_INVALID_ARGUMENT;
        }
        begin = inflated.data();
        end   = begin + inflated.size();
    }
    Tables t;
    Status st;
    if (!parseText(begin, end, t, st)) {
        setLastError(st.msg);
        return st.code;
    }
    { std::string().swap(inflated); }
    const uint32_t     dim = reduced > 0 ? reduced : t.dimension;
    std::vector<float> means, vars;
    if (!reshapeRows(t.meanData, t.meanOff, offset, reduced, dim, 0.0f, "mean", means, st) ||
        !reshapeRows(t.varData, t.varOff, offset, reduced, dim, 1.0f, "covariance", vars, st)) {
        setLastError(st.msg);
        return st.code;
    }
    const uint32_t nMeans = static_cast<uint32_t>(t.meanOff.size() - 1);
    const uint32_t nCovs  = static_cast<uint32_t>(t.varOff.size() - 1);
    const uint32_t nDns   = static_cast<uint32_t>(t.dnsMean.size());
    for (uint32_t d = 0; d < nDns; ++d)
        if (t.dnsMean[d] >= nMeans || t.dnsCov[d] >= nCovs) {
            setLastError("mixture set: density " + std::to_string(d) + " refers to mean " +
                         std::to_string(t.dnsMean[d]) + " / covariance " + std::to_string(t.dnsCov[d]) +
                         " (tables hold " + std::to_string(nMeans) + " / " + std::to_string(nCovs) + ")");
            return GMM_ERR_INVALID_ARGUMENT;
        }
    for (size_t e = 0; e < t.mixDns.size(); ++e)
        if (t.mixDns[e] >= nDns) {
            setLastError("mixture set: mixture entry " + std::to_string(e) + " refers to density " +
                         std::to_string(t.mixDns[e]) + " of " + std::to_string(nDns));
            return GMM_ERR_INVALID_ARGUMENT;
        }
    gmm_mixture_set r;
    r.dimension           = dim;
    r.n_means             = nMeans;
    r.means               = copyOut(means);
    r.n_covariances       = nCovs;
    r.variances           = copyOut(vars);
    r.n_densities         = nDns;
    r.density_mean        = copyOut(t.dnsMean);
    r.density_covariance  = copyOut(t.dnsCov);
    r.n_mixtures          = static_cast<uint32_t>(t.mixOff.size() - 1);
    r.mixture_offsets     = copyOut(t.mixOff);
    r.mixture_densities   = copyOut(t.mixDns);
    r.mixture_log_weights = copyOut(t.mixLogW);
    *out                  = r;
    if (!r.means || !r.variances || !r.density_mean || !r.density_covariance || !r.mixture_offsets ||
        !r.mixture_densities || !r.mixture_log_weights) {
        gmm_mixture_set_free(out);
        setLastError("mixture set: out of host memory");
        return GMM_ERR_OUT_OF_MEMORY;
    }
    return GMM_OK;
}

// ---------------------------------------------------------------------------
// tables -> text (operator<< chain of MixtureSet::write with ostream::precision(p))
// ---------------------------------------------------------------------------
class TextSink {
public:
    TextSink(const char* filename, bool gz) : gz_(gz) {
        if (gz_)
            zf_ = gzopen(filename, "wb");
        else
            f_ = std::fopen(filename, "wb");
        buf_.reserve(kFlush + 4096);
    }
    ~TextSink() { close(); }
    bool ok() const { return (gz_ ? zf_ != nullptr : f_ != nullptr) && good_; }

    void str(const char* s) { buf_.append(s); maybeFlush(); }
    void u32(uint32_t v) {
        char b[16];
        std::snprintf(b, sizeof(b), "%u", v);
        str(b);
    }
    void real(double v, int prec) {  // libstdc++ _M_insert_float, default floatfield: "%.*g"
        char b[64];
        std::snprintf(b, sizeof(b), "%.*g", prec, v);
        str(b);
    }
    bool close() {
        flush();
        bool r = good_;
        if (zf_) {
            r = gzclose(zf_) == Z_OK && r;
            zf_ = nullptr;
        }
        if (f_) {
            r = std::fclose(f_) == 0 && r;
            f_ = nullptr;
        }
        good_ = r;
        return r;
    }

private:
    static constexpr size_t kFlush = 1 << 22;
    void maybeFlush() {
        if (buf_.size() >= kFlush)
            flush();
    }
    void flush() {
        if (buf_.empty() || !ok())
            return;
        if (gz_)
            good_ = gzwrite(zf_, buf_.data(), static_cast<unsigned>(buf_.size())) == static_cast<int>(buf_.size());
        else
            good_ = std::fwrite(buf_.data(), 1, buf_.size(), f_) == buf_.size();
        buf_.clear();
    }

    bool        gz_;
    gzFile      zf_ = nullptr;
    FILE*       f_  = nullptr;
    bool        good_ = true;
    std::string buf_;
};

bool endsWith(const std::string& s, const char* suffix) {
    const size_t n = std::strlen(suffix);
    return s.size() >= n && s.compare(s.size() - n, n, suffix) == 0;
}

}  // namespace

extern "C" {

int gmm_mixture_set_parse(const void* data, uint64_t size, uint32_t dimension_offset, uint32_t reduced_dimension,
                          gmm_mixture_set* out) {
    if (!data && size) {
        setLastError("gmm_mixture_set_parse: null data");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    static const unsigned char empty = 0;
    return parseBytes(data ? static_cast<const unsigned char*>(data) : &empty, static_cast<size_t>(size),
                      dimension_offset, reduced_dimension, out);
}

int gmm_mixture_set_read(const char* filename, uint32_t dimension_offset, uint32_t reduced_dimension,
                         gmm_mixture_set* out) {
    return gmm_mixture_set_read_config(filename, nullptr, dimension_offset, reduced_dimension, out);
}

int gmm_mixture_set_read_config(const char* filename, const gmm_estimator_config* config, uint32_t dimension_offset,
                                uint32_t reduced_dimension, gmm_mixture_set* out) {
    if (!filename || !out) {
        setLastError("gmm_mixture_set_read: null argument");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    std::memset(out, 0, sizeof(*out));
    FILE* f = std::fopen(filename, "rb");
    if (!f) {
        setLastError(std::string("mixture set: cannot open \"") + filename + "\": " + std::strerror(errno));
        return GMM_ERR_INVALID_ARGUMENT;
    }
    std::vector<unsigned char> bytes;
    unsigned char              chunk[1 << 16];
    size_t                     n;
    while ((n = std::fread(chunk, 1, sizeof(chunk), f)) > 0)
        bytes.insert(bytes.end(), chunk, chunk + n);
    const bool readErr = std::ferror(f) != 0;
    std::fclose(f);
    if (readErr) {
        setLastError(std::string("mixture set: read error on \"") + filename + "\"");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    // MixtureSetReader: ".pms" / ".gz" (Core::filenameExtension, the text after the last '.' of the last path
    // component) through the format reader, any other name through the estimator reader
    const std::string name(filename);
    const size_t      dot = name.find_last_of("./");
    const std::string ext = dot != std::string::npos && name[dot] == '.' ? name.substr(dot) : std::string();
    int               rc;
    if (ext == ".pms" || ext == ".gz")
        rc = parseBytes(bytes.empty() ? chunk : bytes.data(), bytes.size(), dimension_offset, reduced_dimension, out);
    else if ((rc = gmm_mixture_set_estimate(bytes.data(), bytes.size(), config, out)) == GMM_OK)
        rc = offsetAndReduce(out, dimension_offset, reduced_dimension);
    if (rc != GMM_OK) {
        const std::string msg = std::string("\"") + filename + "\": ";
        setLastError(msg + gmm_last_error());
    }
    return rc;
}

int gmm_mixture_set_free(gmm_mixture_set* ms) {
    if (!ms)
        return GMM_ERR_INVALID_ARGUMENT;
    std::free(const_cast<float*>(ms->means));
    std::free(const_cast<float*>(ms->variances));
    std::free(const_cast<uint32_t*>(ms->density_mean));
    std::free(const_cast<uint32_t*>(ms->density_covariance));
    std::free(const_cast<uint32_t*>(ms->mixture_offsets));
    std::free(const_cast<uint32_t*>(ms->mixture_densities));
    std::free(const_cast<double*>(ms->mixture_log_weights));
    std::memset(ms, 0, sizeof(*ms));
    return GMM_OK;
}

int gmm_mixture_set_write(const char* filename, const gmm_mixture_set* ms, uint32_t precision) {
    if (!filename || !ms) {
        setLastError("gmm_mixture_set_write: null argument");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    if (ms->n_covariances == 0) {  // MixtureSet::write inspects covariance(0) (MixtureSet.cc:145)
        setLastError("gmm_mixture_set_write: a mixture set without covariances has no covariance type");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    const std::string name(filename);
    TextSink          out(filename, endsWith(name, ".gz") || endsWith(name, ".Z"));
    if (!out.ok()) {
        setLastError(std::string("mixture set: cannot open \"") + filename + "\" for writing");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    const int      p = static_cast<int>(precision);
    const uint32_t D = ms->dimension;
    out.str("#Version: 2.0\n#CovarianceType: DiagonalCovariance\n");
    out.u32(D), out.str(" "), out.u32(ms->n_mixtures), out.str(" "), out.u32(ms->n_densities), out.str(" ");
    out.u32(ms->n_means), out.str(" "), out.u32(ms->n_covariances), out.str("\n");
    for (uint32_t m = 0; m < ms->n_mixtures; ++m) {  // Mixture::write (Mixture.cc:81-88)
        const uint32_t b = ms->mixture_offsets[m], e = ms->mixture_offsets[m + 1];
        out.u32(e - b);
        for (uint32_t k = b; k < e; ++k) {
            out.str(" "), out.u32(ms->mixture_densities[k]), out.str(" ");
            out.real(ms->mixture_log_weights[k], p);
        }
        out.str("\n");
    }
    for (uint32_t d = 0; d < ms->n_densities; ++d) {  // MixtureSetTopology.cc:19-22
        out.u32(ms->density_mean[d]), out.str(" "), out.u32(ms->density_covariance[d]), out.str("\n");
    }
    for (uint32_t i = 0; i < ms->n_means; ++i) {  // Mean::write (GaussDensity.cc:25-31)
        out.u32(D);
        for (uint32_t k = 0; k < D; ++k)
            out.str(" "), out.real(ms->means[size_t(i) * D + k], p);
        out.str("\n");
    }
    for (uint32_t i = 0; i < ms->n_covariances; ++i) {  // " " << DiagonalCovariance (MixtureSet.cc:164-166)
        out.str(" "), out.u32(D);
        for (uint32_t k = 0; k < D; ++k)
            out.str(" "), out.real(ms->variances[size_t(i) * D + k], p), out.str(" 1");
        out.str("\n");
    }
    if (!out.close()) {
        setLastError(std::string("mixture set: write error on \"") + filename + "\"");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    return GMM_OK;
}

}  // extern "C"
