// pms_istream.cc -- TEST INFRASTRUCTURE ONLY (checker, never shipped or called by the product).
//
// Restatement of the reference's mixture-set text reader on std::istream, i.e. with the
// very libstdc++ extraction operators the reference uses, to pin the product's own
// tokenizer (rasr_amd/csrc/host/MixtureSetFile.cc):
//   MixtureSet::read            src/Mm/MixtureSet.cc:170-214
//   Mixture::read / addDensity  src/Mm/Mixture.cc:56-66, 90-107
//   GaussDensityTopology::read  src/Mm/MixtureSetTopology.cc:23-30
//   Mean::read                  src/Mm/GaussDensity.cc:32-43
//   DiagonalCovariance::read    src/Mm/GaussDensity.cc:54-69
//   setOffset / setDimension    src/Mm/MixtureSet.cc:109-126, GaussDensity.hh:187-194
//   CompressedInputStream       src/Core/CompressedStream.cc:37-54 (here: gzread, which also
//                               passes uncompressed files through)
// Returns 0 when the reference's read() would return true (stream.good()), 1 otherwise,
// 2 for a version above 2.0 (criticalError), 3 for a covariance type other than
// DiagonalCovariance (error()), 4 for a header line too short for substr (std::out_of_range).
#include <zlib.h>

#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <string>
#include <vector>

extern "C" {
typedef struct {
    uint32_t        dimension;
    uint32_t        n_means;
    float*          means;
    uint32_t        n_covariances;
    float*          variances;
    uint32_t        n_densities;
    uint32_t*       density_mean;
    uint32_t*       density_covariance;
    uint32_t        n_mixtures;
    uint32_t*       mixture_offsets;
    uint32_t*       mixture_densities;
    double*         mixture_log_weights;
} orc_mixture_set;  // layout of gmm_mixture_set (include/rasr_gmm.h)
}

namespace {

template <class T>
T* out(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc((v.size() + 1) * sizeof(T)));
    if (!v.empty())
        std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

bool slurp(const char* path, std::string& text) {
    gzFile f = gzopen(path, "rb");
    if (!f)
        return false;
    char buf[1 << 16];
    int  n;
    while ((n = gzread(f, buf, sizeof(buf))) > 0)
        text.append(buf, static_cast<size_t>(n));
    gzclose(f);
    return n == 0;
}

}  // namespace

extern "C" int orc_pms_read(const char* path, uint32_t offset, uint32_t reduced, orc_mixture_set* res) {
    std::memset(res, 0, sizeof(*res));
    std::string text;
    if (!slurp(path, text))
        return 1;
    std::istringstream i(text);
    std::string        line;
    std::getline(i, line);
    if (line.size() < 10)
        return 4;
    const float version = static_cast<float>(std::atof(line.substr(10).c_str()));
    if (version > 2.0)
        return 2;
    std::getline(i, line);
    if (line.size() < 17)
        return 4;
    if (line.substr(17).compare("DiagonalCovariance") != 0)
        return 3;
    uint32_t dim, nMix, nDns, nMean, nCov;
    i >> dim >> nMix >> nDns >> nMean >> nCov;

    std::vector<uint32_t> mixOff{0}, mixDns, dnsMean, dnsCov;
    std::vector<double>   logW;
    while (0 < nMix--) {
        uint32_t ndns;
        i >> ndns;
        uint32_t dns;
        double   w;
        while (0 < ndns--) {
            i >> dns >> w;
            if (!i)
                return 1;  // (the reference keeps looping on a failed stream; the outcome is the same)
            mixDns.push_back(dns);
            logW.push_back(version < 2.0 ? (w > 0 ? std::log(w) : -DBL_MAX) : w);
        }
        mixOff.push_back(static_cast<uint32_t>(mixDns.size()));
        if (!i)
            return 1;
    }
    while (0 < nDns--) {
        uint32_t m, c;
        i >> m >> c;
        if (!i)
            return 1;
        dnsMean.push_back(m);
        dnsCov.push_back(c);
    }
    std::vector<std::vector<float>> means, vars;
    while (0 < nMean--) {
        uint32_t d;
        i >> d;
        std::vector<float> mean;
        float              melem;
        while (0 < d) {
            i >> melem;
            if (!i)
                return 1;
            mean.push_back(melem);
            d--;
        }
        means.push_back(mean);
        if (!i)
            return 1;
    }
    while (0 < nCov--) {
        uint32_t d;
        i >> d;
        std::vector<float> v;
        float              velem;
        double             welem;
        while (0 < d) {
            i >> velem >> welem;
            if (!i)
                return 1;
            v.push_back(velem * welem);
            d--;
        }
        vars.push_back(v);
        if (!i)
            return 1;
    }
    if (!i.good())
        return 1;
    // Module_::readMixtureSet: setOffset, then setDimension (means pad 0, covariances pad 1)
    for (auto& m : means) {
        if (offset > m.size())
            return 1;
        m.erase(m.begin(), m.begin() + offset);
    }
    for (auto& v : vars) {
        if (offset > v.size())
            return 1;
        v.erase(v.begin(), v.begin() + offset);
    }
    if (reduced > 0) {
        dim = reduced;
        for (auto& m : means)
            m.resize(dim, 0.0f);
        for (auto& v : vars)
            v.resize(dim, 1.0f);
    }
    std::vector<float> flatM, flatV;
    for (auto& m : means) {
        if (m.size() != dim)
            return 1;
        flatM.insert(flatM.end(), m.begin(), m.end());
    }
    for (auto& v : vars) {
        if (v.size() != dim)
            return 1;
        flatV.insert(flatV.end(), v.begin(), v.end());
    }
    res->dimension           = dim;
    res->n_means             = static_cast<uint32_t>(means.size());
    res->means               = out(flatM);
    res->n_covariances       = static_cast<uint32_t>(vars.size());
    res->variances           = out(flatV);
    res->n_densities         = static_cast<uint32_t>(dnsMean.size());
    res->density_mean        = out(dnsMean);
    res->density_covariance  = out(dnsCov);
    res->n_mixtures          = static_cast<uint32_t>(mixOff.size() - 1);
    res->mixture_offsets     = out(mixOff);
    res->mixture_densities   = out(mixDns);
    res->mixture_log_weights = out(logW);
    return 0;
}

extern "C" void orc_pms_free(orc_mixture_set* ms) {
    std::free(ms->means);
    std::free(ms->variances);
    std::free(ms->density_mean);
    std::free(ms->density_covariance);
    std::free(ms->mixture_offsets);
    std::free(ms->mixture_densities);
    std::free(ms->mixture_log_weights);
    std::memset(ms, 0, sizeof(*ms));
}
