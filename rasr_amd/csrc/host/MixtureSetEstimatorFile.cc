// MixtureSetEstimatorFile.cc -- mixture sets from RASR's binary estimator (accumulator) files.
//
// Every file name whose extension is not ".pms" or ".gz" is read by the reference as a maximum-
// likelihood mixture-set estimator file and the mixture set is estimated from it:
//   MixtureSetReader::read                     src/Mm/MixtureSetReader.hh:105-117 (default reader)
//   MixtureSetEstimatorReader::read            src/Mm/MixtureSetReader.cc:52-74
//   Module_::createMixtureSetEstimator         src/Mm/Module.cc:211-227 ("estimator-type" maximum-likelihood)
//   AbstractMixtureSetEstimator::read          src/Mm/AbstractMixtureSetEstimator.cc:404-414, 433-479
//   AbstractMixtureSetEstimator::estimate      src/Mm/AbstractMixtureSetEstimator.cc:299-337
//   MixtureSetEstimatorIndexMap                src/Mm/AbstractMixtureSetEstimator.cc:804-817
//   Mean/CovarianceEstimator::estimate         src/Mm/GaussDensityEstimator.cc:148-227
//   AbstractMixtureEstimator::read/estimate    src/Mm/MixtureEstimator.cc:47-66, 112-123, 140-161
//   VectorAccumulator::read                    src/Mm/VectorAccumulator.hh (size, f64 sums, weight)
//   Mixture::addDensity / normalizeWeights     src/Mm/Mixture.cc:63-74, logExpNorm Utilities.hh:44-51
// Core::BinaryInputStream: native (little-endian) byte order, no compression.
//
// The arithmetic follows the reference in f64 with the reference's operation order, results stored as
// f32 means / variances and f64 log weights.  One order is not defined by the reference: the covariance
// estimate sums the squared mean statistics of the covariance's means in the iteration order of an
// unordered_set of pointers (GaussDensityEstimator.hh CovarianceToMeanSetMap); here they are summed in mean
// index order (f64 sums of positive terms: the order moves the f32 variance only on an exact rounding tie).
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <set>
#include <string>
#include <vector>

#include "../../../include/rasr_gmm_io.h"

namespace rasr_gmm {
void setLastError(const std::string& msg);
}
using rasr_gmm::setLastError;

namespace {

struct Reader {  // Core::BinaryInputStream over a byte buffer
    const unsigned char* p;
    const unsigned char* end;
    bool                 fail = false;
    template <class T>
    T get() {
        T v{};
        if (static_cast<size_t>(end - p) < sizeof(T)) {
            fail = true;
            p    = end;
            return v;
        }
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
};

struct Accumulator {  // VectorAccumulator<..., Sum = f64>
    std::vector<double> sum;
    double              weight = 0;
    void read(Reader& r, uint32_t version) {
        const uint32_t n = r.get<uint32_t>();
        if (r.fail || static_cast<uint64_t>(n) * 8 > static_cast<uint64_t>(r.end - r.p)) {
            r.fail = true;
            return;
        }
        sum.resize(n);
        for (uint32_t k = 0; k < n; ++k)
            sum[k] = r.get<double>();
        weight = version > 0 ? r.get<double>() : static_cast<double>(r.get<uint32_t>());
    }
};

struct DensityEst {
    uint32_t mean = 0, cov = 0;
};
struct MixtureEst {
    std::vector<uint32_t> dens;     // density estimator indices
    std::vector<double>   weights;  // Weight per density
    double                weight() const {  // getWeight: std::accumulate(..., 0.0)
        double s = 0.0;
        for (double w : weights)
            s += w;
        return s;
    }
};

// Core::differenceUlp(f64, f64), src/Core/Utility.cc:75-87
int64_t differenceUlp(double af, double bf) {
    int64_t a, b;
    std::memcpy(&a, &af, 8);
    std::memcpy(&b, &bf, 8);
    if (a < 0)
        a = static_cast<int64_t>((static_cast<uint64_t>(1) << 63) - static_cast<uint64_t>(a));
    if (b < 0)
        b = static_cast<int64_t>((static_cast<uint64_t>(1) << 63) - static_cast<uint64_t>(b));
    const int64_t d = a - b;
    return d < 0 ? -d : d;
}

template <class T>
T* copyOut(const std::vector<T>& v) {
    T* p = static_cast<T*>(std::malloc(std::max<size_t>(v.size(), 1) * sizeof(T)));
    if (p && !v.empty())
        std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

// first-appearance index of a pointer (PointerIndexMap::add)
struct IndexMap {
    std::vector<int64_t>  index;  // estimator -> new index or -1
    std::vector<uint32_t> order;  // new index -> estimator
    explicit IndexMap(size_t n) : index(n, -1) {}
    void add(uint32_t e) {
        if (index[e] < 0) {
            index[e] = static_cast<int64_t>(order.size());
            order.push_back(e);
        }
    }
};

int fail(int code, const std::string& msg) {
    setLastError("mixture set estimator: " + msg);
    return code;
}

}  // namespace

extern "C" {

void gmm_default_estimator_config(gmm_estimator_config* c) {
    if (!c)
        return;
    c->minimum_observation_weight = 5.0;  // AbstractMixtureSetEstimator.cc:25-28
    c->minimum_relative_weight    = 0.0;  // :30-33
    c->minimum_variance           = 0.0;  // :35-38
    c->allow_zero_weights         = 0;    // :50-53
    c->normalize_mixture_weights  = 1;    // :55-58
}

int gmm_mixture_set_estimate(const void* data, uint64_t size, const gmm_estimator_config* config,
                             gmm_mixture_set* out) {
    if (!out || (!data && size))
        return fail(GMM_ERR_INVALID_ARGUMENT, "null argument");
    std::memset(out, 0, sizeof(*out));
    gmm_estimator_config cfg;
    gmm_default_estimator_config(&cfg);
    if (config)
        cfg = *config;
    static const unsigned char empty = 0;
    Reader r{data ? static_cast<const unsigned char*>(data) : &empty,
             (data ? static_cast<const unsigned char*>(data) : &empty) + size};

    // ---- AbstractMixtureSetEstimator::readHeader / read ----
    char magic[8];
    for (char& c : magic)
        c = static_cast<char>(r.get<uint8_t>());
    // strcmp(_magic, "MIXSET") (MixtureSetEstimator.hh:36): the six letters then a NUL within the 8 bytes
    if (r.fail || std::memcmp(magic, "MIXSET", 7) != 0)
        return fail(GMM_ERR_INVALID_ARGUMENT, "magic \"MIXSET\" expected (criticalError, AbstractMixtureSetEstimator.cc:404-411)");
    const uint32_t version   = r.get<uint32_t>();
    const uint32_t dimension = r.get<uint32_t>();
    const uint32_t nMeans    = r.get<uint32_t>();
    if (r.fail)
        return fail(GMM_ERR_INVALID_ARGUMENT, "error reading mixture set estimator (header)");
    std::vector<Accumulator> means, covs;
    for (uint32_t i = 0; i < nMeans && !r.fail; ++i) {
        means.emplace_back();
        means.back().read(r, version);
    }
    const uint32_t nCovs = r.get<uint32_t>();
    for (uint32_t i = 0; i < nCovs && !r.fail; ++i) {
        covs.emplace_back();
        covs.back().read(r, version);
    }
    const uint32_t          nDens = r.get<uint32_t>();
    std::vector<DensityEst> dens;
    for (uint32_t i = 0; i < nDens && !r.fail; ++i) {
        DensityEst d;
        d.mean = r.get<uint32_t>();
        d.cov  = r.get<uint32_t>();
        if (!r.fail && (d.mean >= nMeans || d.cov >= nCovs))
            return fail(GMM_ERR_INVALID_ARGUMENT, "density estimator " + std::to_string(i) + " refers to mean " +
                                                          std::to_string(d.mean) + " / covariance " + std::to_string(d.cov) +
                                                          " (file holds " + std::to_string(nMeans) + " / " +
                                                          std::to_string(nCovs) + ")");
        dens.push_back(d);
    }
    const uint32_t          nMix = r.get<uint32_t>();
    std::vector<MixtureEst> mix;
    for (uint32_t m = 0; m < nMix && !r.fail; ++m) {
        MixtureEst     x;
        const uint32_t n = r.get<uint32_t>();
        if (r.fail || static_cast<uint64_t>(n) * 8 > static_cast<uint64_t>(r.end - r.p)) {
            r.fail = true;
            break;
        }
        for (uint32_t j = 0; j < n && !r.fail; ++j) {
            const uint32_t di = r.get<uint32_t>();
            const double   w  = version > 0 ? r.get<double>() : static_cast<double>(r.get<uint32_t>());
            if (!r.fail && di >= nDens)
                return fail(GMM_ERR_INVALID_ARGUMENT, "mixture " + std::to_string(m) + " refers to density estimator " +
                                                              std::to_string(di) + " of " + std::to_string(nDens));
            x.dens.push_back(di);
            x.weights.push_back(w);
        }
        mix.push_back(std::move(x));
    }
    if (r.fail)  // is.fail(): "error reading mixture set estimator" (cc:469-471), the reader fails (MixtureSetReader.cc:68-71)
        return fail(GMM_ERR_INVALID_ARGUMENT, "error reading mixture set estimator (truncated file)");
    for (const Accumulator& a : means)
        if (a.sum.size() != dimension)
            return fail(GMM_ERR_INVALID_ARGUMENT, "a mean accumulator has " + std::to_string(a.sum.size()) +
                                                          " components, dimension is " + std::to_string(dimension));
    for (const Accumulator& a : covs)
        if (a.sum.size() != dimension)
            return fail(GMM_ERR_INVALID_ARGUMENT, "a covariance accumulator has " + std::to_string(a.sum.size()) +
                                                          " components, dimension is " + std::to_string(dimension));

    // ---- estimate (cc:305-337) ----
    if (!cfg.allow_zero_weights)  // checkEventsWithZeroWeight (cc:422-431): zero-weight mixture -> criticalError
        for (uint32_t m = 0; m < nMix; ++m)
            if (mix[m].weight() == 0)
                return fail(GMM_ERR_INVALID_ARGUMENT, "Mixture " + std::to_string(m) + " has zero weight.");
    // CovarianceToMeanSetMap over the density estimators in index-map order, before the removal
    std::vector<std::set<uint32_t>> meanSet(nCovs);
    {
        IndexMap dm(nDens);
        for (const MixtureEst& x : mix)
            for (uint32_t d : x.dens)
                dm.add(d);
        for (uint32_t d : dm.order)
            meanSet[dens[d].cov].insert(dens[d].mean);
    }
    // removeDensitiesWithLowWeight (MixtureEstimator.cc:47-66)
    for (uint32_t m = 0; m < nMix; ++m) {
        MixtureEst& x = mix[m];
        if (x.dens.empty())  // densityIndexWithMaxWeight: verify(!densityEstimators_.empty())
            return fail(GMM_ERR_INVALID_ARGUMENT, "mixture " + std::to_string(m) + " has no densities");
        size_t densityMax = 0;
        for (size_t j = 1; j < x.dens.size(); ++j)
            if (x.weights[j] > x.weights[densityMax])
                densityMax = j;
        const double minWeight = std::max(cfg.minimum_observation_weight, x.weight() * cfg.minimum_relative_weight);
        for (size_t j = 0; j < x.dens.size();) {
            if (!(x.weights[j] >= minWeight) && j != densityMax) {
                x.dens.erase(x.dens.begin() + static_cast<long>(j));
                x.weights.erase(x.weights.begin() + static_cast<long>(j));
                if (densityMax > j)
                    --densityMax;
            }
            else
                ++j;
        }
    }
    // MixtureSetEstimatorIndexMap after the removal: first appearance over mixtures, densities in order
    IndexMap meanMap(nMeans), covMap(nCovs), densMap(nDens);
    for (const MixtureEst& x : mix)
        for (uint32_t d : x.dens) {
            meanMap.add(dens[d].mean);
            covMap.add(dens[d].cov);
            densMap.add(d);
        }

    std::vector<uint32_t> mixOff{0}, mixDens;
    std::vector<double>   mixLogW;
    for (const MixtureEst& x : mix) {
        std::vector<double> lw;
        for (size_t j = 0; j < x.dens.size(); ++j) {
            mixDens.push_back(static_cast<uint32_t>(densMap.index[x.dens[j]]));
            // Mixture::addDensity: log(weight), Core::Type<Weight>::min for weight <= 0
            lw.push_back(x.weights[j] > 0 ? std::log(x.weights[j]) : -std::numeric_limits<double>::max());
        }
        if (cfg.normalize_mixture_weights && !lw.empty()) {  // Mixture::normalizeWeights, logExpNorm
            size_t maxIt = 0;
            for (size_t j = 1; j < lw.size(); ++j)
                if (lw[maxIt] < lw[j])
                    maxIt = j;
            double result = 0;
            for (size_t j = 0; j < lw.size(); ++j)
                if (j != maxIt)
                    result += std::exp(lw[j] - lw[maxIt]);
            const double logNorm = std::log1p(result) + lw[maxIt];
            for (double& v : lw)
                v = v - logNorm;
        }
        mixLogW.insert(mixLogW.end(), lw.begin(), lw.end());
        mixOff.push_back(static_cast<uint32_t>(mixDens.size()));
    }
    std::vector<uint32_t> dnsMean, dnsCov;
    for (uint32_t d : densMap.order) {
        dnsMean.push_back(static_cast<uint32_t>(meanMap.index[dens[d].mean]));
        dnsCov.push_back(static_cast<uint32_t>(covMap.index[dens[d].cov]));
    }
    const size_t       D = dimension;
    std::vector<float> meanOut(meanMap.order.size() * D, 0.0f), varOut(covMap.order.size() * D, 1.0f);
    for (size_t i = 0; i < meanMap.order.size(); ++i) {  // MeanEstimator::estimate: sum / weight, zero if weight 0
        const Accumulator& a = means[meanMap.order[i]];
        if (a.weight == 0)
            continue;
        for (size_t k = 0; k < D; ++k)
            meanOut[i * D + k] = static_cast<float>(a.sum[k] / a.weight);
    }
    const float minVariance = static_cast<float>(cfg.minimum_variance);  // VarianceType minVariance_
    for (size_t i = 0; i < covMap.order.size(); ++i) {  // CovarianceEstimator::estimate (cc:201-227)
        const uint32_t     c = covMap.order[i];
        const Accumulator& a = covs[c];
        if (a.weight == 0)  // new DiagonalCovariance(size): variances 1
            continue;
        // GaussDensityEstimator / CovarianceEstimator: verify(accumulator_.weight() > 0) (GaussDensityEstimator.cc:216)
        if (!(a.weight > 0) || !std::isfinite(a.weight))
            return fail(GMM_ERR_INVALID_ARGUMENT, "covariance " + std::to_string(c) + " has weight " +
                                                          std::to_string(a.weight) + " (verify(weight > 0) failed)");
        std::vector<double> wmss(D, 0.0);  // WeighedMeanSquareSum: x + y * y / meanWeight
        double              wmssWeight = 0;
        for (uint32_t mi : meanSet[c]) {
            const Accumulator& ma = means[mi];
            if (ma.weight > 0) {
                for (size_t k = 0; k < D; ++k)
                    wmss[k] = wmss[k] + ma.sum[k] * ma.sum[k] / ma.weight;
                wmssWeight += ma.weight;
            }
        }
        if (differenceUlp(a.weight, wmssWeight) > static_cast<int64_t>(1e12))  // verify(isAlmostEqualUlp(...))
            return fail(GMM_ERR_INVALID_ARGUMENT, "covariance " + std::to_string(c) + " has weight " +
                                                          std::to_string(a.weight) + " but its means weigh " +
                                                          std::to_string(wmssWeight) + " (verify failed)");
        for (size_t k = 0; k < D; ++k) {
            float v = static_cast<float>((a.sum[k] - wmss[k]) / a.weight);  // normalizedMinus<Sum>
            if (minVariance != 0 && v < minVariance)                        // applyMinimumVariance
                v = minVariance;
            varOut[i * D + k] = v;
        }
    }

    gmm_mixture_set res;
    res.dimension           = dimension;
    res.n_means             = static_cast<uint32_t>(meanMap.order.size());
    res.means               = copyOut(meanOut);
    res.n_covariances       = static_cast<uint32_t>(covMap.order.size());
    res.variances           = copyOut(varOut);
    res.n_densities         = static_cast<uint32_t>(densMap.order.size());
    res.density_mean        = copyOut(dnsMean);
    res.density_covariance  = copyOut(dnsCov);
    res.n_mixtures          = nMix;
    res.mixture_offsets     = copyOut(mixOff);
    res.mixture_densities   = copyOut(mixDens);
    res.mixture_log_weights = copyOut(mixLogW);
    *out                    = res;
    if (!res.means || !res.variances || !res.density_mean || !res.density_covariance || !res.mixture_offsets ||
        !res.mixture_densities || !res.mixture_log_weights) {
        gmm_mixture_set_free(out);
        return fail(GMM_ERR_OUT_OF_MEMORY, "out of host memory");
    }
    return GMM_OK;
}

}  // extern "C"
