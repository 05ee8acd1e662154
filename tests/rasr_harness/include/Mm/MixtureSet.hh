// TEST DOUBLE: Mm::MixtureSet with the accessors the adapter's conversion reads
#pragma once
#include <cmath>
#include <vector>
#include <Core/ReferenceCounting.hh>
#include "Types.hh"
namespace Mm {
class AbstractMixtureSet : public Core::ReferenceCounted {
public:
    virtual ~AbstractMixtureSet() {}
};
class Mean : public std::vector<MeanType> {
public:
    explicit Mean(const std::vector<MeanType>& v) : std::vector<MeanType>(v) {}
};
class Covariance {
public:
    explicit Covariance(const std::vector<VarianceType>& d) : d_(d) {}
    const std::vector<VarianceType>& diagonal() const { return d_; }

private:
    std::vector<VarianceType> d_;
};
class GaussDensity {
public:
    GaussDensity(MeanIndex m, CovarianceIndex c) : m_(m), c_(c) {}
    MeanIndex       meanIndex() const { return m_; }
    CovarianceIndex covarianceIndex() const { return c_; }

private:
    MeanIndex       m_;
    CovarianceIndex c_;
};
class Mixture {
public:
    void         addLogDensity(DensityIndex d, Weight logWeight) { d_.push_back(d); w_.push_back(logWeight); }
    DensityIndex nDensities() const { return static_cast<DensityIndex>(d_.size()); }
    DensityIndex densityIndex(DensityIndex j) const { return d_[j]; }
    Weight       logWeight(size_t j) const { return w_[j]; }
    Weight       weight(size_t j) const { return std::exp(w_[j]); }  // Mixture::weight, src/Mm/Mixture.hh

private:
    std::vector<DensityIndex> d_;
    std::vector<Weight>       w_;
};
class MixtureSet : public AbstractMixtureSet {
public:
    explicit MixtureSet(ComponentIndex dimension) : dimension_(dimension) {}
    ComponentIndex      dimension() const { return dimension_; }
    MeanIndex           addMean(const std::vector<MeanType>& m) { means_.push_back(Mean(m)); return static_cast<MeanIndex>(means_.size() - 1); }
    CovarianceIndex     addCovariance(const std::vector<VarianceType>& d) { covs_.push_back(Covariance(d)); return static_cast<CovarianceIndex>(covs_.size() - 1); }
    DensityIndex        addDensity(MeanIndex m, CovarianceIndex c) { dens_.push_back(GaussDensity(m, c)); return static_cast<DensityIndex>(dens_.size() - 1); }
    MixtureIndex        addMixture(const Mixture& x) { mix_.push_back(x); return static_cast<MixtureIndex>(mix_.size() - 1); }
    MeanIndex           nMeans() const { return static_cast<MeanIndex>(means_.size()); }
    const Mean*         mean(MeanIndex i) const { return &means_[i]; }
    CovarianceIndex     nCovariances() const { return static_cast<CovarianceIndex>(covs_.size()); }
    const Covariance*   covariance(CovarianceIndex i) const { return &covs_[i]; }
    DensityIndex        nDensities() const { return static_cast<DensityIndex>(dens_.size()); }
    const GaussDensity* density(DensityIndex i) const { return &dens_[i]; }
    MixtureIndex        nMixtures() const { return static_cast<MixtureIndex>(mix_.size()); }
    const Mixture*      mixture(MixtureIndex m) const { return &mix_[m]; }

private:
    ComponentIndex            dimension_;
    std::vector<Mean>         means_;
    std::vector<Covariance>   covs_;
    std::vector<GaussDensity> dens_;
    std::vector<Mixture>      mix_;
};
}  // namespace Mm
