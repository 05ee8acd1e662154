// TEST DOUBLE: Nn::Prior<T> -- "prior-file" / "priori-scale" (src/Nn/Prior.cc:22-28) and setFromMixtureSet
// (Prior.cc:159-190: f32 per-mixture weight sums, the total accumulated from 0.0 in double, std::log in f32).  A
// prior file is in a format of THIS double (little-endian f32 log priors), not RASR's.
#pragma once
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>
#include <Core/Component.hh>
#include <Core/ReferenceCounting.hh>
#include <Mm/MixtureSet.hh>
#include "ClassLabelWrapper.hh"
namespace Nn {
template <class T>
class Prior : public Core::Component {
public:
    explicit Prior(const Core::Configuration& c) : Core::Component(c) {
        std::string v;
        if (c.get("prior-file", v))
            file_ = v;
        if (c.get("priori-scale", v))
            scale_ = static_cast<T>(std::strtod(v.c_str(), 0));
    }
    T           scale() const { return scale_; }
    std::string fileName() const { return file_; }
    size_t      size() const { return logPrior_.size(); }
    const T&    at(size_t n) const { return logPrior_.at(n); }
    bool        read() {
        FILE* f = std::fopen(file_.c_str(), "rb");
        if (!f)
            return false;
        T x;
        logPrior_.clear();
        while (std::fread(&x, sizeof(T), 1, f) == 1)
            logPrior_.push_back(x);
        std::fclose(f);
        return true;
    }
    void setFromMixtureSet(Core::Ref<const Mm::MixtureSet> ms, const ClassLabelWrapper& labels) {
        std::vector<f32> p(ms->nMixtures(), 0.0f);
        for (size_t m = 0; m < ms->nMixtures(); ++m)
            for (size_t d = 0; d < ms->mixture(m)->nDensities(); ++d)
                p.at(m) += ms->mixture(m)->weight(d);
        logPrior_.assign(labels.nClassesToAccumulate(), T(0));
        for (u32 m = 0; m < ms->nMixtures(); ++m)
            if (labels.isClassToAccumulate(m))
                logPrior_.at(labels.getOutputIndexFromClassIndex(m)) = p.at(m);
        const f32 total = std::accumulate(logPrior_.begin(), logPrior_.end(), 0.0);
        for (T& v : logPrior_)
            v = std::log(v / total);
    }

private:
    std::string    file_;
    T              scale_ = T(1);
    std::vector<T> logPrior_;
};
}  // namespace Nn
