// TEST DOUBLE: Nn::ClassLabelWrapper -- the mapping generated from the configuration (src/Nn/ClassLabelWrapper.cc:
// 35-75): classes listed in "disregard-classes" get no network output, the others consecutive outputs.
#pragma once
#include <cstdlib>
#include <string>
#include <vector>
#include <Core/Component.hh>
#include <Core/Types.hh>
namespace Nn {
class ClassLabelWrapper : public Core::Component {
public:
    ClassLabelWrapper(const Core::Configuration& c, u32 nClasses) : Core::Component(c), mapping_(nClasses, -1) {
        std::vector<u32> disregard;
        std::string      v;
        if (c.get("disregard-classes", v))
            for (char* p = &v[0]; *p;) {
                char*      e = 0;
                const long x = std::strtol(p, &e, 10);
                if (e == p)
                    break;
                disregard.push_back(static_cast<u32>(x));
                p = *e ? e + 1 : e;
            }
        for (u32 k = 0; k < nClasses; ++k) {
            bool skip = false;
            for (u32 d : disregard)
                skip = skip || d == k;
            if (!skip)
                mapping_[k] = static_cast<s32>(nTargets_++);
        }
    }
    bool isOneToOneMapping() const { return nTargets_ == mapping_.size(); }
    u32  nClassesToAccumulate() const { return nTargets_; }
    bool isClassToAccumulate(u32 k) const { return mapping_.at(k) >= 0; }
    u32  getOutputIndexFromClassIndex(u32 k) const { return static_cast<u32>(mapping_.at(k)); }

private:
    std::vector<s32> mapping_;
    u32              nTargets_ = 0;
};
}  // namespace Nn
