// TEST DOUBLE: typed parameters read from a Configuration (Core::ParameterInt / ParameterFloat)
#pragma once
#include <cstdlib>
#include <string>
#include "Configuration.hh"
#include "Assertions.hh"
#include "Types.hh"
namespace Core {
template <class T>
class Parameter {
public:
    Parameter(const char* name, const char* description, T def, T min = std::numeric_limits<T>::lowest(),
              T max = std::numeric_limits<T>::max())
            : name_(name), def_(def), min_(min), max_(max) { (void)description; }
    T operator()(const Configuration& c) const {
        std::string v;
        if (!c.get(name_, v))
            return def_;
        const T x = static_cast<T>(std::strtod(v.c_str(), 0));
        require(x >= min_ && x <= max_);
        return x;
    }
    T operator()(const Configuration& c, T def) const {
        std::string v;
        return c.get(name_, v) ? static_cast<T>(std::strtod(v.c_str(), 0)) : def;
    }

private:
    std::string name_;
    T           def_, min_, max_;
};
typedef Parameter<s32> ParameterInt;
typedef Parameter<f64> ParameterFloat;
}  // namespace Core
