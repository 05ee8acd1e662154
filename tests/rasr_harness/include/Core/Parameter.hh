// TEST DOUBLE: typed parameters read from a Configuration (Core::ParameterInt / ParameterFloat)
#pragma once
#include <cstdlib>
#include <limits>
#include <string>
#include <vector>
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
// Core::ParameterString / ParameterBool: the resource text; "true"/"yes"/"1" for a bool
class ParameterString {
public:
    ParameterString(const char* name, const char* description, const std::string def = "")
            : name_(name), def_(def) { (void)description; }
    std::string operator()(const Configuration& c) const {
        std::string v;
        return c.get(name_, v) ? v : def_;
    }

private:
    std::string name_, def_;
};
class ParameterBool {
public:
    ParameterBool(const char* name, const char* description, bool def = false) : name_(name), def_(def) {
        (void)description;
    }
    bool operator()(const Configuration& c) const {
        std::string v;
        if (!c.get(name_, v))
            return def_;
        return v == "true" || v == "yes" || v == "1";
    }

private:
    std::string name_;
    bool        def_;
};
// Core::ParameterIntVector (Core/Parameter.hh): values split at `delimiter`, each in [min, max]
class ParameterIntVector {
public:
    ParameterIntVector(const char* name, const char* description, const std::string delimiter = " ",
                       s32 min = std::numeric_limits<s32>::lowest(), s32 max = std::numeric_limits<s32>::max())
            : name_(name), delimiter_(delimiter.empty() ? " " : delimiter), min_(min), max_(max) { (void)description; }
    std::vector<s32> operator()(const Configuration& c) const {
        std::vector<s32> out;
        std::string      v;
        if (!c.get(name_, v))
            return out;
        size_t b = 0;
        while (b <= v.size()) {
            size_t e = v.find(delimiter_, b);
            if (e == std::string::npos)
                e = v.size();
            if (e > b) {
                const s32 x = static_cast<s32>(std::strtol(v.substr(b, e - b).c_str(), 0, 10));
                require(x >= min_ && x <= max_);
                out.push_back(x);
            }
            b = e + delimiter_.size();
        }
        return out;
    }

private:
    std::string name_, delimiter_;
    s32         min_, max_;
};
}  // namespace Core
