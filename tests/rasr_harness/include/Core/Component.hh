// TEST DOUBLE: Core::Component (a configured object that logs and reports errors; criticalError aborts)
#pragma once
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <string>
#include "Configuration.hh"
namespace Core {
class Component {
public:
    explicit Component(const Configuration& c) : config(c) {}
    virtual ~Component() {}
    const Configuration& getConfiguration() const { return config; }
    std::string          name() const { return config.getName(); }
    Configuration        select(const std::string& s) const { return Configuration(config, s); }
    void log(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::fprintf(stderr, "[log %s] ", config.getSelection().c_str());
        std::vfprintf(stderr, fmt, ap);
        std::fputc('\n', stderr);
        va_end(ap);
    }
    void warning(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::fprintf(stderr, "[warning %s] ", config.getSelection().c_str());
        std::vfprintf(stderr, fmt, ap);
        std::fputc('\n', stderr);
        va_end(ap);
    }
    void error(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::fprintf(stderr, "[error %s] ", config.getSelection().c_str());
        std::vfprintf(stderr, fmt, ap);
        std::fputc('\n', stderr);
        va_end(ap);
        ++errors_;
    }
    void criticalError(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::fprintf(stderr, "[critical error %s] ", config.getSelection().c_str());
        std::vfprintf(stderr, fmt, ap);
        std::fputc('\n', stderr);
        va_end(ap);
        std::fflush(stderr);
        std::abort();
    }
    int nErrors() const { return errors_; }

protected:
    Configuration config;

private:
    mutable int errors_ = 0;
};
}  // namespace Core
