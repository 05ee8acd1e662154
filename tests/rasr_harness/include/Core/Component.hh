// TEST DOUBLE: Core::Component (a configured object that logs and reports errors; criticalError aborts).  As in
// RASR, log / warning / error return a message that takes further "<< value" parts and is written when it ends.
#pragma once
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include "Configuration.hh"
namespace Core {
class Component {
public:
    class Message {
    public:
        explicit Message(std::string text) { s_ << text; }
        ~Message() { std::fprintf(stderr, "%s\n", s_.str().c_str()); }
        template <class T>
        Message& operator<<(const T& x) {
            s_ << x;
            return *this;
        }

    private:
        std::ostringstream s_;
    };

    explicit Component(const Configuration& c) : config(c) {}
    virtual ~Component() {}
    const Configuration& getConfiguration() const { return config; }
    std::string          name() const { return config.getName(); }
    Configuration        select(const std::string& s) const { return Configuration(config, s); }
    Message log(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::string t = format("log", fmt, ap);
        va_end(ap);
        return Message(t);
    }
    Message warning(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::string t = format("warning", fmt, ap);
        va_end(ap);
        return Message(t);
    }
    Message error(const char* fmt, ...) const {
        va_list ap;
        va_start(ap, fmt);
        std::string t = format("error", fmt, ap);
        va_end(ap);
        ++errors_;
        return Message(t);
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
    std::string format(const char* kind, const char* fmt, va_list ap) const {
        char buf[1024];
        std::vsnprintf(buf, sizeof(buf), fmt, ap);
        return "[" + std::string(kind) + " " + config.getSelection() + "] " + buf;
    }
    mutable int errors_ = 0;
};
}  // namespace Core
