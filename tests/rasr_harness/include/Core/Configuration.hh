// TEST DOUBLE: a selection path plus resource lines "<path>.<parameter> = value"; a parameter resolves to the
// longest resource whose path is a prefix (or "*") of the component's selection (Core::Configuration)
#pragma once
#include <map>
#include <memory>
#include <string>
namespace Core {
class Configuration {
public:
    Configuration() : resources_(std::make_shared<std::map<std::string, std::string>>()) {}
    Configuration(const Configuration& parent, const std::string& selection)
            : resources_(parent.resources_), path_(parent.path_.empty() ? selection : parent.path_ + "." + selection) {}
    void set(const std::string& key, const std::string& value) { (*resources_)[key] = value; }
    bool get(const std::string& parameter, std::string& value) const {
        // exact path first, then every shorter prefix, then "*"
        std::string p = path_;
        for (;;) {
            auto it = resources_->find((p.empty() ? std::string("*") : p) + "." + parameter);
            if (it != resources_->end()) {
                value = it->second;
                return true;
            }
            if (p.empty())
                return false;
            const size_t dot = p.rfind('.');
            p = dot == std::string::npos ? std::string() : p.substr(0, dot);
        }
    }
    const std::string& getSelection() const { return path_; }
    std::string        getName() const {
        const size_t dot = path_.rfind('.');
        return dot == std::string::npos ? path_ : path_.substr(dot + 1);
    }

private:
    std::shared_ptr<std::map<std::string, std::string>> resources_;
    std::string                                         path_;
};
}  // namespace Core
