// TEST DOUBLE: Core::Application -- only us() and the application's configuration (the root the "cache-archive"
// names resolve under, Core/Application.cc:397-400).  The harness sets resources on a copy of it (copies share them).
#pragma once
#include "Component.hh"
namespace Core {
class Application : public Component {
public:
    static Application* us() {
        static Application app;
        return &app;
    }

private:
    Application() : Component(Configuration()) {}
};
}  // namespace Core
