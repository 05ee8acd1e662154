// TEST DOUBLE: intrusive, non-atomic reference counting (Core::ReferenceCounted / Core::Ref)
#pragma once
#include "Assertions.hh"
namespace Core {
class ReferenceCounted {
public:
    ReferenceCounted() : refs_(0) {}
    ReferenceCounted(const ReferenceCounted&) : refs_(0) {}
    virtual ~ReferenceCounted() {}
    void acquireReference() const { ++refs_; }
    bool releaseReference() const { return --refs_ == 0; }
    int  refCount() const { return refs_; }

private:
    mutable int refs_;
};

template <class T>
class Ref {
public:
    Ref() : p_(0) {}
    explicit Ref(T* p) : p_(p) { if (p_) p_->acquireReference(); }
    Ref(const Ref& o) : p_(o.p_) { if (p_) p_->acquireReference(); }
    template <class S>
    Ref(const Ref<S>& o) : p_(o.get()) { if (p_) p_->acquireReference(); }
    ~Ref() { release(); }
    Ref& operator=(const Ref& o) {
        if (o.p_) o.p_->acquireReference();
        release();
        p_ = o.p_;
        return *this;
    }
    T* get() const { return p_; }
    T* operator->() const { require(p_); return p_; }
    T& operator*() const { require(p_); return *p_; }
    operator bool() const { return p_ != 0; }
    void reset() { release(); p_ = 0; }

private:
    void release() {
        if (p_ && p_->releaseReference())
            delete p_;
    }
    T* p_;
};

template <class T>
Ref<T> ref(T* p) { return Ref<T>(p); }
}  // namespace Core
