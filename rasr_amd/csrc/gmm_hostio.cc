// gmm_hostio.cc -- see gmm_hostio.hh.
#include "gmm_hostio.hh"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

namespace rasr_gmm {

HostCopyPool::HostCopyPool(unsigned threads) {
    for (unsigned i = 1; i < std::max(threads, 1u); ++i)
        workers_.emplace_back([this, i] {
            uint64_t seen = 0;
            for (;;) {
                {
                    std::unique_lock<std::mutex> lk(m_);
                    wake_.wait(lk, [&] { return stop_ || gen_ != seen; });
                    if (stop_)
                        return;
                    seen = gen_;
                }
                run(i);
                std::lock_guard<std::mutex> lk(m_);
                if (--pending_ == 0)
                    done_.notify_one();
            }
        });
}

HostCopyPool::~HostCopyPool() {
    {
        std::lock_guard<std::mutex> lk(m_);
        stop_ = true;
    }
    wake_.notify_all();
    for (auto& t : workers_)
        t.join();
}

void HostCopyPool::run(unsigned part) {
    const size_t parts = workers_.size() + 1, b = n_ * part / parts, e = n_ * (part + 1) / parts;
    if (b < e)
        (*job_)(b, e);
}

void HostCopyPool::parallelFor(size_t n, const std::function<void(size_t, size_t)>& fn) {
    if (workers_.empty() || n < 2) {
        if (n)
            fn(0, n);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(m_);
        job_     = &fn;
        n_       = n;
        pending_ = static_cast<unsigned>(workers_.size());
        ++gen_;
    }
    wake_.notify_all();
    run(0);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
}

unsigned hostCopyThreads() {
    const char* e = std::getenv("RASR_GMM_HOST_THREADS");
    const long  v = e ? std::strtol(e, nullptr, 10) : 8;
    return static_cast<unsigned>(std::clamp<long>(v, 1, 64));
}

bool isPinnedHost(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory is reported as an error by some runtimes
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

bool isDeviceMappedHost(const void* p) {
    hipPointerAttribute_t a{};
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost && a.devicePointer == p;
}

}  // namespace rasr_gmm
