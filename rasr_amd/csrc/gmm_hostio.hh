// gmm_hostio.hh -- host-buffer side of the boundary (gmm_score_host): a small copy-thread pool and the
// pinned-memory probe.  The score table of a large batch (n_mixtures x n_frames f32, plus the best
// densities) is what crosses PCIe; gmm_api.cc streams it back in frame chunks overlapped with the
// scoring of the next chunk, straight into the caller's buffer when that buffer is pinned, otherwise
// through a double-buffered pinned staging ring whose host-side copies run on this pool.
#pragma once

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rasr_gmm {

class HostCopyPool {
public:
    explicit HostCopyPool(unsigned threads);
    ~HostCopyPool();
    HostCopyPool(const HostCopyPool&)            = delete;
    HostCopyPool& operator=(const HostCopyPool&) = delete;

    // fn(begin, end) over disjoint parts of [0, n), on the workers and the calling thread; returns
    // when every part is done
    void     parallelFor(size_t n, const std::function<void(size_t, size_t)>& fn);
    unsigned threads() const { return static_cast<unsigned>(workers_.size()) + 1u; }

private:
    void run(unsigned part);

    std::vector<std::thread>                   workers_;
    std::mutex                                 m_;
    std::condition_variable                    wake_, done_;
    const std::function<void(size_t, size_t)>* job_     = nullptr;
    size_t                                     n_       = 0;
    uint64_t                                   gen_     = 0;
    unsigned                                   pending_ = 0;
    bool                                       stop_    = false;
};

// copy threads of gmm_score_host (RASR_GMM_HOST_THREADS, default 8, at least 1)
unsigned hostCopyThreads();

// true when p lies in page-locked host memory known to this HIP runtime (hipHostMalloc /
// hipHostRegister / gmm_host_alloc), i.e. the DMA engines can write it directly
bool isPinnedHost(const void* p);

// true when p is page-locked host memory that kernels can address at p itself (hipHostMalloc / gmm_host_alloc
// on ROCm: the same virtual address on host and device), so a kernel reads and writes it over PCIe
bool isDeviceMappedHost(const void* p);

}  // namespace rasr_gmm
