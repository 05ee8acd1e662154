// gmm_presel.cc -- density clustering for the preselection scorers (see gmm_presel.hh).
#include "gmm_presel.hh"

#include <algorithm>
#include <set>

#include "gmm_kernels.hh"

namespace rasr_gmm {

// srandom_r (TYPE_3): r[0] = seed, r[i] = 16807 r[i-1] mod (2^31 - 1) for i < 31, r[31..33] = r[0..2],
// then r[i] = r[i-31] + r[i-3] (mod 2^32); the first 310 values are discarded, rand() = r[i] >> 1.
GlibcRand::GlibcRand(uint32_t seed) {
    int32_t r[344];
    r[0] = static_cast<int32_t>(seed == 0 ? 1 : seed);
    for (int i = 1; i < 31; ++i) {
        // Schrage: 16807 * r mod (2^31 - 1) without overflow (glibc random_r.c)
        const int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
        int32_t       w  = 16807 * lo - 2836 * hi;
        if (w < 0)
            w += 2147483647;
        r[i] = w;
    }
    for (int i = 31; i < 34; ++i)
        r[i] = r[i - 31];
    for (int i = 34; i < 344; ++i)
        r[i] = static_cast<int32_t>(static_cast<uint32_t>(r[i - 31]) + static_cast<uint32_t>(r[i - 3]));
    for (int i = 0; i < 34; ++i)
        r_[i] = r[310 + i];
    i_ = 0;  // r_[(i_ + k) % 34] = r[310 + i_ + k]
}

int32_t GlibcRand::next() {
    // r[n] = r[n-31] + r[n-3] with the last 34 values in a ring
    const int32_t v = static_cast<int32_t>(static_cast<uint32_t>(r_[(i_ + 3) % 34]) + static_cast<uint32_t>(r_[(i_ + 31) % 34]));
    r_[i_ % 34]     = v;
    i_              = (i_ + 1) % 34;
    return static_cast<int32_t>(static_cast<uint32_t>(v) >> 1);
}

std::vector<uint32_t> clusteringSeeds(uint32_t nEntries, uint32_t nClusters) {
    std::vector<uint32_t> seeds;
    std::set<uint32_t>    used;
    GlibcRand             rng(1);
    for (uint32_t c = 0; c < nClusters; ++c) {
        uint32_t d = 0;
        do {
            d = static_cast<uint32_t>(rng.next()) % nEntries;
        } while (used.count(d));
        used.insert(d);
        seeds.push_back(d);
    }
    return seeds;
}

namespace {

struct DeviceBuffer {
    void* p = nullptr;
    ~DeviceBuffer() {
        if (p)
            (void)hipFree(p);
    }
};

template <class F>
void updateMeans(const F* entries, uint32_t nEntries, uint32_t Dp, const std::vector<uint8_t>& clusterOf,
                 uint32_t nClusters, std::vector<F>& means) {
    // updateClusterMeans (DensityClustering.tcc:101-121): per cluster, f64 sums over its densities in
    // density order, divided by the count and converted to the element type; empty clusters keep theirs
    std::vector<double>   sums(static_cast<size_t>(nClusters) * Dp, 0.0);
    std::vector<uint32_t> count(nClusters, 0);
    for (uint32_t e = 0; e < nEntries; ++e) {
        const uint32_t c = clusterOf[e];
        ++count[c];
        double*  s = sums.data() + static_cast<size_t>(c) * Dp;
        const F* m = entries + static_cast<size_t>(e) * Dp;
        for (uint32_t k = 0; k < Dp; ++k)
            s[k] += static_cast<double>(m[k]);
    }
    for (uint32_t c = 0; c < nClusters; ++c) {
        if (count[c] == 0)
            continue;
        for (uint32_t k = 0; k < Dp; ++k)
            means[static_cast<size_t>(c) * Dp + k] =
                    static_cast<F>(sums[static_cast<size_t>(c) * Dp + k] / static_cast<double>(count[c]));
    }
}

}  // namespace

std::string buildDensityClustering(bool quantized, const void* entryMeans, uint32_t nEntries, uint32_t Dp,
                                   uint32_t nClusters, uint32_t nSelected, uint32_t iterations,
                                   DensityClustering& out) {
    if (nEntries == 0)
        return "density preselection needs at least one density";
    if (nClusters == 0 || nClusters > 256)
        return "clusters must be in [1, 256]";  // paramNumClusters range, DensityClustering.cc:20-21
    if (Dp > 128)
        return "density preselection supports padded dimension <= 128";
    out                 = DensityClustering();
    out.quantized       = quantized;
    out.paddedDimension = Dp;
    out.nClusters       = std::min(nClusters, nEntries);  // "reducing number of clusters", cc:55-59
    out.nSelected       = nSelected;
    if (nSelected == 0 || nSelected > out.nClusters)
        return "select-clusters must be in [1, clusters]";  // verify(nSelected_ <= nClusters_), cc:61
    const size_t elem = quantized ? 1 : 4;
    const size_t nC   = out.nClusters;
    // initializeClusters
    const std::vector<uint32_t> seeds = clusteringSeeds(nEntries, out.nClusters);
    if (quantized) {
        const uint8_t* m = static_cast<const uint8_t*>(entryMeans);
        out.meansQ.resize(nC * Dp);
        for (size_t c = 0; c < nC; ++c)
            std::copy(m + static_cast<size_t>(seeds[c]) * Dp, m + static_cast<size_t>(seeds[c] + 1) * Dp,
                      out.meansQ.begin() + c * Dp);
    }
    else {
        const float* m = static_cast<const float*>(entryMeans);
        out.meansF.resize(nC * Dp);
        for (size_t c = 0; c < nC; ++c)
            std::copy(m + static_cast<size_t>(seeds[c]) * Dp, m + static_cast<size_t>(seeds[c] + 1) * Dp,
                      out.meansF.begin() + c * Dp);
    }
    out.clusterOfEntry.assign(nEntries, 0);  // init(): clusterIndexForDensity_ all 0
    if (iterations == 0)
        return "";
    DeviceBuffer dMeans, dCluster, dAssign;
    const size_t meanBytes = static_cast<size_t>(nEntries) * Dp * elem;
    if (hipMalloc(&dMeans.p, meanBytes) != hipSuccess || hipMalloc(&dCluster.p, nC * Dp * elem) != hipSuccess ||
        hipMalloc(&dAssign.p, nEntries) != hipSuccess)
        return "out of device memory for the density clustering";
    if (hipMemcpy(dMeans.p, entryMeans, meanBytes, hipMemcpyHostToDevice) != hipSuccess)
        return "device copy failed (density clustering)";
    for (uint32_t it = 0; it < iterations; ++it) {
        const void* cm = quantized ? static_cast<const void*>(out.meansQ.data()) : static_cast<const void*>(out.meansF.data());
        if (hipMemcpy(dCluster.p, cm, nC * Dp * elem, hipMemcpyHostToDevice) != hipSuccess ||
            launchAssignDensities(quantized, dMeans.p, nEntries, Dp, dCluster.p, out.nClusters,
                                  static_cast<uint8_t*>(dAssign.p), nullptr) != hipSuccess ||
            hipMemcpy(out.clusterOfEntry.data(), dAssign.p, nEntries, hipMemcpyDeviceToHost) != hipSuccess)
            return "density clustering: device step failed";
        if (quantized)
            updateMeans(static_cast<const uint8_t*>(entryMeans), nEntries, Dp, out.clusterOfEntry, out.nClusters,
                        out.meansQ);
        else
            updateMeans(static_cast<const float*>(entryMeans), nEntries, Dp, out.clusterOfEntry, out.nClusters,
                        out.meansF);
    }
    return "";
}

}  // namespace rasr_gmm
