// gmm_presel.cc -- density clustering for the preselection scorers (see gmm_presel.hh).
#include "gmm_presel.hh"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <set>

#include <unistd.h>

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

// ---------------------------------------------------------------------------
// cache archive (Core::MappedArchive) and the density-clustering item
// ---------------------------------------------------------------------------
namespace {
constexpr uint32_t kArchiveVersion = 0x17231;  // MappedArchive.cc:52

struct ArchiveItem {
    std::string       name;
    std::vector<char> data;
};

// every item of a valid archive (false: no file, or not an archive of this version; a truncated tail ends the list,
// as MappedArchive::loadData stops there)
bool readArchive(const std::string& path, std::vector<ArchiveItem>& items) {
    std::ifstream in(path, std::ios::binary);
    if (!in)
        return false;
    std::vector<char> all((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    uint32_t          ver = 0;
    if (all.size() < sizeof(ver))
        return false;
    std::memcpy(&ver, all.data(), sizeof(ver));
    if (ver != kArchiveVersion)
        return false;
    size_t o = sizeof(ver);
    while (o + sizeof(uint32_t) + sizeof(uint64_t) <= all.size()) {
        uint32_t nl = 0;
        uint64_t ds = 0;
        std::memcpy(&nl, all.data() + o, sizeof(nl));
        std::memcpy(&ds, all.data() + o + sizeof(nl), sizeof(ds));
        o += sizeof(nl) + sizeof(ds);
        if (nl == 0 || nl > all.size() - o || ds > all.size() - o - nl)
            break;
        ArchiveItem it;
        it.name.assign(all.data() + o, nl);
        it.data.assign(all.data() + o + nl, all.data() + o + nl + ds);
        items.push_back(std::move(it));
        o += nl + ds;
    }
    return true;
}

struct ItemWriter {
    std::vector<char> b;
    template <class T>
    void pod(const T& v) {
        const char* p = reinterpret_cast<const char*>(&v);
        b.insert(b.end(), p, p + sizeof(T));
    }
    template <class T>
    void vec(const T* p, size_t n) {
        pod<uint64_t>(n);
        b.insert(b.end(), reinterpret_cast<const char*>(p), reinterpret_cast<const char*>(p) + n * sizeof(T));
    }
    void str(const std::string& s) {
        pod<uint64_t>(s.size() + 1);
        b.insert(b.end(), s.begin(), s.end());
        b.push_back(0);
    }
};

struct ItemReader {
    const std::vector<char>& b;
    size_t                   o  = 0;
    bool                     ok = true;
    template <class T>
    T pod() {
        T v{};
        if (!ok || o + sizeof(T) > b.size()) {
            ok = false;
            return v;
        }
        std::memcpy(&v, b.data() + o, sizeof(T));
        o += sizeof(T);
        return v;
    }
    template <class T>
    std::vector<T> vec() {
        const uint64_t n = pod<uint64_t>();
        std::vector<T> v;
        if (!ok || n > (b.size() - o) / sizeof(T)) {
            ok = false;
            return v;
        }
        v.resize(n);
        std::memcpy(v.data(), b.data() + o, n * sizeof(T));
        o += n * sizeof(T);
        return v;
    }
    std::string str() {  // MappedArchiveReader::operator>>(std::string&): up to the first 0
        const std::vector<char> v = vec<char>();
        return v.empty() ? std::string() : std::string(v.data(), strnlen(v.data(), v.size()));
    }
};
}  // namespace

bool readArchiveItem(const std::string& path, const std::string& name, std::vector<char>& data) {
    std::vector<ArchiveItem> items;
    if (!readArchive(path, items))
        return false;
    for (auto it = items.rbegin(); it != items.rend(); ++it)  // MappedArchive::getItem: the last one of a name
        if (it->name == name) {
            data = it->data;
            return true;
        }
    return false;
}

bool writeArchiveItem(const std::string& path, const std::string& name, const std::vector<char>& data) {
    std::vector<ArchiveItem> items;
    (void)readArchive(path, items);  // keep the archive's other items (a missing or foreign file starts empty)
    // MappedArchive.cc:40-48, 114: "<archive>.temp.<host>.<pid>" -- archives may sit on a shared filesystem
    char host[256] = {0};
    if (gethostname(host, sizeof(host) - 1) != 0)
        std::strcpy(host, "unknown");
    const std::string tmp = path + ".temp." + host + "." + std::to_string(static_cast<long>(getpid()));
    {
        std::ofstream out(tmp, std::ios::binary | std::ios::trunc);
        if (!out)
            return false;
        out.write(reinterpret_cast<const char*>(&kArchiveVersion), sizeof(kArchiveVersion));
        const auto put = [&](const std::string& n, const std::vector<char>& d) {
            const uint32_t nl = static_cast<uint32_t>(n.size());
            const uint64_t ds = d.size();
            out.write(reinterpret_cast<const char*>(&nl), sizeof(nl));
            out.write(reinterpret_cast<const char*>(&ds), sizeof(ds));
            out.write(n.data(), nl);
            out.write(d.data(), static_cast<std::streamsize>(ds));
        };
        for (const ArchiveItem& it : items)
            if (it.name != name)
                put(it.name, it.data);
        put(name, data);
        if (!out.good()) {
            out.close();
            std::remove(tmp.c_str());
            return false;
        }
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        return false;
    }
    return true;
}

std::vector<char> encodeClusteringItem(const DensityClustering& dc, uint32_t nEntries) {
    ItemWriter w;
    w.str("SPRINT-DC");  // DensityClusteringBase::FileMagic, FileFormatVersion (DensityClustering.cc:34-35)
    w.pod<uint32_t>(2);
    w.str(dc.quantized ? "u8" : "f32");  // Core::Type<FeatureType>::name, Core::Type<DistanceType>::name
    w.str(dc.quantized ? "s32" : "f32");
    w.pod<uint32_t>(dc.paddedDimension);
    w.pod<uint32_t>(dc.nClusters);
    w.pod<uint32_t>(nEntries);
    w.vec(dc.clusterOfEntry.data(), dc.clusterOfEntry.size());
    if (dc.quantized)
        w.vec(dc.meansQ.data(), dc.meansQ.size());
    else
        w.vec(dc.meansF.data(), dc.meansF.size());
    return w.b;
}

bool decodeClusteringItem(const std::vector<char>& data, bool quantized, uint32_t Dp, uint32_t nClusters,
                          uint32_t nEntries, uint32_t nSelected, DensityClustering& out) {
    ItemReader r{data};
    if (r.str() != "SPRINT-DC" || r.pod<uint32_t>() != 2u)
        return false;
    if (r.str() != (quantized ? "u8" : "f32") || r.str() != (quantized ? "s32" : "f32"))
        return false;
    if (r.pod<uint32_t>() != Dp || r.pod<uint32_t>() != nClusters || r.pod<uint32_t>() != nEntries || !r.ok)
        return false;
    DensityClustering dc;
    dc.quantized       = quantized;
    dc.nClusters       = nClusters;
    dc.nSelected       = nSelected;
    dc.paddedDimension = Dp;
    dc.clusterOfEntry  = r.vec<uint8_t>();
    if (quantized)
        dc.meansQ = r.vec<uint8_t>();
    else
        dc.meansF = r.vec<float>();
    const size_t nMeans = quantized ? dc.meansQ.size() : dc.meansF.size();
    // readMeans verifies the size (DensityClustering.tcc:36); every assignment must name a cluster
    if (!r.ok || dc.clusterOfEntry.size() != nEntries || nMeans != static_cast<size_t>(nClusters) * Dp)
        return false;
    for (uint8_t c : dc.clusterOfEntry)
        if (c >= nClusters)
            return false;
    out = std::move(dc);
    return true;
}

}  // namespace rasr_gmm
