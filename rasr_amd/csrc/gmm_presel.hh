// gmm_presel.hh -- host side of the density preselection (preselection-batch-float / -int):
// Mm::DensityClustering::build (src/Mm/DensityClustering.tcc:124-149) with the assignment step on the
// GPU (gmm_kernels_presel.hip) and the mean update on the host in the reference's f64 order.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace rasr_gmm {

// glibc random_r TYPE_3 (additive feedback x^31 + x^3 + 1), i.e. rand() after srand(seed): the
// generator DensityClustering::initializeClusters draws from (srand(1), DensityClustering.tcc:64)
class GlibcRand {
public:
    explicit GlibcRand(uint32_t seed);
    int32_t next();

private:
    int32_t  r_[34];
    uint32_t i_ = 0;
};

// initializeClusters (DensityClustering.tcc:60-74): the entry each cluster mean starts from
std::vector<uint32_t> clusteringSeeds(uint32_t nEntries, uint32_t nClusters);

struct DensityClustering {
    bool                 quantized = false;  // u8 means / s32 distances (preselection-batch-int)
    uint32_t             nClusters = 0, nSelected = 0, paddedDimension = 0;
    std::vector<uint8_t> clusterOfEntry;     // clusterIndexForDensity_ [entries]
    std::vector<float>   meansF;             // [nClusters][paddedDimension] (float)
    std::vector<uint8_t> meansQ;             // [nClusters][paddedDimension] (int)
};

// Build the clustering of the entry means (float: [entries][Dp] f32, int: [entries][Dp] u8) on
// `device`.  nClusters is reduced to the entry count (DensityClustering.cc:55-59); nSelected must not
// exceed the result.  Returns "" or an error message.
std::string buildDensityClustering(bool quantized, const void* entryMeans, uint32_t nEntries, uint32_t Dp,
                                   uint32_t nClusters, uint32_t nSelected, uint32_t iterations,
                                   DensityClustering& out);

// ---- RASR's cache archive (Core::MappedArchive, src/Core/MappedArchive.{hh,cc}) ----
// File: u32 version 0x17231, then items: u32 name length, u64 data size, the name, the data (the last item of a
// name wins).  Item data: POD values raw, vectors as a u64 count and the elements, strings as a vector<char> with
// the terminating 0 (MappedArchiveWriter, MappedArchive.hh:401-466).
// Read item `name` of the archive at `path` into `data`; false if the file, its version or the item is missing.
bool readArchiveItem(const std::string& path, const std::string& name, std::vector<char>& data);
// Write item `name` into the archive at `path` (the file is created, or rewritten with the other items kept, through
// a temporary file renamed over it, as MappedArchive::finalize does); false on an I/O error.
bool writeArchiveItem(const std::string& path, const std::string& name, const std::vector<char>& data);
// The "density-clustering" item of DensityClusteringBase::write / load (DensityClustering.cc:59-95,
// DensityClustering.tcc:26-55): magic "SPRINT-DC", version 2, the feature and distance type names ("f32"/"f32"
// float, "u8"/"s32" int), dimension (the padded dimension), clusters, densities, clusterIndexForDensity_ (u8), the
// cluster means.
std::vector<char> encodeClusteringItem(const DensityClustering& dc, uint32_t nEntries);
// Decode and check an item against the scorer's (type, padded dimension, cluster count after the reduction to the
// entry count, entry count); false on any mismatch, as DensityClusteringBase::load rejects one.
bool decodeClusteringItem(const std::vector<char>& data, bool quantized, uint32_t Dp, uint32_t nClusters,
                          uint32_t nEntries, uint32_t nSelected, DensityClustering& out);

}  // namespace rasr_gmm
