// gmm_shard.hh -- the density-sharded layout (BASELINE config 4): which densities each GPU of a group holds.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace rasr_gmm {

// One GPU's part: the mixture entries [entryBegin, entryEnd) = [E r / P, E (r + 1) / P) of the CSR order, the
// mixtures [mixBegin, mixEnd) with entries in that range (an empty mixture goes to the first part whose range
// reaches past its position, else to the last), and the in-mixture index of the part's first entry of mixture
// mixBegin (> 0 when that mixture began on the previous part).  Same plan as rasr_amd/parallel.py
// density_shards, which the tests compare it with.
struct DensityShard {
    uint32_t entryBegin = 0, entryEnd = 0, mixBegin = 0, mixEnd = 0, firstOffset = 0;
};

// empty string on success
std::string planDensityShards(const uint32_t* mixtureOffsets, uint32_t nMixtures, uint32_t world,
                              std::vector<DensityShard>& out);
// mixtures held by more than one part, ascending (the ones the per-frame reduce combines)
std::vector<uint32_t> splitMixtures(const std::vector<DensityShard>& shards);

}  // namespace rasr_gmm
