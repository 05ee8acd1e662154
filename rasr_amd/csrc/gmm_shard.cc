// gmm_shard.cc -- density shard plan (BASELINE config 4) and its host-only C-ABI entry point.
#include "gmm_shard.hh"

#include <algorithm>

#include "../../include/rasr_gmm.h"

namespace rasr_gmm {

void setLastError(const std::string& msg);  // gmm_api.cc

std::string planDensityShards(const uint32_t* off, uint32_t nMixtures, uint32_t world, std::vector<DensityShard>& out) {
    out.clear();
    if (world == 0)
        return "world must be > 0";
    const uint64_t E = off[nMixtures];
    std::vector<std::pair<uint64_t, uint64_t>> ranges(world);
    for (uint32_t r = 0; r < world; ++r)
        ranges[r] = {E * r / world, E * (r + 1) / world};
    std::vector<std::vector<uint32_t>> owners(world);
    for (uint32_t m = 0; m < nMixtures; ++m) {
        const uint64_t a = off[m], b = off[m + 1];
        if (b < a)
            return "mixture_offsets must be non-decreasing";
        if (a == b) {
            uint32_t r = world - 1;
            for (uint32_t q = 0; q < world; ++q)
                if (a < ranges[q].second) {
                    r = q;
                    break;
                }
            owners[r].push_back(m);
            continue;
        }
        for (uint32_t r = 0; r < world; ++r)
            if (a < ranges[r].second && b > ranges[r].first)
                owners[r].push_back(m);
    }
    for (uint32_t r = 0; r < world; ++r) {
        DensityShard s;
        s.entryBegin = static_cast<uint32_t>(ranges[r].first);
        s.entryEnd   = static_cast<uint32_t>(ranges[r].second);
        const std::vector<uint32_t>& o = owners[r];
        if (!o.empty()) {
            s.mixBegin = o.front();
            s.mixEnd   = o.back() + 1;
            if (s.mixEnd - s.mixBegin != o.size())
                return "density shard plan: a part's mixtures are not contiguous";
            s.firstOffset = s.entryBegin > off[s.mixBegin] ? s.entryBegin - off[s.mixBegin] : 0;
        }
        out.push_back(s);
    }
    return {};
}

std::vector<uint32_t> splitMixtures(const std::vector<DensityShard>& shards) {
    std::vector<uint32_t> held, split;
    for (const DensityShard& s : shards)
        for (uint32_t m = s.mixBegin; m < s.mixEnd; ++m)
            held.push_back(m);
    std::sort(held.begin(), held.end());
    for (size_t i = 1; i < held.size(); ++i)
        if (held[i] == held[i - 1] && (split.empty() || split.back() != held[i]))
            split.push_back(held[i]);
    return split;
}

}  // namespace rasr_gmm

extern "C" int gmm_density_shard_plan(const uint32_t* mixture_offsets, uint32_t n_mixtures, uint32_t world,
                                      uint32_t* shard_table, uint32_t* split, uint32_t* n_split) {
    using namespace rasr_gmm;
    if (!mixture_offsets || world == 0) {
        setLastError("null mixture_offsets or world 0");
        return GMM_ERR_INVALID_ARGUMENT;
    }
    std::vector<DensityShard> shards;
    const std::string         err = planDensityShards(mixture_offsets, n_mixtures, world, shards);
    if (!err.empty()) {
        setLastError(err);
        return GMM_ERR_INVALID_ARGUMENT;
    }
    if (shard_table)
        for (uint32_t r = 0; r < world; ++r) {
            const DensityShard& s = shards[r];
            uint32_t* row = shard_table + 5u * r;
            row[0] = s.entryBegin, row[1] = s.entryEnd, row[2] = s.mixBegin, row[3] = s.mixEnd, row[4] = s.firstOffset;
        }
    const std::vector<uint32_t> sp = splitMixtures(shards);
    if (split)
        std::copy(sp.begin(), sp.end(), split);
    if (n_split)
        *n_split = static_cast<uint32_t>(sp.size());
    return GMM_OK;
}
