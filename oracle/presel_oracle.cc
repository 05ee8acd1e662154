// presel_oracle.cc -- TEST INFRASTRUCTURE ONLY (parity checker for the preselection scorers).
//
// CPU restatement of Mm::DensityClustering (src/Mm/DensityClustering.{hh,cc,tcc}) as used by
// "preselection-batch-float" / "preselection-batch-int" (src/Mm/BatchFeatureScorer.cc:238-289,
// 478-533): k-means over the prepared density means, initialised from glibc rand() after srand(1),
// and the per-frame selection of the select-clusters nearest clusters by std::sort.  Written in C++
// on purpose: the selection's tie order is whatever the C++ library's std::sort (introsort) makes of
// equal distances, and this file calls the same std::sort on the same (distance, cluster) pairs with
// the same comparator; the clustering calls the same srand/rand.  Built with the reference's flags
// (oracle/Makefile: -O2 -ffast-math -msse3 -funsigned-char).
//
// Parity status: UNPINNED (gmm_oracle.h); the tie order is pinned to this image's libstdc++ (GCC 11)
// and glibc, the reference build's own runtime on Linux.
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <cstring>
#include <set>
#include <utility>
#include <vector>

namespace {

// Mm::unrolledVectorDistance (src/Mm/Utilities.hh:244-284): the switch only picks the entry point
// of the 8-fold unrolled loop; the components are summed in order 0 .. dimension-1.
template <class T, class D>
D vectorDistance(const T* a, const T* b, uint32_t dimension) {
    D score = 0;
    for (uint32_t cmp = 0; cmp < dimension; ++cmp) {
        D df = (a[cmp] - b[cmp]);
        score += df * df;
    }
    return score;
}

template <class F, class D>
void buildClustering(const F* densities, uint32_t nDensities, uint32_t dimension, uint32_t nClusters,
                     uint32_t iterations, uint8_t* clusterIndexForDensity, F* clusterMeans) {
    // init (DensityClustering.cc:48-61): nClusters_ reduced to nDensities_ by the caller
    std::memset(clusterIndexForDensity, 0, nDensities);
    // initializeClusters (DensityClustering.tcc:60-74)
    std::set<uint32_t> used;
    srand(1);
    for (uint32_t cluster = 0; cluster < nClusters; ++cluster) {
        uint32_t d = 0;
        do {
            d = rand() % nDensities;
        } while (used.count(d));
        used.insert(d);
        std::copy(densities + static_cast<size_t>(d) * dimension, densities + static_cast<size_t>(d + 1) * dimension,
                  clusterMeans + static_cast<size_t>(cluster) * dimension);
    }
    for (uint32_t it = 0; it < iterations; ++it) {
        // assignDensities (DensityClustering.tcc:80-99)
        std::vector<std::vector<uint32_t>> assigned(nClusters);
        for (uint32_t density = 0; density < nDensities; ++density) {
            D        bestDistance = 0;
            uint32_t bestCluster  = 0;
            bool     first        = true;  // Core::Type<D>::max start; strict < keeps the first minimum
            for (uint32_t cluster = 0; cluster < nClusters; ++cluster) {
                D dist = vectorDistance<F, D>(clusterMeans + static_cast<size_t>(cluster) * dimension,
                                              densities + static_cast<size_t>(density) * dimension, dimension);
                if (first || dist < bestDistance) {
                    bestDistance = dist;
                    bestCluster  = cluster;
                    first        = false;
                }
            }
            clusterIndexForDensity[density] = static_cast<uint8_t>(bestCluster);
            assigned[bestCluster].push_back(density);
        }
        // updateClusterMeans (DensityClustering.tcc:101-121): f64 sums in density order / count
        for (uint32_t cluster = 0; cluster < nClusters; ++cluster) {
            const std::vector<uint32_t>& a = assigned[cluster];
            if (a.empty())
                continue;
            std::vector<double> sums(dimension, 0);
            for (uint32_t i : a)
                for (uint32_t k = 0; k < dimension; ++k)
                    sums[k] += densities[static_cast<size_t>(i) * dimension + k];
            for (uint32_t k = 0; k < dimension; ++k)
                clusterMeans[static_cast<size_t>(cluster) * dimension + k] = static_cast<F>(sums[k] / a.size());
        }
    }
}

// selectClusters (DensityClustering.tcc:151-176)
template <class F, class D>
void selectClusters(const F* feature, const F* clusterMeans, uint32_t nClusters, uint32_t dimension, uint32_t nSelected,
                    uint8_t* selection) {
    typedef std::pair<D, uint32_t> Item;
    std::vector<Item>              byDistance(nClusters);
    for (uint32_t cluster = 0; cluster < nClusters; ++cluster)
        byDistance[cluster] = std::make_pair(
                vectorDistance<F, D>(feature, clusterMeans + static_cast<size_t>(cluster) * dimension, dimension), cluster);
    std::sort(byDistance.begin(), byDistance.end(), [](const Item& x, const Item& y) { return x.first < y.first; });
    std::fill(selection, selection + nClusters, 0);
    for (uint32_t i = 0; i < nSelected; ++i)
        selection[byDistance[i].second] = 1;
}

}  // namespace

extern "C" {

/* libc rand() after srand(seed): the generator the reference's initializeClusters draws from */
int orc_libc_rand_sequence(uint32_t seed, uint32_t n, int32_t* out) {
    srand(seed);
    for (uint32_t i = 0; i < n; ++i)
        out[i] = rand();
    return 0;
}

/* means [n_densities][dimension] (dimension = the scorer's padded dimension) */
int orc_cluster_build_f32(const float* means, uint32_t n_densities, uint32_t dimension, uint32_t n_clusters,
                          uint32_t iterations, uint8_t* cluster_of_density, float* cluster_means) {
    if (n_clusters == 0 || n_clusters > 256 || n_clusters > n_densities)
        return -1;
    buildClustering<float, float>(means, n_densities, dimension, n_clusters, iterations, cluster_of_density,
                                  cluster_means);
    return 0;
}

int orc_cluster_build_u8(const uint8_t* means, uint32_t n_densities, uint32_t dimension, uint32_t n_clusters,
                         uint32_t iterations, uint8_t* cluster_of_density, uint8_t* cluster_means) {
    if (n_clusters == 0 || n_clusters > 256 || n_clusters > n_densities)
        return -1;
    buildClustering<uint8_t, int32_t>(means, n_densities, dimension, n_clusters, iterations, cluster_of_density,
                                      cluster_means);
    return 0;
}

/* features [n_frames][dimension] (setFeature output); selection [n_frames][n_clusters] 0/1 */
int orc_select_clusters_f32(const float* features, uint32_t n_frames, const float* cluster_means, uint32_t n_clusters,
                            uint32_t dimension, uint32_t n_selected, uint8_t* selection) {
    for (uint32_t t = 0; t < n_frames; ++t)
        selectClusters<float, float>(features + static_cast<size_t>(t) * dimension, cluster_means, n_clusters,
                                     dimension, n_selected, selection + static_cast<size_t>(t) * n_clusters);
    return 0;
}

int orc_select_clusters_u8(const uint8_t* features, uint32_t n_frames, const uint8_t* cluster_means,
                           uint32_t n_clusters, uint32_t dimension, uint32_t n_selected, uint8_t* selection) {
    for (uint32_t t = 0; t < n_frames; ++t)
        selectClusters<uint8_t, int32_t>(features + static_cast<size_t>(t) * dimension, cluster_means, n_clusters,
                                         dimension, n_selected, selection + static_cast<size_t>(t) * n_clusters);
    return 0;
}

}  // extern "C"
