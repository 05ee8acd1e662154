// refsort_test.cc -- pins rasr_amd/csrc/gmm_refsort.hh (the GPU replay of the reference's std::sort over
// (distance, cluster) pairs, DensityClustering.tcc:151-176) against this image's std::sort: for
// tie-heavy random inputs the full resulting permutation must be identical.  Exit status 0 = pass.
#include <algorithm>
#include <cstdio>
#include <random>
#include <utility>
#include <vector>

#include "../../rasr_amd/csrc/gmm_refsort.hh"

template <class K>
static int check(std::mt19937& rng, int n, int range, bool nanFree) {
    std::vector<std::pair<K, unsigned>> ref(n);
    std::vector<K>                      key(n);
    std::vector<unsigned char>          idx(n);
    std::uniform_int_distribution<int>  d(0, range);
    for (int i = 0; i < n; ++i) {
        key[i] = static_cast<K>(d(rng));
        if (!nanFree && i % 7 == 3)
            key[i] = static_cast<K>(d(rng)) * static_cast<K>(0.5);
        ref[i] = std::make_pair(key[i], static_cast<unsigned>(i));
        idx[i] = static_cast<unsigned char>(i);
    }
    std::sort(ref.begin(), ref.end(),
              [](const std::pair<K, unsigned>& x, const std::pair<K, unsigned>& y) { return x.first < y.first; });
    rasr_gmm::RefSortRange<K, unsigned char> s{key.data(), idx.data()};
    s.sort(n);
    for (int i = 0; i < n; ++i)
        if (ref[i].second != idx[i] || !(ref[i].first == key[i])) {
            std::printf("mismatch n=%d range=%d at %d: std %u, replay %u\n", n, range, i, ref[i].second, idx[i]);
            return 1;
        }
    return 0;
}

int main() {
    std::mt19937 rng(12345);
    int          fails = 0, cases = 0;
    for (int n : {1, 2, 3, 15, 16, 17, 31, 32, 33, 64, 100, 128, 200, 255, 256})
        for (int range : {0, 1, 2, 3, 5, 10, 40, 1000, 1 << 30})
            for (int rep = 0; rep < 40; ++rep) {
                fails += check<int>(rng, n, range, true);
                fails += check<float>(rng, n, range, false);
                cases += 2;
            }
    // adversarial: sorted, reversed, organ-pipe inputs (deep recursion, heapsort fallback)
    for (int n : {64, 200, 256}) {
        std::vector<int> pattern(n);
        for (int kind = 0; kind < 4; ++kind) {
            std::vector<std::pair<int, unsigned>> ref(n);
            std::vector<int>                      key(n);
            std::vector<unsigned char>            idx(n);
            for (int i = 0; i < n; ++i) {
                key[i] = kind == 0 ? i : kind == 1 ? n - i : kind == 2 ? std::min(i, n - i) : (i * 37) % 11;
                ref[i] = std::make_pair(key[i], static_cast<unsigned>(i));
                idx[i] = static_cast<unsigned char>(i);
            }
            std::sort(ref.begin(), ref.end(), [](const std::pair<int, unsigned>& x, const std::pair<int, unsigned>& y) {
                return x.first < y.first;
            });
            rasr_gmm::RefSortRange<int, unsigned char> s{key.data(), idx.data()};
            s.sort(n);
            for (int i = 0; i < n; ++i)
                if (ref[i].second != idx[i]) {
                    std::printf("mismatch pattern %d n=%d at %d\n", kind, n, i);
                    ++fails;
                    break;
                }
            ++cases;
        }
    }
    // the depth-limit fallback (std::partial_sort(first, last, last): heap select + sort_heap)
    for (int n : {2, 3, 17, 100, 256})
        for (int range : {0, 2, 7, 1000})
            for (int rep = 0; rep < 40; ++rep) {
                std::vector<std::pair<int, unsigned>> ref(n);
                std::vector<int>                      key(n);
                std::vector<unsigned char>            idx(n);
                std::uniform_int_distribution<int>    d(0, range);
                for (int i = 0; i < n; ++i) {
                    key[i] = d(rng);
                    ref[i] = std::make_pair(key[i], static_cast<unsigned>(i));
                    idx[i] = static_cast<unsigned char>(i);
                }
                std::partial_sort(ref.begin(), ref.end(), ref.end(),
                                  [](const std::pair<int, unsigned>& x, const std::pair<int, unsigned>& y) {
                                      return x.first < y.first;
                                  });
                rasr_gmm::RefSortRange<int, unsigned char> s{key.data(), idx.data()};
                s.heapSort(0, n);
                for (int i = 0; i < n; ++i)
                    if (ref[i].second != idx[i]) {
                        std::printf("heap mismatch n=%d at %d\n", n, i);
                        ++fails;
                        break;
                    }
                ++cases;
            }
    // selectFirst(n, k): the set std::sort leaves in [0, k)
    for (int n : {2, 3, 16, 17, 40, 100, 255, 256})
        for (int range : {0, 1, 3, 10, 100, 1 << 30})
            for (int rep = 0; rep < 30; ++rep) {
                std::vector<std::pair<int, unsigned>> ref(n);
                std::vector<int>                      key0(n);
                std::uniform_int_distribution<int>    d(0, range);
                for (int i = 0; i < n; ++i) {
                    key0[i] = d(rng);
                    ref[i]  = std::make_pair(key0[i], static_cast<unsigned>(i));
                }
                std::sort(ref.begin(), ref.end(), [](const std::pair<int, unsigned>& x, const std::pair<int, unsigned>& y) {
                    return x.first < y.first;
                });
                for (int k : {1, 2, 5, 16, 17, 32, n / 2, n - 1}) {
                    if (k <= 0 || k >= n)
                        continue;
                    std::vector<int>           key(key0);
                    std::vector<unsigned char> idx(n);
                    for (int i = 0; i < n; ++i)
                        idx[i] = static_cast<unsigned char>(i);
                    rasr_gmm::RefSortRange<int, unsigned char> s{key.data(), idx.data()};
                    s.selectFirst(n, k);
                    std::vector<unsigned> a, b;
                    for (int i = 0; i < k; ++i) {
                        a.push_back(ref[i].second);
                        b.push_back(idx[i]);
                    }
                    std::sort(a.begin(), a.end());
                    std::sort(b.begin(), b.end());
                    if (a != b) {
                        std::printf("selectFirst mismatch n=%d k=%d range=%d\n", n, k, range);
                        ++fails;
                    }
                    ++cases;
                }
            }
    std::printf("refsort: %d cases, %d failures\n", cases, fails);
    return fails ? 1 : 0;
}
