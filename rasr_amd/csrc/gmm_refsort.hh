// gmm_refsort.hh -- the cluster ranking of Mm::DensityClustering::selectClusters
// (src/Mm/DensityClustering.tcc:151-176): std::sort over (distance, cluster) pairs compared by the
// distance only.  std::sort is not stable, so WHICH of several clusters at the same distance land in
// the first select-clusters positions is defined by the sort algorithm itself.  This header replays
// the reference build's std::sort (libstdc++ introsort: median-of-three quicksort down to 16-element
// ranges, heapsort below depth 2*log2(n), final insertion sort) step for step on two parallel arrays,
// so the selection is the reference's on ties too.  The scorer runs it on the GPU only for frames
// whose ranking has a tie across the selection boundary (gmm_kernels_presel.hip); tests/cpp pins it
// against std::sort on the host.
//
// The unguarded scans of the library are bounded here (they never hit the bound for a strict weak
// order; a NaN distance is undefined behaviour in the reference and merely "some order" here).
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define GMM_HD __host__ __device__
#else
#define GMM_HD
#endif

namespace rasr_gmm {

template <class K, class I>
struct RefSortRange {
    K* key;
    I* idx;

    GMM_HD bool lt(int i, int j) const { return key[i] < key[j]; }
    GMM_HD void swap(int i, int j) {
        const K k = key[i];
        key[i]    = key[j];
        key[j]    = k;
        const I x = idx[i];
        idx[i]    = idx[j];
        idx[j]    = x;
    }
    GMM_HD void move(int dst, int src) {
        key[dst] = key[src];
        idx[dst] = idx[src];
    }

    GMM_HD void moveMedianToFirst(int result, int a, int b, int c) {
        if (lt(a, b)) {
            if (lt(b, c))
                swap(result, b);
            else if (lt(a, c))
                swap(result, c);
            else
                swap(result, a);
        }
        else if (lt(a, c))
            swap(result, a);
        else if (lt(b, c))
            swap(result, c);
        else
            swap(result, b);
    }

    GMM_HD int unguardedPartition(int first, int last, int pivot) {
        const int hi = last;
        while (true) {
            while (first < hi - 1 && lt(first, pivot))
                ++first;
            --last;
            while (last > pivot && lt(pivot, last))
                --last;
            if (!(first < last))
                return first;
            swap(first, last);
            ++first;
        }
    }

    GMM_HD int unguardedPartitionPivot(int first, int last) {
        const int mid = first + (last - first) / 2;
        moveMedianToFirst(first, first + 1, mid, last - 1);
        return unguardedPartition(first + 1, last, first);
    }

    // heap primitives (bits/stl_heap.h): positions are relative to `first`
    GMM_HD void pushHeap(int first, int hole, int top, K vk, I vi) {
        int parent = (hole - 1) / 2;
        while (hole > top && key[first + parent] < vk) {
            move(first + hole, first + parent);
            hole   = parent;
            parent = (hole - 1) / 2;
        }
        key[first + hole] = vk;
        idx[first + hole] = vi;
    }
    GMM_HD void adjustHeap(int first, int hole, int len, K vk, I vi) {
        const int top    = hole;
        int       second = hole;
        while (second < (len - 1) / 2) {
            second = 2 * (second + 1);
            if (lt(first + second, first + second - 1))
                --second;
            move(first + hole, first + second);
            hole = second;
        }
        if ((len & 1) == 0 && second == (len - 2) / 2) {
            second = 2 * (second + 1);
            move(first + hole, first + second - 1);
            hole = second - 1;
        }
        pushHeap(first, hole, top, vk, vi);
    }
    GMM_HD void makeHeap(int first, int last) {
        const int len = last - first;
        if (len < 2)
            return;
        int parent = (len - 2) / 2;
        while (true) {
            adjustHeap(first, parent, len, key[first + parent], idx[first + parent]);
            if (parent == 0)
                return;
            --parent;
        }
    }
    GMM_HD void popHeap(int first, int last, int result) {
        const K vk = key[result];
        const I vi = idx[result];
        move(result, first);
        adjustHeap(first, 0, last - first, vk, vi);
    }
    // __partial_sort(first, last, last): __heap_select (make_heap; no element beyond `last`) + __sort_heap
    GMM_HD void heapSort(int first, int last) {
        makeHeap(first, last);
        while (last - first > 1) {
            --last;
            popHeap(first, last, last);
        }
    }

    GMM_HD void unguardedLinearInsert(int last, int lo) {
        const K vk   = key[last];
        const I vi   = idx[last];
        int     next = last - 1;
        while (next >= lo && vk < key[next]) {
            move(last, next);
            last = next;
            --next;
        }
        key[last] = vk;
        idx[last] = vi;
    }
    GMM_HD void insertionSort(int first, int last) {
        if (first == last)
            return;
        for (int i = first + 1; i != last; ++i) {
            if (lt(i, first)) {
                const K vk = key[i];
                const I vi = idx[i];
                for (int j = i; j > first; --j)
                    move(j, j - 1);
                key[first] = vk;
                idx[first] = vi;
            }
            else {
                unguardedLinearInsert(i, first);
            }
        }
    }

    // The set std::sort(key, key + n) leaves in positions [0, k), without the rest of the sort: after a
    // partition every element of [first, cut) is <= every element of [cut, last), and the final
    // insertion sort moves an element only past strictly greater ones, so no element ever leaves the
    // introsort range it ends up in.  Ranges entirely left or right of k are therefore decided, and only
    // the one range containing the boundary is followed (a single partition path, like quickselect):
    // down to <= 16 elements, whose final order is the stable (insertion) order of their positions,
    // or to the depth-limit heapsort, replayed in full.  Positions [0, k) then hold the selection.
    GMM_HD void selectFirst(int n, int k) {
        if (k <= 0 || k >= n)
            return;
        constexpr int kThreshold = 16;
        int           lg         = 0;
        while ((2 << lg) <= n)
            ++lg;
        int first = 0, last = n, depth = 2 * lg;
        while (last - first > kThreshold) {
            if (depth == 0) {
                heapSort(first, last);
                return;
            }
            --depth;
            const int cut = unguardedPartitionPivot(first, last);
            if (cut <= k)      // [first, cut) all selected; the boundary is in the recursion on [cut, last)
                first = cut;
            else               // the loop continues on [first, cut)
                last = cut;
            if (first == k)    // the cut fell on the boundary
                return;
        }
        insertionSort(first, last);
    }

    // std::sort(key, key + n) carrying idx along
    GMM_HD void sort(int n) {
        if (n <= 0)
            return;
        constexpr int kThreshold = 16;
        int           lg         = 0;
        while ((2 << lg) <= n)
            ++lg;
        // __introsort_loop: the recursion on [cut, last) is independent of the loop on [first, cut),
        // so a stack replays it; depths strictly decrease up the stack (<= 2 lg + 1 entries)
        struct Range {
            int first, last, depth;
        };
        Range stack[40];  // n < 2^19
        int   sp    = 0;
        stack[sp++] = Range{0, n, 2 * lg};
        while (sp > 0) {
            Range r     = stack[--sp];
            int   first = r.first, last = r.last, depth = r.depth;
            while (last - first > kThreshold) {
                if (depth == 0) {
                    heapSort(first, last);
                    break;
                }
                --depth;
                const int cut = unguardedPartitionPivot(first, last);
                stack[sp++]   = Range{cut, last, depth};
                last          = cut;
            }
        }
        // __final_insertion_sort
        if (n > kThreshold) {
            insertionSort(0, kThreshold);
            for (int i = kThreshold; i < n; ++i)
                unguardedLinearInsert(i, 0);
        }
        else {
            insertionSort(0, n);
        }
    }
};

}  // namespace rasr_gmm
