// gosort.hpp -- Go 1.24's sort.Sort (pdqsort, sort/zsortinterface.go) for the C++ mirror of core.KNN.Predict
// (knn.go:107-108 sorts its CandidateSet with sort.Sort; go.mod:3 pins go 1.24).  sort.Sort is not stable:
// the order it leaves among equal keys is a property of its exact Less / Swap sequence, which this
// template reproduces call for call, so ties (and with them the top-k boundary and the summation order of
// knn.go:118-130) come out as in the reference.  less(i, j) and swap(i, j) act on positions of the
// sequence being sorted, as Go's sort.Interface does.  The same algorithm is restated in oracle/oracle.c
// (the tests' checker) and on the device in csrc/sim.hip (knn_predict_gosort_kernel).
#pragma once

#include <cstdint>

namespace core {
namespace gosort {

inline int bits_len(uint64_t x) {  // math/bits.Len
    int n = 0;
    for (; x; x >>= 1) ++n;
    return n;
}

template <typename Less, typename Swap>
struct Sorter {
    Less less;
    Swap swap;

    void insertion(int64_t a, int64_t b) {
        for (int64_t i = a + 1; i < b; ++i)
            for (int64_t j = i; j > a && less(j, j - 1); --j) swap(j, j - 1);
    }
    void sift_down(int64_t lo, int64_t hi, int64_t first) {
        int64_t root = lo;
        for (;;) {
            int64_t child = 2 * root + 1;
            if (child >= hi) return;
            if (child + 1 < hi && less(first + child, first + child + 1)) ++child;
            if (!less(first + root, first + child)) return;
            swap(first + root, first + child);
            root = child;
        }
    }
    void heap_sort(int64_t a, int64_t b) {
        const int64_t first = a, lo = 0, hi = b - a;
        for (int64_t i = (hi - 1) / 2; i >= 0; --i) sift_down(i, hi, first);
        for (int64_t i = hi - 1; i >= 0; --i) {
            swap(first, first + i);
            sift_down(lo, i, first);
        }
    }
    void order2(int64_t& a, int64_t& b, int& swaps) {
        if (less(b, a)) {
            const int64_t t = a;
            a = b;
            b = t;
            ++swaps;
        }
    }
    int64_t median(int64_t a, int64_t b, int64_t c, int& swaps) {
        order2(a, b, swaps);
        order2(b, c, swaps);
        order2(a, b, swaps);
        return b;
    }
    // 0 unknown, 1 increasing, 2 decreasing (the sortedHint of the Go source)
    int64_t choose_pivot(int64_t a, int64_t b, int& hint) {
        const int64_t l = b - a;
        int swaps = 0;
        int64_t i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
        if (l >= 8) {
            if (l >= 50) {  // Tukey ninther
                i = median(i - 1, i, i + 1, swaps);
                j = median(j - 1, j, j + 1, swaps);
                k = median(k - 1, k, k + 1, swaps);
            }
            j = median(i, j, k, swaps);
        }
        hint = swaps == 0 ? 1 : (swaps == 12 ? 2 : 0);
        return j;
    }
    void reverse(int64_t a, int64_t b) {
        for (int64_t i = a, j = b - 1; i < j; ++i, --j) swap(i, j);
    }
    bool partial_insertion(int64_t a, int64_t b) {
        int64_t i = a + 1;
        for (int step = 0; step < 5; ++step) {
            while (i < b && !less(i, i - 1)) ++i;
            if (i == b) return true;
            if (b - a < 50) return false;
            swap(i, i - 1);
            if (i - a >= 2)
                for (int64_t j = i - 1; j >= 1; --j) {
                    if (!less(j, j - 1)) break;
                    swap(j, j - 1);
                }
            if (b - i >= 2)
                for (int64_t j = i + 1; j < b; ++j) {
                    if (!less(j, j - 1)) break;
                    swap(j, j - 1);
                }
        }
        return false;
    }
    void break_patterns(int64_t a, int64_t b) {
        const int64_t length = b - a;
        if (length < 8) return;
        uint64_t r = static_cast<uint64_t>(length);  // xorshift seeded with the length
        const uint64_t modulus = uint64_t{1} << bits_len(static_cast<uint64_t>(length));
        const int64_t idx = a + (length / 4) * 2 - 1;
        for (int t = 0; t < 3; ++t) {
            r ^= r << 13;
            r ^= r >> 7;
            r ^= r << 17;
            int64_t other = static_cast<int64_t>(r & (modulus - 1));
            if (other >= length) other -= length;
            swap(idx - 1 + t, a + other);
        }
    }
    int64_t partition_equal(int64_t a, int64_t b, int64_t pivot) {
        swap(a, pivot);
        int64_t i = a + 1, j = b - 1;
        for (;;) {
            while (i <= j && !less(a, i)) ++i;
            while (i <= j && less(a, j)) --j;
            if (i > j) break;
            swap(i, j);
            ++i;
            --j;
        }
        return i;
    }
    int64_t partition(int64_t a, int64_t b, int64_t pivot, bool& already) {
        swap(a, pivot);
        int64_t i = a + 1, j = b - 1;
        while (i <= j && less(i, a)) ++i;
        while (i <= j && !less(j, a)) --j;
        if (i > j) {
            swap(j, a);
            already = true;
            return j;
        }
        swap(i, j);
        ++i;
        --j;
        for (;;) {
            while (i <= j && less(i, a)) ++i;
            while (i <= j && !less(j, a)) --j;
            if (i > j) break;
            swap(i, j);
            ++i;
            --j;
        }
        swap(j, a);
        already = false;
        return j;
    }
    void pdqsort(int64_t a, int64_t b, int limit) {
        bool was_balanced = true, was_partitioned = true;
        for (;;) {
            const int64_t length = b - a;
            if (length <= 12) {
                insertion(a, b);
                return;
            }
            if (limit == 0) {
                heap_sort(a, b);
                return;
            }
            if (!was_balanced) {
                break_patterns(a, b);
                --limit;
            }
            int hint = 0;
            int64_t pivot = choose_pivot(a, b, hint);
            if (hint == 2) {
                reverse(a, b);
                pivot = (b - 1) - (pivot - a);
                hint = 1;
            }
            if (was_balanced && was_partitioned && hint == 1 && partial_insertion(a, b)) return;
            if (a > 0 && !less(a - 1, pivot)) {
                a = partition_equal(a, b, pivot);
                continue;
            }
            bool already = false;
            const int64_t mid = partition(a, b, pivot, already);
            was_partitioned = already;
            const int64_t left_len = mid - a, right_len = b - mid, threshold = length / 8;
            if (left_len < right_len) {
                was_balanced = left_len >= threshold;
                pdqsort(a, mid, limit);
                a = mid + 1;
            } else {
                was_balanced = right_len >= threshold;
                pdqsort(mid + 1, b, limit);
                b = mid;
            }
        }
    }
};

// sort.Sort on n elements
template <typename Less, typename Swap>
void sort(int64_t n, Less less, Swap swap) {
    if (n <= 1) return;
    Sorter<Less, Swap> s{less, swap};
    s.pdqsort(0, n, bits_len(static_cast<uint64_t>(n)));
}

}  // namespace gosort
}  // namespace core
