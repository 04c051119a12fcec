// tests/native/sort_check.cpp — the product's std::sort restatement
// (pl-vi-orbslam3_amd/csrc/std_sort.h) vs the host libstdc++ std::sort with
// the reference comparator (LineExtractor.cc:78), on tie-heavy inputs.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../pl-vi-orbslam3_amd/csrc/std_sort.h"

int main() {
    std::mt19937 rng(42);
    long bad = 0, total = 0;
    for (int trial = 0; trial < 20000; ++trial) {
        int n = (trial % 7 == 0) ? (int)(rng() % 5000) : (int)(rng() % 600);
        int distinct = 1 + (int)(rng() % (trial % 3 == 0 ? 4 : 400));
        std::vector<plvi::SortItem> a(n);
        for (int i = 0; i < n; ++i) a[i] = plvi::SortItem{(float)(rng() % distinct) * 0.01f, i};
        if (trial % 11 == 0) std::sort(a.begin(), a.end(), [](auto& x, auto& y) { return x.key < y.key; });  // adversarial order
        if (trial % 13 == 0) std::reverse(a.begin(), a.end());
        std::vector<plvi::SortItem> b = a;
        std::sort(a.begin(), a.end(), [](const plvi::SortItem& x, const plvi::SortItem& y) { return x.key > y.key; });
        plvi::std_sort(b.data(), b.data() + n);
        for (int i = 0; i < n; ++i)
            if (a[i].idx != b[i].idx) { ++bad; if (bad < 5) printf("trial %d n %d mismatch at %d\n", trial, n, i); break; }
        ++total;
    }
    // heapsort fallback (depth limit exhausted) == std::partial_sort(first, last, last)
    for (int trial = 0; trial < 2000; ++trial) {
        int n = 2 + (int)(rng() % 700);
        int distinct = 1 + (int)(rng() % 50);
        std::vector<plvi::SortItem> a(n);
        for (int i = 0; i < n; ++i) a[i] = plvi::SortItem{(float)(rng() % distinct), i};
        std::vector<plvi::SortItem> b = a;
        std::partial_sort(a.begin(), a.end(), a.end(),
                          [](const plvi::SortItem& x, const plvi::SortItem& y) { return x.key > y.key; });
        plvi::heap_sort_range(b.data(), b.data() + n);
        for (int i = 0; i < n; ++i)
            if (a[i].idx != b[i].idx) { ++bad; break; }
        ++total;
    }
    printf("mismatches=%ld checked=%ld\n", bad, total);
    return bad ? 1 : 0;
}
