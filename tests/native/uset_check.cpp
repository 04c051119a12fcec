// tests/native/uset_check.cpp — the product's libstdc++ unordered_set<int>
// emulation (pl-vi-orbslam3_amd/csrc/stl_uset.h) vs the real container:
// random sequences of range inserts (as GridStructure::get issues them),
// compared on iteration order after every range.
#include <cstdio>
#include <list>
#include <random>
#include <unordered_set>
#include <vector>

#include "../../pl-vi-orbslam3_amd/csrc/stl_uset.h"

// the host libstdc++'s range-insert behaviour (no size hint since GCC 11)
static const int kHint = __GNUC__ >= 11 ? 0 : 1;

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937 rng(7);
    std::vector<int> bkt(20000), nxt(4096), key(4096);
    long bad = 0;
    for (int t = 0; t < trials; ++t) {
        std::unordered_set<int> ref;
        plvi::UsetEmu u;
        plvi::uset_init(u, bkt.data(), (int)bkt.size(), nxt.data(), key.data(), 4096);
        const int ranges = 1 + rng() % 80;
        const int maxKey = 1 + rng() % (t % 3 == 0 ? 50 : (t % 3 == 1 ? 600 : 3000));
        for (int r = 0; r < ranges; ++r) {
            std::list<int> cell;  // GridStructure cell lists are std::list<int>
            const int len = rng() % (r % 5 == 0 ? 12 : 4);
            for (int i = 0; i < len; ++i) cell.push_back(rng() % maxKey);
            ref.insert(cell.begin(), cell.end());
            std::vector<int> v(cell.begin(), cell.end());
            plvi::uset_insert_range(u, v.data(), (int)v.size(), kHint);
            std::vector<int> a(ref.begin(), ref.end()), b;
            for (int p = u.head; p >= 0; p = u.nxt[p]) b.push_back(u.key[p]);
            if (a != b || (int)ref.bucket_count() != u.nbkt || u.overflow) {
                if (bad < 5) fprintf(stderr, "trial %d range %d: size %zu/%zu buckets %zu/%d\n", t, r, a.size(), b.size(),
                                     ref.bucket_count(), u.nbkt);
                ++bad;
                break;
            }
        }
    }
    printf("mismatches=%ld trials=%d\n", bad, trials);
    return bad ? 1 : 0;
}
