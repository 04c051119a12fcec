// tests/native/uset_check.cpp — the product's libstdc++ unordered_set<int>
// emulation (pl-vi-orbslam3_amd/csrc/stl_uset.h) vs the real container:
// random sequences of range inserts (as GridStructure::get issues them),
// compared on iteration order and bucket count after every range.
// Mode "gcc10" (argv[2]): the GCC <= 10 range-insert rule (size hint), with
// the real container driven through merge() from a reverse-ordered
// constant-hash multiset -- libstdc++ 11's _M_merge_unique runs exactly the
// GCC <= 10 _M_insert_range hint loop (see oracle/match_oracle.cpp).
#include <cstdio>
#include <list>
#include <random>
#include <string>
#include <unordered_set>
#include <vector>

#include "../../pl-vi-orbslam3_amd/csrc/stl_uset.h"

// the host libstdc++'s range-insert behaviour (no size hint since GCC 11)
static int kHint = __GNUC__ >= 11 ? 0 : 1;

struct ConstHash {
    size_t operator()(int) const noexcept { return 0; }
};
struct NeverEq {
    bool operator()(int, int) const noexcept { return false; }
};

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20000;
    const bool gcc10 = argc > 2 && std::string(argv[2]) == "gcc10";
    if (gcc10) kHint = 1;
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
            // GridStructure cells hold distinct line indices
            const int len = rng() % (r % 5 == 0 ? 12 : 4);
            for (int i = 0; i < len; ++i) {
                const int k = rng() % maxKey;
                bool dup = false;
                for (int c : cell) dup |= c == k;
                if (!dup || !gcc10) cell.push_back(k);
            }
            if (gcc10) {
                std::unordered_multiset<int, ConstHash, NeverEq> src;
                for (auto it = cell.rbegin(); it != cell.rend(); ++it) src.insert(*it);
                ref.merge(src);
            } else {
                ref.insert(cell.begin(), cell.end());
            }
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
    printf("mismatches=%ld trials=%d mode=%s\n", bad, trials, gcc10 ? "gcc10" : "host");
    return bad ? 1 : 0;
}
