// stl_uset.h — iteration order of libstdc++'s std::unordered_set<int>.
//
// LineMatcher::matchGrid (src/LineMatcher.cpp:191-272) collects its
// candidates in a default-constructed std::unordered_set<int> filled by
// range inserts of grid-cell lists (GridStructure::get,
// src/gridStructure.cpp:64-75) and breaks distance ties by the set's
// iteration order.  This restates libstdc++'s _Hashtable for
// unique int keys: std::hash<int> is the identity, bucket = key % count,
// max_load_factor 1, _Prime_rehash_policy (first allocation of at least 11
// buckets, growth x2 rounded up to the next prime of __prime_list), the
// range-insert size hint (GCC <= 10 only), nodes inserted at the front of their bucket (or
// of the whole list when the bucket was empty) and the rehash relinking.
// Checked against the build host's libstdc++ on random insert sequences
// (tests/native/uset_check.cpp).  __host__ __device__: one lane runs it.
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#define PLVI_UHD __host__ __device__ __forceinline__
#else
#define PLVI_UHD static inline
#endif

namespace plvi {

// libstdc++ __prime_list entries up to 8009 (tools/gen_stl_primes.cpp).
#include "stl_primes.inc"

struct UsetEmu {
    static constexpr int kBB = -2;  // _M_before_begin
    int nbkt;                       // _M_bucket_count
    int count;                      // _M_element_count
    long long next_resize;          // _Prime_rehash_policy::_M_next_resize
    int head;                       // _M_before_begin._M_nxt (node id, -1 = none)
    int* bkt;                       // bucket -> node before its first node (-1 empty, kBB)
    int* nxt;                       // node -> next node (-1 = end)
    int* key;                       // node -> key
    int capN, capB;
    bool overflow;
};

PLVI_UHD void uset_init(UsetEmu& u, int* bkt, int capB, int* nxt, int* key, int capN) {
    u.nbkt = 1;
    u.count = 0;
    u.next_resize = 0;
    u.head = -1;
    u.bkt = bkt;
    u.nxt = nxt;
    u.key = key;
    u.capN = capN;
    u.capB = capB;
    u.overflow = false;
    bkt[0] = -1;
}

PLVI_UHD int uset_next_of(const UsetEmu& u, int before) { return before == UsetEmu::kBB ? u.head : u.nxt[before]; }
PLVI_UHD void uset_set_next(UsetEmu& u, int before, int v) {
    if (before == UsetEmu::kBB) u.head = v;
    else u.nxt[before] = v;
}

// _Prime_rehash_policy::_M_next_bkt
PLVI_UHD int uset_next_bkt(UsetEmu& u, long long n) {
    const unsigned char fast[14] = {2, 2, 2, 3, 5, 5, 7, 7, 11, 11, 11, 11, 13, 13};
    if (n < 14) {
        if (n == 0) return 1;
        u.next_resize = fast[n];
        return fast[n];
    }
    int i = 6;  // lower_bound(__prime_list + 6, last, n)
    while (i < kStlPrimeCount - 1 && (long long)kStlPrimes[i] < n) ++i;
    u.next_resize = kStlPrimes[i];
    return (int)kStlPrimes[i];
}

PLVI_UHD void uset_rehash(UsetEmu& u, int nb) {
    if (nb > u.capB) {
        u.overflow = true;
        return;
    }
    for (int b = 0; b < nb; ++b) u.bkt[b] = -1;
    int p = u.head;
    u.head = -1;
    int bbegin = 0;
    while (p >= 0) {
        const int nx = u.nxt[p];
        const int b = (int)((unsigned)u.key[p] % (unsigned)nb);
        if (u.bkt[b] == -1) {
            u.nxt[p] = u.head;
            u.head = p;
            u.bkt[b] = UsetEmu::kBB;
            if (u.nxt[p] >= 0) u.bkt[bbegin] = p;
            bbegin = b;
        } else {
            const int before = u.bkt[b];
            u.nxt[p] = uset_next_of(u, before);
            uset_set_next(u, before, p);
        }
        p = nx;
    }
    u.nbkt = nb;
}

PLVI_UHD bool uset_find(const UsetEmu& u, int k) {
    const int b = (int)((unsigned)k % (unsigned)u.nbkt);
    if (u.bkt[b] == -1) return false;
    for (int p = uset_next_of(u, u.bkt[b]); p >= 0; p = u.nxt[p]) {
        if (u.key[p] == k) return true;
        if ((int)((unsigned)u.key[p] % (unsigned)u.nbkt) != b) break;
    }
    return false;
}

// _M_insert_unique_node: rehash check with the range hint, then insert at
// the beginning of the bucket.
PLVI_UHD bool uset_insert(UsetEmu& u, int k, long long n_ins) {
    if (uset_find(u, k)) return false;
    if ((long long)u.count + n_ins > u.next_resize) {
        long long want = (long long)u.count + n_ins;
        if (u.next_resize == 0 && want < 11) want = 11;
        const double min_bkts = (double)want;
        if (min_bkts >= (double)u.nbkt) {
            long long a = (long long)min_bkts + 1, b2 = (long long)u.nbkt * 2;
            uset_rehash(u, uset_next_bkt(u, a > b2 ? a : b2));
        } else {
            u.next_resize = u.nbkt;
        }
    }
    if (u.count >= u.capN || u.overflow) {
        u.overflow = true;
        return false;
    }
    const int node = u.count;
    u.key[node] = k;
    const int b = (int)((unsigned)k % (unsigned)u.nbkt);
    if (u.bkt[b] != -1) {
        const int before = u.bkt[b];
        u.nxt[node] = uset_next_of(u, before);
        uset_set_next(u, before, node);
    } else {
        u.nxt[node] = u.head;
        u.head = node;
        if (u.nxt[node] >= 0) u.bkt[(int)((unsigned)u.key[u.nxt[node]] % (unsigned)u.nbkt)] = node;
        u.bkt[b] = UsetEmu::kBB;
    }
    ++u.count;
    return true;
}

// insert(first, last) for a forward range (_Insert_base::_M_insert_range).
// range_hint = 1: libstdc++ up to GCC 10 (the reference's Ubuntu 20.04 /
// GCC 9.3 build) passes the remaining range length as the rehash hint;
// range_hint = 0: GCC 11+ inserts element by element (the build host here,
// against which tests/native/uset_check.cpp validates this emulation).
PLVI_UHD void uset_insert_range(UsetEmu& u, const int* first, int n, int range_hint) {
    long long n_elt = n;
    if (n == 0) return;
    for (int i = 0; i < n; ++i) {
        if (uset_insert(u, first[i], range_hint ? n_elt : 1)) n_elt = 1;
        else if (n_elt != 1) --n_elt;
    }
}

}  // namespace plvi
