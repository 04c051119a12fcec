// std_sort.h — a faithful restatement of libstdc++'s std::sort (introsort:
// median-of-3 to first, unguarded partition, depth limit 2*lg(n), heapsort
// fallback, final insertion sort with threshold 16) for device use.
//
// Lineextractor sorts keylines with std::sort and a `response >` comparator
// (src/LineExtractor.cc:78); std::sort is not stable, so the surviving top-k
// set and its order on ties depend on this exact algorithm.
// __host__ __device__ so tests compare it against the host libstdc++.
#pragma once

#ifdef __HIPCC__
#define PLVI_SORT_HD __host__ __device__
#else
#define PLVI_SORT_HD
#endif

namespace plvi {

struct SortItem {
    float key;  // KeyLine.response
    int idx;    // original position
};

// comp(a, b) = a.response > b.response (sort_lines_by_response)
PLVI_SORT_HD inline bool sort_comp(const SortItem& a, const SortItem& b) { return a.key > b.key; }

PLVI_SORT_HD inline void sort_swap(SortItem* a, SortItem* b) {
    SortItem t = *a;
    *a = *b;
    *b = t;
}

PLVI_SORT_HD inline void move_median_to_first(SortItem* result, SortItem* a, SortItem* b, SortItem* c) {
    if (sort_comp(*a, *b)) {
        if (sort_comp(*b, *c)) sort_swap(result, b);
        else if (sort_comp(*a, *c)) sort_swap(result, c);
        else sort_swap(result, a);
    } else if (sort_comp(*a, *c)) sort_swap(result, a);
    else if (sort_comp(*b, *c)) sort_swap(result, c);
    else sort_swap(result, b);
}

PLVI_SORT_HD inline SortItem* unguarded_partition(SortItem* first, SortItem* last, SortItem* pivot) {
    while (true) {
        while (sort_comp(*first, *pivot)) ++first;
        --last;
        while (sort_comp(*pivot, *last)) --last;
        if (!(first < last)) return first;
        sort_swap(first, last);
        ++first;
    }
}

PLVI_SORT_HD inline void push_heap(SortItem* first, long hole, long top, SortItem value) {
    long parent = (hole - 1) / 2;
    while (hole > top && sort_comp(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

PLVI_SORT_HD inline void adjust_heap(SortItem* first, long hole, long len, SortItem value) {
    const long top = hole;
    long second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (sort_comp(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    push_heap(first, hole, top, value);
}

PLVI_SORT_HD inline void make_heap(SortItem* first, SortItem* last) {
    const long len = last - first;
    if (len < 2) return;
    long parent = (len - 2) / 2;
    while (true) {
        SortItem v = first[parent];
        adjust_heap(first, parent, len, v);
        if (parent == 0) return;
        parent--;
    }
}

PLVI_SORT_HD inline void pop_heap(SortItem* first, SortItem* last, SortItem* result) {
    SortItem v = *result;
    *result = *first;
    adjust_heap(first, 0, last - first, v);
}

PLVI_SORT_HD inline void heap_sort_range(SortItem* first, SortItem* last) {  // __partial_sort(first,last,last)
    make_heap(first, last);
    while (last - first > 1) {
        --last;
        pop_heap(first, last, last);
    }
}

PLVI_SORT_HD inline void unguarded_linear_insert(SortItem* last) {
    SortItem val = *last;
    SortItem* next = last - 1;
    while (sort_comp(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

PLVI_SORT_HD inline void insertion_sort(SortItem* first, SortItem* last) {
    if (first == last) return;
    for (SortItem* i = first + 1; i != last; ++i) {
        if (sort_comp(*i, *first)) {
            SortItem val = *i;
            for (SortItem* p = i; p != first; --p) *p = *(p - 1);
            *first = val;
        } else {
            unguarded_linear_insert(i);
        }
    }
}

PLVI_SORT_HD inline int lg2(long n) {
    int r = 0;
    while (n > 1) { n >>= 1; ++r; }
    return r;
}

// __introsort_loop, iterative form of the right-recursion with an explicit
// stack (the recursion is on [cut, last) first, then the loop continues on
// [first, cut)).  Depth limits travel with each stacked range.
PLVI_SORT_HD inline void introsort_loop(SortItem* first, SortItem* last, int depth_limit) {
    struct Range {
        SortItem *first, *last;
        int depth;
    };
    Range stack[64];
    int sp = 0;
    stack[sp++] = Range{first, last, depth_limit};
    while (sp > 0) {
        Range r = stack[--sp];
        SortItem* f = r.first;
        SortItem* l = r.last;
        int depth = r.depth;
        while (l - f > 16) {
            if (depth == 0) {
                heap_sort_range(f, l);
                break;
            }
            --depth;
            SortItem* mid = f + (l - f) / 2;
            move_median_to_first(f, f + 1, mid, l - 1);
            SortItem* cut = unguarded_partition(f + 1, l, f);
            // recursive call on [cut, l) happens before the loop continues on [f, cut):
            // process it first (LIFO): push the remaining left part, then the right part.
            stack[sp++] = Range{f, cut, depth};
            stack[sp++] = Range{cut, l, depth};
            break;
        }
    }
}

#ifdef __HIPCC__
// The same permutation as std_sort, replayed by a whole workgroup: every
// partition of __introsort_loop reads and writes only its own range, so the
// ranges of one recursion level are independent -- one thread per range,
// level by level (both children carry the decremented depth, as in the
// reference loop; a range at depth 0 is heap-sorted by its thread).  The
// final insertion sort never moves an element across a partition boundary
// (left parts hold keys >= the pivot's, right parts <=, so comp(right,
// left) is false and the linear inserts stop there), so it runs per final
// range, in parallel.  ~2n sequential element steps instead of n log n.
// Any block size; LDS scratch: rng0 / rng1 of 256 ranges each (a level holds
// < n / 17 ranges longer than 16: n <= 4352), `segbits` (n bits), 4 ints.
struct SortRange {
    int first, last, depth;
};

// unguarded_partition(a + f0 + 1, a + l0, a + f0) by the whole block.  The
// sequential loop swaps its k-th left stop (k-th element, from the left, with
// !comp(x, pivot)) with its k-th right stop (from the right, !comp(pivot, x))
// for as long as the left one lies before the right one; the scans never read
// a swapped element before they cross, so the stops are those of the
// original range: rank them with a block scan, swap the first m pairs (m =
// the pairs in order, a monotone test) and return min(L[m], R[m-1]) -- where
// the sequential scans stop after their last swap (L[0] without a swap).
// lpos / rpos: n entries each, scan: blockDim.x ints.
constexpr int kCoopPartition = 128;  // ranges longer than this are partitioned by the block
__device__ inline int block_partition(SortItem* a, int f0, int l0, unsigned short* lpos, unsigned short* rpos,
                                      int* scan, int* ctl) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const SortItem P = a[f0];
    const int b = f0 + 1, len = l0 - b, per = (len + nt - 1) / nt;
    const int s0 = min(b + tid * per, l0), s1 = min(s0 + per, l0);
    int cl = 0, cr = 0;
    for (int i = s0; i < s1; ++i) {
        cl += !sort_comp(a[i], P);
        cr += !sort_comp(P, a[i]);
    }
    // inclusive scan of the packed counts (each < 2^16) over the threads
    int v = cl | (cr << 16);
    scan[tid] = v;
    __syncthreads();
    for (int o = 1; o < nt; o <<= 1) {
        const int u = tid >= o ? scan[tid - o] : 0;
        __syncthreads();
        v += u;
        scan[tid] = v;
        __syncthreads();
    }
    const int tot = scan[nt - 1], nL = tot & 0xffff, nR = tot >> 16;
    int lr = (v & 0xffff) - cl, rseen = (v >> 16) - cr;  // stops before this thread's chunk
    for (int i = s0; i < s1; ++i) {
        if (!sort_comp(a[i], P)) lpos[lr++] = (unsigned short)i;
        if (!sort_comp(P, a[i])) rpos[nR - 1 - rseen++] = (unsigned short)i;  // rank from the right
    }
    if (tid == 0) ctl[2] = 0;
    __syncthreads();
    const int np = min(nL, nR);
    int mc = 0;
    for (int k = tid; k < np; k += nt) mc += lpos[k] < rpos[k];
    if (mc) atomicAdd(&ctl[2], mc);
    __syncthreads();
    const int m = ctl[2];
    for (int k = tid; k < m; k += nt) sort_swap(a + lpos[k], a + rpos[k]);
    const int cut = m == 0 ? lpos[0] : min(m < nL ? (int)lpos[m] : 0x7fffffff, (int)rpos[m - 1]);
    __syncthreads();
    return cut;
}

// Precondition: n <= kSortBlockMax.  block_partition packs a thread's two
// counts into one int (cl | cr << 16, each < 2^15 keeps the scan's sum
// positive) and keeps positions as unsigned short; callers size their arrays
// with a compile-time cap and static_assert it against this limit.
constexpr int kSortBlockMax = 32767;
__device__ inline void std_sort_block(SortItem* a, int n, SortRange* rng0, SortRange* rng1, unsigned* segbits,
                                      int* ctl, unsigned short* lpos, unsigned short* rpos, int* scan,
                                      int depth0 = -1) {  // depth0 >= 0: test override of 2 lg n
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int w = tid; w < (n + 31) / 32; w += nt) segbits[w] = 0u;
    if (tid == 0) {
        ctl[0] = 0;
        if (n > 16) {
            rng0[0] = SortRange{0, n, depth0 >= 0 ? depth0 : lg2(n) * 2};
            ctl[0] = 1;
        } else if (n > 0) {
            segbits[0] = 1u;  // one final range [0, n)
        }
    }
    __syncthreads();
    SortRange* cur = rng0;
    SortRange* nxt = rng1;
    int nr = ctl[0];
    while (nr > 0) {
        if (tid == 0) ctl[1] = 0;
        __syncthreads();
        // long ranges: the whole block partitions them, one after another
        for (int r = 0; r < nr; ++r) {
            const SortRange R = cur[r];
            if (R.depth == 0 || R.last - R.first <= kCoopPartition) continue;
            if (tid == 0) {
                SortItem* f = a + R.first;
                move_median_to_first(f, f + 1, f + (R.last - R.first) / 2, a + R.last - 1);
            }
            __syncthreads();
            const int c = block_partition(a, R.first, R.last, lpos, rpos, scan, ctl);
            if (tid == 0) {
                const SortRange kids[2] = {SortRange{R.first, c, R.depth - 1}, SortRange{c, R.last, R.depth - 1}};
                for (const SortRange& k : kids) {
                    if (k.last - k.first > 16) nxt[atomicAdd(&ctl[1], 1)] = k;
                    else if (k.last > k.first) atomicOr(&segbits[k.first >> 5], 1u << (k.first & 31));
                }
            }
            __syncthreads();
        }
        for (int r = tid; r < nr; r += nt) {
            const SortRange R = cur[r];
            if (R.depth != 0 && R.last - R.first > kCoopPartition) continue;  // done above
            SortItem* f = a + R.first;
            SortItem* l = a + R.last;
            if (R.depth == 0) {  // __partial_sort(first, last, last)
                heap_sort_range(f, l);
                atomicOr(&segbits[R.first >> 5], 1u << (R.first & 31));
                continue;
            }
            SortItem* mid = f + (l - f) / 2;
            move_median_to_first(f, f + 1, mid, l - 1);
            SortItem* cut = unguarded_partition(f + 1, l, f);
            const int c = (int)(cut - a);
            const SortRange kids[2] = {SortRange{R.first, c, R.depth - 1}, SortRange{c, R.last, R.depth - 1}};
            for (const SortRange& k : kids) {
                if (k.last - k.first > 16) nxt[atomicAdd(&ctl[1], 1)] = k;
                else if (k.last > k.first) atomicOr(&segbits[k.first >> 5], 1u << (k.first & 31));
            }
        }
        __syncthreads();
        nr = ctl[1];
        SortRange* t = cur;
        cur = nxt;
        nxt = t;
        __syncthreads();
    }
    // __final_insertion_sort, one thread per final range
    for (int i = tid; i < n; i += nt) {
        if (!((segbits[i >> 5] >> (i & 31)) & 1u)) continue;
        int e = i + 1;
        while (e < n && !((segbits[e >> 5] >> (e & 31)) & 1u)) ++e;
        insertion_sort(a + i, a + e);
    }
    __syncthreads();
}
#endif

PLVI_SORT_HD inline void std_sort(SortItem* first, SortItem* last) {
    if (first == last) return;
    introsort_loop(first, last, lg2(last - first) * 2);
    // __final_insertion_sort
    if (last - first > 16) {
        insertion_sort(first, first + 16);
        for (SortItem* i = first + 16; i != last; ++i) unguarded_linear_insert(i);
    } else {
        insertion_sort(first, last);
    }
}

}  // namespace plvi
