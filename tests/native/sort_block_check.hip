// sort_block_check.hip -- the workgroup replay of libstdc++ std::sort
// (csrc/std_sort.h: std_sort_block, used by line_assemble_kernel's tie path)
// against the host's libstdc++ std::sort (default depth limit) and against
// the sequential restatement with a forced small depth limit (heapsort
// fallback).  Tie-heavy, sorted, reversed, all-equal and random keys, n in
// 0..4096.  Exit 0 = every case identical.  Test infrastructure.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

#include "../../pl-vi-orbslam3_amd/csrc/std_sort.h"

using namespace plvi;

__global__ __launch_bounds__(256) void sort_kernel(SortItem* data, const int* off, const int* depth, int ncase) {
    __shared__ SortItem s[4096];
    __shared__ SortRange r0[256], r1[256];
    __shared__ unsigned seg[4096 / 32];
    __shared__ int ctl[4];
    __shared__ unsigned short lpos[4096], rpos[4096];
    __shared__ int scan[256];
    const int c = blockIdx.x;
    const int o = off[c], n = off[c + 1] - off[c];
    for (int i = threadIdx.x; i < n; i += 256) s[i] = data[o + i];
    __syncthreads();
    std_sort_block(s, n, r0, r1, seg, ctl, lpos, rpos, scan, depth[c]);
    for (int i = threadIdx.x; i < n; i += 256) data[o + i] = s[i];
}

static void seq_sort_depth(SortItem* f, SortItem* l, int depth) {  // std_sort with a forced depth limit
    if (f == l) return;
    introsort_loop(f, l, depth);
    if (l - f > 16) {
        insertion_sort(f, f + 16);
        for (SortItem* i = f + 16; i != l; ++i) unguarded_linear_insert(i);
    } else {
        insertion_sort(f, l);
    }
}

int main() {
    std::mt19937 rng(7);
    std::vector<SortItem> all, expect;
    std::vector<int> off{0}, depth;
    const int sizes[] = {0, 1, 2, 3, 16, 17, 18, 31, 33, 64, 100, 255, 256, 257, 600, 1000, 1500, 2048, 4096};
    for (int rep = 0; rep < 12; ++rep)
        for (int n : sizes)
            for (int kind = 0; kind < 7; ++kind) {
                std::vector<SortItem> v(n);
                for (int i = 0; i < n; ++i) {
                    float k;
                    switch (kind) {
                        case 0: k = (float)(rng() % 4); break;                    // heavy ties
                        case 1: k = (float)(rng() % 50) * 0.01f; break;           // ties, line-response-like
                        case 2: k = 1.0f; break;                                  // all equal
                        case 3: k = (float)i; break;                              // ascending (comp is >)
                        case 4: k = (float)(n - i); break;                        // descending
                        case 5: k = (float)(i < n / 2 ? i : n - i) + (rng() % 3); break;  // organ pipe with ties
                        default: k = std::uniform_real_distribution<float>(0.f, 1.f)(rng); break;
                    }
                    v[i] = SortItem{k, i};
                }
                // default depth vs the host libstdc++; a forced small depth vs the restatement
                const int d = rep % 3 == 2 ? (int)(rng() % 4) : -1;
                std::vector<SortItem> e = v;
                if (d < 0) std::sort(e.begin(), e.end(), [](const SortItem& a, const SortItem& b) { return a.key > b.key; });
                else seq_sort_depth(e.data(), e.data() + n, d);
                all.insert(all.end(), v.begin(), v.end());
                expect.insert(expect.end(), e.begin(), e.end());
                off.push_back((int)all.size());
                depth.push_back(d);
            }
    const int ncase = (int)depth.size();
    SortItem* dd;
    int *doff, *ddep;
    if (hipMalloc(&dd, sizeof(SortItem) * std::max<size_t>(all.size(), 1)) || hipMalloc(&doff, 4 * off.size()) ||
        hipMalloc(&ddep, 4 * depth.size()))
        return 2;
    (void)hipMemcpy(dd, all.data(), sizeof(SortItem) * all.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(doff, off.data(), 4 * off.size(), hipMemcpyHostToDevice);
    (void)hipMemcpy(ddep, depth.data(), 4 * depth.size(), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(sort_kernel, dim3(ncase), dim3(256), 0, nullptr, dd, doff, ddep, ncase);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(all.data(), dd, sizeof(SortItem) * all.size(), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int c = 0; c < ncase; ++c)
        for (int i = off[c]; i < off[c + 1]; ++i)
            if (all[i].idx != expect[i].idx) {
                if (bad < 5) printf("case %d (n %d, depth %d): position %d idx %d vs %d\n", c, off[c + 1] - off[c],
                                    depth[c], i - off[c], all[i].idx, expect[i].idx);
                ++bad;
                break;
            }
    printf("%d cases, %d mismatching\n", ncase, bad);
    return bad ? 1 : 0;
}
