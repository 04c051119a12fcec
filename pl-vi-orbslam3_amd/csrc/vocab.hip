// vocab.hip — DBoW2 TemplatedVocabulary<FORB::TDescriptor, FORB> on the device
// (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h), the vocabulary half of
// Frame::ComputeBoW (src/Frame.cc:1115-1122) / KeyFrame::ComputeBoW
// (src/KeyFrame.cc:111): transform(descriptors, BowVector&, FeatureVector&, 4).
//
// Host: loadFromTextFile (:1338-1424) restated with a single-pass parser
// (same node numbering, word numbering and tail-line behaviour), then the
// tree is laid out breadth-first on the device so the children of every
// node are contiguous: one (first child, count) int2 per node, descriptors as
// 2 x uint4.
//
// Kernel: one workgroup (4 waves) per frame.
//   descent  (:1217-1259)  16 lanes per descriptor, lane j = child j: FORB
//            distance, then a 16-lane min over (distance << 16 | j) = the
//            reference's strict-< first-wins argmin; the winner's child range
//            travels with it through the shuffle, so each level costs one
//            dependent load round.  The node at level L - levelsup is kept.
//   BowVector (:1145-1193, BowVector.cpp:34-84)  bitonic sort of
//            (word << 32 | feature) keys in LDS, run lengths by a block scan;
//            addWeight's repeated sum is replayed per word in feature order,
//            the L1/L2 norm is a single-lane sum in map (word id) order.
//   FeatureVector (FeatureVector.cpp:31-45)  the same sort on
//            (node << 32 | feature): CSR (node, off, idx), map order.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "plvi_common.h"

namespace plvi {

struct VocabDev {
    const int2* range;       // [nd] (first child device index, child count)
    const uint4* desc;       // [nd][2]
    const unsigned* ref_id;  // [nd] reference NodeId
    const unsigned* word;    // [nd] word id (leaves)
    const double* weight;    // [nd]
};

constexpr int kBowThreads = 256;
constexpr int kDescentGroup = 16;
constexpr int kMaxDepth = 64;

__device__ __forceinline__ int popc256(const uint4& a0, const uint4& a1, const uint4& b0, const uint4& b1) {
    return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
           __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Exclusive scan of one int per thread over the 256-thread block.
__device__ int block_excl_scan(int v, int* s_tmp, int* total) {
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_tmp[wv] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kBowThreads / 64; ++w) {
        const int t = s_tmp[w];
        base += w < wv ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

__device__ void bitonic_sort_u64(unsigned long long* a, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < P / 2; t += kBowThreads) {
                const int i = (t / j) * 2 * j + (t % j), ixj = i + j;
                const bool asc = (i & k) == 0;
                const unsigned long long x = a[i], y = a[ixj];
                if ((x > y) == asc) {
                    a[i] = y;
                    a[ixj] = x;
                }
            }
            __syncthreads();
        }
    }
}

// Group runs of equal (key >> 32) among the first m sorted keys: returns the
// number of runs, s_head[r] = index of run r's first key, s_head[runs] = m.
__device__ int runs_of(const unsigned long long* key, int m, int P, int* s_head, int* s_tmp) {
    const int E = P / kBowThreads, j0 = threadIdx.x * E;
    int c = 0;
    for (int j = j0; j < j0 + E; ++j)
        c += j < m && (j == 0 || (key[j] >> 32) != (key[j - 1] >> 32));
    int total;
    int pos = block_excl_scan(c, s_tmp, &total);
    for (int j = j0; j < j0 + E; ++j)
        if (j < m && (j == 0 || (key[j] >> 32) != (key[j - 1] >> 32))) s_head[pos++] = j;
    if (threadIdx.x == 0) s_head[total] = m;
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(kBowThreads) void bow_transform_kernel(
    VocabDev V, int L, int levelsup, int must, int l2, int tf, const uint8_t* __restrict__ fdesc,
    const int* __restrict__ fcount, int cap, int P, unsigned* __restrict__ bow_word, double* __restrict__ bow_value,
    int* __restrict__ bow_n, unsigned* __restrict__ fv_node, int* __restrict__ fv_off, unsigned* __restrict__ fv_idx,
    int* __restrict__ fv_n, unsigned* __restrict__ feat_word, unsigned* __restrict__ feat_nid, int* __restrict__ err) {
    extern __shared__ __align__(16) unsigned long long lds64[];
    unsigned long long* s_key = lds64;                       // [P]
    double* s_w = reinterpret_cast<double*>(lds64 + P);      // [P] word weight per feature
    double* s_val = s_w + P;                                 // [P] BowVector values
    unsigned* s_word = reinterpret_cast<unsigned*>(s_val + P);  // [P]
    unsigned* s_nid = s_word + P;                            // [P]
    int* s_head = reinterpret_cast<int*>(s_nid + P);         // [P + 1]
    __shared__ int s_tmp[kBowThreads / 64];
    __shared__ double s_norm;
    const int f = blockIdx.x, tid = threadIdx.x;
    int n = fcount[f];
    if (n > cap) {
        if (tid == 0) atomicOr(err, 1);
        n = cap;
    }
    const int nid_level = L - levelsup;
    // ---- descent: 16 lanes per feature
    const int grp = tid / kDescentGroup, sub = tid % kDescentGroup;
    const uint8_t* FD = fdesc + (size_t)f * cap * 32;
    for (int i0 = 0; i0 < n; i0 += kBowThreads / kDescentGroup) {
        const int i = i0 + grp;
        const bool valid = i < n;
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
        if (valid) {
            const uint4* q = reinterpret_cast<const uint4*>(FD + (size_t)i * 32);
            q0 = q[0];
            q1 = q[1];
        }
        int2 rng = V.range[0];
        int node = 0, level = 0;
        unsigned nid = 0;  // levels above nid_level: 0 (root); see DESIGN.md (unset in the reference)
        bool done = !valid;
        while (__any(!done)) {
            if (!done) {
                ++level;
                const int c0 = rng.x, nc = rng.y;
                unsigned best = 0xffffffffu;
                int2 brng = make_int2(0, 0);
                for (int base = 0; base < nc; base += kDescentGroup) {
                    const int j = base + sub;
                    unsigned key = 0xffffffffu;
                    int2 r = make_int2(0, 0);
                    if (j < nc) {
                        const uint4* d = V.desc + 2 * (size_t)(c0 + j);
                        r = V.range[c0 + j];
                        key = ((unsigned)popc256(q0, q1, d[0], d[1]) << 16) | (unsigned)j;
                    }
                    unsigned k = key;
#pragma unroll
                    for (int o = kDescentGroup / 2; o > 0; o >>= 1) k = min(k, (unsigned)__shfl_xor((int)k, o, kDescentGroup));
                    const int src = (int)(k & 0xffffu) - base;
                    const int rx = __shfl(r.x, src & (kDescentGroup - 1), kDescentGroup);
                    const int ry = __shfl(r.y, src & (kDescentGroup - 1), kDescentGroup);
                    if (k < best) {
                        best = k;
                        brng = make_int2(rx, ry);
                    }
                }
                node = c0 + (int)(best & 0xffffu);
                if (level == nid_level) nid = V.ref_id[node];
                rng = brng;
                if (rng.y == 0) done = true;
                if (level >= kMaxDepth) {
                    done = true;
                    if (sub == 0) atomicOr(err, 2);
                }
            }
        }
        if (valid && sub == 0) {
            s_word[i] = V.word[node];
            s_w[i] = V.weight[node];
            s_nid[i] = nid;
            if (feat_word) feat_word[(size_t)f * cap + i] = V.word[node];
            if (feat_nid) feat_nid[(size_t)f * cap + i] = nid;
        }
    }
    __syncthreads();
    // ---- BowVector
    int cm = 0;
    for (int j = tid; j < P; j += kBowThreads) {
        const bool live = j < n && s_w[j] > 0;  // "if(w > 0) // not stopped"
        s_key[j] = live ? ((unsigned long long)s_word[j] << 32) | (unsigned)j : ~0ull;
        cm += live;
    }
    int m;
    (void)block_excl_scan(cm, s_tmp, &m);
    bitonic_sort_u64(s_key, P);
    const int nb = runs_of(s_key, m, P, s_head, s_tmp);
    for (int r = tid; r < nb; r += kBowThreads) {
        const int j = s_head[r], c = s_head[r + 1] - j;
        const double w = s_w[(unsigned)(s_key[j] & 0xffffffffu)];
        double v = w;
        if (tf)
            for (int t = 1; t < c; ++t) v += w;  // addWeight, once per feature of the word
        if (tf && !must) v /= (double)nb;
        s_val[r] = v;
        s_word[r] = (unsigned)(s_key[j] >> 32);
    }
    __syncthreads();
    if (must) {
        if (tid == 0) {
            double nrm = 0.0;
            if (!l2) {
                for (int r = 0; r < nb; ++r) nrm += fabs(s_val[r]);
            } else {
                for (int r = 0; r < nb; ++r) nrm += s_val[r] * s_val[r];
                nrm = sqrt(nrm);
            }
            s_norm = nrm;
        }
        __syncthreads();
    }
    const double nrm = must ? s_norm : 0.0;
    for (int r = tid; r < nb; r += kBowThreads) {
        double v = s_val[r];
        if (must && nrm > 0.0) v /= nrm;
        bow_word[(size_t)f * cap + r] = s_word[r];
        bow_value[(size_t)f * cap + r] = v;
    }
    if (tid == 0) bow_n[f] = nb;
    __syncthreads();
    // ---- FeatureVector
    for (int j = tid; j < P; j += kBowThreads) {
        const bool live = j < n && s_w[j] > 0;
        s_key[j] = live ? ((unsigned long long)s_nid[j] << 32) | (unsigned)j : ~0ull;
    }
    __syncthreads();
    bitonic_sort_u64(s_key, P);
    const int nf = runs_of(s_key, m, P, s_head, s_tmp);
    int* FO = fv_off + (size_t)f * (cap + 1);
    for (int r = tid; r <= nf; r += kBowThreads) {
        FO[r] = s_head[r];
        if (r < nf) fv_node[(size_t)f * cap + r] = (unsigned)(s_key[s_head[r]] >> 32);
    }
    for (int j = tid; j < m; j += kBowThreads) fv_idx[(size_t)f * cap + j] = (unsigned)(s_key[j] & 0xffffffffu);
    if (tid == 0) fv_n[f] = nf;
}

static int bow_pow2(int cap) {
    int P = kBowThreads;
    while (P < cap) P <<= 1;
    return P;
}
static size_t bow_smem(int P) { return (size_t)P * (8 + 8 + 8 + 4 + 4 + 4) + 16; }

// ---------------------------------------------------------------------------
// Host: node table (reference numbering) -> breadth-first device layout.
// ---------------------------------------------------------------------------
struct VocabHost {
    int k = 0, L = 0, scoring = 0, weighting = 0;
    std::vector<int> parent;       // [n + 1], node 0 = root
    std::vector<uint8_t> desc;     // [n + 1][32]
    std::vector<double> weight;    // [n + 1]
    std::vector<unsigned> word;    // [n + 1]
    int nwords = 0;
};

struct Vocab {
    int k = 0, L = 0, scoring = 0, weighting = 0, nNodes = 0, nWords = 0, device = 0;
    DevBuf range, desc, refid, word, weight, err;
    hipStream_t stream = nullptr;
    ~Vocab() {
        if (stream) (void)hipStreamDestroy(stream);
    }

    int build(const VocabHost& h, int dev) {
        k = h.k; L = h.L; scoring = h.scoring; weighting = h.weighting;
        nNodes = (int)h.parent.size();
        nWords = h.nwords;
        device = dev;
        const int n = nNodes;
        std::vector<int> cnt(n, 0), first(n + 1, 0);
        for (int i = 1; i < n; ++i) cnt[h.parent[i]]++;
        for (int i = 0; i < n; ++i) first[i + 1] = first[i] + cnt[i];
        std::vector<int> kids(n > 1 ? n - 1 : 1), fill(first.begin(), first.end() - 1);
        for (int i = 1; i < n; ++i) kids[fill[h.parent[i]]++] = i;  // children in push order
        std::vector<int> order;
        order.reserve(n);
        order.push_back(0);
        std::vector<int2> rng(n);
        for (size_t q = 0; q < order.size(); ++q) {
            const int v = order[q];
            rng[q] = make_int2((int)order.size(), cnt[v]);
            for (int c = first[v]; c < first[v + 1]; ++c) order.push_back(kids[c]);
        }
        if ((int)order.size() != n) return PLVI_E_BADARG;
        std::vector<uint8_t> d((size_t)n * 32);
        std::vector<unsigned> rid(n), wd(n);
        std::vector<double> wt(n);
        for (int q = 0; q < n; ++q) {
            const int v = order[q];
            std::memcpy(&d[(size_t)q * 32], &h.desc[(size_t)v * 32], 32);
            rid[q] = (unsigned)v;
            wd[q] = h.word[v];
            wt[q] = h.weight[v];
        }
        PLVI_CHECK(hipSetDevice(device));
        PLVI_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        if (range.alloc(sizeof(int2) * n) || desc.alloc((size_t)32 * n) || refid.alloc(4 * (size_t)n) ||
            word.alloc(4 * (size_t)n) || weight.alloc(8 * (size_t)n) || err.alloc(sizeof(int)))
            return PLVI_E_HIP;
        PLVI_CHECK(hipMemcpy(range.p, rng.data(), sizeof(int2) * n, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(desc.p, d.data(), d.size(), hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(refid.p, rid.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(word.p, wd.data(), 4 * (size_t)n, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(weight.p, wt.data(), 8 * (size_t)n, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemset(err.p, 0, sizeof(int)));
        return PLVI_OK;
    }

    VocabDev dev() const {
        return VocabDev{range.as<int2>(), desc.as<uint4>(), refid.as<unsigned>(), word.as<unsigned>(),
                        weight.as<double>()};
    }
};

// istream-style token cursor over one line: once an extraction fails, every
// later extraction on the line fails too and yields 0 (C++11 operator>>).
struct LineCursor {
    const char* p;
    const char* e;
    bool fail = false;
    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\v' || *p == '\f')) ++p;
    }
    long get_int() {
        ws();
        if (fail || p >= e) { fail = true; return 0; }
        char* q;
        const long v = strtol(p, &q, 10);
        if (q == p) { fail = true; return 0; }
        p = q;
        return v;
    }
    double get_double() {
        ws();
        if (fail || p >= e) { fail = true; return 0; }
        char buf[64];
        const char* t = p;
        while (t < e && !(*t == ' ' || *t == '\t' || *t == '\r' || *t == '\v' || *t == '\f')) ++t;
        const size_t len = std::min<size_t>((size_t)(t - p), sizeof(buf) - 1);
        std::memcpy(buf, p, len);
        buf[len] = 0;
        char* q;
        const double v = strtod(buf, &q);
        if (q == buf) { fail = true; return 0; }
        p += (q - buf);
        return v;
    }
};

// TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424).
static int load_text(const char* path, int emulate_tail, VocabHost& h) {
    FILE* fp = fopen(path, "rb");
    if (!fp) return PLVI_E_BADARG;
    std::vector<char> buf;
    {
        char tmp[1 << 16];
        size_t r;
        while ((r = fread(tmp, 1, sizeof(tmp), fp)) > 0) buf.insert(buf.end(), tmp, tmp + r);
        fclose(fp);
    }
    const char* p = buf.data();
    const char* end = p + buf.size();
    auto next_line = [&](const char*& b, const char*& e) {  // std::getline
        b = p;
        while (p < end && *p != '\n') ++p;
        e = p;
        if (p < end) ++p;  // consume '\n'
    };
    if (buf.empty()) return PLVI_E_BADARG;
    const char *b, *e;
    next_line(b, e);
    {
        LineCursor c{b, e};
        h.k = (int)c.get_int();
        h.L = (int)c.get_int();
        h.scoring = (int)c.get_int();
        h.weighting = (int)c.get_int();
        if (h.k < 0 || h.k > 20 || h.L < 1 || h.L > 10 || h.scoring < 0 || h.scoring > 5 || h.weighting < 0 ||
            h.weighting > 3)
            return PLVI_E_BADARG;
    }
    h.parent.assign(1, 0);
    h.desc.assign(32, 0);
    h.weight.assign(1, 0.0);
    h.word.assign(1, 0u);
    h.nwords = 0;
    // `while(!f.eof()) getline(...)`: after a final '\n' one more (empty) line is read
    bool at_eof = p >= end && (buf.empty() || buf.back() != '\n');
    while (!at_eof) {
        const bool tail = p >= end;  // the empty read after the final newline
        next_line(b, e);
        at_eof = p >= end && (tail || buf.back() != '\n');
        if (tail && !emulate_tail) break;
        const int nid = (int)h.parent.size();
        LineCursor c{b, e};
        const long pid = c.get_int();
        if (pid < 0 || pid >= nid) return PLVI_E_BADARG;
        const long leaf = c.get_int();
        uint8_t d[32] = {0};  // reference: bytes of a failed FORB::fromString stay uninitialised
        for (int i = 0; i < 32; ++i) {
            const long v = c.get_int();
            if (!c.fail) d[i] = (uint8_t)v;
        }
        const double w = c.get_double();
        h.parent.push_back((int)pid);
        h.desc.insert(h.desc.end(), d, d + 32);
        h.weight.push_back(w);
        h.word.push_back(leaf > 0 ? (unsigned)h.nwords : 0u);
        if (leaf > 0) ++h.nwords;
        if (tail) break;
    }
    return PLVI_OK;
}

}  // namespace plvi

struct plvi_vocabulary {
    plvi::Vocab v;
};

using namespace plvi;

extern "C" int plvi_vocab_load_text(const char* path, int emulate_tail, int device, plvi_vocabulary** out) {
    if (!path || !out) return PLVI_E_BADARG;
    *out = nullptr;
    VocabHost h;
    int rc = load_text(path, emulate_tail, h);
    if (rc) return rc;
    auto v = std::make_unique<plvi_vocabulary>();
    rc = v->v.build(h, device);
    if (rc) return rc;
    *out = v.release();
    return PLVI_OK;
}

extern "C" int plvi_vocab_create(int k, int L, int scoring, int weighting, int n_nodes, const int* parent,
                                 const uint8_t* is_leaf, const uint8_t* desc, const double* weight, int device,
                                 plvi_vocabulary** out) {
    if (!out || n_nodes < 0 || (n_nodes > 0 && (!parent || !is_leaf || !desc || !weight))) return PLVI_E_BADARG;
    if (scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3 || L < 1) return PLVI_E_BADARG;
    *out = nullptr;
    VocabHost h;
    h.k = k; h.L = L; h.scoring = scoring; h.weighting = weighting;
    h.parent.assign(1, 0);
    h.desc.assign(32, 0);
    h.weight.assign(1, 0.0);
    h.word.assign(1, 0u);
    for (int i = 0; i < n_nodes; ++i) {
        if (parent[i] < 0 || parent[i] > i) return PLVI_E_BADARG;  // node i+1's parent precedes it
        h.parent.push_back(parent[i]);
        h.desc.insert(h.desc.end(), desc + (size_t)32 * i, desc + (size_t)32 * (i + 1));
        h.weight.push_back(weight[i]);
        h.word.push_back(is_leaf[i] ? (unsigned)h.nwords : 0u);
        if (is_leaf[i]) ++h.nwords;
    }
    auto v = std::make_unique<plvi_vocabulary>();
    int rc = v->v.build(h, device);
    if (rc) return rc;
    *out = v.release();
    return PLVI_OK;
}

extern "C" int plvi_vocab_destroy(plvi_vocabulary* h) {
    if (!h) return PLVI_E_BADARG;
    (void)hipSetDevice(h->v.device);
    (void)hipStreamSynchronize(h->v.stream);
    delete h;
    return PLVI_OK;
}

extern "C" int plvi_vocab_info(plvi_vocabulary* h, int* info) {
    if (!h || !info) return PLVI_E_BADARG;
    const Vocab& v = h->v;
    info[0] = v.k; info[1] = v.L; info[2] = v.scoring; info[3] = v.weighting;
    info[4] = v.nNodes; info[5] = v.nWords;
    return PLVI_OK;
}

extern "C" int plvi_vocab_transform_batch(plvi_vocabulary* h, const uint8_t* d_desc, const int* d_count, int cap,
                                          int n_frames, int levelsup, unsigned* d_bow_word, double* d_bow_value,
                                          int* d_bow_n, unsigned* d_fv_node, int* d_fv_off, unsigned* d_fv_idx,
                                          int* d_fv_n, unsigned* d_feat_word, unsigned* d_feat_nid, void* stream) {
    if (!h || cap < 1 || n_frames < 0) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    const Vocab& v = h->v;
    PLVI_CHECK(hipSetDevice(v.device));
    hipStream_t st = stream ? (hipStream_t)stream : v.stream;
    if (v.nWords == 0) {  // empty(): BowVector and FeatureVector stay cleared (:1134-1137)
        PLVI_CHECK(hipMemsetAsync(d_bow_n, 0, sizeof(int) * n_frames, st));
        PLVI_CHECK(hipMemsetAsync(d_fv_n, 0, sizeof(int) * n_frames, st));
        PLVI_CHECK(hipMemsetAsync(d_fv_off, 0, sizeof(int) * (size_t)n_frames * (cap + 1), st));
        return PLVI_OK;
    }
    const int P = bow_pow2(cap);
    const size_t smem = bow_smem(P);
    if (!lds_fits<bow_transform_kernel>(smem)) return PLVI_E_CAPACITY;
    PLVI_CHECK(hipFuncSetAttribute((const void*)bow_transform_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)smem));
    const int must = v.scoring != 5, l2 = v.scoring == 1, tf = v.weighting == 0 || v.weighting == 1;
    hipLaunchKernelGGL(bow_transform_kernel, dim3(n_frames), dim3(kBowThreads), smem, st, v.dev(), v.L, levelsup,
                       must, l2, tf, d_desc, d_count, cap, P, d_bow_word, d_bow_value, d_bow_n, d_fv_node, d_fv_off,
                       d_fv_idx, d_fv_n, d_feat_word, d_feat_nid, v.err.as<int>());
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// transform(features, BowVector&, FeatureVector&, levelsup) for one frame
// from host memory, synchronous.  Outputs are n-capacity arrays; fv_off has
// n + 1 entries.
extern "C" int plvi_vocab_transform(plvi_vocabulary* h, const uint8_t* desc, int n, int levelsup,
                                    unsigned* bow_word, double* bow_value, int* bow_n, unsigned* fv_node, int* fv_off,
                                    unsigned* fv_idx, int* fv_n) {
    if (!h || n < 0 || (n > 0 && !desc) || !bow_n || !fv_n) return PLVI_E_BADARG;
    *bow_n = 0;
    *fv_n = 0;
    if (fv_off) fv_off[0] = 0;
    const Vocab& v = h->v;
    if (n == 0 || v.nWords == 0) return PLVI_OK;
    PLVI_CHECK(hipSetDevice(v.device));
    const int cap = n;
    DevBuf d;
    const size_t oD = 0, oC = (size_t)32 * cap, oBW = oC + 16, oBV = oBW + ((4 * (size_t)cap + 15) & ~size_t(15));
    const size_t oBN = oBV + 8 * (size_t)cap, oFN = oBN + 16, oFO = oFN + ((4 * (size_t)cap + 15) & ~size_t(15));
    const size_t oFI = oFO + ((4 * (size_t)(cap + 1) + 15) & ~size_t(15)), oFC = oFI + ((4 * (size_t)cap + 15) & ~size_t(15));
    if (d.alloc(oFC + 16)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    PLVI_CHECK(hipMemcpy(B + oD, desc, (size_t)32 * n, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(B + oC, &n, sizeof(int), hipMemcpyHostToDevice));
    int rc = plvi_vocab_transform_batch(h, B + oD, (const int*)(B + oC), cap, 1, levelsup, (unsigned*)(B + oBW),
                                        (double*)(B + oBV), (int*)(B + oBN), (unsigned*)(B + oFN), (int*)(B + oFO),
                                        (unsigned*)(B + oFI), (int*)(B + oFC), nullptr, nullptr, v.stream);
    if (rc) return rc;
    PLVI_CHECK(hipStreamSynchronize(v.stream));
    int errv = 0, nb = 0, nf = 0;
    PLVI_CHECK(hipMemcpy(&errv, v.err.p, sizeof(int), hipMemcpyDeviceToHost));
    if (errv) {
        PLVI_CHECK(hipMemset(v.err.p, 0, sizeof(int)));
        return PLVI_E_OVERFLOW;
    }
    PLVI_CHECK(hipMemcpy(&nb, B + oBN, sizeof(int), hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(&nf, B + oFC, sizeof(int), hipMemcpyDeviceToHost));
    *bow_n = nb;
    *fv_n = nf;
    if (bow_word) PLVI_CHECK(hipMemcpy(bow_word, B + oBW, 4 * (size_t)nb, hipMemcpyDeviceToHost));
    if (bow_value) PLVI_CHECK(hipMemcpy(bow_value, B + oBV, 8 * (size_t)nb, hipMemcpyDeviceToHost));
    if (fv_node) PLVI_CHECK(hipMemcpy(fv_node, B + oFN, 4 * (size_t)nf, hipMemcpyDeviceToHost));
    if (fv_off) PLVI_CHECK(hipMemcpy(fv_off, B + oFO, 4 * (size_t)(nf + 1), hipMemcpyDeviceToHost));
    int m = 0;
    if (fv_off) m = fv_off[nf];
    else PLVI_CHECK(hipMemcpy(&m, B + oFO + 4 * (size_t)nf, sizeof(int), hipMemcpyDeviceToHost));
    if (fv_idx) PLVI_CHECK(hipMemcpy(fv_idx, B + oFI, 4 * (size_t)m, hipMemcpyDeviceToHost));
    return PLVI_OK;
}

// Per-descriptor descent results (word id, NodeId at level L - levelsup) of
// one frame, synchronous (diagnostics and tests).
extern "C" int plvi_vocab_transform_features(plvi_vocabulary* h, const uint8_t* desc, int n, int levelsup,
                                             unsigned* word, unsigned* nid) {
    if (!h || n < 0 || (n > 0 && (!desc || !word || !nid))) return PLVI_E_BADARG;
    if (n == 0) return PLVI_OK;
    const Vocab& v = h->v;
    PLVI_CHECK(hipSetDevice(v.device));
    const size_t c4 = ((4 * (size_t)n + 15) & ~size_t(15));
    DevBuf d;
    if (d.alloc((size_t)32 * n + 16 + c4 * 7 + 8 * (size_t)n + 64)) return PLVI_E_HIP;
    uint8_t* B = d.as<uint8_t>();
    uint8_t* dd = B;
    int* dc = (int*)(B + (size_t)32 * n);
    unsigned* w = (unsigned*)(B + (size_t)32 * n + 16);
    unsigned* ni = (unsigned*)((uint8_t*)w + c4);
    unsigned* bw = (unsigned*)((uint8_t*)ni + c4);
    unsigned* fn = (unsigned*)((uint8_t*)bw + c4);
    unsigned* fi = (unsigned*)((uint8_t*)fn + c4);
    int* fo = (int*)((uint8_t*)fi + c4);
    int* cnts = (int*)((uint8_t*)fo + c4 + 16);
    double* bv = (double*)((uint8_t*)cnts + 16);
    PLVI_CHECK(hipMemcpy(dd, desc, (size_t)32 * n, hipMemcpyHostToDevice));
    PLVI_CHECK(hipMemcpy(dc, &n, sizeof(int), hipMemcpyHostToDevice));
    int rc = plvi_vocab_transform_batch(h, dd, dc, n, 1, levelsup, bw, bv, cnts, fn, fo, fi, cnts + 1, w, ni, v.stream);
    if (rc) return rc;
    PLVI_CHECK(hipStreamSynchronize(v.stream));
    PLVI_CHECK(hipMemcpy(word, w, 4 * (size_t)n, hipMemcpyDeviceToHost));
    PLVI_CHECK(hipMemcpy(nid, ni, 4 * (size_t)n, hipMemcpyDeviceToHost));
    return PLVI_OK;
}
