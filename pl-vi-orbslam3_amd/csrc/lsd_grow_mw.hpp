// lsd_grow_mw.hpp — LK3 for small batches (latency): flsd's region loop
// (lsd.cpp:476-533, region_grow :635-686) with SEVERAL regions of ONE frame
// growing at once, bit-exact with the sequential raster-order loop.
//
// One workgroup of NW waves per (frame, octave).  Seeds are resolved in
// raster order by a single "walk" (the lock holder); the other waves grow
// regions speculatively ahead of it:
//
//  * A region grown from seed s only depends on the USED state of the pixels
//    it tests.  Every defined pixel before s (raster order) is USED when flsd
//    reaches s, so a speculative region treats them as USED; for pixels after
//    s it sees the committed bitmap C (regions already walked) and its own
//    marks.  Earlier regions can only ADD USED pixels, so the region is exactly
//    the reference's iff none of the pixels it accepted is in C when the walk
//    reaches s (validation); otherwise the walker regrows it exactly (all
//    earlier regions are then committed).
//  * The walk goes over the pixels after the last committed seed: committed /
//    NOTDEF pixels (C) are skipped, "trivial" seeds (no forward neighbour
//    aligned with the seed angle: a static property, the region is the seed
//    alone, T) are committed in place, any other seed takes its speculative
//    region (validated) or is grown exactly by the walker when no wave has it.
//  * Waves 1..NW-1 pick the next seed after a shared cursor that is neither
//    in C, T nor claimed by any region so far (H, a hint: skipped seeds are
//    found by the walk) and grow it into their own LDS queue; a finished
//    region is copied into a free slot of a shared pool (first kMwSP points in
//    LDS, the rest in global memory).  Wave 0 is the walker.  A speculative
//    region whose seed the walk passed is dropped.
//
// LDS: C, T, H (whole frame, one bit per pixel), per wave an own-mark window
// of kMwRB rows from the seed row (rows below it spill to a global bitmap)
// and a growth queue (spill to global), the slot pool, the dispatch log (the
// speculative seeds in increasing order with their slots).  Commit order =
// raster seed order, so the region list handed to lsd_rect_lanes_kernel is the
// sequential kernel's.
//
// ---------------------------------------------------------------------------
#pragma once

namespace plvi {

constexpr int kMwRB = 32;           // own-mark window rows
constexpr int kMwGQ = 256;          // LDS growth-queue entries per wave
constexpr int kMwGSpill = 4096;     // global growth-queue entries per speculative wave
constexpr int kMwSP = 64;           // points of a slot kept in LDS
constexpr int kMwSlotSpill = 2048;  // points of a slot beyond kMwSP (global)
constexpr int kMwMaxSlots = 128;
constexpr int kMwLog = 256;         // dispatch log entries (seed order)
#ifndef PLVI_MW_LOOK
#define PLVI_MW_LOOK 16
#endif
// wave priorities (s_setprio) of the walker and the speculative growers: the
// walk is the critical path, the growers fill the issue slots it leaves
#ifndef PLVI_MW_WALKER_PRIO
#define PLVI_MW_WALKER_PRIO 3
#endif
#ifndef PLVI_MW_GROWER_PRIO
#define PLVI_MW_GROWER_PRIO 1
#endif
#ifndef PLVI_MW_CHECKER_PRIO
#define PLVI_MW_CHECKER_PRIO 2
#endif
constexpr int kMwLook = PLVI_MW_LOOK;  // dispatch-log entries ahead of the walk that growers revalidate (0 = off)
// diagnostic variant (tools/build_variant.sh ... -DPLVI_MW_DIAG=1): 32
// counters per task instead of 16 and a commit-epoch map (see the stat list)
#ifndef PLVI_MW_DIAG
#define PLVI_MW_DIAG 0
#endif
constexpr int kMwStatN = PLVI_MW_DIAG ? 32 : 16;

// slot states; COMMITTED: validated and committed, a grower still copies
// its points out (regions of more than kMwSP points); WALKING: the walker
// validates it (claimed from DONE by compare-and-swap, like a grower's
// revalidation, which holds it as GROWING)
// DIRTY: grown, and found invalid by the checker wave (a pixel of it has since
// been committed); the walker regrows it without validating, a grower regrows
// it ahead of the walk
enum : int { kMwFree = 0, kMwGrowing = 1, kMwDone = 2, kMwCommitted = 3, kMwCopying = 4, kMwWalking = 5, kMwDirty = 6 };
// commit-driven revalidation: wave 1 is a checker that, after every commit,
// tests every grown region of the dispatch log ahead of the walk against the
// committed bitmap and marks the invalid ones DIRTY; growers regrow DIRTY
// regions (the earliest first) before growing new ones.  0: the r05 scheme
// (idle growers recheck the first kMwLook log entries after the walk).
#ifndef PLVI_MW_CHECKER
#define PLVI_MW_CHECKER 1
#endif
constexpr bool kMwChecker = PLVI_MW_CHECKER != 0;

struct MwSlot {
    int seed;   // bit index y * (wpr * 32) + x
    int state;  // kMw*
    int n;      // region size
    float deg;  // final region angle (float degrees)
    int ovf;    // queue overflow: the walker regrows it
    int out;    // COMMITTED: offset of its points in the task's point list
    int chk;    // ctl->ncommit when the region was last grown / found valid
};
constexpr int kMwSlotBytes = sizeof(MwSlot) + 4 * kMwSP;
// control block (LDS)
struct MwCtl {
    int lock, dlock, head, cursor, finished, npts, nout, overflow;
    int dlog_n, wptr, ncommit, pad1;  // dispatch log: entries appended / next entry the walk examines;
                                      // regions committed so far (revalidation epoch)
    int stat[kMwStatN];  // [0] dispatched [1] dropped [2] regrown [3] exact (undispatched) [4] trivial [5] committed
                   // speculative [6] walk cycles [7] walker growth cycles [8] walk entries [9] blocked on a
                   // growing head [10] kernel cycles (wave 0) [11] speculative growth cycles (sum over waves)
                   // [12] unused [13] blocks (completed regions) [14] block setup cycles / 16
                   // [15] block round cycles / 16
                   // PLVI_MW_DIAG: [16]/[17] walker waits on a revalidation regrowth (count / cycles)
                   // [18]/[19] waits on a first growth [20..25] walker regrowths by distance (in commits)
                   // from the commit that invalidated them: 1, 2, 3-4, 5-8, 9-16, >16 [26] sum of their
                   // check lag (commits since last check) [27] of them last grown by a revalidation
                   // [28] revalidation checks (r05 scheme) / regions the checker marked DIRTY [29] grower
                   // regrowths [30] sum of waited-on region
                   // sizes [31] sum of (dispatch log entries ahead of the walk) at its waits
};

typedef MwSlot __attribute__((address_space(3))) lds_slot;
typedef MwCtl __attribute__((address_space(3))) lds_ctl;

struct MwQueue {
    lds_u32* lq;
    int lcap;
    unsigned* gq;
    int gcap;
};

struct MwEnv {
    const float* P;    // angle plane (degrees, NOTDEF = -1024)
    const float2* SC;  // cosf / sinf of float(angle)
    lds_u32* C;        // committed or NOTDEF
    lds_u32* T;        // trivial seeds
    lds_u32* H;        // claimed by some region (dispatch hint)
    lds_u32* own;      // this wave's own-mark window (RB rows x wpr)
    unsigned* ownG;    // this wave's own-mark spill (sh x wpr)
    lds_ctl* ctl;
    int* epoch;  // PLVI_MW_DIAG: commit index of every committed pixel (bit index), else null
    int sw, sh, wpr, rowbits;  // rowbits = wpr * 32
    float pdeg;
    double prec;
};

// LDS hand-offs between the waves of the workgroup stay inside the HIP
// memory model: a wave publishes data (slot records, dispatch-log entries,
// the walk position) with a workgroup-scope RELEASE store of a flag and the
// consumer reads the flag with an ACQUIRE load; locks are taken with an
// acquire compare-and-swap and released with a release store.  Locations
// several waves update concurrently (the C / H bitmaps, slot states scanned
// as hints) are only accessed atomically -- relaxed where a later acquire or
// a lock re-checks the value.  On gfx950 (no threadgroup split) a
// workgroup-scope release or acquire on LDS costs an s_waitcnt lgkmcnt(0).
__device__ __forceinline__ unsigned mw_peek(const lds_u32* p) {
    return __hip_atomic_load(const_cast<lds_u32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int mw_peek(const lds_i32* p) {
    return __hip_atomic_load(const_cast<lds_i32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned mw_word(const lds_u32* B, int wpr, int x, int y) {
    return mw_peek(B + y * wpr + (x >> 5));
}
__device__ __forceinline__ bool mw_bit(const lds_u32* B, int wpr, int x, int y) {
    return (mw_word(B, wpr, x, y) >> (x & 31)) & 1u;
}
__device__ __forceinline__ void mw_or(lds_u32* B, int wpr, int x, int y) {
    __atomic_fetch_or(&B[y * wpr + (x >> 5)], 1u << (x & 31), __ATOMIC_RELAXED);
}
__device__ __forceinline__ bool mw_own_get(const MwEnv& E, int x, int y, int sy) {
    const bool inwin = y < sy + kMwRB;
    const int yy = inwin ? y - sy : 0;
    unsigned v = E.own[yy * E.wpr + (x >> 5)];
    if (__builtin_expect(!inwin, 0)) v = gload_l2(E.ownG + (size_t)y * E.wpr + (x >> 5));
    return (v >> (x & 31)) & 1u;
}
__device__ __forceinline__ void mw_own_set(const MwEnv& E, int x, int y, int sy) {
    const unsigned b = 1u << (x & 31);
    if (__builtin_expect(y < sy + kMwRB, 1)) __atomic_fetch_or(&E.own[(y - sy) * E.wpr + (x >> 5)], b, __ATOMIC_RELAXED);
    else __hip_atomic_fetch_or(E.ownG + (size_t)y * E.wpr + (x >> 5), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned mw_qget(const MwQueue& Q, int i) {
    if (__builtin_expect(i < Q.lcap, 1)) return Q.lq[i];
    return gload_l2(Q.gq + (i - Q.lcap));
}
__device__ __forceinline__ void mw_qput(const MwQueue& Q, int i, unsigned v) {
    if (__builtin_expect(i < Q.lcap, 1)) Q.lq[i] = v;
    else gstore_l2(Q.gq + (i - Q.lcap), v);
}
__device__ __forceinline__ void mw_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// acquire load of a flag (pairs with mw_lds_store)
__device__ __forceinline__ int mw_lds_load(lds_i32* p) {
    const int v = __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return v;
}
// release store of a flag: everything this wave wrote before it (after a
// mw_wave_sync when other lanes wrote) is visible to an acquiring wave
__device__ __forceinline__ void mw_lds_store(lds_i32* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// compare-and-swap of a slot state / lock word: acquire on success
__device__ __forceinline__ bool mw_lds_cas(lds_i32* p, int expected, int desired) {
    return __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void mw_stat(lds_ctl* c, int i, int v) {
    __hip_atomic_fetch_add(&c->stat[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wave-uniform try-lock (lane 0 does the CAS)
__device__ __forceinline__ bool mw_try_lock(lds_i32* l, int lane) {
    int got = 0;
    if (lane == 0) got = mw_lds_cas(l, 0, 1) ? 1 : 0;
    got = __builtin_amdgcn_readfirstlane(got);
    return got != 0;
}
__device__ __forceinline__ void mw_unlock(lds_i32* l, int lane) {
    mw_wave_sync();
    if (lane == 0) mw_lds_store(l, 0);
}

// Grow the region of seed (sx, sy) into Q (region_grow, lsd.cpp:635-686).
// SPEC: abandon when the walk passes the seed.  Returns 0 = grown, 1 =
// abandoned, 2 = queue overflow; n = points in Q (own marks set for them).
template <bool SPEC, bool STATS = false>
__device__ int mw_grow(const MwEnv& E, int sx, int sy, const MwQueue& Q, int& n_out, float& deg_out, bool& spilled,
                       int lane) {
    unsigned long long c_setup = 0, c_round = 0, n_blk = 0;
    const int sw = E.sw, sh = E.sh;
    const int seedb = sy * E.rowbits + sx;
    const float pdeg = E.pdeg;
    const double prec = E.prec;
    const int bp = lane / 9, bk = lane % 9;
    const int kdx = bk % 3 - 1, kdy = bk / 3 - 1;
    float reg_deg = E.P[(size_t)sy * sw + sx];
    // the seed direction (lsd.cpp:648-649) is computed in the first block,
    // while its neighbourhood loads are in flight
    float sumdx = 0.f, sumdy = 0.f;
    if (lane == 0) {
        mw_own_set(E, sx, sy, sy);
        mw_or(E.H, E.wpr, sx, sy);
        Q.lq[0] = (unsigned)sx | ((unsigned)sy << 16);
    }
    mw_wave_sync();
    spilled = false;
    int reg_size = 1;
    const int cap = Q.lcap + Q.gcap;
    for (int i = 0; i < reg_size;) {
        // the walk position is read at the top of the block (relaxed: a hint)
        // and tested once the block's loads are in flight, instead of an
        // acquire load that stalls the block first (6.40 -> 6.27 ms at one
        // frame, profiles/r04/mw_helpers_ab.txt)
        const int hd0 = SPEC ? mw_peek(&E.ctl->head) : 0;
        const unsigned long long tb0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
        const int nb = min(7, reg_size - i);
        const bool active = lane < 9 * nb;
        // the block's queue points: one LDS read (inactive lanes read entry i),
        // the global part only once the queue has passed its LDS entries
        unsigned pv;
        if (i + 7 <= Q.lcap) {
            const unsigned v = Q.lq[i + (active ? bp : 0)];
            pv = active ? v : 0u;
        } else {
            pv = active ? mw_qget(Q, i + bp) : 0u;
        }
        const int px = (int)(pv & 0xffffu), py = (int)(pv >> 16);
        const int nx = px + kdx, ny = py + kdy;
        // pixels before the seed in raster order are USED when flsd reaches it
        // in the frame and at or after the seed in raster order
        const bool valid = active & ((unsigned)nx < (unsigned)sw) & (ny < sh) & (ny * sw + nx >= sy * sw + sx);
        float deg = kNotdefF, cc = 0.f, ss = 0.f;
        if (valid) {
            const float2 cs2 = E.SC[(size_t)ny * sw + nx];
            deg = E.P[(size_t)ny * sw + nx];
            cc = cs2.x;
            ss = cs2.y;
        }
        if (i == 0) {
            double ds, dc;
            plvi_sincos((double)reg_deg * kD2R, &ds, &dc);
            sumdx = (float)dc;
            sumdy = (float)ds;
        }
        const unsigned long long dup = dup_lanes(pv, nb, bp, nx, ny);
        if (SPEC) {
            if (hd0 > seedb) {
                n_out = reg_size;
                deg_out = reg_deg;
                return 1;
            }
            // the walk waits on this region: let it win the SIMD's issue
            // arbitration against the other growers until it is done
            if (hd0 == seedb) __builtin_amdgcn_s_setprio(3);
            else __builtin_amdgcn_s_setprio(PLVI_MW_GROWER_PRIO);
        }
        // own marks and the committed bitmap, read once per block (within the
        // block a lane's pixel only changes through an earlier lane's commit
        // of the same pixel: dup / Ccum)
        // committed bit and own mark, read for every lane (clamped), the own
        // marks below the window from the global spill (rare, uniform branch)
        const int ux = valid ? nx : sx, uy = valid ? ny : sy;
        const unsigned cw = mw_word(E.C, E.wpr, ux, uy);
        const bool ofar = uy >= sy + kMwRB;
        unsigned ow = E.own[(ofar ? 0 : uy - sy) * E.wpr + (ux >> 5)];
        if (__builtin_expect(ballot(valid && ofar) != 0ull, 0)) {
            if (ofar) ow = gload_l2(E.ownG + (size_t)uy * E.wpr + (ux >> 5));
        }
        const bool live0 = valid & (deg != kNotdefF) & ((((cw | ow) >> (ux & 31)) & 1u) == 0u);
        unsigned long long tb1 = 0;
        if (STATS) {
            tb1 = __builtin_amdgcn_s_memtime();
            c_setup += tb1 - tb0;
            ++n_blk;
        }
        unsigned long long Ccum = 0;
        int start = 0;
        while (start < 9 * nb) {
            const unsigned long long fromStart = ~0ull << start;
            const bool candl = (lane >= start) & live0 & ((dup & Ccum) == 0ull);
            const bool alg = is_aligned_fast(deg, reg_deg, pdeg, prec);
            const bool al = candl & alg;
            const bool acc = al & ((dup & fromStart) == 0ull);
            const unsigned long long A = ballot(acc);
            if (!A) break;
            const int cl = mbcnt64(A);
            float sx2 = sumdx, sy2 = sumdy, pfx = sumdx, pfy = sumdy;
            int t = 0;
            for (unsigned long long mm = A; mm; mm &= mm - 1) {
                const int bl = __ffsll((long long)mm) - 1;
                sx2 += readlane_f(cc, bl);
                sy2 += readlane_f(ss, bl);
                ++t;
                if (cl == t) {
                    pfx = sx2;
                    pfy = sy2;
                }
            }
            const float tha = plvi_fast_atan2(pfy, pfx);
            const float th = cl > 0 ? tha : reg_deg;
            const bool alth = is_aligned_fast(deg, th, pdeg, prec);
            const bool al2 = candl & ((dup & A) == 0ull) & alth;
            const unsigned long long mism = ballot(al2 != acc) & fromStart;
            const int ls = mism ? __ffsll((long long)mism) - 1 : 63;
            const unsigned long long Cm = A & ((1ull << ls) - 1ull);
            const int nc = __popcll(Cm);
            start = mism ? ls : 9 * nb;
            if (nc > 0) {
                if (reg_size + nc > cap) {  // the slot queue is full: the walker regrows it exactly
                    n_out = reg_size;
                    deg_out = reg_deg;
                    return 2;
                }
                Ccum |= Cm;
                const bool mine = (Cm >> lane) & 1ull;
                const bool sp = ballot(mine && ny >= sy + kMwRB) != 0ull;
                spilled |= sp;
                if (__builtin_expect(!sp && reg_size + nc <= Q.lcap, 1)) {
                    // own mark, claim hint and queue entry in LDS
                    if (mine) {
                        const unsigned b = 1u << (nx & 31);
                        __atomic_fetch_or(&E.own[(ny - sy) * E.wpr + (nx >> 5)], b, __ATOMIC_RELAXED);
                        __atomic_fetch_or(&E.H[ny * E.wpr + (nx >> 5)], b, __ATOMIC_RELAXED);
                        Q.lq[reg_size + mbcnt64(Cm)] = (unsigned)nx | ((unsigned)ny << 16);
                    }
                } else {
                    if (mine) {
                        int sx_ = nx, sy_ = ny;  // opaque: keep the slow path's addressing here
                        asm volatile("" : "+v"(sx_), "+v"(sy_));
                        mw_own_set(E, sx_, sy_, sy);
                        mw_or(E.H, E.wpr, sx_, sy_);
                        mw_qput(Q, reg_size + mbcnt64(Cm), (unsigned)sx_ | ((unsigned)sy_ << 16));
                    }
                    vm_drain();
                }
                reg_size += nc;
                sumdx = readlane_f(pfx, ls);
                sumdy = readlane_f(pfy, ls);
                reg_deg = readlane_f(th, ls);
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (STATS) c_round += __builtin_amdgcn_s_memtime() - tb1;
        i += nb;
    }
    if (STATS && lane == 0) {
        mw_stat(E.ctl, 13, (int)n_blk);
        mw_stat(E.ctl, 14, (int)(c_setup >> 4));
        mw_stat(E.ctl, 15, (int)(c_round >> 4));
    }
    n_out = reg_size;
    deg_out = reg_deg;
    return 0;
}

// Clear the own marks of a region grown from row sy (n points in Q).
__device__ __forceinline__ void mw_own_clear(const MwEnv& E, int sy, const MwQueue& Q, int n, bool spilled, int lane) {
    mw_wave_sync();
    for (int k = lane; k < kMwRB * E.wpr; k += 64) E.own[k] = 0u;
    if (spilled) {
        for (int j = lane; j < n; j += 64) {
            const unsigned v = mw_qget(Q, j);
            const int x = (int)(v & 0xffffu), y = (int)(v >> 16);
            if (y >= sy + kMwRB) gstore_l2(E.ownG + (size_t)y * E.wpr + (x >> 5), 0u);
        }
        vm_drain();
    }
    mw_wave_sync();
}

// A slot's points: the first kMwSP in LDS after its header, the rest in
// global memory.
__device__ __forceinline__ MwQueue mw_slot_queue(lds_u8* pool, unsigned* slotspill, int si) {
    return MwQueue{(lds_u32*)(pool + (size_t)si * kMwSlotBytes + sizeof(MwSlot)), kMwSP,
                   slotspill + (size_t)si * kMwSlotSpill, kMwSlotSpill};
}
__device__ __forceinline__ lds_slot* mw_slot(lds_u8* pool, int si) { return (lds_slot*)(pool + (size_t)si * kMwSlotBytes); }

// The walk (wave 0): resolve seeds from ctl->head in raster order.  Returns
// the slot whose region the next seed waits for, or -1 once every seed is
// resolved.  The dispatch log lists the speculative seeds in increasing
// order, so the region of seed q (if any) is found by advancing one pointer.
template <bool STATS>
__device__ int mw_walk(const MwEnv& E, lds_u8* pool, lds_i32* dlog, unsigned* slotspill, const MwQueue& XQ,
                       int min_reg, LsdRegion* outR, unsigned* outP, int lane) {
    lds_ctl* ctl = E.ctl;
    const int nwords = E.sh * E.wpr;
    const int rowbits = E.rowbits;
    int head = ctl->head;
    int wp = ctl->wptr;
    int blocked = -1;
    while (true) {
        // next non-trivial unresolved pixel >= head.  The trivial seeds before
        // it (one-pixel regions < min_reg_size; every earlier region is
        // committed) are committed in place -- the words wholly before it in
        // one wave-parallel pass, 64 words at a time.  Only the walker writes C.
        int w = head >> 5;
        if (w >= nwords) break;
        unsigned cw = mw_peek(E.C + w), tw = E.T[w];  // T is static after the set-up
        unsigned m = ~cw & (~0u << (head & 31));
        unsigned nt = m & ~tw;
        if (!nt) {
            if ((m & tw) && lane == 0) {
                __atomic_fetch_or(&E.C[w], m & tw, __ATOMIC_RELAXED);
                if (STATS) mw_stat(ctl, 4, __popc(m & tw));
            }
            int found = -1;
            for (int w0 = w + 1; w0 < nwords && found < 0; w0 += 64) {
                const int ww = w0 + lane;
                const bool in = ww < nwords;
                const unsigned c = in ? mw_peek(E.C + ww) : ~0u, t = in ? E.T[ww] : 0u;
                const unsigned long long b = ballot((~c & ~t) != 0u);
                const int fl = b ? __ffsll((long long)b) - 1 : 64;
                const unsigned triv = ~c & t;
                if (lane < fl && triv) {
                    __atomic_fetch_or(&E.C[ww], triv, __ATOMIC_RELAXED);
                    if (STATS) mw_stat(ctl, 4, __popc(triv));
                }
                if (b) found = w0 + fl;
            }
            if (found < 0) {
                head = nwords * 32;
                break;
            }
            w = found;
            cw = mw_peek(E.C + w);
            tw = E.T[w];
            m = ~cw;
            nt = m & ~tw;
        }
        // trivial seeds before the first non-trivial one of word w
        const unsigned run = m & tw & ((nt & (0u - nt)) - 1u);
        if (run && lane == 0) {
            __atomic_fetch_or(&E.C[w], run, __ATOMIC_RELAXED);
            if (STATS) mw_stat(ctl, 4, __popc(run));
        }
        const int q = w * 32 + (__ffs((int)nt) - 1);
        head = q;
        // the speculative region of seed q, if one was dispatched
        const int dn = mw_lds_load(&ctl->dlog_n);
        while (wp < dn && dlog[2 * (wp & (kMwLog - 1))] < q) ++wp;
        int si = -1;
        bool fromLog = false;
        if (wp < dn && dlog[2 * (wp & (kMwLog - 1))] == q) {
            si = dlog[2 * (wp & (kMwLog - 1)) + 1];
            fromLog = true;
        }
        lds_slot* S = si >= 0 ? mw_slot(pool, si) : nullptr;
        int sst = si >= 0 ? mw_lds_load(&S->state) : kMwFree;
        bool dirty = false;  // found invalid by the checker: regrow without validating
        if (sst == kMwDone || sst == kMwDirty) {
            // claim it against a grower's revalidation / regrowth (and, for a
            // DONE region, the checker marking it DIRTY meanwhile: one retry)
            int got = 0;
            if (lane == 0) {
                got = mw_lds_cas(&S->state, sst, kMwWalking) ? sst : 0;
                if (!got && sst == kMwDone) got = mw_lds_cas(&S->state, kMwDirty, kMwWalking) ? kMwDirty : 0;
            }
            got = __builtin_amdgcn_readfirstlane(got);
            if (!got) sst = kMwGrowing;
            else {
                dirty = got == kMwDirty;
                sst = kMwDone;
            }
        }
        if (sst == kMwGrowing) {  // wait for it
            if (STATS && lane == 0) mw_stat(ctl, 9, 1);
#if PLVI_MW_DIAG
            if (STATS && lane == 0) mw_stat(ctl, 31, dn - wp);
#endif
            blocked = si;
            break;
        }
        if (fromLog) ++wp;
        int n = 0;
        bool done = false;
        if (sst == kMwDone) {
            // (now WALKING) validate (none of its pixels committed by an earlier region) and
            // commit; the first kMwSP points stay in registers
            n = S->n;
            const float deg = S->deg;
            const MwQueue Q = mw_slot_queue(pool, slotspill, si);
            bool valid = S->ovf == 0 && !dirty;
            unsigned v0 = 0u;
            if (valid) {
                bool bad = false;
                if (lane < n) {
                    v0 = Q.lq[lane];
                    bad = mw_bit(E.C, E.wpr, (int)(v0 & 0xffffu), (int)(v0 >> 16));
                }
                for (int j = lane + 64; j < n; j += 64) {
                    const unsigned v = mw_qget(Q, j);
                    bad |= mw_bit(E.C, E.wpr, (int)(v & 0xffffu), (int)(v >> 16));
                }
                valid = ballot(bad) == 0ull;
#if PLVI_MW_DIAG
                if (STATS && !valid) {
                    // the earliest commit that took one of its pixels
                    int emin = 0x7fffffff;
                    for (int j = lane; j < n; j += 64) {
                        const unsigned v = mw_qget(Q, j);
                        const int x = (int)(v & 0xffffu), y = (int)(v >> 16);
                        if (mw_bit(E.C, E.wpr, x, y)) emin = min(emin, (int)gload_l2((unsigned*)E.epoch + y * rowbits + x));
                    }
                    for (int o = 32; o > 0; o >>= 1) emin = min(emin, __shfl_xor(emin, o));
                    if (lane == 0) {
                        const int nc = ctl->ncommit, d = nc - emin;
                        mw_stat(ctl, d <= 1 ? 20 : d == 2 ? 21 : d <= 4 ? 22 : d <= 8 ? 23 : d <= 16 ? 24 : 25, 1);
                        mw_stat(ctl, 26, nc - S->chk);
                        if (S->out == -2) mw_stat(ctl, 27, 1);
                    }
                }
#endif
            }
            if (valid) {
                if (lane < n) mw_or(E.C, E.wpr, (int)(v0 & 0xffffu), (int)(v0 >> 16));
                for (int j = lane + 64; j < n; j += 64) {
                    const unsigned v = mw_qget(Q, j);
                    mw_or(E.C, E.wpr, (int)(v & 0xffffu), (int)(v >> 16));
                }
#if PLVI_MW_DIAG
                if (STATS)
                    for (int j = lane; j < n; j += 64) {
                        const unsigned v = mw_qget(Q, j);
                        E.epoch[(int)(v >> 16) * rowbits + (int)(v & 0xffffu)] = ctl->ncommit;
                    }
#endif
                int st_next = kMwFree;
                if (n >= min_reg) {
                    const int nout = ctl->nout, npts = ctl->npts;
                    if (nout < kLsdRawCap) {
                        if (lane == 0) {
                            outR[nout] = LsdRegion{npts, n, (double)deg * kD2R};
                            ctl->npts = npts + n;
                            ctl->nout = nout + 1;
                            S->out = npts;
                        }
                        // up to 64 points now; longer regions are copied by a grower
                        if (n <= 64) {
                            if (lane < n) outP[npts + lane] = v0;
                        } else {
                            st_next = kMwCommitted;
                        }
                    } else if (lane == 0) {
                        ctl->overflow = 1;
                    }
                }
                if (STATS && lane == 0) mw_stat(ctl, 5, 1);
                mw_wave_sync();
                if (lane == 0) {
                    mw_lds_store(&ctl->ncommit, ctl->ncommit + 1);
                    mw_lds_store(&S->state, st_next);
                }
                done = true;
            } else {
                if (STATS && lane == 0) mw_stat(ctl, 2, 1);
                mw_wave_sync();
                if (lane == 0) mw_lds_store(&S->state, kMwFree);
            }
        }
        if (!done) {
            // exact growth: every earlier seed is committed
            bool spilled = false;
            float deg = 0.f;
            const int qx = q % rowbits, qy = q / rowbits;
            const unsigned long long tg0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
            mw_grow<false, STATS>(E, qx, qy, XQ, n, deg, spilled, lane);
            mw_own_clear(E, qy, XQ, n, spilled, lane);
            if (STATS && lane == 0) {
                mw_stat(ctl, 7, (int)(__builtin_amdgcn_s_memtime() - tg0));
                if (si < 0) mw_stat(ctl, 3, 1);
            }
            for (int j = lane; j < n; j += 64) {
                const unsigned v = mw_qget(XQ, j);
                mw_or(E.C, E.wpr, (int)(v & 0xffffu), (int)(v >> 16));
#if PLVI_MW_DIAG
                if (STATS) E.epoch[(int)(v >> 16) * rowbits + (int)(v & 0xffffu)] = ctl->ncommit;
#endif
            }
            mw_wave_sync();
            if (lane == 0) mw_lds_store(&ctl->ncommit, ctl->ncommit + 1);
            // region2rect input for lsd_rect_lanes_kernel (flsd :500-518 order)
            if (n >= min_reg) {
                const int nout = ctl->nout, npts = ctl->npts;
                if (nout < kLsdRawCap) {
                    for (int j = lane; j < n; j += 64) outP[npts + j] = mw_qget(XQ, j);
                    if (lane == 0) {
                        outR[nout] = LsdRegion{npts, n, (double)deg * kD2R};
                        ctl->npts = npts + n;
                        ctl->nout = nout + 1;
                    }
                } else if (lane == 0) {
                    ctl->overflow = 1;
                }
            }
            mw_wave_sync();
        }
        head = q + 1;
        if (lane == 0) {
            mw_lds_store(&ctl->wptr, wp);  // frees log entries for the dispatchers as the walk goes
            mw_lds_store(&ctl->head, head);
        }
    }
    if (lane == 0) {
        mw_lds_store(&ctl->wptr, wp);
        mw_lds_store(&ctl->head, head);
        if ((head >> 5) >= nwords) mw_lds_store(&ctl->finished, 1);
    }
    mw_wave_sync();
    return blocked;
}

// A free slot (FREE, or DONE with a seed the walk passed) and the next seed
// for a speculative region: the first pixel after the cursor (and the walk)
// that is neither committed / NOTDEF, trivial nor claimed; appended to the
// dispatch log with its slot.  Returns the seed (-1: none) and the slot.
template <bool STATS>
__device__ __forceinline__ int mw_dispatch(const MwEnv& E, lds_u8* pool, int nslots, lds_i32* dlog, int& slot,
                                           int lane) {
    lds_ctl* ctl = E.ctl;
    const int nwords = E.sh * E.wpr;
    const int dn = mw_peek(&ctl->dlog_n);  // written under dlock only (held)
    if (dn - mw_lds_load(&ctl->wptr) >= kMwLog - 1) return -1;  // log full: the walk is far behind
    const int head = mw_lds_load(&ctl->head);
    // a free slot (lanes scan the pool), claimed by compare-and-swap: growers
    // claim DIRTY slots without the dispatch lock, and a dead DIRTY slot (seed
    // passed by the walk) is also free here
    slot = -1;
    int st0 = kMwFree;
    for (int b0 = 0; b0 < nslots && slot < 0; b0 += 64) {
        const int si = b0 + lane;
        bool ok = false;
        int st = kMwFree;
        if (si < nslots) {
            lds_slot* S = mw_slot(pool, si);
            st = mw_lds_load(&S->state);
            ok = st == kMwFree || ((st == kMwDone || st == kMwDirty) && S->seed < head);
        }
        for (unsigned long long b = ballot(ok); b && slot < 0; b &= b - 1) {
            const int l = __ffsll((long long)b) - 1;
            const int c = b0 + l, stc = readlane_i(st, l);
            int got = 0;
            if (lane == 0) got = mw_lds_cas(&mw_slot(pool, c)->state, stc, kMwGrowing) ? 1 : 0;
            if (__builtin_amdgcn_readfirstlane(got)) {
                slot = c;
                st0 = stc;
            }
        }
    }
    if (slot < 0) return -1;
    // (no seed: the claimed slot goes back as FREE -- it was free or held a dead region)
    int cur = max(ctl->cursor, head);
    int w = cur >> 5;
    if (w >= nwords) {
        if (lane == 0) mw_lds_store(&mw_slot(pool, slot)->state, kMwFree);
        return -1;
    }
    unsigned m = ~(mw_peek(E.C + w) | E.T[w] | mw_peek(E.H + w)) & (~0u << (cur & 31));
    if (!m) {
        int found = -1;
        for (int w0 = w + 1; w0 < nwords && found < 0; w0 += 64) {
            const int ww = w0 + lane;
            const bool nz = ww < nwords && (mw_peek(E.C + ww) | E.T[ww] | mw_peek(E.H + ww)) != ~0u;
            const unsigned long long b = ballot(nz);
            if (b) found = w0 + __ffsll((long long)b) - 1;
        }
        if (found < 0) {
            if (lane == 0) {
                ctl->cursor = nwords * 32;
                mw_lds_store(&mw_slot(pool, slot)->state, kMwFree);
            }
            return -1;
        }
        w = found;
        m = ~(mw_peek(E.C + w) | E.T[w] | mw_peek(E.H + w));
    }
    const int q = w * 32 + (__ffs((int)m) - 1);
    if (lane == 0) {
        lds_slot* S = mw_slot(pool, slot);
        if (STATS && (st0 == kMwDone || st0 == kMwDirty)) mw_stat(ctl, 1, 1);  // a passed region, dropped
        S->seed = q;
        S->ovf = 0;
        S->chk = mw_peek(&ctl->ncommit);
#if PLVI_MW_DIAG
        S->out = -1;
#endif
        // (GROWING since the claim) the slot record before the log entry that names it
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        ctl->cursor = q + 1;
        dlog[2 * (dn & (kMwLog - 1))] = q;
        dlog[2 * (dn & (kMwLog - 1)) + 1] = slot;
        mw_lds_store(&ctl->dlog_n, dn + 1);
        if (STATS) mw_stat(ctl, 0, 1);
    }
    return q;
}

// Copy region points [0, n) from queue A to queue B (one wave).
__device__ __forceinline__ void mw_copy_points(const MwQueue& A, const MwQueue& B, int n, int lane) {
    bool g = false;
    for (int j = lane; j < n; j += 64) {
        mw_qput(B, j, mw_qget(A, j));
        g |= j >= B.lcap;
    }
    if (ballot(g)) vm_drain();
}


template <int NW, bool STATS>
__global__ __launch_bounds__(NW * 64) void lsd_grow_mw_kernel(
    const LineOctDev* __restrict__ octs, const float* __restrict__ pix, const float2* __restrict__ pixcs,
    unsigned* __restrict__ ownspill, size_t ownspill_task, unsigned* __restrict__ gspill, unsigned* __restrict__ slotspill,
    unsigned* __restrict__ xspill, size_t xspill_task, double prec, LsdRegion* __restrict__ regs,
    unsigned* __restrict__ regpts, size_t regpts_frame, int* __restrict__ nlines, int* __restrict__ err, int nslots,
    int nOct, int oBase, int oCount, int* __restrict__ stats, int nf, int* __restrict__ epochs) {
    extern __shared__ __align__(16) unsigned lds_u[];
    __builtin_amdgcn_s_setprio(PLVI_GROW_SETPRIO);
    const int t = blockIdx.x;
    if (t >= nf * oCount) return;
    const int o = oBase + t / nf, f = t - (o - oBase) * nf;
    const int task = f * nOct + o;
    const LineOctDev& od = octs[o];
    const int sw = od.sw, sh = od.sh, wpr = (sw + 31) >> 5;
    // the wave index read uniformly: the role (walker / grower) and this wave's
    // LDS partitions and spill areas stay scalar
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // LDS carve-up: ctl | dispatch log | C | T | H | own windows | growth queues | slot pool
    lds_ctl* ctl = (lds_ctl*)lds_u;
    lds_i32* dlog = (lds_i32*)(lds_u + sizeof(MwCtl) / 4);
    const int nwords = sh * wpr;
    lds_u32* C = (lds_u32*)(dlog + 2 * kMwLog);
    lds_u32* T = C + nwords;
    lds_u32* H = T + nwords;
    lds_u32* ownAll = H + nwords;
    lds_u32* gqAll = ownAll + NW * kMwRB * wpr;
    lds_u8* pool = (lds_u8*)(gqAll + NW * kMwGQ);

    MwEnv E;
    E.P = pix + od.soff + (size_t)f * od.splane;
    E.SC = pixcs + od.soff + (size_t)f * od.splane;
    E.C = C; E.T = T; E.H = H;
    E.own = ownAll + wv * kMwRB * wpr;
    E.ownG = ownspill + (size_t)task * ownspill_task + (size_t)wv * sh * wpr;
    E.ctl = ctl;
    E.epoch = epochs ? epochs + (size_t)task * sh * (wpr * 32) : nullptr;
    E.sw = sw; E.sh = sh; E.wpr = wpr; E.rowbits = wpr * 32;
    E.pdeg = (float)(prec / kD2R);
    E.prec = prec;
    unsigned* sspill = slotspill + (size_t)task * nslots * kMwSlotSpill;  // the host sizes it by nslots
    // growth queue: LDS part + global part (the walker's spans a whole plane)
    const MwQueue GQ = wv == 0 ? MwQueue{gqAll, kMwGQ, xspill + (size_t)task * xspill_task,
                                         (int)min<size_t>(xspill_task, (size_t)sw * sh)}
                               : MwQueue{gqAll + wv * kMwGQ, kMwGQ,
                                         gspill + ((size_t)task * NW + wv) * kMwGSpill, kMwGSpill};
    LsdRegion* outR = regs + (size_t)task * kLsdRawCap;
    unsigned* outP = regpts + (size_t)task * regpts_frame;

    const unsigned long long t_kernel = STATS ? __builtin_amdgcn_s_memtime() : 0;
    // ---- init: C = NOTDEF (and row padding), T = trivial seeds, H = 0
    // (each wave builds whole 32-pixel words: lanes = 64 consecutive pixels)
    const float pdeg = E.pdeg;
    const int min_reg = od.min_reg_size;
    for (int k = wv; k < sh * ((wpr + 1) >> 1); k += NW) {
        const int y = k / ((wpr + 1) >> 1), xb = (k - y * ((wpr + 1) >> 1)) * 64;
        const int x = xb + lane;
        const float* r0 = E.P + (size_t)y * sw;
        float d0 = kNotdefF, dr = kNotdefF, dbl = kNotdefF, db = kNotdefF, dbr = kNotdefF;
        if (x < sw) {
            d0 = r0[x];
            if (x + 1 < sw) dr = r0[x + 1];
            if (y + 1 < sh) {
                const float* r1 = r0 + sw;
                if (x > 0) dbl = r1[x - 1];
                db = r1[x];
                if (x + 1 < sw) dbr = r1[x + 1];
            }
        }
        const bool def = x < sw && d0 != kNotdefF;
        // forward neighbours of a seed: (x+1,y) (x-1,y+1) (x,y+1) (x+1,y+1);
        // none aligned with its angle -> region = {seed} (< min_reg_size)
        const bool grows = is_aligned_fast(dr, d0, pdeg, prec) || is_aligned_fast(dbl, d0, pdeg, prec) ||
                           is_aligned_fast(db, d0, pdeg, prec) || is_aligned_fast(dbr, d0, pdeg, prec);
        const unsigned long long cm = ballot(!def);
        const unsigned long long tm = ballot(def && !grows && min_reg > 1);
        if (lane < 2 && (xb >> 5) + lane < wpr) {
            const int wi = y * wpr + (xb >> 5) + lane;
            C[wi] = lane == 0 ? (unsigned)cm : (unsigned)(cm >> 32);
            T[wi] = lane == 0 ? (unsigned)tm : (unsigned)(tm >> 32);
            H[wi] = 0u;
        }
    }
    for (int k = threadIdx.x; k < NW * kMwRB * wpr; k += NW * 64) ownAll[k] = 0u;
    for (int k = threadIdx.x; k < nslots; k += NW * 64) {
        mw_slot(pool, k)->state = kMwFree;
        mw_slot(pool, k)->seed = -1;
        mw_slot(pool, k)->n = 0;
        mw_slot(pool, k)->ovf = 0;
    }
    if (threadIdx.x == 0) {
        ctl->lock = ctl->dlock = ctl->head = ctl->cursor = ctl->finished = 0;
        ctl->npts = ctl->nout = ctl->overflow = 0;
        ctl->dlog_n = ctl->wptr = ctl->ncommit = 0;
        for (int i = 0; i < kMwStatN; ++i) ctl->stat[i] = 0;
    }
    __syncthreads();

    if (wv == 0) {
        // ---- the walker: resolves seeds in raster order, waits on the head
        // seed's region while it grows
        __builtin_amdgcn_s_setprio(PLVI_MW_WALKER_PRIO);
        while (true) {
            const unsigned long long tw0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
            const int b = mw_walk<STATS>(E, pool, dlog, sspill, GQ, min_reg, outR, outP, lane);
            if (STATS && lane == 0) {
                mw_stat(ctl, 6, (int)(__builtin_amdgcn_s_memtime() - tw0));
                mw_stat(ctl, 8, 1);
            }
            if (b < 0) break;  // every seed resolved
#if PLVI_MW_DIAG
            const unsigned long long twa = STATS ? __builtin_amdgcn_s_memtime() : 0;
            const bool rg = STATS && mw_slot(pool, b)->out == -2;
#endif
            while (mw_lds_load(&mw_slot(pool, b)->state) == kMwGrowing) __builtin_amdgcn_s_sleep(1);
#if PLVI_MW_DIAG
            if (STATS && lane == 0) {
                mw_stat(ctl, rg ? 16 : 18, 1);
                mw_stat(ctl, rg ? 17 : 19, (int)(__builtin_amdgcn_s_memtime() - twa));
                mw_stat(ctl, 30, mw_slot(pool, b)->n);
            }
#endif
        }
    } else if (kMwChecker && wv == 1) {
        // ---- the checker: after every commit, every grown region of the
        // dispatch log ahead of the walk that was grown or checked before that
        // commit is tested against C; an invalid one is marked DIRTY (a
        // grower regrows it before the walk arrives).  Only a hint: the walker
        // validates whatever it commits, and regrows what it finds DIRTY.
        __builtin_amdgcn_s_setprio(PLVI_MW_CHECKER_PRIO);
        int last = 0;
        while (!mw_lds_load(&ctl->finished)) {
            const int nc = mw_lds_load(&ctl->ncommit);
            if (nc == last) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            last = nc;
            const int wp = mw_lds_load(&ctl->wptr), dn = mw_lds_load(&ctl->dlog_n);
            const int head = mw_lds_load(&ctl->head);
            for (int b0 = wp; b0 < dn; b0 += 64) {
                const int j = b0 + lane;
                int sj = 0, n = 0;
                bool cand = false;
                if (j < dn) {
                    const int e = j & (kMwLog - 1);
                    sj = dlog[2 * e + 1];
                    lds_slot* S = mw_slot(pool, sj);
                    cand = mw_lds_load(&S->state) == kMwDone && S->seed == dlog[2 * e] && S->seed >= head &&
                           S->chk < nc && S->ovf == 0;
                    n = S->n;
                }
                // regions held in LDS: a lane each, first committed point ends the test
                const bool small = cand && n <= kMwSP;
                bool bad = false;
                if (small) {
                    const lds_u32* pts = (const lds_u32*)(pool + (size_t)sj * kMwSlotBytes + sizeof(MwSlot));
                    for (int k = 0; k < n; ++k) {
                        const unsigned v = pts[k];
                        if (mw_bit(E.C, E.wpr, (int)(v & 0xffffu), (int)(v >> 16))) {
                            bad = true;
                            break;
                        }
                    }
                }
                // longer regions: the whole wave, one at a time
                for (unsigned long long big = ballot(cand && !small); big; big &= big - 1) {
                    const int lb = __ffsll((long long)big) - 1;
                    const int sb = readlane_i(sj, lb), nb = readlane_i(n, lb);
                    const MwQueue Q = mw_slot_queue(pool, sspill, sb);
                    bool bb = false;
                    for (int k = lane; k < nb; k += 64) {
                        const unsigned v = mw_qget(Q, k);
                        bb |= mw_bit(E.C, E.wpr, (int)(v & 0xffffu), (int)(v >> 16));
                    }
                    const bool isbad = ballot(bb) != 0ull;
                    if (lane == lb) bad = isbad;
                }
                if (cand) {
                    lds_slot* S = mw_slot(pool, sj);
                    if (bad) {
                        const bool marked = mw_lds_cas(&S->state, kMwDone, kMwDirty);
#if PLVI_MW_DIAG
                        if (STATS && marked) mw_stat(ctl, 28, 1);
#endif
                        (void)marked;
                    } else {
                        S->chk = nc;  // a hint (a racing re-dispatch rewrites it)
                    }
                }
            }
        }
    } else {
        // ---- growers
        __builtin_amdgcn_s_setprio(PLVI_MW_GROWER_PRIO);
        while (true) {
            // copy out a committed long region (the walker wrote its record)
            int cs = -1;
            if (mw_try_lock(&ctl->dlock, lane)) {
                for (int b0 = 0; b0 < nslots && cs < 0; b0 += 64) {
                    const int si = b0 + lane;
                    const bool ok = si < nslots && mw_lds_load(&mw_slot(pool, si)->state) == kMwCommitted;
                    const unsigned long long b = ballot(ok);
                    if (b) cs = b0 + __ffsll((long long)b) - 1;
                }
                if (cs >= 0 && lane == 0) mw_lds_store(&mw_slot(pool, cs)->state, kMwCopying);
                mw_unlock(&ctl->dlock, lane);
            }
            if (cs >= 0) {
                lds_slot* S = mw_slot(pool, cs);
                const MwQueue Q = mw_slot_queue(pool, sspill, cs);
                const int n = S->n, out = S->out;
                for (int k = lane; k < n; k += 64) outP[out + k] = mw_qget(Q, k);
                mw_wave_sync();
                if (lane == 0) mw_lds_store(&S->state, kMwFree);
                continue;
            }
            if (mw_lds_load(&ctl->finished)) break;
            // regrow a region an earlier commit has invalidated, off the
            // walker's path (the walker still validates every region it
            // commits).  With the checker: the earliest DIRTY region of the log
            // ahead of the walk (claimed by compare-and-swap, no lock).  r05
            // scheme: recheck one of the first kMwLook log entries after the
            // walk that was grown or checked before the latest commit.
            if (kMwChecker || kMwLook > 0) {
                int rs = -1;
                if (kMwChecker) {
                    const int wp = mw_lds_load(&ctl->wptr), dn = mw_lds_load(&ctl->dlog_n);
                    const int head = mw_lds_load(&ctl->head);
                    for (int b0 = wp; b0 < dn && rs < 0; b0 += 64) {
                        const int j = b0 + lane;
                        int sj = -1;
                        bool ok = false;
                        if (j < dn) {
                            const int e = j & (kMwLog - 1);
                            sj = dlog[2 * e + 1];
                            lds_slot* S = mw_slot(pool, sj);
                            ok = mw_lds_load(&S->state) == kMwDirty && S->seed == dlog[2 * e] && S->seed >= head;
                        }
                        for (unsigned long long b = ballot(ok); b && rs < 0; b &= b - 1) {
                            const int cand = readlane_i(sj, __ffsll((long long)b) - 1);
                            int got = 0;
                            if (lane == 0) got = mw_lds_cas(&mw_slot(pool, cand)->state, kMwDirty, kMwGrowing) ? 1 : 0;
                            if (__builtin_amdgcn_readfirstlane(got)) rs = cand;
                        }
                    }
                } else if (mw_try_lock(&ctl->dlock, lane)) {
                    const int wp = mw_lds_load(&ctl->wptr), dn = mw_peek(&ctl->dlog_n);
                    const int nc = mw_lds_load(&ctl->ncommit), head = mw_lds_load(&ctl->head);
                    const int j = wp + lane;
                    int sj = -1;
                    bool ok = false;
                    if (lane < kMwLook && j < dn) {
                        const int e = j & (kMwLog - 1);
                        sj = dlog[2 * e + 1];
                        lds_slot* S = mw_slot(pool, sj);
                        ok = mw_lds_load(&S->state) == kMwDone && S->seed == dlog[2 * e] && S->seed >= head &&
                             S->chk < nc;
                    }
                    const unsigned long long b = ballot(ok);
                    if (b) {
                        const int cand = readlane_i(sj, __ffsll((long long)b) - 1);
                        int got = 0;
                        if (lane == 0) got = mw_lds_cas(&mw_slot(pool, cand)->state, kMwDone, kMwGrowing) ? 1 : 0;
                        if (__builtin_amdgcn_readfirstlane(got)) rs = cand;
                    }
                    mw_unlock(&ctl->dlock, lane);
                }
                if (rs >= 0) {
                    lds_slot* S = mw_slot(pool, rs);
                    const int nc0 = mw_lds_load(&ctl->ncommit);
                    const int seed = S->seed, n0 = S->n;
                    const int sx = seed % E.rowbits, sy = seed / E.rowbits;
                    const MwQueue Q = mw_slot_queue(pool, sspill, rs);
                    bool bad = kMwChecker;  // a DIRTY region is known invalid
#if PLVI_MW_DIAG
                    if (STATS && lane == 0 && !kMwChecker) mw_stat(ctl, 28, 1);
#endif
                    if (!kMwChecker)
                        for (int k = lane; k < n0; k += 64) {
                            const unsigned v = mw_qget(Q, k);
                            bad |= mw_bit(E.C, E.wpr, (int)(v & 0xffffu), (int)(v >> 16));
                        }
                    int nst = kMwDone;
                    if (mw_bit(E.C, E.wpr, sx, sy)) {
                        nst = kMwFree;  // the seed itself was taken: the walk never visits it
                    } else if (ballot(bad) == 0ull) {
                        if (lane == 0) S->chk = nc0;
                    } else {
                        int n = 0;
                        float deg = 0.f;
                        bool spilled = false;
                        const unsigned long long ts0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
#if PLVI_MW_DIAG
                        if (STATS && lane == 0) {
                            mw_stat(ctl, 29, 1);
                            S->out = -2;
                        }
#endif
                        int rc = mw_grow<true, STATS>(E, sx, sy, GQ, n, deg, spilled, lane);
                        mw_own_clear(E, sy, GQ, n, spilled, lane);
                        if (rc == 0) {
                            if (n > kMwSP + kMwSlotSpill) rc = 2;
                            else mw_copy_points(GQ, Q, n, lane);
                        }
                        if (STATS && lane == 0) mw_stat(ctl, 11, (int)(__builtin_amdgcn_s_memtime() - ts0));
                        if (lane == 0) {
                            S->n = n;
                            S->deg = deg;
                            S->ovf = rc == 2 ? 1 : 0;
                            S->chk = nc0;
                        }
                        nst = rc == 1 ? kMwFree : kMwDone;
                    }
                    mw_wave_sync();
                    if (lane == 0) mw_lds_store(&S->state, nst);
                    continue;
                }
            }
            // a new speculative region
            int q = -1, si = -1;
            if (mw_try_lock(&ctl->dlock, lane)) {
                q = mw_dispatch<STATS>(E, pool, nslots, dlog, si, lane);
                mw_unlock(&ctl->dlock, lane);
            }
            if (q < 0) {
                __builtin_amdgcn_s_sleep(2);
                continue;
            }
            int n = 0;
            float deg = 0.f;
            bool spilled = false;
            const unsigned long long ts0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
            int rc = mw_grow<true, STATS>(E, q % E.rowbits, q / E.rowbits, GQ, n, deg, spilled, lane);
            mw_own_clear(E, q / E.rowbits, GQ, n, spilled, lane);
            lds_slot* S = mw_slot(pool, si);
            if (rc == 0) {
                if (n > kMwSP + kMwSlotSpill) rc = 2;  // too long for a slot: the walker regrows it
                else mw_copy_points(GQ, mw_slot_queue(pool, sspill, si), n, lane);
            }
            if (STATS && lane == 0) mw_stat(ctl, 11, (int)(__builtin_amdgcn_s_memtime() - ts0));
            if (lane == 0) {
                S->n = n;
                S->deg = deg;
                S->ovf = rc == 2 ? 1 : 0;
                if (STATS && rc == 1) mw_stat(ctl, 1, 1);
            }
            mw_wave_sync();
            if (lane == 0) mw_lds_store(&S->state, rc == 1 ? kMwFree : kMwDone);
        }
    }
    __syncthreads();
    // copy out the long regions committed after the last growers' copy-out
    // scans (a grower skips its scan while another holds dlock, so every
    // grower can miss a region committed just before the walk finishes)
    for (int si = wv; si < nslots; si += NW) {
        lds_slot* S = mw_slot(pool, si);
        if (S->state == kMwCommitted) {
            const MwQueue Q = mw_slot_queue(pool, sspill, si);
            const int n = S->n, out = S->out;
            for (int k = lane; k < n; k += 64) outP[out + k] = mw_qget(Q, k);
        }
    }
    if (threadIdx.x == 0) {
        nlines[task] = ctl->nout;
        if (ctl->overflow) atomicOr(err + f, 4);
        if (STATS) {
            ctl->stat[10] = (int)(__builtin_amdgcn_s_memtime() - t_kernel);
            for (int i = 0; i < kMwStatN; ++i) stats[(size_t)task * kMwStatN + i] = ctl->stat[i];
        }
    }
}

}  // namespace plvi
