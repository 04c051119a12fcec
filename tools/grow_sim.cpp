// Simulator for intra-frame speculative LSD region growing (diagnostic tool,
// not product code).  Input: flsd's angle plane of one scaled image
// (oracle_lsd_planes).  It runs
//   (1) the reference's sequential region loop (lsd.cpp:476-533, 635-686)
//       and reports region statistics;
//   (2) a time-stepped model of K waves growing regions concurrently, one
//       BFS generation per wave per time step, each wave owning `slots`
//       region slots; regions commit in seed order after validation against
//       the committed bitmap, and the committed regions are checked against
//       the sequential ones.
//   view = 0: a growing region sees only committed pixels and its own;
//   view = 1: it also sees the live claims of earlier-seeded regions (an
//             owner plane updated by atomicMin of the seed address).
// The dispatcher skips pixels any region has claimed (a hint).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {
const double NOTDEF = -1024.0;
const double DEG_TO_RADS = M_PI / 180;
const double M_3_2_PI_ = (3 * M_PI) / 2;
const double M_2__PI_ = (2 * M_PI);

float fast_atan2(float y, float x) {  // cv::fastAtan2 (OpenCV 4.2)
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI), p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI), p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = std::abs(x), ay = std::abs(y), a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

struct Planes {
    int w, h;
    const double* ang;
    bool aligned(int a, double theta, double prec) const {
        const double v = ang[a];
        if (v == NOTDEF) return false;
        double n = theta - v;
        if (n < 0) n = -n;
        if (n > M_3_2_PI_) {
            n -= M_2__PI_;
            if (n < 0) n = -n;
        }
        return n <= prec;
    }
};
const uint32_t INF = 0xffffffffu;

// A region growing one BFS generation per step.
struct Grower {
    std::vector<int> pts, seen;
    size_t i = 0, gen_end = 0;
    double reg_angle = 0;
    float sumdx = 0, sumdy = 0;
    int seed = -1, sid = 0, gens = 0;
    bool done = true;
    std::vector<int> stamp;  // private own-region marks (per attempt id)
};

template <class Accept>
void grow_start(Grower& G, const Planes& P, int seed, int sid, Accept accept) {
    G.pts.clear();
    G.seen.clear();
    if ((int)G.stamp.size() < P.w * P.h) G.stamp.assign(P.w * P.h, 0);
    G.pts.push_back(seed);
    G.seed = seed;
    G.sid = sid;
    G.reg_angle = P.ang[seed];
    G.sumdx = (float)std::cos(G.reg_angle);
    G.sumdy = (float)std::sin(G.reg_angle);
    accept(seed);
    G.i = 0;
    G.gen_end = 1;
    G.gens = 0;
    G.done = false;
}
// one generation; returns true when the region is complete
template <class Used, class Accept>
bool grow_step(Grower& G, const Planes& P, double prec, Used used, Accept accept) {
    const size_t end = G.gen_end;
    for (; G.i < end; ++G.i) {
        const int rx = G.pts[G.i] % P.w, ry = G.pts[G.i] / P.w;
        const int x0 = std::max(rx - 1, 0), x1 = std::min(rx + 1, P.w - 1);
        const int y0 = std::max(ry - 1, 0), y1 = std::min(ry + 1, P.h - 1);
        for (int yy = y0; yy <= y1; ++yy)
            for (int xx = x0; xx <= x1; ++xx) {
                const int c = xx + yy * P.w;
                if (!used(c) && P.aligned(c, G.reg_angle, prec)) {
                    accept(c);
                    G.pts.push_back(c);
                    const double a = P.ang[c];
                    G.sumdx += cosf((float)a);
                    G.sumdy += sinf((float)a);
                    G.reg_angle = fast_atan2(G.sumdy, G.sumdx) * DEG_TO_RADS;
                }
            }
    }
    ++G.gens;
    G.gen_end = G.pts.size();
    if (G.i >= G.pts.size()) G.done = true;
    return G.done;
}

struct Slot {
    Grower G;
    bool busy = false;  // holds a region (growing or done, not committed)
};
}  // namespace

extern "C" int grow_sim(const double* ang, int w, int h, int K, int slots, int view, int overhead, double* stats) {
    Planes P{w, h, ang};
    const double prec = M_PI * 22.5 / 180;
    const int N = w * h;
    auto is_seed_px = [&](int a) { return (a % w) < w - 1 && (a / w) < h - 1 && ang[a] != NOTDEF; };
    // (1) sequential reference
    std::vector<uint8_t> used(N, 0);
    std::vector<std::vector<int>> ref;
    double seq_cost = 0, seq_pts = 0, ndef = 0;
    int big = 0;
    {
        Grower G;
        for (int a = 0; a < N; ++a) {
            if (!is_seed_px(a)) continue;
            ndef += 1;
            if (used[a]) continue;
            auto U = [&](int c) { return used[c] == 1; };
            auto A = [&](int c) { used[c] = 1; };
            grow_start(G, P, a, 0, A);
            while (!grow_step(G, P, prec, U, A)) {
            }
            ref.push_back(G.pts);
            seq_cost += overhead + G.gens;
            seq_pts += G.pts.size();
            if (G.pts.size() >= 10) ++big;
        }
    }
    // (2) K waves x `slots` slots, time-stepped
    std::vector<uint32_t> owner(N, INF);  // live claims (atomicMin of the seed address)
    std::vector<uint8_t> C(N, 0);         // committed
    std::vector<uint8_t> hint(N, 0);      // claimed by any region (dispatch hint)
    int next_sid = 0;
    const int S = K * slots;
    std::vector<Slot> sl(S);
    std::vector<int> wave_cur(K, -1);  // slot being grown by each wave
    std::vector<int> wave_busy(K, 0);  // overhead steps left
    std::vector<int> slot_of_seed(N, -1);
    int cursor = 0, head = 0;
    size_t ncommit = 0;
    bool ok = true;
    long long t = 0, dispatched = 0, dropped = 0, regrown = 0, exact_head = 0;
    auto used_fn = [&](Grower& G) {
        return [&, sp = &G](int c) {
            if (sp->stamp[c] == sp->sid) return true;
            if (C[c]) return true;
            if (view && owner[c] < (uint32_t)sp->seed) {
                sp->seen.push_back(c);
                return true;
            }
            return false;
        };
    };
    auto acc_fn = [&](Grower& G) {
        return [&, sp = &G](int c) {
            sp->stamp[c] = sp->sid;
            hint[c] = 1;
            owner[c] = std::min(owner[c], (uint32_t)sp->seed);
        };
    };
    auto release = [&](Grower& G) {
        for (int c : G.pts)
            if (owner[c] == (uint32_t)G.seed) owner[c] = INF;
    };
    Grower headG;
    int committer_busy = 0;  // the commit walk is serial: its regrows cost time
    while (head < N && t < 100000000) {
        ++t;
        // (a) every wave advances its region one generation (or its overhead)
        for (int k = 0; k < K; ++k) {
            if (wave_busy[k] > 0) {
                --wave_busy[k];
                continue;
            }
            int s = wave_cur[k];
            if (s >= 0 && sl[s].busy && !sl[s].G.done) {
                auto U = used_fn(sl[s].G);
                auto A = acc_fn(sl[s].G);
                grow_step(sl[s].G, P, prec, U, A);
                continue;
            }
            int fs = -1;
            for (int j = 0; j < slots; ++j)
                if (!sl[k * slots + j].busy) fs = k * slots + j;
            if (fs < 0) continue;  // every slot waits for its commit
            while (cursor < N && (!is_seed_px(cursor) || hint[cursor] || C[cursor] || cursor < head)) ++cursor;
            if (cursor >= N) continue;
            Slot& X = sl[fs];
            X.busy = true;
            slot_of_seed[cursor] = fs;
            auto A = acc_fn(X.G);
            grow_start(X.G, P, cursor, ++next_sid, A);
            ++dispatched;
            ++cursor;
            wave_cur[k] = fs;
            wave_busy[k] = overhead;
        }
        // (b) commit walk (one committer; a regrow / head growth costs its generations)
        if (committer_busy > 0) {
            --committer_busy;
            continue;
        }
        while (head < N) {
            if (!is_seed_px(head) || C[head]) {
                const int s = slot_of_seed[head];
                if (s >= 0 && sl[s].busy && sl[s].G.seed == head) {  // absorbed seed: abort + drop its region
                    release(sl[s].G);
                    sl[s].G.done = true;
                    sl[s].busy = false;
                    ++dropped;
                }
                slot_of_seed[head] = -1;
                ++head;
                continue;
            }
            int s = slot_of_seed[head];
            if (s < 0) {  // never dispatched (hint): grow it now, exact, costs time
                Grower& G = headG;
                auto U = used_fn(G);
                auto A = acc_fn(G);
                grow_start(G, P, head, ++next_sid, A);
                while (!grow_step(G, P, prec, U, A)) {
                }
                committer_busy += overhead + G.gens;
                ++exact_head;
                for (int c : G.pts) C[c] = 1;
                if (ncommit >= ref.size() || ref[ncommit] != G.pts) ok = false;
                ++ncommit;
                ++head;
                break;
            }
            Slot& X = sl[s];
            if (!X.G.done) break;
            bool valid = !C[X.G.seed];
            for (int c : X.G.pts) valid = valid && !C[c];
            for (int c : X.G.seen) valid = valid && C[c];
            if (!valid) {
                release(X.G);
                auto U = used_fn(X.G);
                auto A = acc_fn(X.G);
                grow_start(X.G, P, head, ++next_sid, A);
                while (!grow_step(X.G, P, prec, U, A)) {
                }
                committer_busy += overhead + X.G.gens;
                ++regrown;
            }
            for (int c : X.G.pts) C[c] = 1;
            if (ncommit >= ref.size() || ref[ncommit] != X.G.pts) ok = false;
            ++ncommit;
            X.busy = false;
            slot_of_seed[head] = -1;
            ++head;
            if (committer_busy) break;
        }
    }
    stats[0] = (double)ref.size();
    stats[1] = seq_pts;
    stats[2] = seq_cost;
    stats[3] = (double)t;
    stats[4] = ok && ncommit == ref.size() ? 1 : 0;
    stats[5] = (double)dispatched;
    stats[6] = (double)dropped;
    stats[7] = (double)regrown;
    stats[8] = ndef;
    stats[9] = big;
    stats[10] = (double)exact_head;
    return 0;
}
