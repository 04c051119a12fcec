// oracle/match_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the Hamming matchers on the path ("parity unpinned":
// no reference test pins them; restated from the cited lines):
//   DescriptorDistance  src/ORBmatcher.cc:2350-2366 (SWAR popcount, >>24)
//   LineMatcher::DescriptorDistance src/LineMatcher.cpp:487-499 (>>25 quirk)
//   BFMatcher::knnMatch(k=2)  OpenCV 4.2 batchDistance K-insertion
//   LineMatcher::matchNNR / match  src/LineMatcher.cpp:41-111
//   ORBmatcher::SearchByBoW(KeyFrame*, Frame&, ...)  src/ORBmatcher.cc:269-471
//   LineMatcher::matchGrid  src/LineMatcher.cpp:191-272 (+ gridStructure.cpp:64-75)
#include <algorithm>
#include <stdexcept>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include "ref_fma.h"

static int descriptor_distance(const uint8_t* a, const uint8_t* b, int shift) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
        int32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        unsigned int v = (unsigned)(pa ^ pb);
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        dist += (int)((((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> shift);
    }
    return dist;
}

extern "C" int oracle_descriptor_distance(const uint8_t* a, const uint8_t* b) { return descriptor_distance(a, b, 24); }
extern "C" int oracle_line_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    return descriptor_distance(a, b, 25);
}

extern "C" void oracle_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int* i0, int* d0, int* i1, int* d1) {
    const int K = 2;
    for (int i = 0; i < nq; ++i) {
        int dist[K] = {INT_MAX, INT_MAX}, nidx[K] = {-1, -1};
        for (int j = 0; j < nt; ++j) {
            int d = descriptor_distance(q + (size_t)i * 32, t + (size_t)j * 32, 24);
            if (d < dist[K - 1]) {
                int k;
                for (k = K - 2; k >= 0 && dist[k] > d; k--) {
                    nidx[k + 1] = nidx[k];
                    dist[k + 1] = dist[k];
                }
                nidx[k + 1] = j;
                dist[k + 1] = d;
            }
        }
        i0[i] = nidx[0]; d0[i] = dist[0]; i1[i] = nidx[1]; d1[i] = dist[1];
    }
}

// LineMatcher::matchNNR / match (LineMatcher.cpp:41-61, :92-111) on a
// std::vector<int> exactly as the reference holds it: resize(rows, -1) keeps
// the caller's existing entries.
static int match_nnr_vec(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, std::vector<int>& m12) {
    m12.resize(n1, -1);
    std::vector<int> i0(n1), a(n1), i1(n1), b(n1);
    oracle_knn2(d1, n1, d2, n2, i0.data(), a.data(), i1.data(), b.data());
    int matches = 0;
    for (int idx = 0; idx < n1; ++idx) {
        if ((float)a[idx] < (float)b[idx] * nnr) {
            m12[idx] = i0[idx];
            ++matches;
        }
    }
    return matches;
}

static int match_vec(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, std::vector<int>& m12) {
    std::vector<int> m21;
    int matches = match_nnr_vec(d1, n1, d2, n2, nnr, m12);
    match_nnr_vec(d2, n2, d1, n1, nnr, m21);
    for (int i1 = 0, nsize = (int)m12.size(); i1 < nsize; ++i1) {
        int& i2 = m12[i1];
        if (i2 >= 0 && m21.at(i2) != i1) {  // .at: a stale out-of-range entry is UB in the reference
            i2 = -1;
            --matches;
        }
    }
    return matches;
}

// m12 holds n_prev existing entries on entry and n1 on return.
extern "C" int oracle_match_nnr_inout(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, int* m12,
                                      int n_prev) {
    std::vector<int> v(m12, m12 + n_prev);
    int r = match_nnr_vec(d1, n1, d2, n2, nnr, v);
    std::copy(v.begin(), v.end(), m12);
    return r;
}

extern "C" int oracle_match_inout(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, int* m12,
                                  int n_prev) {
    std::vector<int> v(m12, m12 + n_prev);
    int r;
    try {
        r = match_vec(d1, n1, d2, n2, nnr, v);
    } catch (const std::out_of_range&) {
        return -2;
    }
    std::copy(v.begin(), v.end(), m12);
    return r;
}

extern "C" int oracle_match_nnr(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, int* m12) {
    return oracle_match_nnr_inout(d1, n1, d2, n2, nnr, m12, 0);
}

extern "C" int oracle_match(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float nnr, int* m12) {
    return oracle_match_inout(d1, n1, d2, n2, nnr, m12, 0);
}

// ORBmatcher::SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
// (src/ORBmatcher.cc:269-471) + ComputeThreeMaxima (:2304-2345), one or two
// cameras (F.Nleft, oracle_search_by_bow2).  The FeatureVectors
// (std::map<NodeId, vector<unsigned>>) arrive as CSR arrays sorted by node
// id; pMP != NULL && !pMP->isBad() arrives as kf_live[realIdxKF].  Output:
// match_kf[iF] = KF keypoint index whose MapPoint the reference stores in
// vpMapPointMatches[iF], or -1.  Returns nmatches.
static int lower_bound_node(const int* ids, int lo, int hi, int key) {
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (ids[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// f_nleft = F.Nleft: -1 = one camera (:321-342); otherwise the two-camera
// branch (:343-366, :404-431): keypoints [0, Nleft) left, [Nleft, N) right,
// a best / second pair per camera, the right best taken (ratio test `|| true`)
// inside the left best's TH_LOW test.
extern "C" int oracle_search_by_bow2(const uint8_t* kf_desc, const float* kf_angle, const uint8_t* kf_live,
                                     const int* kf_node, const int* kf_off, int kf_nnodes, const int* kf_idx,
                                     const uint8_t* f_desc, const float* f_angle, int f_n, const int* f_node,
                                     const int* f_off, int f_nnodes, const int* f_idx, float nnratio,
                                     int check_orientation, int f_nleft, int* match_kf);

extern "C" int oracle_search_by_bow(const uint8_t* kf_desc, const float* kf_angle, const uint8_t* kf_live,
                                    const int* kf_node, const int* kf_off, int kf_nnodes, const int* kf_idx,
                                    const uint8_t* f_desc, const float* f_angle, int f_n, const int* f_node,
                                    const int* f_off, int f_nnodes, const int* f_idx, float nnratio,
                                    int check_orientation, int* match_kf) {
    return oracle_search_by_bow2(kf_desc, kf_angle, kf_live, kf_node, kf_off, kf_nnodes, kf_idx, f_desc, f_angle, f_n,
                                 f_node, f_off, f_nnodes, f_idx, nnratio, check_orientation, -1, match_kf);
}

extern "C" int oracle_search_by_bow2(const uint8_t* kf_desc, const float* kf_angle, const uint8_t* kf_live,
                                     const int* kf_node, const int* kf_off, int kf_nnodes, const int* kf_idx,
                                     const uint8_t* f_desc, const float* f_angle, int f_n, const int* f_node,
                                     const int* f_off, int f_nnodes, const int* f_idx, float nnratio,
                                     int check_orientation, int f_nleft, int* match_kf) {
    const int TH_LOW = 50, HISTO_LENGTH = 30;
    for (int i = 0; i < f_n; ++i) match_kf[i] = -1;
    std::vector<std::vector<int>> rotHist(HISTO_LENGTH);
    const float factor = 1.0f / HISTO_LENGTH;
    int nmatches = 0;
    int KFit = 0, Fit = 0;
    while (KFit < kf_nnodes && Fit < f_nnodes) {
        if (kf_node[KFit] == f_node[Fit]) {
            for (int a = kf_off[KFit]; a < kf_off[KFit + 1]; ++a) {
                const int realIdxKF = kf_idx[a];
                if (!kf_live[realIdxKF]) continue;
                const uint8_t* dKF = kf_desc + (size_t)realIdxKF * 32;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                int bestDist1R = 256, bestIdxFR = -1, bestDist2R = 256;
                for (int b = f_off[Fit]; b < f_off[Fit + 1]; ++b) {
                    const unsigned realIdxF = (unsigned)f_idx[b];
                    if (match_kf[realIdxF] >= 0) continue;
                    const int dist = descriptor_distance(dKF, f_desc + (size_t)realIdxF * 32, 24);
                    if (f_nleft == -1) {
                        if (dist < bestDist1) {
                            bestDist2 = bestDist1;
                            bestDist1 = dist;
                            bestIdxF = (int)realIdxF;
                        } else if (dist < bestDist2) {
                            bestDist2 = dist;
                        }
                    } else {
                        const unsigned nl = (unsigned)f_nleft;
                        if (realIdxF < nl && dist < bestDist1) {
                            bestDist2 = bestDist1;
                            bestDist1 = dist;
                            bestIdxF = (int)realIdxF;
                        } else if (realIdxF < nl && dist < bestDist2) {
                            bestDist2 = dist;
                        }
                        if (realIdxF >= nl && dist < bestDist1R) {
                            bestDist2R = bestDist1R;
                            bestDist1R = dist;
                            bestIdxFR = (int)realIdxF;
                        } else if (realIdxF >= nl && dist < bestDist2R) {
                            bestDist2R = dist;
                        }
                    }
                }
                auto take = [&](int idx) {
                    match_kf[idx] = realIdxKF;
                    if (check_orientation) {
                        float rot = kf_angle[realIdxKF] - f_angle[idx];
                        if (rot < 0.0) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == HISTO_LENGTH) bin = 0;
                        rotHist[bin].push_back(idx);
                    }
                    nmatches++;
                };
                if (bestDist1 <= TH_LOW) {
                    if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) take(bestIdxF);
                    if (bestDist1R <= TH_LOW) {
                        (void)bestDist2R;  // `static_cast<float>(bestDist1R) < mfNNratio * ... || true` (:411)
                        take(bestIdxFR);
                    }
                }
            }
            KFit++;
            Fit++;
        } else if (kf_node[KFit] < f_node[Fit]) {
            KFit = lower_bound_node(kf_node, KFit, kf_nnodes, f_node[Fit]);
        } else {
            Fit = lower_bound_node(f_node, Fit, f_nnodes, kf_node[KFit]);
        }
    }
    if (check_orientation) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        int max1 = 0, max2 = 0, max3 = 0;
        for (int i = 0; i < HISTO_LENGTH; i++) {
            const int s = (int)rotHist[i].size();
            if (s > max1) {
                max3 = max2; max2 = max1; max1 = s;
                ind3 = ind2; ind2 = ind1; ind1 = i;
            } else if (s > max2) {
                max3 = max2; max2 = s;
                ind3 = ind2; ind2 = i;
            } else if (s > max3) {
                max3 = s;
                ind3 = i;
            }
        }
        if (max2 < 0.1f * (float)max1) {
            ind2 = -1;
            ind3 = -1;
        } else if (max3 < 0.1f * (float)max1) {
            ind3 = -1;
        }
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (size_t j = 0; j < rotHist[i].size(); j++) {
                match_kf[rotHist[i][j]] = -1;
                nmatches--;
            }
        }
    }
    return nmatches;
}

// LineMatcher::matchGrid (src/LineMatcher.cpp:191-272) with
// GridStructure::get (src/gridStructure.cpp:64-75): literal restatement on
// std::list cells and std::unordered_set<int> candidates (the host
// libstdc++ decides the candidate iteration order, as the reference's
// does).  lines1[i] = (sp.x, sp.y, ep.x, ep.y) as line_2d = pair<pair<int,int>>
// (coordinates already truncated to grid cells by the caller, Frame.cc:1424-1427);
// the grid is CSR over cells (x * rows + y) in list order.
#include <list>
#include <limits>
#include <unordered_set>

// indices.insert(first, last) as libstdc++ up to GCC 10 performs it (the
// reference's Ubuntu 20.04 / GCC 9.3 build): _M_insert_range
// passes the remaining range length __n_elt as the rehash hint of
// _M_insert_unique_node, reset to 1 after each insertion and decremented
// for each key already present.  GCC 11 (this host) dropped the hint from
// insert(first, last) but keeps exactly that loop in _M_merge_unique, so the
// oracle drives the HOST library's own hashtable through merge(): the
// source is an unordered_multiset with a constant hash and an equality that
// never holds, whose iteration order is the reverse of its insertion order
// (every node is inserted at the front of bucket 0; the multi-key rehash
// keeps bucket order), so inserting the cell reversed makes the merge visit
// it in list order.  Independent of the product's emulation
// (csrc/stl_uset.h): here the host _Hashtable / _Prime_rehash_policy code
// runs the insertion.
struct ConstHash {
    size_t operator()(int) const noexcept { return 0; }
};
struct NeverEq {
    bool operator()(int, int) const noexcept { return false; }
};
static void insert_range_gcc10(std::unordered_set<int>& indices, const std::list<int>& cell) {
    if (cell.empty()) return;
    std::unordered_multiset<int, ConstHash, NeverEq> src;
    for (auto it = cell.rbegin(); it != cell.rend(); ++it) src.insert(*it);
    indices.merge(src);
}

// GridStructure(rows, cols) filled from CSR cells (x * rows + y) in list order
using GridLists = std::vector<std::vector<std::list<int>>>;
static GridLists grid_lists(int cols, int rows, const int* cell_off, const int* cell_idx) {
    GridLists grid(cols, std::vector<std::list<int>>(rows));
    for (int x = 0; x < cols; ++x)
        for (int y = 0; y < rows; ++y)
            for (int k = cell_off[x * rows + y]; k < cell_off[x * rows + y + 1]; ++k) grid[x][y].push_back(cell_idx[k]);
    return grid;
}

// GridStructure::get (src/gridStructure.cpp:67-78)
static void grid_get(const GridLists& grid, int cols, int rows, int x, int y, int w0, int w1, int h0, int h1,
                     int range_hint, std::unordered_set<int>& indices) {
    int min_x = std::max(0, x - w0);
    int max_x = std::min(cols, x + w1 + 1);
    int min_y = std::max(0, y - h0);
    int max_y = std::min(rows, y + h1 + 1);
    for (int x_ = min_x; x_ < max_x; ++x_)
        for (int y_ = min_y; y_ < max_y; ++y_) {
            if (range_hint) insert_range_gcc10(indices, grid[x_][y_]);
            else indices.insert(grid[x_][y_].begin(), grid[x_][y_].end());
        }
}

// The candidate set of one matchGrid line (get at sp, then at ep, into one
// set) in iteration order: the restatement tests/test_ref_grid.py compares
// with the reference's own gridStructure.cpp (oracle/_ref).
extern "C" int oracle_grid_candidates(int cols, int rows, const int* cell_off, const int* cell_idx, int spx, int spy,
                                      int epx, int epy, int w0, int w1, int h0, int h1, int range_hint, int* out,
                                      int cap) {
    const GridLists grid = grid_lists(cols, rows, cell_off, cell_idx);
    std::unordered_set<int> c;
    grid_get(grid, cols, rows, spx, spy, w0, w1, h0, h1, range_hint, c);
    grid_get(grid, cols, rows, epx, epy, w0, w1, h0, h1, range_hint, c);
    int n = 0;
    for (int v : c) {
        if (n < cap) out[n] = v;
        ++n;
    }
    return n;
}

extern "C" int oracle_match_grid2(const int* lines1, const uint8_t* desc1, int n1, int cols, int rows,
                                  const int* cell_off, const int* cell_idx, const uint8_t* desc2,
                                  const double* directions2, int n2, int w0, int w1, int h0, int h1,
                                  int range_hint, int* matches_12) {
    const GridLists grid = grid_lists(cols, rows, cell_off, cell_idx);
    auto get = [&](int x, int y, std::unordered_set<int>& indices) {
        grid_get(grid, cols, rows, x, y, w0, w1, h0, h1, range_hint, indices);
    };
    const double lineSimTh = 0.75, minRatio12L = 0.9;
    int matches = 0;
    for (int i = 0; i < n1; ++i) matches_12[i] = -1;
    std::vector<int> matches_21(n2, -1), distances(n2, std::numeric_limits<int>::max());
    for (int i1 = 0; i1 < n1; ++i1) {
        int best_d = std::numeric_limits<int>::max(), best_d2 = std::numeric_limits<int>::max(), best_idx = -1;
        const int spx = lines1[4 * i1], spy = lines1[4 * i1 + 1], epx = lines1[4 * i1 + 2], epy = lines1[4 * i1 + 3];
        double vx = (double)(epx - spx), vy = (double)(epy - spy);
        const double magnitude = std::sqrt(ref_fma(vx, vx, vy * vy));  // normalize / dot: fused in LineMatcher.cpp.o
        vx /= magnitude;
        vy /= magnitude;
        std::unordered_set<int> candidates;
        get(spx, spy, candidates);
        get(epx, epy, candidates);
        if (candidates.empty()) continue;
        for (const int& i2 : candidates) {
            if (i2 < 0 || i2 >= n2) continue;
            if (std::abs(ref_fma(vx, directions2[2 * i2], vy * directions2[2 * i2 + 1])) < lineSimTh) continue;
            const int d = descriptor_distance(desc1 + (size_t)i1 * 32, desc2 + (size_t)i2 * 32, 24);
            if (d < distances[i2]) {
                distances[i2] = d;
                matches_21[i2] = i1;
            } else {
                continue;
            }
            if (d < best_d) {
                best_d2 = best_d;
                best_d = d;
                best_idx = i2;
            } else if (d < best_d2) {
                best_d2 = d;
            }
        }
        if (best_d < best_d2 * minRatio12L) {
            matches_12[i1] = best_idx;
            matches++;
        }
    }
    for (int i1 = 0; i1 < n1; ++i1) {
        int& i2 = matches_12[i1];
        if (i2 >= 0 && matches_21[i2] != i1) {
            i2 = -1;
            matches--;
        }
    }
    return matches;
}

extern "C" int oracle_match_grid(const int* lines1, const uint8_t* desc1, int n1, int cols, int rows,
                                 const int* cell_off, const int* cell_idx, const uint8_t* desc2,
                                 const double* directions2, int n2, int w0, int w1, int h0, int h1,
                                 int* matches_12) {
    return oracle_match_grid2(lines1, desc1, n1, cols, rows, cell_off, cell_idx, desc2, directions2, n2, w0, w1, h0,
                              h1, 0, matches_12);
}

// Iteration order of a candidate set filled by range inserts (for the
// emulation's own checks): out receives the set's elements in iteration order.
extern "C" int oracle_uset_order(const int* seq_off, const int* seq, int nseq, int range_hint, int* out) {
    std::unordered_set<int> s;
    for (int k = 0; k < nseq; ++k) {
        std::list<int> cell(seq + seq_off[k], seq + seq_off[k + 1]);
        if (range_hint) insert_range_gcc10(s, cell);
        else s.insert(cell.begin(), cell.end());
    }
    int n = 0;
    for (int v : s) out[n++] = v;
    return n;
}

// LineMatcher::SearchByProjection(Frame& CurrentFrame, Frame& LastFrame,
// const GridStructure& grid, th, angth) (src/LineMatcher.cpp:274-372).
// The per-line MapLine state is evaluated by the caller: last_flags bit0 =
// mvpMapLines[i] && !mvbOutlier_Line[i], bit1 = that MapLine's Observations() > 0;
// x3dc = Rcw*x3Dw+tcw of its two endpoints (cv::Mat float, 6 floats);
// last_oct = mvKeys_Line[i].octave.  Current frame: mvKeysUn_Line angles,
// descriptors, blocked = mvpMapLines[i2] && Observations() > 0 on entry,
// grid_Line as CSR cells (x * rows + y) in std::list order.  inv_w / inv_h
// are Frame::inv_width / inv_height (double).  Literal: the second endpoint's
// grid y is uv_ep.x * inv_height (:329), atan2 of floats is the float
// overload (std::atan2(float, float) via the `using namespace std` of
// GeometricCamera.h).  match[i2] = last-frame line whose MapLine is stored in
// mvpMapLines[i2] (-1 untouched); returns matches (every assignment counts).
extern "C" int oracle_line_search_projection(
    int n_cur, const float* cur_angle, const uint8_t* cur_desc, const uint8_t* cur_blocked, int cols, int rows,
    const int* cell_off, const int* cell_idx, int n_last, const uint8_t* last_flags, const float* x3dc,
    const int* last_oct, const uint8_t* ml_desc, float fx, float fy, float cx, float cy, float minX, float maxX,
    float minY, float maxY, double inv_w, double inv_h, const float* scale_l, float th, float angth, int range_hint,
    int* match) {
    std::vector<std::vector<std::list<int>>> grid(cols, std::vector<std::list<int>>(rows));
    for (int x = 0; x < cols; ++x)
        for (int y = 0; y < rows; ++y)
            for (int k = cell_off[x * rows + y]; k < cell_off[x * rows + y + 1]; ++k) grid[x][y].push_back(cell_idx[k]);
    auto get = [&](int x, int y, int win, std::unordered_set<int>& indices) {
        int min_x = std::max(0, x - win), max_x = std::min(cols, x + win + 1);
        int min_y = std::max(0, y - win), max_y = std::min(rows, y + win + 1);
        for (int x_ = min_x; x_ < max_x; ++x_)
            for (int y_ = min_y; y_ < max_y; ++y_) {
                if (range_hint) insert_range_gcc10(indices, grid[x_][y_]);
                else indices.insert(grid[x_][y_].begin(), grid[x_][y_].end());
            }
    };
    std::vector<char> blocked(cur_blocked, cur_blocked + n_cur);
    for (int i = 0; i < n_cur; ++i) match[i] = -1;
    const int TH_HIGH = 120;
    int matches = 0;
    for (int i = 0; i < n_last; i++) {
        if (!(last_flags[i] & 1)) continue;
        const float* sp = x3dc + 6 * (size_t)i;
        const float* ep = sp + 3;
        const float invzc_sp = 1.0 / sp[2];
        const float invzc_ep = 1.0 / ep[2];
        if (invzc_sp < 0 || invzc_ep < 0) continue;
        const float usx = fx * sp[0] / sp[2] + cx, usy = fy * sp[1] / sp[2] + cy;  // Pinhole::project
        const float uex = fx * ep[0] / ep[2] + cx, uey = fy * ep[1] / ep[2] + cy;
        if (usx < minX || usx > maxX || uex < minX || uex > maxX) continue;
        if (usy < minY || usy > maxY || uey < minY || uey > maxY) continue;
        const int nLastOctave = last_oct[i];
        int window = std::floor(th);
        if (scale_l[nLastOctave] > 1) window = std::floor(th + scale_l[nLastOctave]);
        const std::pair<int, int> spoint = std::make_pair(usx * inv_w, usy * inv_h);
        const std::pair<int, int> epoint = std::make_pair(uex * inv_w, uex * inv_h);  // sic (:329)
        std::unordered_set<int> candidates;
        get(spoint.first, spoint.second, window, candidates);
        get(epoint.first, epoint.second, window, candidates);
        if (candidates.empty()) continue;
        int bestDist = 256, bestidx = -1;
        for (const int& i2 : candidates) {
            if (blocked[i2]) continue;
            const int dist = descriptor_distance(ml_desc + 32 * (size_t)i, cur_desc + 32 * (size_t)i2, 24);
            if (dist < bestDist) {
                bestDist = dist;
                bestidx = i2;
            }
        }
        if (bestDist <= TH_HIGH) {
            float theta = cur_angle[bestidx] - std::atan2(uey - usy, uex - usx);  // float overload
            if (theta < -M_PI) theta += 2 * M_PI;
            else if (theta > M_PI) theta -= 2 * M_PI;
            if (std::fabs(theta) < angth) {
                match[bestidx] = i;
                blocked[bestidx] = (last_flags[i] & 2) ? 1 : 0;
                matches++;
            }
        }
    }
    return matches;
}

// LineMatcher::SerachForInitialize (src/LineMatcher.cpp:113-139) with
// Frame::lineDescriptorMAD (src/Frame.cc:1089-1112) and the comparators of
// include/LineMatcher.h:56-76, on std::vector<std::vector<DMatch>> as the
// reference holds them (knnMatch k = 2 of the initial frame's lines against
// the current frame's).  Outputs the LineMatches pairs (query, train) in
// order; mad = {nn_mad, nn12_mad}.  The reference indexes [0] and [1] of
// every knnMatch list: with n1 == 0 or n2 < 2 it is undefined, here 0 pairs.
namespace {
struct DMatchO {
    int queryIdx, trainIdx, imgIdx;
    float distance;
};
typedef std::vector<std::vector<DMatchO>> MatchLists;
struct ByNN {
    bool operator()(const std::vector<DMatchO>& a, const std::vector<DMatchO>& b) const {
        return a[0].distance < b[0].distance;
    }
};
struct ByNN12Desc {
    bool operator()(const std::vector<DMatchO>& a, const std::vector<DMatchO>& b) const {
        return (a[1].distance - a[0].distance) > (b[1].distance - b[0].distance);
    }
};
struct ByQuery {
    bool operator()(const std::vector<DMatchO>& a, const std::vector<DMatchO>& b) const {
        return a[0].queryIdx < b[0].queryIdx;
    }
};
void line_descriptor_mad(MatchLists matches, double& nn_mad, double& nn12_mad) {
    MatchLists matches_nn = matches, matches_12 = matches;
    std::sort(matches_nn.begin(), matches_nn.end(), ByNN());
    const double nn_dist_median = matches_nn[int(matches_nn.size() / 2)][0].distance;
    for (unsigned int i = 0; i < matches_nn.size(); i++)
        matches_nn[i][0].distance = fabsf(matches_nn[i][0].distance - nn_dist_median);
    std::sort(matches_nn.begin(), matches_nn.end(), ByNN());
    nn_mad = 1.4826 * matches_nn[int(matches_nn.size() / 2)][0].distance;
    std::sort(matches_12.begin(), matches_12.end(), ByNN12Desc());
    const double nn12_dist_median = matches_12[int(matches_12.size() / 2)][1].distance -
                                    matches_12[int(matches_12.size() / 2)][0].distance;
    for (unsigned int j = 0; j < matches_12.size(); j++)
        matches_12[j][0].distance = fabsf(matches_12[j][1].distance - matches_12[j][0].distance - nn12_dist_median);
    std::sort(matches_12.begin(), matches_12.end(), ByNN());
    nn12_mad = 1.4826 * matches_12[int(matches_12.size() / 2)][0].distance;
}
}  // namespace

extern "C" int oracle_line_search_init(const uint8_t* d1, int n1, const uint8_t* d2, int n2, int* q_out, int* t_out,
                                       double* mad) {
    if (n1 <= 0 || n2 < 2) return 0;
    std::vector<int> i0(n1), a(n1), i1(n1), b(n1);
    oracle_knn2(d1, n1, d2, n2, i0.data(), a.data(), i1.data(), b.data());
    MatchLists lmatches(n1);
    for (int i = 0; i < n1; ++i) {
        lmatches[i].push_back(DMatchO{i, i0[i], 0, (float)a[i]});
        lmatches[i].push_back(DMatchO{i, i1[i], 0, (float)b[i]});
    }
    double nn_dist_th, nn12_dist_th;
    line_descriptor_mad(lmatches, nn_dist_th, nn12_dist_th);
    if (mad) {
        mad[0] = nn_dist_th;
        mad[1] = nn12_dist_th;
    }
    nn12_dist_th = nn12_dist_th * 0.5;
    std::sort(lmatches.begin(), lmatches.end(), ByQuery());
    int nmatches = 0;
    for (int i = 0; i < (int)lmatches.size(); i++) {
        const int qdx = lmatches[i][0].queryIdx, tdx = lmatches[i][0].trainIdx;
        const double dist_12 = lmatches[i][1].distance - lmatches[i][0].distance;
        if (dist_12 > nn12_dist_th) {
            q_out[nmatches] = qdx;
            t_out[nmatches] = tdx;
            nmatches++;
        }
    }
    return nmatches;
}
