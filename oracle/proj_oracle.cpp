// oracle/proj_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the steady-state frame-to-frame ORB matcher and the grid
// it searches ("parity unpinned": no reference test pins them):
//   Frame::AssignFeaturesToGrid      src/Frame.cc:644-675
//   Frame::PosInGrid                 src/Frame.cc:1077-1087
//   Frame::GetFeaturesInArea         src/Frame.cc:1006-1075
//   ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
//                                    src/ORBmatcher.cc:1962-2178 (Nleft == -1 branch)
//   ORBmatcher::ComputeThreeMaxima   src/ORBmatcher.cc:2304-2345
//   ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
//                                    src/ORBmatcher.cc:44-145 (F.Nleft == -1) + RadiusByViewingCos :216-222
//   ORBmatcher::SearchByProjection(Frame&, KeyFrame*, sAlreadyFound, th, ORBdist)
//                                    src/ORBmatcher.cc:2180-2300 (relocalization)
//   Pinhole::project                 src/CameraModels/Pinhole.cpp:30-39
// The pose product x3Dc = Rcw*x3Dw + tcw (cv::Mat) is an input: it is taken
// from the caller, as the drop-in shim keeps it on the host.
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "ref_fma.h"

namespace {

constexpr int kCols = 64, kRows = 48;  // FRAME_GRID_COLS / FRAME_GRID_ROWS (include/Frame.h:47-48)
constexpr int kThHigh = 100, kHisto = 30;

struct Kp {
    float x, y;
    int octave;
    float angle;
};

struct Grid {
    std::vector<size_t> cell[kCols][kRows];
};

int dist256(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 8; ++i) {
        int32_t pa, pb;
        std::memcpy(&pa, a + 4 * i, 4);
        std::memcpy(&pb, b + 4 * i, 4);
        unsigned v = (unsigned)(pa ^ pb);
        v = v - ((v >> 1) & 0x55555555);
        v = (v & 0x33333333) + ((v >> 2) & 0x33333333);
        d += (((v + (v >> 4)) & 0xF0F0F0F) * 0x1010101) >> 24;
    }
    return d;
}

bool pos_in_grid(const Kp& kp, float minX, float minY, float invW, float invH, int& px, int& py) {
    px = (int)std::round((kp.x - minX) * invW);  // std::round(float)
    py = (int)std::round((kp.y - minY) * invH);
    return !(px < 0 || px >= kCols || py < 0 || py >= kRows);
}

void assign_grid(const std::vector<Kp>& kps, float minX, float minY, float invW, float invH, Grid& g) {
    for (int i = 0; i < (int)kps.size(); ++i) {
        int px, py;
        if (pos_in_grid(kps[i], minX, minY, invW, invH, px, py)) g.cell[px][py].push_back(i);
    }
}

std::vector<size_t> features_in_area(const Grid& g, const std::vector<Kp>& kps, float minX, float minY, float invW,
                                     float invH, const float& x, const float& y, const float& r, int minLevel,
                                     int maxLevel) {
    std::vector<size_t> v;
    const float factorX = r, factorY = r;
    const int nMinCellX = std::max(0, (int)std::floor((x - minX - factorX) * invW));
    if (nMinCellX >= kCols) return v;
    const int nMaxCellX = std::min(kCols - 1, (int)std::ceil((x - minX + factorX) * invW));
    if (nMaxCellX < 0) return v;
    const int nMinCellY = std::max(0, (int)std::floor((y - minY - factorY) * invH));
    if (nMinCellY >= kRows) return v;
    const int nMaxCellY = std::min(kRows - 1, (int)std::ceil((y - minY + factorY) * invH));
    if (nMaxCellY < 0) return v;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
        for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
            const std::vector<size_t>& vCell = g.cell[ix][iy];
            for (size_t j = 0; j < vCell.size(); j++) {
                const Kp& kp = kps[vCell[j]];
                if (bCheckLevels) {
                    if (kp.octave < minLevel) continue;
                    if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                }
                const float distx = kp.x - x, disty = kp.y - y;
                if (std::fabs(distx) < factorX && std::fabs(disty) < factorY) v.push_back(vCell[j]);
            }
        }
    return v;
}

void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
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
}

std::vector<Kp> make_kps(int n, const float* x, const float* y, const int* oct, const float* ang) {
    std::vector<Kp> k(n);
    for (int i = 0; i < n; ++i) k[i] = Kp{x[i], y[i], oct ? oct[i] : 0, ang ? ang[i] : 0.f};
    return k;
}

}  // namespace

// AssignFeaturesToGrid as CSR: cell (ix, iy) = ix*48 + iy, cell_off[3073].
extern "C" int oracle_assign_grid(const float* x, const float* y, int n, float minX, float minY, float invW,
                                  float invH, int* cell_off, int* cell_idx) {
    Grid g;
    assign_grid(make_kps(n, x, y, nullptr, nullptr), minX, minY, invW, invH, g);
    int c = 0;
    cell_off[0] = 0;
    for (int ix = 0; ix < kCols; ++ix)
        for (int iy = 0; iy < kRows; ++iy) {
            for (size_t j : g.cell[ix][iy]) cell_idx[c++] = (int)j;
            cell_off[ix * kRows + iy + 1] = c;
        }
    return c;
}

// GetFeaturesInArea on a grid built from the same keypoints; returns the count.
extern "C" int oracle_features_in_area(const float* kx, const float* ky, const int* oct, int n, float minX,
                                       float minY, float invW, float invH, float x, float y, float r, int minLevel,
                                       int maxLevel, int* out) {
    const std::vector<Kp> kps = make_kps(n, kx, ky, oct, nullptr);
    Grid g;
    assign_grid(kps, minX, minY, invW, invH, g);
    const std::vector<size_t> v = features_in_area(g, kps, minX, minY, invW, invH, x, y, r, minLevel, maxLevel);
    for (size_t i = 0; i < v.size(); ++i) out[i] = (int)v[i];
    return (int)v.size();
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono), Nleft == -1.
//  cur_*: CurrentFrame.mvKeysUn (x, y, octave, angle), mDescriptors, blocked[i2]
//         = mvpMapPoints[i2] && Observations() > 0 on entry, mvuRight (or NULL).
//  last_*: per LastFrame point i: flags bit0 = has a MapPoint and not an
//         outlier, bit1 = that MapPoint's Observations() > 0; x3Dc = Rcw*x3Dw+tcw;
//         octave = LastFrame.mvKeys[i].octave, angle = mvKeysUn[i].angle;
//         mp_desc = pMP->GetDescriptor().
//  out: match[i2] = LastFrame index whose MapPoint mvpMapPoints[i2] holds on
//       return, -2 = set to NULL by the rotation filter, -1 = untouched.
extern "C" int oracle_search_by_projection(
    int n_cur, const float* cx_, const float* cy_, const int* coct, const float* cang, const uint8_t* cdesc,
    const uint8_t* cblocked, const float* curight, float minX, float maxX, float minY, float maxY, float invW,
    float invH, const float* scale_factors, float fx, float fy, float cxp, float cyp, float mbf, int n_last,
    const uint8_t* lflags, const float* x3dc, const int* loct, const float* lang, const uint8_t* mpdesc, float th,
    int bForward, int bBackward, int check_ori, int* match) {
    const std::vector<Kp> kps = make_kps(n_cur, cx_, cy_, coct, cang);
    Grid g;
    assign_grid(kps, minX, minY, invW, invH, g);
    std::vector<int> mp(n_cur, -1);          // index of the LastFrame point whose MapPoint is stored
    std::vector<char> blocked(cblocked, cblocked + n_cur);  // mvpMapPoints[i2] && Observations()>0
    std::vector<int> rotHist[kHisto];
    const float factor = 1.0f / kHisto;
    int nmatches = 0;
    for (int i = 0; i < n_last; i++) {
        if (!(lflags[i] & 1)) continue;
        const float xc = x3dc[3 * i], yc = x3dc[3 * i + 1], zc = x3dc[3 * i + 2];
        const float invzc = 1.0 / zc;
        if (invzc < 0) continue;
        const float u = fx * xc / zc + cxp, v = fy * yc / zc + cyp;
        if (u < minX || u > maxX) continue;
        if (v < minY || v > maxY) continue;
        const int nLastOctave = loct[i];
        const float radius = th * scale_factors[nLastOctave];
        std::vector<size_t> vIndices2;
        if (bForward)
            vIndices2 = features_in_area(g, kps, minX, minY, invW, invH, u, v, radius, nLastOctave, -1);
        else if (bBackward)
            vIndices2 = features_in_area(g, kps, minX, minY, invW, invH, u, v, radius, 0, nLastOctave);
        else
            vIndices2 = features_in_area(g, kps, minX, minY, invW, invH, u, v, radius, nLastOctave - 1,
                                         nLastOctave + 1);
        if (vIndices2.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (blocked[i2]) continue;
            if (curight && curight[i2] > 0) {
                const float ur = ref_fmaf(-mbf, invzc, u);  // fused in ORBmatcher.cc.o
                const float er = std::fabs(ur - curight[i2]);
                if (er > radius) continue;
            }
            const int dist = dist256(mpdesc + 32 * (size_t)i, cdesc + 32 * i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = (int)i2;
            }
        }
        if (bestDist <= kThHigh) {
            mp[bestIdx2] = i;
            blocked[bestIdx2] = (lflags[i] & 2) ? 1 : 0;  // the stored MapPoint's Observations() > 0
            nmatches++;
            if (check_ori) {
                float rot = lang[i] - kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == kHisto) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    std::vector<char> nulled(n_cur, 0);
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, kHisto, ind1, ind2, ind3);
        for (int b = 0; b < kHisto; b++)
            if (b != ind1 && b != ind2 && b != ind3)
                for (int idx : rotHist[b]) {
                    nulled[idx] = 1;
                    nmatches--;
                }
    }
    for (int i2 = 0; i2 < n_cur; ++i2) match[i2] = nulled[i2] ? -2 : mp[i2];
    return nmatches;
}

// CameraModels: Pinhole::project (Pinhole.cpp:30-33) and
// KannalaBrandt8::project(const cv::Point3f&) (KannalaBrandt8.cpp:33-48),
// the host libm as the reference calls it (atan2f, sqrtf; `cos(psi)` with a
// float psi under `using namespace std` is std::cos(float)).
static void project_cam(const float* kb8, float fx, float fy, float cxp, float cyp, float x, float y, float z,
                        float& u, float& v) {
    if (!kb8) {
        u = fx * x / z + cxp;
        v = fy * y / z + cyp;
        return;
    }
    // the seven multiply-adds KannalaBrandt8.cpp.o fuses: x*x + y*y, the four
    // r terms, u and v
    const float x2_plus_y2 = ref_fmaf(x, x, y * y);
    const float theta = atan2f(sqrtf(x2_plus_y2), z);
    const float psi = atan2f(y, x);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r =
        ref_fmaf(kb8[3], theta9, ref_fmaf(kb8[2], theta7, ref_fmaf(kb8[1], theta5, ref_fmaf(kb8[0], theta3, theta))));
    u = ref_fmaf(fx * r, std::cos(psi), cxp);
    v = ref_fmaf(fy * r, std::sin(psi), cyp);
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) with a two-camera
// CurrentFrame (CurrentFrame.Nleft != -1, src/ORBmatcher.cc:1985-2175),
// restated with the reference's indexing: mvpMapPoints / mDescriptors over N
// = Nleft + Nright, mvKeys in mGrid, mvKeysRight in mGridRight
// (right-relative).  kb8 = KannalaBrandt8 k1..k4 (NULL = Pinhole).  LastFrame
// point i: x3Dc, x3Dr = mTrl * x3Dc, octave, angle, descriptor, flags (bit0
// MapPoint and not an outlier, bit1 Observations() > 0).  match[N]: LastFrame
// index held by mvpMapPoints[idx], -2 = NULL by the rotation filter, -1.
extern "C" int oracle_search_by_projection2(
    int n_left, const float* lx, const float* ly, const int* loct_c, const float* lang_c, int n_right, const float* rx,
    const float* ry, const int* roct_c, const float* rang_c, const uint8_t* cdesc, const uint8_t* cblocked,
    float minX, float maxX, float minY, float maxY, float invW, float invH, const float* scale_factors, float fx,
    float fy, float cxp, float cyp, const float* kb8, int n_last, const uint8_t* lflags, const float* x3dc,
    const float* x3dr, const int* loct, const float* lang, const uint8_t* mpdesc, float th, int bForward,
    int bBackward, int check_ori, int* match) {
    const int Nleft = n_left, N = n_left + n_right;
    const std::vector<Kp> keys = make_kps(n_left, lx, ly, loct_c, lang_c);            // mvKeys
    const std::vector<Kp> keysRight = make_kps(n_right, rx, ry, roct_c, rang_c);     // mvKeysRight
    Grid grid, gridRight;
    assign_grid(keys, minX, minY, invW, invH, grid);
    assign_grid(keysRight, minX, minY, invW, invH, gridRight);
    std::vector<int> mp(N, -1);
    std::vector<char> blocked(cblocked, cblocked + N);
    std::vector<int> rotHist[kHisto];
    const float factor = 1.0f / kHisto;
    int nmatches = 0;
    auto area = [&](const Grid& g, const std::vector<Kp>& k, float u, float v, float radius, int nLastOctave) {
        if (bForward) return features_in_area(g, k, minX, minY, invW, invH, u, v, radius, nLastOctave, -1);
        if (bBackward) return features_in_area(g, k, minX, minY, invW, invH, u, v, radius, 0, nLastOctave);
        return features_in_area(g, k, minX, minY, invW, invH, u, v, radius, nLastOctave - 1, nLastOctave + 1);
    };
    auto bin_of = [&](float a, float b) {
        float rot = a - b;
        if (rot < 0.0) rot += 360.0f;
        int bin = (int)std::round(rot * factor);
        if (bin == kHisto) bin = 0;
        return bin;
    };
    for (int i = 0; i < n_last; i++) {
        if (!(lflags[i] & 1)) continue;
        const float xc = x3dc[3 * i], yc = x3dc[3 * i + 1], zc = x3dc[3 * i + 2];
        const float invzc = 1.0 / zc;
        if (invzc < 0) continue;
        float u, v;
        project_cam(kb8, fx, fy, cxp, cyp, xc, yc, zc, u, v);
        if (u < minX || u > maxX) continue;
        if (v < minY || v > maxY) continue;
        const int nLastOctave = loct[i];
        const float radius = th * scale_factors[nLastOctave];
        const std::vector<size_t> vIndices2 = area(grid, keys, u, v, radius, nLastOctave);
        if (vIndices2.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (blocked[i2]) continue;
            const int dist = dist256(mpdesc + 32 * (size_t)i, cdesc + 32 * i2);
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = (int)i2;
            }
        }
        if (bestDist <= kThHigh) {
            mp[bestIdx2] = i;
            blocked[bestIdx2] = (lflags[i] & 2) ? 1 : 0;
            nmatches++;
            if (check_ori) rotHist[bin_of(lang[i], keys[bestIdx2].angle)].push_back(bestIdx2);
        }
        // the right camera (:2084-2150)
        float ur, vr;
        project_cam(kb8, fx, fy, cxp, cyp, x3dr[3 * i], x3dr[3 * i + 1], x3dr[3 * i + 2], ur, vr);
        const std::vector<size_t> vIndicesR = area(gridRight, keysRight, ur, vr, radius, nLastOctave);
        bestDist = 256;
        bestIdx2 = -1;
        for (size_t i2 : vIndicesR) {
            if (blocked[i2 + Nleft]) continue;
            const int dist = dist256(mpdesc + 32 * (size_t)i, cdesc + 32 * (i2 + Nleft));
            if (dist < bestDist) {
                bestDist = dist;
                bestIdx2 = (int)i2;
            }
        }
        if (bestDist <= kThHigh) {
            mp[bestIdx2 + Nleft] = i;
            blocked[bestIdx2 + Nleft] = (lflags[i] & 2) ? 1 : 0;
            nmatches++;
            if (check_ori) rotHist[bin_of(lang[i], keysRight[bestIdx2].angle)].push_back(bestIdx2 + Nleft);
        }
    }
    std::vector<char> nulled(N, 0);
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, kHisto, ind1, ind2, ind3);
        for (int b = 0; b < kHisto; b++)
            if (b != ind1 && b != ind2 && b != ind3)
                for (int idx : rotHist[b]) {
                    nulled[idx] = 1;
                    nmatches--;
                }
    }
    for (int k = 0; k < N; ++k) match[k] = nulled[k] ? -2 : mp[k];
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const
// set<MapPoint*>& sAlreadyFound, th, ORBdist) (src/ORBmatcher.cc:2180-2300),
// the relocalization guided search (Tracking.cc:5857, 5871).  Per KF MapPoint i
// (GetMapPointMatches() order) the caller evaluates the MapPoint state:
// kf_flags bit0 = pMP && !isBad() && !sAlreadyFound.count(pMP); x3dc =
// Rcw*x3Dw+tcw; dist = {cv::norm(x3Dw-Ow), GetMinDistanceInvariance(),
// GetMaxDistanceInvariance()}; level = PredictScale(dist3D, &CurrentFrame);
// kf_angle = pKF->mvKeysUn[i].angle; mp_desc = GetDescriptor().  Frame:
// mvKeysUn (x, y, octave, angle), descriptors, blocked = mvpMapPoints[i2] !=
// NULL on entry.  Output match[i2] = KF index stored by this call, -2 = set to
// NULL by the rotation filter, -1 = untouched.  Returns nmatches.
extern "C" int oracle_search_reloc(int n_cur, const float* cx_, const float* cy_, const int* coct, const float* cang,
                                   const uint8_t* cdesc, const uint8_t* cblocked, float minX, float maxX, float minY,
                                   float maxY, float invW, float invH, const float* scale_factors, int nlevels,
                                   float fx, float fy, float cxp, float cyp, int n_kf, const uint8_t* kf_flags,
                                   const float* x3dc, const float* dist, const int* level, const float* kf_angle,
                                   const uint8_t* mpdesc, float th, int ORBdist, int check_ori, int* match) {
    const std::vector<Kp> kps = make_kps(n_cur, cx_, cy_, coct, cang);
    Grid g;
    assign_grid(kps, minX, minY, invW, invH, g);
    std::vector<int> mp(n_cur, -1);
    std::vector<char> nonnull(n_cur, 0);  // CurrentFrame.mvpMapPoints[i2] != NULL
    for (int i = 0; i < n_cur; ++i) nonnull[i] = cblocked && cblocked[i] ? 1 : 0;
    std::vector<int> rotHist[kHisto];
    for (int i = 0; i < kHisto; i++) rotHist[i].reserve(500);
    const float factor = 1.0f / kHisto;
    int nmatches = 0;
    for (int i = 0; i < n_kf; i++) {
        if (!(kf_flags[i] & 1)) continue;  // pMP, !isBad(), !sAlreadyFound.count(pMP)
        const float xc = x3dc[3 * i], yc = x3dc[3 * i + 1], zc = x3dc[3 * i + 2];
        const float u = fx * xc / zc + cxp, v = fy * yc / zc + cyp;  // Pinhole::project
        if (u < minX || u > maxX) continue;
        if (v < minY || v > maxY) continue;
        const float dist3D = dist[3 * i];
        const float maxDistance = dist[3 * i + 2], minDistance = dist[3 * i + 1];
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = level[i];
        if (nPredictedLevel < 0 || nPredictedLevel >= nlevels) continue;  // PredictScale's clamp range
        const float radius = th * scale_factors[nPredictedLevel];
        const std::vector<size_t> vIndices2 = features_in_area(g, kps, minX, minY, invW, invH, u, v, radius,
                                                               nPredictedLevel - 1, nPredictedLevel + 1);
        if (vIndices2.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            if (nonnull[i2]) continue;
            const int d = dist256(mpdesc + 32 * (size_t)i, cdesc + 32 * i2);
            if (d < bestDist) {
                bestDist = d;
                bestIdx2 = (int)i2;
            }
        }
        if (bestDist <= ORBdist && bestIdx2 >= 0) {  // (ORBdist < 256: bestIdx2 >= 0 whenever bestDist <= ORBdist)
            mp[bestIdx2] = i;
            nonnull[bestIdx2] = 1;
            nmatches++;
            if (check_ori) {
                float rot = kf_angle[i] - kps[bestIdx2].angle;
                if (rot < 0.0) rot += 360.0f;
                int bin = (int)std::round(rot * factor);
                if (bin == kHisto) bin = 0;
                rotHist[bin].push_back(bestIdx2);
            }
        }
    }
    std::vector<char> nulled(n_cur, 0);
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, kHisto, ind1, ind2, ind3);
        for (int b = 0; b < kHisto; b++)
            if (b != ind1 && b != ind2 && b != ind3)
                for (int idx : rotHist[b]) {
                    nulled[idx] = 1;
                    nmatches--;
                }
    }
    for (int i2 = 0; i2 < n_cur; ++i2) match[i2] = nulled[i2] ? -2 : mp[i2];
    return nmatches;
}

// ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints,
// th, bFarPoints, thFarPoints) (src/ORBmatcher.cc:44-145), F.Nleft == -1, the
// local-map search of Tracking::SearchLocalPoints (Tracking.cc:5119/5211).
// Per MapPoint iMP (vector order) the caller evaluates the MapPoint state:
// mp_flags bit0 = it is searched (mbTrackInView && !(bFarPoints && mTrackDepth
// > thFarPoints) && !isBad()), bit1 = Observations() > 0; mTrackProjX/Y,
// mTrackProjXR, mTrackViewCos, mnTrackScaleLevel, GetDescriptor().  Frame:
// mvKeysUn (x, y, octave), descriptors, blocked = mvpMapPoints[idx] &&
// Observations() > 0 on entry, mvuRight (nullable).  Output match[idx] = iMP
// stored in F.mvpMapPoints[idx] by this call, or -1.  Returns nmatches.
extern "C" int oracle_search_local(int n_cur, const float* cx_, const float* cy_, const int* coct,
                                   const uint8_t* cdesc, const uint8_t* cblocked, const float* curight, float minX,
                                   float minY, float invW, float invH, const float* scale_factors, float nnratio,
                                   float th, int n_mp, const uint8_t* mp_flags, const float* px, const float* py,
                                   const float* pxr, const float* view_cos, const int* level, const uint8_t* mpdesc,
                                   int* match) {
    std::vector<float> ang(n_cur, 0.f);
    const std::vector<Kp> kps = make_kps(n_cur, cx_, cy_, coct, ang.data());
    Grid g;
    assign_grid(kps, minX, minY, invW, invH, g);
    std::vector<char> blocked(cblocked, cblocked + n_cur);
    for (int i = 0; i < n_cur; ++i) match[i] = -1;
    const bool bFactor = th != 1.0;
    int nmatches = 0;
    for (int iMP = 0; iMP < n_mp; iMP++) {
        if (!(mp_flags[iMP] & 1)) continue;
        const int nPredictedLevel = level[iMP];
        float r = view_cos[iMP] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos
        if (bFactor) r *= th;
        const std::vector<size_t> vIndices =
            features_in_area(g, kps, minX, minY, invW, invH, px[iMP], py[iMP], r * scale_factors[nPredictedLevel],
                             nPredictedLevel - 1, nPredictedLevel);
        if (vIndices.empty()) continue;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        for (size_t idx : vIndices) {
            if (blocked[idx]) continue;
            if (curight && curight[idx] > 0) {
                const float er = std::fabs(pxr[iMP] - curight[idx]);
                if (er > r * scale_factors[nPredictedLevel]) continue;
            }
            const int dist = dist256(mpdesc + 32 * (size_t)iMP, cdesc + 32 * idx);
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestLevel2 = bestLevel;
                bestLevel = kps[idx].octave;
                bestIdx = (int)idx;
            } else if (dist < bestDist2) {
                bestLevel2 = kps[idx].octave;
                bestDist2 = dist;
            }
        }
        if (bestDist <= kThHigh) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
            if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                match[bestIdx] = iMP;
                blocked[bestIdx] = (mp_flags[iMP] & 2) ? 1 : 0;
                nmatches++;
            }
        }
    }
    return nmatches;
}

// The same function on a two-camera Frame (F.Nleft != -1, src/ORBmatcher.cc:
// 44-214).  Restated with the reference's indexing: one mvpMapPoints /
// mDescriptors space of N = Nleft + Nright entries, left keypoints mvKeys
// [0, Nleft) in mGrid, right keypoints mvKeysRight in mGridRight with
// right-relative indices (Frame.cc:661-674).  blocked[N] = mvpMapPoints[i]
// && Observations() > 0 on entry; l2r[Nleft] / r2l[Nright] =
// mvLeftToRightMatch / mvRightToLeftMatch.  MapPoint flags: bit0 =
// mbTrackInView (and not far, not bad), bit1 = Observations() > 0, bit2 =
// mbTrackInViewR (and not far, not bad).  match[N] = the MapPoint index left
// in mvpMapPoints by the call or -1; returns nmatches.
extern "C" int oracle_search_local2(int n_left, const float* lx, const float* ly, const int* loct, int n_right,
                                    const float* rx, const float* ry, const int* roct, const uint8_t* desc,
                                    const uint8_t* blocked_in, const int* l2r, const int* r2l, float minX, float minY,
                                    float invW, float invH, const float* scale_factors, float nnratio, float th,
                                    int n_mp, const uint8_t* mp_flags, const float* px, const float* py,
                                    const float* view_cos, const int* level, const float* pxr, const float* pyr,
                                    const float* view_cos_r, const int* level_r, const uint8_t* mpdesc, int* match) {
    const int Nleft = n_left, N = n_left + n_right;
    const std::vector<Kp> keys = make_kps(n_left, lx, ly, loct, nullptr);        // mvKeys
    const std::vector<Kp> keysRight = make_kps(n_right, rx, ry, roct, nullptr);  // mvKeysRight
    Grid grid, gridRight;
    assign_grid(keys, minX, minY, invW, invH, grid);
    assign_grid(keysRight, minX, minY, invW, invH, gridRight);
    std::vector<char> blocked(blocked_in, blocked_in + N);  // mvpMapPoints[i] && ->Observations() > 0
    for (int i = 0; i < N; ++i) match[i] = -1;
    const bool bFactor = th != 1.0;
    int nmatches = 0;
    auto store = [&](int i, int iMP) {  // F.mvpMapPoints[i] = pMP
        match[i] = iMP;
        blocked[i] = (mp_flags[iMP] & 2) ? 1 : 0;
    };
    for (int iMP = 0; iMP < n_mp; iMP++) {
        const bool inView = mp_flags[iMP] & 1, inViewR = mp_flags[iMP] & 4;
        if (!inView && !inViewR) continue;
        if (inView) {
            const int nPredictedLevel = level[iMP];
            float r = view_cos[iMP] > 0.998 ? 2.5f : 4.0f;  // RadiusByViewingCos
            if (bFactor) r *= th;
            const std::vector<size_t> vIndices =
                features_in_area(grid, keys, minX, minY, invW, invH, px[iMP], py[iMP], r * scale_factors[nPredictedLevel],
                                 nPredictedLevel - 1, nPredictedLevel);
            if (!vIndices.empty()) {
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (size_t idx : vIndices) {
                    if (blocked[idx]) continue;
                    const int dist = dist256(mpdesc + 32 * (size_t)iMP, desc + 32 * idx);
                    if (dist < bestDist) {
                        bestDist2 = bestDist;
                        bestDist = dist;
                        bestLevel2 = bestLevel;
                        bestLevel = keys[idx].octave;
                        bestIdx = (int)idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = keys[idx].octave;
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= kThHigh) {
                    if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;  // the next MapPoint
                    if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                        store(bestIdx, iMP);
                        if (l2r && l2r[bestIdx] != -1) {  // also the stereo observation in the right camera
                            store(l2r[bestIdx] + Nleft, iMP);
                            nmatches++;
                        }
                        nmatches++;
                    }
                }
            }
        }
        if (inViewR) {
            const int nPredictedLevel = level_r[iMP];
            if (nPredictedLevel != -1) {
                const float r = view_cos_r[iMP] > 0.998 ? 2.5f : 4.0f;
                const std::vector<size_t> vIndices =
                    features_in_area(gridRight, keysRight, minX, minY, invW, invH, pxr[iMP], pyr[iMP],
                                     r * scale_factors[nPredictedLevel], nPredictedLevel - 1, nPredictedLevel);
                if (vIndices.empty()) continue;
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (size_t idx : vIndices) {
                    if (blocked[idx + Nleft]) continue;
                    const int dist = dist256(mpdesc + 32 * (size_t)iMP, desc + 32 * (idx + Nleft));
                    if (dist < bestDist) {
                        bestDist2 = bestDist;
                        bestDist = dist;
                        bestLevel2 = bestLevel;
                        bestLevel = keysRight[idx].octave;
                        bestIdx = (int)idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = keysRight[idx].octave;
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= kThHigh) {
                    if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
                    if (r2l && r2l[bestIdx] != -1) {
                        store(r2l[bestIdx], iMP);
                        nmatches++;
                    }
                    store(bestIdx + Nleft, iMP);
                    nmatches++;
                }
            }
        }
    }
    return nmatches;
}

// ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12,
// windowSize) (src/ORBmatcher.cc:705-814), the monocular initializer's matcher
// (Tracking::MonocularInitialization, Tracking.cc:3023/3111: ORBmatcher(0.9,
// true), windowSize 100).  F1 = mInitialFrame.mvKeysUn (x, y, octave, angle)
// + mDescriptors; prev_xy = vbPrevMatched (in/out, [n1][2]); F2 =
// mCurrentFrame.mvKeysUn + mDescriptors, its mGrid built by
// AssignFeaturesToGrid from the same keypoints.  Output m12 = vnMatches12
// [n1]; returns nmatches.
extern "C" int oracle_search_for_initialization(int n1, const float* x1, const float* y1, const int* oct1,
                                                const float* ang1, const uint8_t* desc1, float* prev_xy, int n2,
                                                const float* x2, const float* y2, const int* oct2, const float* ang2,
                                                const uint8_t* desc2, float minX, float minY, float invW, float invH,
                                                int windowSize, float nnratio, int check_ori, int* m12) {
    const int TH_LOW = 50;
    const std::vector<Kp> K1 = make_kps(n1, x1, y1, oct1, ang1), K2 = make_kps(n2, x2, y2, oct2, ang2);
    Grid g;
    assign_grid(K2, minX, minY, invW, invH, g);
    int nmatches = 0;
    std::vector<int> vnMatches12(n1, -1);
    std::vector<int> rotHist[kHisto];
    for (int i = 0; i < kHisto; i++) rotHist[i].reserve(500);
    const float factor = 1.0f / kHisto;
    std::vector<int> vMatchedDistance(n2, INT_MAX);
    std::vector<int> vnMatches21(n2, -1);
    for (int i1 = 0; i1 < n1; i1++) {
        const Kp kp1 = K1[i1];
        const int level1 = kp1.octave;
        if (level1 > 0) continue;
        const float px = prev_xy[2 * i1], py = prev_xy[2 * i1 + 1];
        const float r = (float)windowSize;
        std::vector<size_t> vIndices2 = features_in_area(g, K2, minX, minY, invW, invH, px, py, r, level1, level1);
        if (vIndices2.empty()) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : vIndices2) {
            const int dist = dist256(desc1 + (size_t)32 * i1, desc2 + (size_t)32 * i2);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) {
                bestDist2 = bestDist;
                bestDist = dist;
                bestIdx2 = (int)i2;
            } else if (dist < bestDist2) {
                bestDist2 = dist;
            }
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) {
                    vnMatches12[vnMatches21[bestIdx2]] = -1;
                    nmatches--;
                }
                vnMatches12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (check_ori) {
                    float rot = K1[i1].angle - K2[bestIdx2].angle;
                    if (rot < 0.0) rot += 360.0f;
                    int bin = (int)std::round(rot * factor);
                    if (bin == kHisto) bin = 0;
                    rotHist[bin].push_back(i1);
                }
            }
        }
    }
    if (check_ori) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, kHisto, ind1, ind2, ind3);
        for (int i = 0; i < kHisto; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (size_t j = 0; j < rotHist[i].size(); j++) {
                const int idx1 = rotHist[i][j];
                if (vnMatches12[idx1] >= 0) {
                    vnMatches12[idx1] = -1;
                    nmatches--;
                }
            }
        }
    }
    for (int i1 = 0; i1 < n1; i1++)
        if (vnMatches12[i1] >= 0) {
            prev_xy[2 * i1] = K2[vnMatches12[i1]].x;
            prev_xy[2 * i1 + 1] = K2[vnMatches12[i1]].y;
        }
    for (int i1 = 0; i1 < n1; i1++) m12[i1] = vnMatches12[i1];
    return nmatches;
}
