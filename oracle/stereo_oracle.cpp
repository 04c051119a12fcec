// oracle/stereo_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the rectified-stereo steps of the stereo Frame
// constructors (src/Frame.cc:95-140, :225-300), "parity unpinned" (no
// reference test pins them):
//   Frame::ComputeStereoMatches          src/Frame.cc:1228-1406
//   Frame::ComputeStereoMatches_Lines    src/Frame.cc:1408-1492
//   Frame::lineSegmentOverlapStereo      src/Frame.cc:1494-1529
//   Frame::filterLineSegmentDisparity    src/Frame.cc:1531-1542
//   getLineCoords / LineIterator         src/gridStructure.cpp:32-40, src/LineIterator.cpp:31-73
//   GridStructure(rows, cols) / at       src/gridStructure.cpp:45-65
//   normalize                            include/LineMatcher.h:48-53
// LineMatcher::matchGrid is the restatement in match_oracle.cpp.
// cv::Mat::rowRange/colRange windows, convertTo(CV_16S), Mat - scalar and
// cv::norm(NORM_L1) are restated on plain arrays (integer arithmetic; the
// 11x11 windows of extractor keypoints never leave their level image).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <list>
#include <utility>
#include <vector>

#include "oracle_api.h"
#include "ref_fma.h"

extern "C" int oracle_match_grid2(const int* lines1, const uint8_t* desc1, int n1, int cols, int rows,
                                  const int* cell_off, const int* cell_idx, const uint8_t* desc2,
                                  const double* directions2, int n2, int w0, int w1, int h0, int h1,
                                  int range_hint, int* matches_12);

namespace {

constexpr int kThHigh = 100, kThLow = 50;   // ORBmatcher::TH_HIGH / TH_LOW (src/ORBmatcher.cc:39-40)
constexpr int kGridRows = 48, kGridCols = 64;  // FRAME_GRID_ROWS / COLS (include/Frame.h:47-48)

int dist256(const uint8_t* a, const uint8_t* b) {  // ORBmatcher::DescriptorDistance (:2350-2366)
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

struct Level {
    const uint8_t* p;
    int w, h;
    int at(int x, int y) const { return p[(size_t)y * w + x]; }
};

// LineIterator (src/LineIterator.cpp:31-73), all state in double / int
void line_coords(double x1, double y1, double x2, double y2, std::list<std::pair<int, int>>& out) {
    out.clear();
    const bool steep = std::abs(y2 - y1) > std::abs(x2 - x1);
    if (steep) { std::swap(x1, y1); std::swap(x2, y2); }
    if (x1 > x2) { std::swap(x1, x2); std::swap(y1, y2); }
    const double dx = x2 - x1, dy = std::abs(y2 - y1);
    double error = dx / 2.0;
    const int ystep = (y1 < y2) ? 1 : -1;
    int x = static_cast<int>(x1), y = static_cast<int>(y1);
    const int maxX = static_cast<int>(x2);
    while (x <= maxX) {
        out.push_back(steep ? std::make_pair(y, x) : std::make_pair(x, y));
        error -= dy;
        if (error < 0) { y += ystep; error += dx; }
        x++;
    }
}

double overlap_stereo(double spl_obs, double epl_obs, double spl_proj, double epl_proj) {  // :1494-1529
    double overlap = 1.f;
    float lineHorizTh = 0.1;
    if (std::fabs(epl_obs - spl_obs) > lineHorizTh) {
        double sln = std::min(spl_obs, epl_obs);
        double eln = std::max(spl_obs, epl_obs);
        double spn = std::min(spl_proj, epl_proj);
        double epn = std::max(spl_proj, epl_proj);
        double length = eln - spn;
        if ((epn < sln) || (spn > eln))
            overlap = 0.f;
        else {
            if ((epn > eln) && (spn < sln))
                overlap = eln - sln;
            else
                overlap = std::min(eln, epn) - std::max(sln, spn);
        }
        if (length > 0.01f)
            overlap = overlap / length;
        else
            overlap = 0.f;
        if (overlap > 1.f) overlap = 1.f;
    }
    return overlap;
}

}  // namespace

// getLineCoords (src/gridStructure.cpp:32-40): the pixels of LineIterator in
// order, as (x, y) pairs; tests/test_ref_grid.py compares it with the
// reference's own LineIterator.cpp (oracle/_ref).
extern "C" int oracle_line_coords(double x1, double y1, double x2, double y2, int* out_xy, int cap) {
    std::list<std::pair<int, int>> l;
    line_coords(x1, y1, x2, y2, l);
    int n = 0;
    for (auto& p : l) {
        if (n < cap) { out_xy[2 * n] = p.first; out_xy[2 * n + 1] = p.second; }
        ++n;
    }
    return n;
}

// Frame::ComputeStereoMatches (src/Frame.cc:1228-1406).  kps*: mvKeys /
// mvKeysRight (cv::KeyPoint layout), desc*: 32 B rows; pyramids: level l of
// each side at pyr + lvl_off[l], lvl_w[l] x lvl_h[l] (mvImagePyramid of the
// left / right extractor); scale / inv_scale: mvScaleFactors /
// mvInvScaleFactors.  Outputs mvuRight / mvDepth (nL floats).  Returns the
// number of left keypoints that keep a depth.
extern "C" int oracle_stereo_match(const plvi_keypoint* kpsL, const uint8_t* descL, int nL, const plvi_keypoint* kpsR,
                                   const uint8_t* descR, int nR, const uint8_t* pyrL, const uint8_t* pyrR,
                                   const long long* lvl_off, const int* lvl_w, const int* lvl_h, const float* scale,
                                   const float* inv_scale, float mb, float mbf, float* uright, float* depth) {
    std::vector<float> mvuRight(nL, -1.0f), mvDepth(nL, -1.0f);
    const int thOrbDist = (kThHigh + kThLow) / 2;
    const int nRows = lvl_h[0];
    std::vector<std::vector<size_t>> vRowIndices(nRows, std::vector<size_t>());
    for (int iR = 0; iR < nR; iR++) {
        const plvi_keypoint& kp = kpsR[iR];
        const float& kpY = kp.y;
        // kpY + r / kpY - r with r = 2*scale: fused in Frame.cc.o
        const int maxr = std::ceil(ref_fmaf(2.0f, scale[kp.octave], kpY));
        const int minr = std::floor(ref_fmaf(-2.0f, scale[kp.octave], kpY));
        if (minr < 0 || maxr >= nRows) return -1;  // vRowIndices[yi] out of range (UB in the reference)
        for (int yi = minr; yi <= maxr; yi++) vRowIndices[yi].push_back(iR);
    }
    const float minZ = mb;
    const float minD = 0;
    const float maxD = mbf / minZ;
    std::vector<std::pair<int, int>> vDistIdx;
    for (int iL = 0; iL < nL; iL++) {
        const plvi_keypoint& kpL = kpsL[iL];
        const int& levelL = kpL.octave;
        const float& vL = kpL.y;
        const float& uL = kpL.x;
        if ((size_t)vL >= (size_t)nRows) return -1;
        const std::vector<size_t>& vCandidates = vRowIndices[(size_t)vL];
        if (vCandidates.empty()) continue;
        const float minU = uL - maxD;
        const float maxU = uL - minD;
        if (maxU < 0) continue;
        int bestDist = kThHigh;
        size_t bestIdxR = 0;
        const uint8_t* dL = descL + (size_t)iL * 32;
        for (size_t iC = 0; iC < vCandidates.size(); iC++) {
            const size_t iR = vCandidates[iC];
            const plvi_keypoint& kpR = kpsR[iR];
            if (kpR.octave < levelL - 1 || kpR.octave > levelL + 1) continue;
            const float& uR = kpR.x;
            if (uR >= minU && uR <= maxU) {
                const int dist = dist256(dL, descR + iR * 32);
                if (dist < bestDist) {
                    bestDist = dist;
                    bestIdxR = iR;
                }
            }
        }
        if (bestDist < thOrbDist) {
            const float uR0 = kpsR[bestIdxR].x;
            const float scaleFactor = inv_scale[kpL.octave];
            const float scaleduL = std::round(kpL.x * scaleFactor);
            const float scaledvL = std::round(kpL.y * scaleFactor);
            const float scaleduR0 = std::round(uR0 * scaleFactor);
            const int w = 5;
            const Level IL0{pyrL + lvl_off[kpL.octave], lvl_w[kpL.octave], lvl_h[kpL.octave]};
            const Level IR0{pyrR + lvl_off[kpL.octave], lvl_w[kpL.octave], lvl_h[kpL.octave]};
            const int r0 = (int)scaledvL - w, c0 = (int)scaleduL - w;
            // rowRange/colRange bounds (CV_Assert in the reference)
            if (r0 < 0 || r0 + 2 * w + 1 > IL0.h || c0 < 0 || c0 + 2 * w + 1 > IL0.w) return -1;
            // IL.convertTo(IL, CV_16S); IL = IL - IL.at<short>(w,w)
            short IL[11][11];
            const int cL = IL0.at(c0 + w, r0 + w);
            for (int y = 0; y < 11; ++y)
                for (int x = 0; x < 11; ++x) IL[y][x] = (short)(IL0.at(c0 + x, r0 + y) - cL);
            int bestDist = INT_MAX;
            int bestincR = 0;
            const int L = 5;
            std::vector<float> vDists(2 * L + 1);
            const float iniu = scaleduR0 + L - w;
            const float endu = scaleduR0 + L + w + 1;
            if (iniu < 0 || endu >= IR0.w) continue;
            for (int incR = -L; incR <= +L; incR++) {
                const int cr0 = (int)(scaleduR0 + incR - w);
                if (cr0 < 0 || cr0 + 2 * w + 1 > IR0.w) return -1;
                const int cR = IR0.at(cr0 + w, r0 + w);
                long long s = 0;  // cv::norm(IL, IR, NORM_L1) over CV_16S
                for (int y = 0; y < 11; ++y)
                    for (int x = 0; x < 11; ++x) s += std::abs(IL[y][x] - (short)(IR0.at(cr0 + x, r0 + y) - cR));
                float dist = (float)(double)s;
                if (dist < bestDist) {
                    bestDist = dist;
                    bestincR = incR;
                }
                vDists[L + incR] = dist;
            }
            if (bestincR == -L || bestincR == L) continue;
            const float dist1 = vDists[L + bestincR - 1];
            const float dist2 = vDists[L + bestincR];
            const float dist3 = vDists[L + bestincR + 1];
            const float deltaR = (dist1 - dist3) / (2.0f * ref_fmaf(-2.0f, dist2, dist1 + dist3));
            if (deltaR < -1 || deltaR > 1) continue;
            float bestuR = scale[kpL.octave] * ((float)scaleduR0 + (float)bestincR + deltaR);
            float disparity = (uL - bestuR);
            if (disparity >= minD && disparity < maxD) {
                if (disparity <= 0) {
                    disparity = 0.01;
                    bestuR = uL - 0.01;
                }
                mvDepth[iL] = mbf / disparity;
                mvuRight[iL] = bestuR;
                vDistIdx.push_back(std::pair<int, int>(bestDist, iL));
            }
        }
    }
    if (!vDistIdx.empty()) {  // the reference reads vDistIdx[0] of an empty vector (UB); nothing to reject
        std::sort(vDistIdx.begin(), vDistIdx.end());
        const float median = vDistIdx[vDistIdx.size() / 2].first;
        const float thDist = 1.5f * 1.4f * median;
        for (int i = (int)vDistIdx.size() - 1; i >= 0; i--) {
            if (vDistIdx[i].first < thDist)
                break;
            else {
                mvuRight[vDistIdx[i].second] = -1;
                mvDepth[vDistIdx[i].second] = -1;
            }
        }
    }
    int n = 0;
    for (int i = 0; i < nL; ++i) {
        uright[i] = mvuRight[i];
        depth[i] = mvDepth[i];
        n += mvDepth[i] > 0;
    }
    return n;
}

// KeyLine fields used here (descriptor_custom.hpp:107-146): start/end points.
struct KLpts {
    float sx, sy, ex, ey;
};

// Frame::ComputeStereoMatches_Lines (src/Frame.cc:1408-1492) for a frame of
// width x height (inv_width / inv_height, :208-209).  kl*: 4 floats per line
// (startPointX, startPointY, endPointX, endPointY) of mvKeys_Line,
// mvKeysRight_Line and mvKeysUn_Line.  Outputs: matches_12 (nL ints, the
// matchGrid result), disparity / depth (2 floats per left line: mvDisparity_l,
// mvDepth_l), le (3 doubles per left line: mvle_l).  Returns the number of
// lines with a depth.
extern "C" int oracle_stereo_lines(const float* klL, const uint8_t* descL, int nL, const float* klR,
                                   const uint8_t* descR, int nR, const float* klUn, int width, int height,
                                   float mbf, int range_hint, int* matches_12, float* disparity, float* depth,
                                   double* le) {
    for (int i = 0; i < nL; ++i) {
        matches_12[i] = -1;
        disparity[2 * i] = disparity[2 * i + 1] = -1;
        depth[2 * i] = depth[2 * i + 1] = -1.0f;
        le[3 * i] = le[3 * i + 1] = le[3 * i + 2] = 0;
    }
    if (nL == 0 || nR == 0) return 0;
    const KLpts* L = reinterpret_cast<const KLpts*>(klL);
    const KLpts* R = reinterpret_cast<const KLpts*>(klR);
    const KLpts* U = reinterpret_cast<const KLpts*>(klUn);
    const double inv_width = kGridCols / static_cast<double>(width);
    const double inv_height = kGridRows / static_cast<double>(height);
    std::vector<int> coords(4 * (size_t)nL);
    for (int i = 0; i < nL; ++i) {  // make_pair(make_pair(double, double), ...) -> line_2d (int)
        coords[4 * i] = (int)(L[i].sx * inv_width);
        coords[4 * i + 1] = (int)(L[i].sy * inv_height);
        coords[4 * i + 2] = (int)(L[i].ex * inv_width);
        coords[4 * i + 3] = (int)(L[i].ey * inv_height);
    }
    std::vector<std::vector<std::vector<int>>> grid(kGridCols, std::vector<std::vector<int>>(kGridRows));
    std::vector<double> directions(2 * (size_t)nR);
    std::list<std::pair<int, int>> lc;
    for (int idx = 0; idx < nR; ++idx) {
        double vx = (R[idx].ex - R[idx].sx) * inv_width, vy = (R[idx].ey - R[idx].sy) * inv_height;
        const double magnitude = std::sqrt(ref_fma(vx, vx, vy * vy));  // fused in Frame.cc.o
        vx /= magnitude;
        vy /= magnitude;
        directions[2 * idx] = vx;
        directions[2 * idx + 1] = vy;
        line_coords(R[idx].sx * inv_width, R[idx].sy * inv_height, R[idx].ex * inv_width, R[idx].ey * inv_height, lc);
        for (const auto& p : lc)
            if (p.first >= 0 && p.first < kGridCols && p.second >= 0 && p.second < kGridRows)
                grid[p.first][p.second].push_back(idx);
    }
    std::vector<int> off(kGridCols * kGridRows + 1, 0), idxs;
    for (int x = 0; x < kGridCols; ++x)
        for (int y = 0; y < kGridRows; ++y) {
            idxs.insert(idxs.end(), grid[x][y].begin(), grid[x][y].end());
            off[x * kGridRows + y + 1] = (int)idxs.size();
        }
    if (idxs.empty()) idxs.push_back(0);
    oracle_match_grid2(coords.data(), descL, nL, kGridCols, kGridRows, off.data(), idxs.data(), descR,
                       directions.data(), nR, 7, 0, 2, 2, range_hint, matches_12);
    int nd = 0;
    for (int i1 = 0; i1 < nL; ++i1) {
        const int i2 = matches_12[i1];
        if (i2 < 0) continue;
        const double spl0 = L[i1].sx, spl1 = L[i1].sy, epl0 = L[i1].ex, epl1 = L[i1].ey;
        double spr0 = R[i2].sx, spr1 = R[i2].sy, epr0 = R[i2].ex, epr1 = R[i2].ey;
        const double overlap = overlap_stereo(spl1, epl1, spr1, epr1);
        // sp_r << ..., sp_l(1), 1.0;  then ep_r << ... reads the UPDATED sp_r
        spr0 = ref_fma(spr0, spl1 - epr1, epr0 * (spr1 - spl1)) / (spr1 - epr1);  // left products fused
        spr1 = spl1;
        epr0 = ref_fma(spr0, epl1 - epr1, epr0 * (spr1 - epl1)) / (spr1 - epr1);
        epr1 = epl1;
        double disp_s = spl0 - spr0, disp_e = epl0 - epr0;  // filterLineSegmentDisparity (:1531-1542)
        float lsMinDispRatio = 0.7;
        if (std::min(disp_s, disp_e) / std::max(disp_s, disp_e) < lsMinDispRatio) {
            disp_s = -1.0;
            disp_e = -1.0;
        }
        int minDisp = 1;
        float lineHorizTh = 0.1;
        float stereoOverlapTh = 0.75;
        if (disp_s >= minDisp && disp_e >= minDisp && std::abs(spl1 - epl1) > lineHorizTh &&
            std::abs(spr1 - epr1) > lineHorizTh && overlap > stereoOverlapTh) {
            disparity[2 * i1] = (float)disp_s;
            disparity[2 * i1 + 1] = (float)disp_e;
            depth[2 * i1] = mbf / float(disp_s);
            depth[2 * i1 + 1] = mbf / float(disp_e);
            nd++;
        }
    }
    for (int i = 0; i < nL; i++) {  // mvle_l from mvKeysUn_Line (Eigen cross + normalise)
        const double a0 = U[i].sx, a1 = U[i].sy, a2 = 1.0, b0 = U[i].ex, b1 = U[i].ey, b2 = 1.0;
        double l0 = a1 * b2 - a2 * b1, l1 = a2 * b0 - a0 * b2, l2 = ref_fma(a0, b1, -(a1 * b0));
        const double s = std::sqrt(ref_fma(l0, l0, l1 * l1));  // both fused in Frame.cc.o
        le[3 * i] = l0 / s;
        le[3 * i + 1] = l1 / s;
        le[3 * i + 2] = l2 / s;
    }
    return nd;
}
