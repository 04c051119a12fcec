// oracle/orb_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of ORB_SLAM3::ORBextractor (reference src/ORBextractor.cc,
// include/ORBextractor.h) on top of the OpenCV primitives restated in
// cvprim.cpp.  Parity status: "parity unpinned" — the reference ships no
// golden vectors for this path and cannot be built here (OpenCV absent,
// SURVEY.md §8c); this restatement follows the cited lines and is locked by
// KATs + the exhaustive libm checks in tests/.
//
// Determinism: DistributeOctTree's phase-2 sort of (size, ExtractorNode*)
// breaks ties by heap address (src/ORBextractor.cc:679-683).  We adopt the
// canonical rule of SURVEY.md B.1: addresses are taken from a monotone bump
// allocator, i.e. ties are ordered by node creation sequence.
#include <algorithm>
#include <list>
#include <utility>

#include "cvprim.h"
#include "oracle_api.h"
#include "ref_fma.h"

namespace oracle {

static const int PATCH_SIZE = 31;       // ORBextractor.cc:70
static const int HALF_PATCH_SIZE = 15;  // :71
static const int EDGE_THRESHOLD = 19;   // :72

static const signed char kPattern[512 * 2] = {
#include "orb_pattern.inc"
};

struct KP {  // cv::KeyPoint
    float x, y, size, angle, response;
    int octave, class_id;
};

// ---------------------------------------------------------------- FAST (A.3)
// cv::FAST(roi, kps, threshold, nonmax=true) on a sub-image [x0,x1)x[y0,y1)
// of `img`.  Detection window rows/cols [3, dim-4] of the ROI, NMS against
// the 8 neighbours inside the ROI's score buffer (neighbours that were not
// detected in THIS call count as 0).  Row-major output, ROI coordinates.
static void fast_roi(const ImageU8& img, int x0, int y0, int x1, int y1, int threshold,
                     std::vector<KP>& out) {
    out.clear();
    threshold = std::min(std::max(threshold, 0), 255);
    const int rw = x1 - x0, rh = y1 - y0;
    if (rw < 7 || rh < 7) return;
    std::vector<int> score((size_t)rw * rh, 0);
    for (int i = 3; i < rh - 3; ++i)
        for (int j = 3; j < rw - 3; ++j) {
            const uint8_t* p = img.row(y0 + i) + x0 + j;
            int S = fast_score(p, img.w);
            if (S > threshold) score[(size_t)i * rw + j] = S - 1;
        }
    for (int i = 3; i < rh - 3; ++i)
        for (int j = 3; j < rw - 3; ++j) {
            int s = score[(size_t)i * rw + j];
            if (!s) continue;
            bool keep = true;
            for (int dy = -1; dy <= 1 && keep; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    if (!dx && !dy) continue;
                    if (!(s > score[(size_t)(i + dy) * rw + j + dx])) { keep = false; break; }
                }
            if (keep) out.push_back(KP{(float)j, (float)i, 7.f, -1.f, (float)s, 0, -1});
        }
}

// ---------------------------------------------------------------- octree
// ExtractorNode (include/ORBextractor.h:31-42) + DivideNode (ORBextractor.cc:479-535).
struct Node {
    std::vector<KP> vKeys;
    int ULx, ULy, URx, URy, BLx, BLy, BRx, BRy;
    std::list<Node>::iterator lit;
    bool bNoMore = false;
    long seq = 0;  // creation sequence == bump-allocator address order (B.1)
};

static thread_local long g_seq = 0;  // per thread: the bench runs the oracle on several host threads

static void divide_node(const Node& P, Node& n1, Node& n2, Node& n3, Node& n4) {
    const int halfX = (int)std::ceil((float)(P.URx - P.ULx) / 2);
    const int halfY = (int)std::ceil((float)(P.BRy - P.ULy) / 2);
    n1.ULx = P.ULx; n1.ULy = P.ULy;
    n1.URx = P.ULx + halfX; n1.URy = P.ULy;
    n1.BLx = P.ULx; n1.BLy = P.ULy + halfY;
    n1.BRx = P.ULx + halfX; n1.BRy = P.ULy + halfY;
    n2.ULx = n1.URx; n2.ULy = n1.URy;
    n2.URx = P.URx; n2.URy = P.URy;
    n2.BLx = n1.BRx; n2.BLy = n1.BRy;
    n2.BRx = P.URx; n2.BRy = P.ULy + halfY;
    n3.ULx = n1.BLx; n3.ULy = n1.BLy;
    n3.URx = n1.BRx; n3.URy = n1.BRy;
    n3.BLx = P.BLx; n3.BLy = P.BLy;
    n3.BRx = n1.BRx; n3.BRy = P.BLy;
    n4.ULx = n3.URx; n4.ULy = n3.URy;
    n4.URx = n2.BRx; n4.URy = n2.BRy;
    n4.BLx = n3.BRx; n4.BLy = n3.BRy;
    n4.BRx = P.BRx; n4.BRy = P.BRy;
    for (const KP& kp : P.vKeys) {
        if (kp.x < n1.URx) {
            if (kp.y < n1.BRy) n1.vKeys.push_back(kp);
            else n3.vKeys.push_back(kp);
        } else if (kp.y < n1.BRy) n2.vKeys.push_back(kp);
        else n4.vKeys.push_back(kp);
    }
    if (n1.vKeys.size() == 1) n1.bNoMore = true;
    if (n2.vKeys.size() == 1) n2.bNoMore = true;
    if (n3.vKeys.size() == 1) n3.bNoMore = true;
    if (n4.vKeys.size() == 1) n4.bNoMore = true;
}

typedef std::pair<int, long> SizeKey;  // (size, creation seq) — canonical (size, pointer)

// SURVEY §8c diagnostic: the reference orders equal-size nodes by heap address
// (B.1).  0 = creation order (a bump allocator: the canonical rule the HIP
// path follows), 1 = reverse creation order, 2 = a pseudo-random address per
// node (freed list nodes reused by malloc).
static int g_tie_mode = 0;
static long tie_key(long seq) {
    if (g_tie_mode == 1) return -seq;
    if (g_tie_mode == 2) {
        unsigned long long z = (unsigned long long)seq + 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return (long)((z ^ (z >> 31)) >> 1);
    }
    return seq;
}

// ORBextractor::DistributeOctTree (src/ORBextractor.cc:537-761).
static std::vector<KP> distribute_octtree(const std::vector<KP>& keys, int minX, int maxX, int minY,
                                          int maxY, int N) {
    const int nIni = (int)std::round((float)(maxX - minX) / (maxY - minY));
    const float hX = (float)(maxX - minX) / nIni;
    std::list<Node> lNodes;
    std::vector<Node*> ini(nIni);
    for (int i = 0; i < nIni; ++i) {
        Node ni;
        ni.ULx = (int)(hX * (float)i); ni.ULy = 0;
        ni.URx = (int)(hX * (float)(i + 1)); ni.URy = 0;
        ni.BLx = ni.ULx; ni.BLy = maxY - minY;
        ni.BRx = ni.URx; ni.BRy = maxY - minY;
        ni.seq = g_seq++;
        lNodes.push_back(ni);
        ini[i] = &lNodes.back();
    }
    for (const KP& kp : keys) ini[(size_t)(kp.x / hX)]->vKeys.push_back(kp);
    for (auto lit = lNodes.begin(); lit != lNodes.end();) {
        if (lit->vKeys.size() == 1) { lit->bNoMore = true; ++lit; }
        else if (lit->vKeys.empty()) lit = lNodes.erase(lit);
        else ++lit;
    }
    bool bFinish = false;
    // (size, node) pairs; the node is identified by its seq, looked up via map
    std::vector<std::pair<SizeKey, Node*>> vSize;
    auto push_child = [&](Node& c, std::vector<std::pair<SizeKey, Node*>>* rec, int* nToExpand) {
        if (c.vKeys.empty()) return;
        c.seq = g_seq++;
        lNodes.push_front(c);
        if (c.vKeys.size() > 1) {
            if (nToExpand) ++*nToExpand;
            rec->push_back({SizeKey((int)c.vKeys.size(), tie_key(lNodes.front().seq)), &lNodes.front()});
            lNodes.front().lit = lNodes.begin();
        }
    };
    while (!bFinish) {
        int prevSize = (int)lNodes.size();
        auto lit = lNodes.begin();
        int nToExpand = 0;
        vSize.clear();
        while (lit != lNodes.end()) {
            if (lit->bNoMore) { ++lit; continue; }
            Node n1, n2, n3, n4;
            divide_node(*lit, n1, n2, n3, n4);
            push_child(n1, &vSize, &nToExpand);
            push_child(n2, &vSize, &nToExpand);
            push_child(n3, &vSize, &nToExpand);
            push_child(n4, &vSize, &nToExpand);
            lit = lNodes.erase(lit);
        }
        if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) {
            bFinish = true;
        } else if ((int)lNodes.size() + nToExpand * 3 > N) {
            while (!bFinish) {
                prevSize = (int)lNodes.size();
                auto vPrev = vSize;
                vSize.clear();
                std::sort(vPrev.begin(), vPrev.end(),
                          [](const std::pair<SizeKey, Node*>& a, const std::pair<SizeKey, Node*>& b) {
                              return a.first < b.first;
                          });
                for (int j = (int)vPrev.size() - 1; j >= 0; --j) {
                    Node n1, n2, n3, n4;
                    divide_node(*vPrev[j].second, n1, n2, n3, n4);
                    push_child(n1, &vSize, nullptr);
                    push_child(n2, &vSize, nullptr);
                    push_child(n3, &vSize, nullptr);
                    push_child(n4, &vSize, nullptr);
                    lNodes.erase(vPrev[j].second->lit);
                    if ((int)lNodes.size() >= N) break;
                }
                if ((int)lNodes.size() >= N || (int)lNodes.size() == prevSize) bFinish = true;
            }
        }
    }
    std::vector<KP> res;
    for (auto& n : lNodes) {
        const KP* best = &n.vKeys[0];
        float maxResponse = best->response;
        for (size_t k = 1; k < n.vKeys.size(); ++k)
            if (n.vKeys[k].response > maxResponse) { best = &n.vKeys[k]; maxResponse = best->response; }
        res.push_back(*best);
    }
    return res;
}

// ---------------------------------------------------------------- extractor
struct OrbParams {
    int nfeatures, nlevels, iniTh, minTh;
    double scaleFactor;
    std::vector<float> scale, invScale, sigma2, invSigma2;
    std::vector<int> perLevel, umax;
};

// ORBextractor::ORBextractor (src/ORBextractor.cc:408-468).
static OrbParams make_params(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh) {
    OrbParams P;
    P.nfeatures = nfeatures; P.nlevels = nlevels; P.iniTh = iniTh; P.minTh = minTh;
    P.scaleFactor = scaleFactor;  // double member (include/ORBextractor.h:97)
    P.scale.resize(nlevels); P.sigma2.resize(nlevels);
    P.scale[0] = 1.0f; P.sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; ++i) {
        P.scale[i] = (float)(P.scale[i - 1] * P.scaleFactor);
        P.sigma2[i] = P.scale[i] * P.scale[i];
    }
    P.invScale.resize(nlevels); P.invSigma2.resize(nlevels);
    for (int i = 0; i < nlevels; ++i) {
        P.invScale[i] = 1.0f / P.scale[i];
        P.invSigma2[i] = 1.0f / P.sigma2[i];
    }
    P.perLevel.resize(nlevels);
    float factor = (float)(1.0f / P.scaleFactor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; ++l) {
        P.perLevel[l] = cv_round(nDesired);
        sum += P.perLevel[l];
        nDesired *= factor;
    }
    P.perLevel[nlevels - 1] = std::max(nfeatures - sum, 0);
    P.umax.resize(HALF_PATCH_SIZE + 1);
    int v, v0, vmax = cv_floor(HALF_PATCH_SIZE * std::sqrt(2.f) / 2 + 1);
    int vmin = cv_ceil(HALF_PATCH_SIZE * std::sqrt(2.f) / 2);
    const double hp2 = HALF_PATCH_SIZE * HALF_PATCH_SIZE;
    for (v = 0; v <= vmax; ++v) P.umax[v] = cv_round(std::sqrt(hp2 - v * v));
    for (v = HALF_PATCH_SIZE, v0 = 0; v >= vmin; --v) {
        while (P.umax[v0] == P.umax[v0 + 1]) ++v0;
        P.umax[v] = v0;
        ++v0;
    }
    return P;
}

// IC_Angle (src/ORBextractor.cc:75-102).
static float ic_angle(const ImageU8& img, float px, float py, const std::vector<int>& umax) {
    int m_01 = 0, m_10 = 0;
    const int cx = cv_round(px), cy = cv_round(py);
    for (int u = -HALF_PATCH_SIZE; u <= HALF_PATCH_SIZE; ++u) m_10 += u * img.at(cx + u, cy);
    for (int v = 1; v <= HALF_PATCH_SIZE; ++v) {
        int v_sum = 0, d = umax[v];
        for (int u = -d; u <= d; ++u) {
            int vp = img.at(cx + u, cy + v), vm = img.at(cx + u, cy - v);
            v_sum += vp - vm;
            m_10 += u * (vp + vm);
        }
        m_01 += v * v_sum;
    }
    return fast_atan2((float)m_01, (float)m_10);
}

// computeOrbDescriptor (src/ORBextractor.cc:105-145): cosf/sinf from host glibc.
static void orb_descriptor(const KP& kpt, const ImageU8& img, uint8_t* desc) {
    const float factorPI = (float)(M_PI / 180.f);
    float angle = (float)kpt.angle * factorPI;
    float a = cosf(angle), b = sinf(angle);
    const int cx = cv_round(kpt.x), cy = cv_round(kpt.y);
    auto get = [&](int idx) -> int {
        int x = kPattern[2 * idx], y = kPattern[2 * idx + 1];
        // GET_VALUE (:116-118): the left product fused (ORBextractor.cc.o)
        int r = cv_round(ref_fmaf((float)x, b, (float)y * a));
        int c = cv_round(ref_fmaf((float)x, a, -((float)y * b)));
        return img.at(cx + c, cy + r);
    };
    for (int i = 0; i < 32; ++i) {
        int val = 0;
        for (int bit = 0; bit < 8; ++bit) {
            int t0 = get(16 * i + 2 * bit), t1 = get(16 * i + 2 * bit + 1);
            val |= (t0 < t1) << bit;
        }
        desc[i] = (uint8_t)val;
    }
}

struct OrbResult {
    std::vector<ImageU8> pyramid, blurred;
    std::vector<std::vector<KP>> candidates;  // per level, level-relative (minus minBorder)
    std::vector<std::vector<KP>> levelKps;    // per level, after octree + orientation (level coords)
    std::vector<KP> kps;
    std::vector<uint8_t> desc;
    int monoIndex = 0;
};

// ORBextractor::operator() (src/ORBextractor.cc:1068-1150) with
// ComputePyramid (:1152-1177) and ComputeKeyPointsOctTree (:763-878).
static int orb_extract(const ImageU8& image, const OrbParams& P, int lap0, int lap1, OrbResult& R) {
    if (image.w == 0 || image.h == 0) return -1;
    g_seq = 0;
    const int L = P.nlevels;
    R.pyramid.assign(L, ImageU8());
    for (int l = 0; l < L; ++l) {
        float sc = P.invScale[l];
        int w = cv_round((float)image.w * sc), h = cv_round((float)image.h * sc);
        if (l == 0) R.pyramid[0] = image;
        else resize_linear_u8(R.pyramid[l - 1], R.pyramid[l], w, h);
    }
    R.candidates.assign(L, {});
    R.levelKps.assign(L, {});
    const float W = 30;
    for (int level = 0; level < L; ++level) {
        const ImageU8& im = R.pyramid[level];
        const int minBorderX = EDGE_THRESHOLD - 3, minBorderY = minBorderX;
        const int maxBorderX = im.w - EDGE_THRESHOLD + 3, maxBorderY = im.h - EDGE_THRESHOLD + 3;
        std::vector<KP>& toDist = R.candidates[level];
        const float width = (float)(maxBorderX - minBorderX), height = (float)(maxBorderY - minBorderY);
        const int nCols = (int)(width / W), nRows = (int)(height / W);
        if (nCols <= 0 || nRows <= 0) return -2;
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        std::vector<KP> cell;
        for (int i = 0; i < nRows; ++i) {
            const float iniY = (float)(minBorderY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= maxBorderY - 3) continue;
            if (maxY > maxBorderY) maxY = (float)maxBorderY;
            for (int j = 0; j < nCols; ++j) {
                const float iniX = (float)(minBorderX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= maxBorderX - 6) continue;
                if (maxX > maxBorderX) maxX = (float)maxBorderX;
                fast_roi(im, (int)iniX, (int)iniY, (int)maxX, (int)maxY, P.iniTh, cell);
                if (cell.empty()) fast_roi(im, (int)iniX, (int)iniY, (int)maxX, (int)maxY, P.minTh, cell);
                for (KP kp : cell) {
                    kp.x += j * wCell;
                    kp.y += i * hCell;
                    toDist.push_back(kp);
                }
            }
        }
        std::vector<KP> kps =
            distribute_octtree(toDist, minBorderX, maxBorderX, minBorderY, maxBorderY, P.perLevel[level]);
        const int scaledPatchSize = (int)(PATCH_SIZE * P.scale[level]);
        for (KP& kp : kps) {
            kp.x += minBorderX;
            kp.y += minBorderY;
            kp.octave = level;
            kp.size = (float)scaledPatchSize;
        }
        R.levelKps[level] = kps;
    }
    for (int level = 0; level < L; ++level)
        for (KP& kp : R.levelKps[level]) kp.angle = ic_angle(R.pyramid[level], kp.x, kp.y, P.umax);

    int nk = 0;
    for (int level = 0; level < L; ++level) nk += (int)R.levelKps[level].size();
    R.kps.assign(nk, KP{0, 0, 0, 0, 0, 0, 0});
    R.desc.assign((size_t)nk * 32, 0);
    R.blurred.assign(L, ImageU8());
    int monoIndex = 0, stereoIndex = nk - 1;
    for (int level = 0; level < L; ++level) {
        std::vector<KP>& kps = R.levelKps[level];
        gaussian_blur_u8(R.pyramid[level], R.blurred[level], 7, 2.0);
        if (kps.empty()) continue;
        std::vector<uint8_t> d(kps.size() * 32);
        for (size_t i = 0; i < kps.size(); ++i) orb_descriptor(kps[i], R.blurred[level], &d[i * 32]);
        const float scale = P.scale[level];
        for (size_t i = 0; i < kps.size(); ++i) {
            KP kp = kps[i];
            if (level != 0) { kp.x *= scale; kp.y *= scale; }
            int slot;
            if (kp.x >= lap0 && kp.x <= lap1) slot = stereoIndex--;
            else slot = monoIndex++;
            R.kps[slot] = kp;
            std::memcpy(&R.desc[(size_t)slot * 32], &d[i * 32], 32);
        }
    }
    R.monoIndex = monoIndex;
    return monoIndex;
}

}  // namespace oracle

using namespace oracle;

extern "C" int oracle_orb_extract(const uint8_t* img, int w, int h, int stride, int nfeatures, float scaleFactor,
                                  int nlevels, int iniTh, int minTh, int lap0, int lap1, plvi_keypoint* kps,
                                  uint8_t* desc, int cap, int* n) {
    ImageU8 im;
    im.create(w, h);
    for (int y = 0; y < h; ++y) std::memcpy(im.row(y), img + (size_t)y * stride, w);
    OrbParams P = make_params(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    OrbResult R;
    int mono = orb_extract(im, P, lap0, lap1, R);
    if (mono < 0) { *n = 0; return mono; }
    *n = (int)R.kps.size();
    if ((int)R.kps.size() > cap) return -3;
    for (size_t i = 0; i < R.kps.size(); ++i) {
        const KP& k = R.kps[i];
        kps[i] = plvi_keypoint{k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id};
    }
    std::memcpy(desc, R.desc.data(), R.desc.size());
    return mono;
}

// Diagnostics for per-stage parity: pyramid level `level` (u8, w*h), its 7x7
// blur, and the level's octree input candidate list (x,y,response relative to
// minBorder) / octree output (level coords, angle filled).
extern "C" int oracle_orb_stage(const uint8_t* img, int w, int h, int nfeatures, float scaleFactor, int nlevels,
                                int iniTh, int minTh, int level, uint8_t* pyr, uint8_t* blur, int* lw, int* lh,
                                float* cand, int cand_cap, int* ncand, float* lvkps, int lv_cap, int* nlv) {
    ImageU8 im;
    im.create(w, h);
    std::memcpy(im.px.data(), img, (size_t)w * h);
    OrbParams P = make_params(nfeatures, scaleFactor, nlevels, iniTh, minTh);
    OrbResult R;
    int rc = orb_extract(im, P, 0, 0, R);
    if (rc < 0) return rc;
    const ImageU8& L = R.pyramid[level];
    *lw = L.w; *lh = L.h;
    if (pyr) std::memcpy(pyr, L.px.data(), L.px.size());
    if (blur) std::memcpy(blur, R.blurred[level].px.data(), L.px.size());
    const auto& c = R.candidates[level];
    *ncand = (int)c.size();
    for (int i = 0; i < (int)c.size() && i < cand_cap; ++i) {
        cand[3 * i] = c[i].x; cand[3 * i + 1] = c[i].y; cand[3 * i + 2] = c[i].response;
    }
    const auto& k = R.levelKps[level];
    *nlv = (int)k.size();
    for (int i = 0; i < (int)k.size() && i < lv_cap; ++i) {
        lvkps[4 * i] = k[i].x; lvkps[4 * i + 1] = k[i].y; lvkps[4 * i + 2] = k[i].response;
        lvkps[4 * i + 3] = k[i].angle;
    }
    return 0;
}

extern "C" void oracle_orb_set_tie_mode(int mode) { g_tie_mode = mode; }

extern "C" void oracle_orb_params(int nfeatures, float scaleFactor, int nlevels, float* scale, int* perLevel,
                                  int* umax) {
    OrbParams P = make_params(nfeatures, scaleFactor, nlevels, 20, 7);
    for (int i = 0; i < nlevels; ++i) { scale[i] = P.scale[i]; perLevel[i] = P.perLevel[i]; }
    for (int i = 0; i <= HALF_PATCH_SIZE; ++i) umax[i] = P.umax[i];
}

extern "C" void oracle_resize_u8(const uint8_t* src, int sw, int sh, uint8_t* dst, int dw, int dh) {
    ImageU8 s, d;
    s.create(sw, sh);
    std::memcpy(s.px.data(), src, (size_t)sw * sh);
    resize_linear_u8(s, d, dw, dh);
    std::memcpy(dst, d.px.data(), (size_t)dw * dh);
}

extern "C" void oracle_gaussian_blur_u8(const uint8_t* src, int w, int h, int ksize, double sigma, uint8_t* dst) {
    ImageU8 s, d;
    s.create(w, h);
    std::memcpy(s.px.data(), src, (size_t)w * h);
    gaussian_blur_u8(s, d, ksize, sigma);
    std::memcpy(dst, d.px.data(), (size_t)w * h);
}

extern "C" void oracle_set_compat(unsigned bits) { g_compat = bits; }
extern "C" unsigned oracle_get_compat(void) { return g_compat; }
extern "C" double oracle_cv_exp_table(double x) { return cv_exp_table(x); }
extern "C" void oracle_gaussian_taps_u8(int ksize, double sigma, int* taps) { gaussian_taps_u8(ksize, sigma, taps); }
extern "C" void oracle_gaussian_kernel_f64(int ksize, double sigma, double* k) { gaussian_kernel_f64(ksize, sigma, k); }
extern "C" float oracle_fast_atan2(float y, float x) { return fast_atan2(y, x); }
extern "C" int oracle_fast_score(const uint8_t* p, int stride) { return fast_score(p, stride); }
