// orb_pipeline.hip — host orchestration of the ORB kernels and the ORB part
// of the C-ABI (include/plvi_frontend.h).  Geometry is derived exactly as
// ORBextractor does (src/ORBextractor.cc:408-468 ctor, :1152-1177 pyramid,
// :763-878 cells/borders, :537-561 octree roots).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "orb_device.h"
#include "plvi_common.h"
#include "orb_kernels.hpp"

namespace plvi {

static inline int cv_round_h(float v) { return (int)lrintf(v); }
static inline int cv_round_h(double v) { return (int)lrint(v); }
static inline int cv_floor_h(float v) { int i = (int)v; return i - (i > v); }
static inline int cv_ceil_h(float v) { int i = (int)v; return i + (i < v); }

// cv::resize INTER_LINEAR 8U column coefficients (imgproc/src/resize.cpp,
// OpenCV 4.2: scale_x = 1/inv_scale_x, fx = (float)((dx+0.5)*scale_x-0.5),
// sx = cvFloor(fx), border clamps, cvRound(... * INTER_RESIZE_COEF_SCALE)),
// packed for orb_pyramid_kernel; dx >= xmax columns use S[sx] * 2048 only.
static int append_xtab(std::vector<uint32_t>& tab, int sw, int dw) {
    const double scale_x = 1. / ((double)dw / sw);
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor_h(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        const bool clampR = sx + 1 >= sw;
        if (clampR && sx >= sw - 1) { fx = 0; sx = sw - 1; }
        const int a0 = cv_round_h((1.f - fx) * 2048), a1 = cv_round_h(fx * 2048);
        if (sx > 1023 || a0 + a1 < 2047 || a0 + a1 > 2049) return PLVI_E_BADARG;
        tab.push_back(pyr_xtab_pack(sx, a0, a1, clampR));
    }
    return PLVI_OK;
}

// Split [0, n) into the fewest pieces whose interior cuts are taken from
// `cand` (ascending) and that all satisfy fits(a, b), as even as possible:
// the smallest piece-length bound for which the greedy cut still needs no
// more pieces.  out = {0, cuts..., n}.
template <class Fits>
static int plan_splits(int n, const std::vector<int>& cand, Fits fits, std::vector<int>& out) {
    auto greedy = [&](int bound, std::vector<int>& o) {
        o.assign(1, 0);
        int a = 0;
        while (a < n) {
            int b = -1;
            if (fits(a, n) && n - a <= bound) b = n;
            else
                for (int c : cand)
                    if (c > a && fits(a, c) && c - a <= bound) b = c;
            if (b < 0) return false;
            o.push_back(b);
            a = b;
        }
        return true;
    };
    std::vector<int> best;
    if (!greedy(n, best)) return PLVI_E_BADARG;
    const size_t k = best.size();
    int lo = 1, hi = n;  // smallest bound with <= k pieces
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        std::vector<int> t;
        if (greedy(mid, t) && t.size() <= k) hi = mid;
        else lo = mid + 1;
    }
    if (!greedy(lo, out)) out = best;
    return PLVI_OK;
}

struct OrbPipeline {
    plvi_orb_params prm{};
    int W = 0, H = 0, Bcap = 0, device = 0, L = 0;
    hipStream_t stream = nullptr;
    std::vector<float> scale, invScale, sigma2, invSigma2;
    std::vector<int> quota, umax;
    std::vector<OrbLevelDev> lv;
    std::vector<OrbCellDev> cells;
    std::vector<OrbStripDev> strips;
    int taps[7]{};
    int resizeGeneric = 0;  // A.1 vertical-pass switch (PLVI_COMPAT_RESIZE_V_GENERIC)
    int kpCapFrame = 0, nodeCapMax = 0;
    size_t pyrBytesFrameTotal = 0, blurBytesTotal = 0;
    int listFrame = 0, listMax = 0;  // NMS candidate lists: entries per frame, largest level
    DevBuf d_lv, d_cells, d_strips, d_xtab, pyr, blur, score, clist, ccount, rectCnt, lvkp, lvdesc, okp, odesc, ocount,
        omono, err, staging;
    size_t pyrSmem = 0;  // orb_pyramid_kernel LDS: column table + source-level row rings
    int xtabN = 0, pyrFrameLds = 0;
    int octLcap = 0;      // candidates a (frame, level) octree wave stages in LDS
    int octLdsMax = kOctListLds;  // PLVI_ORB_OCT_LDS (0: every level's octree scans its list in memory)
    size_t octSmem = 0;   // orb_octree_kernel dynamic LDS
    // batches of at most this many frames build the pyramid level by level
    // (orb_resize_level_kernel, one launch per level) instead of streaming it
    // (PLVI_PYR_LEVELWISE overrides)
    int pyrLevelwiseMax = 1024;
    int lastFrames = 0;
    // Level 0 of the pyramid (mvImagePyramid[0]) is the input frame itself.
    // When the batch's rows are packed (row stride = width) it stays a view of
    // the caller's frames (no copy: 1 B/pixel of level-0 writes less in the
    // blur + FAST pass); otherwise, or with PLVI_ORB_L0_COPY=1, blur + FAST
    // copies it into the pyramid buffer as before.
    const uint8_t* l0view = nullptr;  // the last run's frames when level 0 is a view
    size_t l0fs = 0;
    bool l0forceCopy = false;
    // Stage timing with HIP events on the launch stream (bench.py roofline).
    static constexpr int kStages = 7, kRing = 512;
    bool prof = false;
    int profRuns = 0;
    std::vector<hipEvent_t> evs;  // kRing * (kStages+1)

    ~OrbPipeline() {
        for (auto e : evs) (void)hipEventDestroy(e);
        for (auto e : kev) (void)hipEventDestroy(e);
        for (auto e : kevP) (void)hipEventDestroy(e);
        if (stream) (void)hipStreamDestroy(stream);
    }

    // Per-launch timing of the blur + FAST kernel (bench.py's roofline kernel)
    // and of the pyramid kernel (roofline_pyramid): an event pair on the
    // launch stream around every launch while enabled.
    static constexpr int kKRing = 4096;
    bool ktime = false;
    int kn = 0, knP = 0;
    hipEvent_t evAfterBlur = nullptr;  // frame schedule hook (plvi_orb_internal_blur_event)
    int gateStage = 1;  // PLVI_GROW_GATE: the hook fires after the pyramid (0), blur + FAST (1), NMS (2) or the SAT (3)
    hipEvent_t evStage = nullptr;  // second hook (plvi_orb_internal_stage_event): fires after stage `evStageAt`
    int evStageAt = -1;
    std::vector<hipEvent_t> kev, kevP;
    int ktiming(int on) {
        if (on && kev.empty()) {
            kev.resize(2 * kKRing);
            kevP.resize(2 * kKRing);
            for (auto& e : kev) PLVI_CHECK(hipEventCreate(&e));
            for (auto& e : kevP) PLVI_CHECK(hipEventCreate(&e));
        }
        ktime = on != 0;
        if (on) kn = knP = 0;
        return PLVI_OK;
    }
    // kind 0: blur + FAST, 1: pyramid
    int ktiming_read(int kind, float* total_ms, int* launches) {
        const std::vector<hipEvent_t>& E = kind ? kevP : kev;
        const int n = kind ? knP : kn;
        float tot = 0.f;
        for (int i = 0; i < n; ++i) {
            PLVI_CHECK(hipEventSynchronize(E[2 * i + 1]));
            float t = 0.f;
            PLVI_CHECK(hipEventElapsedTime(&t, E[2 * i], E[2 * i + 1]));
            tot += t;
        }
        if (total_ms) *total_ms = tot;
        if (launches) *launches = n;
        return PLVI_OK;
    }

    int profile(int on) {
        if (on && evs.empty()) {
            evs.resize((size_t)kRing * (kStages + 1));
            for (auto& e : evs) PLVI_CHECK(hipEventCreate(&e));
        }
        prof = on != 0;
        profRuns = 0;
        return PLVI_OK;
    }
    void mark(int stage, hipStream_t st) {
        if (prof && profRuns < kRing) (void)hipEventRecord(evs[(size_t)profRuns * (kStages + 1) + stage], st);
    }
    int profile_read(float* ms, int* runs) {
        for (int k = 0; k < kStages; ++k) ms[k] = 0.f;
        for (int r = 0; r < profRuns; ++r) {
            PLVI_CHECK(hipEventSynchronize(evs[(size_t)r * (kStages + 1) + kStages]));
            for (int k = 0; k < kStages; ++k) {
                float t = 0.f;
                PLVI_CHECK(hipEventElapsedTime(&t, evs[(size_t)r * (kStages + 1) + k],
                                               evs[(size_t)r * (kStages + 1) + k + 1]));
                ms[k] += t;
            }
        }
        if (runs) *runs = profRuns;
        return PLVI_OK;
    }

    int init(const plvi_orb_params* p, int width, int height, int max_batch, int dev) {
        if (!p || width <= 0 || height <= 0 || max_batch <= 0 || p->nlevels <= 0 ||
            p->nlevels > kOrbMaxLevels || p->nfeatures < 0 || !(p->scale_factor > 1.0f))
            return PLVI_E_BADARG;
        prm = *p;
        W = width; H = height; Bcap = max_batch; device = dev; L = p->nlevels;
        if (const char* e = getenv("PLVI_GROW_GATE")) gateStage = std::min(3, std::max(0, atoi(e)));
        if (const char* e = getenv("PLVI_PYR_LEVELWISE")) pyrLevelwiseMax = atoi(e);
        if (const char* e = getenv("PLVI_ORB_L0_COPY")) l0forceCopy = atoi(e) != 0;
        if (const char* e = getenv("PLVI_ORB_OCT_LDS")) octLdsMax = std::max(0, std::min(kOctListLds, atoi(e)));
        PLVI_CHECK(hipSetDevice(device));
        {
            // the handle's own stream (single-frame calls, batches without a
            // caller stream) at the least priority (PLVI_ORB_STREAM_PRIO=0:
            // normal): the runtime keeps a separate hardware-queue pool per
            // priority, so the ORB thread of Frame does not share a queue with
            // the line extractor's normal-priority stream and hold up its
            // critical path (ORB finishes in half the lines' time anyway)
            int least = 0, greatest = 0;
            PLVI_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            const char* e = getenv("PLVI_ORB_STREAM_PRIO");
            const bool low = !e || atoi(e) != 0;
            PLVI_CHECK(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, low ? least : 0));
        }
        // ORBextractor ctor (ORBextractor.cc:413-444): scaleFactor is a double member.
        const double sf = (double)p->scale_factor;
        scale.assign(L, 1.f); sigma2.assign(L, 1.f);
        for (int i = 1; i < L; ++i) {
            scale[i] = (float)(scale[i - 1] * sf);
            sigma2[i] = scale[i] * scale[i];
        }
        invScale.resize(L); invSigma2.resize(L);
        for (int i = 0; i < L; ++i) { invScale[i] = 1.0f / scale[i]; invSigma2[i] = 1.0f / sigma2[i]; }
        quota.assign(L, 0);
        float factor = (float)(1.0f / sf);
        float nDesired = p->nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)L));
        int sum = 0;
        for (int l = 0; l < L - 1; ++l) {
            quota[l] = cv_round_h(nDesired);
            sum += quota[l];
            nDesired *= factor;
        }
        quota[L - 1] = std::max(p->nfeatures - sum, 0);
        umax.assign(16, 0);
        {
            int v, v0, vmax = cv_floor_h(15 * std::sqrt(2.f) / 2 + 1);
            int vmin = cv_ceil_h(15 * std::sqrt(2.f) / 2);
            const double hp2 = 15 * 15;
            for (v = 0; v <= vmax; ++v) umax[v] = cv_round_h(std::sqrt(hp2 - v * v));
            for (v = 15, v0 = 0; v >= vmin; --v) {
                while (umax[v0] == umax[v0 + 1]) ++v0;
                umax[v] = v0;
                ++v0;
            }
        }
        // 7x7 sigma=2 fixed-point taps: error-diffused
        // [18,34,48,56,48,34,18] (default) or plainly rounded [18,34,49,55,...]
        const int t7ed[7] = {18, 34, 48, 56, 48, 34, 18}, t7r[7] = {18, 34, 49, 55, 49, 34, 18};
        std::memcpy(taps, (p->compat & PLVI_COMPAT_GAUSS_ROUNDED) ? t7r : t7ed, sizeof(taps));
        resizeGeneric = (p->compat & PLVI_COMPAT_RESIZE_V_GENERIC) ? 1 : 0;
        // Levels
        lv.resize(L);
        size_t off = 0, boffAll = 0;
        long long listOff = 0;
        std::vector<uint32_t> xtab;
        int kpOff = 0;
        nodeCapMax = 0;
        for (int l = 0; l < L; ++l) {
            OrbLevelDev& d = lv[l];
            std::memset(&d, 0, sizeof(d));
            d.w = cv_round_h((float)W * invScale[l]);
            d.h = cv_round_h((float)H * invScale[l]);
            d.plane = (long long)d.w * d.h;
            d.off = (long long)off;
            off += (size_t)d.plane * Bcap;
            d.bpitch = (d.w + kBfAlign - 1) / kBfAlign * kBfAlign;
            d.bplane = (long long)d.bpitch * d.h;
            d.boff = (long long)boffAll;
            boffAll += (size_t)d.bplane * Bcap;
            d.minB = 16;
            const int maxBX = d.w - 16, maxBY = d.h - 16;
            d.rw = maxBX - d.minB;
            d.rh = maxBY - d.minB;
            const float width = (float)d.rw, height = (float)d.rh;
            d.nCols = (int)(width / 30.f);
            d.nRows = (int)(height / 30.f);
            if (d.nCols <= 0 || d.nRows <= 0) return PLVI_E_BADARG;
            // the node maximum's tie-break key (cell, row, column) must fit 32 bits
            if ((double)d.nRows * d.nCols * d.rh * d.rw >= 4294967296.0) return PLVI_E_BADARG;
            d.wCell = (int)std::ceil(width / d.nCols);
            d.hCell = (int)std::ceil(height / d.nRows);
            if (d.wCell + 6 > kOrbCellMax || d.hCell + 6 > kOrbCellMax) return PLVI_E_BADARG;
            // candidate entries pack x (11 bits) and y (10 bits) relative to the region
            if (d.rw >= 2048 || d.rh >= 1024) return PLVI_E_BADARG;
            d.quota = quota[l];
            d.scale = scale[l];
            d.size = (float)(int)(31 * scale[l]);
            // octree roots (ORBextractor.cc:541-567)
            const int nIni = (int)std::round((float)(maxBX - d.minB) / (maxBY - d.minB));
            if (nIni <= 0 || nIni > kOrbMaxRoots) return PLVI_E_BADARG;
            d.nIni = nIni;
            const float hX = (float)(maxBX - d.minB) / nIni;
            for (int i = 0; i <= nIni; ++i) d.rootGx[i] = (int)(hX * (float)i);
            // membership boundaries: root(x) = (int)(x / hX) for integer x
            d.rootB[0] = 0;
            for (int i = 1; i <= nIni; ++i) {
                int b = d.rootB[i - 1];
                while (b < d.rw && (int)((float)b / hX) < i) ++b;
                d.rootB[i] = b;
            }
            d.rootB[nIni] = d.rw;
            d.nodeCap = std::max(d.quota, 4 * nIni) + 8;
            d.kpOff = kpOff;
            kpOff += d.nodeCap;
            nodeCapMax = std::max(nodeCapMax, d.nodeCap);
            // cells (ORBextractor.cc:787-806): FAST detection windows
            for (int i = 0; i < d.nRows; ++i) {
                const float iniY = (float)(d.minB + i * d.hCell);
                float maxY = iniY + d.hCell + 6;
                if (iniY >= maxBY - 3) continue;
                if (maxY > maxBY) maxY = (float)maxBY;
                for (int j = 0; j < d.nCols; ++j) {
                    const float iniX = (float)(d.minB + j * d.wCell);
                    float maxX = iniX + d.wCell + 6;
                    if (iniX >= maxBX - 6) continue;
                    if (maxX > maxBX) maxX = (float)maxBX;
                    OrbCellDev c;
                    c.level = l;
                    c.x0 = (int)iniX + 3; c.y0 = (int)iniY + 3;
                    c.x1 = (int)maxX - 3; c.y1 = (int)maxY - 3;
                    if (c.x1 > c.x0 && c.y1 > c.y0) {
                        cells.push_back(c);
                        // survivors are strict maxima over their 8 neighbours
                        // inside the window: at most one per 2 x 2 block
                        d.listCap += ((c.x1 - c.x0 + 1) / 2) * ((c.y1 - c.y0 + 1) / 2);
                    }
                }
            }
            // cv::resize scale from level l-1 (resize.cpp: scale_x = 1 / inv_scale_x)
            if (l > 0) {
                d.rsx = 1. / ((double)d.w / lv[l - 1].w);
                d.rsy = 1. / ((double)d.h / lv[l - 1].h);
                d.xtab = (int)xtab.size();
                if (append_xtab(xtab, lv[l - 1].w, d.w)) return PLVI_E_BADARG;
                // LDS: a kPyrRing-row ring of level 0, two rows of every other source level
                pyrSmem += (l == 1 ? kPyrRing : 2) * (size_t)((lv[l - 1].w + 3) & ~3);
            }
            // strips of the blur + FAST kernel, cut at kBfAlign-aligned columns
            // so that each strip writes whole aligned segments of the blur /
            // score rows (cuts at cell windows leave partial segments that two
            // strips write at different times: 12.48 vs 11.57 GB of HBM
            // traffic per launch)
            {
                std::vector<int> cx, cy;  // interior split candidates
                for (int x = kBfAlign; x < d.w; x += kBfAlign) cx.push_back(x);
                for (int y = 1; y < d.h; ++y) cy.push_back(y);
                std::vector<int> sx, sy;
                if (plan_splits(d.w, cx, [](int a, int b) { return b - (a & ~3) <= kBfCols; }, sx) ||
                    plan_splits(d.h, cy, [](int a, int b) { return b - a <= kBfRowsPlain; }, sy))
                    return PLVI_E_BADARG;
                for (size_t ri = 0; ri + 1 < sy.size(); ++ri)
                    for (size_t ci = 0; ci + 1 < sx.size(); ++ci)
                        strips.push_back(OrbStripDev{l, sx[ci], sx[ci + 1], sy[ri], sy[ri + 1]});
            }
        }
        kpCapFrame = kpOff;
        pyrBytesFrameTotal = off;
        blurBytesTotal = boffAll;
        for (auto& d : lv) {
            d.listOff = (int)listOff;
            listOff += d.listCap;
            listMax = std::max(listMax, d.listCap);
        }
        if (listOff >= (1LL << 31) / 8) return PLVI_E_BADARG;
        listFrame = (int)listOff;
        // device tables
        if (d_lv.alloc(sizeof(OrbLevelDev) * L) || d_cells.alloc(sizeof(OrbCellDev) * cells.size()) ||
            d_strips.alloc(sizeof(OrbStripDev) * strips.size()))
            return PLVI_E_HIP;
        PLVI_CHECK(hipMemcpy(d_strips.p, strips.data(), sizeof(OrbStripDev) * strips.size(), hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(d_lv.p, lv.data(), sizeof(OrbLevelDev) * L, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(d_cells.p, cells.data(), sizeof(OrbCellDev) * cells.size(), hipMemcpyHostToDevice));
        xtabN = (int)xtab.size();
        pyrFrameLds = (int)((pyrSmem + 15) & ~size_t(15));
        pyrSmem = 4 * (size_t)xtabN + (size_t)kPyrFrames * pyrFrameLds;
        if (W > 4 * 64 * kPyrDw || pyrSmem > 64 * 1024) return PLVI_E_BADARG;  // orb_pyramid_kernel limits
        if (xtab.empty()) xtab.push_back(0);
        if (d_xtab.alloc(4 * xtab.size())) return PLVI_E_HIP;
        PLVI_CHECK(hipMemcpy(d_xtab.p, xtab.data(), 4 * xtab.size(), hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_umax), umax.data(), 16 * sizeof(int)));
        // work buffers
        if (pyr.alloc(off) || blur.alloc(boffAll) || score.alloc(boffAll) ||
            clist.alloc(sizeof(uint32_t) * (size_t)listFrame * Bcap) || ccount.alloc(sizeof(int) * kOrbCountPad * L * Bcap) ||
            rectCnt.alloc(sizeof(int) * L * Bcap) || lvkp.alloc(sizeof(float4) * (size_t)kpCapFrame * Bcap) ||
            lvdesc.alloc((size_t)32 * kpCapFrame * Bcap) || okp.alloc(sizeof(plvi_keypoint) * (size_t)kpCapFrame * Bcap) ||
            odesc.alloc((size_t)32 * kpCapFrame * Bcap) || ocount.alloc(sizeof(int) * Bcap) ||
            omono.alloc(sizeof(int) * Bcap) || err.alloc(sizeof(int) * Bcap) || staging.alloc((size_t)W * H))
            return PLVI_E_HIP;
        PLVI_CHECK(hipMemset(err.p, 0, sizeof(int) * Bcap));
        octLcap = std::min(listMax, octLdsMax);
        octSmem = orb_octree_lds(nodeCapMax, octLcap);
        if (octSmem > 160 * 1024) return PLVI_E_BADARG;
        PLVI_CHECK(hipFuncSetAttribute((const void*)orb_octree_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)octSmem));
        return PLVI_OK;
    }

    // The whole batch pipeline, asynchronous on `st`.
    int run(const uint8_t* d_frames, int nf, size_t frame_stride, size_t row_stride, int lap0, int lap1,
            hipStream_t st) {
        if (nf <= 0 || nf > Bcap) return PLVI_E_BADARG;
        if (!st) st = stream;
        lastFrames = nf;
        const bool copy0 = l0forceCopy || row_stride != (size_t)W;
        l0view = copy0 ? nullptr : d_frames;
        l0fs = frame_stride;
        const int tmin = std::max(0, std::min(std::min(prm.ini_th_fast, prm.min_th_fast), 255));
        const int t1 = std::max(0, std::min(prm.ini_th_fast, 255)), t2 = std::max(0, std::min(prm.min_th_fast, 255));
        uint8_t* P = pyr.as<uint8_t>();
        uint8_t* Bl = blur.as<uint8_t>();
        uint8_t* Sc = score.as<uint8_t>();
        // the NMS appends to the (frame, level) candidate lists from zero
        PLVI_CHECK(hipMemsetAsync(ccount.p, 0, sizeof(int) * kOrbCountPad * (size_t)L * nf, st));
        mark(0, st);
        auto hook = [&](int k, hipStream_t s_) {
            if (evAfterBlur && gateStage == k) PLVI_CHECK(hipEventRecord(evAfterBlur, s_));
            if (evStage && evStageAt == k) PLVI_CHECK(hipEventRecord(evStage, s_));
            return PLVI_OK;
        };
        // K1a: the pyramid (ComputePyramid, chained resize: level l from l-1):
        // small batches level by level over the whole chip, large ones in one
        // streaming launch (a loader and a resizer wave per frame)
        if (L > 1) {
            const bool ktP = ktime && knP < kKRing;
            if (ktP) PLVI_CHECK(hipEventRecord(kevP[2 * knP], st));
            if (nf <= pyrLevelwiseMax) {
                for (int l = 1; l < L; ++l) {
                    const OrbLevelDev& s = lv[l - 1];
                    const OrbLevelDev& d = lv[l];
                    const uint8_t* src = l == 1 ? d_frames : P + s.off;
                    const size_t sfr = l == 1 ? frame_stride : (size_t)s.plane, srow = l == 1 ? row_stride : (size_t)s.w;
                    const int items = ((d.w + 3) >> 2) * d.h;
                    hipLaunchKernelGGL(orb_resize_level_kernel, dim3((items + 255) / 256, nf), dim3(256), 0, st, src, sfr,
                                       srow, s.w, s.h, P + d.off, (size_t)d.plane, d.w, d.h, d.rsy,
                                       (const uint32_t*)d_xtab.as<uint32_t>() + d.xtab, resizeGeneric);
                }
            } else {
                hipLaunchKernelGGL(orb_pyramid_kernel, dim3((nf + kPyrFrames - 1) / kPyrFrames), dim3(64 * (kPyrFrames + 1)),
                                   pyrSmem, st, d_lv.as<OrbLevelDev>(), L, d_frames, frame_stride, row_stride, nf, P,
                                   (const uint32_t*)d_xtab.as<uint32_t>(), xtabN, pyrFrameLds, resizeGeneric);
            }
            if (ktP) {
                PLVI_CHECK(hipEventRecord(kevP[2 * knP + 1], st));
                ++knP;
            }
        }
        if (const int hrc = hook(0, st)) return hrc;
        // K1b: blur + FAST score of every level (level 0 also copies the frame into its plane)
        const bool kt = ktime && kn < kKRing;
        if (kt) PLVI_CHECK(hipEventRecord(kev[2 * kn], st));
        hipLaunchKernelGGL(orb_blur_fast_kernel, dim3((unsigned)(strips.size() * 8 * ((nf + 7) / 8))), dim3(64), 0, st,
                           d_lv.as<OrbLevelDev>(), d_strips.as<OrbStripDev>(), d_frames, frame_stride, row_stride, P,
                           Bl, Sc, taps[0], taps[1], taps[2], taps[3], tmin, t1, t2, (int)strips.size(),
                           nf, copy0 ? 1 : 0);
        if (kt) {
            PLVI_CHECK(hipEventRecord(kev[2 * kn + 1], st));
            ++kn;
        }
        if (const int hrc = hook(1, st)) return hrc;
        mark(1, st);
        // K2 cell NMS -> the (frame, level) candidate lists
        hipLaunchKernelGGL(orb_cell_nms_kernel, dim3((unsigned)cells.size(), nf), dim3(64), 0, st,
                           d_cells.as<OrbCellDev>(), (int)cells.size(), d_lv.as<OrbLevelDev>(), (const uint8_t*)Sc,
                           clist.as<uint32_t>(), listFrame, ccount.as<int>(), L, err.as<int>(), t1, t2);
        mark(2, st);
        if (const int hrc = hook(2, st)) return hrc;
        // (K3, the r01-r05 summed-area table of the candidate plane, is gone:
        // stage 3 stays as an empty profiling slot)
        mark(3, st);
        if (const int hrc = hook(3, st)) return hrc;
        // K4 octree + the best candidate of every node (K5 in r01-r05)
        hipLaunchKernelGGL(orb_octree_kernel, dim3(nf, L), dim3(64), octSmem, st, d_lv.as<OrbLevelDev>(),
                           (const uint32_t*)clist.as<uint32_t>(), listFrame, (const int*)ccount.as<int>(), lvkp.as<float4>(),
                           kpCapFrame, rectCnt.as<int>(), nodeCapMax, L, err.as<int>(), octLcap);
        mark(4, st);
        if (const int hrc = hook(4, st)) return hrc;
        mark(5, st);
        if (const int hrc = hook(5, st)) return hrc;
        // K6 orientation + rBRIEF
        hipLaunchKernelGGL(orb_describe_kernel, dim3((kpCapFrame + 15) / 16, nf), dim3(256), 0, st,
                           d_lv.as<OrbLevelDev>(), L, (const uint8_t*)P, (const uint8_t*)Bl,
                           (const int*)rectCnt.as<int>(), lvkp.as<float4>(), lvdesc.as<uint8_t>(), kpCapFrame,
                           copy0 ? nullptr : d_frames, frame_stride, row_stride);
        mark(6, st);
        // K7 assemble
        hipLaunchKernelGGL(orb_assemble_kernel, dim3(nf), dim3(256), 0, st, d_lv.as<OrbLevelDev>(), L,
                           (const int*)rectCnt.as<int>(), (const float4*)lvkp.as<float4>(),
                           (const uint8_t*)lvdesc.as<uint8_t>(), kpCapFrame, lap0, lap1, okp.as<plvi_keypoint>(),
                           odesc.as<uint8_t>(), ocount.as<int>(), omono.as<int>());
        mark(7, st);
        if (prof && profRuns < kRing) ++profRuns;
        PLVI_CHECK(hipGetLastError());
        return PLVI_OK;
    }

};

}  // namespace plvi

using plvi::OrbPipeline;

// The handle owns its pipeline by pointer: ORBextractor::operator() takes
// frames of any size (ORBextractor.cc:1152-1160), so a size change builds a
// new plan for it (geometry, tables, buffers) and retires the old one.
struct plvi_orb_extractor {
    std::unique_ptr<OrbPipeline> up;
    OrbPipeline& p() { return *up; }
    int replan(int width, int height) {
        if (width == up->W && height == up->H) return PLVI_OK;
        PLVI_CHECK(hipStreamSynchronize(up->stream));
        auto np = std::make_unique<OrbPipeline>();
        int rc = np->init(&up->prm, width, height, up->Bcap, up->device);
        if (rc) return rc;
        up = std::move(np);
        return PLVI_OK;
    }
};

// Read and clear per-frame device error flags (shared by both extractors).
int plvi::read_frame_errors(int* d_err, int nslots, int* frame_flags, int* any, hipStream_t st) {
    std::vector<int> f((size_t)nslots);
    PLVI_CHECK(hipMemcpyAsync(f.data(), d_err, sizeof(int) * nslots, hipMemcpyDeviceToHost, st));
    PLVI_CHECK(hipMemsetAsync(d_err, 0, sizeof(int) * nslots, st));
    PLVI_CHECK(hipStreamSynchronize(st));
    int a = 0;
    for (int i = 0; i < nslots; ++i) {
        a |= f[i];
        if (frame_flags) frame_flags[i] = f[i];
    }
    if (any) *any = a;
    return PLVI_OK;
}

extern "C" int plvi_orb_create(const plvi_orb_params* p, int width, int height, int max_batch, int device,
                               plvi_orb_extractor** out) {
    if (!out) return PLVI_E_BADARG;
    *out = nullptr;
    auto h = std::make_unique<plvi_orb_extractor>();
    h->up = std::make_unique<OrbPipeline>();
    int rc = h->p().init(p, width, height, max_batch, device);
    if (rc) return rc;
    *out = h.release();
    return PLVI_OK;
}

extern "C" int plvi_orb_destroy(plvi_orb_extractor* h) {
    if (!h) return PLVI_E_BADARG;
    (void)hipSetDevice(h->p().device);
    (void)hipStreamSynchronize(h->p().stream);
    delete h;
    return PLVI_OK;
}

extern "C" int plvi_orb_extract_batch(plvi_orb_extractor* h, const uint8_t* d_frames, int n_frames,
                                      size_t frame_stride, size_t row_stride, int lap0, int lap1, void* stream) {
    if (!h || !d_frames) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().run(d_frames, n_frames, frame_stride, row_stride, lap0, lap1, (hipStream_t)stream);
}

extern "C" int plvi_orb_errors(plvi_orb_extractor* h, int* frame_flags, int* any, void* stream) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    hipStream_t st = stream ? (hipStream_t)stream : h->p().stream;
    return plvi::read_frame_errors(h->p().err.as<int>(), h->p().Bcap, frame_flags, any, st);
}

extern "C" int plvi_orb_outputs(plvi_orb_extractor* h, plvi_keypoint** d_kps, uint8_t** d_desc, int** d_count,
                                int** d_mono, int* cap) {
    if (!h) return PLVI_E_BADARG;
    if (d_kps) *d_kps = h->p().okp.as<plvi_keypoint>();
    if (d_desc) *d_desc = h->p().odesc.as<uint8_t>();
    if (d_count) *d_count = h->p().ocount.as<int>();
    if (d_mono) *d_mono = h->p().omono.as<int>();
    if (cap) *cap = h->p().kpCapFrame;
    return PLVI_OK;
}

extern "C" int plvi_orb_extract(plvi_orb_extractor* h, const uint8_t* img, int width, int height, size_t stride,
                                int lap0, int lap1, plvi_keypoint* kps, uint8_t* desc, int cap, int* n,
                                int* mono_index) {
    if (!h) return PLVI_E_BADARG;
    if (n) *n = 0;
    if (!img || width <= 0 || height <= 0) return PLVI_E_EMPTY;  // _image.empty() -> -1
    PLVI_CHECK(hipSetDevice(h->p().device));
    if (int rc = h->replan(width, height)) return rc;
    OrbPipeline& P = h->p();
    PLVI_CHECK(hipMemcpy2DAsync(P.staging.p, (size_t)P.W, img, stride, (size_t)P.W, (size_t)P.H,
                                hipMemcpyHostToDevice, P.stream));
    int rc = P.run(P.staging.as<uint8_t>(), 1, (size_t)P.W * P.H, (size_t)P.W, lap0, lap1, P.stream);
    if (rc) return rc;
    int cnt = 0, mono = 0, errv = 0;
    PLVI_CHECK(hipMemcpyAsync(&cnt, P.ocount.p, sizeof(int), hipMemcpyDeviceToHost, P.stream));
    PLVI_CHECK(hipMemcpyAsync(&mono, P.omono.p, sizeof(int), hipMemcpyDeviceToHost, P.stream));
    PLVI_CHECK(hipMemcpyAsync(&errv, P.err.p, sizeof(int), hipMemcpyDeviceToHost, P.stream));
    PLVI_CHECK(hipStreamSynchronize(P.stream));
    if (errv) {
        PLVI_CHECK(hipMemset(P.err.p, 0, sizeof(int) * P.Bcap));
        return PLVI_E_OVERFLOW;
    }
    if (n) *n = cnt;
    if (mono_index) *mono_index = mono;
    if (cnt > cap) return PLVI_E_CAPACITY;
    if (cnt > 0) {
        if (kps) PLVI_CHECK(hipMemcpy(kps, P.okp.p, sizeof(plvi_keypoint) * cnt, hipMemcpyDeviceToHost));
        if (desc) PLVI_CHECK(hipMemcpy(desc, P.odesc.p, (size_t)32 * cnt, hipMemcpyDeviceToHost));
    }
    return PLVI_OK;
}

extern "C" int plvi_orb_pyramid_level(plvi_orb_extractor* h, int frame, int level, uint8_t* dst, int* w, int* hgt) {
    if (!h || level < 0 || level >= h->p().L || frame < 0 || frame >= h->p().Bcap) return PLVI_E_BADARG;
    const auto& d = h->p().lv[level];
    if (w) *w = d.w;
    if (hgt) *hgt = d.h;
    if (!dst) return PLVI_OK;
    PLVI_CHECK(hipSetDevice(h->p().device));
    PLVI_CHECK(hipStreamSynchronize(h->p().stream));
    const uint8_t* src = h->p().pyr.as<uint8_t>() + d.off;
    size_t fs = (size_t)d.plane;
    if (level == 0 && h->p().l0view) {  // level 0 is a view of the last run's frames
        src = h->p().l0view;
        fs = h->p().l0fs;
    }
    PLVI_CHECK(hipMemcpy(dst, src + (size_t)frame * fs, (size_t)d.plane, hipMemcpyDeviceToHost));
    return PLVI_OK;
}

extern "C" int plvi_orb_pyramid_device(plvi_orb_extractor* h, int level, const uint8_t** d_frame0,
                                       size_t* frame_stride, int* w, int* hgt, int* nlevels) {
    if (!h || level < -1 || level >= h->p().L) return PLVI_E_BADARG;
    if (nlevels) *nlevels = h->p().L;
    if (level < 0) return PLVI_OK;
    const auto& d = h->p().lv[level];
    const bool view = level == 0 && h->p().l0view;
    if (d_frame0) *d_frame0 = view ? h->p().l0view : h->p().pyr.as<uint8_t>() + d.off;
    if (frame_stride) *frame_stride = view ? h->p().l0fs : (size_t)d.plane;
    if (w) *w = d.w;
    if (hgt) *hgt = d.h;
    return PLVI_OK;
}

extern "C" int plvi_orb_scale_tables(plvi_orb_extractor* h, float* scale, float* inv_scale, float* sigma2,
                                     float* inv_sigma2) {
    if (!h) return PLVI_E_BADARG;
    const auto& P = h->p();
    for (int i = 0; i < P.L; ++i) {
        if (scale) scale[i] = P.scale[i];
        if (inv_scale) inv_scale[i] = P.invScale[i];
        if (sigma2) sigma2[i] = P.sigma2[i];
        if (inv_sigma2) inv_sigma2[i] = P.invSigma2[i];
    }
    return PLVI_OK;
}

extern "C" int plvi_orb_level_quota(plvi_orb_extractor* h, int* q) {
    if (!h || !q) return PLVI_E_BADARG;
    for (int i = 0; i < h->p().L; ++i) q[i] = h->p().quota[i];
    return PLVI_OK;
}

extern "C" int plvi_orb_profile(plvi_orb_extractor* h, int enable) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().profile(enable);
}

extern "C" int plvi_orb_profile_read(plvi_orb_extractor* h, float* stage_ms, int* runs) {
    if (!h || !stage_ms) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().profile_read(stage_ms, runs);
}

// Internal (frame schedule): record `ev` on the batch stream right after the
// blur + FAST launch of every later batch (nullptr: off).
extern "C" int plvi_orb_internal_stage_event(plvi_orb_extractor* h, int stage, hipEvent_t ev) {
    if (!h) return PLVI_E_BADARG;
    h->p().evStage = ev;
    h->p().evStageAt = stage;
    return PLVI_OK;
}

extern "C" int plvi_orb_internal_blur_event(plvi_orb_extractor* h, hipEvent_t ev) {
    if (!h) return PLVI_E_BADARG;
    h->p().evAfterBlur = ev;
    return PLVI_OK;
}

extern "C" int plvi_orb_kernel_timing(plvi_orb_extractor* h, int enable) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().ktiming(enable);
}

extern "C" int plvi_orb_kernel_timing_read(plvi_orb_extractor* h, float* total_ms, int* launches) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().ktiming_read(0, total_ms, launches);
}

extern "C" int plvi_orb_kernel_timing_read_kind(plvi_orb_extractor* h, int kind, float* total_ms, int* launches) {
    if (!h || kind < 0 || kind > 1) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().ktiming_read(kind, total_ms, launches);
}

extern "C" int plvi_orb_debug_node_cap(plvi_orb_extractor* h, int cap) {
    if (!h) return PLVI_E_BADARG;
    OrbPipeline& p = h->p();
    PLVI_CHECK(hipSetDevice(p.device));
    PLVI_CHECK(hipStreamSynchronize(p.stream));
    std::vector<plvi::OrbLevelDev> v = p.lv;
    if (cap > 0)
        for (auto& d : v) d.nodeCap = std::min(d.nodeCap, cap);
    PLVI_CHECK(hipMemcpy(p.d_lv.p, v.data(), sizeof(plvi::OrbLevelDev) * v.size(), hipMemcpyHostToDevice));
    return PLVI_OK;
}
