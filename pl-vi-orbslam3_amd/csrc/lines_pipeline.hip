// lines_pipeline.hip — host orchestration of the line kernels and the line
// part of the C-ABI.  Replaces ORB_SLAM3::Lineextractor::operator()
// (src/LineExtractor.cc:45-117, LSD branch) with the reference's constants:
// LSD sigma_scale 0.6, quant 2, ang_th 22.5, log_eps 1, density 0.6,
// n_bins 1024 (:56-61), min_length 0.025*min(w,h) (:72).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "lines_device.h"
#include "lines_kernels.hpp"
#include "lsd_grow_mw.hpp"
#include "plvi_common.h"

// internal hook of the ORB pipeline (orb_pipeline.hip): event after the blur + FAST launch
extern "C" int plvi_orb_internal_blur_event(plvi_orb_extractor* h, hipEvent_t ev);
extern "C" int plvi_orb_internal_stage_event(plvi_orb_extractor* h, int stage, hipEvent_t ev);

namespace plvi {

static inline int lround_h(float v) { return (int)lrintf(v); }
static inline int lround_h(double v) { return (int)lrint(v); }
static inline int lfloor_h(float v) { int i = (int)v; return i - (i > v); }

// exp64f of OpenCV (mathfuncs_core; softfloat's f64_exp uses the same
// scheme): v = cvRound(x * 64/ln2), 2^(v>>6) in the exponent bits, the table
// entry 2^((v&63)/64) * EXPPOLY_32F_A0 and a degree-5 polynomial of the
// remainder.  SURVEY A.6 switch (PLVI_COMPAT_EXP_CV_TABLE).
static double cv_exp64f(double x) {
    const double a0s = .9670371139572337719125840413672004409288e-2;
    const double k5 = .99999999999999999998285227504999 / a0s, k4 = .69314718055994546743029643825322 / a0s,
                 k3 = .24022650695886477918181338054308 / a0s, k2 = .55504108793649567998466049042729e-1 / a0s,
                 k1 = .96180973140732918010002372686186e-2 / a0s, k0 = .13369713757180123244806654839424e-2 / a0s;
    const double pre = 1.4426950408889634073599246810019 * 64;
    double y = x * pre;
    const int v = (int)lrint(y);
    int e = (v >> 6) + 1023;
    e = e < 0 ? 0 : e > 2047 ? 2047 : e;
    const double p2 = std::ldexp(1.0, e - 1023);
    const double tab = (double)exp2l((long double)(v & 63) / 64.0L) * a0s;
    y = (y - v) * (1. / 64);
    return p2 * tab * (((((k0 * y + k1) * y + k2) * y + k3) * y + k4) * y + k5);
}

// getGaussianKernelBitExact (OpenCV 4.2 smooth.dispatch.cpp) in double.
static void gauss_kernel_f64(int n, double sigma, double* k, bool cvExp) {
    const double scale2X = -0.125 / (sigma * sigma);
    const int n2 = (n - 1) / 2;
    std::vector<double> values(n2 + 1);
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
        const double a = (double)(x * x) * scale2X;
        double t = cvExp ? cv_exp64f(a) : std::exp(a);
        values[i] = t;
        sum += t;
    }
    sum *= 2;
    sum += 1.0;
    const double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; ++i) k[i] = k[n - 1 - i] = values[i] * mul1;
    k[n2] = 1.0 * mul1;
}

struct LinePipeline {
    plvi_line_params prm{};
    int W = 0, H = 0, Bcap = 0, device = 0, nOct = 0, fcap = 0;
    hipStream_t stream = nullptr;
    hipStream_t aux[2] = {nullptr, nullptr};  // frame mode: ORB and LBD-Sobel streams
    hipEvent_t evSobelGo = nullptr;
    hipEvent_t evFork = nullptr, evPrep = nullptr, evSobel = nullptr, evOrb = nullptr, evCrit = nullptr,
               evBlur = nullptr, evGate = nullptr, evGrow2 = nullptr, evPair = nullptr;
    bool growAfterBlur = true, sobelWithGrow = false, growSplit = false;
    int sobelGate = -1;  // PLVI_SOBEL_GATE: ORB stage after which the Sobel pyramid starts (-1: with growth)
    bool sobelAfterGrow = false;
    hipStream_t critStream = nullptr;  // frame schedule: prep -> grow -> describe
    hipStream_t crit2 = nullptr;       // frame schedule: octave-1 region growing (split mode)
    hipStream_t octStream = nullptr;   // small batches: prep + growth of octaves >= 1 beside octave 0's
    int orbAfterPrep = 1;
    std::vector<LineOctDev> oct;
    std::vector<float> scaleF, invScaleF;
    double SCALE = 0.8, prec = 0, rho = 0, min_length = 0;
    double gk[7]{};
    int lbdTaps[3] = {14, 62, 104};
    DevBuf d_oct, d_tabs, octImg, pix, modg, seedcs, gbits, qspill, regs, regpts, rawLines, nlines, klTmp, klOut, fnOut, cntOut, descOut, lbdBlur,
        lbdG, err, staging, mwOwn, mwSlot, mwGrow, sortPos;
    size_t qspillFrame = 0, gbitsFrame = 0, lbdPlaneTotal = 0;
    int lastFrames = 0;
    static constexpr int kStages = 5, kRing = 512;
    bool prof = false;
    int profRuns = 0;
    std::vector<hipEvent_t> evs;

    // Per-launch timing of lsd_prep_kernel (bench.py's LSD-pass roofline): an
    // event pair on the launch stream around every launch while enabled.
    static constexpr int kKRing = 4096;
    bool ktime = false;
    int kn = 0;
    std::vector<hipEvent_t> kev;
    // and around every LBD Gaussian + Sobel launch: [0] lbd_sobel0_kernel, [1] lbd_sobel1_kernel
    std::vector<hipEvent_t> kevS[2];
    int knS[2] = {0, 0};
    int ktiming(int on) {
        if (on && kev.empty()) {
            kev.resize(2 * kKRing);
            for (auto& e : kev) PLVI_CHECK(hipEventCreate(&e));
            for (auto& v : kevS) {
                v.resize(2 * kKRing);
                for (auto& e : v) PLVI_CHECK(hipEventCreate(&e));
            }
        }
        ktime = on != 0;
        if (on) kn = knS[0] = knS[1] = 0;
        return PLVI_OK;
    }
    void ktimeS(int k, int edge, hipStream_t st) {  // edge 0 = before, 1 = after launch k
        if (!ktime || knS[k] >= kKRing) return;
        (void)hipEventRecord(kevS[k][2 * knS[k] + edge], st);
        if (edge) ++knS[k];
    }
    int ktiming_read_kind(int kind, float* total_ms, int* launches) {
        if (kind == 0) return ktiming_read(total_ms, launches);
        if (kind < 1 || kind > 2) return PLVI_E_BADARG;
        const int k = kind - 1;
        float tot = 0.f;
        for (int i = 0; i < knS[k]; ++i) {
            PLVI_CHECK(hipEventSynchronize(kevS[k][2 * i + 1]));
            float t = 0.f;
            PLVI_CHECK(hipEventElapsedTime(&t, kevS[k][2 * i], kevS[k][2 * i + 1]));
            tot += t;
        }
        if (total_ms) *total_ms = tot;
        if (launches) *launches = knS[k];
        return PLVI_OK;
    }
    int ktiming_read(float* total_ms, int* launches) {
        float tot = 0.f;
        for (int i = 0; i < kn; ++i) {
            PLVI_CHECK(hipEventSynchronize(kev[2 * i + 1]));
            float t = 0.f;
            PLVI_CHECK(hipEventElapsedTime(&t, kev[2 * i], kev[2 * i + 1]));
            tot += t;
        }
        if (total_ms) *total_ms = tot;
        if (launches) *launches = kn;
        return PLVI_OK;
    }

    ~LinePipeline() {
        for (auto e : kev) (void)hipEventDestroy(e);
        for (auto e : evs) (void)hipEventDestroy(e);
        for (auto e : {evFork, evPrep, evSobel, evOrb, evCrit, evBlur, evGate, evGrow2, evPair, evSobelGo})
            if (e) (void)hipEventDestroy(e);
        if (critStream) (void)hipStreamDestroy(critStream);
        if (crit2) (void)hipStreamDestroy(crit2);
        if (octStream) (void)hipStreamDestroy(octStream);
        for (auto a : aux)
            if (a) (void)hipStreamDestroy(a);
        if (stream) (void)hipStreamDestroy(stream);
    }

    int init(const plvi_line_params* p, int width, int height, int max_batch, int dev) {
        if (!p || width <= 0 || height <= 0 || max_batch <= 0) return PLVI_E_BADARG;
        if (p->refine != 0 || p->extractor != 0) return PLVI_E_BADARG;  // config: lsd_refine 0, extractor 0 (LSD)
        if (p->nlevels <= 0 || p->nlevels > kLineMaxOct || p->nfeatures < 0) return PLVI_E_BADARG;
        prm = *p;
        W = width; H = height; Bcap = max_batch; device = dev; nOct = p->nlevels;
        PLVI_CHECK(hipSetDevice(device));
        PLVI_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        {
            // frame schedule streams: PLVI_STREAM_PRIO=1 (default) puts the critical
            // path on the greatest priority and ORB / Sobel on the least
            int least = 0, greatest = 0;
            PLVI_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            const char* e1 = getenv("PLVI_STREAM_PRIO");
            const bool prio = !e1 || atoi(e1) != 0;
            // PLVI_ORB_AFTER_PREP: ORB waits for the LSD prep -- 1 in batches
            // below 1024 frames, 2 (default since late r06) in every batch, 0
            // never.  In r04, with two 3072-frame batches in flight, starting
            // ORB at once was 2-3 % faster (profiles/r04/ab_sched_inflight2.txt);
            // at the end of r06 (one growth task per wave, ORB the busier chain)
            // waiting is +0.2-0.6 % over two A/Bs and blur + FAST's in-window
            // time steadier (profiles/r06/ab_sched_orbprio.txt, ab_final_knobs.txt)
            const char* e2 = getenv("PLVI_ORB_AFTER_PREP");
            orbAfterPrep = e2 ? atoi(e2) : 2;
            // PLVI_GROW_AFTER_BLUR=0: region growing starts right after the prep
            // (default 1: it waits for the ORB blur + FAST launch, whose 81-VGPR /
            // 9 KB-LDS waves cannot share a CU with the region-growing waves; the
            // rest of the ORB chain then runs alongside region growing)
            const char* e3 = getenv("PLVI_GROW_AFTER_BLUR");
            growAfterBlur = !e3 || atoi(e3) != 0;
            // PLVI_ORB_PRIO (default 1): the ORB stream at the greatest priority as
            // well (its pyramid + blur gate region growing from 1024 frames on).
            // r06: 0 (least) with ORB after the prep gives the same headline
            // step and blur + FAST 8-10 instead of 16-22 ms in the window, but
            // a batch-64 pair created later in the same process then steps in
            // 7.9 instead of 7.45 ms -- even with its own ORB stream at the
            // greatest priority (profiles/r06/ab_sched_orbprio.txt); kept at 1
            const char* e4 = getenv("PLVI_ORB_PRIO");
            const bool orbHigh = !e4 || atoi(e4) != 0;
            for (int a = 0; a < 2; ++a)
                PLVI_CHECK(hipStreamCreateWithPriority(&aux[a], hipStreamNonBlocking,
                                                       prio ? (a == 0 && orbHigh ? greatest : least) : 0));
            // PLVI_SOBEL_WITH_GROW (default 1): the LBD Sobel pyramid (needed only
            // by the LBD describe at the end) starts with region growing instead
            // of competing with the prep and the ORB pyramid
            const char* e5 = getenv("PLVI_SOBEL_WITH_GROW");
            sobelWithGrow = !e5 || atoi(e5) != 0;
            // PLVI_SOBEL_GATE=k (batches from 1024 frames): the Sobel pyramid waits
            // for ORB stage k instead (2: NMS, 3: SAT, 4: octree, 5: node best),
            // so it does not take wave slots from the ORB chain while that chain
            // runs beside region growing
            if (const char* e7 = getenv("PLVI_SOBEL_GATE")) sobelGate = std::min(5, std::max(-1, atoi(e7)));
            // PLVI_SOBEL_AFTER_GROW=1 (batches from 1024 frames): the Sobel
            // pyramid runs on the critical stream after region growing + rect +
            // assemble instead of beside growth on a low-priority stream.  The
            // r04 default (flat then: 47.4K vs 47.6K FPS, lbd_sobel0 3.0-3.3
            // instead of 23-29 ms per launch); since r06, when the ORB chain and
            // not region growing is the longest chain of the two-slot schedule,
            // the line chain's extra work costs more than the Sobel waves beside
            // growth: off by default, 52.6-52.8K -> 53.3-53.5K FPS
            // (profiles/r06/ab_combo.txt)
            if (const char* e8 = getenv("PLVI_SOBEL_AFTER_GROW")) sobelAfterGrow = atoi(e8) != 0;
            if (prio) PLVI_CHECK(hipStreamCreateWithPriority(&critStream, hipStreamNonBlocking, greatest));
            // PLVI_GROW_SPLIT=1: octave 0 grows right after the prep, octave 1
            // after blur + FAST (batches from 1024 frames; +1 % in a 3-way
            // sweep, within run-to-run noise, so off by default)
            const char* e6 = getenv("PLVI_GROW_SPLIT");
            growSplit = e6 && atoi(e6) != 0;
            // crit2 only when split: every greatest-priority stream takes a slot
            // in the runtime's pool of hardware queues, and a pool shared by many
            // handles can put two streams of one schedule on one queue
            if (prio && growSplit)
                PLVI_CHECK(hipStreamCreateWithPriority(&crit2, hipStreamNonBlocking, greatest));
            // normal priority: the octave-1 growth is not the long pole, and the
            // greatest-priority pool stays at two streams per handle
            PLVI_CHECK(hipStreamCreateWithFlags(&octStream, hipStreamNonBlocking));
        }
        for (auto* e : {&evFork, &evPrep, &evSobel, &evOrb, &evCrit, &evBlur, &evGate, &evGrow2, &evPair, &evSobelGo})
            PLVI_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        fcap = p->nfeatures > 0 ? p->nfeatures : kKlCap;
        SCALE = (double)p->lsd_scale;  // LSDOptions::scale is float
        if (!(SCALE > 0) || SCALE > 1) return PLVI_E_BADARG;
        const double ANG_TH = 22.5, QUANT = 2.0, SIGMA_SCALE = 0.6;
        prec = M_PI * ANG_TH / 180;
        const double pp = ANG_TH / 180;
        rho = QUANT / std::sin(prec);
        min_length = 0.025 * std::min(W, H);
        const double sigma = (SCALE < 1) ? (SIGMA_SCALE / SCALE) : SIGMA_SCALE;
        const unsigned hk = (unsigned)std::ceil(sigma * std::sqrt(2 * 3.0 * std::log(10.0)));
        if (SCALE != 1 && 1 + 2 * hk != 7) return PLVI_E_BADARG;  // tile kernel is specialised to 7 taps
        gauss_kernel_f64(7, sigma, gk, (p->compat & PLVI_COMPAT_EXP_CV_TABLE) != 0);
        // SCALE == 1: flsd uses the image as is (lsd.cpp:460-463); identity
        // taps keep every f64 sum exact (0 * I adds +0)
        if (SCALE == 1) gk[0] = gk[1] = gk[2] = 0.0, gk[3] = 1.0;
        // LBD 5x5 sigma 1 fixed-point taps (A.4): error-diffused or rounded
        lbdTaps[0] = 14;
        lbdTaps[1] = (p->compat & PLVI_COMPAT_GAUSS_ROUNDED) ? 63 : 62;
        lbdTaps[2] = (p->compat & PLVI_COMPAT_GAUSS_ROUNDED) ? 103 : 104;
        // ComputePyramid(image, scale, nlevels) (LSDDetector_custom.cpp:76-109)
        scaleF.assign(nOct, 1.f); invScaleF.assign(nOct, 1.f);
        for (int l = 0; l < nOct; ++l) {
            if (l > 0) scaleF[l] = scaleF[l - 1] * p->scale;
            invScaleF[l] = 1.0f / scaleF[l];
        }
        oct.resize(nOct);
        size_t imgOff = 0, sOff = 0, lOff = 0, maxSplane = 0;
        std::vector<uint8_t> tabs;
        auto put = [&](const void* src, size_t n) {
            size_t o = (tabs.size() + 15) & ~size_t(15);
            tabs.resize(o + n);
            std::memcpy(tabs.data() + o, src, n);
            return (long long)o;
        };
        for (int l = 0; l < nOct; ++l) {
            LineOctDev& d = oct[l];
            std::memset(&d, 0, sizeof(d));
            d.w = lround_h((float)W * invScaleF[l]);
            d.h = lround_h((float)H * invScaleF[l]);
            if (l > 0) {
                // exact factor 2 required (INTER_AREA fast path): 640x480, 752x480
                if (d.w * 2 != oct[l - 1].w || d.h * 2 != oct[l - 1].h) return PLVI_E_BADARG;
                if (std::fabs(scaleF[l] / scaleF[l - 1] - 2.0f) > 0) return PLVI_E_BADARG;
            }
            d.plane = (long long)d.w * d.h;
            d.off = (long long)imgOff;
            if (l > 0) imgOff += (size_t)d.plane * Bcap;
            d.sw = SCALE != 1 ? lround_h(d.w * SCALE) : d.w;
            d.sh = SCALE != 1 ? lround_h(d.h * SCALE) : d.h;
            d.splane = (long long)d.sw * d.sh;
            d.soff = (long long)sOff;
            sOff += (size_t)d.splane * Bcap;
            maxSplane = std::max(maxSplane, (size_t)d.splane);
            // lsd.cpp.o computes 5*(.)/2 + log10(11.0) as one fused
            // multiply-add by 0.5 with GCC's folded constant log10(11.0)
            const double LOG_NT = rfma(5 * (std::log10((double)d.sw) + std::log10((double)d.sh)), 0.5,
                                       kLog10Of11);
            d.min_reg_size = (int)(-LOG_NT / std::log10(pp));
            d.octaveScale = (float)std::pow(p->scale, l);
            d.maxWH = std::max(d.w, d.h);
            // resize x SCALE tables (f64 INTER_LINEAR, float coefficients)
            {
                const double sx = 1. / SCALE, sy = 1. / SCALE;
                std::vector<int> xofs(d.sw), yrow(2 * d.sh);
                std::vector<float> xa(2 * d.sw), yb(2 * d.sh);
                int xmax = d.sw;
                for (int dx = 0; dx < d.sw; ++dx) {
                    float fx = (float)((dx + 0.5) * sx - 0.5);
                    int s = lfloor_h(fx);
                    fx -= s;
                    if (s < 0) { fx = 0; s = 0; }
                    if (s + 1 >= d.w) {
                        xmax = std::min(xmax, dx);
                        if (s >= d.w - 1) { fx = 0; s = d.w - 1; }
                    }
                    xofs[dx] = s;
                    xa[2 * dx] = 1.f - fx;
                    xa[2 * dx + 1] = fx;
                }
                for (int dy = 0; dy < d.sh; ++dy) {
                    float fy = (float)((dy + 0.5) * sy - 0.5);
                    int s = lfloor_h(fy);
                    fy -= s;
                    yrow[2 * dy] = std::min(std::max(s, 0), d.h - 1);
                    yrow[2 * dy + 1] = std::min(std::max(s + 1, 0), d.h - 1);
                    yb[2 * dy] = 1.f - fy;
                    yb[2 * dy + 1] = fy;
                }
                d.xmax = xmax;
                // streaming prep strips: scaled columns [X0, X1) plus the
                // gradient's right neighbour, every G column they read
                // (xofs, xofs + 1 where interpolated) on lanes 3..60
                std::vector<int> strips;
                for (int X0 = 0; X0 < d.sw;) {
                    const int gx0 = xofs[X0];
                    int E = X0;
                    while (E < d.sw && xofs[E] + (E < xmax ? 1 : 0) - gx0 + 3 <= 60) ++E;
                    const int X1 = E == d.sw ? E : E - 1;
                    if (X1 <= X0) return PLVI_E_BADARG;
                    strips.insert(strips.end(), {X0, X1, gx0, E - X0});
                    X0 = X1;
                }
                // each G row completes scaled rows whose two source rows are g - 1 or g
                for (int dy = 0; dy < d.sh; ++dy) {
                    const int r1 = yrow[2 * dy + 1], r0 = yrow[2 * dy];
                    if (r0 > r1 || r1 - r0 > 1 || (dy > 0 && r1 < yrow[2 * dy - 1])) return PLVI_E_BADARG;
                }
                d.nstrips = (int)strips.size() / 4;
                d.tabStrips = put(strips.data(), strips.size() * 4);
                // row bands: scaled rows [dyA, dyB) and the first source row
                // a band streams (its first G row needs source rows from
                // yrow[2 dyA] - 3); one band per strip for large batches,
                // kPrepBands for small ones (latency: more waves per frame)
                for (int nb : {1, kPrepBands}) {
                    std::vector<int> bands;
                    for (int b = 0; b < nb; ++b) {
                        const int dyA = (int)((long long)d.sh * b / nb), dyB = (int)((long long)d.sh * (b + 1) / nb);
                        bands.insert(bands.end(), {dyA, dyB, dyA == 0 ? -3 : yrow[2 * dyA] - 3, 0});
                    }
                    (nb == 1 ? d.tabBands1 : d.tabBandsK) = put(bands.data(), bands.size() * 4);
                }
                d.tabXofs = put(xofs.data(), xofs.size() * 4);
                d.tabXa = put(xa.data(), xa.size() * 4);
                d.tabYrow = put(yrow.data(), yrow.size() * 4);
                d.tabYb = put(yb.data(), yb.size() * 4);
            }
            // LBD pyramid (computeGaussianPyramid: pyrDown to (cols/2, rows/2))
            d.lw = l == 0 ? W : oct[l - 1].lw / 2;
            d.lh = l == 0 ? H : oct[l - 1].lh / 2;
            d.lplane = (long long)d.lw * d.lh;
            d.loff = (long long)lOff;
            lOff += (size_t)d.lplane * Bcap;
        }
        lbdPlaneTotal = lOff;
        qspillFrame = maxSplane;
        for (auto& d : oct) gbitsFrame = std::max(gbitsFrame, (size_t)d.sh * (size_t)((d.sw + 31) / 32));
        if (d_oct.alloc(sizeof(LineOctDev) * nOct) || d_tabs.alloc(tabs.size())) return PLVI_E_HIP;
        PLVI_CHECK(hipMemcpy(d_oct.p, oct.data(), sizeof(LineOctDev) * nOct, hipMemcpyHostToDevice));
        PLVI_CHECK(hipMemcpy(d_tabs.p, tabs.data(), tabs.size(), hipMemcpyHostToDevice));
        // LBD tables (BinaryDescriptor ctor, binary_descriptor_custom.cpp:231-260)
        {
            float gL[21], gG[63];
            double u = (7 * 3 - 1) / 2, sg = (7 * 2 + 1) / 2, inv = -1 / (2 * sg * sg);
            for (int i = 0; i < 21; ++i) { double dis = i - u; gL[i] = (float)std::exp(dis * dis * inv); }
            u = (9 * 7 - 1) / 2; sg = u; inv = -1 / (2 * sg * sg);
            for (int i = 0; i < 63; ++i) { double dis = i - u; gG[i] = (float)std::exp(dis * dis * inv); }
            static const unsigned char comb[64] = {0, 1, 0, 2, 0, 3, 0, 4, 0, 5, 0, 6, 1, 2, 1, 3, 1, 4, 1, 5, 1, 6,
                                                   2, 3, 2, 4, 2, 5, 2, 6, 2, 7, 2, 8, 3, 4, 3, 5, 3, 6, 3, 7, 3, 8,
                                                   4, 5, 4, 6, 4, 7, 4, 8, 5, 6, 5, 7, 5, 8, 6, 7, 6, 8, 7, 8};
            PLVI_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_gaussL), gL, sizeof(gL)));
            PLVI_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_gaussG), gG, sizeof(gG)));
            PLVI_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_comb), comb, sizeof(comb)));
        }
        if (octImg.alloc(std::max<size_t>(imgOff, 16)) || pix.alloc(sizeof(float) * sOff) ||
            modg.alloc(sizeof(double) * sOff) || seedcs.alloc(sizeof(float2) * sOff) ||
            gbits.alloc(sizeof(unsigned) * gbitsFrame * nOct * Bcap) || qspill.alloc(sizeof(unsigned) * qspillFrame * nOct * Bcap) ||
            rawLines.alloc(sizeof(LsdLine) * (size_t)kLsdRawCap * nOct * Bcap) ||
            regs.alloc(sizeof(LsdRegion) * (size_t)kLsdRawCap * nOct * Bcap) ||
            regpts.alloc(sizeof(unsigned) * qspillFrame * nOct * Bcap) ||
            nlines.alloc(sizeof(int) * nOct * Bcap) || klTmp.alloc(sizeof(plvi_keyline) * (size_t)kKlCap * Bcap) ||
            sortPos.alloc(sizeof(unsigned short) * 2 * (size_t)kKlCap * Bcap) ||
            klOut.alloc(sizeof(plvi_keyline) * (size_t)fcap * Bcap) || fnOut.alloc(sizeof(double) * 3 * fcap * Bcap) ||
            cntOut.alloc(sizeof(int) * Bcap) || descOut.alloc((size_t)32 * fcap * Bcap) ||
            lbdBlur.alloc((size_t)W * H * Bcap) || lbdG.alloc(sizeof(short2) * lbdPlaneTotal) ||
            err.alloc(sizeof(int) * Bcap) || staging.alloc((size_t)W * H))
            return PLVI_E_HIP;
        PLVI_CHECK(hipMemset(err.p, 0, sizeof(int) * Bcap));
        // region-growing LDS: USED-bits ring (RB rows) + queue + angle ring (R
        // rows, 0 = angles straight from the plane), sized so that every wave of
        // a 3072-frame batch is resident with the kernels that run concurrently.
        // PLVI_GROW_RB: bits rows (power of two >= 2, default 64: regions rarely
        // reach 32 rows below their seed, so USED updates stay in LDS);
        // PLVI_GROW_LDS: total budget (default 6 KB) from which R takes the
        // largest power of two that fits; PLVI_GROW_RD overrides R.
        size_t maxSw = 0;
        for (auto& d : oct) maxSw = std::max(maxSw, (size_t)d.sw);
        const size_t wprMax = (maxSw + 31) / 32;
        size_t budget = 6 * 1024;
        if (const char* e = getenv("PLVI_GROW_LDS")) budget = (size_t)atol(e);
        budget = std::min<size_t>(budget, 160 * 1024);
        growRB = 64;
        if (const char* e = getenv("PLVI_GROW_RB")) growRB = atoi(e);
        if (growRB < 2 || (growRB & (growRB - 1)) || growRB > 1024) return PLVI_E_BADARG;
        growQL = budget >= 32 * 1024 ? 1024 : 256;
        const size_t fixed = (size_t)growQL * sizeof(unsigned) + (size_t)growRB * wprMax * sizeof(unsigned);
        const size_t perRow = maxSw * sizeof(float);
        growR = 0;
        if (fixed + perRow * 2 <= budget) {
            growR = 2;
            while (growR * 2 <= 1024 && fixed + perRow * growR * 2 <= budget) growR *= 2;
        }
        if (const char* e = getenv("PLVI_GROW_RD")) growR = atoi(e);
        if (growR < 0 || (growR & (growR - 1)) || growR == 1 || growR > 1024) return PLVI_E_BADARG;
        growSmem = (fixed + perRow * growR + 15) & ~size_t(15);  // per wave
        if (growSmem > 160 * 1024) return PLVI_E_BADARG;
        // tasks (waves) per workgroup: kGrowWaves, fewer when their LDS
        // partitions would not fit one CU (large PLVI_GROW_LDS budgets)
        growWPW = (int)std::max<size_t>(1, std::min<size_t>(kGrowWaves, (160 * 1024) / growSmem));
        for (const void* k : {(const void*)lsd_grow_kernel<false, false>, (const void*)lsd_grow_kernel<true, false>,
                              (const void*)lsd_grow_kernel<false, true>, (const void*)lsd_grow_kernel<true, true>,
                              (const void*)lsd_grow_kernel<false, true, true>})
            PLVI_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(growSmem * growWPW)));
        // Small batches (latency): lsd_grow_mw_kernel, kMwWaves waves per
        // (frame, octave) growing regions of one frame concurrently.
        // PLVI_GROW_MW = largest batch that takes it (default 256; 0 = off).
        mwMaxFrames = 256;
        if (const char* e = getenv("PLVI_GROW_MW")) mwMaxFrames = atoi(e);
        if (const char* e = getenv("PLVI_GROW_TPW")) growTPW = std::max(0, atoi(e));
        mwMaxFrames = std::min(mwMaxFrames, Bcap);
        if (mwMaxFrames > 0) {
            // LDS: ctl + dispatch log + C/T/H bitmaps + own windows + growth
            // queues, the rest for the slot pool (up to kMwMaxSlots)
            const size_t nwords = gbitsFrame;  // max over octaves of sh * wpr
            const size_t fixedMw = sizeof(MwCtl) + 8 * kMwLog +
                                   4 * (3 * nwords + (size_t)kMwWaves * kMwRB * wprMax + (size_t)kMwWaves * kMwGQ);
            const size_t ldsMax = 160 * 1024;
            mwSlots = fixedMw < ldsMax ? (int)std::min<size_t>(kMwMaxSlots, (ldsMax - fixedMw) / kMwSlotBytes) : 0;
            mwSmem = fixedMw + (size_t)mwSlots * kMwSlotBytes;
            if (mwSlots < 2 * kMwWaves) {
                mwMaxFrames = 0;  // frame too large for the LDS bitmaps: sequential kernel only
            } else {
                const size_t tasks = (size_t)mwMaxFrames * nOct;
                mwOwnTask = (size_t)kMwWaves * gbitsFrame;
                if (mwOwn.alloc(sizeof(unsigned) * mwOwnTask * tasks) ||
                    mwSlot.alloc(sizeof(unsigned) * (size_t)mwSlots * kMwSlotSpill * tasks) ||
                    mwGrow.alloc(sizeof(unsigned) * (size_t)kMwWaves * kMwGSpill * tasks))
                    return PLVI_E_HIP;
                PLVI_CHECK(hipMemset(mwOwn.p, 0, mwOwn.bytes));  // kept zero by every launch
                for (const void* k : {(const void*)lsd_grow_mw_kernel<kMwWaves, false>,
                                      (const void*)lsd_grow_mw_kernel<kMwWaves, true>})
                    PLVI_CHECK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mwSmem));
            }
        }
        return PLVI_OK;
    }
#ifndef PLVI_MW_WAVES
#define PLVI_MW_WAVES 16
#endif
    static constexpr int kMwWaves = PLVI_MW_WAVES;  // waves per (frame, octave) of the multi-wave kernel
    int mwMaxFrames = 0, mwSlots = 0;
    size_t mwSmem = 0, mwOwnTask = 0;
    int* mwStats = nullptr;  // diagnostic counters (plvi_lines_debug_mw_stats)
    DevBuf mwEpoch;          // PLVI_MW_DIAG variant: commit-epoch map per task
    size_t growSmem = 0;
    int growWPW = 1;  // region-growing tasks (waves) per workgroup
    // region-growing tasks per wave of the large-batch kernel: 2 = octave 0
    // and octave 1 of a frame in one wave, half the resident growth waves
    // (3 per SIMD at 3072 frames instead of 6, so the two batches in flight
    // can grow at once and blur + FAST shares a SIMD with 3 growth waves
    // instead of 6).  PLVI_GROW_TPW=0 selects the rule: 2 in the frame
    // schedule (run_with_orb) from 2048 frames, else 1 -- a lines-only batch
    // alone on the chip grows faster with every task in its own wave (30 vs
    // 40 ms at 3072 frames).  The rule was the default while the ORB chain
    // was the longer chain of a slot (52.9-53.0K -> 53.0-53.3K FPS, blur +
    // FAST in the timed window 15-17 -> 10-12 ms, profiles/r06/ab_knn_tpw.txt);
    // after the candidate-list ORB middle the line chain is the longer one
    // and one task per wave is faster again (54.9K -> 55.9K FPS, blur + FAST
    // in the window 12 -> 16-17 ms, profiles/r06/ab_resweep.txt): default 1
    int growTPW = 1;  // 0: the rule above
    bool inSchedule = false;  // run_with_orb is issuing
    int growR = 0, growRB = 0, growQL = 0;
    unsigned long long* growStats = nullptr;  // diagnostic cycle counters (plvi_lines_debug_stats)

    int profile(int on) {
        if (on && evs.empty()) {
            evs.resize((size_t)kRing * (kStages + 1));
            for (auto& e : evs) PLVI_CHECK(hipEventCreate(&e));
        }
        prof = on != 0;
        profRuns = 0;
        return PLVI_OK;
    }
    void mark(int s, hipStream_t st) {
        if (prof && profRuns < kRing) (void)hipEventRecord(evs[(size_t)profRuns * (kStages + 1) + s], st);
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

    // Phase A: octave pyramid + LSD prep (LK1, LK2).
    void launch_prep(const uint8_t* d_frames, int nf, size_t frame_stride, size_t row_stride, hipStream_t st,
                     int lFirst = 0, int lEnd = -1) {
        const uint8_t* T = d_tabs.as<uint8_t>();
        if (lEnd < 0) lEnd = nOct;
        for (int l = 1; l < nOct && lFirst == 0; ++l) {
            const LineOctDev& d = oct[l];
            const uint8_t* s = l == 1 ? d_frames : octImg.as<uint8_t>() + oct[l - 1].off;
            const size_t sf = l == 1 ? frame_stride : (size_t)oct[l - 1].plane;
            const size_t sr = l == 1 ? row_stride : (size_t)oct[l - 1].w;
            hipLaunchKernelGGL(lsd_half_kernel, dim3((d.w * d.h + 255) / 256, nf), dim3(256), 0, st, s, sf, sr,
                               octImg.as<uint8_t>() + d.off, d.w, d.h, (size_t)d.plane);
        }
        if (lFirst == 0) mark(1, st);
        for (int l = lFirst; l < lEnd; ++l) {
            const LineOctDev& d = oct[l];
            const uint8_t* s = l == 0 ? d_frames : octImg.as<uint8_t>() + d.off;
            const size_t sf = l == 0 ? frame_stride : (size_t)d.plane;
            const size_t sr = l == 0 ? row_stride : (size_t)d.w;
            const bool kt = ktime && kn < kKRing;
            if (kt) (void)hipEventRecord(kev[2 * kn], st);
            const bool banded = nf <= kPrepBandMax;
            hipLaunchKernelGGL(lsd_prep_kernel, dim3(d.nstrips, nf, banded ? kPrepBands : 1), dim3(64), 0, st, s, sf,
                               sr, d.w, d.h, d.sw, d.sh, (const int4*)(T + d.tabStrips),
                               (const int4*)(T + (banded ? d.tabBandsK : d.tabBands1)), (const int*)(T + d.tabXofs),
                               (const float*)(T + d.tabXa), d.xmax, (const int*)(T + d.tabYrow),
                               (const float*)(T + d.tabYb), gk[0], gk[1], gk[2], gk[3], rho,
                               pix.as<float>() + d.soff, modg.as<double>() + d.soff, seedcs.as<float2>() + d.soff,
                               (size_t)d.splane);
            if (kt) {
                (void)hipEventRecord(kev[2 * kn + 1], st);
                ++kn;
            }
        }
        if (lEnd == nOct) mark(2, st);
    }

    // Phase B: region growing (LK3) + keyline assembly / top-k (LK4).
    // region growing of octaves [oBase, oBase + oCount) (LK3)
    void launch_grow(int nf, int oBase, int oCount, hipStream_t st) {
        if (nf <= mwMaxFrames) {
            auto mwK = mwStats ? lsd_grow_mw_kernel<kMwWaves, true> : lsd_grow_mw_kernel<kMwWaves, false>;
            hipLaunchKernelGGL(mwK, dim3(oCount * nf), dim3(kMwWaves * 64), mwSmem, st, d_oct.as<LineOctDev>(),
                               (const float*)pix.as<float>(), (const float2*)seedcs.as<float2>(),
                               mwOwn.as<unsigned>(), mwOwnTask, mwGrow.as<unsigned>(), mwSlot.as<unsigned>(),
                               qspill.as<unsigned>(), qspillFrame, prec, regs.as<LsdRegion>(), regpts.as<unsigned>(),
                               qspillFrame, nlines.as<int>(), err.as<int>(), mwSlots, nOct, oBase, oCount, mwStats, nf,
                               mwStats && PLVI_MW_DIAG ? mwEpoch.as<int>() : nullptr);
            return;
        }
        const bool fixedWin = growR == 0 && growRB == kGrowRB && growQL == kGrowQL;
        // (the multi-task loop is built for the default windows only)
        const int tpwWant = growTPW > 0 ? growTPW : (inSchedule && nf >= 2048 ? 2 : 1);
        const int tpw = tpwWant > 1 && !growStats && fixedWin ? tpwWant : 1;
        auto growK = growStats ? (fixedWin ? lsd_grow_kernel<true, true> : lsd_grow_kernel<true, false>)
                               : (fixedWin ? (tpw > 1 ? lsd_grow_kernel<false, true, true> : lsd_grow_kernel<false, true>)
                                           : lsd_grow_kernel<false, false>);
        const int waves = (oCount * nf + tpw - 1) / tpw;
        hipLaunchKernelGGL(growK, dim3((waves + growWPW - 1) / growWPW), dim3(64 * growWPW),
                           growSmem * growWPW, st, d_oct.as<LineOctDev>(),
                           (const float*)pix.as<float>(), (const double*)modg.as<double>(),
                           (const float2*)seedcs.as<float2>(), gbits.as<unsigned>(), gbitsFrame,
                           qspill.as<unsigned>(), qspillFrame, prec, regs.as<LsdRegion>(), regpts.as<unsigned>(),
                           qspillFrame, nlines.as<int>(), err.as<int>(), growR, growRB, growQL, nOct, oBase, oCount,
                           growStats, nf, (int)growSmem, growWPW);
    }
    // region2rect (lane = region) of octaves [oBase, oBase + oCount); small
    // batches spread a frame's regions over more workgroups (latency)
    void launch_rect(int nf, int oBase, int oCount, hipStream_t st) {
        const int bx = nf <= 16 ? 8 : kRectLaneBlocks;
        auto rectK = nf <= kRectSmallNf ? lsd_rect_lanes_kernel<kRectUSmall> : lsd_rect_lanes_kernel<kRectU>;
        hipLaunchKernelGGL(rectK, dim3(bx, nf, oCount), dim3(256), 0, st, d_oct.as<LineOctDev>(),
                           (const double*)modg.as<double>(), (const LsdRegion*)regs.as<LsdRegion>(),
                           (const unsigned*)regpts.as<unsigned>(), qspillFrame, (const int*)nlines.as<int>(), prec,
                           SCALE, rawLines.as<LsdLine>(), oBase, nOct);
    }
    // grown: region growing already launched; rect0: only octave 0's
    // region2rect is left (the other octaves' ran behind their growth on
    // the side stream, which the caller joined)
    void launch_grow_assemble(int nf, hipStream_t st, bool grown = false, bool rect0 = false) {
        if (!grown) launch_grow(nf, 0, nOct, st);
        launch_rect(nf, 0, rect0 ? 1 : nOct, st);
        mark(3, st);
        hipLaunchKernelGGL(line_assemble_kernel, dim3(nf), dim3(256), 0, st, d_oct.as<LineOctDev>(), nOct,
                           (const LsdLine*)rawLines.as<LsdLine>(), (const int*)nlines.as<int>(), min_length,
                           prm.nfeatures, fcap, klOut.as<plvi_keyline>(), fnOut.as<double>(), cntOut.as<int>(),
                           klTmp.as<plvi_keyline>(), err.as<int>(), sortPos.as<unsigned short>());
        mark(4, st);
    }

    // LB1/LB2: LBD Gaussian pyramid + Sobel (depends on the frames only).
    int launch_sobel(const uint8_t* d_frames, int nf, size_t frame_stride, size_t row_stride, hipStream_t st) {
        const LineOctDev& d0 = oct[0];
        {
            // column strips of at most kLbOutLanes * 4 columns, balanced, multiples of 4
            const int ns = (d0.lw + 4 * kLbOutLanes - 1) / (4 * kLbOutLanes);
            const int sw4 = ((d0.lw + ns - 1) / ns + 3) & ~3;
            ktimeS(0, 0, st);
            hipLaunchKernelGGL(lbd_sobel0_kernel, dim3((d0.lw + sw4 - 1) / sw4, nf, kLbBands), dim3(64), 0, st, d_frames,
                               frame_stride, row_stride, d0.lw, d0.lh, sw4, lbdBlur.as<uint8_t>(),
                               lbdG.as<short2>() + d0.loff, (size_t)d0.lplane, lbdTaps[0], lbdTaps[1], lbdTaps[2]);
            ktimeS(0, 1, st);
        }
        for (int l = 1; l < nOct; ++l) {
            const LineOctDev& d = oct[l];
            if (l > 1) return PLVI_E_BADARG;  // pyrDown chain beyond octave 1 not wired (config: 2 levels)
            const int ns = (d.lw + 2 * kLb2OutLanes - 1) / (2 * kLb2OutLanes);
            const int sw2 = ((d.lw + ns - 1) / ns + 1) & ~1;
            ktimeS(1, 0, st);
            hipLaunchKernelGGL(lbd_sobel1_kernel, dim3((d.lw + sw2 - 1) / sw2, nf), dim3(64), 0, st,
                               (const uint8_t*)lbdBlur.as<uint8_t>(), d0.lw, d0.lh, (size_t)d0.lplane, d.lw, d.lh,
                               sw2, lbdG.as<short2>() + d.loff, (size_t)d.lplane);
            ktimeS(1, 1, st);
        }
        return PLVI_OK;
    }

    // LB3: LBD descriptors of the assembled keylines.
    void launch_describe(int nf, hipStream_t st) {
        hipLaunchKernelGGL(lbd_describe_kernel, dim3(fcap, nf), dim3(64), 0, st, d_oct.as<LineOctDev>(),
                           (const short2*)lbdG.as<short2>(),
                           (const plvi_keyline*)klOut.as<plvi_keyline>(), (const int*)cntOut.as<int>(), fcap,
                           descOut.as<uint8_t>());
        mark(5, st);
    }

    int run(const uint8_t* d_frames, int nf, size_t frame_stride, size_t row_stride, hipStream_t st) {
        if (nf <= 0 || nf > Bcap) return PLVI_E_BADARG;
        if (!st) st = stream;
        lastFrames = nf;
        // the LBD Sobel pyramid depends on the frames only: it runs on aux[1]
        // beside prep + region growing and joins before the LBD describe
        // (stage profiling and stream capture keep the sequential order)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        PLVI_CHECK(hipStreamIsCapturing(st, &cs));
        const bool fork = !prof && aux[1] && cs == hipStreamCaptureStatusNone;
        int rc = PLVI_OK;
        if (fork) {
            PLVI_CHECK(hipEventRecord(evFork, st));
            PLVI_CHECK(hipStreamWaitEvent(aux[1], evFork, 0));
            rc = launch_sobel(d_frames, nf, frame_stride, row_stride, aux[1]);
            PLVI_CHECK(hipEventRecord(evSobel, aux[1]));
        }
        mark(0, st);
        if (fork && nOct > 1 && nf <= mwMaxFrames) {
            // small batches (latency): octave 0's region growing, the long
            // pole, starts right after its own prep; the other octaves are
            // prepared and grown on aux[0] beside it
            launch_prep(d_frames, nf, frame_stride, row_stride, st, 0, 1);
            PLVI_CHECK(hipEventRecord(evPrep, st));
            PLVI_CHECK(hipStreamWaitEvent(aux[0], evPrep, 0));
            launch_prep(d_frames, nf, frame_stride, row_stride, aux[0], 1, nOct);
            launch_grow(nf, 1, nOct - 1, aux[0]);
            launch_rect(nf, 1, nOct - 1, aux[0]);  // beside octave 0's growth
            PLVI_CHECK(hipEventRecord(evGrow2, aux[0]));
            launch_grow(nf, 0, 1, st);
            PLVI_CHECK(hipStreamWaitEvent(st, evGrow2, 0));
            launch_grow_assemble(nf, st, true, true);
        } else {
            launch_prep(d_frames, nf, frame_stride, row_stride, st);
            launch_grow_assemble(nf, st);
        }
        if (fork) {
            PLVI_CHECK(hipStreamWaitEvent(st, evSobel, 0));
        } else {
            rc = launch_sobel(d_frames, nf, frame_stride, row_stride, st);
        }
        if (rc) return rc;
        launch_describe(nf, st);
        if (prof && profRuns < kRing) ++profRuns;
        PLVI_CHECK(hipGetLastError());
        return PLVI_OK;
    }

    // Frame::Frame's two extractor threads (Frame.cc:558-561) as one
    // schedule: the latency-bound region growing runs while the ORB
    // extractor and the LBD Sobel pyramid fill the machine on two more
    // streams; everything joins back on `st`.
    // the step's matching, issued inside the schedule (plvi_frame_extract_match_batch)
    struct StepMatch {
        int *idx0, *d0, *idx1, *d1;
        float nnr;
        int *lscratch, *lm12, *lnm;
    };
    int run_with_orb(const uint8_t* d_frames, int nf, size_t frame_stride, size_t row_stride, hipStream_t st,
                     plvi_orb_extractor* orb, int lap0, int lap1, const StepMatch* sm = nullptr) {
        if (nf <= 0 || nf > Bcap) return PLVI_E_BADARG;
        if (!st) st = stream;
        lastFrames = nf;
        const bool p0 = prof;
        prof = false;  // stage events are meaningless across streams
        inSchedule = true;
        // the critical path (prep -> region growing -> LBD describe) runs on
        // the high-priority stream `crit`; ORB and the Sobel pyramid on the
        // low-priority aux streams, started after prep (orbAfterPrep) or at once
        hipStream_t crit = critStream ? critStream : st;
        PLVI_CHECK(hipEventRecord(evFork, st));
        if (crit != st) PLVI_CHECK(hipStreamWaitEvent(crit, evFork, 0));
        // small batches (multi-wave growth): octave 0, the long pole, grows
        // right after its own prep; the other octaves are prepared and grown
        // on octStream beside it
        const bool octFirst = nf <= mwMaxFrames && nOct > 1 && octStream;
        launch_prep(d_frames, nf, frame_stride, row_stride, crit, 0, octFirst ? 1 : nOct);
        PLVI_CHECK(hipEventRecord(evPrep, crit));
        if (octFirst) {
            PLVI_CHECK(hipStreamWaitEvent(octStream, evPrep, 0));
            launch_prep(d_frames, nf, frame_stride, row_stride, octStream, 1, nOct);
            launch_grow(nf, 1, nOct - 1, octStream);
            launch_rect(nf, 1, nOct - 1, octStream);  // beside octave 0's growth
            PLVI_CHECK(hipEventRecord(evGrow2, octStream));
        }
        hipEvent_t auxStart = (orbAfterPrep >= 2 || (orbAfterPrep == 1 && nf < 1024)) ? evPrep : evFork;
        PLVI_CHECK(hipStreamWaitEvent(aux[0], auxStart, 0));
        // only a batch whose region-growing waves fill the SIMDs (>= 2 per SIMD
        // from 1024 frames on) starves blur + FAST; a small batch is latency-bound
        // and starts region growing right after the prep
        const bool waitBlur = growAfterBlur && nf >= 1024;
        const bool sobelLate = waitBlur && sobelGate >= 0;
        if (waitBlur) plvi_orb_internal_blur_event(orb, evBlur);
        if (sobelLate) plvi_orb_internal_stage_event(orb, sobelGate, evSobelGo);
        int rc = plvi_orb_extract_batch(orb, d_frames, nf, frame_stride, row_stride, lap0, lap1, aux[0]);
        if (waitBlur) plvi_orb_internal_blur_event(orb, nullptr);
        if (sobelLate) plvi_orb_internal_stage_event(orb, -1, nullptr);
        if (sm && !rc) {
            // ORB kNN-2 of frame t vs t-1 right behind the ORB chain
            plvi_keypoint* kp = nullptr;
            uint8_t* de = nullptr;
            int *co = nullptr, *mo = nullptr, cap = 0;
            rc = plvi_orb_outputs(orb, &kp, &de, &co, &mo, &cap);
            if (!rc)
                rc = plvi_hamming_knn2_batch(de + (size_t)cap * 32, co + 1, cap, de, co, cap, nf - 1, sm->idx0, sm->d0,
                                             sm->idx1, sm->d1, aux[0]);
        }
        PLVI_CHECK(hipEventRecord(evOrb, aux[0]));
        // split: octave 0 (the long waves, 3 per SIMD at 3072 frames) grows
        // right after the prep and leaves room for the ORB pyramid and blur +
        // FAST; the shorter octave-1 waves start after blur + FAST on crit2
        const bool split = waitBlur && growSplit && nOct == 2 && crit2 && !rc;
        hipStream_t gate = split ? crit2 : crit;
        if (split) {
            launch_grow(nf, 0, 1, crit);
            PLVI_CHECK(hipStreamWaitEvent(crit2, evPrep, 0));
        }
        if (waitBlur && !rc) PLVI_CHECK(hipStreamWaitEvent(gate, evBlur, 0));
        // evGate: everything the (last) region-growing launch waits for
        PLVI_CHECK(hipEventRecord(evGate, gate));
        const bool sobelAfter = sobelAfterGrow && waitBlur;
        if (!sobelAfter) {
            PLVI_CHECK(hipStreamWaitEvent(aux[1], sobelLate ? evSobelGo : sobelWithGrow ? evGate : auxStart, 0));
            if (!rc) rc = launch_sobel(d_frames, nf, frame_stride, row_stride, aux[1]);
            PLVI_CHECK(hipEventRecord(evSobel, aux[1]));
        }
        if (split) {
            launch_grow(nf, 1, 1, crit2);
            PLVI_CHECK(hipEventRecord(evGrow2, crit2));
            PLVI_CHECK(hipStreamWaitEvent(crit, evGrow2, 0));
        }
        if (octFirst) {
            launch_grow(nf, 0, 1, crit);
            PLVI_CHECK(hipStreamWaitEvent(crit, evGrow2, 0));
            launch_grow_assemble(nf, crit, true, true);
        } else {
            launch_grow_assemble(nf, crit, split);
        }
        if (sobelAfter) {
            if (!rc) rc = launch_sobel(d_frames, nf, frame_stride, row_stride, crit);
        } else {
            PLVI_CHECK(hipStreamWaitEvent(crit, evSobel, 0));
        }
        launch_describe(nf, crit);
        if (sm && !rc) {
            // LineMatcher::match of frame t vs t-1 right behind the LBD descriptors
            uint8_t* ld = descOut.as<uint8_t>();
            int* lc = cntOut.as<int>();
            rc = plvi_line_match_batch(ld + (size_t)fcap * 32, lc + 1, fcap, ld, lc, fcap, nf - 1, sm->nnr,
                                       sm->lscratch, sm->lm12, sm->lnm, crit);
        }
        if (crit != st) {
            PLVI_CHECK(hipEventRecord(evCrit, crit));
            PLVI_CHECK(hipStreamWaitEvent(st, evCrit, 0));
        }
        PLVI_CHECK(hipStreamWaitEvent(st, evOrb, 0));
        prof = p0;
        inSchedule = false;
        PLVI_CHECK(hipGetLastError());
        return rc;
    }
};

}  // namespace plvi

using plvi::LinePipeline;

// Pipeline held by pointer so a frame-size change can re-plan the handle
// (Lineextractor::operator() takes any image, LineExtractor.cc:45).
struct plvi_line_extractor {
    std::unique_ptr<LinePipeline> up;
    LinePipeline& p() { return *up; }
    int replan(int width, int height) {
        if (width == up->W && height == up->H) return PLVI_OK;
        PLVI_CHECK(hipStreamSynchronize(up->stream));
        auto np = std::make_unique<LinePipeline>();
        int rc = np->init(&up->prm, width, height, up->Bcap, up->device);
        if (rc) return rc;
        np->growStats = nullptr;
        up = std::move(np);
        return PLVI_OK;
    }
};

extern "C" int plvi_lines_create(const plvi_line_params* p, int width, int height, int max_batch, int device,
                                 plvi_line_extractor** out) {
    if (!out) return PLVI_E_BADARG;
    *out = nullptr;
    auto h = std::make_unique<plvi_line_extractor>();
    h->up = std::make_unique<LinePipeline>();
    int rc = h->p().init(p, width, height, max_batch, device);
    if (rc) return rc;
    *out = h.release();
    return PLVI_OK;
}

extern "C" int plvi_lines_destroy(plvi_line_extractor* h) {
    if (!h) return PLVI_E_BADARG;
    (void)hipSetDevice(h->p().device);
    (void)hipStreamSynchronize(h->p().stream);
    delete h;
    return PLVI_OK;
}

extern "C" int plvi_lines_extract_batch(plvi_line_extractor* h, const uint8_t* d_frames, int n_frames,
                                        size_t frame_stride, size_t row_stride, void* stream) {
    if (!h || !d_frames) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().run(d_frames, n_frames, frame_stride, row_stride, (hipStream_t)stream);
}

extern "C" int plvi_frame_extract_batch(plvi_orb_extractor* orb, plvi_line_extractor* lines, const uint8_t* d_frames,
                                        int n_frames, size_t frame_stride, size_t row_stride, int lap0, int lap1,
                                        void* stream) {
    if (!orb || !lines || !d_frames) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(lines->p().device));
    if (stream) {
        // Capturing the fork/join of this schedule crashes inside
        // hipStreamEndCapture on the HIP 7.0 runtime that PyTorch bundles
        // (torch/lib/libamdhip64.so, mapped by any process that imports torch
        // first); ROCm 7.2's runtime captures and replays it bit-exactly
        // (tests/test_frame_gpu.py, tools/graph_probe.py).  Refuse the capture
        // on older runtimes instead of letting it crash later.
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        PLVI_CHECK(hipStreamIsCapturing((hipStream_t)stream, &cs));
        int ver = 0;
        PLVI_CHECK(hipRuntimeGetVersion(&ver));
        if (cs != hipStreamCaptureStatusNone && ver < 70200000) return PLVI_E_CAPTURE;
    }
    return lines->p().run_with_orb(d_frames, n_frames, frame_stride, row_stride, (hipStream_t)stream, orb, lap0, lap1);
}

extern "C" int plvi_frame_extract_match_batch(plvi_orb_extractor* orb, plvi_line_extractor* lines,
                                              const uint8_t* d_frames, int n_frames, size_t frame_stride,
                                              size_t row_stride, int lap0, int lap1, int* d_idx0, int* d_d0,
                                              int* d_idx1, int* d_d1, float nnr, int* d_line_scratch,
                                              int* d_line_matches, int* d_line_nmatch, void* stream) {
    if (!orb || !lines || !d_frames || n_frames < 2 || !d_idx0 || !d_d0 || !d_idx1 || !d_d1 || !d_line_scratch ||
        !d_line_matches || !d_line_nmatch)
        return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(lines->p().device));
    if (stream) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        PLVI_CHECK(hipStreamIsCapturing((hipStream_t)stream, &cs));
        int ver = 0;
        PLVI_CHECK(hipRuntimeGetVersion(&ver));
        if (cs != hipStreamCaptureStatusNone && ver < 70200000) return PLVI_E_CAPTURE;
    }
    const LinePipeline::StepMatch sm{d_idx0, d_d0, d_idx1, d_d1, nnr, d_line_scratch, d_line_matches, d_line_nmatch};
    return lines->p().run_with_orb(d_frames, n_frames, frame_stride, row_stride, (hipStream_t)stream, orb, lap0,
                                   lap1, &sm);
}

extern "C" int plvi_frame_orb_event(plvi_line_extractor* lines, void** event) {
    if (!lines || !event) return PLVI_E_BADARG;
    *event = (void*)lines->p().evOrb;
    return PLVI_OK;
}

// The stereo-line Frame (src/Frame.cc:200-249): ORB left || right and lines
// left || right as two frame schedules that run concurrently, the right one
// forked from the caller's stream onto the right line handle's own stream and
// joined back, so the caller's stream holds all four extractions (stereo
// matching follows on it: plvi_stereo_match_batch / plvi_stereo_lines_batch).
extern "C" int plvi_stereo_frame_extract_batch(plvi_orb_extractor* orb_left, plvi_orb_extractor* orb_right,
                                               plvi_line_extractor* lines_left, plvi_line_extractor* lines_right,
                                               const uint8_t* d_left, const uint8_t* d_right, int n_frames,
                                               size_t frame_stride, size_t row_stride, int lap0, int lap1,
                                               void* stream) {
    if (!orb_left || !orb_right || !lines_left || !lines_right || !d_left || !d_right) return PLVI_E_BADARG;
    if (orb_left == orb_right || lines_left == lines_right) return PLVI_E_BADARG;  // each side owns its tables
    LinePipeline& L = lines_left->p();
    LinePipeline& R = lines_right->p();
    if (L.device != R.device) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(L.device));
    hipStream_t st = stream ? (hipStream_t)stream : L.stream;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    PLVI_CHECK(hipStreamIsCapturing(st, &cs));
    int ver = 0;
    PLVI_CHECK(hipRuntimeGetVersion(&ver));
    if (cs != hipStreamCaptureStatusNone && ver < 70200000) return PLVI_E_CAPTURE;  // see plvi_frame_extract_batch
    // fork the right side off the caller's stream
    PLVI_CHECK(hipEventRecord(R.evPair, st));
    PLVI_CHECK(hipStreamWaitEvent(R.stream, R.evPair, 0));
    int rc = L.run_with_orb(d_left, n_frames, frame_stride, row_stride, st, orb_left, lap0, lap1);
    int rc2 = R.run_with_orb(d_right, n_frames, frame_stride, row_stride, R.stream, orb_right, lap0, lap1);
    // join it back
    PLVI_CHECK(hipEventRecord(L.evPair, R.stream));
    PLVI_CHECK(hipStreamWaitEvent(st, L.evPair, 0));
    return rc ? rc : rc2;
}

extern "C" int plvi_lines_outputs(plvi_line_extractor* h, plvi_keyline** d_kl, uint8_t** d_desc, double** d_fn,
                                  int** d_count, int* cap) {
    if (!h) return PLVI_E_BADARG;
    if (d_kl) *d_kl = h->p().klOut.as<plvi_keyline>();
    if (d_desc) *d_desc = h->p().descOut.as<uint8_t>();
    if (d_fn) *d_fn = h->p().fnOut.as<double>();
    if (d_count) *d_count = h->p().cntOut.as<int>();
    if (cap) *cap = h->p().fcap;
    return PLVI_OK;
}

extern "C" int plvi_lines_errors(plvi_line_extractor* h, int* frame_flags, int* any, void* stream) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    hipStream_t st = stream ? (hipStream_t)stream : h->p().stream;
    return plvi::read_frame_errors(h->p().err.as<int>(), h->p().Bcap, frame_flags, any, st);
}

extern "C" int plvi_lines_extract(plvi_line_extractor* h, const uint8_t* img, int width, int height, size_t stride,
                                  plvi_keyline* kl, uint8_t* desc, double* line_fns, int cap, int* n) {
    if (!h) return PLVI_E_BADARG;
    if (n) *n = 0;
    if (!img || width <= 0 || height <= 0) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    if (int rc = h->replan(width, height)) return rc;
    LinePipeline& P = h->p();
    PLVI_CHECK(hipMemcpy2DAsync(P.staging.p, (size_t)P.W, img, stride, (size_t)P.W, (size_t)P.H,
                                hipMemcpyHostToDevice, P.stream));
    int rc = P.run(P.staging.as<uint8_t>(), 1, (size_t)P.W * P.H, (size_t)P.W, P.stream);
    if (rc) return rc;
    int cnt = 0, errv = 0;
    PLVI_CHECK(hipMemcpyAsync(&cnt, P.cntOut.p, sizeof(int), hipMemcpyDeviceToHost, P.stream));
    PLVI_CHECK(hipMemcpyAsync(&errv, P.err.p, sizeof(int), hipMemcpyDeviceToHost, P.stream));
    PLVI_CHECK(hipStreamSynchronize(P.stream));
    if (errv) {
        PLVI_CHECK(hipMemset(P.err.p, 0, sizeof(int) * P.Bcap));
        return PLVI_E_OVERFLOW;
    }
    if (n) *n = cnt;
    if (cnt > cap) return PLVI_E_CAPACITY;
    if (cnt > 0) {
        if (kl) PLVI_CHECK(hipMemcpy(kl, P.klOut.p, sizeof(plvi_keyline) * cnt, hipMemcpyDeviceToHost));
        if (desc) PLVI_CHECK(hipMemcpy(desc, P.descOut.p, (size_t)32 * cnt, hipMemcpyDeviceToHost));
        if (line_fns) PLVI_CHECK(hipMemcpy(line_fns, P.fnOut.p, sizeof(double) * 3 * cnt, hipMemcpyDeviceToHost));
    }
    return PLVI_OK;
}

extern "C" int plvi_lines_pyramid_level(plvi_line_extractor* h, int frame, int level, uint8_t* dst, int* w,
                                        int* hgt) {
    if (!h || level < 0 || level >= h->p().nOct || frame < 0 || frame >= h->p().Bcap) return PLVI_E_BADARG;
    const auto& d = h->p().oct[level];
    if (w) *w = d.w;
    if (hgt) *hgt = d.h;
    if (!dst) return PLVI_OK;
    if (level == 0) return PLVI_E_BADARG;  // level 0 is the caller's own image (gaussianPyrs[0] == image)
    PLVI_CHECK(hipSetDevice(h->p().device));
    PLVI_CHECK(hipStreamSynchronize(h->p().stream));
    PLVI_CHECK(hipMemcpy(dst, h->p().octImg.as<uint8_t>() + d.off + (size_t)frame * d.plane, (size_t)d.plane,
                         hipMemcpyDeviceToHost));
    return PLVI_OK;
}

extern "C" int plvi_lines_scale_tables(plvi_line_extractor* h, float* scale, float* inv_scale, float* sigma2,
                                       float* inv_sigma2) {
    if (!h) return PLVI_E_BADARG;
    const auto& P = h->p();
    for (int i = 0; i < P.nOct; ++i) {
        // Lineextractor (LineExtractor.cc:88-99): sigma2[0] = 1, sigma2[i] = s*s
        const float s = P.scaleF[i];
        const float s2 = i > 0 ? s * s : 1.0f;
        if (scale) scale[i] = s;
        if (inv_scale) inv_scale[i] = P.invScaleF[i];
        if (sigma2) sigma2[i] = s2;
        if (inv_sigma2) inv_sigma2[i] = 1.0f / s2;
    }
    return PLVI_OK;
}

extern "C" int plvi_lines_profile(plvi_line_extractor* h, int enable) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().profile(enable);
}

extern "C" int plvi_lines_profile_read(plvi_line_extractor* h, float* stage_ms, int* runs) {
    if (!h || !stage_ms) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().profile_read(stage_ms, runs);
}

// Diagnostic: enable per-task cycle accounting of the region-growing kernel
// into a caller-provided device buffer of n_frames*nlevels*24 uint64 (NULL disables):
// [0..15] cycle counters, [16] HW_ID, [17] XCC_ID, [18] start time (s_memtime).
extern "C" int plvi_lines_debug_stats(plvi_line_extractor* h, unsigned long long* d_stats) {
    if (!h) return PLVI_E_BADARG;
    h->p().growStats = d_stats;
    return PLVI_OK;
}

// Diagnostic: counters of the multi-wave region-growing kernel per (frame,
// octave): 16 ints (plvi_frontend.h) into a caller-provided device buffer
// (NULL disables).
extern "C" int plvi_lines_debug_mw_stats(plvi_line_extractor* h, int* d_stats) {
    if (!h) return PLVI_E_BADARG;
    h->p().mwStats = d_stats;
    // the diagnostic variant's commit-epoch map: one int per bit of every
    // (frame, octave) task's bitmaps
    if (PLVI_MW_DIAG && d_stats && !h->p().mwEpoch.p &&
        h->p().mwEpoch.alloc(sizeof(int) * 32 * h->p().gbitsFrame * (size_t)h->p().mwMaxFrames * h->p().nOct))
        return PLVI_E_HIP;
    return PLVI_OK;
}

// Diagnostic: the LSD planes of the last batch for one (frame, octave):
// angle in degrees (float, NOTDEF = -1024), modgrad (f64) and the per-pixel
// cos/sin pairs (valid where the angle is defined), copied to host memory.
extern "C" int plvi_lines_debug_planes(plvi_line_extractor* h, int frame, int octave, float* deg, double* modgrad,
                                       float* cs, int* sw, int* sh) {
    if (!h || octave < 0 || octave >= h->p().nOct || frame < 0 || frame >= h->p().Bcap) return PLVI_E_BADARG;
    LinePipeline& P = h->p();
    PLVI_CHECK(hipSetDevice(P.device));
    const plvi::LineOctDev& d = P.oct[octave];
    const size_t n = (size_t)d.splane, o = (size_t)d.soff + (size_t)frame * n;
    if (sw) *sw = d.sw;
    if (sh) *sh = d.sh;
    PLVI_CHECK(hipDeviceSynchronize());
    if (deg) PLVI_CHECK(hipMemcpy(deg, P.pix.as<float>() + o, n * sizeof(float), hipMemcpyDeviceToHost));
    if (modgrad) PLVI_CHECK(hipMemcpy(modgrad, P.modg.as<double>() + o, n * sizeof(double), hipMemcpyDeviceToHost));
    if (cs) PLVI_CHECK(hipMemcpy(cs, P.seedcs.as<float2>() + o, n * sizeof(float2), hipMemcpyDeviceToHost));
    return PLVI_OK;
}

// Diagnostic: the LBD Sobel plane (interleaved int16 dx, dy) of the last
// batch for one (frame, octave), copied to host memory.
extern "C" int plvi_lines_debug_sobel(plvi_line_extractor* h, int frame, int octave, short* dxdy, int* w, int* hgt) {
    if (!h || octave < 0 || octave >= h->p().nOct || frame < 0 || frame >= h->p().Bcap) return PLVI_E_BADARG;
    LinePipeline& P = h->p();
    PLVI_CHECK(hipSetDevice(P.device));
    const plvi::LineOctDev& d = P.oct[octave];
    if (w) *w = d.lw;
    if (hgt) *hgt = d.lh;
    PLVI_CHECK(hipDeviceSynchronize());
    if (dxdy)
        PLVI_CHECK(hipMemcpy(dxdy, P.lbdG.as<short2>() + d.loff + (size_t)frame * d.lplane,
                             (size_t)d.lplane * sizeof(short2), hipMemcpyDeviceToHost));
    return PLVI_OK;
}

extern "C" int plvi_lines_kernel_timing(plvi_line_extractor* h, int enable) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().ktiming(enable);
}

extern "C" int plvi_lines_kernel_timing_read(plvi_line_extractor* h, float* total_ms, int* launches) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().ktiming_read(total_ms, launches);
}

extern "C" int plvi_lines_kernel_timing_read_kind(plvi_line_extractor* h, int kind, float* total_ms, int* launches) {
    if (!h) return PLVI_E_BADARG;
    PLVI_CHECK(hipSetDevice(h->p().device));
    return h->p().ktiming_read_kind(kind, total_ms, launches);
}
