// oracle/lines_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the line front end ("parity unpinned": no golden
// vectors exist in the reference and it cannot be built here):
//   Lineextractor::operator()              src/LineExtractor.cc:45-117 (LSD branch)
//   LSDDetectorC::ComputePyramid/detectImpl Thirdparty/line_descriptor/src/LSDDetector_custom.cpp:76-109, 263-362
//   LineSegmentDetectorImpl::flsd & helpers src/LSD/lsd.cpp:412-782, 1136-1152 (refine = 0)
//   BinaryDescriptor::computeImpl/computeLBD Thirdparty/line_descriptor/src/binary_descriptor_custom.cpp:219-261,
//                                            351-414, 540-688, 1027-1373
// OpenCV primitives from cvprim.cpp; libm from the host glibc (as the
// reference).  Compiled with -ffp-contract=off.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "cvprim.h"
#include "ref_fma.h"

namespace oracle {

struct KeyLine {  // line_descriptor::KeyLine (descriptor_custom.hpp:107-146)
    float angle;
    int class_id;
    int octave;
    float pt_x, pt_y;
    float response;
    float size;
    float startPointX, startPointY, endPointX, endPointY;
    float sPointInOctaveX, sPointInOctaveY, ePointInOctaveX, ePointInOctaveY;
    float lineLength;
    int numOfPixels;
};

struct LineParams {
    int nfeatures = 200;    // lsd_nfeatures
    int refine = 0;         // lsd_refine (only 0 supported: the config)
    float lsd_scale = 0.8f; // LSDOptions::scale is a float (descriptor_custom.hpp:919)
    int nlevels = 2;
    float scale = 2.0f;
};

// ----------------------------------------------------------------- f64 image ops
struct ImageF64 {
    int w = 0, h = 0;
    std::vector<double> px;
    double& at(int x, int y) { return px[(size_t)y * w + x]; }
    double at(int x, int y) const { return px[(size_t)y * w + x]; }
};

// GaussianBlur on CV_64F: RowFilter<double,double> (sequential sum) then
// SymmColumnFilter (center + k*(up+down)), BORDER_REFLECT_101.
static void gaussian_blur_f64(const ImageF64& src, ImageF64& dst, int n, double sigma) {
    std::vector<double> k(n);
    gaussian_kernel_f64(n, sigma, k.data());
    const int r = n / 2, w = src.w, h = src.h;
    ImageF64 H;
    H.w = w; H.h = h; H.px.assign((size_t)w * h, 0.0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double s = k[0] * src.at(reflect101(x - r, w), y);
            for (int i = 1; i < n; ++i) s += k[i] * src.at(reflect101(x - r + i, w), y);
            H.at(x, y) = s;
        }
    dst.w = w; dst.h = h; dst.px.assign((size_t)w * h, 0.0);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            double s = k[r] * H.at(x, y) + 0.0;
            for (int i = 1; i <= r; ++i) s += k[r + i] * (H.at(x, reflect101(y + i, h)) + H.at(x, reflect101(y - i, h)));
            dst.at(x, y) = s;
        }
}

// cv::resize(src, dst, Size(), fx, fx) INTER_LINEAR on CV_64F: float
// coefficients, double accumulation (HResizeLinear/VResizeLinear, no FMA).
static void resize_f64(const ImageF64& src, ImageF64& dst, double inv_scale) {
    const int sw = src.w, sh = src.h;
    const int dw = cv_round(sw * inv_scale), dh = cv_round(sh * inv_scale);
    const double scale_x = 1. / inv_scale, scale_y = 1. / inv_scale;
    std::vector<int> xofs(dw);
    std::vector<float> al(2 * dw);
    int xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        xofs[dx] = sx;
        al[2 * dx] = 1.f - fx;
        al[2 * dx + 1] = fx;
    }
    std::vector<double> H0(dw), H1(dw);
    auto hres = [&](int row, double* D) {
        const double* S = src.px.data() + (size_t)row * sw;
        int dx = 0;
        for (; dx < xmax; ++dx) D[dx] = S[xofs[dx]] * (double)al[2 * dx] + S[xofs[dx] + 1] * (double)al[2 * dx + 1];
        for (; dx < dw; ++dx) D[dx] = S[xofs[dx]] * 1.0;
    };
    dst.w = dw; dst.h = dh; dst.px.assign((size_t)dw * dh, 0.0);
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = cv_floor(fy);
        fy -= sy;
        float b0 = 1.f - fy, b1 = fy;
        hres(std::min(std::max(sy, 0), sh - 1), H0.data());
        hres(std::min(std::max(sy + 1, 0), sh - 1), H1.data());
        for (int x = 0; x < dw; ++x) dst.at(x, dy) = H0[x] * (double)b0 + H1[x] * (double)b1;
    }
}

// ----------------------------------------------------------------- LSD (lsd.cpp)
static const double NOTDEF = -1024.0;
static const double DEG_TO_RADS = M_PI / 180;
static const double M_3_2_PI_ = (3 * M_PI) / 2;
static const double M_2__PI_ = (2 * M_PI);

struct RegionPoint {
    int x, y;
    double angle, modgrad;
};

struct LSD {
    double SCALE, SIGMA_SCALE = 0.6, QUANT = 2.0, ANG_TH = 22.5;
    int img_width = 0, img_height = 0;
    ImageF64 scaled, angles, modgrad;
    std::vector<unsigned char> used;
    std::vector<RegionPoint> reg;

    bool isAligned(int address, double theta, double prec) const {  // :1136-1152
        if (address < 0) return false;
        const double a = angles.px[address];
        if (a == NOTDEF) return false;
        double n_theta = theta - a;
        if (n_theta < 0) n_theta = -n_theta;
        if (n_theta > M_3_2_PI_) {
            n_theta -= M_2__PI_;
            if (n_theta < 0) n_theta = -n_theta;
        }
        return n_theta <= prec;
    }

    void ll_angle(double threshold) {  // :536-584 (the bucket list is never consumed: see flsd)
        img_width = scaled.w;
        img_height = scaled.h;
        angles.w = modgrad.w = img_width;
        angles.h = modgrad.h = img_height;
        angles.px.assign((size_t)img_width * img_height, NOTDEF);
        modgrad.px.assign((size_t)img_width * img_height, 0.0);
        for (int y = 0; y < img_height - 1; ++y)
            for (int x = 0; x < img_width - 1; ++x) {
                const size_t addr = (size_t)y * img_width + x;
                double DA = scaled.px[addr + img_width + 1] - scaled.px[addr];
                double BC = scaled.px[addr + 1] - scaled.px[addr + img_width];
                double gx = DA + BC, gy = DA - BC;
                double norm = std::sqrt(ref_fma(gx, gx, gy * gy) / 4);  // fused in lsd.cpp.o
                modgrad.px[addr] = norm;
                if (norm <= threshold) angles.px[addr] = NOTDEF;
                else angles.px[addr] = fast_atan2((float)gx, (float)-gy) * DEG_TO_RADS;
            }
    }

    void region_grow(int sx, int sy, int& reg_size, double& reg_angle, double prec) {  // :635-686
        reg_size = 1;
        reg[0].x = sx; reg[0].y = sy;
        int addr = sx + sy * img_width;
        reg_angle = angles.px[addr];
        reg[0].angle = reg_angle;
        reg[0].modgrad = modgrad.px[addr];
        double seed_s, seed_c;  // lsd.cpp:648-649, one sincos call as in the reference object
        ::sincos(reg_angle, &seed_s, &seed_c);
        float sumdx = (float)seed_c;
        float sumdy = (float)seed_s;
        used[addr] = 1;
        for (int i = 0; i < reg_size; ++i) {
            const RegionPoint rp = reg[i];
            int xx_min = std::max(rp.x - 1, 0), xx_max = std::min(rp.x + 1, img_width - 1);
            int yy_min = std::max(rp.y - 1, 0), yy_max = std::min(rp.y + 1, img_height - 1);
            for (int yy = yy_min; yy <= yy_max; ++yy) {
                int c_addr = xx_min + yy * img_width;
                for (int xx = xx_min; xx <= xx_max; ++xx, ++c_addr) {
                    if (used[c_addr] != 1 && isAligned(c_addr, reg_angle, prec)) {
                        used[c_addr] = 1;
                        RegionPoint& p = reg[reg_size];
                        p.x = xx; p.y = yy;
                        p.modgrad = modgrad.px[c_addr];
                        const double angle = angles.px[c_addr];
                        p.angle = angle;
                        ++reg_size;
                        sumdx += cosf((float)angle);
                        sumdy += sinf((float)angle);
                        reg_angle = fast_atan2(sumdy, sumdx) * DEG_TO_RADS;
                    }
                }
            }
        }
    }

    static double angle_diff(double a, double b) {
        double diff = a - b;
        while (diff <= -M_PI) diff += M_2__PI_;
        while (diff > M_PI) diff -= M_2__PI_;
        return std::fabs(diff);
    }

    double get_theta(int reg_size, double x, double y, double reg_angle, double prec) const {  // :746-782
        double Ixx = 0.0, Iyy = 0.0, Ixy = 0.0;
        for (int i = 0; i < reg_size; ++i) {
            const double regx = reg[i].x, regy = reg[i].y, weight = reg[i].modgrad;
            double dx = regx - x, dy = regy - y;
            // lsd.cpp.o get_theta: three fused accumulations + the root's
            Ixx = ref_fma(dy * dy, weight, Ixx);
            Iyy = ref_fma(dx * dx, weight, Iyy);
            Ixy = ref_fma(-(dx * dy), weight, Ixy);
        }
        double lambda = 0.5 * (Ixx + Iyy - std::sqrt(ref_fma(Ixx - Iyy, Ixx - Iyy, 4.0 * Ixy * Ixy)));
        double theta = (std::fabs(Ixx) > std::fabs(Iyy)) ? (double)fast_atan2((float)(lambda - Ixx), (float)Ixy)
                                                         : (double)fast_atan2((float)Ixy, (float)(lambda - Iyy));
        theta *= DEG_TO_RADS;
        if (angle_diff(theta, reg_angle) > prec) theta += M_PI;
        return theta;
    }

    void region2rect(int reg_size, double reg_angle, double prec, double* r) const {  // :688-744
        double x = 0, y = 0, sum = 0;
        for (int i = 0; i < reg_size; ++i) {
            const double weight = reg[i].modgrad;
            x = ref_fma((double)reg[i].x, weight, x);  // fused in lsd.cpp.o region2rect
            y = ref_fma((double)reg[i].y, weight, y);
            sum += weight;
        }
        x /= sum;
        y /= sum;
        double theta = get_theta(reg_size, x, y, reg_angle, prec);
        // lsd.cpp:710-711: GCC merges the pair into one glibc sincos call (the
        // reference object's `call sincos`; x86-64 sincos has no FMA ifunc)
        double dx, dy;
        ::sincos(theta, &dy, &dx);
        double l_min = 0, l_max = 0, w_min = 0, w_max = 0;
        for (int i = 0; i < reg_size; ++i) {
            double regdx = (double)reg[i].x - x, regdy = (double)reg[i].y - y;
            double l = ref_fma(regdx, dx, regdy * dy);
            double w = ref_fma(-regdx, dy, regdy * dx);
            if (l > l_max) l_max = l;
            else if (l < l_min) l_min = l;
            if (w > w_max) w_max = w;
            else if (w < w_min) w_min = w;
        }
        r[0] = ref_fma(l_min, dx, x);  // one vfmadd132pd over the four
        r[1] = ref_fma(l_min, dy, y);
        r[2] = ref_fma(l_max, dx, x);
        r[3] = ref_fma(l_max, dy, y);
    }

    // LineSegmentDetectorImpl::detect + flsd (:412-534), refine = LSD_REFINE_NONE.
    std::vector<float> detect(const ImageU8& img) {
        ImageF64 image;
        image.w = img.w; image.h = img.h;
        image.px.resize((size_t)img.w * img.h);
        for (size_t i = 0; i < image.px.size(); ++i) image.px[i] = img.px[i];
        const double prec = M_PI * ANG_TH / 180;
        const double p = ANG_TH / 180;
        const double rho = QUANT / std::sin(prec);
        if (SCALE != 1) {
            const double sigma = (SCALE < 1) ? (SIGMA_SCALE / SCALE) : SIGMA_SCALE;
            const double sprec = 3;
            const unsigned h = (unsigned)std::ceil(sigma * std::sqrt(2 * sprec * std::log(10.0)));
            ImageF64 g;
            gaussian_blur_f64(image, g, 1 + 2 * h, sigma);
            resize_f64(g, scaled, SCALE);
        } else {
            scaled = image;
        }
        ll_angle(rho);
        // lsd.cpp.o: fma(5*(lw + lh), 0.5, log10(11.0) folded by GCC); the
        // literal below is that .rodata constant (glibc's log10(11.0) is one
        // ulp lower)
        const double LOG_NT = ref_fma(5 * (std::log10((double)img_width) + std::log10((double)img_height)), 0.5,
                                      0x1.0a98b6050c56fp+0);
        const int min_reg_size = (int)(-LOG_NT / std::log10(p));
        used.assign((size_t)img_width * img_height, 0);
        reg.assign((size_t)img_width * img_height, RegionPoint{0, 0, 0, 0});
        std::vector<float> lines;
        // flsd iterates the coorlist *vector* (raster order of insertion,
        // lsd.cpp:476-479); the pseudo-ordered linked list is never walked.
        for (int y = 0; y < img_height - 1; ++y)
            for (int x = 0; x < img_width - 1; ++x) {
                const int adx = x + y * img_width;
                if (used[adx] == 0 && angles.px[adx] != NOTDEF) {
                    int reg_size;
                    double reg_angle;
                    region_grow(x, y, reg_size, reg_angle, prec);
                    if (reg_size < min_reg_size) continue;
                    double r[4];
                    region2rect(reg_size, reg_angle, prec, r);
                    r[0] += 0.5; r[1] += 0.5; r[2] += 0.5; r[3] += 0.5;
                    if (SCALE != 1) { r[0] /= SCALE; r[1] /= SCALE; r[2] /= SCALE; r[3] /= SCALE; }
                    lines.push_back((float)r[0]); lines.push_back((float)r[1]);
                    lines.push_back((float)r[2]); lines.push_back((float)r[3]);
                }
            }
        return lines;
    }
};

// ----------------------------------------------------------------- LineIterator count
static bool clip_line(long long W, long long H, long long& x1, long long& y1, long long& x2, long long& y2) {
    int c1, c2;
    long long right = W - 1, bottom = H - 1;
    if (W <= 0 || H <= 0) return false;
    c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        long long a;
        if (c1 & 12) {
            a = c1 < 8 ? 0 : bottom;
            x1 += (long long)((double)(a - y1) * (x2 - x1) / (y2 - y1));
            y1 = a;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            a = c2 < 8 ? 0 : bottom;
            x2 += (long long)((double)(a - y2) * (x2 - x1) / (y2 - y1));
            y2 = a;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                a = c1 == 1 ? 0 : right;
                y1 += (long long)((double)(a - x1) * (y2 - y1) / (x2 - x1));
                x1 = a;
                c1 = 0;
            }
            if (c2) {
                a = c2 == 1 ? 0 : right;
                y2 += (long long)((double)(a - x2) * (y2 - y1) / (x2 - x1));
                x2 = a;
                c2 = 0;
            }
        }
    }
    return (c1 | c2) == 0;
}

// cv::LineIterator(img, Point(pt1), Point(pt2), 8).count.
static int line_iterator_count(int W, int H, float fx1, float fy1, float fx2, float fy2) {
    int x1 = cv_round(fx1), y1 = cv_round(fy1), x2 = cv_round(fx2), y2 = cv_round(fy2);
    if ((unsigned)x1 >= (unsigned)W || (unsigned)x2 >= (unsigned)W || (unsigned)y1 >= (unsigned)H ||
        (unsigned)y2 >= (unsigned)H) {
        long long a = x1, b = y1, c = x2, d = y2;
        if (!clip_line(W, H, a, b, c, d)) return 0;
        x1 = (int)a; y1 = (int)b; x2 = (int)c; y2 = (int)d;
    }
    int dx = std::abs(x2 - x1), dy = std::abs(y2 - y1);
    return std::max(dx, dy) + 1;
}

// ----------------------------------------------------------------- LBD
static const int kCombinations[32][2] = {{0, 1}, {0, 2}, {0, 3}, {0, 4}, {0, 5}, {0, 6}, {1, 2}, {1, 3},
                                         {1, 4}, {1, 5}, {1, 6}, {2, 3}, {2, 4}, {2, 5}, {2, 6}, {2, 7},
                                         {2, 8}, {3, 4}, {3, 5}, {3, 6}, {3, 7}, {3, 8}, {4, 5}, {4, 6},
                                         {4, 7}, {4, 8}, {5, 6}, {5, 7}, {5, 8}, {6, 7}, {6, 8}, {7, 8}};

struct LBD {
    static const int NB = 9, WB = 7;
    std::vector<double> gaussCoefL, gaussCoefG;
    std::vector<ImageU8> octaves;
    std::vector<std::vector<int16_t>> dxs, dys;

    LBD() {  // BinaryDescriptor ctor (:219-261)
        gaussCoefL.resize(WB * 3);
        double u = (WB * 3 - 1) / 2;
        double sigma = (WB * 2 + 1) / 2;
        double invsigma2 = -1 / (2 * sigma * sigma);
        for (int i = 0; i < WB * 3; ++i) {
            double dis = i - u;
            gaussCoefL[i] = std::exp(dis * dis * invsigma2);
        }
        gaussCoefG.resize(NB * WB);
        u = (NB * WB - 1) / 2;
        sigma = u;
        invsigma2 = -1 / (2 * sigma * sigma);
        for (int i = 0; i < NB * WB; ++i) {
            double dis = i - u;
            gaussCoefG[i] = std::exp(dis * dis * invsigma2);
        }
    }

    void sobel_pyramid(const ImageU8& image, int numOctaves) {  // computeGaussianPyramid + computeSobel
        octaves.clear();
        ImageU8 cur;
        gaussian_blur_u8(image, cur, 5, 1.0);
        octaves.push_back(cur);
        for (int o = 1; o < numOctaves; ++o) {
            ImageU8 nxt;
            pyr_down_u8(cur, nxt, cur.w / 2, cur.h / 2);
            cur = nxt;
            octaves.push_back(cur);
        }
        dxs.assign(octaves.size(), {});
        dys.assign(octaves.size(), {});
        for (size_t o = 0; o < octaves.size(); ++o) sobel_s16(octaves[o], dxs[o], dys[o]);
    }

    // computeLBD for one line (:1073-1342); returns the 72-float descriptor.
    void describe(const KeyLine& kl, float* desVec) const {
        const int o = kl.octave;
        const short* pdx = dxs[o].data();
        const short* pdy = dys[o].data();
        const short realWidth = (short)octaves[o].w;
        const short imageWidth = realWidth - 1;
        const short imageHeight = (short)(octaves[o].h - 1);
        float pL[NB] = {0}, nL[NB] = {0}, pL2[NB] = {0}, nL2[NB] = {0};
        float pO[NB] = {0}, nO[NB] = {0}, pO2[NB] = {0}, nO2[NB] = {0};
        const short heightOfLSP = (short)(WB * NB);
        const short halfHeight = (heightOfLSP - 1) / 2;
        const short lengthOfLSP = (short)kl.numOfPixels;
        const short halfWidth = (lengthOfLSP - 1) / 2;
        const float mX = (float)(0.5 * (kl.sPointInOctaveX + kl.ePointInOctaveX));
        const float mY = (float)(0.5 * (kl.sPointInOctaveY + kl.ePointInOctaveY));
        float dL[2], dO[2];
        dL[0] = cosf(kl.angle);
        dL[1] = sinf(kl.angle);
        dO[0] = -dL[1];
        dO[1] = dL[0];
        float sCorX0 = -dL[0] * halfWidth + dL[1] * halfHeight + mX;
        float sCorY0 = -dL[1] * halfWidth - dL[0] * halfHeight + mY;
        for (short hID = 0; hID < heightOfLSP; hID++) {
            float sCorX = sCorX0, sCorY = sCorY0;
            float pLr = 0, nLr = 0, pOr = 0, nOr = 0;
            for (short wID = 0; wID < lengthOfLSP; wID++) {
                short tempCor = (short)roundf(sCorX);
                short xCor = (tempCor < 0) ? 0 : (tempCor > imageWidth) ? imageWidth : tempCor;
                tempCor = (short)roundf(sCorY);
                short yCor = (tempCor < 0) ? 0 : (tempCor > imageHeight) ? imageHeight : tempCor;
                short dx = pdx[yCor * realWidth + xCor];
                short dy = pdy[yCor * realWidth + xCor];
                float gDL = dx * dL[0] + dy * dL[1];
                float gDO = dx * dO[0] + dy * dO[1];
                if (gDL > 0) pLr += gDL;
                else nLr -= gDL;
                if (gDO > 0) pOr += gDO;
                else nOr -= gDO;
                sCorX += dL[0];
                sCorY += dL[1];
            }
            sCorX0 -= dL[1];
            sCorY0 += dL[0];
            float c = (float)gaussCoefG[hID];
            pLr = c * pLr; nLr = c * nLr;
            float pL2r = pLr * pLr, nL2r = nLr * nLr;
            pOr = c * pOr; nOr = c * nOr;
            float pO2r = pOr * pOr, nO2r = nOr * nOr;
            short band = (short)(hID / WB);
            c = (float)gaussCoefL[hID % WB + WB];
            pL[band] += c * pLr; nL[band] += c * nLr;
            pL2[band] += c * c * pL2r; nL2[band] += c * c * nL2r;
            pO[band] += c * pOr; nO[band] += c * nOr;
            pO2[band] += c * c * pO2r; nO2[band] += c * c * nO2r;
            band--;
            if (band >= 0) {
                c = (float)gaussCoefL[hID % WB + 2 * WB];
                pL[band] += c * pLr; nL[band] += c * nLr;
                pL2[band] += c * c * pL2r; nL2[band] += c * c * nL2r;
                pO[band] += c * pOr; nO[band] += c * nOr;
                pO2[band] += c * c * pO2r; nO2[band] += c * c * nO2r;
            }
            band = band + 2;
            if (band < NB) {
                c = (float)gaussCoefL[hID % WB];
                pL[band] += c * pLr; nL[band] += c * nLr;
                pL2[band] += c * c * pL2r; nL2[band] += c * c * nL2r;
                pO[band] += c * pOr; nO[band] += c * nOr;
                pO2[band] += c * c * pO2r; nO2[band] += c * c * nO2r;
            }
        }
        const float invN2 = (float)(1.0 / (WB * 2.0)), invN3 = (float)(1.0 / (WB * 3.0));
        for (int b = 0; b < NB; ++b) {
            const float invN = (b == 0 || b == NB - 1) ? invN2 : invN3;
            const int d = b * 8;
            float t = pL[b] * invN;
            desVec[d] = t;
            desVec[d + 4] = std::sqrt(pL2[b] * invN - t * t);
            t = nL[b] * invN;
            desVec[d + 1] = t;
            desVec[d + 5] = std::sqrt(nL2[b] * invN - t * t);
            t = pO[b] * invN;
            desVec[d + 2] = t;
            desVec[d + 6] = std::sqrt(pO2[b] * invN - t * t);
            t = nO[b] * invN;
            desVec[d + 3] = t;
            desVec[d + 7] = std::sqrt(nO2[b] * invN - t * t);
        }
        float tempM = 0, tempS = 0;
        for (int b = 0; b < NB; ++b) {
            const float* v = desVec + 8 * b;
            tempM += v[0] * v[0]; tempM += v[1] * v[1]; tempM += v[2] * v[2]; tempM += v[3] * v[3];
            tempS += v[4] * v[4]; tempS += v[5] * v[5]; tempS += v[6] * v[6]; tempS += v[7] * v[7];
        }
        tempM = 1 / std::sqrt(tempM);
        tempS = 1 / std::sqrt(tempS);
        for (int b = 0; b < NB; ++b) {
            float* v = desVec + 8 * b;
            v[0] = v[0] * tempM; v[1] = v[1] * tempM; v[2] = v[2] * tempM; v[3] = v[3] * tempM;
            v[4] = v[4] * tempS; v[5] = v[5] * tempS; v[6] = v[6] * tempS; v[7] = v[7] * tempS;
        }
        for (int i = 0; i < NB * 8; ++i)
            if (desVec[i] > 0.4) desVec[i] = (float)0.4;
        float temp = 0;
        for (int i = 0; i < NB * 8; ++i) temp += desVec[i] * desVec[i];
        temp = 1 / std::sqrt(temp);
        for (int i = 0; i < NB * 8; ++i) desVec[i] = desVec[i] * temp;
    }

    static void binarize(const float* desVec, uint8_t* row) {  // binaryConversion (:402-414), :663-667
        for (int comb = 0; comb < 32; ++comb) {
            const float* f1 = desVec + 8 * kCombinations[comb][0];
            const float* f2 = desVec + 8 * kCombinations[comb][1];
            uint8_t r = 0;
            for (int i = 0; i < 8; ++i)
                if (f1[i] > f2[i]) r += (uint8_t)(1 << i);
            row[comb] = r;
        }
    }
};

// ----------------------------------------------------------------- Lineextractor
struct LinesResult {
    std::vector<KeyLine> keylines;
    std::vector<uint8_t> desc;
    std::vector<double> lineFns;
    std::vector<ImageU8> pyramid;
    std::vector<float> rawLines[4];  // per octave, LSD Vec4f output
};

static void line_extract(const ImageU8& img, const LineParams& P, LinesResult& R) {
    // LSDDetectorC::ComputePyramid(image, scale, nlevels) (LSDDetector_custom.cpp:76-109)
    std::vector<float> sf(P.nlevels), isf(P.nlevels);
    R.pyramid.assign(P.nlevels, ImageU8());
    sf[0] = 1.0f;
    for (int l = 0; l < P.nlevels; ++l) {
        if (l > 0) sf[l] = sf[l - 1] * P.scale;
        isf[l] = 1.0f / sf[l];
        int w = cv_round((float)img.w * isf[l]), h = cv_round((float)img.h * isf[l]);
        if (l == 0) R.pyramid[0] = img;
        else resize_linear_u8(R.pyramid[l - 1], R.pyramid[l], w, h);
    }
    // detectImpl(opts) (:263-362)
    const double min_length = 0.025 * std::min(img.w, img.h);  // LineExtractor.cc:72
    std::vector<KeyLine>& kls = R.keylines;
    kls.clear();
    int class_counter = -1;
    for (int o = 0; o < P.nlevels; ++o) {
        LSD lsd;
        lsd.SCALE = (double)P.lsd_scale;
        std::vector<float> lines = lsd.detect(R.pyramid[o]);
        if (o < 4) R.rawLines[o] = lines;
        const float octaveScale = (float)std::pow((float)P.scale, o);
        const int W = R.pyramid[o].w, H = R.pyramid[o].h;
        for (size_t k = 0; k + 3 < lines.size(); k += 4) {
            float e[4] = {lines[k], lines[k + 1], lines[k + 2], lines[k + 3]};
            if (e[0] < 0) e[0] = 0;
            if (e[0] >= W) e[0] = (float)W - 1.0f;
            if (e[2] < 0) e[2] = 0;
            if (e[2] >= W) e[2] = (float)W - 1.0f;
            if (e[1] < 0) e[1] = 0;
            if (e[1] >= H) e[1] = (float)H - 1.0f;
            if (e[3] < 0) e[3] = 0;
            if (e[3] >= H) e[3] = (float)H - 1.0f;
            double length = (float)std::sqrt(std::pow((double)(e[0] - e[2]), 2.0) + std::pow((double)(e[1] - e[3]), 2.0));
            if (!(length > min_length)) continue;
            KeyLine kl;
            kl.startPointX = e[0] * octaveScale;
            kl.startPointY = e[1] * octaveScale;
            kl.endPointX = e[2] * octaveScale;
            kl.endPointY = e[3] * octaveScale;
            kl.sPointInOctaveX = e[0];
            kl.sPointInOctaveY = e[1];
            kl.ePointInOctaveX = e[2];
            kl.ePointInOctaveY = e[3];
            kl.lineLength = (float)length;
            kl.numOfPixels = line_iterator_count(W, H, e[0], e[1], e[2], e[3]);
            kl.angle = atan2f(kl.endPointY - kl.startPointY, kl.endPointX - kl.startPointX);
            kl.class_id = ++class_counter;
            kl.octave = o;
            kl.size = (kl.endPointX - kl.startPointX) * (kl.endPointY - kl.startPointY);
            kl.response = kl.lineLength / std::max(W, H);
            kl.pt_x = (kl.endPointX + kl.startPointX) / 2;
            kl.pt_y = (kl.endPointY + kl.startPointY) / 2;
            kls.push_back(kl);
        }
    }
    // filter keyline (LineExtractor.cc:75-84): libstdc++ std::sort (unstable) by response desc
    if ((int)kls.size() > P.nfeatures && P.nfeatures != 0) {
        std::sort(kls.begin(), kls.end(), [](const KeyLine& a, const KeyLine& b) { return a.response > b.response; });
        kls.resize(P.nfeatures);
        for (int i = 0; i < P.nfeatures; ++i) kls[i].class_id = i;
    }
    // lbd->compute(img, keylines, descriptors) (binary_descriptor_custom.cpp:540-688)
    R.desc.assign(kls.size() * 32, 0);
    if (!kls.empty()) {
        int octaveIndex = -1;
        for (auto& k : kls) octaveIndex = std::max(octaveIndex, k.octave);
        LBD lbd;
        lbd.sobel_pyramid(img, octaveIndex + 1);
        float dv[72];
        for (size_t i = 0; i < kls.size(); ++i) {
            lbd.describe(kls[i], dv);
            LBD::binarize(dv, &R.desc[i * 32]);
        }
    }
    // line equations (LineExtractor.cc:106-115): (sp x ep) / ||(a,b)||, double
    R.lineFns.clear();
    for (auto& k : kls) {
        double sx = k.startPointX, sy = k.startPointY, ex = k.endPointX, ey = k.endPointY;
        double a = sy * 1.0 - 1.0 * ey, b = 1.0 * ex - sx * 1.0, c = ref_fma(sx, ey, -(sy * ex));
        double n = std::sqrt(ref_fma(a, a, b * b));  // both fused in LineExtractor.cc.o
        R.lineFns.push_back(a / n);
        R.lineFns.push_back(b / n);
        R.lineFns.push_back(c / n);
    }
}

}  // namespace oracle

using namespace oracle;

extern "C" int oracle_line_extract(const uint8_t* img, int w, int h, int stride, int nfeatures, float lsd_scale,
                                   int nlevels, float scale, void* keylines /*KeyLine[cap]*/, uint8_t* desc,
                                   double* lineFns, int cap, int* n) {
    ImageU8 im;
    im.create(w, h);
    for (int y = 0; y < h; ++y) std::memcpy(im.row(y), img + (size_t)y * stride, w);
    LineParams P;
    P.nfeatures = nfeatures; P.lsd_scale = lsd_scale; P.nlevels = nlevels; P.scale = scale;
    LinesResult R;
    line_extract(im, P, R);
    *n = (int)R.keylines.size();
    if (*n > cap) return -3;
    std::memcpy(keylines, R.keylines.data(), sizeof(KeyLine) * R.keylines.size());
    std::memcpy(desc, R.desc.data(), R.desc.size());
    std::memcpy(lineFns, R.lineFns.data(), R.lineFns.size() * sizeof(double));
    return 0;
}

// Raw LSD output (Vec4f list) for one image at the given LSD scale.
extern "C" int oracle_lsd_raw(const uint8_t* img, int w, int h, float lsd_scale, float* lines, int cap, int* n) {
    ImageU8 im;
    im.create(w, h);
    std::memcpy(im.px.data(), img, (size_t)w * h);
    LSD lsd;
    lsd.SCALE = (double)lsd_scale;
    std::vector<float> l = lsd.detect(im);
    *n = (int)l.size() / 4;
    if (*n > cap) return -3;
    std::memcpy(lines, l.data(), l.size() * sizeof(float));
    return 0;
}

// Intermediate LSD planes (scaled f64 image, angle, modgrad) for per-kernel parity.
extern "C" int oracle_lsd_planes(const uint8_t* img, int w, int h, float lsd_scale, double* scaled, double* angles,
                                 double* modgrad, int* sw, int* sh) {
    ImageU8 im;
    im.create(w, h);
    std::memcpy(im.px.data(), img, (size_t)w * h);
    LSD lsd;
    lsd.SCALE = (double)lsd_scale;
    lsd.detect(im);
    *sw = lsd.scaled.w; *sh = lsd.scaled.h;
    const size_t n = lsd.scaled.px.size();
    if (scaled) std::memcpy(scaled, lsd.scaled.px.data(), n * 8);
    if (angles) std::memcpy(angles, lsd.angles.px.data(), n * 8);
    if (modgrad) std::memcpy(modgrad, lsd.modgrad.px.data(), n * 8);
    return 0;
}

// LBD Sobel planes for per-kernel parity.
extern "C" int oracle_lbd_sobel(const uint8_t* img, int w, int h, int octave, int16_t* dx, int16_t* dy, int* ow,
                                int* oh) {
    ImageU8 im;
    im.create(w, h);
    std::memcpy(im.px.data(), img, (size_t)w * h);
    LBD lbd;
    lbd.sobel_pyramid(im, octave + 1);
    *ow = lbd.octaves[octave].w; *oh = lbd.octaves[octave].h;
    std::memcpy(dx, lbd.dxs[octave].data(), lbd.dxs[octave].size() * 2);
    std::memcpy(dy, lbd.dys[octave].data(), lbd.dys[octave].size() * 2);
    return 0;
}

extern "C" int oracle_line_iterator_count(int W, int H, float x1, float y1, float x2, float y2) {
    return line_iterator_count(W, H, x1, y1, x2, y2);
}
