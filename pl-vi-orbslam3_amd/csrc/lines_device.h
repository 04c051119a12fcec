// lines_device.h — device tables of the line front end (Lineextractor,
// LSDDetectorC, LineSegmentDetectorImpl, BinaryDescriptor).  Geometry is
// derived on the host exactly as the reference does.
#pragma once
#include <cstdint>

namespace plvi {

constexpr int kLineMaxOct = 2;      // Lineextractor nlevels (config: 2)
constexpr int kLsdRawCap = 8192;    // LSD segments per (frame, octave)
constexpr int kPrepBands = 8;       // row bands of the LSD prep for batches <= kPrepBandMax frames
constexpr int kPrepBandMax = 256;


struct LineOctDev {
    int w, h;             // octave image (LSD input) dims
    long long off;        // byte offset of frame-0 plane in the octave image buffer
    long long plane;      // bytes per frame plane
    int sw, sh;           // LSD scaled image dims (x SCALE)
    long long soff;       // element offset of frame-0 plane in the scaled-plane buffers
    long long splane;     // elements per frame plane (sw*sh)
    int min_reg_size;     // int(-LOG_NT/log10(p)) (lsd.cpp:466-467)
    float octaveScale;    // pow(scale, octave) (LSDDetector_custom.cpp:322)
    int maxWH;            // max(w,h) for KeyLine.response
    // resize x0.8 tables (offsets in the table buffer)
    long long tabXofs, tabXa, tabYrow, tabYb;
    int xmax;
    // lsd_prep2_kernel column strips (int4 {X0, X1, gx0, nc}, offset in the table buffer)
    long long tabStrips;
    int nstrips;
    // lsd_prep_kernel row bands (int4 {dyA, dyB, ybase0, 0}): one band, or
    // kPrepBands for small batches (offsets in the table buffer)
    long long tabBands1, tabBandsK;
    // Sobel/LBD pyramid (computeGaussianPyramid): dims and offsets
    int lw, lh;
    long long loff, lplane;
};

struct LsdLine {
    float x1, y1, x2, y2;
};

// A region kept by region growing: its points (x | y << 16, queue order) at
// [start, start + n) of the task's point list, and its final reg_angle.
struct LsdRegion {
    int start, n;
    double angle;
};

// Per-pixel static data for region growing: fastAtan2 angle in degrees
// (float; NOTDEF encoded as -1024), and cosf/sinf of float(angle rad)
// exactly as region_grow computes them (lsd.cpp:678-679).
struct LsdPix {
    float deg;
    float c, s;
    float pad;
};

}  // namespace plvi
