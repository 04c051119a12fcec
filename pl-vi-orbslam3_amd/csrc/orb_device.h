// orb_device.h — device-side tables shared by the ORB kernels and the host
// pipeline (orb.hip).  All geometry is precomputed on the host exactly as
// ORBextractor does it (src/ORBextractor.cc:408-468, 771-785, 1156-1157).
#pragma once
#include <cstdint>

namespace plvi {

constexpr int kOrbMaxLevels = 16;
constexpr int kOrbMaxRoots = 8;
constexpr int kOrbCellMax = 64;  // max detection-window side (wCell+2 < 64)
#ifndef PLVI_BF_ALIGN
#define PLVI_BF_ALIGN 32
#endif
constexpr int kBfAlign = PLVI_BF_ALIGN;  // byte alignment of the blur / score rows and strips

struct OrbLevelDev {
    int w, h;
    long long off;    // byte offset of this level's frame-0 plane in pyr
    long long plane;  // bytes per frame plane (w*h) of the pyramid
    // blur / FAST score planes: rows padded to bpitch (a multiple
    // of kBfAlign) so that every blur+FAST strip writes whole aligned segments
    int bpitch;
    long long boff, bplane;
    int minB;         // EDGE_THRESHOLD-3 = 16
    int rw, rh;       // relative region (maxBorder-minBorder)
    int nCols, nRows, wCell, hCell;
    int listOff;         // offset (entries) of this level's candidate list in a frame's block
    int listCap;         // its capacity: no two NMS survivors of a cell window are 8-adjacent
    int quota;           // mnFeaturesPerLevel
    int nodeCap;         // octree output capacity (>= quota+3)
    int kpOff;           // offset of this level in the per-frame level-keypoint table
    float scale;         // mvScaleFactor
    float size;          // (float)(int)(PATCH_SIZE*scale)
    int nIni;
    int rootGx[kOrbMaxRoots + 1];  // geometric root x: (int)(hX*i)
    int rootB[kOrbMaxRoots + 1];   // membership: root i holds x in [rootB[i], rootB[i+1])
    double rsx, rsy;               // cv::resize scale_x / scale_y from level l-1 (1 / ((double)dw / sw))
    int xtab;                      // offset of this level's packed column table (orb_pyramid_kernel)
};

// One strip of a level for the blur + FAST kernel: output columns [x0, x1),
// rows [y0, y1).  Lane L holds the four columns (x0 & ~3) - 4 + 4L .. +3
// (x1 - (x0 & ~3) <= kBfCols).  Strips are cut at kBfAlign-aligned columns.
struct OrbStripDev {
    int level, x0, x1, y0, y1;
};

struct OrbCellDev {
    int level;
    int x0, y0, x1, y1;  // FAST detection window [x0,x1)x[y0,y1) in level coords
};

}  // namespace plvi
