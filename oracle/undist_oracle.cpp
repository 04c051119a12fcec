// oracle/undist_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the keypoint / keyline undistortion that runs right after
// extraction ("parity unpinned": OpenCV 4.2's cv::undistortPoints is not in
// this image; restated from its published source, cvUndistortPointsInternal,
// default criteria TermCriteria(COUNT, 5, 0.01), no tilt, R = I, P = K):
//   Frame::UndistortKeyPoints   src/Frame.cc:1124-1157
//   Frame::UndistortKeyLines    src/Frame.cc:1159-1197 (endpoints only)
//   Frame::ComputeImageBounds   src/Frame.cc:1199-1226
#include <algorithm>
#include <cstdint>

namespace {

struct Cam {
    double fx, fy, cx, cy;
    double k[14];
};

Cam make_cam(const float* K4, const float* dist, int nd) {
    Cam c{};
    c.fx = K4[0]; c.fy = K4[1]; c.cx = K4[2]; c.cy = K4[3];
    for (int i = 0; i < 14; ++i) c.k[i] = 0.0;
    for (int i = 0; i < nd && i < 14; ++i) c.k[i] = dist[i];
    return c;
}

void undistort(const Cam& c, float sx, float sy, float& ox, float& oy) {
    const double ifx = 1. / c.fx, ify = 1. / c.fy;
    const double* k = c.k;
    double x = sx, y = sy;
    x = (x - c.cx) * ifx;
    y = (y - c.cy) * ify;
    // identity tilt: vecUntilt = (x, y, 1), invProj = 1
    const double ux = 1.0 * x + 0.0 * y + 0.0 * 1.0, uy = 0.0 * x + 1.0 * y + 0.0 * 1.0;
    const double uz = 0.0 * x + 0.0 * y + 1.0 * 1.0;
    const double invProj = uz ? 1. / uz : 1;
    double x0 = x = invProj * ux;
    double y0 = y = invProj * uy;
    for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I = K
    const double xx = c.fx * x + 0.0 * y + c.cx;
    const double yy = 0.0 * x + c.fy * y + c.cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    ox = (float)(xx * ww);
    oy = (float)(yy * ww);
}

}  // namespace

// K4 = fx, fy, cx, cy; dist = mDistCoef (k1, k2, p1, p2[, k3]).
extern "C" void oracle_undistort_points(const float* K4, const float* dist, int nd, const float* xy, int n,
                                        float* out) {
    const Cam c = make_cam(K4, dist, nd);
    for (int i = 0; i < n; ++i) {
        if (dist[0] == 0.0f) {  // mDistCoef.at<float>(0)==0.0: mvKeysUn = mvKeys
            out[2 * i] = xy[2 * i];
            out[2 * i + 1] = xy[2 * i + 1];
        } else {
            undistort(c, xy[2 * i], xy[2 * i + 1], out[2 * i], out[2 * i + 1]);
        }
    }
}

// bounds = mnMinX, mnMaxX, mnMinY, mnMaxY
extern "C" void oracle_image_bounds(const float* K4, const float* dist, int nd, int cols, int rows, float* bounds) {
    if (dist[0] == 0.0f) {
        bounds[0] = 0.0f; bounds[1] = (float)cols; bounds[2] = 0.0f; bounds[3] = (float)rows;
        return;
    }
    const Cam c = make_cam(K4, dist, nd);
    float p[4][2];
    const float in[4][2] = {{0.0f, 0.0f}, {(float)cols, 0.0f}, {0.0f, (float)rows}, {(float)cols, (float)rows}};
    for (int i = 0; i < 4; ++i) undistort(c, in[i][0], in[i][1], p[i][0], p[i][1]);
    bounds[0] = std::min(p[0][0], p[2][0]);
    bounds[1] = std::max(p[1][0], p[3][0]);
    bounds[2] = std::min(p[0][1], p[1][1]);
    bounds[3] = std::max(p[2][1], p[3][1]);
}
