// undistort.hip — keypoint / keyline undistortion right after extraction:
//   Frame::UndistortKeyPoints (src/Frame.cc:1124-1157)
//   Frame::UndistortKeyLines  (src/Frame.cc:1159-1197, endpoints)
//   Frame::ComputeImageBounds (src/Frame.cc:1199-1226)
// = cv::undistortPoints (OpenCV 4.2 cvUndistortPointsInternal) with the
// default TermCriteria(COUNT, 5, 0.01), no tilt, R = I, P = K: five
// fixed-point iterations in double, per point, in the library's exact
// operation order (-ffp-contract=off).  Element-wise: one thread per point.
#include <hip/hip_runtime.h>

#include "plvi_common.h"

namespace plvi {

struct UndistCam {
    double fx, fy, cx, cy, ifx, ify;
    double k[12];
    int active;  // mDistCoef.at<float>(0) != 0
};

static UndistCam undist_cam(const plvi_camera* c) {
    UndistCam u{};
    u.fx = c->fx; u.fy = c->fy; u.cx = c->cx; u.cy = c->cy;
    u.ifx = 1. / u.fx;
    u.ify = 1. / u.fy;
    for (int i = 0; i < 12; ++i) u.k[i] = i < c->ndist && i < 5 ? (double)c->dist[i] : 0.0;
    u.active = c->dist[0] != 0.0f;
    return u;
}

__device__ __forceinline__ float2 undistort_pt(const UndistCam& c, float sx, float sy) {
    if (!c.active) return make_float2(sx, sy);
    const double* k = c.k;
    double x = sx, y = sy;
    x = (x - c.cx) * c.ifx;
    y = (y - c.cy) * c.ify;
    const double ux = 1.0 * x + 0.0 * y + 0.0 * 1.0, uy = 0.0 * x + 1.0 * y + 0.0 * 1.0;
    const double uz = 0.0 * x + 0.0 * y + 1.0 * 1.0;
    const double invProj = uz ? 1. / uz : 1;
    const double x0 = invProj * ux, y0 = invProj * uy;
    x = x0;
    y = y0;
#pragma unroll 1
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist =
            (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    const double xx = c.fx * x + 0.0 * y + c.cx;
    const double yy = 0.0 * x + c.fy * y + c.cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    return make_float2((float)(xx * ww), (float)(yy * ww));
}

__global__ __launch_bounds__(256) void undistort_points_kernel(UndistCam c, const float2* __restrict__ in, int n,
                                                               float2* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = undistort_pt(c, in[i].x, in[i].y);
}

// mvKeysUn of keypoint tables [n_frames][cap]: the keypoint with pt replaced.
__global__ __launch_bounds__(256) void undistort_keypoints_kernel(UndistCam c, const plvi_keypoint* __restrict__ in,
                                                                  const int* __restrict__ counts, int cap,
                                                                  plvi_keypoint* __restrict__ out) {
    const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= min(counts[f], cap)) return;
    plvi_keypoint k = in[(size_t)f * cap + i];
    const float2 p = undistort_pt(c, k.x, k.y);
    k.x = p.x;
    k.y = p.y;
    out[(size_t)f * cap + i] = k;
}

// mvKeysUn_Line endpoints (startPointX/Y, endPointX/Y) of keyline tables.
__global__ __launch_bounds__(256) void undistort_keylines_kernel(UndistCam c, const plvi_keyline* __restrict__ in,
                                                                 const int* __restrict__ counts, int cap,
                                                                 float4* __restrict__ out) {
    const int f = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
    if (i >= min(counts[f], cap)) return;
    const plvi_keyline& kl = in[(size_t)f * cap + i];
    const float2 s = undistort_pt(c, kl.startPointX, kl.startPointY);
    const float2 e = undistort_pt(c, kl.endPointX, kl.endPointY);
    out[(size_t)f * cap + i] = make_float4(s.x, s.y, e.x, e.y);
}

}  // namespace plvi

using namespace plvi;

extern "C" int plvi_undistort_points(const plvi_camera* cam, const float* d_xy, int n, float* d_out, void* stream) {
    if (!cam || n < 0 || cam->ndist < 4 || cam->ndist > 5) return PLVI_E_BADARG;
    if (n == 0) return PLVI_OK;
    hipLaunchKernelGGL(undistort_points_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       undist_cam(cam), reinterpret_cast<const float2*>(d_xy), n, reinterpret_cast<float2*>(d_out));
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_undistort_keypoints_batch(const plvi_camera* cam, const plvi_keypoint* d_kps, const int* d_count,
                                              int cap, int n_frames, plvi_keypoint* d_out, void* stream) {
    if (!cam || cap < 1 || n_frames < 0 || cam->ndist < 4 || cam->ndist > 5) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    hipLaunchKernelGGL(undistort_keypoints_kernel, dim3((cap + 255) / 256, n_frames), dim3(256), 0,
                       (hipStream_t)stream, undist_cam(cam), d_kps, d_count, cap, d_out);
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

extern "C" int plvi_undistort_keylines_batch(const plvi_camera* cam, const plvi_keyline* d_kl, const int* d_count,
                                             int cap, int n_frames, float* d_endpoints, void* stream) {
    if (!cam || cap < 1 || n_frames < 0 || cam->ndist < 4 || cam->ndist > 5) return PLVI_E_BADARG;
    if (n_frames == 0) return PLVI_OK;
    hipLaunchKernelGGL(undistort_keylines_kernel, dim3((cap + 255) / 256, n_frames), dim3(256), 0,
                       (hipStream_t)stream, undist_cam(cam), d_kl, d_count, cap, reinterpret_cast<float4*>(d_endpoints));
    PLVI_CHECK(hipGetLastError());
    return PLVI_OK;
}

// ComputeImageBounds: the four image corners undistorted on the device.
extern "C" int plvi_image_bounds(const plvi_camera* cam, int cols, int rows, float* bounds) {
    if (!cam || !bounds || cols <= 0 || rows <= 0) return PLVI_E_BADARG;
    if (cam->dist[0] == 0.0f) {
        bounds[0] = 0.0f; bounds[1] = (float)cols; bounds[2] = 0.0f; bounds[3] = (float)rows;
        return PLVI_OK;
    }
    const float in[8] = {0.0f, 0.0f, (float)cols, 0.0f, 0.0f, (float)rows, (float)cols, (float)rows};
    DevBuf d;
    if (d.alloc(64)) return PLVI_E_HIP;
    PLVI_CHECK(hipMemcpy(d.p, in, sizeof(in), hipMemcpyHostToDevice));
    int rc = plvi_undistort_points(cam, d.as<float>(), 4, d.as<float>() + 8, nullptr);
    if (rc) return rc;
    float p[8];
    PLVI_CHECK(hipMemcpy(p, d.as<float>() + 8, sizeof(p), hipMemcpyDeviceToHost));
    bounds[0] = std::min(p[0], p[4]);  // mnMinX = min(mat(0,0), mat(2,0))
    bounds[1] = std::max(p[2], p[6]);  // mnMaxX = max(mat(1,0), mat(3,0))
    bounds[2] = std::min(p[1], p[3]);  // mnMinY = min(mat(0,1), mat(1,1))
    bounds[3] = std::max(p[5], p[7]);  // mnMaxY = max(mat(2,1), mat(3,1))
    return PLVI_OK;
}
