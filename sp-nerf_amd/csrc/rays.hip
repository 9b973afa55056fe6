// RPC camera rays on gfx950 — datasets/satellite_scene.py:21-68 (get_rays), :415-425
// (normalize_rays), :449-473 (get_sun_dirs) with modules/utils.py:59-100 (rescale_rpc,
// geodetic_to_ecef), one thread per pixel.
//
// Localization (image → ground) restates rpcm's iterative inversion of the RPC00B projection
// in fp64 (see oracle/rpc_ref.py): project the estimate and two offset points (lon + EPS,
// lat + EPS), decompose the image residual on the offset vectors, step; EPS = 2 then 0.1; stop
// at a squared normalised residual < 1e-18 (rpcm iterates its whole batch until every point
// converges; here each pixel stops on its own and takes two extra refinement steps).
// Precision sequence of the reference: ECEF in fp64 → cast to fp32 (satellite_scene.py:66) →
// centring and scaling in fp32 (:415-425), so the 0.5 m fp32 quantisation of ECEF at
// 5.45e6 m is reproduced, not removed.
#include "common.h"

namespace spn {

struct RpcArgs {
    double off[10];  // row_offset col_offset lat_offset lon_offset alt_offset row_scale col_scale lat_scale lon_scale alt_scale
    double rn[20], rd[20], cn[20], cd[20];
    double min_alt, max_alt;
    int row0, col0, nrows, ncols;
    const int32_t* pix;  // optional (n, 2) [col, row] pixel list instead of the rectangle
    int64_t n;
    float center[3], range, sun[3];
    int normalize;
    float* out;
    int stride;
};

__device__ __forceinline__ double rpoly(const double* c, double x, double y, double z) {
    // x = lat, y = lon, z = alt (normalised); RPC00B monomial order
    return c[0] + c[1] * y + c[2] * x + c[3] * z + c[4] * y * x + c[5] * y * z + c[6] * x * z + c[7] * y * y +
           c[8] * x * x + c[9] * z * z + c[10] * x * y * z + c[11] * y * y * y + c[12] * y * x * x +
           c[13] * y * z * z + c[14] * y * y * x + c[15] * x * x * x + c[16] * x * z * z + c[17] * y * y * z +
           c[18] * x * x * z + c[19] * z * z * z;
}

__device__ __forceinline__ void proj_n(const RpcArgs& a, double lat, double lon, double alt, double& col, double& row) {
    col = rpoly(a.cn, lat, lon, alt) / rpoly(a.cd, lat, lon, alt);
    row = rpoly(a.rn, lat, lon, alt) / rpoly(a.rd, lat, lon, alt);
}

// normalised image (cn, rn) at normalised altitude an → degrees (lon, lat)
__device__ void localize(const RpcArgs& a, double cn, double rn, double an, double& lon_d, double& lat_d) {
    double lon = -1.0, lat = -1.0, eps = 2.0;
    int extra = -1;
    for (int it = 0; it <= 100; ++it) {
        double x0, y0;
        proj_n(a, lat, lon, an, x0, y0);
        const double res = (x0 - cn) * (x0 - cn) + (y0 - rn) * (y0 - rn);
        if (res < 1e-18) {
            if (extra < 0) extra = 2;
            if (extra-- == 0) break;
        }
        double x1, y1, x2, y2;
        proj_n(a, lat, lon + eps, an, x1, y1);
        proj_n(a, lat + eps, lon, an, x2, y2);
        const double e1x = x1 - x0, e1y = y1 - y0, e2x = x2 - x0, e2y = y2 - y0;
        const double ux = cn - x0, uy = rn - y0;
        const double a1 = (ux * e1x + uy * e1y) / (e1x * e1x + e1y * e1y);
        const double a2 = (ux * e2x + uy * e2y) / (e2x * e2x + e2y * e2y);
        lon += a1 * eps;
        lat += a2 * eps;
        eps = 0.1;
    }
    lon_d = lon * a.off[8] + a.off[3];
    lat_d = lat * a.off[7] + a.off[2];
}

__device__ void ecef(double lat_deg, double lon_deg, double alt, double& x, double& y, double& z) {
    const double A = 6378137.0, Bm = 6356752.314245;
    const double ba = (Bm * Bm) / (A * A);
    const double e2 = 1.0 - ba;
    const double la = lat_deg * (M_PI / 180.0), lo = lon_deg * (M_PI / 180.0);
    const double sl = sin(la);
    const double N = A / sqrt(1.0 - e2 * (sl * sl));
    x = (N + alt) * cos(la) * cos(lo);
    y = (N + alt) * cos(la) * sin(lo);
    z = (ba * N + alt) * sl;
}

__global__ __launch_bounds__(256) void k_rpc_rays(RpcArgs a) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    double col, row;
    if (a.pix) {
        col = a.pix[2 * i];
        row = a.pix[2 * i + 1];
    } else {
        col = a.col0 + (double)(i % a.ncols);
        row = a.row0 + (double)(i / a.ncols);
    }
    const double cnm = (col - a.off[1]) / a.off[6], rnm = (row - a.off[0]) / a.off[5];
    double lon, lat, xn, yn, zn, xf, yf, zf;
    localize(a, cnm, rnm, (a.max_alt - a.off[4]) / a.off[9], lon, lat);
    ecef(lat, lon, a.max_alt, xn, yn, zn);
    localize(a, cnm, rnm, (a.min_alt - a.off[4]) / a.off[9], lon, lat);
    ecef(lat, lon, a.min_alt, xf, yf, zf);
    const double dx = xf - xn, dy = yf - yn, dz = zf - zn;
    const double nrm = sqrt((dx * dx + dy * dy) + dz * dz);
    float* o = a.out + i * a.stride;
    float v[8] = {(float)xn, (float)yn, (float)zn, (float)(dx / nrm), (float)(dy / nrm), (float)(dz / nrm), 0.f,
                  (float)nrm};
    if (a.normalize) {
        for (int k = 0; k < 3; ++k) v[k] = __fdiv_rn(__fsub_rn(v[k], a.center[k]), a.range);
        v[6] = __fdiv_rn(v[6], a.range);
        v[7] = __fdiv_rn(v[7], a.range);
    }
    for (int k = 0; k < 8; ++k) o[k] = v[k];
    if (a.stride >= 11)
        for (int k = 0; k < 3; ++k) o[8 + k] = a.sun[k];
}

}  // namespace spn

using namespace spn;

extern "C" int32_t spnerf_rpc_rays(const double* rpc, double downscale, double min_alt, double max_alt, int32_t row0,
                                   int32_t col0, int32_t n_rows, int32_t n_cols, const int32_t* pixels, int64_t n_pixels,
                                   const float* center, float range, const float* sun, float* rays, int32_t ray_stride,
                                   void* stream) {
    SPN_ARG(rpc && rays, "rpc_rays: NULL pointer");
    SPN_ARG(ray_stride >= 8 && downscale > 0, "rpc_rays: bad stride / downscale");
    SPN_ARG(ray_stride < 11 || sun, "rpc_rays: an 11-wide ray needs the sun direction");
    RpcArgs a{};
    for (int k = 0; k < 10; ++k) a.off[k] = rpc[k];
    for (int k = 0; k < 20; ++k) {
        a.rn[k] = rpc[10 + k];
        a.rd[k] = rpc[30 + k];
        a.cn[k] = rpc[50 + k];
        a.cd[k] = rpc[70 + k];
    }
    const double s = 1.0 / downscale;  // utils.rescale_rpc(rpc, 1/downscale)
    a.off[5] *= s;
    a.off[6] *= s;
    a.off[0] *= s;
    a.off[1] *= s;
    a.min_alt = min_alt;
    a.max_alt = max_alt;
    a.row0 = row0;
    a.col0 = col0;
    a.nrows = n_rows;
    a.ncols = n_cols;
    a.pix = pixels;
    a.n = pixels ? n_pixels : (int64_t)n_rows * n_cols;
    a.normalize = center != nullptr;
    if (center)
        for (int k = 0; k < 3; ++k) a.center[k] = center[k];
    a.range = range;
    if (sun)
        for (int k = 0; k < 3; ++k) a.sun[k] = sun[k];
    a.out = rays;
    a.stride = ray_stride;
    if (a.n == 0) return SPNERF_OK;
    ProfScope prof("rpc_rays", (hipStream_t)stream, 0.0, 4.0 * ray_stride * a.n);
    hipLaunchKernelGGL(k_rpc_rays, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}
