// DSM extraction from a rendered depth image: the reference's
// get_latlonalt_from_nerf_prediction / get_dsm_from_nerf_prediction
// (datasets/satellite_scene.py:475-568) with modules/utils.py:103-139, on the GPU in fp64.
//  * k_dsm_points — one thread per ray: x = o + d·depth in the normalised scene, denormalised to
//    ECEF (× range + center), geodetic lat / lon / alt by the reference's closed form
//    (ecef_to_latlon_custom, utils.py:103-122), then UTM easting / northing in the zone of the
//    first point (utils.py:125-139 calls pyproj "+proj=utm"; restated here as the 6th-order
//    Krüger series of the transverse Mercator projection on WGS-84 — pyproj / PROJ are absent
//    offline: parity unpinned beyond the oracle restatement, oracle/dsm_ref.py).
//  * k_dsm_splat / k_dsm_finish — plyflatten(cloud, xoff, yoff, resolution, xsize, ysize,
//    radius, sigma = inf) (satellite_scene.py:547; the plyflatten package is absent: its
//    rasterisation restated, parity unpinned): each point lands in cell (floor((e − xoff)/res),
//    floor((yoff − n)/res)) and adds its altitude with weight exp(−d²/2σ²) (1 for σ = ∞) to every
//    cell of the (2·radius + 1)² window around it; a cell is the weighted mean, NaN when empty.
//    Sums and weights accumulate with fp64 vector atomics (order-dependent only in the last
//    bits of a double).
// HBM-bound and tiny next to a render (≈ 60 B per ray in, 16 B per cell).
#include <cmath>

#include "common.h"

namespace spn {

struct DsmPointArgs {
    const float* rays; int rs;
    const float* depth;
    int64_t n;
    double cx, cy, cz, range;
    int zone, south;
    double* lla;  // [n][3] lat, lon (degrees), alt, or null
    double* ena;  // [n][3] easting, northing, alt, or null
};

// WGS-84 transverse Mercator (UTM) by Krüger's series to 6th order in n (utm_krueger in
// oracle/dsm_ref.py is the same arithmetic in numpy)
__device__ __forceinline__ void utm_forward(double lat_deg, double lon_deg, int zone, int south, double* e, double* nn) {
    const double a = 6378137.0, f = 1.0 / 298.257223563, k0 = 0.9996;
    const double n = f / (2.0 - f), n2 = n * n, n3 = n2 * n, n4 = n3 * n, n5 = n4 * n, n6 = n5 * n;
    const double A = a / (1.0 + n) * (1.0 + n2 / 4.0 + n4 / 64.0 + n6 / 256.0);
    const double al[6] = {n / 2.0 - 2.0 * n2 / 3.0 + 5.0 * n3 / 16.0 + 41.0 * n4 / 180.0 - 127.0 * n5 / 288.0 +
                              7891.0 * n6 / 37800.0,
                          13.0 * n2 / 48.0 - 3.0 * n3 / 5.0 + 557.0 * n4 / 1440.0 + 281.0 * n5 / 630.0 -
                              1983433.0 * n6 / 1935360.0,
                          61.0 * n3 / 240.0 - 103.0 * n4 / 140.0 + 15061.0 * n5 / 26880.0 + 167603.0 * n6 / 181440.0,
                          49561.0 * n4 / 161280.0 - 179.0 * n5 / 168.0 + 6601661.0 * n6 / 7257600.0,
                          34729.0 * n5 / 80640.0 - 3418889.0 * n6 / 1995840.0,
                          212378941.0 * n6 / 319334400.0};
    const double deg = M_PI / 180.0;
    const double phi = lat_deg * deg;
    const double lam = (lon_deg - (6.0 * zone - 183.0)) * deg;
    const double c = 2.0 * sqrt(n) / (1.0 + n);
    const double t = sinh(atanh(sin(phi)) - c * atanh(c * sin(phi)));
    const double xi = atan2(t, cos(lam));
    const double eta = atanh(sin(lam) / sqrt(1.0 + t * t));
    double se = eta, sn = xi;
    for (int j = 1; j <= 6; ++j) {
        se += al[j - 1] * cos(2.0 * j * xi) * sinh(2.0 * j * eta);
        sn += al[j - 1] * sin(2.0 * j * xi) * cosh(2.0 * j * eta);
    }
    *e = 500000.0 + k0 * A * se;
    *nn = (south ? 10000000.0 : 0.0) + k0 * A * sn;
}

__global__ void k_dsm_points(DsmPointArgs g) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const float* r = g.rays + i * g.rs;
    const double d = (double)g.depth[i];
    // satellite_scene.py:488-500: in double, xyz_n = o + d·depth, then × range + center
    const double x = ((double)r[0] + (double)r[3] * d) * g.range + g.cx;
    const double y = ((double)r[1] + (double)r[4] * d) * g.range + g.cy;
    const double z = ((double)r[2] + (double)r[5] * d) * g.range + g.cz;
    // utils.py:103-122
    const double a = 6378137.0, e = 8.1819190842622e-2;
    const double asq = a * a, esq = e * e;
    const double b = sqrt(asq * (1.0 - esq)), bsq = b * b;
    const double ep = sqrt((asq - bsq) / bsq);
    const double p = sqrt(x * x + y * y);
    const double th = atan2(a * z, b * p);
    const double lon = atan2(y, x);
    const double st = sin(th), ct = cos(th);
    const double lat = atan2(z + ep * ep * b * st * st * st, p - esq * a * ct * ct * ct);
    const double sl = sin(lat);
    const double N = a / sqrt(1.0 - esq * sl * sl);
    const double alt = p / cos(lat) - N;
    const double lat_d = lat * 180.0 / M_PI, lon_d = lon * 180.0 / M_PI;
    if (g.lla) {
        g.lla[3 * i] = lat_d;
        g.lla[3 * i + 1] = lon_d;
        g.lla[3 * i + 2] = alt;
    }
    if (g.ena) {
        double east, north;
        utm_forward(lat_d, lon_d, g.zone, g.south, &east, &north);
        g.ena[3 * i] = east;
        g.ena[3 * i + 1] = north;
        g.ena[3 * i + 2] = alt;
    }
}

struct DsmRasterArgs {
    const double* ena; int64_t n;
    double xoff, yoff, res;
    int xsize, ysize, radius;
    double inv2s2;   // 1 / (2σ²); 0 for σ = ∞ (weight 1)
    double* acc;     // [2][ysize][xsize]: weighted sums, weights
    double* dsm;     // [ysize][xsize]
};

__global__ void k_dsm_splat(DsmRasterArgs g) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const double xx = (g.ena[3 * i] - g.xoff) / g.res, yy = (g.yoff - g.ena[3 * i + 1]) / g.res;
    const double v = g.ena[3 * i + 2];
    if (!(isfinite(xx) && isfinite(yy) && isfinite(v))) return;
    const double fx = floor(xx), fy = floor(yy);
    if (fx < -g.radius - 1 || fy < -g.radius - 1 || fx > g.xsize + g.radius || fy > g.ysize + g.radius) return;
    const int ci = (int)fx, cj = (int)fy;
    const int64_t cells = (int64_t)g.xsize * g.ysize;
    for (int dj = -g.radius; dj <= g.radius; ++dj)
        for (int di = -g.radius; di <= g.radius; ++di) {
            const int ii = ci + di, jj = cj + dj;
            if (ii < 0 || jj < 0 || ii >= g.xsize || jj >= g.ysize) continue;
            double w = 1.0;
            if (g.inv2s2 > 0.0) {
                const double dx = xx - (ii + 0.5), dy = yy - (jj + 0.5);
                w = exp(-(dx * dx + dy * dy) * g.inv2s2);
            }
            const int64_t k = (int64_t)jj * g.xsize + ii;
            atomicAdd(g.acc + k, w * v);
            atomicAdd(g.acc + cells + k, w);
        }
}

__global__ void k_dsm_finish(DsmRasterArgs g) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t cells = (int64_t)g.xsize * g.ysize;
    if (k >= cells) return;
    const double w = g.acc[cells + k];
    g.dsm[k] = w > 0.0 ? g.acc[k] / w : NAN;
}

}  // namespace spn

using namespace spn;

extern "C" int32_t spnerf_dsm_points(const float* rays, int32_t rs, int64_t n, const float* depth, const double* center,
                                     double range, int32_t utm_zone, int32_t south, double* lla, double* ena,
                                     void* stream) {
    hipStream_t s = (hipStream_t)stream;
    SPN_ARG(rays && depth && center && rs >= 6 && n >= 0, "dsm_points: bad arguments");
    SPN_ARG(utm_zone >= 1 && utm_zone <= 60, "dsm_points: UTM zone %d", utm_zone);
    if (n == 0) return SPNERF_OK;
    DsmPointArgs g{rays, rs, depth, n, center[0], center[1], center[2], range, utm_zone, south ? 1 : 0, lla, ena};
    ProfScope prof("dsm", s, 0.0, (double)n * (4.0 * rs + 4.0 + 24.0 * ((lla ? 1 : 0) + (ena ? 1 : 0))));
    hipLaunchKernelGGL(k_dsm_points, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_dsm_rasterize(const double* ena, int64_t n, double xoff, double yoff, double resolution,
                                        int32_t xsize, int32_t ysize, int32_t radius, double sigma, double* acc,
                                        double* dsm, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    SPN_ARG(ena && acc && dsm && n >= 0 && xsize > 0 && ysize > 0 && radius >= 0 && resolution > 0.0,
            "dsm_rasterize: bad arguments");
    SPN_ARG(!(sigma <= 0.0), "dsm_rasterize: sigma must be > 0 (inf for plain means)");
    const int64_t cells = (int64_t)xsize * ysize;
    DsmRasterArgs g{ena, n, xoff, yoff, resolution, xsize, ysize, radius,
                    std::isinf(sigma) ? 0.0 : 1.0 / (2.0 * sigma * sigma), acc, dsm};
    ProfScope prof("dsm", s, 0.0, (double)n * 24.0 + (double)cells * 24.0);
    SPN_HIP(hipMemsetAsync(acc, 0, 2 * cells * sizeof(double), s));
    if (n > 0) hipLaunchKernelGGL(k_dsm_splat, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, g);
    hipLaunchKernelGGL(k_dsm_finish, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, g);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}
