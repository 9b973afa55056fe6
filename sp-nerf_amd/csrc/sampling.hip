// Sample generation of the SP-NeRF render path (modules/rendering.py) on gfx950:
//  * k_stratified  — jittered stratified depths (render_rays :131-144, perturb = 1)
//  * k_guided      — GenerateGuidedSamples (:92-116: 3σ window around the pass-1 depth or
//                    the GT depth, sample_3sigma :58-73, sample_pdf :14-55), then sort of the
//                    guided depths and merge with the stratified ones (:165-167), all fused,
//                    one wavefront per ray, with NO host synchronisation (the reference copies
//                    valid_depth to the host every step, :101-104)
//  * k_sample_pdf / k_sample_3sigma / k_sort_rows — the standalone drop-ins.
//  * k_merge_rows  — the main pass's MLP rows gathered into the sorted depth order from pass 1's
//                    rows and the guided samples' rows (each point evaluated once), and back.
// Inverse-CDF sampling keeps the CDF in LDS and binary-searches it per sample; cumsum is
// accumulated in double as torch's CPU cumsum does.
#include "common.h"
#include "wave.h"

namespace spn {

// u: the draws, or null: drawn on the device from rng (spnerf_rng)
__global__ void k_stratified(int64_t B, int S, const float* __restrict__ rays, int rs, const float* __restrict__ u,
                             float* __restrict__ z, spnerf_rng rng) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= B * S) return;
    const int64_t ray = i / S;
    const int k = (int)(i % S);
    const float nr = rays[ray * rs + 6], fr = rays[ray * rs + 7];
    auto zl = [&](int q) {  // near*(1-t) + far*t  (rendering.py:133)
        const float t = linspace_at(0.f, 1.f, S, q);
        return __fadd_rn(__fmul_rn(nr, __fsub_rn(1.f, t)), __fmul_rn(fr, t));
    };
    const float zc = zl(k);
    const float hi = k < S - 1 ? __fmul_rn(0.5f, __fadd_rn(zc, zl(k + 1))) : zc;
    const float lo = k > 0 ? __fmul_rn(0.5f, __fadd_rn(zl(k - 1), zc)) : zc;
    const float ui = u ? u[i] : rng_uniform(rng, ray, k);
    z[i] = __fadd_rn(lo, __fmul_rn(__fsub_rn(hi, lo), ui));
}

struct WaveLds {
    float cdf[256];
    float bins[256];
    float buf[256];
};

// Build the CDF of (w + eps) over nb bins into L.cdf[0..nb] (cdf[0] = 0).  Lane l owns bins
// l*EPL .. l*EPL+EPL-1.  Returns nothing; caller syncs.
template <int EPL>
__device__ void build_cdf(WaveLds& L, const float (&w)[EPL], int nb, int lane, float eps) {
    float wl[EPL];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        wl[j] = e < nb ? w[j] + eps : 0.f;
        s += wl[j];
    }
    const float tot = wave_sum(s);
    double run = 0.0, loc[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        run += (double)(wl[j] / tot);
        loc[j] = run;
    }
    const double incl = wave_scan_add(run, lane);
    double base = __shfl_up(incl, 1, 64);
    if (lane == 0) base = 0.0;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        if (e < nb) L.cdf[e + 1] = (float)(base + loc[j]);
    }
    if (lane == 0) L.cdf[0] = 0.f;
}

// sample_pdf inner step for one u: searchsorted(right=True) + gather + interpolation
__device__ __forceinline__ float invert_cdf(const WaveLds& L, int nb, float u, float eps) {
    int lo = 0, hi = nb + 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L.cdf[mid] <= u) lo = mid + 1;
        else hi = mid;
    }
    const int below = lo - 1 > 0 ? lo - 1 : 0;
    const int above = lo < nb ? lo : nb;
    const float c0 = L.cdf[below], c1 = L.cdf[above];
    const float b0 = L.bins[below], b1 = L.bins[above];
    float den = c1 - c0;
    if (den < eps) den = 1.f;
    return b0 + (u - c0) / den * (b1 - b0);
}

// sample_3sigma bin edges / Gaussian bin weights of one ray into L.bins and w (N edges, N-1 bins)
template <int EPL>
__device__ void window_bins(WaveLds& L, float (&w)[EPL], float low, float high, int N, float nr, float fr, int lane) {
    const float step = (high - low) / (float)(N - 1);
    float edge[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        const float t = linspace_at(0.f, 1.f, N, e < N ? e : 0);
        float v = __fadd_rn(__fmul_rn(low, __fsub_rn(1.f, t)), __fmul_rn(high, t));
        v = fminf(fmaxf(v, nr), fr);  // Tensor.clamp(near, far)
        edge[j] = v;
        if (e < N) L.bins[e] = v;
    }
    const float en0 = __shfl_down(edge[0], 1, 64);
    const float gc = (float)(1.0 / 2.5066282746310002);  // 1/sqrt(2π) as an fp32 scalar
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        w[j] = 0.f;
        if (e < N - 1) {
            const float en = j + 1 < EPL ? edge[j + 1] : en0;
            const float factor = (en - edge[j]) / step;
            const float x = linspace_at(-3.f, 3.f, N - 1, e);
            w[j] = factor * (gc * expf(-0.5f * (x * x)));
        }
    }
}

struct GuidedArgs {
    int64_t B;
    int S;
    const float *z, *depth, *weights, *clamp_nf;
    const int64_t* valid;
    const float *tdepth, *tstd;
    int td_stride;
    const float *u_pred, *u_gt;   // or null: drawn from rng, slots rng.slot (pred) / rng.slot + 1 (GT)
    float *z_sorted, *z_unsort;
    spnerf_rng rng;
};

template <int EPL>
__global__ __launch_bounds__(256) void k_guided(GuidedArgs a) {
    __shared__ WaveLds lds[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ray = (int64_t)blockIdx.x * 4 + wv;
    const bool active = ray < a.B;
    const int64_t rr = active ? ray : 0;
    WaveLds& L = lds[wv];
    // each wave sorts in its own LDS slice: a wave barrier orders its LDS writes and reads (the
    // block barriers made the four rays of a block wait for each other at every sort stage)
    const auto wsync = [] {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    };
    const int S = a.S, N = S;
    // predicted-depth spread: std = sqrt(Σ (z - depth)^2 w)   (rendering.py:81)
    const float dep = a.depth[rr];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        if (e < S) {
            const float dz = a.z[rr * S + e] - dep;
            s += (dz * dz) * a.weights[rr * S + e];
        }
    }
    const float sd = sqrtf(wave_sum(s));
    float low = dep - 3.f * sd, high = dep + 3.f * sd;
    const bool dev_rng = a.u_pred == nullptr;
    const float* u = dev_rng ? nullptr : a.u_pred + rr * N;
    spnerf_rng rk = a.rng;
    if (a.valid && a.valid[rr] > 0) {  // GT window replaces the predicted one (:98-114)
        const float gt = a.tdepth[rr * a.td_stride], gs = a.tstd[rr];
        low = gt - 3.f * gs;
        high = gt + 3.f * gs;
        if (dev_rng) rk.slot += 1;
        else u = a.u_gt + rr * N;
    }
    const float nr = a.clamp_nf[0], fr = a.clamp_nf[1];
    float w[EPL];
    window_bins<EPL>(L, w, low, high, N, nr, fr, lane);
    build_cdf<EPL>(L, w, N - 1, lane, 1e-5f);
    wsync();
    // 2N slots: [0,N) guided samples (sorted first, rendering.py:165), [N,2N) stratified
    int n2 = 1;
    while (n2 < 2 * N) n2 <<= 1;
    for (int e = lane; e < n2; e += 64)
        L.buf[e] = e < N ? invert_cdf(L, N - 1, dev_rng ? rng_uniform(rk, rr, e) : u[e], 1e-5f) : INFINITY;
    wsync();
    int n1 = 1;
    while (n1 < N) n1 <<= 1;
    // sort the guided half (padded with +inf up to n1 ≤ n2)
    for (int e = lane + N; e < n1; e += 64) L.buf[e] = INFINITY;
    wsync();
    wave_bitonic_sort(L.buf, n1, lane, wsync);
    if (active) {
        for (int e = lane; e < 2 * N; e += 64)
            a.z_unsort[ray * 2 * N + e] = e < N ? a.z[ray * N + e] : L.buf[e - N];
    }
    wsync();
    // merge: [sorted guided | stratified | +inf pad] → full sort of n2 slots
    for (int e = lane; e < n2; e += 64) {
        float v = INFINITY;
        if (e < N) v = L.buf[e];
        else if (e < 2 * N) v = a.z[rr * N + (e - N)];
        L.cdf[e & 255] = v;  // stage in cdf (free now)
    }
    wsync();
    wave_bitonic_sort(L.cdf, n2, lane, wsync);
    if (active)
        for (int e = lane; e < 2 * N; e += 64) a.z_sorted[ray * 2 * N + e] = L.cdf[e];
}

struct PdfArgs {
    int64_t B;
    int nb, n_imp;
    const float *bins, *w, *u;   // u null: drawn from rng
    float eps;
    float* out;
    const float *low, *high, *clamp_nf;  // sample_3sigma mode when low != nullptr
    spnerf_rng rng;
};

template <int EPL>
__global__ __launch_bounds__(256) void k_sample_pdf(PdfArgs a) {
    __shared__ WaveLds lds[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ray = (int64_t)blockIdx.x * 4 + wv;
    if (ray >= a.B) return;  // no block barriers below
    WaveLds& L = lds[wv];
    float w[EPL];
    int nb = a.nb;
    if (a.low) {
        nb = a.n_imp - 1;
        window_bins<EPL>(L, w, a.low[ray], a.high[ray], a.n_imp, a.clamp_nf[0], a.clamp_nf[1], lane);
    } else {
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
            const int e = lane * EPL + j;
            w[j] = e < nb ? a.w[ray * nb + e] : 0.f;
        }
        for (int e = lane; e <= nb; e += 64) L.bins[e] = a.bins[ray * (nb + 1) + e];
    }
    build_cdf<EPL>(L, w, nb, lane, a.eps);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int e = lane; e < a.n_imp; e += 64)
        a.out[ray * a.n_imp + e] = invert_cdf(L, nb, a.u ? a.u[ray * a.n_imp + e] : rng_uniform(a.rng, ray, e), a.eps);
}

__global__ __launch_bounds__(256) void k_sort_rows(int64_t B, int n, const float* __restrict__ in, float* __restrict__ out) {
    __shared__ float buf[4][256];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ray = (int64_t)blockIdx.x * 4 + wv;
    const bool active = ray < B;
    int n2 = 1;
    while (n2 < n) n2 <<= 1;
    for (int e = lane; e < n2; e += 64) buf[wv][e] = (active && e < n) ? in[ray * n + e] : INFINITY;
    __syncthreads();
    wave_bitonic_sort(buf[wv], n2, lane, [] { __syncthreads(); });
    if (active)
        for (int e = lane; e < n; e += 64) out[ray * n + e] = buf[wv][e];
}

// The main pass's samples are the union of the stratified depths and the guided ones, sorted
// (rendering.py:165-168).  Its points at the stratified depths are pass 1's points (:147, :168:
// the same o + d·z), so their MLP rows are computed once: the rows of the two segments (pass 1's
// s1 per ray, then the guided s2 per ray, spnerf_mlp_forward_window) are gathered into the sorted
// order here, and the backward scatters the sorted rows' gradients back to the segments.  The
// sorted position of element e of z_unsort = [z | sorted z_2] (the reference's z_vals_unsort) is
// its rank #{f : z[f] < z[e]} + #{f < e : z[f] == z[e]} — a permutation into ascending order, so
// the rows land where torch.sort puts their depths (equal depths are the same point: equal rows).
// One 128-thread block per ray (n = s1 + s2 <= 256: up to two elements per thread for the ranks;
// small blocks: every ray of a 4 096-ray batch resident at once, one latency round).  The
// ray's rows move through LDS so that every global access is a contiguous run of the ray's rows,
// all issued up front: forward the two segments' runs (s1·n_out and s2·n_out floats) in and the
// sorted run out, backward the reverse.  The ranks are formed while the rows are in flight.
// bwd = 0: sorted ← segments; 1: segments ← sorted (the pointers' roles swap, not their types)
__global__ __launch_bounds__(128) void k_merge_rows(int64_t B, int s1, int s2, const float* __restrict__ zu,
                                                    float* __restrict__ seg1, float* __restrict__ seg2,
                                                    float* __restrict__ sorted, int n_out, int bwd) {
    extern __shared__ __attribute__((aligned(16))) float msm[];
    const int tid = threadIdx.x;
    const int64_t ray = blockIdx.x;
    const int n = s1 + s2;
    const int n4 = (n + 3) & ~3;  // z padded with +inf to whole float4s (never below a finite depth)
    float* zs = msm;                                    // [n4]
    int* rank_of = reinterpret_cast<int*>(msm + n4);    // [n]
    int* src = rank_of + n;                             // [n]: sorted position → element
    float* rows = msm + n4 + 2 * n;                     // [n · n_out]
    const float inv = 1.f / (float)n_out;
    const int n1 = s1 * n_out, nn = n * n_out;
    float* g1 = seg1 + ray * (int64_t)n1;
    float* g2 = seg2 + ray * (int64_t)(s2 * n_out);
    float* gs = sorted + ray * (int64_t)nn;
    // the depths first, then (up to 128·U values) the rows: the depths' wait does not wait for them
    constexpr int NT = 128, U = 16;
    float zv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) zv[h] = tid + NT * h < n ? zu[ray * n + tid + NT * h] : INFINITY;
    const bool fits = nn <= NT * U;
    auto src_of = [&](int i) -> float* { return bwd ? gs + i : (i < n1 ? g1 + i : g2 + (i - n1)); };
    float v[U];
    if (fits) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = tid + NT * u;
            v[u] = i < nn ? *src_of(i) : 0.f;
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
        if (tid + NT * h < n4) zs[tid + NT * h] = zv[h];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int e = tid + NT * h;
        if (e < n) {
            int rank = 0;
#pragma unroll 4
            for (int f = 0; f < n4; f += 4) {
                const f32x4 w = *reinterpret_cast<const f32x4*>(zs + f);
#pragma unroll
                for (int q = 0; q < 4; ++q) rank += (w[q] < zv[h]) || (w[q] == zv[h] && f + q < e);
            }
            rank_of[e] = rank;
            src[rank] = e;
        }
    }
    // the rows into LDS (element e's row at rows[e · n_out]: segment order forward, sorted order
    // backward)
    if (fits) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (tid + NT * u < nn) rows[tid + NT * u] = v[u];
    } else {
        for (int i = tid; i < nn; i += NT) rows[i] = *src_of(i);
    }
    __syncthreads();
    if (!bwd) {
        for (int i = tid; i < nn; i += NT) {
            const int t = (int)(((float)i + 0.5f) * inv), col = i - t * n_out;  // i / n_out (exact: i < 2^16)
            gs[i] = rows[src[t] * n_out + col];
        }
    } else {
        for (int i = tid; i < nn; i += NT) {
            const int e = (int)(((float)i + 0.5f) * inv), col = i - e * n_out;
            const float x = rows[rank_of[e] * n_out + col];
            if (i < n1) g1[i] = x;
            else g2[i - n1] = x;
        }
    }
}

}  // namespace spn

using namespace spn;

static int32_t merge_rows(int64_t n_rays, int32_t s1, int32_t s2, const float* z_unsort, float* seg1, float* seg2,
                          float* sorted, int32_t n_out, int bwd, hipStream_t s) {
    SPN_ARG(z_unsort && seg1 && seg2 && sorted, "merge_samples: NULL pointer");
    SPN_ARG(s1 >= 1 && s2 >= 1 && s1 + s2 <= 256 && n_out >= 1 && n_rays >= 0, "merge_samples: bad sizes");
    if (n_rays == 0) return SPNERF_OK;
    ProfScope prof("merge_samples", s, 0.0, (double)n_rays * (s1 + s2) * (8.0 * n_out + 4.0));
    const size_t lds = sizeof(float) * ((size_t)(s1 + s2) * (3 + n_out) + 3);
    SPN_ARG(lds <= 64 * 1024, "merge_samples: %d samples x %d outputs too large", s1 + s2, n_out);
    hipLaunchKernelGGL(k_merge_rows, dim3((unsigned)n_rays), dim3(128), lds, s, n_rays, s1, s2, z_unsort, seg1, seg2, sorted,
                       n_out, bwd);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_merge_samples(int64_t n_rays, int32_t s1, int32_t s2, const float* z_unsort, const float* out1,
                                        const float* out2, int32_t n_out, float* out_sorted, void* stream) {
    return merge_rows(n_rays, s1, s2, z_unsort, const_cast<float*>(out1), const_cast<float*>(out2), out_sorted, n_out, 0,
                      (hipStream_t)stream);
}

extern "C" int32_t spnerf_merge_samples_backward(int64_t n_rays, int32_t s1, int32_t s2, const float* z_unsort,
                                                 const float* d_sorted, int32_t n_out, float* d_out1, float* d_out2,
                                                 void* stream) {
    return merge_rows(n_rays, s1, s2, z_unsort, d_out1, d_out2, const_cast<float*>(d_sorted), n_out, 1, (hipStream_t)stream);
}

static spnerf_rng rng_or_null(const spnerf_rng* r) { return r ? *r : spnerf_rng{nullptr, 0, 0, 0}; }

extern "C" int32_t spnerf_sample_stratified(int64_t n_rays, int32_t n_samples, const float* rays, int32_t ray_stride,
                                            const float* u, float* z, const spnerf_rng* rng, void* stream) {
    SPN_ARG(rays && z && (u || (rng && rng->state)), "sample_stratified: NULL pointer");
    SPN_ARG(n_samples >= 2 && ray_stride >= 8 && n_rays >= 0, "sample_stratified: bad sizes");
    const int64_t n = n_rays * n_samples;
    if (n == 0) return SPNERF_OK;
    hipLaunchKernelGGL(k_stratified, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n_rays,
                       n_samples, rays, ray_stride, u, z, rng_or_null(rng));
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_sample_guided(int64_t n_rays, int32_t n_samples, const float* z, const float* depth,
                                        const float* weights, const float* clamp_nf, const int64_t* valid_depth,
                                        const float* target_depths, int32_t td_stride, const float* target_std,
                                        const float* u_pred, const float* u_gt, float* z_sorted, float* z_unsort,
                                        const spnerf_rng* rng, void* stream) {
    const bool dev_rng = u_pred == nullptr;
    SPN_ARG(z && depth && weights && clamp_nf && z_sorted && z_unsort && (!dev_rng || (rng && rng->state)),
            "sample_guided: NULL pointer");
    SPN_ARG(!valid_depth || (target_depths && target_std && (u_gt || dev_rng)), "sample_guided: train mode needs GT inputs");
    SPN_ARG(n_samples >= 2 && n_samples <= 128, "sample_guided: n_samples %d must be in [2, 128]", n_samples);
    if (n_rays == 0) return SPNERF_OK;
    GuidedArgs a{n_rays, n_samples, z, depth, weights, clamp_nf, valid_depth, target_depths, target_std, td_stride,
                 u_pred, dev_rng ? nullptr : u_gt, z_sorted, z_unsort, rng_or_null(rng)};
    const dim3 g((unsigned)((n_rays + 3) / 4)), b(256);
    ProfScope prof("sample_guided", (hipStream_t)stream, 0.0, (double)n_rays * n_samples * 4.0 * 7.0);
    if (n_samples <= 64) hipLaunchKernelGGL(k_guided<1>, g, b, 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL(k_guided<2>, g, b, 0, (hipStream_t)stream, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

static int32_t launch_pdf(const PdfArgs& a, int nbins, hipStream_t s) {
    const dim3 g((unsigned)((a.B + 3) / 4)), b(256);
    if (nbins <= 64) hipLaunchKernelGGL(k_sample_pdf<1>, g, b, 0, s, a);
    else if (nbins <= 128) hipLaunchKernelGGL(k_sample_pdf<2>, g, b, 0, s, a);
    else hipLaunchKernelGGL(k_sample_pdf<4>, g, b, 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_sample_pdf(int64_t n_rays, int32_t n_bins, const float* bins, const float* weights,
                                     int32_t n_imp, const float* u, float eps, float* samples, const spnerf_rng* rng,
                                     void* stream) {
    SPN_ARG(bins && weights && samples && (u || (rng && rng->state)), "sample_pdf: NULL pointer");
    SPN_ARG(n_bins >= 1 && n_bins + 1 <= 256 && n_imp >= 1, "sample_pdf: n_bins %d / n_imp %d out of range", n_bins, n_imp);
    if (n_rays == 0) return SPNERF_OK;
    PdfArgs a{n_rays, n_bins, n_imp, bins, weights, u, eps, samples, nullptr, nullptr, nullptr, rng_or_null(rng)};
    return launch_pdf(a, n_bins, (hipStream_t)stream);
}

extern "C" int32_t spnerf_sample_3sigma(int64_t n_rays, int32_t n, const float* low, const float* high,
                                        const float* clamp_nf, const float* u, float* out, void* stream) {
    SPN_ARG(low && high && clamp_nf && u && out, "sample_3sigma: NULL pointer");
    SPN_ARG(n >= 2 && n <= 256, "sample_3sigma: n %d out of range", n);
    if (n_rays == 0) return SPNERF_OK;
    PdfArgs a{n_rays, n - 1, n, nullptr, nullptr, u, 1e-5f, out, low, high, clamp_nf, spnerf_rng{nullptr, 0, 0, 0}};
    return launch_pdf(a, n, (hipStream_t)stream);
}

extern "C" int32_t spnerf_sort_rows(int64_t n_rays, int32_t n, const float* in, float* out, void* stream) {
    SPN_ARG(in && out, "sort_rows: NULL pointer");
    SPN_ARG(n >= 1 && n <= 256, "sort_rows: n %d out of range", n);
    if (n_rays == 0) return SPNERF_OK;
    hipLaunchKernelGGL(k_sort_rows, dim3((unsigned)((n_rays + 3) / 4)), dim3(256), 0, (hipStream_t)stream, n_rays, n, in, out);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}
