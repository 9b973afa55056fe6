// σ→α volumetric compositing with the solar-visibility irradiance term
// (inference(), models/spnerf.py:115-134,156), forward and backward, one wavefront per ray.
//
// Lane l holds the EPL consecutive samples l*EPL .. l*EPL+EPL-1 (S ≤ 64*EPL); the exclusive
// cumprod of (1-α+1e-10) is a lane-local product + a 6-step wavefront scan, the backward's
// reversed cumsum a lane-local suffix sum + a 6-step suffix scan.  A ray's S x NO block of MLP
// outputs is contiguous in HBM: the wave copies it into its own LDS slice with 16-B loads
// (coalesced) and every per-sample column is read from there (a lane reading its samples' rows
// straight from HBM walks them at a 44-56 B stride); the backward assembles the ray's d_out block
// in LDS the same way and writes it out with 16-B stores.  The backward follows torch
// autograd's formulas exactly where they differ from the textbook derivative: cumprod's
// no-zero fast path  dIn_m = (Σ_{j≥m} out_j·gOut_j) / In_m  (FunctionsManual cumprod_backward),
// clamp's inclusive pass-through mask, relu's result>0 mask, mean's division by S.
#include "common.h"
#include "wave.h"

namespace spn {

struct CompArgs {
    int64_t B;
    int S, NO, sem_col, n_sem, weights_only;
    const float *z, *out, *noise;
    float noise_std;
    spnerf_rng rng;   // noise drawn on the device when rng.state is set (and noise is null)
    float *rgb, *depth, *w, *T, *sem;
    const float *g_rgb, *g_depth, *g_w, *g_T, *g_sem;
    float* d_out;
    // weights-only passes with SPNERF_COMP_SUN_COLUMN: the sun-visibility column out (forward),
    // its gradient into d_out's sun column (backward) — the solar pass's sun_sc (rendering.py:177)
    float* sun_out;
    const float* g_sun;
};

__device__ __forceinline__ float relu_t(float x) { return x != x ? x : (x > 0.f ? x : 0.f); }

template <int EPL>
struct RayState {
    float z[EPL], al[EPL], t[EPL], T[EPL], w[EPL], r[EPL], E[EPL], dl[EPL];
};

// per-sample alpha / transparency / weights of one ray (spnerf.py:116-128)
// rows: the ray's S x NO output block (LDS copy)
template <int EPL>
__device__ __forceinline__ void march(const CompArgs& a, int64_t ray, int lane, const float* rows, RayState<EPL>& st) {
    const int S = a.S;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        st.z[j] = e < S ? a.z[ray * S + e] : 0.f;
    }
    const float zn0 = __shfl_down(st.z[0], 1, 64);
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        if (e < S) {
            const int64_t p = ray * S + e;
            float sg = rows[e * a.NO + 3];
            if (a.noise) sg = sg + a.noise[p] * a.noise_std;
            else if (a.rng.state) sg = sg + rng_normal(a.rng, ray, e) * a.noise_std;
            const float zn = j + 1 < EPL ? st.z[j + 1] : zn0;
            const float dl = e == S - 1 ? 1e10f : zn - st.z[j];
            const float r = relu_t(sg);
            const float E = expf(-dl * r);
            const float al = 1.f - E;
            st.dl[j] = dl;
            st.r[j] = r;
            st.E[j] = E;
            st.al[j] = al;
            st.t[j] = (1.f - al) + 1e-10f;
        } else {
            st.dl[j] = st.r[j] = st.E[j] = st.al[j] = 0.f;
            st.t[j] = 1.f;
        }
    }
    // exclusive cumprod in double (torch's CPU cumprod accumulates in double), rounded once
    double run = 1.0, excl[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        excl[j] = run;
        run *= (double)st.t[j];
    }
    const double incl = wave_scan_mul(run, lane);
    double lane_excl = __shfl_up(incl, 1, 64);
    if (lane == 0) lane_excl = 1.0;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        st.T[j] = (float)(lane_excl * excl[j]);
        st.w[j] = st.al[j] * st.T[j];
    }
}

// the ray's contiguous S·NO floats: HBM → this wave's LDS slice, 16-B pieces when aligned, up to
// 8 loads per lane in flight before their LDS stores
__device__ __forceinline__ void stage_rows(const float* __restrict__ src, float* dst, int n, int lane) {
    if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        const int nq = n >> 2;
        for (int base = 0; base < nq; base += 512) {
            f32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = min(base + lane + 64 * k, nq - 1);  // clamped: unconditional loads
                v[k] = ld4(src + 4 * i);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int i = base + lane + 64 * k;
                if (i < nq) reinterpret_cast<f32x4*>(dst)[i] = v[k];
            }
        }
    } else {
        for (int i = lane; i < n; i += 64) dst[i] = src[i];
    }
    wave_lds_sync();
}

template <int EPL>
__global__ __launch_bounds__(256) void k_composite_fwd(CompArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sh_rows[];
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (ray >= a.B) return;  // wave-uniform; the LDS slices are wave-private (no block barrier)
    const int S = a.S, NO = a.NO;
    float* rows = sh_rows + (threadIdx.x >> 6) * (S * NO);
    if (a.weights_only) {   // σ is the only column read: stride loads of one column
        for (int e = lane; e < S; e += 64) rows[e * NO + 3] = a.out[(ray * S + e) * NO + 3];
        if (a.sun_out)
            for (int e = lane; e < S; e += 64) a.sun_out[ray * S + e] = a.out[(ray * S + e) * NO + 4];
        wave_lds_sync();
    } else {
        stage_rows(a.out + ray * (int64_t)(S * NO), rows, S * NO, lane);
    }
    RayState<EPL> st;
    march<EPL>(a, ray, lane, rows, st);
    float dsum = 0.f, c0 = 0.f, c1 = 0.f, c2 = 0.f;
    float wv[EPL], tv[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        wv[j] = st.w[j];
        tv[j] = st.T[j];
        if (e >= S) continue;
        dsum += st.w[j] * st.z[j];
        if (!a.weights_only) {
            const float* o = rows + e * NO;
            const float sun = o[4], om = 1.f - sun;
            c0 += (st.w[j] * o[0]) * (sun + om * o[5]);
            c1 += (st.w[j] * o[1]) * (sun + om * o[6]);
            c2 += (st.w[j] * o[2]) * (sun + om * o[7]);
        }
    }
    // w, T: a lane's EPL consecutive samples as one store each
    if (lane * EPL + EPL <= S && ((ray * S) % EPL) == 0) {
        if constexpr (EPL == 4) {
            *reinterpret_cast<f32x4*>(a.w + ray * S + lane * 4) = f32x4{wv[0], wv[1], wv[2], wv[3]};
            *reinterpret_cast<f32x4*>(a.T + ray * S + lane * 4) = f32x4{tv[0], tv[1], tv[2], tv[3]};
        } else {
#pragma unroll
            for (int j = 0; j < EPL; ++j) {
                a.w[ray * S + lane * EPL + j] = wv[j];
                a.T[ray * S + lane * EPL + j] = tv[j];
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
            const int e = lane * EPL + j;
            if (e < S) {
                a.w[ray * S + e] = wv[j];
                a.T[ray * S + e] = tv[j];
            }
        }
    }
    dsum = wave_sum(dsum);
    if (lane == 0) a.depth[ray] = dsum;
    if (a.weights_only) return;
    c0 = wave_sum(c0);
    c1 = wave_sum(c1);
    c2 = wave_sum(c2);
    if (lane == 0) {
        a.rgb[ray * 3 + 0] = fminf(fmaxf(c0, 0.f), 1.f);
        a.rgb[ray * 3 + 1] = fminf(fmaxf(c1, 0.f), 1.f);
        a.rgb[ray * 3 + 2] = fminf(fmaxf(c2, 0.f), 1.f);
    }
    for (int c = 0; c < a.n_sem; ++c) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
            const int e = lane * EPL + j;
            if (e < S) s += rows[e * NO + a.sem_col + c];
        }
        s = wave_sum(s);
        if (lane == 0) a.sem[ray * a.n_sem + c] = s / (float)S;
    }
}

template <int EPL>
__global__ __launch_bounds__(256) void k_composite_bwd(CompArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sh_rows[];
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (ray >= a.B) return;  // wave-uniform; wave-private LDS slices
    const int S = a.S, NO = a.NO;
    float* rows = sh_rows + (threadIdx.x >> 6) * (2 * S * NO);
    float* drows = rows + S * NO;   // the ray's d_out block, assembled here and stored whole
    const bool col = !a.weights_only;
    if (col) {
        stage_rows(a.out + ray * (int64_t)(S * NO), rows, S * NO, lane);
    } else {
        for (int e = lane; e < S; e += 64) rows[e * NO + 3] = a.out[(ray * S + e) * NO + 3];
        wave_lds_sync();
    }
    for (int i = lane; i < S * NO; i += 64) drows[i] = 0.f;
    RayState<EPL> st;
    march<EPL>(a, ray, lane, rows, st);
    // clamp mask of rgb = clamp(Σ w·albedo·irr, 0, 1) (recomputed pre-clamp value)
    float gp[3] = {0.f, 0.f, 0.f};
    if (col && a.g_rgb) {
        float c[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < EPL; ++j) {
            const int e = lane * EPL + j;
            if (e >= S) continue;
            const float* o = rows + e * NO;
            const float sun = o[4], om = 1.f - sun;
            for (int q = 0; q < 3; ++q) c[q] += (st.w[j] * o[q]) * (sun + om * o[5 + q]);
        }
        for (int q = 0; q < 3; ++q) {
            const float v = wave_sum(c[q]);
            const float g = a.g_rgb[ray * 3 + q];
            gp[q] = (v >= 0.f && v <= 1.f) ? g : 0.f;
        }
    }
    const float gd = a.g_depth ? a.g_depth[ray] : 0.f;
    float dal[EPL], q[EPL];
    wave_lds_sync();   // the zero fill of drows is complete
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        dal[j] = 0.f;
        q[j] = 0.f;
        if (e >= S) continue;
        const int64_t p = ray * S + e;
        float* dO = drows + e * NO;
        float dw = gd * st.z[j] + (a.g_w ? a.g_w[p] : 0.f);
        if (col) {
            const float* o = rows + e * NO;
            const float sun = o[4], om = 1.f - sun;
            float dsun = 0.f, dsun2 = 0.f;
            for (int c = 0; c < 3; ++c) {
                const float sky = o[5 + c];
                const float irr = sun + om * sky;
                const float du = gp[c] * irr;
                dw += du * o[c];
                dO[c] = du * st.w[j];
                const float dirr = gp[c] * (st.w[j] * o[c]);
                dsun += dirr;
                dsun2 += dirr * sky;
                dO[5 + c] = dirr * om;
            }
            dO[4] = dsun - dsun2;
        }
        if (col && a.g_sem)
            for (int c = 0; c < a.n_sem; ++c) dO[a.sem_col + c] = a.g_sem[ray * a.n_sem + c] / (float)S;
        if (!col && a.g_sun) dO[4] = a.g_sun[p];
        const float dT = dw * st.al[j] + (a.g_T ? a.g_T[p] : 0.f);
        dal[j] = dw * st.T[j];
        q[j] = st.T[j] * dT;
    }
    // reversed cumsum R_e = Σ_{j≥e} q_j (double accumulation like torch's CPU cumsum)
    double suf[EPL];
    double run = 0.0;
#pragma unroll
    for (int j = EPL - 1; j >= 0; --j) {
        run += (double)q[j];
        suf[j] = run;
    }
    const double incl = wave_suffix_add(run, lane);
    double nxt = __shfl_down(incl, 1, 64);
    if (lane == 63) nxt = 0.0;
    float R[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) R[j] = (float)(suf[j] + nxt);
    const float Rn0 = __shfl_down(R[0], 1, 64);
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
        const int e = lane * EPL + j;
        if (e >= S) continue;
        const float Rnext = e == S - 1 ? 0.f : (j + 1 < EPL ? R[j + 1] : Rn0);
        const float dt = Rnext / st.t[j];
        const float da = dal[j] - dt;
        const float dX = (-da) * st.E[j];
        const float dr = dX * (-st.dl[j]);
        drows[e * NO + 3] = st.r[j] > 0.f ? dr : 0.f;
    }
    wave_lds_sync();
    float* dst = a.d_out + ray * (int64_t)(S * NO);
    const int n = S * NO;
    if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int i = lane; i < n / 4; i += 64) reinterpret_cast<f32x4*>(dst)[i] = reinterpret_cast<const f32x4*>(drows)[i];
    } else {
        for (int i = lane; i < n; i += 64) dst[i] = drows[i];
    }
}

template <int EPL>
static int32_t launch_comp(const CompArgs& a, bool fwd, hipStream_t s) {
    // 4 waves (rays) per block, fewer when their LDS row blocks would not fit
    const size_t per_wave = (size_t)(fwd ? 1 : 2) * a.S * a.NO * sizeof(float);
    const int wpb = per_wave * 4 <= 64 * 1024 ? 4 : 1;
    const dim3 grid((unsigned)((a.B + wpb - 1) / wpb)), block(64 * wpb);
    const size_t lds = per_wave * wpb;
    if (fwd) hipLaunchKernelGGL(k_composite_fwd<EPL>, grid, block, lds, s, a);
    else hipLaunchKernelGGL(k_composite_bwd<EPL>, grid, block, lds, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

static int32_t run_comp(const CompArgs& a, bool fwd, hipStream_t s) {
    SPN_ARG(a.S > 0 && a.S <= 256, "composite: n_samples %d must be in [1, 256]", a.S);
    SPN_ARG(a.NO >= 8 && a.sem_col + a.n_sem <= a.NO, "composite: bad output layout");
    SPN_ARG((size_t)2 * a.S * a.NO * sizeof(float) <= 64 * 1024, "composite: n_samples x n_out = %d x %d too large", a.S,
            a.NO);
    if (a.B == 0) return SPNERF_OK;
    const double P = (double)a.B * a.S;
    ProfScope prof(fwd ? "composite_fwd" : "composite_bwd", s, 0.0,
                   fwd ? P * (a.weights_only ? 16.0 : 44.0) + a.B * 16.0 : P * (a.NO * 8.0 + 24.0));
    if (a.S <= 64) return launch_comp<1>(a, fwd, s);
    if (a.S <= 128) return launch_comp<2>(a, fwd, s);
    return launch_comp<4>(a, fwd, s);
}

}  // namespace spn

using namespace spn;

extern "C" int32_t spnerf_composite_forward(int64_t n_rays, int32_t n_samples, const float* z, const float* out,
                                            int32_t n_out, const float* noise, float noise_std, int32_t sem_col,
                                            int32_t n_sem, int32_t flags, float* rgb, float* depth, float* weights,
                                            float* transparency, float* sem_logits, const spnerf_rng* rng, void* stream) {
    const bool wo = flags & SPNERF_COMP_WEIGHTS_ONLY;
    SPN_ARG(z && out && depth && weights && transparency, "composite_forward: NULL pointer");
    SPN_ARG(wo || rgb, "composite_forward: rgb is NULL");
    SPN_ARG(wo || n_sem == 0 || sem_logits, "composite_forward: sem_logits is NULL");
    CompArgs a{};
    a.B = n_rays; a.S = n_samples; a.NO = n_out; a.sem_col = sem_col; a.n_sem = wo ? 0 : n_sem; a.weights_only = wo;
    a.z = z; a.out = out; a.noise = noise; a.noise_std = noise_std;
    if (!noise && rng && noise_std != 0.f) a.rng = *rng;
    a.rgb = rgb; a.depth = depth; a.w = weights; a.T = transparency; a.sem = sem_logits;
    if (flags & SPNERF_COMP_SUN_COLUMN) {
        SPN_ARG(wo && rgb, "composite_forward: SPNERF_COMP_SUN_COLUMN needs SPNERF_COMP_WEIGHTS_ONLY and rgb");
        a.sun_out = rgb;
        a.rgb = nullptr;
    }
    return run_comp(a, true, (hipStream_t)stream);
}

extern "C" int32_t spnerf_composite_backward(int64_t n_rays, int32_t n_samples, const float* z, const float* out,
                                             int32_t n_out, const float* noise, float noise_std, int32_t sem_col,
                                             int32_t n_sem, int32_t flags, const float* g_rgb, const float* g_depth,
                                             const float* g_weights, const float* g_transparency, const float* g_sem,
                                             float* d_out, const spnerf_rng* rng, void* stream) {
    const bool wo = flags & SPNERF_COMP_WEIGHTS_ONLY;
    SPN_ARG(z && out && d_out, "composite_backward: NULL pointer");
    CompArgs a{};
    a.B = n_rays; a.S = n_samples; a.NO = n_out; a.sem_col = sem_col; a.n_sem = wo ? 0 : n_sem; a.weights_only = wo;
    a.z = z; a.out = out; a.noise = noise; a.noise_std = noise_std;
    if (!noise && rng && noise_std != 0.f) a.rng = *rng;
    a.g_rgb = g_rgb; a.g_depth = g_depth; a.g_w = g_weights; a.g_T = g_transparency; a.g_sem = g_sem;
    a.d_out = d_out;
    if (flags & SPNERF_COMP_SUN_COLUMN) {
        SPN_ARG(wo, "composite_backward: SPNERF_COMP_SUN_COLUMN needs SPNERF_COMP_WEIGHTS_ONLY");
        a.g_sun = g_rgb;
        a.g_rgb = nullptr;
    }
    return run_comp(a, false, (hipStream_t)stream);
}
