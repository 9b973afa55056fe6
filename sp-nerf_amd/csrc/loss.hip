// The training step's losses over the render dictionary (reference modules/metrics.py, as the
// trainer combines them in main.py:125-174) and their gradients, in two small kernels instead of
// ~60 ATen launches:
//   colour   SNerfLoss            mean((rgb - t)^2)                                :27-45
//   solar    solar_correction     λ_sc/3 · mean_r Σ_s (T_sc - sun)^2                :17-24
//                                 λ_sc/3 · mean_r (1 - Σ_s w_sc · sun)   (T_sc, w_sc detached)
//   depth    DepthLoss subset MSE λ_ds/3 · Σ_{valid ∧ outside} tw (d - td)^2 / B   :82-132,151-153
//            (outside = |d - td| > σ_t  or  sqrt(Σ w (z - d)^2) > σ_t, :78-80; no gradient
//             through that selection)
//   semantic SemanticLoss         λ_ss · Σ_{label ≠ -100} nll / n_valid            :162-183
// Data parallelism (no reference counterpart): the CE mean runs over the GLOBAL batch's valid
// labels (denominator n_valid_global / world), so the ranks' losses average to the global one.
// Labels: -100 is ignored; any other label outside [0, C) — where torch's CrossEntropyLoss raises
// (a device-side assert on the GPU) — makes the loss, its CE term and that ray's logit gradients
// NaN (no host synchronisation; a graph-captured step cannot raise).  A global batch without a
// valid label gives a NaN CE term as torch's mean over zero elements does, and zero logit
// gradients.
//
// k_loss_rays: one wavefront per ray (S ≤ 256 samples, 4 per lane), a block of 4 waves walks a
// fixed ray range and writes its partial sums — fixed order, deterministic.  k_loss_final: one
// block adds the partials in block order, counts the global valid labels, writes the loss (and
// its terms).  k_loss_grad: the upstream gradients × dL (device scalar), one wavefront per ray.
#include "common.h"
#include "wave.h"

namespace spn {

struct LossArgs {
    int64_t B;
    int S, C;
    const float *rgb, *target;                  // (B,3)
    float lambda_sc;
    const float* sun_sc; int ld_sun;            // sun_sc[ray*S + s] at stride ld_sun (a view of out)
    const float *T_sc, *w_sc;                   // (B,S)
    float lambda_ds;
    const float *depth, *z, *w;                 // (B), (B,S), (B,S)
    const float* tdepth; int ld_td;             // target depth / weight columns (stride ld_td)
    const float* tweight;
    const int64_t* valid;                       // (B) int64 (> 0 = prior)
    const float* tstd;                          // (B)
    float lambda_ss;
    const float* logits;                        // (B,C)
    const int64_t* labels;                      // (B)
    const int64_t* labels_global; int64_t n_global; int world;
    float* partial;                             // [nblocks][8]
    int nblocks;
    float* result;                              // [0] loss, [1..5] terms, [6] CE denominator
    const float* g;                             // dL (device scalar) for the gradients
    float *d_rgb, *d_sun, *d_depth, *d_logits;  // (B,3), (B,S), (B), (B,C)
};

constexpr int kLossWaves = 4;
constexpr int kLossParts = 6;  // colour, sc2, sc3, depth, nll sum, out-of-range labels

// per-ray quantities shared by the loss and its gradient
struct RayLoss {
    float col, sc2, sc3, dep, nll, bad;
    bool apply;
};

__device__ __forceinline__ RayLoss ray_loss(const LossArgs& a, int64_t r, int lane, float* sm_logit) {
    RayLoss o{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, false};
    if (a.rgb) {
        float c = 0.f;
        if (lane < 3) {
            const float d = a.rgb[r * 3 + lane] - a.target[r * 3 + lane];
            c = d * d;
        }
        o.col = wave_sum(c);
    }
    if (a.lambda_sc > 0.f) {
        float s2 = 0.f, s3 = 0.f;
        for (int s = lane; s < a.S; s += 64) {
            const float sun = a.sun_sc[(r * a.S + s) * (int64_t)a.ld_sun];
            const float dt = a.T_sc[r * a.S + s] - sun;
            s2 += dt * dt;
            s3 += a.w_sc[r * a.S + s] * sun;
        }
        o.sc2 = wave_sum(s2);
        o.sc3 = 1.f - wave_sum(s3);
    }
    if (a.lambda_ds > 0.f) {
        const float d = a.depth[r];
        float v = 0.f;
        for (int s = lane; s < a.S; s += 64) {
            const float e = a.z[r * a.S + s] - d;
            v += e * e * a.w[r * a.S + s];
        }
        const float pstd = sqrtf(wave_sum(v));
        const float td = a.tdepth[r * a.ld_td], ts = a.tstd[r];
        const float diff = d - td;
        o.apply = a.valid[r] > 0 && (fabsf(diff) > ts || pstd > ts);
        o.dep = o.apply ? a.tweight[r * a.ld_td] * diff * diff : 0.f;
    }
    if (a.logits) {
        const int64_t lab = a.labels[r];
        if (lab != -100 && (lab < 0 || lab >= a.C)) o.bad = 1.f;
        if (lab != -100) {
            // log-softmax over C classes (lane c holds logit c; C ≤ 64)
            const float x = lane < a.C ? a.logits[r * a.C + lane] : -INFINITY;
            float m = x;
            for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
            const float lse = m + logf(wave_sum(lane < a.C ? expf(x - m) : 0.f));
            const float xl = __shfl(x, (int)min<int64_t>(max<int64_t>(lab, 0), a.C - 1), 64);
            o.nll = lse - xl;
            if (sm_logit) *sm_logit = lane < a.C ? expf(x - lse) : 0.f;
        }
    }
    return o;
}

__global__ __launch_bounds__(64 * kLossWaves) void k_loss_rays(LossArgs a) {
    __shared__ float part[kLossWaves][kLossParts];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t per = (a.B + a.nblocks - 1) / a.nblocks;
    const int64_t r0 = blockIdx.x * per, r1 = min(a.B, r0 + per);
    float acc[kLossParts] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t r = r0 + wv; r < r1; r += kLossWaves) {
        const RayLoss o = ray_loss(a, r, lane, nullptr);
        acc[0] += o.col; acc[1] += o.sc2; acc[2] += o.sc3; acc[3] += o.dep; acc[4] += o.nll; acc[5] += o.bad;
    }
    if (lane == 0)
        for (int k = 0; k < kLossParts; ++k) part[wv][k] = acc[k];
    __syncthreads();
    if (threadIdx.x < kLossParts) {
        float s = 0.f;
        for (int v = 0; v < kLossWaves; ++v) s += part[v][threadIdx.x];
        a.partial[blockIdx.x * 8 + threadIdx.x] = s;
    }
}

__global__ __launch_bounds__(256) void k_loss_final(LossArgs a) {
    __shared__ float red[kLossParts + 1][256];
    const int t = threadIdx.x;
    float s[kLossParts] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int b = t; b < a.nblocks; b += 256)
        for (int k = 0; k < kLossParts; ++k) s[k] += a.partial[b * 8 + k];
    float nv = 0.f;
    if (a.logits)
        for (int64_t i = t; i < a.n_global; i += 256) nv += a.labels_global[i] != -100 ? 1.f : 0.f;
    for (int k = 0; k < kLossParts; ++k) red[k][t] = s[k];
    red[kLossParts][t] = nv;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (t < st)
            for (int k = 0; k <= kLossParts; ++k) red[k][t] += red[k][t + st];
        __syncthreads();
    }
    if (t == 0) {
        const float B = (float)a.B;
        const float col = a.rgb ? red[0][0] / (3.f * B) : 0.f;
        const float sc2 = a.lambda_sc > 0.f ? a.lambda_sc / 3.f * (red[1][0] / B) : 0.f;
        const float sc3 = a.lambda_sc > 0.f ? a.lambda_sc / 3.f * (red[2][0] / B) : 0.f;
        const float dep = a.lambda_ds > 0.f ? a.lambda_ds / 3.f * red[3][0] / B : 0.f;
        // CE mean over the global batch's valid labels, per rank: Σ nll / (n_valid_global / world)
        const float den = red[kLossParts][0] / (float)a.world;
        float ce = 0.f;
        if (a.logits) ce = (den > 0.f && red[5][0] == 0.f) ? a.lambda_ss * (red[4][0] / den) : NAN;
        a.result[1] = col; a.result[2] = sc2; a.result[3] = sc3; a.result[4] = dep; a.result[5] = ce;
        a.result[6] = den;
        a.result[0] = (((col + sc2) + sc3) + dep) + ce;
    }
}

__global__ __launch_bounds__(64 * kLossWaves) void k_loss_grad(LossArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * kLossWaves + (threadIdx.x >> 6);
    if (r >= a.B) return;  // wave-uniform
    const float g = *a.g, B = (float)a.B;
    float sm = 0.f;
    const RayLoss o = ray_loss(a, r, lane, a.logits ? &sm : nullptr);
    if (a.rgb && lane < 3)
        a.d_rgb[r * 3 + lane] = g * (2.f * (a.rgb[r * 3 + lane] - a.target[r * 3 + lane]) / (3.f * B));
    if (a.lambda_sc > 0.f) {
        const float k = g * (a.lambda_sc / 3.f) / B;
        for (int s = lane; s < a.S; s += 64) {
            const float sun = a.sun_sc[(r * a.S + s) * (int64_t)a.ld_sun];
            a.d_sun[r * a.S + s] = k * (-2.f * (a.T_sc[r * a.S + s] - sun) - a.w_sc[r * a.S + s]);
        }
    }
    if (a.lambda_ds > 0.f && lane == 0)
        a.d_depth[r] = o.apply ? g * (a.lambda_ds / 3.f) * 2.f * a.tweight[r * a.ld_td] * (a.depth[r] - a.tdepth[r * a.ld_td]) / B
                               : 0.f;
    if (a.logits && lane < a.C) {
        const int64_t lab = a.labels[r];
        const float den = a.result[6];
        float d = 0.f;
        if (o.bad != 0.f) d = NAN;
        else if (lab != -100 && den > 0.f) d = g * a.lambda_ss * (sm - (lane == lab ? 1.f : 0.f)) / den;
        a.d_logits[r * a.C + lane] = d;
    }
}

}  // namespace spn

using namespace spn;

static int32_t loss_check(const LossArgs& a) {
    SPN_ARG(a.B > 0 && a.S > 0 && a.S <= 4096, "render_loss: bad sizes B=%lld S=%d", (long long)a.B, a.S);
    SPN_ARG(a.partial && a.result && a.nblocks >= 1 && a.nblocks <= 4096, "render_loss: NULL workspace / loss_out");
    SPN_ARG(!a.rgb || a.target, "render_loss: rgb without target");
    SPN_ARG(a.lambda_sc <= 0.f || (a.sun_sc && a.T_sc && a.w_sc && a.ld_sun > 0), "render_loss: solar inputs");
    SPN_ARG(a.lambda_ds <= 0.f || (a.depth && a.z && a.w && a.tdepth && a.tweight && a.valid && a.tstd), "render_loss: depth inputs");
    SPN_ARG(!a.logits || (a.labels && a.labels_global && a.C >= 1 && a.C <= 64 && a.world >= 1), "render_loss: semantic inputs");
    return SPNERF_OK;
}

static LossArgs loss_args(int64_t n_rays, int32_t n_samples, int32_t n_classes, const float* rgb, const float* target,
                          float lambda_sc, const float* sun_sc, int32_t ld_sun, const float* T_sc, const float* w_sc,
                          float lambda_ds, const float* depth, const float* z, const float* w, const float* tdepth,
                          const float* tweight, int32_t ld_td, const int64_t* valid, const float* tstd, float lambda_ss,
                          const float* logits, const int64_t* labels, const int64_t* labels_global, int64_t n_global,
                          int32_t world, float* workspace, int32_t nblocks) {
    LossArgs a{};
    a.B = n_rays; a.S = n_samples; a.C = n_classes;
    a.rgb = rgb; a.target = target;
    a.lambda_sc = sun_sc ? lambda_sc : 0.f; a.sun_sc = sun_sc; a.ld_sun = ld_sun; a.T_sc = T_sc; a.w_sc = w_sc;
    a.lambda_ds = depth ? lambda_ds : 0.f; a.depth = depth; a.z = z; a.w = w;
    a.tdepth = tdepth; a.tweight = tweight; a.ld_td = ld_td; a.valid = valid; a.tstd = tstd;
    a.lambda_ss = lambda_ss; a.logits = logits; a.labels = labels; a.labels_global = labels_global;
    a.n_global = n_global; a.world = world;
    a.nblocks = nblocks;
    a.partial = workspace;
    return a;
}

// a block of 4 waves per 4 rays (a wave per ray: the per-ray terms are a chain of dependent
// loads and wave sums, so 4 rays per wave took 18 us at any batch), at most 4096 blocks
static int loss_blocks(int64_t n_rays) { return (int)std::min<int64_t>(std::max<int64_t>((n_rays + 3) / 4, 1), 4096); }

extern "C" int64_t spnerf_render_loss_workspace_bytes(int64_t n_rays) {
    if (n_rays < 0) return -1;
    return 8 * (int64_t)loss_blocks(n_rays) * (int64_t)sizeof(float);
}

extern "C" int32_t spnerf_render_loss_forward(int64_t n_rays, int32_t n_samples, int32_t n_classes, const float* rgb,
                                             const float* target, float lambda_sc, const float* sun_sc, int32_t ld_sun,
                                             const float* T_sc, const float* w_sc, float lambda_ds, const float* depth,
                                             const float* z, const float* w, const float* tdepth, const float* tweight,
                                             int32_t ld_td, const int64_t* valid, const float* tstd, float lambda_ss,
                                             const float* logits, const int64_t* labels, const int64_t* labels_global,
                                             int64_t n_global, int32_t world, void* workspace, float* loss_out,
                                             void* stream) {
    const int nb = loss_blocks(n_rays);
    LossArgs a = loss_args(n_rays, n_samples, n_classes, rgb, target, lambda_sc, sun_sc, ld_sun, T_sc, w_sc, lambda_ds,
                           depth, z, w, tdepth, tweight, ld_td, valid, tstd, lambda_ss, logits, labels, labels_global,
                           n_global, world, (float*)workspace, nb);
    a.result = loss_out;  // [0] loss, [1..5] terms, [6] CE denominator (read back by the gradient)
    SPN_TRY(loss_check(a));
    hipStream_t s = (hipStream_t)stream;
    ProfScope prof("render_loss", s, 0.0, 0.0);
    hipLaunchKernelGGL(k_loss_rays, dim3(nb), dim3(64 * kLossWaves), 0, s, a);
    SPN_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(256), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_render_loss_backward(int64_t n_rays, int32_t n_samples, int32_t n_classes, const float* rgb,
                                              const float* target, float lambda_sc, const float* sun_sc, int32_t ld_sun,
                                              const float* T_sc, const float* w_sc, float lambda_ds, const float* depth,
                                              const float* z, const float* w, const float* tdepth, const float* tweight,
                                              int32_t ld_td, const int64_t* valid, const float* tstd, float lambda_ss,
                                              const float* logits, const int64_t* labels, const float* loss_out,
                                              const float* g_loss, float* d_rgb, float* d_sun, float* d_depth,
                                              float* d_logits, void* stream) {
    LossArgs a = loss_args(n_rays, n_samples, n_classes, rgb, target, lambda_sc, sun_sc, ld_sun, T_sc, w_sc, lambda_ds,
                           depth, z, w, tdepth, tweight, ld_td, valid, tstd, lambda_ss, logits, labels, labels, n_rays, 1,
                           const_cast<float*>(loss_out), 1);   // (the partials are not read here)
    a.result = const_cast<float*>(loss_out);
    SPN_TRY(loss_check(a));
    SPN_ARG(g_loss && (!rgb || d_rgb) && (a.lambda_sc <= 0.f || d_sun) && (a.lambda_ds <= 0.f || d_depth) &&
                (!logits || d_logits), "render_loss_backward: NULL gradient pointer");
    a.g = g_loss; a.d_rgb = d_rgb; a.d_sun = d_sun; a.d_depth = d_depth; a.d_logits = d_logits;
    hipStream_t s = (hipStream_t)stream;
    ProfScope prof("render_loss", s, 0.0, 0.0);
    hipLaunchKernelGGL(k_loss_grad, dim3((unsigned)((n_rays + kLossWaves - 1) / kLossWaves)), dim3(64 * kLossWaves), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}
