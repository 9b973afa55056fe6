// Adam over a list of fp32 parameter tensors in one launch (the optimizer step of the training
// loop, reference main.py:97: torch.optim.Adam(parameters, lr, weight_decay=0), default betas / eps).
// torch's fused multi-tensor Adam took ~100 us per C2 step for 2.7 M parameters (0.75 TB/s):
// here every block owns 4096 consecutive elements of one tensor (found by a binary search over
// the per-tensor block prefix held in the kernel arguments), each thread 4 x float4.
#include <cmath>

#include "common.h"

namespace spn {

constexpr int kAdamSeg = 48;           // tensors per launch (kernel-argument budget)
constexpr int kAdamChunk = 256 * 16;   // elements per block

struct AdamSeg {
    float* p;
    const float* g;
    float* m;
    float* v;
    int64_t n;
};
struct AdamArgs {
    AdamSeg s[kAdamSeg];
    int64_t first_block[kAdamSeg + 1];  // prefix of per-tensor block counts
    int nseg;
    float w1, beta2, w2, eps, step_size, bc2_sqrt;  // w = 1 - beta, rounded from double like torch's scalars
};

// torch's single-tensor Adam arithmetic (torch/optim/adam.py _single_tensor_adam):
// m.lerp_(g, 1-b1); v = v*b2 + (1-b2)*g*g; p -= step_size * m / (sqrt(v)/sqrt(bc2) + eps)
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, const AdamArgs& a) {
    const float w = a.w1;
    m = w < 0.5f ? m + w * (g - m) : g - (g - m) * (1.f - w);
    v = v * a.beta2 + (a.w2 * g) * g;
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    p = p + (-a.step_size) * (m / denom);
}

__global__ __launch_bounds__(256) void k_adam(AdamArgs a) {
    typedef const __attribute__((address_space(4))) AdamArgs* KArgs;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    const int64_t b = blockIdx.x;
    int lo = 0, hi = a.nseg - 1;  // last segment with first_block <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ka->first_block[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const AdamSeg sg{ka->s[lo].p, ka->s[lo].g, ka->s[lo].m, ka->s[lo].v, ka->s[lo].n};  // scalar loads
    const int64_t base = (b - ka->first_block[lo]) * kAdamChunk;
    const bool vec = ((reinterpret_cast<uintptr_t>(sg.p) | reinterpret_cast<uintptr_t>(sg.g) |
                       reinterpret_cast<uintptr_t>(sg.m) | reinterpret_cast<uintptr_t>(sg.v)) & 15) == 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t i = base + (int64_t)(q * 256 + threadIdx.x) * 4;
        if (vec && i + 3 < sg.n) {
            f32x4 p = ld4(sg.p + i), g = ld4(sg.g + i), m = ld4(sg.m + i), v = ld4(sg.v + i);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float pe = p[e], me = m[e], ve = v[e];
                adam1(pe, g[e], me, ve, a);
                p[e] = pe;
                m[e] = me;
                v[e] = ve;
            }
            st4(sg.p + i, p);
            st4(sg.m + i, m);
            st4(sg.v + i, v);
        } else {
            for (int64_t j = i; j < i + 4 && j < sg.n; ++j) {
                float p = sg.p[j], m = sg.m[j], v = sg.v[j];
                adam1(p, sg.g[j], m, v, a);
                sg.p[j] = p;
                sg.m[j] = m;
                sg.v[j] = v;
            }
        }
    }
}

}  // namespace spn

using namespace spn;

extern "C" int32_t spnerf_adam_step(int32_t n, void* const* params, const void* const* grads, void* const* exp_avg,
                                    void* const* exp_avg_sq, const int64_t* numel, double lr, double beta1, double beta2,
                                    double eps, int32_t step, void* stream) {
    SPN_ARG(n >= 0 && (n == 0 || (params && grads && exp_avg && exp_avg_sq && numel)), "adam_step: bad lists");
    SPN_ARG(step >= 1 && lr >= 0.0 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps > 0.0,
            "adam_step: bad hyper-parameters");
    hipStream_t s = (hipStream_t)stream;
    const double bc1 = 1.0 - std::pow(beta1, step), bc2 = 1.0 - std::pow(beta2, step);
    for (int i = 0; i < n;) {
        AdamArgs a{};
        a.w1 = (float)(1.0 - beta1);
        a.beta2 = (float)beta2;
        a.w2 = (float)(1.0 - beta2);
        a.eps = (float)eps;
        a.step_size = (float)(lr / bc1);
        a.bc2_sqrt = (float)std::sqrt(bc2);
        int64_t blocks = 0;
        for (; i < n && a.nseg < kAdamSeg; ++i) {
            SPN_ARG(numel[i] >= 0, "adam_step: tensor %d has negative size", i);
            if (numel[i] == 0) continue;
            a.s[a.nseg] = AdamSeg{(float*)params[i], (const float*)grads[i], (float*)exp_avg[i], (float*)exp_avg_sq[i],
                                  numel[i]};
            a.first_block[a.nseg] = blocks;
            blocks += (numel[i] + kAdamChunk - 1) / kAdamChunk;
            ++a.nseg;
        }
        a.first_block[a.nseg] = blocks;
        if (blocks == 0) continue;
        SPN_ARG(blocks < (1ll << 31), "adam_step: too many elements");
        ProfScope prof("adam", s, 0.0, 0.0);
        hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(256), 0, s, a);
        SPN_HIP(hipGetLastError());
    }
    return SPNERF_OK;
}
