// Wavefront (64-lane) scan / reduce / sort helpers for the per-ray kernels.
#pragma once
#include "common.h"

namespace spn {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// inclusive prefix product / sum over lanes 0..63 (T = float or double: torch's CPU cumsum /
// cumprod accumulate in double, at::acc_type<float, false>)
template <typename T>
__device__ __forceinline__ T wave_scan_mul(T v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T t = __shfl_up(v, off, 64);
        if (lane >= off) v *= t;
    }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_scan_add(T v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}
// inclusive suffix sum over lanes (lane i gets Σ_{j >= i})
template <typename T>
__device__ __forceinline__ T wave_suffix_add(T v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const T t = __shfl_down(v, off, 64);
        if (lane + off < 64) v += t;
    }
    return v;
}

// torch.sort ordering on floats: NaN sorts last
__device__ __forceinline__ bool fless(float a, float b) { return a < b || (b != b && a == a); }

// In-place ascending bitonic sort of s[0..n) (n a power of two ≤ 256) by the 64 lanes of one
// wave; `sync` is called between dependent steps (a block barrier when several waves share a
// block, so every wave must call this with the same n).
template <typename Sync>
__device__ void wave_bitonic_sort(float* s, int n, int lane, Sync sync) {
    for (int k = 2; k <= n; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int e = lane; e < n; e += 64) {
                const int q = e ^ j;
                if (q > e) {
                    const float a = s[e], b = s[q];
                    const bool up = (e & k) == 0;
                    if (up ? fless(b, a) : fless(a, b)) {
                        s[e] = b;
                        s[q] = a;
                    }
                }
            }
            sync();
        }
    }
}

// torch.linspace(start, end, steps)[i] with ATen's CPU formula (two halves, RangeFactories)
__device__ __forceinline__ float linspace_at(float start, float end, int steps, int i) {
    if (steps == 1) return start;
    const float step = (end - start) / (float)(steps - 1);
    return i < steps / 2 ? __fadd_rn(start, __fmul_rn(step, (float)i))
                         : __fsub_rn(end, __fmul_rn(step, (float)(steps - 1 - i)));
}

}  // namespace spn
