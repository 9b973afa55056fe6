// Shared host/device helpers of the SP-NeRF gfx950 library.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/spnerf_amd.h"

namespace spn {

// ---- errors (thread-local last-error text, see spnerf_last_error) -------------------------
void set_error(const char* fmt, ...);

#define SPN_ARG(cond, ...)                 \
    do {                                   \
        if (!(cond)) {                     \
            ::spn::set_error(__VA_ARGS__); \
            return SPNERF_E_ARG;           \
        }                                  \
    } while (0)

#define SPN_HIP(call)                                                                   \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            ::spn::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),      \
                             __FILE__, __LINE__);                                       \
            return SPNERF_E_HIP;                                                        \
        }                                                                               \
    } while (0)

#define SPN_TRY(expr)              \
    do {                           \
        int32_t rc_ = (expr);      \
        if (rc_ != SPNERF_OK)      \
            return rc_;            \
    } while (0)

// ---- profiling: HIP events around each launch of a kernel class, on the launch stream ----
// compute units of the current device (hipDeviceProp_t::multiProcessorCount, cached per device):
// the resident grid of the persistent kernels
int num_cus();
// CU count the weight-gradient split counts are sized for: the workspace layout sizes its slabs
// for kLayoutCus (a pure function of the model dimensions, whatever device is current), and a
// launch never uses more splits than that (split_cus: the device's CUs, capped at kLayoutCus)
constexpr int kLayoutCus = 256;
// Profiling-ablation arguments of the kernels (dbg, nt) vary only in a -DSPN_ABLATIONS build; the
// product build folds them to their defaults, so no runtime flag branches a hot loop
#ifdef SPN_ABLATIONS
constexpr bool kAblBuild = true;
#else
constexpr bool kAblBuild = false;
#endif
inline int split_cus() {
    const int n = num_cus();
    return n < kLayoutCus ? n : kLayoutCus;
}

// option prof_shapes: each launch's class is keyed by its FLOP count too ("class#<MFLOP>"), so
// the in-library timer separates the launch shapes of one kernel function
extern int g_prof_shapes;
struct ProfScope {
    ProfScope(const char* cls, hipStream_t s, double flop, double bytes);
    ~ProfScope();
    void* rec_;
    hipStream_t s_;
};

// ---- small device helpers -----------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef __bf16 bf16;
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__host__ __device__ inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// 4 consecutive activations as fp32 (the MLP keeps activations in fp32 or bf16, cfg.dtype)
__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 ld4(const bf16* p) {
    const u32x2 v = *reinterpret_cast<const u32x2*>(p);
    return f32x4{__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u), __uint_as_float(v[1] << 16),
                 __uint_as_float(v[1] & 0xffff0000u)};
}
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void st4(bf16* p, f32x4 v) {
    const __bf16 a = (__bf16)v[0], b = (__bf16)v[1], c = (__bf16)v[2], d = (__bf16)v[3];
    *reinterpret_cast<u32x2*>(p) =
        u32x2{(uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16),
              (uint32_t)__builtin_bit_cast(uint16_t, c) | ((uint32_t)__builtin_bit_cast(uint16_t, d) << 16)};
}
__device__ __forceinline__ float ld1(const float* p) { return *p; }
__device__ __forceinline__ float ld1(const bf16* p) { return (float)*p; }

// ---- 8-wide bf16 rows, fast sin/cos, wave-local LDS ordering (bf16 GEMM epilogues) --------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldg16(const bf16* p) { return *reinterpret_cast<const u32x4*>(p); }

__device__ __forceinline__ void unpack8(u32x4 v, float (&f)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(v[i] << 16);
        f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
    }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 (round to nearest even): one v_cvt_pk_bf16_f32 (converting the
// scalars separately costs a convert, a shift and an or per pair)
__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
    return u32x4{pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7])};
}

// sin / cos for bf16 outputs: the hardware v_sin_f32 / v_cos_f32 on the argument in revolutions,
// as LLVM lowers native sin for gfx9 (whose sine unit reduces the full input range itself: no
// v_fract, unlike GCN1-3).  Absolute error ~1e-6 for |x| < 1e3, far below the bf16 rounding of
// the result (2^-9 relative).
#ifndef SPN_PK_EPI
#define SPN_PK_EPI 1  // sine epilogues: (acc + b [+ row]) · 1/2π as packed fp32 pairs (0: scalar, A/B builds)
#endif
__device__ __forceinline__ float revs(float x) { return x * 0.15915494309189535f; }
__device__ __forceinline__ void fast_sincos(float x, float* s, float* c) {
    const float r = revs(x);
    *s = __builtin_amdgcn_sinf(r);
    *c = __builtin_amdgcn_cosf(r);
}

// the sine / cosine halves of fast_sincos (bit-identical results)
__device__ __forceinline__ float fast_sin(float x) { return __builtin_amdgcn_sinf(revs(x)); }
__device__ __forceinline__ float fast_cos(float x) { return __builtin_amdgcn_cosf(revs(x)); }

// The saved pre-activation Z of a bf16 trunk layer is stored as fp16 (11-bit significand: 4x
// finer than bf16 at the same 2 bytes; hidden-layer |Z| is O(1), far inside fp16's range), and
// the layer computes H = sin(Z), D = cos(Z) from that rounded Z, so every consumer recomputes
// them bit-identically.  zr16: x rounded to fp16 and back.
__device__ __forceinline__ float zr16(float x) { return (float)(_Float16)x; }
__device__ __forceinline__ uint32_t pack2_f16(float lo, float hi) {
    const _Float16 a = (_Float16)lo, b = (_Float16)hi;
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}
__device__ __forceinline__ u32x4 pack8_f16(const float (&f)[8]) {
    return u32x4{pack2_f16(f[0], f[1]), pack2_f16(f[2], f[3]), pack2_f16(f[4], f[5]), pack2_f16(f[6], f[7])};
}
__device__ __forceinline__ void unpack8_f16(u32x4 v, float (&f)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = (float)__builtin_bit_cast(_Float16, (uint16_t)(v[i] & 0xffffu));
        f[2 * i + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(v[i] >> 16));
    }
}
// 8 saved Z (fp16) -> 8 bf16 sin(Z): the H a saved-Z trunk layer stands for
__device__ __forceinline__ u32x4 sin8_z(u32x4 v) {
    float f[8];
    unpack8_f16(v, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fast_sin(f[e]);
    return pack8(f);
}

// a copy of x the compiler cannot see through: lane-derived addresses computed from it are
// recomputed where used instead of being hoisted out of every loop and kept live across the
// MFMA main loop (where the accumulators need the registers)
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

// order LDS accesses of one wavefront (LDS is in order per wave; this stops the compiler
// from moving accesses across the point)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Bijective XCD-aware remap of a 1-D grid: blocks b and b+8 share an XCD (round-robin
// dispatch), so hand each XCD a contiguous run of tiles (cdna_hip_programming.md T1).
__device__ __forceinline__ int xcd_remap(int id, int nb) {
    const int xcd = id & 7, loc = id >> 3;
    const int q = nb >> 3, r = nb & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// ---- on-device draws: Philox4x32-10 keyed by (seed, step, ray, slot, index) (spnerf_rng) ----
__device__ __forceinline__ void philox_round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t hi0 = __umulhi(M0, c[0]), lo0 = M0 * c[0];
    const uint32_t hi1 = __umulhi(M1, c[2]), lo1 = M1 * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k[0], n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}
// the four 32-bit words of draw `idx` of ray `ray` in `slot`
__device__ __forceinline__ void philox_words(const spnerf_rng& r, int64_t ray, int idx, uint32_t (&c)[4]) {
    const uint64_t seed = (uint64_t)r.state[0], step = (uint64_t)r.state[1];
    const uint64_t id = (uint64_t)(r.ray0 + ray);
    c[0] = (uint32_t)id; c[1] = (uint32_t)(id >> 32);
    c[2] = ((uint32_t)r.slot << 16) | (uint32_t)idx; c[3] = (uint32_t)step;
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(step >> 32)};
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        philox_round(c, k);
        k[0] += 0x9E3779B9u;
        k[1] += 0xBB67AE85u;
    }
}
// uniform in [0, 1) with 24 random bits (torch's float uniform resolution)
__device__ __forceinline__ float rng_uniform(const spnerf_rng& r, int64_t ray, int idx) {
    uint32_t c[4];
    philox_words(r, ray, idx, c);
    return (float)(c[0] >> 8) * (1.0f / 16777216.0f);
}
// standard normal (Box–Muller of two words; u1 in (0, 1])
__device__ __forceinline__ float rng_normal(const spnerf_rng& r, int64_t ray, int idx) {
    uint32_t c[4];
    philox_words(r, ray, idx, c);
    const float u1 = (float)((c[1] >> 8) + 1u) * (1.0f / 16777216.0f);
    const float u2 = (float)(c[2] >> 8) * (1.0f / 16777216.0f);
    return sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795865f * u2);
}

// torch-compatible elementwise pieces (ATen CPU formulas)
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float softplusf_(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float softplus_grad(float g, float x) {
    if (x > 20.0f) return g;
    const float z = expf(x);
    return g * z / (z + 1.0f);
}

}  // namespace spn
