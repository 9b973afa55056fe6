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

// torch-compatible elementwise pieces (ATen CPU formulas)
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float softplusf_(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float softplus_grad(float g, float x) {
    if (x > 20.0f) return g;
    const float z = expf(x);
    return g * z / (z + 1.0f);
}

}  // namespace spn
