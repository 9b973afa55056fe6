// bf16 MFMA GEMMs for the SIREN MLP in mixed precision (cfg.dtype = 1; BASELINE.json config 3).
// bf16 activations / weights, fp32 accumulation on v_mfma_f32_32x32x16_bf16, fp32 gradients.
//
//  * k_gemm_nt_bf16 — forward layers (sine / linear epilogue, bf16 C and derivative D) and the
//    backward dX GEMMs (× Dmul).  Same geometry as the fp32 kernel: 128x128 tile, 4 waves of
//    2x2 32x32 tiles, K-step 64 bf16 (128-B rows padded to 144 B → conflict-free
//    ds_read_b128), double-buffered LDS, XCD-aware tile order.
//  * k_gemm_tn_bf16 — weight gradients dW = dZᵀ·X summed over points.  Both operands stay in
//    their natural [point][feature] layout: tiles are staged row-major (coalesced 16-B loads) in
//    an XOR-swizzled LDS image and read back column-wise with ds_read_b64_tr_b16, so no
//    activation is ever transposed in HBM.  Points are split over blockIdx.y into fp32 slabs
//    reduced in a fixed order by k_reduce_slabs (deterministic).
#include "common.h"
#include "gemm_bf16.h"

namespace spn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int HB = 128, HK = 64, HLK = HK + 8;  // NT LDS row: 72 bf16 = 144 B

__device__ __forceinline__ u32x4 ldg16(const bf16* p) { return *reinterpret_cast<const u32x4*>(p); }

__device__ __forceinline__ void unpack8(u32x4 v, float (&f)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(v[i] << 16);
        f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
    }
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
    const __bf16 a = (__bf16)lo, b = (__bf16)hi;
    return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
    return u32x4{pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7])};
}

// ------------------------------------------------------------------------------------------
// NT
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gemm_nt_bf16(NT16Args g) {
    __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * HB * HLK];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nN = (g.N + HB - 1) / HB;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int bm = (t / nN) * HB, bn = (t % nN) * HB;
    const int lr = tid >> 3, lc = (tid & 7) * 8;  // loader: row (+32 i), bf16 column within the K-step

    u32x4 ra[4], rb[4];
    auto gload = [&](int k0) {
        const int k = k0 + lc;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = bm + lr + 32 * i;
            u32x4 v = {0u, 0u, 0u, 0u};
            if (row < g.M && k < g.K) v = k < g.K1 ? ldg16(g.A + (int64_t)row * g.lda + k) : ldg16(g.A2 + (int64_t)row * g.lda2 + (k - g.K1));
            ra[i] = v;
            const int col = bn + lr + 32 * i;
            u32x4 w = {0u, 0u, 0u, 0u};
            if (col < g.N && k < g.K) w = ldg16(g.B + (int64_t)col * g.ldb + k);
            rb[i] = w;
        }
    };
    auto sstore = [&](int stg) {
        bf16* sA = smem + stg * 2 * HB * HLK;
        bf16* sB = sA + HB * HLK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            *reinterpret_cast<u32x4*>(sA + (lr + 32 * i) * HLK + lc) = ra[i];
            *reinterpret_cast<u32x4*>(sB + (lr + 32 * i) * HLK + lc) = rb[i];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wr = wid >> 1, wc = wid & 1, r32 = lane & 31, h = lane >> 5;
    auto compute = [&](int stg) {
        const bf16* sA = smem + stg * 2 * HB * HLK;
        const bf16* pa0 = sA + (wr * 64 + r32) * HLK + 8 * h;
        const bf16* pa1 = pa0 + 32 * HLK;
        const bf16* pb0 = sA + HB * HLK + (wc * 64 + r32) * HLK + 8 * h;
        const bf16* pb1 = pb0 + 32 * HLK;
#pragma unroll
        for (int ks = 0; ks < HK / 16; ++ks) {
            const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(pa0 + 16 * ks);
            const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(pa1 + 16 * ks);
            const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(pb0 + 16 * ks);
            const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(pb1 + 16 * ks);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
        }
    };

    gload(0);
    sstore(0);
    __syncthreads();
    const int nk = (g.K + HK - 1) / HK;
    for (int kt = 0; kt < nk; ++kt) {
        const bool more = kt + 1 < nk;
        if (more) gload((kt + 1) * HK);
        compute(kt & 1);
        if (more) sstore((kt + 1) & 1);
        __syncthreads();
    }

    // Epilogue: each wave stages one 32x32 fp32 sub-tile at a time in LDS; a lane then owns two
    // 8-column row chunks → 16-B bf16 loads (Dmul) and stores (C, D).
    float* stage = reinterpret_cast<float*>(smem) + wid * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + r32] = acc[i][j][r];
            __syncthreads();
#pragma unroll
            for (int q2 = 0; q2 < 2; ++q2) {
                const int q = lane + 64 * q2;
                const int rr = q >> 2, c8 = (q & 3) * 8;
                const int row = bm + wr * 64 + i * 32 + rr;
                const int col = bn + wc * 64 + j * 32 + c8;
                if (row >= g.M || col >= g.N) continue;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = stage[rr * 32 + c8 + e];
                if (g.bias) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += g.bias[col + e];
                }
                if (g.rowbias) {
                    const float* rb = g.rowbias + (int64_t)(row / g.rows_per_ray) * g.ld_rb + col;
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += rb[e];
                }
                if (g.r1_a) {
                    const float a = g.r1_a[(int64_t)row * g.r1_lda];
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += a * g.r1_v[col + e];
                }
                if (g.act == 1 && col >= g.n_lin) {  // n_lin is a multiple of 8
                    float d[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float sn, cs;
                        sincosf(g.w0 * v[e], &sn, &cs);
                        v[e] = sn;
                        d[e] = g.w0 * cs;
                    }
                    if (g.Dout) *reinterpret_cast<u32x4*>(g.Dout + (int64_t)row * g.ld_dout + col) = pack8(d);
                } else if (g.Dout) {
                    const uint32_t one = 0x3f803f80u;
                    *reinterpret_cast<u32x4*>(g.Dout + (int64_t)row * g.ld_dout + col) = u32x4{one, one, one, one};
                }
                if (g.Dmul) {
                    float dm[8];
                    unpack8(ldg16(g.Dmul + (int64_t)row * g.ld_dmul + col), dm);
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] *= dm[e];
                }
                *reinterpret_cast<u32x4*>(g.C + (int64_t)row * g.ldc + col) = pack8(v);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// TN (weight gradients)
// ------------------------------------------------------------------------------------------
// LDS image of a [64 points][128 features] bf16 tile: 256-B rows, 16-B chunk ch of row r at
// chunk ch ^ (((r&3)<<2) | ((r>>2)&3)) — conflict-free for the 32x32x16 transposed reads
// (cdna_hip_programming.md T10, image (b)).
__device__ __forceinline__ int tn_off(int row, int ch) {
    return 256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

__global__ __launch_bounds__(256) void k_gemm_tn_bf16(TN16Args g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 256];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nK = (g.K + HB - 1) / HB;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int n0 = (t / nK) * HB, k0 = (t % nK) * HB;
    const int p_beg = blockIdx.y * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const int ch = tid & 15, lrow = tid >> 4;  // loader: 8 features (chunk ch), rows lrow + 16 i
    const bool do_bias = g.slab_b != nullptr && k0 == 0;

    u32x4 ra[4], rb[4];
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto gload = [&](int p0) {
        const int n = n0 + 8 * ch, k = k0 + 8 * ch;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = p0 + lrow + 16 * i;
            u32x4 v = {0u, 0u, 0u, 0u}, w = {0u, 0u, 0u, 0u};
            if (p < p_end) {
                if (n < g.N) v = ldg16(g.A + (int64_t)p * g.lda + n);
                if (k < g.K) w = k < g.K1 ? ldg16(g.B + (int64_t)p * g.ldb + k) : ldg16(g.B2 + (int64_t)p * g.ldb2 + (k - g.K1));
            }
            ra[i] = v;
            rb[i] = w;
        }
        if (do_bias) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float f[8];
                unpack8(ra[i], f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[e] += f[e];
            }
        }
    };
    auto sstore = [&](int stg) {
        char* sA = smem + stg * 2 * 64 * 256;
        char* sB = sA + 64 * 256;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int o = tn_off(lrow + 16 * i, ch);
            *reinterpret_cast<u32x4*>(sA + o) = ra[i];
            *reinterpret_cast<u32x4*>(sB + o) = rb[i];
        }
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wr = wid >> 1, wc = wid & 1, h = lane >> 5, grp = (lane >> 4) & 1;
    const int q = (lane & 15) >> 2, pp = lane & 3;
    // ds_read_b64_tr_b16 of rows [r0, r0+4) x features [col, col+16): lane 4q+pp of each 16-lane
    // group addresses row r0+q, features col+4pp..+3; lane i receives feature col+i of the 4 rows
    auto trd = [&](const char* base, int r0, int col) -> s16x4 {
        const int o = tn_off(r0 + q, (col >> 3) + (pp >> 1)) + 8 * (pp & 1);
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o));
    };
    // 32x32x16 operand: lane (r32, h) holds rows 8h..8h+7 of the 16-point step for feature r32
    auto operand = [&](const char* base, int r0, int col) -> bf16x8 {
        const s16x4 lo = trd(base, r0, col), hi = trd(base, r0 + 4, col);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    auto compute = [&](int stg) {
        const char* sA = smem + stg * 2 * 64 * 256;
        const char* sB = sA + 64 * 256;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int r0 = 16 * ks + 8 * h;
            const bf16x8 a0 = operand(sA, r0, wr * 64 + 16 * grp);
            const bf16x8 a1 = operand(sA, r0, wr * 64 + 32 + 16 * grp);
            const bf16x8 b0 = operand(sB, r0, wc * 64 + 16 * grp);
            const bf16x8 b1 = operand(sB, r0, wc * 64 + 32 + 16 * grp);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
        }
    };

    if (p_beg < p_end) {
        gload(p_beg);
        sstore(0);
        __syncthreads();
        int stg = 0;
        for (int p0 = p_beg; p0 < p_end; p0 += 64) {
            const bool more = p0 + 64 < p_end;
            if (more) gload(p0 + 64);
            compute(stg);
            if (more) sstore(stg ^ 1);
            __syncthreads();
            stg ^= 1;
        }
    }

    float* slab = g.slab + (int64_t)blockIdx.y * g.slab_stride;
    const int r32 = lane & 31;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = k0 + wc * 64 + j * 32 + r32;
        if (k >= g.K) continue;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wr * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < g.N) slab[(int64_t)n * g.ld_slab + k] = acc[i][j][r];
            }
    }
    if (do_bias) {  // block-uniform; combine the 16 row phases of every chunk in a fixed order
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [16 phases][128 features]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lrow * 128 + 8 * ch + e] = bs[e];
        __syncthreads();
        if (tid < 128 && n0 + tid < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 16; ++ph) s += red[ph * 128 + tid];
            g.slab_b[(int64_t)blockIdx.y * g.N + n0 + tid] = s;
        }
    }
}

// ------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------
int32_t gemm_nt_bf16(const NT16Args& a, hipStream_t s) {
    SPN_ARG(a.M >= 0 && a.N > 0 && a.K > 0, "gemm_nt_bf16: bad shape M=%d N=%d K=%d", a.M, a.N, a.K);
    SPN_ARG(a.K % 8 == 0 && a.N % 8 == 0 && a.n_lin % 8 == 0, "gemm_nt_bf16: K, N, n_lin must be multiples of 8");
    SPN_ARG(a.K1 <= a.K && (a.K1 == a.K || (a.A2 != nullptr && a.K1 % HK == 0)),
            "gemm_nt_bf16: a split K1=%d must be a multiple of %d with A2 set", a.K1, HK);
    SPN_ARG(a.lda % 8 == 0 && a.ldb % 8 == 0 && a.ldc % 8 == 0 && (a.K1 == a.K || a.lda2 % 8 == 0),
            "gemm_nt_bf16: leading dims must be multiples of 8");
    SPN_ARG(!a.Dout || a.ld_dout % 8 == 0, "gemm_nt_bf16: ld_dout");
    SPN_ARG(!a.Dmul || a.ld_dmul % 8 == 0, "gemm_nt_bf16: ld_dmul");
    SPN_ARG(a.rowbias == nullptr || a.rows_per_ray > 0, "gemm_nt_bf16: rows_per_ray");
    if (a.M == 0) return SPNERF_OK;
    const int nb = cdiv(a.M, HB) * cdiv(a.N, HB);
    ProfScope prof("gemm_nt_bf16", s, 2.0 * a.M * a.N * a.K,
                   2.0 * ((double)a.M * a.K + (double)a.N * a.K + (2.0 + (a.Dmul ? 1 : 0)) * a.M * a.N));
    hipLaunchKernelGGL(k_gemm_nt_bf16, dim3(nb), dim3(256), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int tn_splits_bf16(int P, int N, int K) {
    const int tiles = cdiv(N, HB) * cdiv(K, HB);
    int splits = cdiv(512, tiles);
    if (splits > 64) splits = 64;
    const int max_splits = cdiv(P, 1024);
    if (splits > max_splits) splits = max_splits;
    return splits < 1 ? 1 : splits;
}

int32_t gemm_tn_bf16(const TN16Args& a0, int splits, hipStream_t s) {
    TN16Args a = a0;
    SPN_ARG(a.N > 0 && a.K > 0 && a.P >= 0 && splits >= 1, "gemm_tn_bf16: bad shape");
    SPN_ARG(a.N % 8 == 0 && a.K % 8 == 0 && a.K1 % 8 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0,
            "gemm_tn_bf16: dims must be multiples of 8");
    SPN_ARG(a.K1 >= a.K || (a.B2 != nullptr && a.ldb2 % 8 == 0), "gemm_tn_bf16: second B segment missing");
    int pps = cdiv(a.P, splits);
    pps = (pps + 63) / 64 * 64;
    a.p_per_split = pps < 64 ? 64 : pps;
    const int nb = cdiv(a.N, HB) * cdiv(a.K, HB);
    ProfScope prof("gemm_tn_bf16", s, 2.0 * a.P * a.N * a.K,
                   2.0 * (double)a.P * (a.N + a.K) + 4.0 * splits * (double)a.N * a.K);
    hipLaunchKernelGGL(k_gemm_tn_bf16, dim3(nb, splits), dim3(256), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

}  // namespace spn
