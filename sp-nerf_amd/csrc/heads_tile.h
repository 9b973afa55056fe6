// The fused inference heads' per-tile computation (models/spnerf.py:332-367), shared by the
// heads kernel (k_heads_bf16, heads_bf16.hip: H_L staged from HBM) and the fused trunk + heads
// kernel (k_trunk2_bf16 with HEADS, trunk2_bf16.hip: H_L is the trunk's last LDS image).  What
// each layer computes and why: heads_bf16.hip.
#pragma once
#include <algorithm>

#include "mlp_layout.h"
#include "trunk.h"

namespace spn {
namespace hd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int TM = 128;                 // points per tile
constexpr int HW = 512, HH = 256;
constexpr int NJ = TM / 32;             // 32-point MFMA tiles per wave
constexpr int TPD = 4;                  // weight prefetch depth (k-steps)
constexpr int IMG = TM * HW * 2;        // the [128][512] bf16 image
constexpr int OST_LD = 16;              // output staging row (floats), NO <= 16
constexpr int RQ_RAYS = 4;                         // per-ray Q rows staged for tiles of <= 4 rays

__device__ __forceinline__ int img_off(int row, int ch) { return row * 1024 + ((ch ^ (row & 15)) << 4); }

// acc[a][j] (features 32·NA·w + 32a.., points 32j..) = Σ_k W[n][k] · image[point][k] over nks
// k-steps of 16; wsrc = this wave's fragment stream (+ lane · 8)
// the first TPD k-steps of a layer's weight stream (issuing them one phase early, before the
// previous layer's epilogue, measured slower: the live ring across the epilogue spills)
template <int NA>
__device__ __forceinline__ void layer_prime(const bf16* __restrict__ wsrc, u32x4 (&ring)[TPD][NA]) {
#pragma unroll
    for (int d = 0; d < TPD; ++d)
#pragma unroll
        for (int a = 0; a < NA; ++a) ring[d][a] = ldg16(wsrc + (d * NA + a) * 512);
}

template <int NA>
__device__ __forceinline__ void layer_mm(const bf16* __restrict__ wsrc, int nks, const char* smem, int lane,
                                         f32x16 (&acc)[NA][NJ], u32x4 (&ring)[TPD][NA]) {
    const int r32 = lane & 31, h = lane >> 5, sw = r32 & 15;
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
    const char* brow = smem + r32 * 1024;
    bf16x8 bc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bc[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((h ^ sw) << 4));
#pragma unroll 1
    for (int ks0 = 0; ks0 < nks; ks0 += TPD) {
#pragma unroll
        for (int d = 0; d < TPD; ++d) {
            const int ks = ks0 + d;
            // the next step's B fragments (past the last step: an in-bounds read, unused)
            const int offn = ((2 * (ks + 1) + h) ^ sw) << 4;
            bf16x8 bn[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) bn[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + offn);
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int a = 0; a < NA; ++a)
                    acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ring[d][a]), bc[j],
                                                                      acc[a][j], 0, 0, 0);
            const int kn = min(ks + TPD, nks - 1);
#pragma unroll
            for (int a = 0; a < NA; ++a) ring[d][a] = ldg16(wsrc + (kn * NA + a) * 512);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, NA, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x020, NA, 0);
#pragma unroll
            for (int j = 0; j < NJ; ++j) bc[j] = bn[j];
        }
    }
}

// A narrow head on MFMA: the [32][K] hi/lo-row A operand a (PackedOffs::Fnar16, fragment order,
// 32 features per wave-tile) times the image columns from k-step kb, K split over the 8 waves
// (wave w takes k-steps [w·KPER, (w+1)·KPER)) for all 128 points.  Row pairs (0, 1), (2, 3) and
// (8, 9) are the hi and lo halves of up to three weight rows; their sums are this wave's partial
// outputs, written to part[w][point][0..2] (summed over the waves in wave order by the caller).
template <int KPER>
__device__ __forceinline__ void narrow_mm(const bf16* __restrict__ a, int kb, const char* smem, int lane_, int w,
                                          float* part) {
    const int lane = opaque(lane_), r32 = lane & 31, h = lane >> 5, sw = r32 & 15;
    u32x4 af[KPER];
#pragma unroll
    for (int d = 0; d < KPER; ++d) af[d] = ldg16(a + (w * KPER + d) * 512 + lane * 8);
    f32x16 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const char* brow = smem + r32 * 1024;
#pragma unroll
    for (int d = 0; d < KPER; ++d) {
        const int off = ((2 * (kb + w * KPER + d) + h) ^ sw) << 4;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const bf16x8 b = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + off);
            acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, af[d]), b, acc[j], 0, 0, 0);
        }
    }
    // rows 0..3 are elements 0..3 and rows 8, 9 elements 4, 5 of lanes 0..31 (point = lane)
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            *reinterpret_cast<f32x4*>(part + (w * TM + 32 * j + r32) * 4) =
                f32x4{acc[j][0] + acc[j][1], acc[j][2] + acc[j][3], acc[j][4] + acc[j][5], 0.f};
    }
}
__device__ __forceinline__ int64_t narrow_off(int head) {  // σ, albedo, sun within Fnar16
    return head == 0 ? 0 : head == 1 ? (int64_t)32 * HW : (int64_t)32 * (HW + HH);
}

constexpr int OST_BYTES = TM * OST_LD * 4;        // output staging [TM][OST_LD] floats
constexpr int PART_BYTES = 8 * TM * 4 * 4;         // narrow / semantic partials [wave][point][4]
constexpr int RQ_BYTES = RQ_RAYS * 2 * HH * 4;     // per-ray Q rows of up to RQ_RAYS rays

// One 128-point tile of the heads.  On entry the tile's H_L (rows p0 .. p0 + 127) is the [128][512]
// bf16 image at smem (img_off layout), complete and visible (after a barrier); ost / part (and,
// RQ, srq) are LDS areas of the sizes above.  Writes the tile's output rows; every thread of the
// 8-wave workgroup calls it (it contains barriers); on return the image may be overwritten.
// GA / KA: HeadsFusedArgs / PackedOffs, possibly address-space qualified (the fused trunk passes
// references into the kernarg segment)
template <bool RQ, typename GA, typename KA>
__device__ __forceinline__ void heads_tile(GA& g, KA& k, char* smem, float* ost, float* part, float* srq, int64_t p0) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const float* Pk = g.packed;
    const bf16* P16 = reinterpret_cast<const bf16*>(g.packed);
    const bool full = g.mode == 0;
    const int C = g.C;
    auto stream = [&](int64_t off, int nks, int NA) {
        return P16 + off + (int64_t)w * nks * NA * 512 + opaque(lane) * 8;
    };

    // epilogue walk: for each accumulator element group, f0 = first of 4 features, row = point
    // (the trunk kernel's accumulator geometry); fn(a, j, gq, f0, row, v[4]) with the raw sums
    auto epi = [&](auto kna, auto& acc, auto fn) {
        constexpr int NA = decltype(kna)::value;
        const int el = opaque(lane), er32 = el & 31, eh = el >> 5;  // opaque: no hoisted lane math
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * NA * w + 32 * a + 8 * gq + 4 * eh;
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * gq + e];
                    fn(a, j, gq, f0, 32 * j + er32, v);
                }
                __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted loads
            }
    };
    auto put4 = [&](int row, int f0, const float (&y)[4]) {
        *reinterpret_cast<u32x2*>(smem + img_off(row, f0 >> 3) + 8 * ((f0 >> 2) & 1)) =
            u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
    };

    // the tile's rays' sun rows of Q into LDS when they are few (one ray per tile at 128
    // samples per ray): the Q epilogue then reads LDS instead of an L2 round trip per row (read
    // after the barriers that follow the σ head)
    const int64_t ray0 = p0 / g.S;
    const int nray = (int)((std::min<int64_t>(p0 + TM, (int64_t)g.P) - 1) / g.S - ray0) + 1;
    const bool rq_lds = RQ && full && nray <= RQ_RAYS && !(g.dbg & 4);  // block-uniform (dbg 4: A/B)
    if (rq_lds)
        for (int i = tid; i < nray * 2 * HH; i += 512) srq[i] = g.rbQ[ray0 * (2 * HH) + i];
    // σ on MFMA (narrow_mm), the 8 waves' partials summed in wave order
    narrow_mm<HW / 16 / 8>(P16 + k.Fnar16 + narrow_off(0), 0, smem, lane, w, part);
    __syncthreads();
    if (tid < TM) {
        float t = 0.f;
        for (int v = 0; v < 8; ++v) t += part[(v * TM + tid) * 4];
        ost[tid * OST_LD + 3] = softplusf_(t + Pk[k.bsig]);
    }
    __syncthreads();  // the semantic epilogue reuses part
    if (full) {
        // semantic hidden (256) → logits through W_m2 in the epilogue
        if (C > 0) {
            f32x16 acc[1][NJ];
            u32x4 ring1[TPD][1];
            layer_prime<1>(stream(k.Fsem16, HW / 16, 1), ring1);
            layer_mm<1>(stream(k.Fsem16, HW / 16, 1), HW / 16, smem, lane, acc, ring1);
            // logits partials over this wave's 32 features, per point (lane halves hold 4 + 4)
            const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
            float sacc[NJ][4];
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int c = 0; c < 4; ++c) sacc[j][c] = 0.f;
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                const f32x4 bv = ld4(Pk + k.bG + HW + f0);
                f32x4 wm[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) wm[c] = c < C ? ld4(Pk + k.Wm2 + c * HH + f0) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    float y[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) y[e] = (float)(bf16)fast_sin(acc[0][j][4 * gq + e] + bv[e]);
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        sacc[j][c] += (y[0] * wm[c][0] + y[1] * wm[c][1]) + (y[2] * wm[c][2] + y[3] * wm[c][3]);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float s = sacc[j][c] + __shfl_xor(sacc[j][c], 32, 64);
                    if (eh == 0 && c < C) part[(w * TM + 32 * j + er32) * 4 + c] = s;
                }
        }
        // feat (linear, 512) → the image
        __builtin_amdgcn_sched_barrier(0);
        {
            f32x16 acc[2][NJ];
            u32x4 ring2[TPD][2];
            layer_prime<2>(stream(k.Ffeat16, HW / 16, 2), ring2);
            layer_mm<2>(stream(k.Ffeat16, HW / 16, 2), HW / 16, smem, lane, acc, ring2);
            __syncthreads();  // every wave is done reading H_L
            epi(std::integral_constant<int, 2>{}, acc, [&](int, int, int, int f0, int row, const float (&v)[4]) {
                const f32x4 bv = ld4(Pk + k.bG + f0);
                const float y[4] = {v[0] + bv[0], v[1] + bv[1], v[2] + bv[2], v[3] + bv[3]};
                put4(row, f0, y);
            });
            __syncthreads();
        }
        // [sun1 | rgb1] = sin(W_Q feat + b + per-ray sun rows) → the image
        {
            f32x16 acc[2][NJ];
            u32x4 ring2[TPD][2];
            layer_prime<2>(stream(k.FQ16, HW / 16, 2), ring2);
            layer_mm<2>(stream(k.FQ16, HW / 16, 2), HW / 16, smem, lane, acc, ring2);
            __syncthreads();
            // each accumulator row's ray, relative to ray0 (P < 2^31: host check)
            const int er32 = opaque(lane) & 31;
            int rrel[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) rrel[j] = (int)(std::min<int64_t>(p0 + 32 * j + er32, g.P - 1) / g.S - ray0);
            // two instances of the epilogue (block-uniform choice): one select between the LDS
            // and the global row made hipcc emit a flat load, waited with vmcnt(0) lgkmcnt(0)
            // per 4 outputs
            auto qepi = [&](auto klds) {
                epi(std::integral_constant<int, 2>{}, acc, [&](int, int j, int, int f0, int row, const float (&v)[4]) {
                    const f32x4 bv = ld4(Pk + k.bQ + f0);
                    const f32x4 rv = decltype(klds)::value ? *reinterpret_cast<const f32x4*>(srq + rrel[j] * (2 * HH) + f0)
                                                           : ld4(g.rbQ + (ray0 + rrel[j]) * (2 * HH) + f0);
                    float y[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) y[e] = fast_sin((v[e] + bv[e]) + rv[e]);
                    put4(row, f0, y);
                });
            };
            if (rq_lds) qepi(std::true_type{});
            else qepi(std::false_type{});
            __syncthreads();
        }
        // semantic logits: the 8 waves' partials in wave order
        __builtin_amdgcn_sched_barrier(0);
        for (int i = tid; i < TM * C; i += 512) {
            const int r = i / C, c = i % C;
            float s = 0.f;
            for (int v = 0; v < 8; ++v) s += part[(v * TM + r) * 4 + c];
            ost[r * OST_LD + g.sem_col + c] = s + Pk[k.bm2 + c];
        }
        // albedo from rgb1 (image k-steps 16..31) on MFMA
        __syncthreads();  // the logits are read from part
        narrow_mm<HH / 16 / 8>(P16 + k.Fnar16 + narrow_off(1), HH / 16, smem, lane, w, part);
        __syncthreads();  // rgb1 read before sun_v 2 overwrites the image's first half
        if (tid < TM) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float t = 0.f;
                for (int v = 0; v < 8; ++v) t += part[(v * TM + tid) * 4 + c];
                ost[tid * OST_LD + c] = __fsub_rn(__fmul_rn(sigmoidf_(t + Pk[k.br2 + c]), 1.002f), 0.001f);
            }
        }
        // sun_v 2 and 3 on image columns 0..255
        for (int l = 0; l < 2; ++l) {
            f32x16 acc[1][NJ];
            u32x4 ring1[TPD][1];
            layer_prime<1>(stream(l == 0 ? k.Fs2_16 : k.Fs3_16, HH / 16, 1), ring1);
            layer_mm<1>(stream(l == 0 ? k.Fs2_16 : k.Fs3_16, HH / 16, 1), HH / 16, smem, lane, acc, ring1);
            __syncthreads();
            const int64_t boff = l == 0 ? k.bs2 : k.bs3;
            epi(std::integral_constant<int, 1>{}, acc, [&](int, int, int, int f0, int row, const float (&v)[4]) {
                const f32x4 bv = ld4(Pk + boff + f0);
                float y[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) y[e] = fast_sin(v[e] + bv[e]);
                put4(row, f0, y);
            });
            __syncthreads();
        }
        // sun visibility (MFMA) and the ray's sky colour; part's albedo partials were read
        // before the sun_v layers' barriers
        narrow_mm<HH / 16 / 8>(P16 + k.Fnar16 + narrow_off(2), 0, smem, lane, w, part);
        __syncthreads();
        if (tid < TM) {
            float t = 0.f;
            for (int v = 0; v < 8; ++v) t += part[(v * TM + tid) * 4];
            ost[tid * OST_LD + 4] = sigmoidf_(t + Pk[k.bs4]);
            const float* sk = g.sky + (std::min<int64_t>(p0 + tid, g.P - 1) / g.S) * 4;
#pragma unroll
            for (int c = 0; c < 3; ++c) ost[tid * OST_LD + 5 + c] = sk[c];
        }
    }
    __syncthreads();
    // the tile's output rows, contiguous in HBM
    const int rows = (int)std::min<int64_t>(TM, g.P - p0);
    if (full) {
        for (int i = tid; i < rows * g.NO; i += 512) g.out[p0 * g.NO + i] = ost[(i / g.NO) * OST_LD + i % g.NO];
    } else {
        for (int i = tid; i < rows; i += 512) g.out[(p0 + i) * g.NO + 3] = ost[i * OST_LD + 3];
    }
}

}  // namespace hd

// The argument of a fused trunk launch that runs the heads on its last image: the trunk's (first,
// so the kernarg-segment reads of TrunkArgs stay valid) and the heads'
struct TrunkHeadsArgs : TrunkArgs {
    HeadsFusedArgs hg;
    PackedOffs hk;
};
static_assert(sizeof(TrunkHeadsArgs) <= 4096, "a kernel argument: within the 4 KB kernarg segment");

}  // namespace spn
