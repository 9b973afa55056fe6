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
    const int64_t ray0 = (int)p0 / g.S;  // P < 2^31 / 512 (host checks): 32-bit divisions
    const int nray = (int)((int)(std::min<int64_t>(p0 + TM, (int64_t)g.P) - 1) / g.S - ray0) + 1;
    const bool rq_lds = RQ && full && nray <= RQ_RAYS && !((kTrunkAbl ? g.dbg : 0) & 4);  // block-uniform (dbg 4: A/B)
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
            for (int j = 0; j < NJ; ++j) rrel[j] = (int)std::min<int64_t>(p0 + 32 * j + er32, g.P - 1) / g.S - (int)ray0;
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
            const float* sk = g.sky + (int64_t)((int)std::min<int64_t>(p0 + tid, g.P - 1) / g.S) * 4;
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

// ---- training (option heads_epi 2, k_heads_train_bf16): the same layers after the SAVING trunk,
// with every activation the backward reads stored at the layer-by-layer GEMMs' addresses
// (HeadsFusedArgs G / DG / Q / DQ / S2 / DS2 / S3 / DS3, hsave).  The wide layers run the
// layer-by-layer GEMMs' arithmetic — the same MFMA (32x32x16 bf16, the K-steps of 16 in
// ascending order, weights and activations in swapped operand roles: the same products in the
// same order), then + bias (+ the per-ray row), fast_sincos, RNE to bf16 — so G, Q, sun_v 2 / 3
// and their D equal the DMA NT GEMMs' (k_gemm_nt_bf16d) bit for bit; the narrow heads run on
// MFMA (narrow_mm, hi / lo weight rows) as in inference instead of in those GEMMs' epilogues.
//
// The stores are kept off the MFMAs' critical path the way the training trunk does it: a
// layer's image leaves for HBM in slices inside the NEXT layer's k-loop, each slice after that
// k-step group's weight refills (so no ring wait counts it), and the next layer's weight ring is
// primed before a layer's epilogue, so the register stores of D there (v_permlane32_swap-joined
// 16-B pieces) are younger than every load the next k-loop waits for.

// 16-B stores of one accumulator tile's 16-feature group pairs: cq[gq] holds the bf16 of
// features fbase + 8·gq + 4·eh .. +3 at tile row `row`; pairs (0, 1) and (2, 3) are joined by
// v_permlane32_swap so lane l < 32 stores features fbase + 8k .. +7 and lane l + 32 the next 8
// (the training trunk's register-D store).  Rows past P fall outside the descriptor: dropped.
__device__ __forceinline__ void store_rows16(__amdgpu_buffer_rsrc_t rs, int ld, int fbase, int row, int eh, u32x2 (&cq)[4]) {
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const auto r = __builtin_amdgcn_permlane32_swap(cq[k][e], cq[k + 1][e], false, false);
            cq[k][e] = r[0];
            cq[k + 1][e] = r[1];
        }
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{cq[k][0], cq[k][1], cq[k + 1][0], cq[k + 1][1]}, rs,
                                               (row * ld + fbase + 8 * k + 8 * eh) * 2, 0, 0);
    }
}

// chunks [q0, q0 + N) (per thread) of image columns [0, 8·NCH) to the rows of a descriptor (ld
// elements): chunk c = tid + 512·q, consecutive lanes on consecutive 16-B pieces of a row
#ifndef SPN_HEADS_NT
#define SPN_HEADS_NT 3  // training heads' stores non-temporal (glc slc): 1 = image copy-outs (whole rows), 2 = the D columns
#endif
template <int NCH, int N>
__device__ __forceinline__ void image_out(const char* smem, __amdgpu_buffer_rsrc_t rs, int ld, int tid_, int q0) {
    const int tid = opaque(tid_);  // per-thread offsets computed here, not hoisted across the tile loop
    u32x4 v[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const int c = tid + 512 * (q0 + q);
        v[q] = *reinterpret_cast<const u32x4*>(smem + img_off(c / NCH, c % NCH));
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
        const int c = tid + 512 * (q0 + q);
        __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, ((c / NCH) * ld + 8 * (c % NCH)) * 2, 0, (SPN_HEADS_NT & 1) ? 3 : 0);
    }
}

#ifndef SPN_HEADS_DCOLS
#define SPN_HEADS_DCOLS 1  // the wide layers' D (cos) through the wave's own image columns (0: register stores)
#endif
// rows 32j .. 32j + 31 of this wave's own image columns [fb, fb + 32·NA) (written by this wave
// only, after the barrier that ends every wave's reads of the image) to a descriptor (ld
// elements): 4·NA lanes store one row's whole 64·NA-byte piece (the register stores of
// store_rows16 write 32 B per row and instruction).  One wave's LDS accesses run in order; the
// memory clobbers keep the compiler from moving the epilogue's image writes across the reads.
template <int NA>
__device__ __forceinline__ void cols_out(const char* smem, __amdgpu_buffer_rsrc_t rs, int ld, int fb, int j, int lane_) {
    constexpr int LPR = 4 * NA;    // lanes per row (16 B each)
    constexpr int RPI = 64 / LPR;  // rows per instruction
    constexpr int N = 32 / RPI;    // instructions
    const int l = opaque(lane_);
    const int ch = (fb >> 3) + l % LPR, r0 = 32 * j + l / LPR;
    asm volatile("" ::: "memory");
    u32x4 v[N];
#pragma unroll
    for (int q = 0; q < N; ++q) v[q] = *reinterpret_cast<const u32x4*>(smem + img_off(r0 + RPI * q, ch));
#pragma unroll
    for (int q = 0; q < N; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, ((r0 + RPI * q) * ld + 8 * ch) * 2, 0, (SPN_HEADS_NT & 2) ? 3 : 0);
    asm volatile("" ::: "memory");
}

#ifndef SPN_HEADS_RQ_OST
#define SPN_HEADS_RQ_OST 1  // training heads: when every tile lies within one ray, its Q rows from LDS (ost)
#endif
#ifndef SPN_HEADS_WM_OST
#define SPN_HEADS_WM_OST 1  // ... and the semantic logits' weights W_m2 from ost too
#endif
#ifndef SPN_HEADS_ZC
#define SPN_HEADS_ZC 0  // 1: layer_mm_d k-step 0 with the MFMA C = 0 (no accumulator zeroing) — spills 172 B, heads 2.56 -> 3.0 ms per C4 step
#endif
// layer_prime / layer_mm with a ring of DEPTH k-steps (the 256-wide layers run 8 deep: half the
// MFMAs per k-step of the 512-wide ones, the same register cost and time of cover), drain(group)
// after each group of DEPTH k-steps (behind that group's refills); the ring must be primed
// (layer_prime_n) by the caller
template <int NA, int DEPTH>
__device__ __forceinline__ void layer_prime_n(const bf16* __restrict__ wsrc, u32x4 (&ring)[DEPTH][NA]) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int a = 0; a < NA; ++a) ring[d][a] = ldg16(wsrc + (d * NA + a) * 512);
}
template <int NA, int DEPTH, typename Drain>
__device__ __forceinline__ void layer_mm_d(const bf16* __restrict__ wsrc, int nks, const char* smem, int lane,
                                           f32x16 (&acc)[NA][NJ], u32x4 (&ring)[DEPTH][NA], Drain&& drain) {
    constexpr int TPD = DEPTH;
    const int r32 = lane & 31, h = lane >> 5, sw = r32 & 15;
    const char* brow = smem + r32 * 1024;
    bf16x8 bc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bc[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((h ^ sw) << 4));
    // one k-step; k-step 0 (kfirst) takes the accumulators' C operand as the inline constant 0
    // instead of zeroed registers (no v_mov per accumulator register per layer; the same sums)
    auto kstep = [&](int ks, int d, auto kfirst) {
        constexpr bool FIRST = decltype(kfirst)::value;
        const int offn = ((2 * (ks + 1) + h) ^ sw) << 4;
        bf16x8 bn[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bn[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + offn);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int a = 0; a < NA; ++a)
                acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ring[d][a]), bc[j],
                                                                  FIRST ? f32x16{} : acc[a][j], 0, 0, 0);
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
    };
#if SPN_HEADS_ZC
    // the first group peeled (k-step 0 with C = 0), then groups TPD.. as before
    kstep(0, 0, std::true_type{});
#pragma unroll
    for (int d = 1; d < TPD; ++d) kstep(d, d, std::false_type{});
    drain(0);
    constexpr int kfirst = TPD;
#else
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
    constexpr int kfirst = 0;
#endif
#pragma unroll 1
    for (int ks0 = kfirst; ks0 < nks; ks0 += TPD) {
#pragma unroll
        for (int d = 0; d < TPD; ++d) kstep(ks0 + d, d, std::false_type{});
        drain(ks0 / TPD);
    }
}

// narrow_mm's A fragments loaded ahead (before an epilogue's stores) and the MFMAs on them
template <int KPER>
__device__ __forceinline__ void narrow_load(const bf16* __restrict__ a, int lane_, int w, u32x4 (&af)[KPER]) {
    const int lane = opaque(lane_);
#pragma unroll
    for (int d = 0; d < KPER; ++d) af[d] = ldg16(a + (w * KPER + d) * 512 + lane * 8);
}
template <int KPER>
__device__ __forceinline__ void narrow_run(const u32x4 (&af)[KPER], int kb, const char* smem, int lane_, int w, float* part) {
    const int lane = opaque(lane_), r32 = lane & 31, h = lane >> 5, sw = r32 & 15;
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
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            *reinterpret_cast<f32x4*>(part + (w * TM + 32 * j + r32) * 4) =
                f32x4{acc[j][0] + acc[j][1], acc[j][2] + acc[j][3], acc[j][4] + acc[j][5], 0.f};
    }
}

// ring depth of the training heads' 512-wide layers (8: 43 VGPRs spilled, main pass 1.69 against
// 1.50 ms per 524 288 points)
#ifndef SPN_HEADS_D2
#define SPN_HEADS_D2 4
#endif
// the heads' biases staged once per launch (floats): G = [feat | sem hidden], Q, sun_v 2, sun_v 3
constexpr int SB_G = 0, SB_Q = HW + HH, SB_S2 = SB_Q + 2 * HH, SB_S3 = SB_S2 + HH, SB_N = SB_S3 + HH;

// One 128-point tile of the training heads.  On entry H_L is the [128][512] image at smem,
// complete and visible; ost[row][3] = softplus(σ pre-activation) of each row (from the trunk's
// hsave[p·8]); sbias holds the SB_* biases.  mode 0: every head; mode 2 (the solar pass): feat,
// sun1, sun_v 2 / 3 and the sun, the other output columns zero.  Writes the tile's output rows;
// every thread of the 8-wave workgroup calls it (it contains barriers).
// (g.dbg, profiling ablations of the -DSPN_ABLATIONS build, outputs invalid: 1 = no image
// copy-outs, 2 = no register stores (D, semantic hidden), 8 = no sin / cos in the wide layers'
// epilogues)
// The training heads' per-tile staging in ost (the caller's, before the barrier that precedes
// heads_tile_train<true>; every tile within one ray): the ray's Q rows rbQ[ray][0..512) in columns
// 8..15 of rows 0..63 and (SPN_HEADS_WM_OST) the semantic logits' weights W_m2 [C][HH], C <= 3:
// entries q < 512 in columns 4..7 (rows q / 4), the rest in columns 8..15 of rows 64 + (q - 512) / 8
// — every f32x4 the epilogues read is one aligned piece of a row.  Columns 0..2 and 4..15 are free
// until the semantic logits and the outputs are written, after the Q epilogue.
template <typename GA, typename KA>
__device__ __forceinline__ void stage_rows_ost(GA& g, KA& k, float* ost, int64_t p0, int tid_) {
    const int f = opaque(tid_);  // 512 threads: the 2·HH floats of the row
    ost[(f >> 3) * OST_LD + 8 + (f & 7)] = g.rbQ[(int64_t)((int)p0 / g.S) * (2 * HH) + f];
    if constexpr (SPN_HEADS_WM_OST) {
        if (g.mode == 0)  // block-uniform (the solar pass has no semantic head)
            for (int q = f; q < g.C * HH; q += 512)
                ost[q < 512 ? (q >> 2) * OST_LD + 4 + (q & 3) : (64 + ((q - 512) >> 3)) * OST_LD + 8 + ((q - 512) & 7)] =
                    g.packed[k.Wm2 + q];
    }
}

// SOL: the solar pass (g.mode 2), its own instance: sun1 alone in Q, no semantic / albedo heads
template <bool RQ1, bool SOL, typename GA, typename KA, typename Prefetch>
__device__ __forceinline__ void heads_tile_train(GA& g, KA& k, char* smem, float* ost, float* part, const float* sbias,
                                                 int64_t p0, Prefetch&& prefetch) {
    constexpr int D1 = 8;  // ring depth of the 256-wide layers (sem hidden, sun_v 2 / 3)
    constexpr int D2 = SPN_HEADS_D2;  // ... of the 512-wide ones (feat, Q)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // (product build: 0 — a runtime flag here made every sine epilogue compute sin, cos AND the
    // ablation's alternative, then select per element: two v_cndmask per element)
    const int dbg = kTrunkAbl ? g.dbg : 0;
    const float* Pk = g.packed;
    const bf16* P16 = reinterpret_cast<const bf16*>(g.packed);
    constexpr bool full = !SOL;   // (g.mode == 0 in the full instance, 2 in the solar one)
    const int C = full ? g.C : 0;
    const int rows = (int)std::min<int64_t>(TM, g.P - p0);
    auto stream = [&](int64_t off, int nks, int NA) {
        return P16 + off + (int64_t)w * nks * NA * 512 + opaque(lane) * 8;
    };
    auto rsrc = [&](bf16* base, int ld) {
        return __builtin_amdgcn_make_buffer_rsrc(base + p0 * ld, 0, (dbg & 1) ? 0 : rows * ld * 2, 0x00020000);
    };
    auto rsrc_r = [&](bf16* base, int ld) {  // register stores (dbg 2: dropped)
        return __builtin_amdgcn_make_buffer_rsrc(base + p0 * ld, 0, (dbg & 2) ? 0 : rows * ld * 2, 0x00020000);
    };
    auto sincos = [&](float x, float* sn, float* cs) {
        if (dbg & 8) {
            *sn = x;
            *cs = -x;
        } else {
            fast_sincos(x, sn, cs);
        }
    };
    auto put4 = [&](int row, int f0, const float (&y)[4]) {
        *reinterpret_cast<u32x2*>(smem + img_off(row, f0 >> 3) + 8 * ((f0 >> 2) & 1)) =
            u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
    };
    auto nodrain = [](int) {};
    const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
    // RQ1 (every tile within one ray: S a multiple of TM, the launch's choice): the tile's ray's Q
    // rows (and W_m2) were staged in ost by the caller before its barrier (stage_rows_ost)
    static_assert(!RQ1 || (OST_LD >= 16 && 2 * HH == 512), "the Q row staging: 512 floats in ost columns 8..15");

    u32x4 ring2f[D2][2];  // feat's weights
    // semantic hidden = sin(W_m1 H_L + b) → G[:, W..W+H) and DG; its logits' partials → part
    if (C > 0) {
        f32x16 acc[1][NJ];
        u32x4 ring1[D1][1];
        layer_prime_n<1, D1>(stream(k.Fsem16, HW / 16, 1), ring1);
        layer_mm_d<1, D1>(stream(k.Fsem16, HW / 16, 1), HW / 16, smem, lane, acc, ring1, nodrain);
        layer_prime_n<2, D2>(stream(k.Ffeat16, HW / 16, 2), ring2f);
        const auto rsG = rsrc_r(g.G, g.ldG), rsD = rsrc_r(g.DG, g.ldG);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            u32x2 yq[4], cq[4];
            float sacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_G + HW + f0);
                float y[4], cs[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) sincos(acc[0][j][4 * gq + e] + bv[e], &y[e], &cs[e]);
                yq[gq] = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                cq[gq] = u32x2{pack2(cs[0], cs[1]), pack2(cs[2], cs[3])};
                const f32x4 yb = raw_f32(yq[gq]);  // the stored (bf16) values feed the logits
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    f32x4 wm = f32x4{0.f, 0.f, 0.f, 0.f};
                    if (c < C) {
                        if constexpr (RQ1 && SPN_HEADS_WM_OST)  // staged in ost (see the top of the tile)
                            wm = *reinterpret_cast<const f32x4*>(
                                ost + (c < 2 ? (c * 64 + 8 * w + 2 * gq + eh) * OST_LD + 4 : (64 + 4 * w + gq) * OST_LD + 8 + 4 * eh));
                        else
                            wm = ld4(Pk + k.Wm2 + c * HH + f0);
                    }
                    sacc[c] += (yb[0] * wm[0] + yb[1] * wm[1]) + (yb[2] * wm[2] + yb[3] * wm[3]);
                }
            }
            store_rows16(rsG, g.ldG, HW + 32 * w, 32 * j + er32, eh, yq);
            store_rows16(rsD, g.ldG, HW + 32 * w, 32 * j + er32, eh, cq);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float t = sacc[c] + __shfl_xor(sacc[c], 32, 64);
                if (eh == 0 && c < C) part[(w * TM + 32 * j + er32) * 4 + c] = t;
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    } else {
        layer_prime_n<2, D2>(stream(k.Ffeat16, HW / 16, 2), ring2f);
    }
    // feat = W_f H_L + b (linear) → the image (to G[:, 0..W) during Q's k-loop)
    u32x4 ring2q[D2][2];  // Q's weights
    u32x4 ring1q[D1][1];  // ... the solar pass's: sun1 alone, 32 features per wave (FQs16)
    {
        f32x16 acc[2][NJ];
        layer_mm_d<2, D2>(stream(k.Ffeat16, HW / 16, 2), HW / 16, smem, lane, acc, ring2f, nodrain);
        if constexpr (full) layer_prime_n<2, D2>(stream(k.FQ16, HW / 16, 2), ring2q);
        else layer_prime_n<1, D1>(stream(k.FQs16, HW / 16, 1), ring1q);
        __syncthreads();  // every wave is done reading H_L
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_G + f0);
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const float y[4] = {acc[a][j][4 * gq] + bv[0], acc[a][j][4 * gq + 1] + bv[1],
                                        acc[a][j][4 * gq + 2] + bv[2], acc[a][j][4 * gq + 3] + bv[3]};
                    put4(32 * j + er32, f0, y);
                }
            }
        __syncthreads();
    }
    // [sun1 | rgb1] = sin(W_Q feat + b + per-ray sun rows) → the image and DQ; feat leaves for G
    // in 8 slices behind Q's k-step groups.  The solar pass needs sun1 alone: its 256 features
    // over the 8 waves (32 each, the same MFMA per feature: the same sums), half the MFMAs
    u32x4 ring1s2[D1][1];  // sun_v 2's weights
    u32x4 afr[HH / 16 / 8];  // albedo's narrow A fragments
    if constexpr (!full) {
        f32x16 acc[1][NJ];
        const auto rsF = rsrc(g.G, g.ldG);
        layer_mm_d<1, D1>(stream(k.FQs16, HW / 16, 1), HW / 16, smem, lane, acc, ring1q,
                          [&](int grp) {
                              constexpr int PER = 16 / (HW / 16 / D1);  // feat's 16 chunks per thread over the groups
                              image_out<64, PER>(smem, rsF, g.ldG, tid, PER * grp);
                          });
        layer_prime_n<1, D1>(stream(k.Fs2_16, HH / 16, 1), ring1s2);
        __syncthreads();  // every wave is done reading feat (its copy-out included)
        const auto rsD = rsrc_r(g.DQ, g.ldQ);
        const int rlast = (int)(g.P - 1 - p0);  // P < 2^31 / 512 (host check)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            u32x2 yq[4];
            const int64_t ray = ((int)p0 + std::min(32 * j + er32, rlast)) / g.S;
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_Q + f0);
                // (RQ1: the tile's one ray's row staged in ost, f0 >> 3 = 4w + gq, f0 & 7 = 4·eh)
                const f32x4 rv = RQ1 ? *reinterpret_cast<const f32x4*>(ost + (4 * w + gq) * OST_LD + 8 + 4 * eh)
                                     : ld4(g.rbQ + ray * (2 * HH) + f0);
                float y[4], cs[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) sincos((acc[0][j][4 * gq + e] + bv[e]) + rv[e], &y[e], &cs[e]);
#if SPN_HEADS_DCOLS
                put4(32 * j + er32, f0, cs);
#else
                put4(32 * j + er32, f0, y);
#endif
                yq[gq] = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                if (!SPN_HEADS_DCOLS) yq[gq] = u32x2{pack2(cs[0], cs[1]), pack2(cs[2], cs[3])};
            }
#if SPN_HEADS_DCOLS
            cols_out<1>(smem, rsD, g.ldQ, 32 * w, j, lane);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                *reinterpret_cast<u32x2*>(smem + img_off(32 * j + er32, f0 >> 3) + 8 * ((f0 >> 2) & 1)) = yq[gq];
            }
#else
            store_rows16(rsD, g.ldQ, 32 * w, 32 * j + er32, eh, yq);
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
    } else {
        f32x16 acc[2][NJ];
        const auto rsF = rsrc(g.G, g.ldG);
        layer_mm_d<2, D2>(stream(k.FQ16, HW / 16, 2), HW / 16, smem, lane, acc, ring2q,
                           [&](int grp) {
                               constexpr int PER = 16 / (HW / 16 / D2);  // feat's 16 chunks per thread over Q's groups
                               image_out<64, PER>(smem, rsF, g.ldG, tid, PER * grp);
                           });
        layer_prime_n<1, D1>(stream(k.Fs2_16, HH / 16, 1), ring1s2);
        if (full) narrow_load<HH / 16 / 8>(P16 + k.Fnar16 + narrow_off(1), lane, w, afr);
        __syncthreads();  // every wave is done reading feat (its copy-out included)
        const auto rsD = rsrc_r(g.DQ, g.ldQ);
        const bool dq = full || w < 4;  // wave-uniform
        const int rlast = (int)(g.P - 1 - p0);  // P < 2^31 / 512 (host check)
#if SPN_HEADS_DCOLS
        // per point tile j: cos into the wave's own image columns, those rows out to DQ, then sin
        // over them (the sines wait in registers).  KOST: the tile's one ray's row of rbQ staged in
        // ost (no global load per feature group, whose wait would also wait for the D stores)
        auto qepi = [&](auto kost) {
            constexpr bool KOST = decltype(kost)::value;
            const float* rqb = ost + 8 * w * OST_LD + 8 + 4 * eh;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                u32x2 yq[2][4];
                const int64_t ray = ((int)p0 + std::min(32 * j + er32, rlast)) / g.S;
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                        const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_Q + f0);
                        // (f0 >> 3 = 8w + 4a + gq, f0 & 7 = 4·eh: one lane base, the group as an immediate)
                        const f32x4 rv = KOST ? *reinterpret_cast<const f32x4*>(rqb + (4 * a + gq) * OST_LD)
                                              : ld4(g.rbQ + ray * (2 * HH) + f0);
                        float y[4], cs[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) sincos((acc[a][j][4 * gq + e] + bv[e]) + rv[e], &y[e], &cs[e]);
                        put4(32 * j + er32, f0, cs);
                        yq[a][gq] = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                    }
                if (dq) cols_out<2>(smem, rsD, g.ldQ, 64 * w, j, lane);
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                        *reinterpret_cast<u32x2*>(smem + img_off(32 * j + er32, f0 >> 3) + 8 * ((f0 >> 2) & 1)) = yq[a][gq];
                    }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        qepi(std::integral_constant<bool, RQ1>{});
#else
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                u32x2 cq[4];
                const int64_t ray = ((int)p0 + std::min(32 * j + er32, rlast)) / g.S;
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                    const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_Q + f0);
                    const f32x4 rv = ld4(g.rbQ + ray * (2 * HH) + f0);
                    float y[4], cs[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) sincos((acc[a][j][4 * gq + e] + bv[e]) + rv[e], &y[e], &cs[e]);
                    put4(32 * j + er32, f0, y);
                    cq[gq] = u32x2{pack2(cs[0], cs[1]), pack2(cs[2], cs[3])};
                }
                if (dq) store_rows16(rsD, g.ldQ, 64 * w + 32 * a, 32 * j + er32, eh, cq);
                __builtin_amdgcn_sched_barrier(0);
            }
#endif
        __syncthreads();
    }
    if (full) {
        // semantic logits: the 8 waves' partials in wave order
        for (int i = opaque(tid); i < TM * C; i += 512) {
            const int r = i / C, c = i % C;
            float t = 0.f;
            for (int v = 0; v < 8; ++v) t += part[(v * TM + r) * 4 + c];
            ost[r * OST_LD + g.sem_col + c] = t + Pk[k.bm2 + c];
        }
        __syncthreads();  // the logits are read from part
        // albedo from rgb1 (image k-steps 16..31) on MFMA; its gates saved for the backward
        narrow_run<HH / 16 / 8>(afr, HH / 16, smem, lane, w, part);
        __syncthreads();
        const int r = opaque(tid);  // (row addresses computed here, not hoisted across the tile loop)
        if (r < TM) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float t = 0.f;
                for (int v = 0; v < 8; ++v) t += part[(v * TM + r) * 4 + c];
                const float gv = sigmoidf_(t + Pk[k.br2 + c]);
                ost[r * OST_LD + c] = __fsub_rn(__fmul_rn(gv, 1.002f), 0.001f);
                if (r < rows) g.hsave[(p0 + r) * 8 + 1 + c] = gv;
            }
        }
    }
    // sun_v 2 on image columns 0..255 → the image and DS2; Q leaves for HBM behind its k-step groups
    u32x4 ring1s3[D1][1];
    {
        f32x16 acc[1][NJ];
        const auto rsQ = rsrc(g.Q, g.ldQ);
        if (full)
            layer_mm_d<1, D1>(stream(k.Fs2_16, HH / 16, 1), HH / 16, smem, lane, acc, ring1s2,
                              [&](int grp) { image_out<64, 8>(smem, rsQ, g.ldQ, tid, 8 * grp); });
        else
            layer_mm_d<1, D1>(stream(k.Fs2_16, HH / 16, 1), HH / 16, smem, lane, acc, ring1s2,
                              [&](int grp) { image_out<32, 4>(smem, rsQ, g.ldQ, tid, 4 * grp); });
        layer_prime_n<1, D1>(stream(k.Fs3_16, HH / 16, 1), ring1s3);
        __syncthreads();  // every wave is done reading sun1 (and rgb1: the albedo head; Q's copy-out)
        const auto rsD = rsrc_r(g.DS2, HH);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            u32x2 cq[4];
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_S2 + f0);
                float y[4], cs[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) sincos(acc[0][j][4 * gq + e] + bv[e], &y[e], &cs[e]);
#if SPN_HEADS_DCOLS  // cos through the own columns, then sin over them (cq holds the sines)
                put4(32 * j + er32, f0, cs);
                cq[gq] = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
#else
                put4(32 * j + er32, f0, y);
                cq[gq] = u32x2{pack2(cs[0], cs[1]), pack2(cs[2], cs[3])};
#endif
            }
#if SPN_HEADS_DCOLS
            cols_out<1>(smem, rsD, HH, 32 * w, j, lane);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                *reinterpret_cast<u32x2*>(smem + img_off(32 * j + er32, f0 >> 3) + 8 * ((f0 >> 2) & 1)) = cq[gq];
            }
#else
            store_rows16(rsD, HH, 32 * w, 32 * j + er32, eh, cq);
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
    }
    // sun_v 3 → the image and DS3; S2 leaves behind its k-step groups
    u32x4 afs[HH / 16 / 8];  // the sun head's narrow A fragments
    {
        f32x16 acc[1][NJ];
        const auto rsS2 = rsrc(g.S2, HH);
        layer_mm_d<1, D1>(stream(k.Fs3_16, HH / 16, 1), HH / 16, smem, lane, acc, ring1s3,
                          [&](int grp) { image_out<32, 4>(smem, rsS2, HH, tid, 4 * grp); });
        narrow_load<HH / 16 / 8>(P16 + k.Fnar16 + narrow_off(2), lane, w, afs);
        __syncthreads();
        const auto rsD = rsrc_r(g.DS3, HH);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            u32x2 cq[4];
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                const f32x4 bv = *reinterpret_cast<const f32x4*>(sbias + SB_S3 + f0);
                float y[4], cs[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) sincos(acc[0][j][4 * gq + e] + bv[e], &y[e], &cs[e]);
#if SPN_HEADS_DCOLS  // cos through the own columns, then sin over them (cq holds the sines)
                put4(32 * j + er32, f0, cs);
                cq[gq] = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
#else
                put4(32 * j + er32, f0, y);
                cq[gq] = u32x2{pack2(cs[0], cs[1]), pack2(cs[2], cs[3])};
#endif
            }
#if SPN_HEADS_DCOLS
            cols_out<1>(smem, rsD, HH, 32 * w, j, lane);
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
                const int f0 = 32 * w + 8 * gq + 4 * eh;
                *reinterpret_cast<u32x2*>(smem + img_off(32 * j + er32, f0 >> 3) + 8 * ((f0 >> 2) & 1)) = cq[gq];
            }
#else
            store_rows16(rsD, HH, 32 * w, 32 * j + er32, eh, cq);
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
    }
    // the next tile's H_L rows start loading (into the caller's registers) under the last phases
    prefetch();
    // the sun visibility (MFMA) on S3, then S3 to HBM and, for the main pass, the ray's sky colour
    narrow_run<HH / 16 / 8>(afs, 0, smem, lane, w, part);
    image_out<32, 8>(smem, rsrc(g.S3, HH), HH, tid, 0);
    __syncthreads();
    const int r = opaque(tid);
    if (r < TM) {
        float t = 0.f;
        for (int v = 0; v < 8; ++v) t += part[(v * TM + r) * 4];
        const float sun = sigmoidf_(t + Pk[k.bs4]);
        ost[r * OST_LD + 4] = sun;
        if (r < rows) g.hsave[(p0 + r) * 8 + 4] = sun;
        if (full) {
            const float* sk = g.sky + (int64_t)((int)std::min<int64_t>(p0 + r, g.P - 1) / g.S) * 4;
#pragma unroll
            for (int c = 0; c < 3; ++c) ost[r * OST_LD + 5 + c] = sk[c];
        } else {
            for (int c = 0; c < g.NO; ++c)
                if (c != 3 && c != 4) ost[r * OST_LD + c] = 0.f;
        }
    }
    __syncthreads();
    for (int i = opaque(tid); i < rows * g.NO; i += 512) g.out[p0 * g.NO + i] = ost[(i / g.NO) * OST_LD + i % g.NO];
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
