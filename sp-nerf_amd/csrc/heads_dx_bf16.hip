// The training heads' dX chain in ONE persistent launch (bf16 MLP, W = 512, H = 256, no β) —
// the backward of models/spnerf.py:332-369 from the narrow heads' gradients to the trunk's top
// pre-activation gradient, a 64-point tile resident in LDS from the first GEMM to the last:
//
//   dS2  = (dS3 · Ws3) ⊙ DS2                     [256]   sun_v_net.4 → .2   (spnerf.py:358-360)
//   dZQs = (dS2 · Ws2) ⊙ DQ[:, :H]               [256]   sun_v_net.2 → .0
//   dF   = [dZQs | dZQ_rgb] · WQ                 [512]   Q = [sun_v.0 ; rgb.0] → feat (linear)
//   dZL  = ([dF | dZG_sem] · WG + dσ ⊗ w_σ) ⊙ D_L [512]  G = [feat ; semantic hidden] → H_L
//
// (the solar pass: K of Q = H, of G = W).  The layer-by-layer path runs these as four DMA GEMMs
// (k_gemm_nt_bf16d, two with the ×D epilogue, one with the rank-1 σ term), each writing its output
// to HBM and the next reading it back (≈ 3.5 KB per point of re-reads); here every intermediate
// stays in LDS and only what the weight gradients read (dS2, dZQ's sun half, dF) and dZL leave.
// The arithmetic is the GEMMs': the same 32x32x16 bf16 MFMAs over the K-steps of 16 in ascending
// order (weights and activations in swapped operand roles, as the fused forward heads), the
// epilogues' (acc + 0) [+ dσ·w_σ] [· D] in fp32, RNE to bf16 — bit for bit the GEMMs' outputs.
//
// Two [64][512] bf16 images A and B alternate as the MFMA B operand and the epilogues' target:
//   top   A ← [dS3 | DS2]
//   P1    dS3 (A) → B[:, 0:256) = dS2, ×DS2 from A[:, 256:512);   B[:, 256:512) ← DQ_s
//   P2    dS2 (B) → A[:, 0:256) = dZQs, ×DQ_s from B;             A[:, 256:512) ← dZQ_rgb
//   P3    dZQ (A) → B = dF;                                      A[:, 0:256) ← dZG_sem
//   P4    dF (B) then dZG_sem (A) → ×D_L (staged in B) → B = dZL
// Each input is loaded into registers one phase ahead and written into the free half of an image
// under a k-loop; each output leaves for HBM behind the next phase's k-step groups.  The weights
// (transposed, fragment order: PackedOffs Bs3_16 / Bs2_16 / BQ16 / BG16) stream from L2 through
// a register ring as the A operand, as in the fused trunk and heads.
#include <algorithm>

#include "heads_dx.h"

namespace spn {

#ifdef SPN_ABLATIONS   // measured slower than the four GEMMs: an ablation-build kernel

// option "heads_dx" (ablation build): 1 = this launch (where heads_dx_bf16_ok), 0 (default) = the four
// GEMMs — this launch measured slower in the step (C4 22.05 -> 22.26 ms, same call)
int g_heads_dx = 0;

#ifndef HDX_ABL
#define HDX_ABL 0  // profiling ablations (variant builds only, outputs invalid): 1 no copy-outs, 2 no input loads, 4 no MFMAs, 8 no epilogue math
#endif
#ifndef SPN_HDX_D1
#define SPN_HDX_D1 8
#endif
#ifndef SPN_HDX_D2
#define SPN_HDX_D2 4
#endif

namespace hx {

constexpr int TM = 64;                 // points per tile
constexpr int NJ = TM / 32;            // 32-point MFMA tiles per wave
constexpr int IMG = TM * 1024;         // a [64][512] bf16 image
constexpr int HW = 512, HH = 256;
constexpr int D1 = SPN_HDX_D1, D2 = SPN_HDX_D2;  // weight-ring depths of the 256-wide (NA 1) and 512-wide (NA 2) layers
constexpr int G1 = 16 / D1;                      // k-step groups of the 256-wide layers
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int img_off(int row, int ch) { return row * 1024 + ((ch ^ (row & 15)) << 4); }
// the 8-byte piece of 4 consecutive features f0.. (f0 % 4 == 0) of one row
__device__ __forceinline__ int img4(int row, int f0) { return img_off(row, f0 >> 3) + 8 * ((f0 >> 2) & 1); }

template <int NA, int DEPTH>
__device__ __forceinline__ void prime(const bf16* __restrict__ wsrc, u32x4 (&ring)[DEPTH][NA]) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
        for (int a = 0; a < NA; ++a) ring[d][a] = ldg16(wsrc + (d * NA + a) * 512);
}

// acc[a][j] (+)= Σ_ks W-fragment(ks) · image columns: k-steps [0, nks) of this wave's stream wsrc
// (NA fragments of 512 bf16 per k-step), k-step ks reading image img_of(ks) at its k-step kk_of(ks)
// (block-uniform per group of DEPTH k-steps); the ring holds the stream's next DEPTH k-steps and
// must be primed.  drain(group) runs after each group's refills.
template <int NA, int DEPTH, typename ImgOf, typename Drain>
__device__ __forceinline__ void kloop(const bf16* __restrict__ wsrc, int nks, ImgOf&& img_of, int lane,
                                      f32x16 (&acc)[NA][NJ], u32x4 (&ring)[DEPTH][NA], bool zero, Drain&& drain) {
    const int r32 = lane & 31, h = lane >> 5, sw = r32 & 15;
    if (zero) {
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
    }
#pragma unroll 1
    for (int ks0 = 0; ks0 < nks; ks0 += DEPTH) {
        int kk0;
        const char* img = img_of(ks0, &kk0);   // the group's image and its first k-step there
        const char* brow = img + r32 * 1024;
        bf16x8 bc[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) bc[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((2 * kk0 + h) ^ sw) * 16);
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int ks = ks0 + d, kk = kk0 + d;
            bf16x8 bn[NJ];
            if (d + 1 < DEPTH) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) bn[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((2 * (kk + 1) + h) ^ sw) * 16);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int a = 0; a < NA; ++a)
                    if (!(HDX_ABL & 4))
                        acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ring[d][a]), bc[j],
                                                                          acc[a][j], 0, 0, 0);
            const int kn = min(ks + DEPTH, nks - 1);
#pragma unroll
            for (int a = 0; a < NA; ++a) ring[d][a] = ldg16(wsrc + (kn * NA + a) * 512);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, NA, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x020, NA, 0);
            if (d + 1 < DEPTH) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) bc[j] = bn[j];
            }
        }
        drain(ks0 / DEPTH);
    }
}

}  // namespace hx

using namespace hx;

__global__ __launch_bounds__(512) void k_heads_dx_bf16(HeadsDxArgs g, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[2 * IMG + (HW + 2 * TM) * 4];
    char* const A = smem;
    char* const Bm = smem + IMG;
    float* const wsg = reinterpret_cast<float*>(smem + 2 * IMG);  // w_σ [512]
    float* const hs0 = wsg + HW;   // the tile's dσ [64], double-buffered by tile parity (the next tile's top
                                   // writes its rows while slower waves still read this tile's)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bool full = g.mode == 0, semk = full && g.sem;
    const int nksQ = full ? g.kQ / 16 : HH / 16;   // Q's K: [sun_v.0 | rgb.0] or sun_v.0 alone
    const int nksG = semk ? g.kG / 16 : HW / 16;   // G's K: [feat | semantic hidden] or feat alone
    const bf16* P16 = g.packed16;
    const int l8 = opaque(lane) * 8;
    const bf16* s3 = P16 + g.Bs3 + (int64_t)w * (HH / 16) * 512 + l8;
    const bf16* s2 = P16 + g.Bs2 + (int64_t)w * (HH / 16) * 512 + l8;
    const bf16* sq = P16 + g.BQ + (int64_t)w * (g.kQ / 16) * 2 * 512 + l8;
    const bf16* sg = P16 + g.BG + (int64_t)w * (g.kG / 16) * 2 * 512 + l8;
    for (int i = tid; i < HW; i += 512) wsg[i] = g.wsig[i];
    const int el = opaque(lane), er32 = el & 31, eh = el >> 5;

    // a tile's rows of a [P][ld] bf16 tensor from column c0: chunk c (16 B) of the NCH per row,
    // rows past P read a clamped row (never stored)
    auto ld_rows = [&](const bf16* base, int ld, int c0, int64_t p0, int nch, int c) -> u32x4 {
        const int row = c / nch, ch = c % nch;
        const bf16* src = base + std::min<int64_t>(p0 + row, g.P - 1) * ld + c0 + ch * 8;
        if (HDX_ABL & 2) return u32x4{0u, 0u, 0u, 0u};
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src));
    };
    // the rows of a [P][ld] tensor as a buffer resource (rows past P dropped; null: every store dropped)
    auto rsrc = [&](bf16* base, int ld, int64_t p0) {
        const int rows = (int)std::min<int64_t>(TM, g.P - p0);
        return __builtin_amdgcn_make_buffer_rsrc(base ? base + p0 * ld : g.dZL, 0, base ? rows * ld * 2 : 0, 0x00020000);
    };
    // image columns [8·ch0, 8·(ch0 + nch)) to columns [c0, ..) of the rows: chunks q0.. of this thread
    auto out_rows = [&](const char* img, __amdgpu_buffer_rsrc_t rs, int ld, int c0, int ch0, int nch, int q0, int n) {
        if (HDX_ABL & 1) return;
        const int t = opaque(tid);
        for (int q = q0; q < q0 + n; ++q) {
            const int c = t + 512 * q, row = c / nch, ch = c % nch;
            const u32x4 v = *reinterpret_cast<const u32x4*>(img + img_off(row, ch0 + ch));
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (row * ld + c0 + ch * 8) * 2, 0, 0);
        }
    };

    int tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;  // block-uniform
    // the next tile's [dS3 | DS2] rows (64 rows x 64 chunks: 8 per thread)
    u32x4 rA[8];
    auto load_top = [&](int64_t q0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int c = opaque(tid) + 512 * q;
            rA[q] = (c & 63) < 32 ? ld_rows(g.dS3, HH, 0, q0, 64, c) : ld_rows(g.DS2, HH, -32 * 8, q0, 64, c);
        }
    };
    load_top((int64_t)tile * TM);
    u32x4 ring1[D1][1];
    prime<1, D1>(s3, ring1);
    int64_t pp0 = -1;  // the previous tile (its dZL in B, copied out under this tile's P1)
    for (int it = 0; tile < ntiles; tile += gridDim.x, ++it) {
        const int64_t p0 = (int64_t)tile * TM;
        float* const hs = hs0 + (it & 1) * TM;
        const int64_t next = std::min(tile + (int)gridDim.x, ntiles - 1);
        {
            const int t = opaque(tid);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = t + 512 * q;
                *reinterpret_cast<u32x4*>(A + img_off(c >> 6, c & 63)) = rA[q];
            }
            if (t < TM) hs[t] = g.hpre[std::min<int64_t>(p0 + t, g.P - 1) * g.HP];
        }
        __syncthreads();  // A complete; B (the previous dZL) complete
        // ---- P1: dS2 = (dS3 · Ws3) ⊙ DS2 → B[:, 0:256); the previous dZL leaves under the k-loop
        u32x4 rq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) rq[q] = ld_rows(g.DQ, g.ldQ, 0, p0, 32, opaque(tid) + 512 * q);
        {
            f32x16 acc[1][NJ];
            const auto rsL = rsrc(pp0 >= 0 ? g.dZL : nullptr, HW, std::max<int64_t>(pp0, 0));
            kloop<1, D1>(s3, HH / 16, [&](int ks0, int* kk) { *kk = ks0; return (const char*)A; }, lane, acc, ring1, true,
                         [&](int grp) { out_rows(Bm, rsL, HW, 0, 0, 64, 8 * grp / G1, 8 * (grp + 1) / G1 - 8 * grp / G1); });
            prime<1, D1>(s2, ring1);
            __syncthreads();  // every wave is done reading dS3 (A) and the previous dZL (B)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int f0 = 32 * w + 8 * gq + 4 * eh, row = 32 * j + er32;
                    const f32x4 m = ld4(reinterpret_cast<const bf16*>(A + img4(row, HH + f0)));
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = (acc[0][j][4 * gq + e] + 0.f) * m[e];
                    *reinterpret_cast<u32x2*>(Bm + img4(row, f0)) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
                }
            const int t = opaque(tid);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int c = t + 512 * q;
                *reinterpret_cast<u32x4*>(Bm + img_off(c >> 5, 32 + (c & 31))) = rq[q];
            }
        }
        __syncthreads();  // B = [dS2 | DQ_s]
        // ---- P2: dZQs = (dS2 · Ws2) ⊙ DQ_s → A[:, 0:256); dS2 leaves; A[:, 256:512) ← dZQ_rgb
        u32x4 rr[4];
        if (full) {  // block-uniform
#pragma unroll
            for (int q = 0; q < 4; ++q) rr[q] = ld_rows(g.dZQ, g.ldQ, HH, p0, 32, opaque(tid) + 512 * q);
        }
        u32x4 ring2[D2][2];
        {
            f32x16 acc[1][NJ];
            const auto rsS2 = rsrc(g.dS2, HH, p0);
            kloop<1, D1>(s2, HH / 16, [&](int ks0, int* kk) { *kk = ks0; return (const char*)Bm; }, lane, acc, ring1, true,
                         [&](int grp) { out_rows(Bm, rsS2, HH, 0, 0, 32, 4 * grp / G1, 4 * (grp + 1) / G1 - 4 * grp / G1); });
            prime<2, D2>(sq, ring2);
            if (full) {
                const int t = opaque(tid);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = t + 512 * q;
                    *reinterpret_cast<u32x4*>(A + img_off(c >> 5, 32 + (c & 31))) = rr[q];
                }
            }
            __syncthreads();  // every wave is done reading dS2 (B), its copy-out included
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) {
                    const int f0 = 32 * w + 8 * gq + 4 * eh, row = 32 * j + er32;
                    const f32x4 m = ld4(reinterpret_cast<const bf16*>(Bm + img4(row, HH + f0)));
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = (acc[0][j][4 * gq + e] + 0.f) * m[e];
                    *reinterpret_cast<u32x2*>(A + img4(row, f0)) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
                }
        }
        __syncthreads();  // A = dZQ
        // ---- P3: dF = dZQ · WQ → B; dZQ's sun half leaves; A[:, 0:256) ← dZG_sem
        u32x4 rs[4];
        if (semk) {
#pragma unroll
            for (int q = 0; q < 4; ++q) rs[q] = ld_rows(g.dZG, g.ldG, HW, p0, 32, opaque(tid) + 512 * q);
        }
        {
            f32x16 acc[2][NJ];
            const auto rsQ = rsrc(g.dZQ, g.ldQ, p0);
            // the 4 chunks per thread spread over the k-step groups
            const int G3 = nksQ / D2;
            kloop<2, D2>(sq, nksQ, [&](int ks0, int* kk) { *kk = ks0; return (const char*)A; }, lane, acc, ring2, true,
                         [&](int grp) { out_rows(A, rsQ, g.ldQ, 0, 0, 32, 4 * grp / G3, 4 * (grp + 1) / G3 - 4 * grp / G3); });
            prime<2, D2>(sg, ring2);
            __syncthreads();  // every wave is done reading dZQ (A), its copy-out included
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh, row = 32 * j + er32;
                        float v[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * gq + e] + 0.f;
                        *reinterpret_cast<u32x2*>(Bm + img4(row, f0)) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
                    }
            if (semk) {
                const int t = opaque(tid);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = t + 512 * q;
                    *reinterpret_cast<u32x4*>(A + img_off(c >> 5, c & 31)) = rs[q];
                }
            }
        }
        __syncthreads();  // B = dF; A[:, 0:256) = dZG_sem
        // ---- P4: dZL = ([dF | dZG_sem] · WG + dσ ⊗ w_σ) ⊙ D_L → B; dF leaves
        u32x4 rd[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) rd[q] = ld_rows(g.DL, HW, 0, p0, 64, opaque(tid) + 512 * q);
        {
            f32x16 acc[2][NJ];
            const auto rsF = rsrc(g.dZG, g.ldG, p0);
            kloop<2, D2>(sg, nksG,
                         [&](int ks0, int* kk) {
                             *kk = ks0 < HW / 16 ? ks0 : ks0 - HW / 16;
                             return (const char*)(ks0 < HW / 16 ? Bm : A);
                         },
                         lane, acc, ring2, true,
                         [&](int grp) {
                             constexpr int G4 = HW / 16 / D2;   // the 8 chunks over dF's k-step groups
                             if (grp < G4) out_rows(Bm, rsF, g.ldG, 0, 0, 64, 8 * grp / G4, 8 * (grp + 1) / G4 - 8 * grp / G4);
                         });
            // the next tile's [dS3 | DS2] rows (past the last tile: this tile's rows again, never used)
            load_top(next * TM);
            __syncthreads();  // every wave is done reading dF (B), its copy-out, and A
            {
                const int t = opaque(tid);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int c = t + 512 * q;
                    *reinterpret_cast<u32x4*>(Bm + img_off(c >> 6, c & 63)) = rd[q];
                }
            }
            __syncthreads();  // B = D_L
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh, row = 32 * j + er32;
                        const f32x4 m = ld4(reinterpret_cast<const bf16*>(Bm + img4(row, f0)));
                        const f32x4 wv = *reinterpret_cast<const f32x4*>(wsg + f0);
                        const float hv = hs[row];
                        float v[4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            v[e] = acc[a][j][4 * gq + e] + 0.f;
                            v[e] += hv * wv[e];
                            v[e] *= m[e];
                        }
                        *reinterpret_cast<u32x2*>(Bm + img4(row, f0)) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
                    }
        }
        prime<1, D1>(s3, ring1);   // the next tile's P1 stream
        pp0 = p0;
    }
    __syncthreads();  // the last tile's dZL is complete
    out_rows(Bm, rsrc(g.dZL, HW, pp0), HW, 0, 0, 64, 0, 8);
}

bool heads_dx_bf16_ok(const HeadsDxArgs& a) {
    return a.packed16 && a.Bs3 >= 0 && a.Bs2 >= 0 && a.BQ >= 0 && a.BG >= 0 && (a.mode == 0 || a.mode == 2) &&
           a.kQ == 2 * HH && a.kG == (a.sem ? HW + HH : HW) && a.ldQ == a.kQ && a.ldG == a.kG && a.dS3 && a.DS2 && a.DQ &&
           a.dS2 && a.dZQ && a.dZG && a.dZL && a.DL && a.hpre && a.wsig;
}

int32_t heads_dx_bf16(const HeadsDxArgs& a, hipStream_t s, double flop, double bytes) {
    SPN_ARG(heads_dx_bf16_ok(a), "heads_dx_bf16: bad arguments");
    if (a.P == 0) return SPNERF_OK;
    SPN_ARG(a.P < (1ll << 31) / HW, "heads_dx_bf16: too many points (%lld)", (long long)a.P);
    const int ntiles = cdiv(a.P, TM);
    ProfScope prof("heads_dx", s, flop, bytes);
    hipLaunchKernelGGL(k_heads_dx_bf16, dim3(std::min(ntiles, num_cus())), dim3(512), 0, s, a, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

#else   // product build: the heads' dX runs as the four GEMMs
int g_heads_dx = 0;
bool heads_dx_bf16_ok(const HeadsDxArgs&) { return false; }
int32_t heads_dx_bf16(const HeadsDxArgs&, hipStream_t, double, double) {
    SPN_ARG(false, "heads_dx_bf16: the fused heads dX chain is an ablation-build kernel (-DSPN_ABLATIONS)");
    return SPNERF_OK;
}
#endif

}  // namespace spn
