// Fused inference heads of the bf16 MLP (cfg.dtype = 1, W = 512, no β): everything after the
// trunk's last layer (models/spnerf.py:332-367) in ONE persistent launch, a tile of 128 points
// resident in LDS from the trunk output to the output row — instead of four GEMMs writing the
// G / Q / sun_v activations to HBM (≈5 KB per point) and a heads kernel reading them back.
//
//   σ        = softplus(w_σ · H + b_σ)                (narrow_mm: a 32-row MFMA, hi/lo weight rows)
//   semh     = sin(W_m1 H + b_m1)          [256]  → logits = W_m2 semh + b_m2 in its epilogue
//   feat     = W_f H + b_f                 [512]  → the image
//   [s1 | r1]= sin(W_Q feat + b_Q + sun rows[ray])  [256 | 256] → the image
//   albedo   = sigmoid(W_r2 r1 + b_r2)·1.002 − 0.001                     (narrow_mm)
//   s2, s3   = sin(W_s2 s1 + b), sin(W_s3 s2 + b)   [256] → image columns 0..255
//   sun      = sigmoid(w_s4 · s3 + b)                                    (narrow_mm)
//   sky      = the ray's sky colour (per-ray rows)
//
// The GEMM layers use the fused trunk's formulation (trunk_bf16.hip): weights are the MFMA A
// operand streamed from L2 in fragment order (frag_off) through a 4-deep register ring, the
// [128][512] bf16 activation image (16-B chunks XOR-swizzled by row) the B operand, a
// 32x32x16 accumulator holds 4 runs of 4 consecutive features of one point; 8 waves own 64
// (512-wide layers) or 32 (256-wide layers) output features each.  Activations round to bf16
// like the layer-by-layer path's GEMM outputs.  The narrow heads (σ, albedo, sun: 1–3 outputs)
// are 32-row MFMA tiles whose rows are the bf16 hi and lo halves of the fp32 weight rows, K split
// over the 8 waves and the partials summed in wave order (other summation order than
// k_heads_fwd_v: not bit-identical, within bf16 rounding); as per-point dot products with wave
// reductions they took a quarter of the kernel.
#include <algorithm>

#include "mlp_layout.h"
#include "trunk.h"

namespace spn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

int g_fused_heads = 1;
int g_heads_dbg = 0;

namespace {
constexpr int TM = 128;                 // points per tile
constexpr int HW = 512, HH = 256;
constexpr int NJ = TM / 32;             // 32-point MFMA tiles per wave
constexpr int TPD = 4;                  // weight prefetch depth (k-steps)
constexpr int IMG = TM * HW * 2;        // the [128][512] bf16 image
constexpr int OST_LD = 16;              // output staging row (floats), NO <= 16
constexpr int OST_OFF = IMG;
constexpr int PART_OFF = OST_OFF + TM * OST_LD * 4;
constexpr int RQ_OFF = PART_OFF + 8 * TM * 4 * 4;  // semantic partials [wave][point][4]
constexpr int RQ_RAYS = 4;                         // per-ray Q rows staged for tiles of <= 4 rays
constexpr int LDS = RQ_OFF + RQ_RAYS * 2 * HH * 4;

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

}  // namespace

__global__ __launch_bounds__(512) void k_heads_bf16(HeadsFusedArgs g, PackedOffs k, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    float* ost = reinterpret_cast<float*>(smem + OST_OFF);
    float* part = reinterpret_cast<float*>(smem + PART_OFF);
    float* srq = reinterpret_cast<float*>(smem + RQ_OFF);
    const float* Pk = g.packed;
    const bf16* P16 = reinterpret_cast<const bf16*>(g.packed);
    const bool full = g.mode == 0;
    const int C = g.C;

    // this wave's fragment streams (NA · 1 KB per k-step)
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

    for (int tile = xcd_remap(blockIdx.x, gridDim.x); tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TM;
        // the tile's rays' sun rows of Q into LDS when they are few (one ray per tile at 128
        // samples per ray): the Q epilogue then reads LDS instead of an L2 round trip per row
        const int64_t ray0 = p0 / g.S;
        const int nray = (int)((std::min<int64_t>(p0 + TM, g.P) - 1) / g.S - ray0) + 1;
        const bool rq_lds = full && nray <= RQ_RAYS && !(g.dbg & 4);  // block-uniform (dbg 4: A/B)
        if (rq_lds)
            for (int i = tid; i < nray * 2 * HH; i += 512) srq[i] = g.rbQ[ray0 * (2 * HH) + i];
        // stage H_L (rows past P read a clamped row; their outputs are never stored)
#pragma unroll
        for (int q0 = 0; q0 < 16; q0 += 8) {
            u32x4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = tid + 512 * (q0 + q), row = c >> 6, ch = c & 63;
                const u32x4* src = reinterpret_cast<const u32x4*>(g.HL + std::min<int64_t>(p0 + row, g.P - 1) * HW + ch * 8);
                v[q] = (g.dbg & 2) ? u32x4{0u, 0u, 0u, 0u} : g.nt ? __builtin_nontemporal_load(src) : *src;  // block-uniform
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = tid + 512 * (q0 + q), row = c >> 6, ch = c & 63;
                *reinterpret_cast<u32x4*>(smem + img_off(row, ch)) = v[q];
            }
        }
        __syncthreads();

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
        __syncthreads();  // the next tile restages the image
    }
}

bool heads_bf16_shape_ok(const Dims& d) {
    return d.bf && d.W == HW && d.H == HH && !d.beta && d.C <= 4 && d.NQ == 2 * d.H && d.NO <= OST_LD && d.sem_col == 8;
}
bool heads_bf16_supported(const Dims& d) { return g_fused_heads && heads_bf16_shape_ok(d); }

int32_t heads_bf16(const HeadsFusedArgs& a, const PackedOffs& k, hipStream_t s, double flop, double bytes) {
    SPN_ARG(a.P >= 0 && a.S > 0 && a.NO <= OST_LD && a.C <= 4, "heads_bf16: bad sizes");
    SPN_ARG(k.Fnar16 >= 0, "heads_bf16: narrow heads not packed");
    SPN_ARG(a.mode == 1 || (k.Ffeat16 >= 0 && k.FQ16 >= 0 && k.Fs2_16 >= 0 && k.Fs3_16 >= 0 && (a.C == 0 || k.Fsem16 >= 0)),
            "heads_bf16: weights not packed for the fused heads");
    if (a.P == 0) return SPNERF_OK;
    const int ntiles = (int)((a.P + TM - 1) / TM);
    HeadsFusedArgs ad = a;
    ad.nt = (g_trunk_nt >> 1) & 1;
    ad.dbg = g_heads_dbg;
    ProfScope prof("heads_fused", s, flop, bytes);
    hipLaunchKernelGGL(k_heads_bf16, dim3(std::min(ntiles, num_cus())), dim3(512), 0, s, ad, k, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

}  // namespace spn
