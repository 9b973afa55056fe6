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

#include "heads_tile.h"

namespace spn {

int g_fused_heads = 1;
int g_heads_dbg = 0;

using namespace hd;
constexpr int OST_OFF = IMG;
constexpr int PART_OFF = OST_OFF + OST_BYTES;
constexpr int RQ_OFF = PART_OFF + PART_BYTES;
constexpr int LDS = RQ_OFF + RQ_BYTES;

__global__ __launch_bounds__(512) void k_heads_bf16(HeadsFusedArgs g, PackedOffs k, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int tid = threadIdx.x;
    float* ost = reinterpret_cast<float*>(smem + OST_OFF);
    float* part = reinterpret_cast<float*>(smem + PART_OFF);
    float* srq = reinterpret_cast<float*>(smem + RQ_OFF);
    for (int tile = xcd_remap(blockIdx.x, gridDim.x); tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TM;
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
        heads_tile<true>(g, k, smem, ost, part, srq, p0);
        __syncthreads();  // the next tile restages the image
    }
}

// Training (option heads_epi 2): the same tile loop with hd::heads_tile_train — H_L staged from
// HBM (the saving trunk writes it for the weight gradients anyway), σ from the trunk's hsave[p·8],
// every activation the backward reads stored, the layers' biases staged once in the RQ area.  Its
// own launch keeps the heads' registers out of the trunk's allocation: inside the trunk launch
// the trunk's tile loop spilled (64-bit values reloaded from scratch behind the copy-out stores)
// and the main pass took 5.78 ms against 2.78 + 1.72 ms for the two launches.
static_assert(SB_N * 4 <= RQ_BYTES, "the training heads' biases in the RQ area");
template <bool RQ1, bool SOL>
__global__ __launch_bounds__(512) void k_heads_train_bf16(HeadsFusedArgs g, PackedOffs k, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[LDS];
    const int tid = threadIdx.x;
    float* ost = reinterpret_cast<float*>(smem + OST_OFF);
    float* part = reinterpret_cast<float*>(smem + PART_OFF);
    float* sbias = reinterpret_cast<float*>(smem + RQ_OFF);
    for (int i = tid; i < SB_N; i += 512) {
        const float* P = g.packed;
        sbias[i] = i < SB_Q ? (g.C > 0 || i < HW ? P[k.bG + i] : 0.f)
                 : i < SB_S2 ? P[k.bQ + (i - SB_Q)] : i < SB_S3 ? P[k.bs2 + (i - SB_S2)] : P[k.bs3 + (i - SB_S3)];
    }
    __syncthreads();
    // H_L rows of a tile into registers (the next tile's under the current tile's last phases)
    u32x4 hv[16];
    auto load_hl = [&](int64_t q0) {
        const int t = opaque(tid);
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = t + 512 * q, row = c >> 6, ch = c & 63;
            hv[q] = *reinterpret_cast<const u32x4*>(g.HL + std::min<int64_t>(q0 + row, g.P - 1) * HW + ch * 8);
        }
    };
    int tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile < ntiles) load_hl((int64_t)tile * TM);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TM;
        {
            const int t = opaque(tid);
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int c = t + 512 * q, row = c >> 6, ch = c & 63;
                *reinterpret_cast<u32x4*>(smem + img_off(row, ch)) = hv[q];
            }
        }
        const int r = opaque(tid);
        if (r < TM) ost[r * OST_LD + 3] = softplusf_(g.hsave[std::min<int64_t>(p0 + r, g.P - 1) * 8]);
        if constexpr (RQ1) stage_rows_ost(g, k, ost, p0, tid);
        __syncthreads();
        const int next = tile + (int)gridDim.x;
        // (past the last tile: this tile's rows again, never stored — no branch around the loads)
        heads_tile_train<RQ1, SOL>(g, k, smem, ost, part, sbias, p0, [&] { load_hl((int64_t)std::min(next, ntiles - 1) * TM); });
        __syncthreads();  // the next tile restages the image
    }
}

bool heads_train_bf16_ok(const HeadsFusedArgs& h, const PackedOffs& k) {
    return h.HL && (h.mode == 0 || h.mode == 2) && h.NO <= OST_LD && h.C <= 3 && h.G && h.Q && h.DQ && h.S2 && h.DS2 &&
           h.S3 && h.DS3 && h.hsave && (h.mode != 0 || h.C == 0 || h.DG) && h.ldG % 8 == 0 && h.ldQ % 8 == 0 &&
           k.Fnar16 >= 0 && k.Ffeat16 >= 0 && k.FQ16 >= 0 && k.FQs16 >= 0 && k.Fs2_16 >= 0 && k.Fs3_16 >= 0 &&
           (h.C == 0 || k.Fsem16 >= 0);
}

int32_t heads_train_bf16(const HeadsFusedArgs& a, const PackedOffs& k, hipStream_t s, double flop, double bytes) {
    SPN_ARG(a.P >= 0 && a.S > 0 && heads_train_bf16_ok(a, k), "heads_train_bf16: bad arguments");
    if (a.P == 0) return SPNERF_OK;
    SPN_ARG(a.P < (1ll << 31) / HW, "heads_train_bf16: too many points (%lld)", (long long)a.P);
    const int ntiles = (int)((a.P + TM - 1) / TM);
    HeadsFusedArgs ad = a;
    ad.nt = 0;
#ifdef SPN_ABLATIONS
    ad.dbg = g_heads_dbg;
#else
    ad.dbg = 0;
#endif
    ProfScope prof("heads_train", s, flop, bytes);
    // every 128-point tile within one ray (S a multiple of 128): the Q epilogue's per-ray rows from LDS
    // the solar pass (mode 2) in its own instance (sun1 alone in Q: half its MFMAs)
    const dim3 grid(std::min(ntiles, num_cus())), block(512);
    const bool rq1 = SPN_HEADS_RQ_OST && a.S % TM == 0;
    if (a.mode == 2) {
        if (rq1) hipLaunchKernelGGL((k_heads_train_bf16<true, true>), grid, block, 0, s, ad, k, ntiles);
        else hipLaunchKernelGGL((k_heads_train_bf16<false, true>), grid, block, 0, s, ad, k, ntiles);
    } else {
        if (rq1) hipLaunchKernelGGL((k_heads_train_bf16<true, false>), grid, block, 0, s, ad, k, ntiles);
        else hipLaunchKernelGGL((k_heads_train_bf16<false, false>), grid, block, 0, s, ad, k, ntiles);
    }
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
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
    SPN_ARG(a.P < (1ll << 31) / HW, "heads_bf16: too many points (%lld)", (long long)a.P);
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
