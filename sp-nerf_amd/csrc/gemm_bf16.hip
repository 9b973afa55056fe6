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
//    activation is ever transposed in HBM.  Points are split over blocks into fp32 slabs
//    reduced in a fixed order by k_reduce_slabs (deterministic).
#include <algorithm>

#include "common.h"
#include "gemm_bf16.h"

namespace spn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int HB = 128, HK = 64, HLK = HK + 8;  // NT LDS row: 72 bf16 = 144 B

// ------------------------------------------------------------------------------------------
// NT
// ------------------------------------------------------------------------------------------
// Persistent over tiles: block b walks tiles slot(b), slot(b) + G, ... (slot = XCD-aware remap,
// so the column tiles of a row block run together on one XCD and share its L2).  The first
// K-step of the next tile is loaded before the current tile's epilogue, so the epilogue's
// stores overlap the next tile's load latency (two co-resident blocks otherwise run in lockstep
// and never overlap loop and epilogue).  PF = register prefetch depth in K-steps (1 or 2).
template <int PF>
__global__ __launch_bounds__(256) void k_gemm_nt_bf16(NT16Args g, int ntiles) {
    __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * HB * HLK];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nN = (g.N + HB - 1) / HB;
    const int G = gridDim.x;
    const int lr = tid >> 3, lc = (tid & 7) * 8;  // loader: row (+32 i), bf16 column within the K-step
    int t = xcd_remap(blockIdx.x, G);
    if (t >= ntiles) return;  // block-uniform

    // Loads are unconditional (no branch → no per-load vmcnt(0)): rows past M / columns past N
    // read a clamped row (they only feed output rows / columns that are never stored); the K
    // tail past K is zeroed when the registers are written to LDS, after the K-step's MFMAs, so
    // the loads stay in flight across them.  K1 is a multiple of the K-step, so the A / A2
    // segment is uniform per step.
    const int lda1 = g.lda, lda2 = g.lda2, K1 = g.K1, Kt = g.K;
    struct Regs {
        u32x4 a[4], b[4];
        bool kin;
    };
    auto gload = [&](Regs& r, int tile, int k0) {
        const int bm = (tile / nN) * HB, bn = (tile % nN) * HB;
        const int k = k0 + lc;
        r.kin = k < Kt;
        const int kc = r.kin ? k : Kt - 8;
        const bool seg2 = k0 >= K1;
        const bf16* pa = seg2 ? g.A2 + (kc - K1) : g.A + kc;
        const int lda = seg2 ? lda2 : lda1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = min(bm + lr + 32 * i, g.M - 1);
            r.a[i] = ldg16(pa + (int64_t)row * lda);
            const int col = min(bn + lr + 32 * i, g.N - 1);
            r.b[i] = ldg16(g.B + (int64_t)col * g.ldb + kc);
        }
    };
    auto sstore = [&](const Regs& r, int stg) {
        bf16* sA = smem + stg * 2 * HB * HLK;
        bf16* sB = sA + HB * HLK;
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            *reinterpret_cast<u32x4*>(sA + (lr + 32 * i) * HLK + lc) = r.kin ? r.a[i] : z;
            *reinterpret_cast<u32x4*>(sB + (lr + 32 * i) * HLK + lc) = r.kin ? r.b[i] : z;
        }
    };

    f32x16 acc[2][2];
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

    // Epilogue geometry: a wave owns 64 rows x 64 columns, staged 32 rows at a time as a
    // [32][68] fp32 image in its own LDS slice; lane (lane & 7) owns columns cq..cq+7 of rows
    // (lane >> 3) + 8 q4, so each store instruction writes 8 full 128-B row segments.
    const int cq = (lane & 7) * 8;
    constexpr int SLD = 68;
    float* stage = reinterpret_cast<float*>(smem) + wid * (32 * SLD);
    const int nk = (g.K + HK - 1) / HK;

    Regs r0, r1;
    gload(r0, t, 0);
    if constexpr (PF == 2) gload(r1, t, min(1, nk - 1) * HK);
    sstore(r0, 0);
    __syncthreads();
    while (true) {
        const int bm = (t / nN) * HB, bn = (t % nN) * HB;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        // No branch around a load (a join point makes hipcc drain vmcnt(0)): past the last
        // K-step the loader re-reads the last step (L2 hit, never computed on).
        if constexpr (PF == 1) {
            for (int kt = 0; kt < nk; ++kt) {
                gload(r0, t, min(kt + 1, nk - 1) * HK);
                __builtin_amdgcn_sched_barrier(0);  // issue the loads before the MFMAs
                compute(kt & 1);
                __builtin_amdgcn_sched_barrier(0);  // LDS writes (and their vmcnt waits) after the MFMAs
                sstore(r0, (kt + 1) & 1);
                __syncthreads();
            }
        } else {
            int kt = 0;
            for (; kt + 1 < nk; kt += 2) {
                gload(r0, t, min(kt + 2, nk - 1) * HK);
                __builtin_amdgcn_sched_barrier(0);
                compute(0);
                __builtin_amdgcn_sched_barrier(0);
                sstore(r1, 1);
                __syncthreads();
                gload(r1, t, min(kt + 3, nk - 1) * HK);
                __builtin_amdgcn_sched_barrier(0);
                compute(1);
                __builtin_amdgcn_sched_barrier(0);
                sstore(r0, 0);
                __syncthreads();
            }
            if (kt < nk) {  // odd step count: the last step sits in stage 0
                compute(0);
                __syncthreads();  // the epilogue reuses stage 0
            }
        }
        // next tile: its first K-step(s) load during this tile's epilogue (clamped, unconditional)
        const int tn = t + G;
        const bool more = tn < ntiles;
        const int tl = more ? tn : t;
        gload(r0, tl, 0);
        if constexpr (PF == 2) gload(r1, tl, min(1, nk - 1) * HK);

        // ---- epilogue of tile t: all global loads first (vmcnt counts loads and stores in
        // issue order, so a load issued after a store would wait for the store)
        const int col = bn + wc * 64 + cq;
        const bool colok = col < g.N;
        const int colc = colok ? col : g.N - 8;
        float bias8[8], r1v8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            bias8[e] = g.bias ? g.bias[colc + e] : 0.f;
            r1v8[e] = g.r1_a ? g.r1_v[colc + e] : 0.f;
        }
        u32x4 dm[2][4];
        float r1a[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int row = min(bm + wr * 64 + i * 32 + (lane >> 3) + 8 * q4, g.M - 1);
                dm[i][q4] = g.Dmul ? ldg16(g.Dmul + (int64_t)row * g.ld_dmul + colc) : u32x4{0u, 0u, 0u, 0u};
                r1a[i][q4] = g.r1_a ? g.r1_a[(int64_t)row * g.r1_lda] : 0.f;
            }
        const bool sine_cols = g.act == 1 && col >= g.n_lin;  // n_lin is a multiple of 8
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * h) * SLD + j * 32 + r32] = acc[i][j][r];
            wave_lds_sync();
            u32x4 oc[4], od[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int rr = (lane >> 3) + 8 * q4;
                const int row = bm + wr * 64 + i * 32 + rr;
                float v[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = stage[rr * SLD + cq + e] + bias8[e];
                if (g.rowbias) {
                    const float* rb = g.rowbias + (int64_t)(min(row, g.M - 1) / g.rows_per_ray) * g.ld_rb + colc;
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += rb[e];
                }
                if (g.r1_a) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += r1a[i][q4] * r1v8[e];
                }
                float d[8];
                if (sine_cols) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float sn, cs;
                        const float z = g.zround ? zr16(v[e]) : v[e];
                        fast_sincos(g.w0 * z, &sn, &cs);
                        v[e] = sn;
                        d[e] = g.dout_z ? z : g.w0 * cs;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) d[e] = 1.f;
                }
                if (g.Dmul) {
                    float m[8];
                    if (g.dmul_z) {  // Dmul holds the saved Z (fp16): D = cos(Z)
                        unpack8_f16(dm[i][q4], m);
#pragma unroll
                        for (int e = 0; e < 8; ++e) m[e] = fast_cos(m[e]);
                    } else {
                        unpack8(dm[i][q4], m);
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] *= m[e];
                }
                oc[q4] = pack8(v);
                od[q4] = g.dout_z ? pack8_f16(d) : pack8(d);
            }
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int row = bm + wr * 64 + i * 32 + (lane >> 3) + 8 * q4;
                if (row < g.M && colok) {
                    *reinterpret_cast<u32x4*>(g.C + (int64_t)row * g.ldc + col) = oc[q4];
                    if (g.Dout && sine_cols) *reinterpret_cast<u32x4*>(g.Dout + (int64_t)row * g.ld_dout + col) = od[q4];
                }
            }
        }
        if (!more) break;  // block-uniform
        __syncthreads();   // every wave is done with its staging slice
        sstore(r0, 0);
        __syncthreads();
        t = tn;
    }
}

// Generalised NT tile: BM x BN per block, WGM x WGN waves each owning (BM/WGM) x (BN/WGN) =
// MI x NJ 32x32 MFMA tiles.  Bigger wave tiles re-use every LDS fragment more (LDS bytes per
// MFMA: (MI + NJ) / (MI · NJ) KB) and bigger block tiles halve the L2 re-reads of the weights;
// with 256 x 256 / 8 waves one block fills a CU (147 KB of LDS).  Same loader, fences,
// persistence and store-last epilogue as k_gemm_nt_bf16.
template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN) void k_gemm_nt_bf16w(NT16Args g, int ntiles) {
    constexpr int T = 64 * WGM * WGN;
    constexpr int MI = BM / WGM / 32, NJ = BN / WGN / 32;
    constexpr int RP = T / 8;                       // rows per loader pass (8 16-B chunks per row)
    constexpr int PA = BM / RP, PB = BN / RP;       // loader passes per operand
    static_assert(BM % RP == 0 && BN % RP == 0, "loader geometry");
    __shared__ __attribute__((aligned(16))) bf16 smem[2 * (BM + BN) * HLK];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nN = (g.N + BN - 1) / BN;
    const int G = gridDim.x;
    const int lr = tid >> 3, lc = (tid & 7) * 8;
    int t = xcd_remap(blockIdx.x, G);
    if (t >= ntiles) return;  // block-uniform

    const int lda1 = g.lda, lda2 = g.lda2, K1 = g.K1, Kt = g.K;
    struct Regs {
        u32x4 a[PA], b[PB];
        bool kin;
    };
    auto gload = [&](Regs& r, int tile, int k0) {
        const int bm = (tile / nN) * BM, bn = (tile % nN) * BN;
        const int k = k0 + lc;
        r.kin = k < Kt;
        const int kc = r.kin ? k : Kt - 8;
        const bool seg2 = k0 >= K1;
        const bf16* pa = seg2 ? g.A2 + (kc - K1) : g.A + kc;
        const int lda = seg2 ? lda2 : lda1;
#pragma unroll
        for (int i = 0; i < PA; ++i) r.a[i] = ldg16(pa + (int64_t)min(bm + lr + RP * i, g.M - 1) * lda);
#pragma unroll
        for (int i = 0; i < PB; ++i) r.b[i] = ldg16(g.B + (int64_t)min(bn + lr + RP * i, g.N - 1) * g.ldb + kc);
    };
    auto sstore = [&](const Regs& r, int stg) {
        bf16* sA = smem + stg * (BM + BN) * HLK;
        bf16* sB = sA + BM * HLK;
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < PA; ++i) *reinterpret_cast<u32x4*>(sA + (lr + RP * i) * HLK + lc) = r.kin ? r.a[i] : z;
#pragma unroll
        for (int i = 0; i < PB; ++i) *reinterpret_cast<u32x4*>(sB + (lr + RP * i) * HLK + lc) = r.kin ? r.b[i] : z;
    };

    f32x16 acc[MI][NJ];
    const int wr = wid / WGN, wc = wid % WGN, r32 = lane & 31, h = lane >> 5;
    auto compute = [&](int stg) {
        const bf16* sA = smem + stg * (BM + BN) * HLK + (wr * MI * 32 + r32) * HLK + 8 * h;
        const bf16* sB = smem + stg * (BM + BN) * HLK + BM * HLK + (wc * NJ * 32 + r32) * HLK + 8 * h;
#pragma unroll
        for (int ks = 0; ks < HK / 16; ++ks) {
            bf16x8 a[MI], b[NJ];
#pragma unroll
            for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(sA + i * 32 * HLK + 16 * ks);
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(sB + j * 32 * HLK + 16 * ks);
#pragma unroll
            for (int i = 0; i < MI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    };

    const int cq = (lane & 7) * 8;
    constexpr int SLD = 68;
    static_assert(WGM * WGN * 32 * SLD * 4 <= 2 * (BM + BN) * HLK * 2, "epilogue staging fits in the LDS");
    float* stage = reinterpret_cast<float*>(smem) + wid * (32 * SLD);
    const int nk = (g.K + HK - 1) / HK;

    Regs r0;
    gload(r0, t, 0);
    sstore(r0, 0);
    __syncthreads();
    while (true) {
        const int bm = (t / nN) * BM, bn = (t % nN) * BN;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        for (int kt = 0; kt < nk; ++kt) {
            gload(r0, t, min(kt + 1, nk - 1) * HK);
            __builtin_amdgcn_sched_barrier(0);
            compute(kt & 1);
            __builtin_amdgcn_sched_barrier(0);
            sstore(r0, (kt + 1) & 1);
            __syncthreads();
        }
        const int tn = t + G;
        const bool more = tn < ntiles;
        gload(r0, more ? tn : t, 0);

        // epilogue: the wave's (MI·32) x (NJ·32) outputs, 32 rows x 64 columns at a time
        const int col0 = bn + wc * NJ * 32;
        float bias8[NJ / 2][8], r1v8[NJ / 2][8];
#pragma unroll
        for (int jp = 0; jp < NJ / 2; ++jp) {
            const int colc = min(col0 + 64 * jp + cq, g.N - 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                bias8[jp][e] = g.bias ? g.bias[colc + e] : 0.f;
                r1v8[jp][e] = g.r1_a ? g.r1_v[colc + e] : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#pragma unroll
            for (int jp = 0; jp < NJ / 2; ++jp) {
                const int col = col0 + 64 * jp + cq;
                const bool colok = col < g.N;
                const int colc = colok ? col : g.N - 8;
                // global loads of this 32 x 64 piece before its stores
                u32x4 dm[4];
                float r1a[4];
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int row = min(bm + wr * MI * 32 + i * 32 + (lane >> 3) + 8 * q4, g.M - 1);
                    dm[q4] = g.Dmul ? ldg16(g.Dmul + (int64_t)row * g.ld_dmul + colc) : u32x4{0u, 0u, 0u, 0u};
                    r1a[q4] = g.r1_a ? g.r1_a[(int64_t)row * g.r1_lda] : 0.f;
                }
                wave_lds_sync();
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        stage[((r & 3) + 8 * (r >> 2) + 4 * h) * SLD + j2 * 32 + r32] = acc[i][2 * jp + j2][r];
                wave_lds_sync();
                const bool sine_cols = g.act == 1 && col >= g.n_lin;
                u32x4 oc[4], od[4];
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int rr = (lane >> 3) + 8 * q4;
                    const int row = bm + wr * MI * 32 + i * 32 + rr;
                    float v[8], d[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = stage[rr * SLD + cq + e] + bias8[jp][e];
                    if (g.rowbias) {
                        const float* rb = g.rowbias + (int64_t)(min(row, g.M - 1) / g.rows_per_ray) * g.ld_rb + colc;
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] += rb[e];
                    }
                    if (g.r1_a) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] += r1a[q4] * r1v8[jp][e];
                    }
                    if (sine_cols) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            float sn, cs;
                            const float z = g.zround ? zr16(v[e]) : v[e];
                            fast_sincos(g.w0 * z, &sn, &cs);
                            v[e] = sn;
                            d[e] = g.dout_z ? z : g.w0 * cs;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) d[e] = 1.f;
                    }
                    if (g.Dmul) {
                        float m[8];
                        if (g.dmul_z) {  // Dmul holds the saved Z (fp16): D = cos(Z)
                            unpack8_f16(dm[q4], m);
#pragma unroll
                            for (int e = 0; e < 8; ++e) m[e] = fast_cos(m[e]);
                        } else {
                            unpack8(dm[q4], m);
                        }
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] *= m[e];
                    }
                    oc[q4] = pack8(v);
                    od[q4] = g.dout_z ? pack8_f16(d) : pack8(d);
                }
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int row = bm + wr * MI * 32 + i * 32 + (lane >> 3) + 8 * q4;
                    if (row < g.M && colok) {
                        *reinterpret_cast<u32x4*>(g.C + (int64_t)row * g.ldc + col) = oc[q4];
                        if (g.Dout && sine_cols) *reinterpret_cast<u32x4*>(g.Dout + (int64_t)row * g.ld_dout + col) = od[q4];
                    }
                }
            }
        }
        if (!more) break;
        __syncthreads();
        sstore(r0, 0);
        __syncthreads();
        t = tn;
    }
}

// 256 x 256 NT tile fed by LDS-DMA through a ring that runs across tile boundaries
// (nt_bf16_variant 8).  k_gemm_nt_bf16w keeps one K-step of loads in flight and leaves HBM idle
// through each tile's epilogue, whose Dmul loads then wait one full latency per 32 x 64 piece
// (C4's backward dX GEMMs ran at 41% of HBM).  Here:
//  * K-steps of 32 (64-B rows, 16-B chunk c of row r at c ^ ((r >> 2) & 3): conflict-free
//    ds_read_b128 for the 32x32x16 fragments) land by global_load_lds_dwordx4 in four 32 KB
//    stages, three steps in flight; the step sequence is flat over the block's tiles, so the
//    next tile's first three steps are loading while this tile's epilogue runs;
//  * the epilogue stages 32 x 64 fp32 pieces (256-B rows, chunks XOR row & 1) in the stage the
//    tile's last step was read from (waves 4..7) and in a 32 KB area outside the ring (waves
//    0..3), and the next piece's Dmul rows load while a piece is finished.
// Same k order as k_gemm_nt_bf16w (16-wide k blocks in increasing k): bit-identical outputs.
// K and K1 must be multiples of 32 (host-checked).
constexpr int ND_K = 32, ND_STAGES = 4, ND_STG = 512 * 64;
#ifndef SPN_NT_ADDR
#define SPN_NT_ADDR 1  // DMA sources as a uniform base + 32-bit lane offset (0: 64-bit per-lane pointers, A/B builds)
#endif
#ifndef SPN_NT16_NT
// the DMA NT GEMM's C / Dout stores non-temporal (glc slc; whole 128-B row pieces): round 3, C4 26.20 /
// 26.19 -> 26.13 / 26.11 ms (off then: within the spread); round 6, C4 23.66 / 23.69 -> 23.58 /
// 23.63 ms, C4@512 3.390 / 3.394 -> 3.374 / 3.390 (tools/ab_libs.sh, one call): on
#define SPN_NT16_NT 1
#endif
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }
#ifdef ND_STAMPS
// diagnostic build only (tools/gemm_bench_bf16 -DND_STAMPS): lane 0 of waves 0 and 4 of block 0
// record s_memtime at the phase boundaries; never compiled into the library
#define ND_STAMP(slot)                                                                          \
    do {                                                                                        \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        unsigned long long t_;                                                                  \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");             \
        __builtin_amdgcn_sched_barrier(0);                                                      \
        if (st_on) g.stamps[st_base + st_n] = t_ * 16 + (slot);                                \
        ++st_n;                                                                                 \
    } while (0)
#else
#define ND_STAMP(slot) \
    do {               \
    } while (0)
#endif
// DM: the backward dX epilogue only (C = acc · Dmul, no bias / rank-1 / sine).
// IP: issue placement of the next K-step's DMAs, as k_gemm_tn_bf16d (option nt_bf16_ip; the
// backward xDmul epilogue only, 2 by default: 536 -> 429 us on 524 288 x 512 x 512 in isolation,
// within noise in the C4 step)
// EV: the epilogue's inputs as COMPILE-TIME choices.  An epilogue load behind a runtime branch
// (`g.Dmul ? load : 0`, `if (g.rowbias)`, the zsave option's `g.dmul_z ? cos(Z) : D`) makes hipcc
// wait vmcnt(0) at the join — for the next tile's in-flight DMAs and every earlier store — once per
// 32 x 64 piece (16 per tile; counted in the --save-temps assembly).  Every load of a non-generic
// variant is unconditional:
//   DM:  0 = Dmul holds D (bf16), 1 = Dmul holds the saved Z (fp16; option zsave): D = cos(Z);
//   !DM: 0 = generic (runtime flags: zsave rounding, rank-1, Dmul, rowbias), 1 = bias + sine/linear
//        columns, 2 = the same + per-ray rows (rows_per_ray % 32 == 0: a 32-row piece lies in one
//        ray, each lane loads one column of the wave's ray row at the tile start and the piece
//        takes its 8 values by ds_bpermute), 3 = bias + rank-1 + Dmul (no sine).
// The bias of variants 1-3 is read from a zero row when absent: + 0.f, which the generic
// epilogue also adds (bit-identical).
__device__ const float kZeroRow[2048 + 8] = {};
// a float through an explicitly GLOBAL pointer: a generic (flat) load may alias LDS, so hipcc
// makes it wait for the in-flight LDS-DMA writes (vmcnt(0)) — which a select between a kernel
// argument and kZeroRow otherwise compiles to
typedef const __attribute__((address_space(1))) float* gfloat_ptr;
__device__ __forceinline__ float ldgf(const float* p) { return *(gfloat_ptr)p; }
// HD: the narrow output heads of NT16Args::hd in the epilogue (EV 1 / 2 only): a head tile's
// lanes dot their 8 bf16-rounded outputs per row with the head weights, the 8 lanes of a row
// reduce by xor butterfly, the 4 column waves' partials meet in the staging LDS after a barrier
// and are summed in wave order (deterministic).
template <bool DM, int IP = 0, int EV = 0, bool HD = false>
__global__ __launch_bounds__(512) void k_gemm_nt_bf16d(NT16Args g, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[ND_STAGES * ND_STG + 8 * 4096];
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    constexpr int MI = 4, NJ = 2;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int gdbg = kAblBuild ? g.dbg : 0;  // (product: no ablation branch in the k-loop)
    const int nN = (g.N + 255) / 256;
    const int G = gridDim.x;
    int t = xcd_remap(blockIdx.x, G);
    if (t >= ntiles) return;  // block-uniform
    const int nk = g.K / ND_K;

    // DMA: instruction q = wid + 8 i fills stage rows 16 q .. 16 q + 15 (rows < 256: A, else B);
    // lane l lands at row 16 q + l / 4, chunk position l % 4, so it loads the logical chunk
    // (l % 4) ^ ((row >> 2) & 3)
    int is_t = t, is_k = 0;  // issue pointer: tile, K-step
    // instruction i of the step at the issue pointer (i = 3 advances the pointer)
    auto issue1 = [&](int stg, int i) {
        const int tile = is_t < ntiles ? is_t : t;  // past the last tile: re-reads, never consumed
        const int bm = (tile / nN) * 256, bn = (tile % nN) * 256;
        const int k0 = is_k * ND_K;
        const bool seg2 = k0 >= g.K1;
        const bf16* pa = seg2 ? g.A2 + (k0 - g.K1) : g.A + k0;
        const int lda = seg2 ? g.lda2 : g.lda;
        const int el = opaque(lane);
        const int ni = (gdbg & 16) ? 2 : 4;  // ablation: A only
        if (i < ni) {
            const int q = wid + 8 * i;
            const int row = 16 * q + (el >> 2);
            const int c8 = ((el & 3) ^ ((row >> 2) & 3)) * 8;
#if SPN_NT_ADDR
            // a wave-uniform 64-bit base and a 32-bit per-lane byte offset (P·K < 2^31 / 2 is host-
            // checked): the saddr + voffset form, no 64-bit VALU address per DMA
            const char* base = i < 2 ? reinterpret_cast<const char*>(pa) : reinterpret_cast<const char*>(g.B + k0);
            const uint32_t off = i < 2 ? (uint32_t)(min(bm + row, g.M - 1) * lda + c8) * 2u
                                       : (uint32_t)(min(bn + row - 256, g.N - 1) * g.ldb + c8) * 2u;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(base + off), (lds_ptr_t)(smem + stg * ND_STG + q * 1024), 16, 0, 0);
#else
            const bf16* src = i < 2 ? pa + (int64_t)min(bm + row, g.M - 1) * lda + c8
                                    : g.B + (int64_t)min(bn + row - 256, g.N - 1) * g.ldb + k0 + c8;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(smem + stg * ND_STG + q * 1024), 16, 0, 0);
#endif
        }
        if (i == 3 && ++is_k == nk) {
            is_k = 0;
            is_t += G;
        }
    };
    auto issue = [&](int stg) {
#pragma unroll
        for (int i = 0; i < 4; ++i) issue1(stg, i);
    };

    f32x16 acc[MI][NJ];
    const int wr = wid >> 2, wc = wid & 3, r32 = lane & 31, h = lane >> 5;
    auto compute = [&](int stg, auto&& mid) {
        const int swz = (r32 >> 2) & 3;
        const char* sA = smem + stg * ND_STG + (wr * 128 + r32) * 64;
        const char* sB = smem + stg * ND_STG + (256 + wc * 64 + r32) * 64;
#pragma unroll
        for (int ks = 0; ks < ND_K / 16; ++ks) {
            const int off = ((2 * ks + h) ^ swz) * 16;
            bf16x8 a[MI], b[NJ];
#pragma unroll
            for (int i = 0; i < MI; ++i) a[i] = *reinterpret_cast<const bf16x8*>(sA + i * 32 * 64 + off);
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(sB + j * 32 * 64 + off);
#pragma unroll
            for (int i = 0; i < MI; ++i) {
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
                if constexpr (IP == 3) {
                    // IP 3: the next step's 4 DMA instructions one per two MFMA groups
                    if (i & 1) {
                        __builtin_amdgcn_sched_barrier(0);
                        mid(2 * ks + (i >> 1));
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
            if constexpr (IP != 3) {
                if (ks == 0) mid(0);
            }
        }
    };

#ifdef ND_STAMPS
    const bool st_on = g.stamps && blockIdx.x == 0 && (wid == 0 || wid == 4) && lane == 0;
    const int st_base = (wid >> 2) * 4096;
    int st_n = 0;
#endif
    constexpr bool GEN = !DM && EV == 0;           // runtime epilogue flags
    constexpr bool RBL = !DM && EV == 2;           // per-ray rows by lane loads
    constexpr bool R1D = !DM && EV == 3;           // rank-1 + Dmul
    int gs = 0;  // flat step counter: step gs sits in stage gs % ND_STAGES
    issue(0);
    issue(1);
    issue(2);
    while (true) {
        const int bm = (t / nN) * 256, bn = (t % nN) * 256;
        const int tn = t + G;
        const bool more = tn < ntiles;
        // variants 1-3: the tile's bias (and rank-1 / per-ray row) values load before its K-loop,
        // so no epilogue wait covers the next tile's DMAs
        float bias8[8], r1v8[8], rbl[4];
        // HD: this tile's head group (block-uniform) and this lane's 8 columns' head weights
        // (the group's fields picked by unrolled compares: a dynamic index into the kernel
        // argument would copy it to scratch)
        int hg = -1, hno = 0, hkind = 0;
        const float* hwp = nullptr;
        const float* hbp = nullptr;
        int hldw = 0;
        float hw[3][8];
        if constexpr (HD) {
#pragma unroll
            for (int i = 0; i < kNTHeads; ++i)
                if (i < g.hd.n && g.hd.col0[i] == bn) {
                    hg = i;
                    hno = g.hd.nout[i];
                    hkind = g.hd.kind[i];
                    hwp = g.hd.w[i];
                    hbp = g.hd.b[i];
                    hldw = g.hd.ldw[i];
                }
            if (hg >= 0) {
                const int cq0 = (opaque(lane) & 7) * 8;
                const int cl = wc * 64 + cq0;  // column within the head's 256
                const bool ok = bn + cl < g.N;
#pragma unroll
                for (int o = 0; o < 3; ++o)
#pragma unroll
                    for (int e = 0; e < 8; ++e) hw[o][e] = (o < hno && ok) ? ldgf(hwp + (int64_t)o * hldw + cl + e) : 0.f;
            }
        }
        float hpart[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};  // this lane's two kept rows
        {
            const int cq0 = (opaque(lane) & 7) * 8;
            const int colc0 = min(bn + wc * 64 + cq0, g.N - 8);
            if constexpr (!DM && !GEN) {
                const float* bp = g.bias ? g.bias : kZeroRow;
#pragma unroll
                for (int e = 0; e < 8; ++e) bias8[e] = ldgf(bp + colc0 + e);
            }
            if constexpr (R1D) {
#pragma unroll
                for (int e = 0; e < 8; ++e) r1v8[e] = ldgf(g.r1_v + colc0 + e);
            }
            if constexpr (RBL) {
                const int cl = min(bn + wc * 64 + opaque(lane), g.N - 1);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int ray = min(bm + wr * 128 + i * 32, g.M - 1) / g.rows_per_ray;
                    rbl[i] = ldgf(g.rowbias + (int64_t)ray * g.ld_rb + cl);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        for (int kt = 0; kt < nk; ++kt, ++gs) {
            // step gs has landed when at most the two newer steps' DMAs (4 each) are outstanding
            // (after an epilogue its stores are newer still: the wait is then stricter, not
            // wrong); the barrier publishes every wave's DMAs and retires the reads of stage
            // (gs + 3) % 4 (step gs - 1, or the previous epilogue's staging)
            ND_STAMP(0);
            if (gdbg & 16) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if (!(gdbg & 4)) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            ND_STAMP(1);
            __builtin_amdgcn_s_barrier();
            ND_STAMP(2);
            if constexpr (IP == 3) {  // spread over this step's MFMAs
                compute(gs % ND_STAGES, [&](int i) { issue1((gs + 3) % ND_STAGES, i); });
            } else if constexpr (IP == 2) {  // the next step's DMAs between this step's two k-halves
                compute(gs % ND_STAGES, [&](int) { issue((gs + 3) % ND_STAGES); });
            } else if constexpr (IP == 1) {  // after this step's MFMAs
                compute(gs % ND_STAGES, [](int) {});
                issue((gs + 3) % ND_STAGES);
            } else {
                issue((gs + 3) % ND_STAGES);
                ND_STAMP(3);
                if (!(gdbg & 1)) compute(gs % ND_STAGES, [](int) {});
            }
        }
        ND_STAMP(4);
        if (gdbg & 2) {
            if (tn >= ntiles) break;
            t = tn;
            continue;
        }
        // ---- epilogue: the wave's 128 x 64 outputs as four 32 x 64 pieces
        const int el = opaque(lane), cq = (el & 7) * 8, erow = el >> 3, er32 = el & 31, eh = el >> 5;
        const int col = bn + wc * 64 + cq;
        const bool colok = col < g.N;
        const int colc = colok ? col : g.N - 8;
        const int rbase = bm + wr * 128 + erow;
        auto dload = [&](u32x4 (&dm)[4], float (&r1a)[4], int i) {
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int row = min(rbase + i * 32 + 8 * q4, g.M - 1);
                if constexpr (DM) {
                    dm[q4] = ldg16(g.Dmul + (int64_t)row * g.ld_dmul + colc);
                    r1a[q4] = 0.f;
                } else if constexpr (R1D) {
                    dm[q4] = ldg16(g.Dmul + (int64_t)row * g.ld_dmul + colc);
                    r1a[q4] = ldgf(g.r1_a + (int64_t)row * g.r1_lda);
                } else if constexpr (GEN) {
                    dm[q4] = g.Dmul ? ldg16(g.Dmul + (int64_t)row * g.ld_dmul + colc) : u32x4{0u, 0u, 0u, 0u};
                    r1a[q4] = g.r1_a ? g.r1_a[(int64_t)row * g.r1_lda] : 0.f;
                } else {
                    dm[q4] = u32x4{0u, 0u, 0u, 0u};
                    r1a[q4] = 0.f;
                }
            }
        };
        // Dmul rows in flight one piece ahead
        constexpr int NB = 2;  // all four at once measured slower (546 vs 510 us, 524 288 x 512 x 512)
        u32x4 dm[NB][4];
        float r1a[NB][4];
#pragma unroll
        for (int p = 0; p + 1 < NB; ++p) dload(dm[p], r1a[p], p);
        if constexpr (DM || GEN) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                bias8[e] = !DM && g.bias ? g.bias[colc + e] : 0.f;
                r1v8[e] = !DM && g.r1_a ? g.r1_v[colc + e] : 0.f;
            }
        }
        // every wave is done reading stage (gs - 1) % 4 before waves 4..7 stage into it
        ND_STAMP(5);
        __builtin_amdgcn_s_barrier();
        ND_STAMP(6);
        float* stage = wid < 4 ? reinterpret_cast<float*>(smem + ND_STAGES * ND_STG + wid * 8192)
                               : reinterpret_cast<float*>(smem + ((gs + 3) % ND_STAGES) * ND_STG + (wid - 4) * 8192);
        const bool sine_cols = !DM && !R1D && g.act == 1 && col >= g.n_lin;  // n_lin is a multiple of 8
        // store descriptors over the tile's rows of C and (sine layers) Dout
        const int trows = min(256, g.M - bm);
        const __amdgpu_buffer_rsrc_t rsC =
            __builtin_amdgcn_make_buffer_rsrc(g.C + (int64_t)bm * g.ldc, 0, trows * g.ldc * 2, 0x00020000);
        const bool dout_on = !DM && g.Dout && g.act == 1;
        const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc(
            dout_on ? g.Dout + (int64_t)bm * g.ld_dout : g.C, 0, dout_on ? trows * g.ld_dout * 2 : 0, 0x00020000);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            if (i + NB - 1 < MI) dload(dm[(i + NB - 1) % NB], r1a[(i + NB - 1) % NB], i + NB - 1);
            lds_order();
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int rr = (r & 3) + 8 * (r >> 2) + 4 * eh, cc = j * 32 + er32;
                    stage[rr * 64 + ((((cc >> 2) ^ (rr & 1)) << 2) | (cc & 3))] = acc[i][j][r];
                }
            lds_order();
            // variant 2: the piece's per-ray row (one ray per 32-row piece) from the lanes holding it
            float rbv[8];
            if constexpr (RBL) {
#pragma unroll
                for (int e = 0; e < 8; ++e) rbv[e] = __shfl(rbl[i], cq + e);
            }
            u32x4 oc[4], od[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int rr = erow + 8 * q4;
                const int row = rbase + i * 32 + 8 * q4;
                const f32x4 lo = ld4(stage + rr * 64 + (((cq >> 2) ^ (rr & 1)) << 2));
                const f32x4 hi = ld4(stage + rr * 64 + ((((cq >> 2) + 1) ^ (rr & 1)) << 2));
                float v[8], d[8];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[e] = lo[e] + bias8[e];
                    v[e + 4] = hi[e] + bias8[e + 4];
                }
                if constexpr (RBL) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += rbv[e];
                } else if constexpr (GEN) {
                    if (g.rowbias) {
                        const float* rb = g.rowbias + (int64_t)(min(row, g.M - 1) / g.rows_per_ray) * g.ld_rb + colc;
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] += rb[e];
                    }
                }
                if (R1D || (GEN && g.r1_a)) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += r1a[i % NB][q4] * r1v8[e];
                }
                if (sine_cols) {
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        float sn, cs;
                        const float z = (GEN && g.zround) ? zr16(v[e]) : v[e];
                        fast_sincos(g.w0 * z, &sn, &cs);
                        v[e] = sn;
                        d[e] = (GEN && g.dout_z) ? z : g.w0 * cs;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 8; ++e) d[e] = 1.f;
                }
                if (DM || R1D || (GEN && g.Dmul)) {
                    float m[8];
                    if ((DM && EV == 1) || (GEN && g.dmul_z)) {  // Dmul holds the saved Z (fp16): D = cos(Z)
                        unpack8_f16(dm[i % NB][q4], m);
#pragma unroll
                        for (int e = 0; e < 8; ++e) m[e] = fast_cos(m[e]);
                    } else {
                        unpack8(dm[i % NB][q4], m);
                    }
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] *= m[e];
                }
                oc[q4] = pack8(v);
                od[q4] = (GEN && g.dout_z) ? pack8_f16(d) : pack8(d);
                if constexpr (HD) {
                    if (hg >= 0) {  // block-uniform
                        float y[8];
                        unpack8(oc[q4], y);
                        const int combo = i * 4 + q4;   // lane (combo % 8) of the row keeps the row's sums
#pragma unroll
                        for (int o = 0; o < 3; ++o) {
                            float t = 0.f;
#pragma unroll
                            for (int e = 0; e < 8; ++e) t += y[e] * hw[o][e];
                            t += __shfl_xor(t, 1, 64);
                            t += __shfl_xor(t, 2, 64);
                            t += __shfl_xor(t, 4, 64);
                            if ((el & 7) == (combo & 7)) hpart[combo >> 3][o] = t;
                        }
                    }
                }
                // materialise the piece's results here: hipcc otherwise sinks the arithmetic
                // (and the Dmul waits, as vmcnt(0)) into the guarded stores below
                asm volatile("" : "+v"(oc[q4]));
                if constexpr (!DM) asm volatile("" : "+v"(od[q4]));
            }
            // unconditional stores through the tile's buffer descriptors: rows past M fall outside
            // the descriptor's range and invalid lanes get an out-of-range offset, so the hardware
            // drops them — a branch around the stores would make every later load wait vmcnt(0)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int lr = wr * 128 + erow + i * 32 + 8 * q4;   // row within the tile
                const uint32_t oc_off = colok ? (uint32_t)(((int64_t)lr * g.ldc + col) * 2) : 0x7FFFFFF0u;
                __builtin_amdgcn_raw_buffer_store_b128(oc[q4], rsC, oc_off, 0, SPN_NT16_NT ? 3 : 0);
                if constexpr (!DM && !R1D) {
                    const uint32_t od_off = (colok && sine_cols) ? (uint32_t)(((int64_t)lr * g.ld_dout + col) * 2) : 0x7FFFFFF0u;
                    __builtin_amdgcn_raw_buffer_store_b128(od[q4], rsD, od_off, 0, SPN_NT16_NT ? 3 : 0);
                }
            }
            ND_STAMP(8);
        }
        ND_STAMP(7);
        if constexpr (HD) {
            if (hg >= 0) {  // block-uniform: the 4 column waves' row partials, summed in wave order
                __syncthreads();  // every wave is done with its staging
                float* part = reinterpret_cast<float*>(smem + ND_STAGES * ND_STG);  // [4 wc][256 rows][4]
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int combo = 8 * k + (el & 7), pi = combo >> 2, pq = combo & 3;
                    const int row = wr * 128 + pi * 32 + erow + 8 * pq;
#pragma unroll
                    for (int o = 0; o < 3; ++o) part[(wc * 256 + row) * 4 + o] = hpart[k][o];
                }
                __syncthreads();
                const int row = tid;
                const int64_t p = (int64_t)bm + row;
                if (row < 256 && p < g.M) {
                    const NTHeads& H = g.hd;
                    const int kind = hkind;
                    float x[3];
#pragma unroll
                    for (int o = 0; o < 3; ++o)
                        x[o] = ((part[(0 * 256 + row) * 4 + o] + part[(1 * 256 + row) * 4 + o]) + part[(2 * 256 + row) * 4 + o]) +
                               part[(3 * 256 + row) * 4 + o];
                    // explicitly global accesses: a flat one would wait for the next tile's DMAs
                    typedef __attribute__((address_space(1))) float* gfloat_w;
                    const gfloat_w out = (gfloat_w)(H.out + p * H.NO);
                    const gfloat_w hs = (gfloat_w)(H.hsave + p * 8);
                    const float* bb = hbp;
                    if (kind == 0) {          // rgb
#pragma unroll
                        for (int c = 0; c < 3; ++c) {
                            const float gv = sigmoidf_(x[c] + ldgf(bb + c));
                            out[c] = __fsub_rn(__fmul_rn(gv, 1.002f), 0.001f);
                            hs[1 + c] = gv;
                        }
                    } else if (kind == 1) {   // sun, and σ / sky
                        const float sun = sigmoidf_(x[0] + ldgf(bb));
                        out[4] = sun;
                        hs[4] = sun;
                        out[3] = softplusf_(hs[0]);
                        if (H.full) {
#pragma unroll
                            for (int c = 0; c < 3; ++c) out[5 + c] = ldgf(H.sky + (int64_t)((int)p / H.S) * 4 + c);
                        } else {
                            for (int c = 0; c < H.NO; ++c)
                                if (c != 3 && c != 4) out[c] = 0.f;
                        }
                    } else if (kind == 2) {   // beta
                        const float bpre = x[0] + ldgf(bb);
                        out[8] = softplusf_(bpre);
                        hs[5] = bpre;
                    } else {                  // semantic logits
#pragma unroll
                        for (int o = 0; o < 3; ++o)
                            if (o < hno) out[H.sem_col + o] = x[o] + ldgf(bb + o);
                    }
                }
            }
        }
        if (!more) break;  // block-uniform
        t = tn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-read DMAs land before the block exits
#ifdef ND_STAMPS
    if (st_on) g.stamps[st_base + 4095] = st_n;
#endif
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
    // 1-D grid of tiles x splits, split-major after the XCD remap: all tiles of one split run
    // on one XCD, roughly in step through the points, so each operand slice is fetched into
    // that XCD's L2 once (a (tile, split) grid spread every split over the 8 XCDs: 2.5x the
    // algorithmic HBM/fabric traffic, profiles/r01/traffic_c3.json before this change)
    const int nK = (g.K + HB - 1) / HB;
    const int ntiles = cdiv(g.N, HB) * nK;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * HB, k0 = (t % nK) * HB;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const int ch = tid & 15, lrow = tid >> 4;  // loader: 8 features (chunk ch), rows lrow + 16 i
    const bool do_bias = g.slab_b != nullptr && k0 == 0;

    // Unconditional loads (see k_gemm_nt_bf16): features past N / K read a clamped column (their
    // outputs are never stored); points past the split are zeroed, and the bias sums taken, when
    // the registers are written to LDS, after the step's MFMAs.
    u32x4 ra[4], rb[4];
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int nc = min(n0 + 8 * ch, g.N - 8);
    const int kc = min(k0 + 8 * ch, g.K - 8);
    const bf16* pb = kc < g.K1 ? g.B + kc : g.B2 + (kc - g.K1);
    const bf16* pb2 = kc < g.K1 ? g.B_s2 + kc : g.B2_s2 + (kc - g.K1);  // second segment
    const bool bsin = g.b_sin && kc < g.K1;  // this thread's B chunk is a saved Z: stage sin(Z)
    const int ldb = kc < g.K1 ? g.ldb : g.ldb2;
    const int lda = g.lda;
    int p_ld = 0;
    auto gload = [&](int p0) {
        p_ld = p0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = min(p0 + lrow + 16 * i, p_end - 1);
            const bool s2 = pc >= g.P1;
            ra[i] = ldg16((s2 ? g.A_s2 : g.A) + (int64_t)pc * lda + nc);
            rb[i] = ldg16((s2 ? pb2 : pb) + (int64_t)pc * ldb);
        }
    };
    auto sstore = [&](int stg) {
        char* sA = smem + stg * 2 * 64 * 256;
        char* sB = sA + 64 * 256;
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool pin = p_ld + lrow + 16 * i < p_end;
            const u32x4 v = pin ? ra[i] : z;
            if (do_bias) {
                float f[8];
                unpack8(v, f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[e] += f[e];
            }
            const int o = tn_off(lrow + 16 * i, ch);
            *reinterpret_cast<u32x4*>(sA + o) = v;
            *reinterpret_cast<u32x4*>(sB + o) = pin ? (bsin ? sin8_z(rb[i]) : rb[i]) : z;
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

    if (p_beg < p_end) {  // block-uniform
        const int ns = (p_end - p_beg + 63) / 64;
        gload(p_beg);
        sstore(0);
        __syncthreads();
        for (int st = 0; st < ns; ++st) {
            // unconditional (no branch around a load): past the split the addresses clamp and
            // sstore zeroes the rows
            gload(p_beg + 64 * (st + 1));
            __builtin_amdgcn_sched_barrier(0);  // issue the loads before the MFMAs
            compute(st & 1);
            __builtin_amdgcn_sched_barrier(0);  // LDS writes (and their vmcnt waits) after the MFMAs
            sstore((st + 1) & 1);
            __syncthreads();
        }
    }

    float* slab = g.slab + (int64_t)split * g.slab_stride;
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
            g.slab_b[(int64_t)split * g.N + n0 + tid] = s;
        }
    }
}

// Narrow TN (option tn_bf16_k64): N = 512 A features x K = 64 B features — fc_net.0's weight
// gradient over the PE and the skip layer's PE tail.  One block per split holds the whole
// 512 x 64 output (8 waves of 64 x 64, 2x2 32x32 accumulators), so every operand row is read
// from HBM exactly once; the 128x128 kernel above ran 4 N-tiles per split, each with a 128-wide
// K tile of which 64 columns were clamped duplicates (twice the MFMA work, dZ fetched per tile).
// 32-point steps: A as four [32][128] tn_off images, B in a fifth (its chunks 0..7), two LDS
// stages (80 KB); register loads two steps ahead (two sets, 72 KB in flight per CU) — the
// kernel is HBM-bound (1.1 KB per point, 64 K MAC per point).  Steps past the split read
// clamped rows that are stored as zeros (an even step count, so the loop has no branch).
constexpr int T64_STEP = 32, T64_IMG = T64_STEP * 256, T64_STG = 5 * T64_IMG;
// (a group launch: blocks [start[gi], start[gi + 1]) are the splits of GEMM gi)
__global__ __launch_bounds__(512) void k_gemm_tn_bf16_k64(TN16Group G) {
    __shared__ __attribute__((aligned(16))) char smem[2 * T64_STG];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int gi = 0;
    while (gi + 1 < G.n && (int)blockIdx.x >= G.start[gi + 1]) ++gi;
    const TN16Args& g = G.g[gi];
    const int split = blockIdx.x - G.start[gi];
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const int ach = tid & 63, arow = tid >> 6;         // A: features 8·ach.., rows arow + 8i
    const int bch = tid & 7, brow = (tid >> 3) & 31;   // B: features 8·bch.., row brow (tid >= 256 repeat tid - 256)
    const bool do_bias = g.slab_b != nullptr;
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

    u32x4 ra0[4], ra1[4], rb0, rb1;
    auto gload = [&](u32x4 (&ra)[4], u32x4& rb, int p0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = min(p0 + arow + 8 * i, p_end - 1);
            ra[i] = ldg16((pc >= g.P1 ? g.A_s2 : g.A) + (int64_t)pc * g.lda + 8 * ach);
        }
        const int pb = min(p0 + brow, p_end - 1);
        rb = ldg16((pb >= g.P1 ? g.B_s2 : g.B) + (int64_t)pb * g.ldb + 8 * bch);
    };
    auto sstore = [&](int stg, const u32x4 (&ra)[4], const u32x4& rb, int p0) {
        char* sA = smem + stg * T64_STG;
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = arow + 8 * i;
            const u32x4 v = p0 + row < p_end ? ra[i] : z;
            if (do_bias) {  // block-uniform
                float f[8];
                unpack8(v, f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[e] += f[e];
            }
            *reinterpret_cast<u32x4*>(sA + (ach >> 4) * T64_IMG + tn_off(row, ach & 15)) = v;
        }
        // threads tid and tid + 256 write the same chunk (same value: no branch around the store)
        *reinterpret_cast<u32x4*>(sA + 4 * T64_IMG + tn_off(brow, bch)) = p0 + brow < p_end ? rb : z;
    };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int h = lane >> 5, grp = (lane >> 4) & 1;
    const int q = (lane & 15) >> 2, pp = lane & 3;
    auto trd = [&](const char* base, int r0, int col) -> s16x4 {
        const int o = tn_off(r0 + q, (col >> 3) + (pp >> 1)) + 8 * (pp & 1);
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o));
    };
    auto operand = [&](const char* base, int r0, int col) -> bf16x8 {
        const s16x4 lo = trd(base, r0, col), hi = trd(base, r0 + 4, col);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    // wave w: A features [64w, 64w + 64) = image w / 2, columns 64·(w & 1) ..; all 64 B features
    const int aimg = wid >> 1, acol = (wid & 1) * 64;
    auto compute = [&](int stg) {
        const char* sA = smem + stg * T64_STG + aimg * T64_IMG;
        const char* sB = smem + stg * T64_STG + 4 * T64_IMG;
#pragma unroll
        for (int ks = 0; ks < T64_STEP / 16; ++ks) {
            const int r0 = 16 * ks + 8 * h;
            const bf16x8 a0 = operand(sA, r0, acol + 16 * grp);
            const bf16x8 a1 = operand(sA, r0, acol + 32 + 16 * grp);
            const bf16x8 b0 = operand(sB, r0, 16 * grp);
            const bf16x8 b1 = operand(sB, r0, 32 + 16 * grp);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
        }
    };

    if (p_beg < p_end) {  // block-uniform
        const int ns = ((p_end - p_beg + T64_STEP - 1) / T64_STEP + 1) & ~1;  // even
        gload(ra0, rb0, p_beg);
        gload(ra1, rb1, p_beg + T64_STEP);
        sstore(0, ra0, rb0, p_beg);
        __syncthreads();
        for (int st = 0; st < ns; st += 2) {
            const int p = p_beg + T64_STEP * st;
            gload(ra0, rb0, p + 2 * T64_STEP);
            __builtin_amdgcn_sched_barrier(0);  // issue the loads before the MFMAs
            compute(0);
            __builtin_amdgcn_sched_barrier(0);  // LDS writes (and their waits) after the MFMAs
            sstore(1, ra1, rb1, p + T64_STEP);
            __syncthreads();
            gload(ra1, rb1, p + 3 * T64_STEP);
            __builtin_amdgcn_sched_barrier(0);
            compute(1);
            __builtin_amdgcn_sched_barrier(0);
            sstore(0, ra0, rb0, p + 2 * T64_STEP);
            __syncthreads();
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (unused) prefetch
    }

    float* slab = g.slab + (int64_t)split * g.slab_stride;
    const int r32 = lane & 31;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = j * 32 + r32;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = 64 * wid + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                slab[(int64_t)n * g.ld_slab + k] = acc[i][j][r];
            }
    }
    if (do_bias) {  // block-uniform; the 8 row phases of every chunk in a fixed order
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [8 phases][512 features]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[arow * 512 + 8 * ach + e] = bs[e];
        __syncthreads();
        float s = 0.f;
#pragma unroll
        for (int ph = 0; ph < 8; ++ph) s += red[ph * 512 + tid];
        g.slab_b[(int64_t)split * 512 + tid] = s;
    }
}

int g_tn16_k64 = 1;  // option tn_bf16_k64: the narrow kernel above for N = 512, K = 64
static bool tn_k64(int N, int K) { return g_tn16_k64 && N == 512 && K == 64; }

// Wide TN: 256 (A features) x 256 (B features) per block, 8 waves of 128x64 (4x2 32x32
// accumulators, 128 AGPRs), one block per CU.  Per 64-point step a block stages 2 x 32 KB and
// runs 8 x 32 MFMAs: half the L2 bytes per FLOP of the 128x128 kernel above, whose two
// co-resident blocks need ≈39 TB/s of L2 at MFMA peak (more than the ≈34.5 TB/s the XCDs give),
// and 1.5 transposed LDS reads per MFMA instead of 2.  Each operand tile is staged as two
// [64][128] halves in the tn_off image, so the conflict-free read pattern is the one above.
// Selected (g_tn16_variant = 2) for N, K multiples of 256; other shapes use k_gemm_tn_bf16.
constexpr int TW = 256;
__global__ __launch_bounds__(512) void k_gemm_tn_bf16w(TN16Args g) {
    __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 2 * 64 * 256];  // [stage][A|B][half]
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nK = (g.K + TW - 1) / TW;
    const int ntiles = cdiv(g.N, TW) * nK;
    const int w = xcd_remap(blockIdx.x, gridDim.x);  // split-major, as k_gemm_tn_bf16
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * TW, k0 = (t % nK) * TW;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const int ch = tid & 31, lrow = tid >> 5;  // loader: 8 features (chunk ch of 32), rows lrow + 16 i
    const bool do_bias = g.slab_b != nullptr && k0 == 0;

    u32x4 ra[4], rb[4];
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int nc = min(n0 + 8 * ch, g.N - 8);
    const int kc = min(k0 + 8 * ch, g.K - 8);
    const bf16* pb = kc < g.K1 ? g.B + kc : g.B2 + (kc - g.K1);
    const bf16* pb2 = kc < g.K1 ? g.B_s2 + kc : g.B2_s2 + (kc - g.K1);  // second segment
    const bool bsin = g.b_sin && kc < g.K1;  // this thread's B chunk is a saved Z: stage sin(Z)
    const int ldb = kc < g.K1 ? g.ldb : g.ldb2;
    const int lda = g.lda;
    const int soff = (ch >> 4) * 64 * 256;  // half of the tile this thread's chunk lands in
    int p_ld = 0;
    auto gload = [&](int p0) {
        p_ld = p0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = min(p0 + lrow + 16 * i, p_end - 1);
            const bool s2 = pc >= g.P1;
            ra[i] = ldg16((s2 ? g.A_s2 : g.A) + (int64_t)pc * lda + nc);
            rb[i] = ldg16((s2 ? pb2 : pb) + (int64_t)pc * ldb);
        }
    };
    auto sstore = [&](int stg) {
        char* sA = smem + stg * 4 * 64 * 256 + soff;
        char* sB = sA + 2 * 64 * 256;
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool pin = p_ld + lrow + 16 * i < p_end;
            const u32x4 v = pin ? ra[i] : z;
            if (do_bias) {
                float f[8];
                unpack8(v, f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[e] += f[e];
            }
            const int o = tn_off(lrow + 16 * i, ch & 15);
            *reinterpret_cast<u32x4*>(sA + o) = v;
            *reinterpret_cast<u32x4*>(sB + o) = pin ? (bsin ? sin8_z(rb[i]) : rb[i]) : z;
        }
    };

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wa = wid >> 2, wb = wid & 3, h = lane >> 5, grp = (lane >> 4) & 1;
    const int q = (lane & 15) >> 2, pp = lane & 3;
    auto trd = [&](const char* base, int r0, int col) -> s16x4 {
        const int o = tn_off(r0 + q, (col >> 3) + (pp >> 1)) + 8 * (pp & 1);
        return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + o));
    };
    auto operand = [&](const char* base, int r0, int col) -> bf16x8 {
        const s16x4 lo = trd(base, r0, col), hi = trd(base, r0 + 4, col);
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    auto compute = [&](int stg) {
        const char* sA = smem + stg * 4 * 64 * 256 + wa * 64 * 256;                  // half wa of A
        const char* sB = smem + stg * 4 * 64 * 256 + (2 + (wb >> 1)) * 64 * 256;     // half wb/2 of B
        const int cb = (wb & 1) * 64;
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            const int r0 = 16 * ks + 8 * h;
            bf16x8 a[4], b[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = operand(sB, r0, cb + 32 * j + 16 * grp);
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = operand(sA, r0, 32 * i + 16 * grp);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    };

    if (p_beg < p_end) {  // block-uniform
        const int ns = (p_end - p_beg + 63) / 64;
        gload(p_beg);
        sstore(0);
        __syncthreads();
        for (int st = 0; st < ns; ++st) {
            gload(p_beg + 64 * (st + 1));
            __builtin_amdgcn_sched_barrier(0);
            if (!(g.dbg & 1)) compute(st & 1);
            __builtin_amdgcn_sched_barrier(0);
            sstore((st + 1) & 1);
            __syncthreads();
        }
    }

    float* slab = g.slab + (int64_t)split * g.slab_stride;
    const int r32 = lane & 31;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = k0 + wb * 64 + j * 32 + r32;
        if (k >= g.K) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wa * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < g.N) slab[(int64_t)n * g.ld_slab + k] = acc[i][j][r];
            }
    }
    if (do_bias) {  // block-uniform; the 16 row phases of every chunk combined in a fixed order
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [16 phases][256 features]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lrow * 256 + 8 * ch + e] = bs[e];
        __syncthreads();
        if (tid < 256 && n0 + tid < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 16; ++ph) s += red[ph * 256 + tid];
            g.slab_b[(int64_t)split * g.N + n0 + tid] = s;
        }
    }
}

// Wide TN fed by LDS-DMA (g_tn16_variant = 3): the tiling of k_gemm_tn_bf16w, but 32-point
// steps land by global_load_lds_dwordx4 straight into four 32 KB stages, three steps in flight
// (the register-staged kernel has one step in flight and waits a full HBM latency per step).
// A wave instruction fills 4 rows x 256 B of one half image; lane l lands at chunk position
// l % 16 of row l / 16, so it loads the logical chunk (l % 16) ^ swizzle(row) — the tn_off image
// is built by permuting source addresses.  DMA cannot zero rows, so the host uses this kernel
// only when every split holds whole 32-point steps (P % 32 == 0).  Bias sums are read back from
// the landed stage (k0 == 0 blocks only).
constexpr int TD_STEP = 32, TD_STAGES = 4, TD_STG = 4 * TD_STEP * 256;  // bytes per stage
#ifndef SPN_TN_NT
// the weight-gradient GEMM's DMA loads non-temporal (glc slc; A/B builds): slower — TN 5.88 -> 6.07 ms
// per C4 step, PMC reads 4.59 -> 6.12 GB per launch (the two tiles that share operand rows then
// fetch them twice)
#define SPN_TN_NT 0
#endif
#ifndef SPN_TN_ADDR
// 1: the IP 3 main loop reads its fragments at 12 lane offsets computed once per block, one
// v_add per offset per stage and the k-step as the ds_read immediate (the same reads, MFMAs and
// order: bit-identical); 0: every read's address from tn_off per k-step (≈ 48 VALU per stage
// beside 16 MFMAs: the SIMD's issue port, not the MFMA pipe, was the kernel's limit)
#define SPN_TN_ADDR 1
#endif
// IP: where a step issues the next DMA step: 0 = before its MFMAs, 1 = after them, 2 = between
// its two k-halves (default, option tn_bf16_ip: a wave stalled on the DMA issue then has MFMAs
// in flight; 393 -> 365 us on 524 288 x 512 x 512, C4 TN 7.18 -> 6.81 ms/step)
// A group launch (gemm_tn_bf16_group) runs G.n GEMMs in one grid, blocks [start[gi],
// start[gi + 1]) on GEMM gi — consecutive after the XCD remap, so a split keeps its tiles
// (which share operand rows) on one XCD as in a single launch.
// PF (option tn_bf16_pf): the next k-step's fragments are read from LDS while the current
// k-step's MFMAs run (two register sets), and a step's barrier sits between its two k-halves —
// the same MFMAs in the same order (bit-identical); without it every k-step waits out its own
// LDS reads (on-chip ceiling of the kernel with one-row operands: 0.44 of the MFMA peak).
template <int IP, bool PF = false>
__global__ __launch_bounds__(512) void k_gemm_tn_bf16d(TN16Group G) {
    __shared__ __attribute__((aligned(16))) char smem[TD_STAGES * TD_STG];  // [stage][A0|A1|B0|B1]
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    const int tid = threadIdx.x, lane = tid & 63;
#if SPN_TN_ADDR
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: DMA destinations in SGPRs
#else
    const int wid = tid >> 6;
#endif
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    int gi = 0;
    while (gi + 1 < G.n && wg >= G.start[gi + 1]) ++gi;
    const int w = wg - G.start[gi];
    const TN16Args& g = G.g[gi];
#ifdef ND_STAMPS
    // diagnostic build: lane 0 of waves 0 and 4 of blocks 0 and 128 stamp the IP = 1 main loop
    const bool st_on = g.stamps && (blockIdx.x == 0 || blockIdx.x == 128) && (wid == 0 || wid == 4) && lane == 0;
    const int st_base = ((blockIdx.x ? 2 : 0) + (wid >> 2)) * 4096;
    int st_n = 0;
#endif
    const int nK = (g.K + TW - 1) / TW;
    const int ntiles = cdiv(g.N, TW) * nK;
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * TW, k0 = (t % nK) * TW;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    // bias_split (nK == 2): the two tiles of a column range [n0, n0 + 256) read the same A rows;
    // each sums the bias of one 128-column half (k-tile kt: half kt), so both do the same work and
    // stay in step — with the whole bias on the k0 == 0 tile it fell behind its partner and the
    // shared A rows were fetched twice (PMC: 1.46x the algorithmic bytes)
    const bool bsplit = g.bias_split && nK == 2;
    const int kt = t % nK;
    const bool do_bias = g.slab_b != nullptr && (bsplit || k0 == 0);
    // IP 4 / 5: the bias sums from the A fragments already in registers (no LDS row reads): wave
    // (wa, wb) sums A fragment i = wb — feature 128 wa + 32 wb + lane % 32, 8 points per k-step per
    // lane — when its half wa is summed by this tile (bsplit: wa == kt; else every wave of the
    // k0 == 0 tile); lanes l and l + 32 (the two point halves) are added at the end
    constexpr bool BR = IP >= 4;
    const bool rb_on = BR && do_bias && (!bsplit || (wid >> 2) == kt);  // wave-uniform
    float rbias = 0.f;
    const int ns = p_end > p_beg ? (p_end - p_beg) / TD_STEP : 0;  // whole steps (host-checked)

    // this lane's 4 DMA sources (instructions q = wid + 8 i: i < 2 → A, else B), advanced by
    // TD_STEP rows per step
    // second point segment (g.P1 a multiple of TD_STEP, host-checked): a step lies in one segment
    // src: this lane's source in the first segment (VGPRs); dl: the wave-uniform byte offset to the
    // second segment's (readfirstlane: a B column range never straddles K1, host-checked K1 % 128)
    const bf16* src[4];
    int64_t dl[4];
    int ld[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = wid + 8 * i, X = q >> 4, hf = (q >> 3) & 1, rg = q & 7;
        const int row = rg * 4 + (lane >> 4);
        const int chl = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int f = (X ? k0 : n0) + hf * 128 + 8 * chl;
        if (X == 0) {
            src[i] = g.A + (int64_t)row * g.lda + min(f, g.N - 8);
            dl[i] = (int64_t)((intptr_t)g.A_s2 - (intptr_t)g.A);
            ld[i] = g.lda;
        } else {
            const int kc = min(f, g.K - 8);
            const bool s2 = __builtin_amdgcn_readfirstlane(kc >= g.K1 ? 1 : 0) != 0;
            ld[i] = s2 ? g.ldb2 : g.ldb;
            src[i] = (s2 ? g.B2 + (kc - g.K1) : g.B + kc) + (int64_t)row * ld[i];
            dl[i] = s2 ? (int64_t)((intptr_t)g.B2_s2 - (intptr_t)g.B2) : (int64_t)((intptr_t)g.B_s2 - (intptr_t)g.B);
        }
    }
    const int64_t P1 = g.P1;  // (a local: no scalar loads from the argument inside the loops)
#if SPN_TN_ADDR
    // the row strides and segment offsets are wave-uniform (ld: readfirstlane'd segment choice):
    // a step's byte offset is scalar arithmetic and each DMA address one 64-bit VALU add
    int ldu[4];
    int64_t dlu[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        ldu[i] = __builtin_amdgcn_readfirstlane(ld[i]);
        const uint64_t d = (uint64_t)dl[i];
        dlu[i] = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(d >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)d));
    }
#endif
    // one of the lane's 4 DMA instructions (IP 3 spreads them over a step's MFMAs)
    auto issue1 = [&](int st, int stg, int i) {
        const int64_t p0 = p_beg + (int64_t)TD_STEP * st;
        const bool sg2 = p0 >= P1;
        const int q = wid + 8 * i;
#if SPN_TN_ADDR
        const int64_t boff = p0 * ldu[i] * (int64_t)sizeof(bf16) + (sg2 ? dlu[i] : 0);
        const char* a = reinterpret_cast<const char*>(src[i]) + boff;
#else
        const char* a = reinterpret_cast<const char*>(src[i] + p0 * ld[i]) + (sg2 ? dl[i] : 0);
#endif
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)a, (lds_ptr_t)(smem + stg * TD_STG + q * 1024), 16, 0, SPN_TN_NT ? 3 : 0);
    };
    auto issue = [&](int st, int stg) {
#pragma unroll
        for (int i = 0; i < 4; ++i) issue1(st, stg, i);
    };

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wa = wid >> 2, wb = wid & 3, h = lane >> 5, grp = (lane >> 4) & 1;
    const int q4 = (lane & 15) >> 2, pp = lane & 3;
    // The transposed LDS reads are inline asm here: through the builtin, the compiler cannot tell
    // them from the in-flight DMA's LDS writes and drains vmcnt(0) before every step's first read
    // (no DMA would ever be in flight across the MFMAs).  Their results are therefore invisible to
    // its lgkmcnt tracking: one explicit wait, tied to every value it guards, precedes the MFMAs.
    auto trd = [&](const char* base, int r0, int col) -> s16x4 {
        const int o = tn_off(r0 + q4, (col >> 3) + (pp >> 1)) + 8 * (pp & 1);
        const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(base + o);
        s16x4 v;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr) : "memory");
        return v;
    };
    auto join = [](s16x4 lo, s16x4 hi) -> bf16x8 {
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    constexpr int HALF = TD_STEP * 256;
    auto compute = [&](int stg, auto&& mid) {
        const char* sA = smem + stg * TD_STG + wa * HALF;
        const char* sB = smem + stg * TD_STG + (2 + (wb >> 1)) * HALF;
        const int cb = (wb & 1) * 64;
#pragma unroll
        for (int ks = 0; ks < TD_STEP / 16; ++ks) {
            const int r0 = 16 * ks + 8 * h;
            s16x4 al[4], ah[4], bl[2], bh[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                bl[j] = trd(sB, r0, cb + 32 * j + 16 * grp);
                bh[j] = trd(sB, r0 + 4, cb + 32 * j + 16 * grp);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                al[i] = trd(sA, r0, 32 * i + 16 * grp);
                ah[i] = trd(sA, r0 + 4, 32 * i + 16 * grp);
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(al[0]), "+v"(al[1]), "+v"(al[2]), "+v"(al[3]), "+v"(ah[0]), "+v"(ah[1]),
                           "+v"(ah[2]), "+v"(ah[3]), "+v"(bl[0]), "+v"(bl[1]), "+v"(bh[0]), "+v"(bh[1])
                         :
                         : "memory");
            ND_STAMP(3 + 2 * ks);   // this k-step's fragments in registers
            bf16x8 a[4], b[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = join(bl[j], bh[j]);
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = join(al[i], ah[i]);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
                if constexpr (IP == 3) {
                    // IP 3: the next DMA step's 4 instructions one per two MFMA groups, each issued
                    // among MFMAs already in flight instead of in one burst with every other wave
                    if (i & 1) {
                        __builtin_amdgcn_sched_barrier(0);
                        mid(2 * ks + (i >> 1));
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
            }
            ND_STAMP(4 + 2 * ks);   // its MFMAs issued
            if constexpr (IP != 3) {
                if (ks == 0) mid(0);
            }
        }
    };
#if SPN_TN_ADDR
    // lane offsets (bytes from smem) of the 12 fragment reads of k-step 0 of stage 0: A fragments
    // i lo / hi, then B fragments j lo / hi.  Rows 16·ks + 8h + q4 (+ 4 for hi): k-step 1 adds 16
    // rows = 4096 bytes, and tn_off's swizzle reads only row bits 0..3, which 16·ks leaves alone
    uint32_t fo[12];
    {
        const uint32_t sbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
        const int cb = (wb & 1) * 64;
        auto off = [&](int half, int r0, int col) {
            return sbase + (uint32_t)(half * HALF + tn_off(r0 + q4, (col >> 3) + (pp >> 1)) + 8 * (pp & 1));
        };
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            fo[2 * i] = off(wa, 8 * h, 32 * i + 16 * grp);
            fo[2 * i + 1] = off(wa, 8 * h + 4, 32 * i + 16 * grp);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            fo[8 + 2 * j] = off(2 + (wb >> 1), 8 * h, cb + 32 * j + 16 * grp);
            fo[8 + 2 * j + 1] = off(2 + (wb >> 1), 8 * h + 4, cb + 32 * j + 16 * grp);
        }
    }
    // the compute() schedule of IP 3 on those offsets: va = fo + the stage's byte offset (12 VALU
    // per stage), k-step ks as the instruction's immediate offset
    auto compute_fo = [&](int stg, auto&& mid) {
        const uint32_t so = (uint32_t)(stg * TD_STG);
        uint32_t va[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) va[r] = fo[r] + so;
        auto kst = [&](auto kks) {
            constexpr int ks = decltype(kks)::value;
            s16x4 al[4], ah[4], bl[2], bh[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(bl[j]) : "v"(va[8 + 2 * j]), "i"(4096 * ks) : "memory");
                asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(bh[j]) : "v"(va[9 + 2 * j]), "i"(4096 * ks) : "memory");
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(al[i]) : "v"(va[2 * i]), "i"(4096 * ks) : "memory");
                asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(ah[i]) : "v"(va[2 * i + 1]), "i"(4096 * ks) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(al[0]), "+v"(al[1]), "+v"(al[2]), "+v"(al[3]), "+v"(ah[0]), "+v"(ah[1]),
                           "+v"(ah[2]), "+v"(ah[3]), "+v"(bl[0]), "+v"(bl[1]), "+v"(bh[0]), "+v"(bh[1])
                         :
                         : "memory");
            bf16x8 a[4], b[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = join(bl[j], bh[j]);
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = join(al[i], ah[i]);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
                if (i & 1) {
                    __builtin_amdgcn_sched_barrier(0);
                    mid(2 * ks + (i >> 1));
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        };
        kst(std::integral_constant<int, 0>{});
        kst(std::integral_constant<int, 1>{});
    };
#endif
    // one 16-point k-step of stage stg (IP 4's shifted schedule)
    auto kstep = [&](int stg, int ks) {
        const char* sA = smem + stg * TD_STG + wa * HALF;
        const char* sB = smem + stg * TD_STG + (2 + (wb >> 1)) * HALF;
        const int cb = (wb & 1) * 64;
        const int r0 = 16 * ks + 8 * h;
        s16x4 al[4], ah[4], bl[2], bh[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            bl[j] = trd(sB, r0, cb + 32 * j + 16 * grp);
            bh[j] = trd(sB, r0 + 4, cb + 32 * j + 16 * grp);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            al[i] = trd(sA, r0, 32 * i + 16 * grp);
            ah[i] = trd(sA, r0 + 4, 32 * i + 16 * grp);
        }
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(al[0]), "+v"(al[1]), "+v"(al[2]), "+v"(al[3]), "+v"(ah[0]), "+v"(ah[1]), "+v"(ah[2]),
                       "+v"(ah[3]), "+v"(bl[0]), "+v"(bl[1]), "+v"(bh[0]), "+v"(bh[1])
                     :
                     : "memory");
        if constexpr (BR) {
            if (rb_on) {  // wave-uniform
                // the fragment of A column block wb (a compile-time index per branch)
                s16x4 xl = al[0], xh = ah[0];
                if (wb == 1) xl = al[1], xh = ah[1];
                if (wb == 2) xl = al[2], xh = ah[2];
                if (wb == 3) xl = al[3], xh = ah[3];
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) rbias += __uint_as_float((uint32_t)(uint16_t)xl[e2] << 16);
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) rbias += __uint_as_float((uint32_t)(uint16_t)xh[e2] << 16);
            }
        }
        bf16x8 av[4], bv[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = join(bl[j], bh[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = join(al[i], ah[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    };
    // bias: thread (chunk ch of 32, row phase lrow of 16) sums rows lrow, lrow + 16 of each step;
    // bsplit: thread (chunk ch of the tile's 16, row phase lrow of 32) sums row lrow
    const int ch = bsplit ? 16 * kt + (tid & 15) : tid & 31, lrow = bsplit ? tid >> 4 : tid >> 5;
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto bias_rows = [&](int stg) {
        const char* sA = smem + stg * TD_STG + (ch >> 4) * HALF;
        if (bsplit) {  // block-uniform
            float f[8];
            unpack8(*reinterpret_cast<const u32x4*>(sA + tn_off(lrow, ch & 15)), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) bs[e] += f[e];
            return;
        }
#pragma unroll
        for (int i = 0; i < TD_STEP / 16; ++i) {
            float f[8];
            unpack8(*reinterpret_cast<const u32x4*>(sA + tn_off(lrow + 16 * i, ch & 15)), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) bs[e] += f[e];
        }
    };
    // the same sums split in two: the stage's rows read at its top (their latency runs with the
    // fragment reads' and is covered by the same waits), added after its MFMAs — read and added in
    // one place, each read was waited for on its own (lgkmcnt(0)) after the MFMAs: 8% of the kernel
    // (tools/tn_lab mode 8).  Same rows, same order of additions: bitwise the same sums
    auto bias_load = [&](int stg, u32x4 (&v)[TD_STEP / 16]) {
        const char* sA = smem + stg * TD_STG + (ch >> 4) * HALF;
#pragma unroll
        for (int i = 0; i < TD_STEP / 16; ++i)
            if (i == 0 || !bsplit) v[i] = *reinterpret_cast<const u32x4*>(sA + tn_off(lrow + 16 * i, ch & 15));
    };
    auto bias_add = [&](const u32x4 (&v)[TD_STEP / 16]) {
#pragma unroll
        for (int i = 0; i < TD_STEP / 16; ++i) {
            if (i > 0 && bsplit) break;
            float f[8];
            unpack8(v[i], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) bs[e] += f[e];
        }
    };

    // PF: fragments of one k-step (16 points) of stage stg into a register set; MFMAs from one
    struct Frag {
        s16x4 al[4], ah[4], bl[2], bh[2];
    };
    auto fread = [&](Frag& f, int stg, int ks) {
        const char* sA = smem + stg * TD_STG + wa * HALF;
        const char* sB = smem + stg * TD_STG + (2 + (wb >> 1)) * HALF;
        const int cb = (wb & 1) * 64;
        const int r0 = 16 * ks + 8 * h;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            f.bl[j] = trd(sB, r0, cb + 32 * j + 16 * grp);
            f.bh[j] = trd(sB, r0 + 4, cb + 32 * j + 16 * grp);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f.al[i] = trd(sA, r0, 32 * i + 16 * grp);
            f.ah[i] = trd(sA, r0 + 4, 32 * i + 16 * grp);
        }
    };
    // wait until at most `later` LDS reads (the other set's, issued after f's) are outstanding
    auto fwait12 = [](Frag& f) {
        asm volatile("s_waitcnt lgkmcnt(12)"
                     : "+v"(f.al[0]), "+v"(f.al[1]), "+v"(f.al[2]), "+v"(f.al[3]), "+v"(f.ah[0]), "+v"(f.ah[1]),
                       "+v"(f.ah[2]), "+v"(f.ah[3]), "+v"(f.bl[0]), "+v"(f.bl[1]), "+v"(f.bh[0]), "+v"(f.bh[1])
                     :
                     : "memory");
    };
    auto fwait0 = [](Frag& f) {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(f.al[0]), "+v"(f.al[1]), "+v"(f.al[2]), "+v"(f.al[3]), "+v"(f.ah[0]), "+v"(f.ah[1]),
                       "+v"(f.ah[2]), "+v"(f.ah[3]), "+v"(f.bl[0]), "+v"(f.bl[1]), "+v"(f.bh[0]), "+v"(f.bh[1])
                     :
                     : "memory");
    };
    auto fmma = [&](const Frag& f) {
        bf16x8 a[4], b[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = join(f.bl[j], f.bh[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = join(f.al[i], f.ah[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    };

    if (IP == 4 && ns > 0) {  // block-uniform
        // IP 4 (ablation build): the two waves of a SIMD (wid and wid + 4, the halves wa = 0 / 1)
        // run one k-step apart, so one waits on its LDS reads, the DMA or the barrier while the
        // other issues MFMAs (with one barrier per stage the two otherwise run in lockstep and wait
        // together).  The lagging half still reads stage st - 1 after stage st's barrier, so the
        // ring keeps two stages ahead (slots: st - 1, st, st + 1, st + 2).  Same MFMAs in the same
        // order per wave (bit-identical).
        issue(0, 0);
        issue(min(1, ns - 1), 1);
        const int lag = wa;
        for (int it = 0; it <= 2 * ns; ++it) {
            if ((it & 1) == 0 && it < 2 * ns) {  // uniform: every wave meets ns barriers
                const int st = it >> 1;
                // stage st landed (own DMAs: st + 1 outstanding); the barrier publishes it and
                // retires every wave's reads of stage st - 2 (the lagging half's last: iteration 2st-2)
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                issue(min(st + 2, ns - 1), (st + 2) % TD_STAGES);
            }
            const int hs = it - lag;  // this wave's half-step (wave-uniform)
            if (hs >= 0 && hs < 2 * ns) {
                kstep((hs >> 1) % TD_STAGES, hs & 1);
                if (!BR && do_bias && (hs & 1)) bias_rows((hs >> 1) % TD_STAGES);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    } else if (IP == 5 && ns > 0) {  // block-uniform
        // IP 5 (ablation build): IP 1's schedule (4 stages, 3 in flight, DMAs after the MFMAs) with
        // the bias sums from the fragments in registers
        issue(0, 0);
        issue(min(1, ns - 1), 1);
        issue(min(2, ns - 1), 2);
        for (int st = 0; st < ns; ++st) {
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            kstep(st % TD_STAGES, 0);
            kstep(st % TD_STAGES, 1);
            issue(min(st + 3, ns - 1), (st + 3) % TD_STAGES);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    } else if (PF && ns > 0) {  // block-uniform
        issue(0, 0);
        issue(min(1, ns - 1), 1);
        issue(min(2, ns - 1), 2);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // step 0 landed (own DMAs)
        __builtin_amdgcn_s_barrier();
        Frag f0, f1;
        fread(f0, 0, 0);
        for (int st = 0; st < ns; ++st) {
            const int stg = st % TD_STAGES;
            // the stage's bias rows as asm reads issued before f1's fragments: the fragment wait
            // below (at most f1's 12 reads outstanding) retires them too, and no compiler wait for
            // them (which, counting in order, would have waited for f1's reads as well) remains
            u32x4 bv[2] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
            if (do_bias) {  // block-uniform
                const char* sA = smem + stg * TD_STG + (ch >> 4) * HALF;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if (i > 0 && bsplit) break;
                    const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(sA + tn_off(lrow + 16 * i, ch & 15));
                    asm volatile("ds_read_b128 %0, %1" : "=v"(bv[i]) : "v"(addr) : "memory");
                }
            }
            fread(f1, stg, 1);
            fwait12(f0);
            asm volatile("" : "+v"(bv[0]), "+v"(bv[1])::"memory");  // (after the wait that retired them)
            fmma(f0);
            if (do_bias) bias_add(bv);
            // step st+1 landed (own DMAs: st+1, st+2 outstanding, st+3 not yet issued); the barrier
            // publishes it and retires every wave's reads of stage (st+3) % 4 = (st-1) % 4
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            issue(min(st + 3, ns - 1), (st + 3) % TD_STAGES);
            if (st + 1 < ns) fread(f0, (st + 1) % TD_STAGES, 0);
            if (st + 1 < ns) fwait12(f1);
            else fwait0(f1);
            fmma(f1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    } else if (ns > 0) {  // block-uniform
        issue(0, 0);
        issue(min(1, ns - 1), 1);  // past the end: re-reads of the last step, never consumed
        issue(min(2, ns - 1), 2);
        for (int st = 0; st < ns; ++st) {
            // step st has landed when at most steps st+1, st+2 (4 DMAs each) are outstanding; the
            // barrier publishes every wave's DMAs and retires step st-1's reads of stage (st+3)%4
            ND_STAMP(0);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            ND_STAMP(1);
            __builtin_amdgcn_s_barrier();
            ND_STAMP(2);
            auto nxt = [&](int) { issue(min(st + 3, ns - 1), (st + 3) % TD_STAGES); };
            auto nxt1 = [&](int i) { issue1(min(st + 3, ns - 1), (st + 3) % TD_STAGES, i); };
            if constexpr (IP == 3) {
                u32x4 bv[TD_STEP / 16];
                if (do_bias) bias_load(st % TD_STAGES, bv);  // block-uniform
#if SPN_TN_ADDR
                compute_fo(st % TD_STAGES, nxt1);
#else
                compute(st % TD_STAGES, nxt1);
#endif
                ND_STAMP(7);
                if (do_bias) bias_add(bv);
                ND_STAMP(8);
                continue;
            } else if constexpr (IP == 2) {
                compute(st % TD_STAGES, nxt);
            } else if constexpr (IP == 1) {
                compute(st % TD_STAGES, [](int) {});
                nxt(0);
                ND_STAMP(7);
            } else {
                nxt(0);
                if (!(g.dbg & 1)) compute(st % TD_STAGES, [](int) {});
            }
            if (do_bias) bias_rows(st % TD_STAGES);
            ND_STAMP(8);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    }
#ifdef ND_STAMPS
    if (st_on) g.stamps[st_base + 4095] = st_n;
#endif

    float* slab = g.slab + (int64_t)split * g.slab_stride;
    const int r32 = lane & 31;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = k0 + wb * 64 + j * 32 + r32;
        if (k >= g.K) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wa * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < g.N) slab[(int64_t)n * g.ld_slab + k] = acc[i][j][r];
            }
    }
    if constexpr (BR) {
        if (rb_on) {  // wave-uniform: lanes l and l + 32 hold the two point halves of one feature
            const float other = __shfl_down(rbias, 32, 64);
            if (lane < 32) g.slab_b[(int64_t)split * g.N + n0 + 128 * (wid >> 2) + 32 * wb + lane] = rbias + other;
        }
    } else if (do_bias && bsplit) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [32 phases][128 features]
        const int cl = ch & 15;
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lrow * 128 + 8 * cl + e] = bs[e];
        __syncthreads();
        const int n = n0 + 128 * kt + tid;
        if (tid < 128 && n < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 32; ++ph) s += red[ph * 128 + tid];
            g.slab_b[(int64_t)split * g.N + n] = s;
        }
    } else if (do_bias) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [16 phases][256 features]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lrow * 256 + 8 * ch + e] = bs[e];
        __syncthreads();
        if (tid < 256 && n0 + tid < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 16; ++ph) s += red[ph * 256 + tid];
            g.slab_b[(int64_t)split * g.N + n0 + tid] = s;
        }
    }
}

#ifdef SPN_ABLATIONS
// Weight-gradient kernels measured slower than k_gemm_tn_bf16d in the C4 step: the
// 16x16x32 pipelined kernels (8 and 16 waves) and the quad-wave kernel — compiled only into
// -DSPN_ABLATIONS builds (tools/tn_lab, the A/B variant libraries).
// Weight gradients on v_mfma_f32_16x16x32_bf16 (option tn_bf16_m16): k_gemm_tn_bf16d's 256 x 256
// block tile, 32-point LDS-DMA stages and bias sums, but a wave's 128 x 64 is 8 x 4 accumulators
// of 16 x 16 and one stage is exactly one 32-point k-step.  The same LDS bytes per FLOP as the
// 32x32x16 form (a fragment is 8 points of one feature per lane either way), at a lower energy
// per FLOP (MI355X_MICROARCH.md, DVFS item 7: 1.12-1.15x the FLOP/s of 32x32x16 at equal cycles).
// The fragments are software-pipelined: a[i + 2]'s transposed reads are issued before a[i]'s four
// MFMAs, each group waits only for its own fragment (counted lgkmcnt, LDS returns in order), and
// the stage barrier sits before the last two groups, so the next stage's B and first two A
// fragments are read under this stage's last MFMAs — no group waits for a read issued in its own
// gap, and no wave drains its LDS queue at the barrier.  The DMA of stage st + NSTG - 1 is issued
// right after stage st's barrier into the slot stage st - 1 used (every wave has consumed it).
// Each output element sums its points in 32-point MFMA blocks in point order: fixed and
// deterministic, but not k_gemm_tn_bf16d's 16-point blocks, so the fp32 slabs round differently.
template <int NSTG>
__global__ __launch_bounds__(512) void k_gemm_tn_bf16m(TN16Group G) {
    static_assert(NSTG == 4 || NSTG == 5, "4 or 5 DMA stages (5 x 32 KB = the whole LDS)");
    __shared__ __attribute__((aligned(16))) char smem[NSTG * TD_STG];  // [stage][A0|A1|B0|B1]
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    int gi = 0;
    while (gi + 1 < G.n && wg >= G.start[gi + 1]) ++gi;
    const int w = wg - G.start[gi];
    const TN16Args& g = G.g[gi];
    const int nK = (g.K + TW - 1) / TW;
    const int ntiles = cdiv(g.N, TW) * nK;
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * TW, k0 = (t % nK) * TW;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const bool bsplit = g.bias_split && nK == 2;
    const int kt = t % nK;
    const bool do_bias = g.slab_b != nullptr && (bsplit || k0 == 0);
    const int ns = p_end > p_beg ? (p_end - p_beg) / TD_STEP : 0;  // whole steps (host-checked)

    // DMA sources: as k_gemm_tn_bf16d
    const bf16* src[4];
    int64_t dl[4];
    int ld[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = wid + 8 * i, X = q >> 4, hf = (q >> 3) & 1, rg = q & 7;
        const int row = rg * 4 + (lane >> 4);
        const int chl = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int f = (X ? k0 : n0) + hf * 128 + 8 * chl;
        if (X == 0) {
            src[i] = g.A + (int64_t)row * g.lda + min(f, g.N - 8);
            dl[i] = (int64_t)((intptr_t)g.A_s2 - (intptr_t)g.A);
            ld[i] = g.lda;
        } else {
            const int kc = min(f, g.K - 8);
            const bool s2 = __builtin_amdgcn_readfirstlane(kc >= g.K1 ? 1 : 0) != 0;
            ld[i] = s2 ? g.ldb2 : g.ldb;
            src[i] = (s2 ? g.B2 + (kc - g.K1) : g.B + kc) + (int64_t)row * ld[i];
            dl[i] = s2 ? (int64_t)((intptr_t)g.B2_s2 - (intptr_t)g.B2) : (int64_t)((intptr_t)g.B_s2 - (intptr_t)g.B);
        }
    }
    const int64_t P1 = g.P1;
    auto issue = [&](int st, int stg) {
        const int64_t p0 = p_beg + (int64_t)TD_STEP * st;
        const bool sg2 = p0 >= P1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = wid + 8 * i;
            const char* a = reinterpret_cast<const char*>(src[i] + p0 * ld[i]) + (sg2 ? dl[i] : 0);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)a, (lds_ptr_t)(smem + stg * TD_STG + q * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int wa = wid >> 2, wb = wid & 3;
    const int g16 = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
    constexpr int HALF = TD_STEP * 256;
    // 16x16x32 operand of 16 features (cols 16m .. 16m + 15 of a half image) x 32 points: lane l
    // holds feature 16m + l % 16, points 8 (l / 16) .. + 7 — the 16-lane group g reads rows
    // 8g .. 8g + 3 (lo) and 8g + 4 .. 8g + 7 (hi) transposed; lane 4q + p of the group addresses
    // row + q, columns 16m + 4p .. + 3 (cdna_hip_programming.md T10: a half's two blocks 8 rows
    // apart in the same columns, conflict-free).  In tn_off's swizzle, column block m only flips
    // address bits 5..7: off(m) = off(0) ^ 32m, so a read is one v_xor from a per-stage lane address
    // (24 hoisted per-fragment addresses spilled, and a spill reload's vmcnt(0) drains the DMA ring)
    const int rlo = 8 * g16 + q4;
    const int olo = tn_off(rlo, pp >> 1) + 8 * (pp & 1), ohi = tn_off(rlo + 4, pp >> 1) + 8 * (pp & 1);
    auto lds_addr = [&](int stg, int half, int o) -> uint32_t {
        return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(smem + stg * TD_STG + half * HALF) +
               (uint32_t)opaque(o);
    };
    auto trd = [](uint32_t base, int m) -> s16x4 {
        s16x4 v;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(base ^ (uint32_t)(32 * m)) : "memory");
        return v;
    };
    auto join = [](s16x4 lo, s16x4 hi) -> bf16x8 {
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    const int mb = (wb & 1) * 4;  // B column blocks of this wave: 4 (wb & 1) + j
    auto readB = [&](s16x4& bl, s16x4& bh, int stg, int j) {
        bl = trd(lds_addr(stg, 2 + (wb >> 1), olo), mb + j);
        bh = trd(lds_addr(stg, 2 + (wb >> 1), ohi), mb + j);
    };
    auto readA = [&](s16x4& al, s16x4& ah, int stg, int i) {
        al = trd(lds_addr(stg, wa, olo), i);
        ah = trd(lds_addr(stg, wa, ohi), i);
    };
    auto mma = [&](int i, s16x4 al, s16x4 ah, int j, s16x4 bl, s16x4 bh) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(join(al, ah), join(bl, bh), acc[i][j], 0, 0, 0);
    };
#define TNM_WAIT(N, x, y) asm volatile("s_waitcnt lgkmcnt(" #N ")" : "+v"(x), "+v"(y) : : "memory")

    // bias: thread (chunk ch of 32, row phase lrow of 16) sums rows lrow, lrow + 16 of each stage;
    // bsplit: thread (chunk ch of the tile's 16, row phase lrow of 32) sums row lrow — read by asm
    // (ordered among the fragment reads; consumed behind a later fragment wait)
    const int ch = bsplit ? 16 * kt + (tid & 15) : tid & 31, lrow = bsplit ? tid >> 4 : tid >> 5;
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto brd = [&](int stg, int row) -> u32x4 {
        const uint32_t addr = lds_addr(stg, ch >> 4, tn_off(row, ch & 15));
        u32x4 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
        return v;
    };
    auto badd = [&](u32x4 v) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) bs[e] += f[e];
    };

    if (ns > 0) {  // block-uniform
#pragma unroll
        for (int s = 0; s < NSTG - 1; ++s) issue(min(s, ns - 1), s);  // past the end: re-reads, never consumed
        if constexpr (NSTG == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // stage 0 landed (own DMAs)
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        s16x4 bl[4], bh[4], al[8], ah[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) readB(bl[j], bh[j], 0, j);
        readA(al[0], ah[0], 0, 0);
        readA(al[1], ah[1], 0, 1);
        for (int st = 0; st < ns; ++st) {
            const int stg = st % NSTG;
            u32x4 bv0 = u32x4{0u, 0u, 0u, 0u}, bv1 = u32x4{0u, 0u, 0u, 0u};
            // i = 0 .. 5: a[i + 2] read, a[i] waited (4 younger reads — the bias reads, older than
            // a[2], only make the wait stricter), four MFMAs
            if (do_bias) {  // block-uniform
                bv0 = brd(stg, lrow);
                if (!bsplit) bv1 = brd(stg, lrow + 16);
            }
            readA(al[2], ah[2], stg, 2);
            asm volatile("s_waitcnt lgkmcnt(4)"
                         : "+v"(al[0]), "+v"(ah[0]), "+v"(bl[0]), "+v"(bl[1]), "+v"(bl[2]), "+v"(bl[3]), "+v"(bh[0]),
                           "+v"(bh[1]), "+v"(bh[2]), "+v"(bh[3])
                         :
                         : "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(0, al[0], ah[0], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            readA(al[3], ah[3], stg, 3);
            TNM_WAIT(4, al[1], ah[1]);
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(1, al[1], ah[1], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            readA(al[4], ah[4], stg, 4);
            asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(al[2]), "+v"(ah[2]), "+v"(bv0), "+v"(bv1) : : "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(2, al[2], ah[2], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            if (do_bias) {
                badd(bv0);
                if (!bsplit) badd(bv1);
            }
            readA(al[5], ah[5], stg, 5);
            TNM_WAIT(4, al[3], ah[3]);
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(3, al[3], ah[3], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            readA(al[6], ah[6], stg, 6);
            TNM_WAIT(4, al[4], ah[4]);
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(4, al[4], ah[4], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            readA(al[7], ah[7], stg, 7);
            TNM_WAIT(4, al[5], ah[5]);
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(5, al[5], ah[5], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            const bool more = st + 1 < ns;
            if (more) {  // block-uniform
                // stage st + 1 landed (own DMAs: at most NSTG - 3 younger stages outstanding); the
                // barrier publishes it and retires every wave's reads of slot (st - 1) % NSTG
                if constexpr (NSTG == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                issue(min(st + NSTG - 1, ns - 1), (st + NSTG - 1) % NSTG);
            }
            // the last two groups column by column: b[j] is free after (a6, bj), (a7, bj), and the
            // next stage's b[j] is read into it (then its a[0], a[1])
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(al[6]), "+v"(ah[6]), "+v"(al[7]), "+v"(ah[7]) : : "memory");
            const int nstg = (st + 1) % NSTG;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                mma(6, al[6], ah[6], j, bl[j], bh[j]);
                mma(7, al[7], ah[7], j, bl[j], bh[j]);
                __builtin_amdgcn_sched_barrier(0);
                if (more) readB(bl[j], bh[j], nstg, j);
            }
            if (more) {
                readA(al[0], ah[0], nstg, 0);
                readA(al[1], ah[1], nstg, 1);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    }
#undef TNM_WAIT

    float* slab = g.slab + (int64_t)split * g.slab_stride;
    const int c16 = lane & 15;
    // (N and K are multiples of 256 on this kernel: tn_wide, host-checked)
    const int64_t lds_ = g.ld_slab;
    float* sp = slab + (int64_t)(n0 + wa * 128 + 4 * g16) * lds_ + k0 + wb * 64 + c16;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) sp[(int64_t)(i * 16 + r) * lds_ + j * 16] = acc[i][j][r];
    if (do_bias && bsplit) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [32 phases][128 features]
        const int cl = ch & 15;
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lrow * 128 + 8 * cl + e] = bs[e];
        __syncthreads();
        const int n = n0 + 128 * kt + tid;
        if (tid < 128 && n < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 32; ++ph) s += red[ph * 128 + tid];
            g.slab_b[(int64_t)split * g.N + n] = s;
        }
    } else if (do_bias) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [16 phases][256 features]
#pragma unroll
        for (int e = 0; e < 8; ++e) red[lrow * 256 + 8 * ch + e] = bs[e];
        __syncthreads();
        if (tid < 256 && n0 + tid < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 16; ++ph) s += red[ph * 256 + tid];
            g.slab_b[(int64_t)split * g.N + n0 + tid] = s;
        }
    }
}

// Weight gradients with 16 waves per block (option tn_bf16_m16 3 / 4): the 256 x 256 block tile and
// 32-point LDS-DMA stages of k_gemm_tn_bf16d (the L2 -> CU bytes per FLOP of a 256 x 256 tile), but
// 16 waves of 64 x 64 (4 x 4 accumulators of v_mfma_f32_16x16x32_bf16, 64 registers): four waves
// per SIMD instead of two, so a wave waiting on its LDS reads, the DMA or the barrier leaves three
// others to issue MFMAs.  Per stage a wave reads its 4 B fragments once and streams its A
// fragments one ahead (counted lgkmcnt); the barrier sits before the last A fragment's MFMAs, which
// run column by column so each freed B register pair takes the next stage's fragment at once.
// The bias sums ride along: one 16-B row chunk per thread and stage, read among the fragments.
template <int NSTG>
__global__ __launch_bounds__(1024) void k_gemm_tn_bf16x(TN16Group G) {
    static_assert(NSTG == 4 || NSTG == 5, "4 or 5 DMA stages");
    __shared__ __attribute__((aligned(16))) char smem[NSTG * TD_STG];  // [stage][A0|A1|B0|B1]
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    int gi = 0;
    while (gi + 1 < G.n && wg >= G.start[gi + 1]) ++gi;
    const int w = wg - G.start[gi];
    const TN16Args& g = G.g[gi];
    const int nK = (g.K + TW - 1) / TW;
    const int ntiles = cdiv(g.N, TW) * nK;
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * TW, k0 = (t % nK) * TW;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const bool bsplit = g.bias_split && nK == 2;
    const int kt = t % nK;
    // bias: !bsplit — thread (row tid / 32, chunk tid % 32) of the stage's 32 x 256 A rows;
    // bsplit — threads < 512: (row tid / 16, chunk 16 kt + tid % 16), the tile's 128-feature half
    const bool do_bias = g.slab_b != nullptr && (bsplit || k0 == 0);
    const bool t_bias = do_bias && (!bsplit || tid < 512);  // wave-uniform
    const int ns = p_end > p_beg ? (p_end - p_beg) / TD_STEP : 0;  // whole steps (host-checked)

    // DMA: instruction q = wid + 16 i (i = 0: A, 1: B) fills 4 rows x 256 B of one half image
    const bf16* src[2];
    int64_t dl[2];
    int ld[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = wid + 16 * i, hf = (q >> 3) & 1, rg = q & 7;
        const int row = rg * 4 + (lane >> 4);
        const int chl = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int f = (i ? k0 : n0) + hf * 128 + 8 * chl;
        if (i == 0) {
            src[i] = g.A + (int64_t)row * g.lda + min(f, g.N - 8);
            dl[i] = (int64_t)((intptr_t)g.A_s2 - (intptr_t)g.A);
            ld[i] = g.lda;
        } else {
            const int kc = min(f, g.K - 8);
            const bool s2 = __builtin_amdgcn_readfirstlane(kc >= g.K1 ? 1 : 0) != 0;
            ld[i] = s2 ? g.ldb2 : g.ldb;
            src[i] = (s2 ? g.B2 + (kc - g.K1) : g.B + kc) + (int64_t)row * ld[i];
            dl[i] = s2 ? (int64_t)((intptr_t)g.B2_s2 - (intptr_t)g.B2) : (int64_t)((intptr_t)g.B_s2 - (intptr_t)g.B);
        }
    }
    const int64_t P1 = g.P1;
    auto issue = [&](int st, int stg) {
        const int64_t p0 = p_beg + (int64_t)TD_STEP * st;
        const bool sg2 = p0 >= P1;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = wid + 16 * i;
            const char* a = reinterpret_cast<const char*>(src[i] + p0 * ld[i]) + (sg2 ? dl[i] : 0);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)a, (lds_ptr_t)(smem + stg * TD_STG + q * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int wa = wid >> 2, wb = wid & 3;
    const int g16 = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
    constexpr int HALF = TD_STEP * 256;
    // fragment reads as k_gemm_tn_bf16m: off(column block m) = off(0) ^ 32 m
    const int rlo = 8 * g16 + q4;
    const int olo = tn_off(rlo, pp >> 1) + 8 * (pp & 1), ohi = tn_off(rlo + 4, pp >> 1) + 8 * (pp & 1);
    auto lds_addr = [&](int stg, int half, int o) -> uint32_t {
        return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(smem + stg * TD_STG + half * HALF) +
               (uint32_t)opaque(o);
    };
    auto trd = [](uint32_t base, int m) -> s16x4 {
        s16x4 v;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(base ^ (uint32_t)(32 * m)) : "memory");
        return v;
    };
    auto join = [](s16x4 lo, s16x4 hi) -> bf16x8 {
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    // A: features wa * 64 + 16 i (half wa / 2, column block 4 (wa & 1) + i); B likewise with wb
    auto readB = [&](s16x4& bl, s16x4& bh, int stg, int j) {
        bl = trd(lds_addr(stg, 2 + (wb >> 1), olo), 4 * (wb & 1) + j);
        bh = trd(lds_addr(stg, 2 + (wb >> 1), ohi), 4 * (wb & 1) + j);
    };
    auto readA = [&](s16x4& al, s16x4& ah, int stg, int i) {
        al = trd(lds_addr(stg, wa >> 1, olo), 4 * (wa & 1) + i);
        ah = trd(lds_addr(stg, wa >> 1, ohi), 4 * (wa & 1) + i);
    };
    auto mma = [&](int i, s16x4 al, s16x4 ah, int j, s16x4 bl, s16x4 bh) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(join(al, ah), join(bl, bh), acc[i][j], 0, 0, 0);
    };

    const int brow = bsplit ? (tid >> 4) & 31 : tid >> 5;
    const int bch = bsplit ? 16 * kt + (tid & 15) : tid & 31;
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto brd = [&](int stg) -> u32x4 {
        const uint32_t addr = lds_addr(stg, bch >> 4, tn_off(brow, bch & 15));
        u32x4 v;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
        return v;
    };

    if (ns > 0) {  // block-uniform
#pragma unroll
        for (int s = 0; s < NSTG - 1; ++s) issue(min(s, ns - 1), s);  // past the end: re-reads, never consumed
        if constexpr (NSTG == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // stage 0 landed (own DMAs)
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        s16x4 bl[4], bh[4], al[4], ah[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) readB(bl[j], bh[j], 0, j);
        readA(al[0], ah[0], 0, 0);
        for (int st = 0; st < ns; ++st) {
            const int stg = st % NSTG;
            readA(al[1], ah[1], stg, 1);
            asm volatile("s_waitcnt lgkmcnt(2)"
                         : "+v"(al[0]), "+v"(ah[0]), "+v"(bl[0]), "+v"(bl[1]), "+v"(bl[2]), "+v"(bl[3]), "+v"(bh[0]),
                           "+v"(bh[1]), "+v"(bh[2]), "+v"(bh[3])
                         :
                         : "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(0, al[0], ah[0], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            readA(al[2], ah[2], stg, 2);
            asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(al[1]), "+v"(ah[1]) : : "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(1, al[1], ah[1], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            u32x4 bv = u32x4{0u, 0u, 0u, 0u};
            if (t_bias) bv = brd(stg);  // wave-uniform; older than a[3]: covered by the next wait
            readA(al[3], ah[3], stg, 3);
            asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(al[2]), "+v"(ah[2]), "+v"(bv) : : "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) mma(2, al[2], ah[2], j, bl[j], bh[j]);
            __builtin_amdgcn_sched_barrier(0);
            if (t_bias) {
                float f[8];
                unpack8(bv, f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[e] += f[e];
            }
            const bool more = st + 1 < ns;
            if (more) {  // block-uniform
                // stage st + 1 landed (own DMAs: at most NSTG - 3 younger stages outstanding); the
                // barrier publishes it and retires every wave's reads of slot (st - 1) % NSTG
                if constexpr (NSTG == 4) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                issue(min(st + NSTG - 1, ns - 1), (st + NSTG - 1) % NSTG);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(al[3]), "+v"(ah[3]) : : "memory");
            const int nstg = (st + 1) % NSTG;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                mma(3, al[3], ah[3], j, bl[j], bh[j]);
                __builtin_amdgcn_sched_barrier(0);
                if (more) readB(bl[j], bh[j], nstg, j);
            }
            if (more) readA(al[0], ah[0], nstg, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    }

    float* slab = g.slab + (int64_t)split * g.slab_stride;
    const int c16 = lane & 15;
    // (N and K are multiples of 256 on this kernel: tn_wide, host-checked)
    const int64_t lds_ = g.ld_slab;
    float* sp = slab + (int64_t)(n0 + wa * 64 + 4 * g16) * lds_ + k0 + wb * 64 + c16;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) sp[(int64_t)(i * 16 + r) * lds_ + j * 16] = acc[i][j][r];
    if (do_bias) {  // block-uniform
        const int nf = bsplit ? 128 : 256;  // features summed by this tile
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [32 row phases][nf features]
        if (t_bias) {
            const int cl = bsplit ? (bch & 15) : bch;
#pragma unroll
            for (int e = 0; e < 8; ++e) red[brow * nf + 8 * cl + e] = bs[e];
        }
        __syncthreads();
        const int n = n0 + (bsplit ? 128 * kt : 0) + tid;
        if (tid < nf) {
            float s = 0.f;
            for (int ph = 0; ph < 32; ++ph) s += red[ph * nf + tid];
            g.slab_b[(int64_t)split * g.N + n] = s;
        }
    }
}

// Quad-wave DMA weight-gradient GEMM (option tn_bf16_quad): the 256x256 tile and LDS-DMA ring
// of k_gemm_tn_bf16d, but 4 waves (one per SIMD) of 128x128 each (4 x 4 32x32 accumulators, 256
// registers): 16 MFMAs per 16 fragment reads instead of 8 per 12, and the next k-step's fragments
// read while the current k-step's MFMAs run (two register sets) — a single wave per SIMD has no
// partner to hide its LDS latency. Same per-element k-order as k_gemm_tn_bf16d (bit-identical).
__global__ __launch_bounds__(256) void k_gemm_tn_bf16q(TN16Group G) {
    __shared__ __attribute__((aligned(16))) char smem[TD_STAGES * TD_STG];  // [stage][A0|A1|B0|B1]
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    int gi = 0;
    while (gi + 1 < G.n && wg >= G.start[gi + 1]) ++gi;
    const int w = wg - G.start[gi];
    const TN16Args& g = G.g[gi];
    const int nK = (g.K + TW - 1) / TW;
    const int ntiles = cdiv(g.N, TW) * nK;
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * TW, k0 = (t % nK) * TW;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const bool bsplit = g.bias_split && nK == 2;
    const int kt = t % nK;
    const bool do_bias = g.slab_b != nullptr && (bsplit || k0 == 0);
    const int ns = p_end > p_beg ? (p_end - p_beg) / TD_STEP : 0;

    // this lane's 8 DMA sources (wave-instructions q = wid + 4 i of the stage's 32)
    const bf16* src[8];
    int64_t dl[8];
    int ld[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int q = wid + 4 * i, X = q >> 4, hf = (q >> 3) & 1, rg = q & 7;
        const int row = rg * 4 + (lane >> 4);
        const int chl = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
        const int f = (X ? k0 : n0) + hf * 128 + 8 * chl;
        if (X == 0) {
            src[i] = g.A + (int64_t)row * g.lda + min(f, g.N - 8);
            dl[i] = (int64_t)((intptr_t)g.A_s2 - (intptr_t)g.A);
            ld[i] = g.lda;
        } else {
            const int kc = min(f, g.K - 8);
            const bool s2 = __builtin_amdgcn_readfirstlane(kc >= g.K1 ? 1 : 0) != 0;
            ld[i] = s2 ? g.ldb2 : g.ldb;
            src[i] = (s2 ? g.B2 + (kc - g.K1) : g.B + kc) + (int64_t)row * ld[i];
            dl[i] = s2 ? (int64_t)((intptr_t)g.B2_s2 - (intptr_t)g.B2) : (int64_t)((intptr_t)g.B_s2 - (intptr_t)g.B);
        }
    }
    const int64_t P1 = g.P1;
    auto issue = [&](int st, int stg) {
        const int64_t p0 = p_beg + (int64_t)TD_STEP * st;
        const bool sg2 = p0 >= P1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int q = wid + 4 * i;
            const char* a = reinterpret_cast<const char*>(src[i] + p0 * ld[i]) + (sg2 ? dl[i] : 0);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)a, (lds_ptr_t)(smem + stg * TD_STG + q * 1024), 16, 0, 0);
        }
    };

    f32x16 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int wa = wid >> 1, wb = wid & 1, h = lane >> 5, grp = (lane >> 4) & 1;
    const int q4 = (lane & 15) >> 2, pp = lane & 3;
    auto trd = [&](const char* base, int r0, int col) -> s16x4 {
        const int o = tn_off(r0 + q4, (col >> 3) + (pp >> 1)) + 8 * (pp & 1);
        const uint32_t addr = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(base + o);
        s16x4 v;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr) : "memory");
        return v;
    };
    auto join = [](s16x4 lo, s16x4 hi) -> bf16x8 {
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        return __builtin_bit_cast(bf16x8, v);
    };
    constexpr int HALF = TD_STEP * 256;
    struct Frag {
        s16x4 al[4], ah[4], bl[4], bh[4];
    };
    auto fread = [&](Frag& f, int stg, int ks) {
        const char* sA = smem + stg * TD_STG + wa * HALF;
        const char* sB = smem + stg * TD_STG + (2 + wb) * HALF;
        const int r0 = 16 * ks + 8 * h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            f.bl[j] = trd(sB, r0, 32 * j + 16 * grp);
            f.bh[j] = trd(sB, r0 + 4, 32 * j + 16 * grp);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f.al[i] = trd(sA, r0, 32 * i + 16 * grp);
            f.ah[i] = trd(sA, r0 + 4, 32 * i + 16 * grp);
        }
    };
    // at most 15 LDS operations (the other set's reads, issued after f's) left in flight
    auto fwait = [](Frag& f, auto cnt) {
        if constexpr (decltype(cnt)::value == 15)
            asm volatile("s_waitcnt lgkmcnt(15)"
                         : "+v"(f.al[0]), "+v"(f.al[1]), "+v"(f.al[2]), "+v"(f.al[3]), "+v"(f.ah[0]), "+v"(f.ah[1]),
                           "+v"(f.ah[2]), "+v"(f.ah[3]), "+v"(f.bl[0]), "+v"(f.bl[1]), "+v"(f.bl[2]), "+v"(f.bl[3]),
                           "+v"(f.bh[0]), "+v"(f.bh[1]), "+v"(f.bh[2]), "+v"(f.bh[3])
                         :
                         : "memory");
        else
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(f.al[0]), "+v"(f.al[1]), "+v"(f.al[2]), "+v"(f.al[3]), "+v"(f.ah[0]), "+v"(f.ah[1]),
                           "+v"(f.ah[2]), "+v"(f.ah[3]), "+v"(f.bl[0]), "+v"(f.bl[1]), "+v"(f.bl[2]), "+v"(f.bl[3]),
                           "+v"(f.bh[0]), "+v"(f.bh[1]), "+v"(f.bh[2]), "+v"(f.bh[3])
                         :
                         : "memory");
    };
    auto fmma = [&](const Frag& f) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = join(f.bl[j], f.bh[j]);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = join(f.al[i], f.ah[i]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    };
    // bias: the per-phase sums of k_gemm_tn_bf16d in the same order (bit-identical), two phases per
    // thread: bsplit: chunk ch of the tile's 16, phases lrow and lrow + 16 (row = phase);
    // else chunk ch of 32, phases lrow and lrow + 8 (rows phase and phase + 16)
    const int ch = bsplit ? 16 * kt + (tid & 15) : tid & 31, lrow = bsplit ? tid >> 4 : tid >> 5;
    float bs[2][8] = {{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
    auto bias_rows = [&](int stg) {
        const char* sA = smem + stg * TD_STG + (ch >> 4) * HALF;
        if (bsplit) {  // block-uniform
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float f[8];
                unpack8(*reinterpret_cast<const u32x4*>(sA + tn_off(lrow + 16 * i, ch & 15)), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[i][e] += f[e];
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                float f[8];
                unpack8(*reinterpret_cast<const u32x4*>(sA + tn_off(lrow + 8 * i + 16 * r, ch & 15)), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) bs[i][e] += f[e];
            }
    };
    using I0 = std::integral_constant<int, 0>;

    if (ns > 0) {  // block-uniform
        issue(0, 0);
        issue(min(1, ns - 1), 1);  // past the end: re-reads of the last step, never consumed
        issue(min(2, ns - 1), 2);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step 0 landed (own DMAs)
        __builtin_amdgcn_s_barrier();
        Frag f0, f1;
        fread(f0, 0, 0);
        // each set is waited for (lgkmcnt(0): issued a whole MFMA burst earlier) just before the
        // other set's reads are issued, so they run under this set's MFMAs
        for (int st = 0; st < ns; ++st) {
            const int stg = st % TD_STAGES;
            fwait(f0, I0{});
            fread(f1, stg, 1);
            fmma(f0);
            if (do_bias) bias_rows(stg);
            // step st+1 landed (own DMAs of st+1, st+2 outstanding); the barrier publishes it and
            // retires every wave's reads of stage (st+3) % 4 = (st-1) % 4 before it is refilled
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            issue(min(st + 3, ns - 1), (st + 3) % TD_STAGES);
            fwait(f1, I0{});
            if (st + 1 < ns) fread(f0, (st + 1) % TD_STAGES, 0);
            fmma(f1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing may land in the reused LDS
        __builtin_amdgcn_s_barrier();
    }

    float* slab = g.slab + (int64_t)split * g.slab_stride;
    const int r32 = lane & 31;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int k = k0 + wb * 128 + j * 32 + r32;
        if (k >= g.K) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wa * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (n < g.N) slab[(int64_t)n * g.ld_slab + k] = acc[i][j][r];
            }
    }
    if (do_bias && bsplit) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [32 phases][128 features]
        const int cl = ch & 15;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) red[(lrow + 16 * i) * 128 + 8 * cl + e] = bs[i][e];
        __syncthreads();
        const int n = n0 + 128 * kt + tid;
        if (tid < 128 && n < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 32; ++ph) s += red[ph * 128 + tid];
            g.slab_b[(int64_t)split * g.N + n] = s;
        }
    } else if (do_bias) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [16 phases][256 features]
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 8; ++e) red[(lrow + 8 * i) * 256 + 8 * ch + e] = bs[i][e];
        __syncthreads();
        if (n0 + tid < g.N) {
            float s = 0.f;
            for (int ph = 0; ph < 16; ++ph) s += red[ph * 256 + tid];
            g.slab_b[(int64_t)split * g.N + n0 + tid] = s;
        }
    }
}
#endif  // SPN_ABLATIONS

// ------------------------------------------------------------------------------------------
// host
// ------------------------------------------------------------------------------------------
int g_nt16_variant = 8;
int g_nt16_ip = 2;  // DMA NT / TN: where a K-step issues the next step's DMAs (0 before its MFMAs, 1 after, 2 between the k-halves)
// the weight-gradient GEMM: 1 (after a step's MFMAs) re-measured on the final round-3 tree: C4 26.69 /
// 26.72 / 26.71 -> 26.62 / 26.64 / 26.61 ms, the TN class 6.20 -> 6.09 ms per step, C4@512 level
// (tools/gpu_r3zf.sh); 2 was the better placement when the TN was measured in isolation (r02)
// round 5: 3 = the four DMA instructions of the next step one per two MFMA groups (bit-identical):
// C4 25.92 / 25.96 / 25.96 -> 25.65 / 25.77 ms, the TN class 6.52 -> 6.30 ms per step, C4@512
// 3.844 / 3.826 -> 3.812 / 3.808 ms (pairs in one call); the product build compiles only this one
constexpr int kTn16IpDefault = 3;
int g_tn16_ip = kTn16IpDefault;
int g_tn16_bias_split = 1;
int g_nt16_ip_gen = 2;  // the same for the general (bias / sine / rank-1) epilogue instances
int g_nt16_epi = 1;     // option "nt_bf16_epi": 1 = compile-time epilogue variants of the DMA NT, 0 = the generic one
int g_tn16_variant = 3;

int g_tn16_few_tiles = 1;  // option tn_bf16_few_tiles: 256x256 tiles also for 1-3 tile shapes, with more splits

static bool tn_wide(int N, int K, int variant, int few = -1) {
    const int v = variant > 0 ? variant : g_tn16_variant;
    // fewer than 4 wide tiles cannot fill the chip within the 64-split cap (N = K = 256: 64
    // blocks, 76 us against 40 us for 256 blocks of the 128x128 kernel) — so such shapes take
    // 256 / tiles splits instead (tn_splits_bf16, option tn_bf16_few_tiles): every operand row is
    // then read once (the 128x128 tiling of N = K = 256 reads each twice).  A skip-layer K (512 +
    // K0p) stays on the 128x128 kernel: a wide part + narrow tail re-reads dZ for the tail and
    // needs 64 splits (K = 576: 143 + 18 us reduction against 152 + 7)
    const int tiles = (N / TW) * (K / TW);
    return (v == 2 || v == 3) && N % TW == 0 && K % TW == 0 && (tiles >= 4 || ((few < 0 ? g_tn16_few_tiles : few) && tiles >= 1));
}

// The DMA NT GEMM's issue placement of the next K-step (IP, k_gemm_nt_bf16d): the product build
// compiles the default only; -DSPN_ABLATIONS builds every placement (options nt_bf16_ip, nt_bf16_ip_gen)
constexpr int kNt16IpDefault = 2;
template <bool DM, int EV, bool HD>
static void launch_nt16d(int ip, dim3 grid, dim3 block, hipStream_t s, const NT16Args& a, int nt) {
#ifdef SPN_ABLATIONS
    if (ip == 3) {
        hipLaunchKernelGGL((k_gemm_nt_bf16d<DM, 3, EV, HD>), grid, block, 0, s, a, nt);
        return;
    }
    if (ip == 1) {
        hipLaunchKernelGGL((k_gemm_nt_bf16d<DM, 1, EV, HD>), grid, block, 0, s, a, nt);
        return;
    }
    if (ip == 0) {
        hipLaunchKernelGGL((k_gemm_nt_bf16d<DM, 0, EV, HD>), grid, block, 0, s, a, nt);
        return;
    }
#endif
    (void)ip;
    hipLaunchKernelGGL((k_gemm_nt_bf16d<DM, kNt16IpDefault, EV, HD>), grid, block, 0, s, a, nt);
}

int32_t gemm_nt_bf16(const NT16Args& a, hipStream_t s, int variant) {
    SPN_ARG(a.M >= 0 && a.N > 0 && a.K > 0, "gemm_nt_bf16: bad shape M=%d N=%d K=%d", a.M, a.N, a.K);
    SPN_ARG(a.K % 8 == 0 && a.N % 8 == 0 && a.n_lin % 8 == 0, "gemm_nt_bf16: K, N, n_lin must be multiples of 8");
    SPN_ARG(a.K1 <= a.K && (a.K1 == a.K || (a.A2 != nullptr && a.K1 % HK == 0)),
            "gemm_nt_bf16: a split K1=%d must be a multiple of %d with A2 set", a.K1, HK);
    SPN_ARG(a.lda % 8 == 0 && a.ldb % 8 == 0 && a.ldc % 8 == 0 && (a.K1 == a.K || a.lda2 % 8 == 0),
            "gemm_nt_bf16: leading dims must be multiples of 8");
    SPN_ARG((int64_t)a.M * std::max(a.lda, a.K1 == a.K ? 0 : a.lda2) < (1ll << 31) && (int64_t)a.N * a.ldb < (1ll << 31),
            "gemm_nt_bf16: operands past 2^31 elements (32-bit DMA offsets)");
    SPN_ARG(!a.Dout || a.ld_dout % 8 == 0, "gemm_nt_bf16: ld_dout");
    SPN_ARG(!a.Dmul || a.ld_dmul % 8 == 0, "gemm_nt_bf16: ld_dmul");
    SPN_ARG(a.rowbias == nullptr || (a.rows_per_ray > 0 && a.ld_rb % 4 == 0), "gemm_nt_bf16: rowbias");
    if (a.M == 0) return SPNERF_OK;
    const int ntiles = cdiv(a.M, HB) * cdiv(a.N, HB);
    // algorithmic bytes: A and B once, C, the derivative of the sine columns, the Dmul read
    const double dcols = (a.Dout && a.act == 1) ? (double)(a.N - std::min(a.n_lin, a.N)) : 0.0;
    // variants: 1 / 2 = one block per tile, prefetch depth 1 / 2; 3 / 4 = persistent grid of
    // two blocks per CU (the LDS limit), depth 1 / 2
    int v = variant > 0 ? variant : g_nt16_variant;
    if (v == 8 && (a.K % ND_K != 0 || (a.K1 != a.K && a.K1 % ND_K != 0))) v = 5;  // DMA needs whole 32-wide K-steps
    SPN_ARG(a.hd.n == 0 || v == 8, "gemm_nt_bf16: output heads need the DMA kernel (variant 8)");
    const bool dm = a.Dmul && !a.bias && !a.rowbias && !a.r1_a && a.act == 0 && !a.Dout;
    // one profiling class per kernel function: the DMA kernel's two epilogue instances apart
    ProfScope prof(v == 8 ? (dm ? "gemm_nt_bf16d_dmul" : "gemm_nt_bf16d") : v >= 5 ? "gemm_nt_bf16w" : "gemm_nt_bf16", s,
                   2.0 * a.M * a.N * (a.k_alg > 0 ? a.k_alg : a.K),
                   2.0 * ((double)a.M * a.K + (double)a.N * a.K + (double)a.M * a.N * (1.0 + (a.Dmul ? 1.0 : 0.0)) +
                          (double)a.M * dcols));
    if (v == 8) {
        const int nt = cdiv(a.M, 256) * cdiv(a.N, 256);
        const dim3 grid(std::min(nt, num_cus())), block(512);
        if (dm) {
            const bool z = a.dmul_z != 0;   // zsave: Dmul holds Z
            const int ip = (a.dbg & 64) ? 2 : (a.dbg & 32) ? 1 : g_nt16_ip;
#ifndef SPN_ABLATIONS
            // product build: the default issue placement and no saved-Z (zsave) epilogue
            SPN_ARG(!z, "gemm_nt_bf16: a saved-Z Dmul (zsave) needs the ablation build");
            (void)ip;
            launch_nt16d<true, 0, false>(kNt16IpDefault, grid, block, s, a, nt);
#else
            if (z) launch_nt16d<true, 1, false>(ip, grid, block, s, a, nt);
            else launch_nt16d<true, 0, false>(ip, grid, block, s, a, nt);
#endif
        } else {
            // the epilogue's inputs as a compile-time variant (see k_gemm_nt_bf16d); option
            // nt_bf16_epi 0 forces the generic one
            const bool zs = a.zround || a.dout_z || a.dmul_z;
            const bool bias_ok = a.bias || a.N <= 2048;   // the zero row covers the columns
            int ev = 0;
            if (!zs && bias_ok && g_nt16_epi) {
                if (!a.Dmul && !a.r1_a && !a.rowbias) ev = 1;
                else if (!a.Dmul && !a.r1_a && a.rowbias && a.rows_per_ray % 32 == 0) ev = 2;
                else if (a.Dmul && a.r1_a && !a.rowbias && a.act == 0 && !a.Dout) ev = 3;
            }
            const int ip = g_nt16_ip_gen;
            if (a.hd.n > 0) {
                SPN_ARG((ev == 1 || ev == 2) && a.hd.n <= kNTHeads && a.hd.out && a.hd.hsave && a.N % 256 == 0,
                        "gemm_nt_bf16: output heads need the bias / per-ray-row DMA epilogue");
                for (int i = 0; i < a.hd.n; ++i)
                    SPN_ARG(a.hd.col0[i] % 256 == 0 && a.hd.col0[i] + 256 <= a.N && a.hd.nout[i] >= 1 && a.hd.nout[i] <= 3,
                            "gemm_nt_bf16: head group %d", i);
                if (ev == 1) launch_nt16d<false, 1, true>(ip, grid, block, s, a, nt);
                else launch_nt16d<false, 2, true>(ip, grid, block, s, a, nt);
            } else if (ev == 1) {
                launch_nt16d<false, 1, false>(ip, grid, block, s, a, nt);
            } else if (ev == 2) {
                launch_nt16d<false, 2, false>(ip, grid, block, s, a, nt);
            } else if (ev == 3) {
                launch_nt16d<false, 3, false>(ip, grid, block, s, a, nt);
            } else {
                launch_nt16d<false, 0, false>(ip, grid, block, s, a, nt);
            }
        }
        SPN_HIP(hipGetLastError());
        return SPNERF_OK;
    }
    if (v >= 5) {  // generalised tiles, persistent with one block per CU
        if (v == 5) {
            const int nt = cdiv(a.M, 256) * cdiv(a.N, 256);
            hipLaunchKernelGGL((k_gemm_nt_bf16w<256, 256, 2, 4>), dim3(std::min(nt, num_cus())), dim3(512), 0, s, a, nt);
        } else if (v == 6) {
            const int nt = cdiv(a.M, 256) * cdiv(a.N, 128);
            hipLaunchKernelGGL((k_gemm_nt_bf16w<256, 128, 4, 2>), dim3(std::min(nt, num_cus())), dim3(512), 0, s, a, nt);
        } else {
            const int nt = cdiv(a.M, 128) * cdiv(a.N, 256);
            hipLaunchKernelGGL((k_gemm_nt_bf16w<128, 256, 2, 2>), dim3(std::min(nt, num_cus())), dim3(256), 0, s, a, nt);
        }
        SPN_HIP(hipGetLastError());
        return SPNERF_OK;
    }
    const int resident = 2 * num_cus();
    const int grid = v >= 3 ? std::min(ntiles, resident) : ntiles;
    if (v == 1 || v == 3) hipLaunchKernelGGL(k_gemm_nt_bf16<1>, dim3(grid), dim3(256), 0, s, a, ntiles);
    else hipLaunchKernelGGL(k_gemm_nt_bf16<2>, dim3(grid), dim3(256), 0, s, a, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int g_tn16_min_points = 1024;  // fewest points per split of a bf16 weight-gradient GEMM
int g_tn16_rounds = 1;         // option tn_bf16_rounds (tn_splits_bf16): 2 measured level in the bench (C4 6.24 vs 6.19 ms TN)

int tn_splits_bf16(int P, int N, int K, int variant, int few, int cus_) {
    // the narrow kernel: one block per CU, at least half the usual points per split
    const int cus = cus_ > 0 ? cus_ : split_cus();
    if (tn_k64(N, K)) return std::max(1, std::min(cus, cdiv(P, g_tn16_min_points / 2)));
    const bool wide = tn_wide(N, K, variant, few);
    const int tiles = wide ? cdiv(N, TW) * cdiv(K, TW) : cdiv(N, HB) * cdiv(K, HB);
    // one wide block per CU, two 128x128 ones: as many splits as fill the CUs (256 on MI355X)
    // WITHOUT a second round (N = 768, K = 512 rounded up to 258 wide blocks: 221 us, two rounds)
    // (option tn_bf16_rounds: wide blocks per CU — 2 lets the blocks' ring fills and slab writes
    // fall at different times; 1 M x 512 x 512 in isolation: 750 -> 646 us)
    const int rounds = wide && tiles >= 4 && g_tn16_rounds > 1 ? 2 : 1;
    int splits = (wide ? rounds * cus : 2 * cus) / tiles;
    if (splits > (wide && tiles < 4 ? cus : 64 * rounds)) splits = wide && tiles < 4 ? cus : 64 * rounds;
    // (few wide tiles: half the points per split, so small batches still spread over the chip)
    const int max_splits = cdiv(P, wide && tiles < 4 ? g_tn16_min_points / 2 : g_tn16_min_points);
    if (splits > max_splits) splits = max_splits;
    return splits < 1 ? 1 : splits;
}

// option tn_bf16_pf: the prefetched-fragment main loop of k_gemm_tn_bf16d (1; 2 = only for launches
// of at most one block per CU). Bit-identical; in isolation (tools/tn_lab, 1 M x 512 x 512, 64
// splits) 762 -> 672 us, but in the bench slower: C4 TN class 6.17 / 6.21 -> 6.47 / 6.46 ms (1) and
// 6.20 / 6.17 -> 6.25 / 6.24 (2), C4@512 3.744 -> 3.766 (2) / 3.799 (1) — the grouped launch already
// runs two blocks per CU (as 128 splits does in isolation: 669 us) and the two do not stack. Off.
int g_tn16_pf = 0;
// option tn_bf16_quad: k_gemm_tn_bf16q (4 waves of 128x128) for the DMA weight gradients —
// bit-identical, but slower: 1 M x 512 x 512 in isolation 778 vs 792 us, with one-row (on-chip)
// operands 710 vs 498 us (MFMA busy 34% against 50%: one wave per SIMD leaves its waits and
// issue stalls uncovered; tools/pmc_tn_lab.sh); C4 TN 6.30 -> 7.9 ms per step, C4@512 3.956 -> 4.22
int g_tn16_quad = 0;
// option tn_bf16_m16: k_gemm_tn_bf16m (16x16x32 MFMAs, pipelined fragments) — 1: 4 DMA stages, 2: 5
int g_tn16_m16 = 0;

static void launch_tn_bf16d(const TN16Args* a, int n, const int* blocks, int ip, hipStream_t s) {
    TN16Group G;
    G.n = n;
    G.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        G.g[i] = a[i];
        G.start[i + 1] = G.start[i] + blocks[i];
    }
    const dim3 grid(G.start[n]), block(512);
#ifdef SPN_ABLATIONS
    if (g_tn16_m16 >= 3) {
        if (g_tn16_m16 == 4) hipLaunchKernelGGL(k_gemm_tn_bf16x<5>, grid, dim3(1024), 0, s, G);
        else hipLaunchKernelGGL(k_gemm_tn_bf16x<4>, grid, dim3(1024), 0, s, G);
        return;
    }
    if (g_tn16_m16) {
        if (g_tn16_m16 == 2) hipLaunchKernelGGL(k_gemm_tn_bf16m<5>, grid, block, 0, s, G);
        else hipLaunchKernelGGL(k_gemm_tn_bf16m<4>, grid, block, 0, s, G);
        return;
    }
    if (g_tn16_quad) {
        hipLaunchKernelGGL(k_gemm_tn_bf16q, grid, dim3(256), 0, s, G);
        return;
    }
    if (g_tn16_pf == 1 || (g_tn16_pf == 2 && G.start[n] <= num_cus())) {
        hipLaunchKernelGGL((k_gemm_tn_bf16d<1, true>), grid, block, 0, s, G);
        return;
    }
    if (ip == 2) {
        hipLaunchKernelGGL(k_gemm_tn_bf16d<2>, grid, block, 0, s, G);
        return;
    }
    if (ip == 4) {
        hipLaunchKernelGGL(k_gemm_tn_bf16d<4>, grid, block, 0, s, G);
        return;
    }
    if (ip == 5) {
        hipLaunchKernelGGL(k_gemm_tn_bf16d<5>, grid, block, 0, s, G);
        return;
    }
    if (ip == 0) {
        hipLaunchKernelGGL(k_gemm_tn_bf16d<0>, grid, block, 0, s, G);
        return;
    }
    if (ip == 1) {
        hipLaunchKernelGGL(k_gemm_tn_bf16d<1>, grid, block, 0, s, G);
        return;
    }
#else
    (void)ip;   // the product build: the default placement only, no variant kernels
#endif
    hipLaunchKernelGGL(k_gemm_tn_bf16d<kTn16IpDefault>, grid, block, 0, s, G);
}

bool tn_k64_ok(int N, int K) { return tn_k64(N, K); }

int32_t gemm_tn_bf16_k64_group(const TN16Args* a0, int n, const int* splits, hipStream_t s) {
    SPN_ARG(n >= 1 && n <= kTnGroup, "gemm_tn_bf16_k64_group: %d GEMMs (at most %d)", n, kTnGroup);
    TN16Group G;
    G.n = n;
    G.start[0] = 0;
    double flop = 0.0, bytes = 0.0;
    for (int i = 0; i < n; ++i) {
        TN16Args& q = G.g[i];
        q = a0[i];
        SPN_ARG(tn_k64(q.N, q.K) && q.K1 >= q.K && !q.b_sin && q.ld_slab == q.K && splits[i] >= 1 && q.A && q.B && q.slab,
                "gemm_tn_bf16_k64_group: GEMM %d is not a narrow N = 512, K = 64 one", i);
        SPN_ARG(q.P1 >= q.P || (q.A_s2 && q.B_s2), "gemm_tn_bf16_k64_group: second segment");
        int pps = cdiv(q.P, splits[i]);
        pps = (pps + 63) / 64 * 64;
        q.p_per_split = pps < 64 ? 64 : pps;
        G.start[i + 1] = G.start[i] + (q.P > 0 ? splits[i] : 0);
        flop += 2.0 * q.P * q.N * q.K;
        bytes += 2.0 * (double)q.P * (q.N + q.K) + 4.0 * splits[i] * ((double)q.N * q.K + (q.slab_b ? q.N : 0));
    }
    if (G.start[n] == 0) return SPNERF_OK;
    ProfScope prof("gemm_tn_bf16k", s, flop, bytes);
    hipLaunchKernelGGL(k_gemm_tn_bf16_k64, dim3(G.start[n]), dim3(512), 0, s, G);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

bool tn_group_ok(int P, int N, int K) { return g_tn16_variant == 3 && !tn_k64(N, K) && tn_wide(N, K, -1) && P % TD_STEP == 0; }
int tn_tiles_bf16(int N, int K) { return cdiv(N, TW) * cdiv(K, TW); }

int32_t gemm_tn_bf16_group(const TN16Args* a0, int n, const int* splits, hipStream_t s) {
    SPN_ARG(n >= 1 && n <= kTnGroup, "gemm_tn_bf16_group: %d GEMMs (at most %d)", n, kTnGroup);
    TN16Args a[kTnGroup];
    int blocks[kTnGroup];
    double flop = 0.0, bytes = 0.0;
    for (int i = 0; i < n; ++i) {
        a[i] = a0[i];
        const TN16Args& q = a[i];
        SPN_ARG(splits[i] >= 1 && q.K1 >= q.K && !q.b_sin, "gemm_tn_bf16_group: GEMM %d: one B segment, >= 1 split", i);
        SPN_ARG(q.lda % 8 == 0 && q.ldb % 8 == 0 && q.A && q.B && q.slab && q.slab_b, "gemm_tn_bf16_group: operands");
        const bool two = q.P1 < q.P;
        SPN_ARG(!two || (q.A_s2 && q.B_s2 && q.P1 % TD_STEP == 0), "gemm_tn_bf16_group: second segment");
        SPN_ARG(tn_group_ok(q.P, q.N, q.K), "gemm_tn_bf16_group: shape N=%d K=%d P=%d not on the DMA tiles", q.N, q.K, q.P);
        int pps = cdiv(q.P, splits[i]);
        pps = (pps + 63) / 64 * 64;
        a[i].p_per_split = pps < 64 ? 64 : pps;
        a[i].bias_split = g_tn16_bias_split;
        blocks[i] = q.P > 0 ? tn_tiles_bf16(q.N, q.K) * splits[i] : 0;
        flop += 2.0 * q.P * q.N * q.K;
        bytes += 2.0 * (double)q.P * (q.N + q.K) + 4.0 * splits[i] * (double)q.N * q.K;
    }
    int total = 0;
    for (int i = 0; i < n; ++i) total += blocks[i];
    if (total == 0) return SPNERF_OK;
    ProfScope prof("gemm_tn_bf16d", s, flop, bytes);
    launch_tn_bf16d(a, n, blocks, g_tn16_ip, s);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
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
    const bool wide = tn_wide(a.N, a.K, -1);
    const bool two = a.P1 < a.P;
    SPN_ARG(!two || (a.A_s2 && a.B_s2 && (a.K1 >= a.K || a.B2_s2)), "gemm_tn_bf16: second segment incomplete");
    if (tn_k64(a.N, a.K) && a.K1 >= a.K && !a.b_sin && a.ld_slab == a.K) {
        ProfScope prof("gemm_tn_bf16k", s, 2.0 * a.P * a.N * a.K,
                       2.0 * (double)a.P * (a.N + a.K) + 4.0 * splits * ((double)a.N * a.K + a.N));
        TN16Group G;
        G.g[0] = a;
        G.n = 1;
        G.start[0] = 0;
        G.start[1] = splits;
        hipLaunchKernelGGL(k_gemm_tn_bf16_k64, dim3(splits), dim3(512), 0, s, G);
        SPN_HIP(hipGetLastError());
        return SPNERF_OK;
    }
    // DMA: whole 32-point steps (and a segment boundary on a step)
    const bool dma = wide && g_tn16_variant == 3 && a.P % TD_STEP == 0 && !a.b_sin && (!two || a.P1 % TD_STEP == 0) &&
                     (a.K1 >= a.K || a.K1 % 128 == 0);
    ProfScope prof(dma ? "gemm_tn_bf16d" : wide ? "gemm_tn_bf16w" : "gemm_tn_bf16", s, 2.0 * a.P * a.N * a.K,
                   2.0 * (double)a.P * (a.N + a.K) + 4.0 * splits * (double)a.N * a.K);
    if (wide) {
        const int nb = cdiv(a.N, TW) * cdiv(a.K, TW);
        if (dma)  // B staged as is
        {
            a.bias_split = g_tn16_bias_split;
            const int blocks = nb * splits;
            launch_tn_bf16d(&a, 1, &blocks, (a.dbg & 4) ? 2 : (a.dbg & 2) ? 1 : g_tn16_ip, s);
        }
        else
            hipLaunchKernelGGL(k_gemm_tn_bf16w, dim3(nb * splits), dim3(512), 0, s, a);
    } else {
        const int nb = cdiv(a.N, HB) * cdiv(a.K, HB);
        hipLaunchKernelGGL(k_gemm_tn_bf16, dim3(nb * splits), dim3(256), 0, s, a);
    }
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

}  // namespace spn
