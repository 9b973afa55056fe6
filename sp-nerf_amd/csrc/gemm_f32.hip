// fp32 MFMA GEMMs for the SIREN MLP on gfx950 (v_mfma_f32_32x32x2_f32: exact f32 fmaf
// chains at the 157 TF/s f32 matrix rate, MI355X_MICROARCH.md "Matrix cores").
//
//  * k_gemm_nt  C[M,N] = epi( A[M,K] · B[N,K]^T )   forward layers (B = torch weight, K-contig)
//                                                    and backward dX (B = pre-transposed weight)
//  * k_gemm_tn  slab[s][N,K] = Σ_{p in split s} A[p,N]^T · B[p,K]   weight gradients, split over
//                                                    the point dimension, partial slabs reduced in
//                                                    a fixed order (deterministic) by k_reduce_slabs
//
// Tiles: 128x128 per 256-thread workgroup, 4 waves each owning 64x64 = 2x2 MFMA 32x32 tiles,
// BK = 32 staged through LDS with a register prefetch of the next K-step.  K is walked in
// groups of 8 with lane-half h handling k = 8g+4h+s at MFMA step s: that permutation lets a
// lane fetch its 4 operands of 4 consecutive MFMAs with one ds_read_b128 (the sum over k is
// order-free up to rounding).  LDS rows padded to 36 floats → conflict-free b128 reads.
#include "common.h"
#include "gemm_f32.h"

namespace spn {

constexpr int BM = 128, BN = 128, BK = 32;

// NT main loop variants: KS = K-step depth (32 or 64), ST = LDS stages (1: register prefetch,
// two barriers per K-step; 2: double-buffered LDS, one barrier per K-step).
template <int KS, int ST>
__global__ __launch_bounds__(256) void k_gemm_nt(NTArgs g) {
    constexpr int LK = KS + 4;                    // padded LDS row (floats): conflict-free b128 reads
    constexpr int NLD = KS / 8;                   // float4 loads per thread per operand per K-step
    __shared__ __attribute__((aligned(16))) float smem[ST * 2 * BM * LK];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nN = (g.N + BN - 1) / BN;
    const int t = xcd_remap(blockIdx.x, gridDim.x);
    const int bm = (t / nN) * BM, bn = (t % nN) * BN;
    const int lr = tid / (KS / 4), lk = (tid % (KS / 4)) * 4;
    constexpr int RSTEP = 256 / (KS / 4);         // rows covered by one pass of the block

    // Unconditional loads (a branch around a load makes hipcc drain vmcnt(0) in the K-loop):
    // rows past M / columns past N read a clamped row; they only feed outputs never stored.
    // K and K1 are multiples of KS, so the A / A2 segment is uniform per K-step.
    const int lda1 = g.lda, lda2 = g.lda2, K1 = g.K1;
    f32x4 ra[NLD], rb[NLD];
    auto gload = [&](int k0) {
        const bool seg2 = k0 >= K1;
        const float* pa = seg2 ? g.A2 + (k0 - K1) + lk : g.A + k0 + lk;
        const int lda = seg2 ? lda2 : lda1;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int row = min(bm + lr + RSTEP * i, g.M - 1);
            ra[i] = ld4(pa + (int64_t)row * lda);
            const int col = min(bn + lr + RSTEP * i, g.N - 1);
            rb[i] = ld4(g.B + (int64_t)col * g.ldb + k0 + lk);
        }
    };
    auto sstore = [&](int stg) {
        float* sA = smem + stg * 2 * BM * LK;
        float* sB = sA + BM * LK;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            *reinterpret_cast<f32x4*>(sA + (lr + RSTEP * i) * LK + lk) = ra[i];
            *reinterpret_cast<f32x4*>(sB + (lr + RSTEP * i) * LK + lk) = rb[i];
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
        const float* sA = smem + stg * 2 * BM * LK;
        const float* pa0 = sA + (wr * 64 + r32) * LK + 4 * h;
        const float* pa1 = pa0 + 32 * LK;
        const float* pb0 = sA + BM * LK + (wc * 64 + r32) * LK + 4 * h;
        const float* pb1 = pb0 + 32 * LK;
#pragma unroll
        for (int kg = 0; kg < KS / 8; ++kg) {
            const f32x4 a0 = ld4(pa0 + kg * 8), a1 = ld4(pa1 + kg * 8);
            const f32x4 b0 = ld4(pb0 + kg * 8), b1 = ld4(pb1 + kg * 8);
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b0[s], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b1[s], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b0[s], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b1[s], acc[1][1], 0, 0, 0);
            }
        }
    };

    const int nk = g.K / KS;
    gload(0);
    if (ST == 1) {
        for (int kt = 0; kt < nk; ++kt) {
            __syncthreads();
            sstore(0);
            __syncthreads();
            if (kt + 1 < nk) gload((kt + 1) * KS);
            compute(0);
        }
    } else {
        // past the last step the loader re-reads it (L2 hit, never computed on): no branch
        sstore(0);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            gload(min(kt + 1, nk - 1) * KS);
            __builtin_amdgcn_sched_barrier(0);  // issue the loads before the MFMAs
            compute(kt & 1);
            __builtin_amdgcn_sched_barrier(0);  // LDS writes (and their vmcnt waits) after them
            sstore((kt + 1) & 1);
            __syncthreads();
        }
    }

    const int row0 = bm + wr * 64 + 4 * h;  // + i*32 + (r&3) + 8(r>>2)
    if (g.act == 0 || bn + BN <= g.n_lin) {
        // Linear epilogue (backward dX, feature layer): applied in the accumulator layout —
        // for a fixed register r the 32 lanes of a half-wave touch 32 consecutive columns of one
        // row, so every Dmul / rowbias / C access is a 128-B segment and, fully unrolled, all
        // loads of the tile are in flight together.
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = bn + wc * 64 + j * 32 + r32;
            if (col >= g.N) continue;
            const float bias = g.bias ? g.bias[col] : 0.f;
            const float r1v = g.r1_a ? g.r1_v[col] : 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float dm[16], rbv[16], r1[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row0 + i * 32 + (r & 3) + 8 * (r >> 2);
                    const bool ok = row < g.M;
                    dm[r] = (g.Dmul && ok) ? g.Dmul[(int64_t)row * g.ld_dmul + col] : 1.f;
                    rbv[r] = (g.rowbias && ok) ? g.rowbias[(int64_t)(row / g.rows_per_ray) * g.ld_rb + col] : 0.f;
                    r1[r] = (g.r1_a && ok) ? g.r1_a[(int64_t)row * g.r1_lda] : 0.f;
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row0 + i * 32 + (r & 3) + 8 * (r >> 2);
                    if (row >= g.M) continue;
                    float v = acc[i][j][r] + bias;
                    v += rbv[r];
                    if (g.r1_a) v += r1[r] * r1v;
                    g.C[(int64_t)row * g.ldc + col] = g.Dmul ? v * dm[r] : v;
                }
            }
        }
        return;
    }
    if (g.C16) {
        // bf16 outputs (layer 0 of the bf16 MLP, sine epilogue only): as k_gemm_nt_bf16 — a
        // wave stages 32 x 64 of its tile at a time, a lane owns 8 consecutive columns of rows
        // (lane >> 3) + 8 q4, so every store is a full 128-B row segment; hardware sin/cos
        // after range reduction (|w0 v| ~ 1e2 → ~1e-5 absolute, below bf16 rounding).
        __syncthreads();  // every wave is done with the K-loop's LDS stages
        constexpr int SLD = 68;
        float* st = smem + wid * (32 * SLD);
        const int cq = (lane & 7) * 8;
        const int col = bn + wc * 64 + cq;
        const bool colok = col < g.N;
        const int colc = colok ? col : g.N - 8;
        float bias8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) bias8[e] = g.bias ? g.bias[colc + e] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            wave_lds_sync();
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) st[((r & 3) + 8 * (r >> 2) + 4 * h) * SLD + j * 32 + r32] = acc[i][j][r];
            wave_lds_sync();
            u32x4 oc[4], od[4];
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int rr = (lane >> 3) + 8 * q4;
                const int row = bm + wr * 64 + i * 32 + rr;
                float v[8], d[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = st[rr * SLD + cq + e] + bias8[e];
                if (g.rowbias) {
                    const float* rb = g.rowbias + (int64_t)(min(row, g.M - 1) / g.rows_per_ray) * g.ld_rb + colc;
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] += rb[e];
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    float sn, cs;
                    fast_sincos(g.w0 * v[e], &sn, &cs);
                    v[e] = sn;
                    d[e] = g.w0 * cs;
                }
                oc[q4] = pack8(v);
                od[q4] = pack8(d);
            }
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int row = bm + wr * 64 + i * 32 + (lane >> 3) + 8 * q4;
                if (row < g.M && colok) {
                    *reinterpret_cast<u32x4*>(g.C16 + (int64_t)row * g.ldc + col) = oc[q4];
                    if (g.D16) *reinterpret_cast<u32x4*>(g.D16 + (int64_t)row * g.ld_dout + col) = od[q4];
                }
            }
        }
        return;
    }
    // Sine epilogue: each wave stages one 32x32 accumulator tile at a time in LDS and walks it
    // back row-major, so global accesses are 128-B row segments and sincos is not unrolled 64x.
    float* stage = smem + wid * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < 16; ++r) stage[((r & 3) + 8 * (r >> 2) + 4 * h) * 32 + r32] = acc[i][j][r];
            __syncthreads();
            const int col = bn + wc * 64 + j * 32 + r32;
            if (col >= g.N) continue;
            const float bias = g.bias ? g.bias[col] : 0.f;
            const bool sine = g.act == 1 && col >= g.n_lin;
            const float r1v = g.r1_a ? g.r1_v[col] : 0.f;
#pragma unroll 4
            for (int e = 0; e < 16; ++e) {
                const int rr = 2 * e + h;
                const int row = bm + wr * 64 + i * 32 + rr;
                if (row >= g.M) continue;
                float v = stage[rr * 32 + r32] + bias;
                if (g.rowbias) v += g.rowbias[(int64_t)(row / g.rows_per_ray) * g.ld_rb + col];
                if (g.r1_a) v += g.r1_a[(int64_t)row * g.r1_lda] * r1v;
                float y = v, dv = 1.f;
                if (sine) {
                    const float a = g.w0 * v;
                    float sn, cs;
                    sincosf(a, &sn, &cs);
                    y = sn;
                    dv = g.w0 * cs;
                }
                if (g.Dmul) y *= g.Dmul[(int64_t)row * g.ld_dmul + col];
                if (g.C16) {
                    if (g.D16 && sine) g.D16[(int64_t)row * g.ld_dout + col] = (bf16)dv;
                    g.C16[(int64_t)row * g.ldc + col] = (bf16)y;
                } else {
                    if (g.Dout && sine) g.Dout[(int64_t)row * g.ld_dout + col] = dv;
                    g.C[(int64_t)row * g.ldc + col] = y;
                }
            }
        }
    }
}

// Wide NT tile: BM x BN per block, WGM x WGN waves each owning (BM/WGM) x (BN/WGN) = MI x NJ
// 32x32 MFMA tiles; K-step 32, double-buffered LDS (rows padded to 36 floats), persistent over
// tiles (one block per CU at 256 x 256: 147 KB of LDS), the next tile's first K-step loading
// during the epilogue.  Same k permutation as k_gemm_nt (lane half h takes k = 8g + 4h + s at
// MFMA step s), so the accumulation order — and every output bit — equals k_gemm_nt's.
// Epilogue: a wave stages 32 rows x 64 columns at a time in its own LDS slice; a lane owns 8
// consecutive columns of rows (lane >> 3) + 8 q4, so every access is a 256-B (fp32) or 128-B
// (bf16) row segment; all global loads of a piece are issued before its stores.
// PIPE 1 (P2): operand loads run two K-steps ahead in two register sets, and step k+1's LDS
// stores sit between the two halves of step k's MFMAs instead of before the barrier (loads one
// step ahead would make those stores wait on HBM mid-step).
// PIPE 2: LDS-DMA (global_load_lds_dwordx4) into three unpadded stages, two K-steps in flight,
// one counted vmcnt + raw barrier per step and no register staging; 128-B rows with 16-B chunks
// XOR-swizzled by (row >> 1) & 7 (the DMA writes lane-linearly, so the swizzle goes on the
// source address) keep the fragment ds_read_b128s conflict-free.
// PIPE 3: PIPE 2 with K-steps of 16 (64-B rows, chunks swizzled by (row >> 2) & 3) for 4-wave
// blocks, two per CU (72 KB of LDS each): one block's epilogue overlaps the other's MFMAs.
template <int BM, int BN, int WGM, int WGN, int PIPE = 0>
__global__ __launch_bounds__(64 * WGM * WGN) __attribute__((amdgpu_waves_per_eu(2))) void k_gemm_nt_w(NTArgs g,
                                                                                                    int ntiles) {
    constexpr bool P2 = PIPE == 1;
    constexpr bool DMA = PIPE >= 2;
    constexpr int T = 64 * WGM * WGN;
    constexpr int MI = BM / WGM / 32, NJ = BN / WGN / 32;
    constexpr int KS = PIPE == 3 ? 16 : 32, LK = KS + 4;
    constexpr int CH = KS / 4, SH = KS == 32 ? 1 : 2;  // 16-B chunks per DMA row, swizzle row shift
    constexpr int RP = T / 8;                  // rows per loader pass (8 float4 chunks per row)
    constexpr int PA = BM / RP, PB = BN / RP;  // loader passes per operand
    static_assert(BM % RP == 0 && BN % RP == 0 && NJ % 2 == 0, "tile geometry");
    constexpr int STGF = (BM + BN) * KS;       // floats per DMA stage (PIPE 2)
    constexpr int SMEM = DMA ? 3 * STGF : 2 * (BM + BN) * LK;
    __shared__ __attribute__((aligned(16))) float smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nN = (g.N + BN - 1) / BN;
    const int G = gridDim.x;
    const int lr = tid >> 3, lk = (tid & 7) * 4;
    int t = xcd_remap(blockIdx.x, G);
    if (t >= ntiles) return;  // block-uniform

    // unconditional loads from clamped rows (see k_gemm_nt); K, K1 are multiples of KS
    const int lda1 = g.lda, lda2 = g.lda2, K1 = g.K1;
    struct Regs {
        f32x4 a[PA], b[PB];
    };
    auto gload = [&](Regs& r, int tile, int k0) {
        const int bm = (tile / nN) * BM, bn = (tile % nN) * BN;
        const bool seg2 = k0 >= K1;
        const float* pa = seg2 ? g.A2 + (k0 - K1) + lk : g.A + k0 + lk;
        const int lda = seg2 ? lda2 : lda1;
#pragma unroll
        for (int i = 0; i < PA; ++i) r.a[i] = ld4(pa + (int64_t)min(bm + lr + RP * i, g.M - 1) * lda);
#pragma unroll
        for (int i = 0; i < PB; ++i) r.b[i] = ld4(g.B + (int64_t)min(bn + lr + RP * i, g.N - 1) * g.ldb + k0 + lk);
    };
    auto sstore = [&](const Regs& r, int stg) {
        float* sA = smem + stg * (BM + BN) * LK;
        float* sB = sA + BM * LK;
#pragma unroll
        for (int i = 0; i < PA; ++i) *reinterpret_cast<f32x4*>(sA + (lr + RP * i) * LK + lk) = r.a[i];
#pragma unroll
        for (int i = 0; i < PB; ++i) *reinterpret_cast<f32x4*>(sB + (lr + RP * i) * LK + lk) = r.b[i];
    };

    f32x16 acc[MI][NJ];
    const int wr = wid / WGN, wc = wid % WGN, r32 = lane & 31, h = lane >> 5;
    // k-groups [lo, hi) of a K-step (8 k each)
    auto compute_kg = [&](int stg, auto klo, auto khi) {
        constexpr int lo = decltype(klo)::value, hi = decltype(khi)::value;
        const float* sA = smem + stg * (BM + BN) * LK + (wr * MI * 32 + r32) * LK + 4 * h;
        const float* sB = smem + stg * (BM + BN) * LK + BM * LK + (wc * NJ * 32 + r32) * LK + 4 * h;
#pragma unroll
        for (int kg = lo; kg < hi; ++kg) {
            f32x4 a[MI], b[NJ];
#pragma unroll
            for (int i = 0; i < MI; ++i) a[i] = ld4(sA + i * 32 * LK + kg * 8);
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = ld4(sB + j * 32 * LK + kg * 8);
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
        }
    };
    auto compute = [&](int stg) {
        compute_kg(stg, std::integral_constant<int, 0>{}, std::integral_constant<int, KS / 8>{});
    };
    // PIPE 2: one K-step from DMA stage s (rows of 32 floats, chunk c of row r at c ^ ((r>>1)&7))
    const int swz = (r32 >> SH) & (CH - 1);
    // fragments double-buffered across k-groups: group kg+1's ds_reads are issued ahead of group
    // kg's MFMAs (with one set, every group started with an exposed LDS latency)
    auto compute_g = [&](int s) {
        const float* sA = smem + s * STGF + (wr * MI * 32 + r32) * KS;
        const float* sB = smem + s * STGF + (BM + wc * NJ * 32 + r32) * KS;
        f32x4 a[2][MI], b[2][NJ];
        auto frag = [&](int kg, f32x4* fa, f32x4* fb) {
            const int off = ((2 * kg + h) ^ swz) * 4;
#pragma unroll
            for (int i = 0; i < MI; ++i) fa[i] = ld4(sA + i * 32 * KS + off);
#pragma unroll
            for (int j = 0; j < NJ; ++j) fb[j] = ld4(sB + j * 32 * KS + off);
        };
        frag(0, a[0], b[0]);
#pragma unroll
        for (int kg = 0; kg < KS / 8; ++kg) {
            const int cur = kg & 1;
            if (kg + 1 < KS / 8) frag(kg + 1, a[cur ^ 1], b[cur ^ 1]);
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] =
                            __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][i][s4], b[cur][j][s4], acc[i][j], 0, 0, 0);
        }
    };
    // PIPE 2: DMA K-step k0 of a tile into stage s; wave w's i-th instruction fills rows
    // 8q .. 8q+7 (q = i·(T/64) + w), lane l row 8q + l/8, LDS chunk l%8
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    auto gissue = [&](int tile, int k0, int s) {
        const int bm = (tile / nN) * BM, bn = (tile % nN) * BN;
        const bool seg2 = k0 >= K1;
        const float* pa = seg2 ? g.A2 + (k0 - K1) : g.A + k0;
        const int lda = seg2 ? lda2 : lda1;
        constexpr int NI = (BM + BN) * CH / T;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int q = i * (T / 64) + wid;
            const int row = q * (64 / CH) + lane / CH;
            const int gc = ((lane % CH) ^ ((row >> SH) & (CH - 1))) * 4;
            const float* src = i < BM * CH / T ? pa + (int64_t)min(bm + row, g.M - 1) * lda + gc
                                              : g.B + (int64_t)min(bn + row - BM, g.N - 1) * g.ldb + k0 + gc;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(smem + s * STGF + q * 256), 16, 0, 0);
        }
    };

    constexpr int SLD = 68;
    static_assert(WGM * WGN * 32 * SLD <= SMEM, "epilogue staging fits in the LDS");
    // PIPE 2 stages the epilogue at the top of the LDS, clear of DMA stage 0
    static_assert(!DMA || WGM * WGN * 32 * SLD <= SMEM - STGF, "epilogue staging clear of stage 0");
    float* stage = smem + (DMA ? SMEM - WGM * WGN * 32 * SLD : 0) + wid * (32 * SLD);
    const int nk = g.K / KS;
    const bool out16 = g.C16 != nullptr;

    Regs r0, r1;
    if constexpr (DMA) {
        gissue(t, 0, 0);
        gissue(t, min(1, nk - 1) * KS, 1);
    } else {
        gload(r0, t, 0);
        sstore(r0, 0);
        if constexpr (P2) gload(r1, t, min(1, nk - 1) * KS);
        __syncthreads();
    }
    // P2 step kt: stage kt & 1 holds step kt, rn holds step kt+1, rl receives step kt+2
    auto step2 = [&](int kt, Regs& rn, Regs& rl) {
        gload(rl, t, min(kt + 2, nk - 1) * KS);
        __builtin_amdgcn_sched_barrier(0);
        compute_kg(kt & 1, std::integral_constant<int, 0>{}, std::integral_constant<int, KS / 16>{});
        __builtin_amdgcn_sched_barrier(0);
        sstore(rn, (kt + 1) & 1);  // stage (kt+1) & 1 was last read in step kt-1 (before the barrier)
        __builtin_amdgcn_sched_barrier(0);
        compute_kg(kt & 1, std::integral_constant<int, KS / 16>{}, std::integral_constant<int, KS / 8>{});
        __syncthreads();
    };
    while (true) {
        const int bm = (t / nN) * BM, bn = (t % nN) * BN;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        if constexpr (DMA) {
            constexpr int NI = (BM + BN) * CH / T;  // DMA instructions per thread per K-step
            static_assert(NI == 6, "vmcnt below counts 6 DMAs per K-step");
            for (int kt = 0; kt < nk; ++kt) {
                // step kt has landed when at most step kt+1's DMAs are outstanding; the barrier
                // makes every wave's DMA visible and retires step kt-1's readers of stage (kt+2)%3
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                gissue(t, min(kt + 2, nk - 1) * KS, (kt + 2) % 3);  // past the end: re-reads, unused
                compute_g(kt % 3);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land in the staging area
            __builtin_amdgcn_s_barrier();
        } else if constexpr (P2) {
            // whole pairs (a conditional second step makes the register sets merge at the
            // back edge, with a wait on the in-flight loads), then an odd last step
            int kt = 0;
            for (; kt + 1 < nk; kt += 2) {
                step2(kt, r1, r0);
                step2(kt + 1, r0, r1);
            }
            if (kt < nk) step2(kt, r1, r0);  // block-uniform
        } else {
            for (int kt = 0; kt < nk; ++kt) {
                gload(r0, t, min(kt + 1, nk - 1) * KS);  // past the last step: re-read it (L2 hit)
                __builtin_amdgcn_sched_barrier(0);         // issue the loads before the MFMAs
                compute(kt & 1);
                __builtin_amdgcn_sched_barrier(0);         // LDS writes (and their vmcnt waits) after
                sstore(r0, (kt + 1) & 1);
                __syncthreads();
            }
        }
        const int tn = t + G;
        const bool more = tn < ntiles;
        if constexpr (!DMA) gload(r0, more ? tn : t, 0);  // the next tile's first K-step loads during the epilogue

        // epilogue lane geometry from an opaque lane id (recomputed per tile, not held live
        // across the main loop)
        const int el = opaque(lane), cq = (el & 7) * 8, er32 = el & 31, eh = el >> 5, erow = el >> 3;
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
                const int rbase = bm + wr * MI * 32 + i * 32 + erow;
                f32x4 dm[4][2];
                float r1a[4];
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int row = min(rbase + 8 * q4, g.M - 1);
                    if (g.Dmul) {
                        dm[q4][0] = ld4(g.Dmul + (int64_t)row * g.ld_dmul + colc);
                        dm[q4][1] = ld4(g.Dmul + (int64_t)row * g.ld_dmul + colc + 4);
                    }
                    r1a[q4] = g.r1_a ? g.r1_a[(int64_t)row * g.r1_lda] : 0.f;
                }
                wave_lds_sync();
#pragma unroll
                for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        stage[((r & 3) + 8 * (r >> 2) + 4 * eh) * SLD + j2 * 32 + er32] = acc[i][2 * jp + j2][r];
                wave_lds_sync();
                const bool sine_cols = g.act == 1 && col >= g.n_lin;  // n_lin is a multiple of 8
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const int rr = erow + 8 * q4;
                    const int row = rbase + 8 * q4;
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
                            if (out16) {
                                fast_sincos(g.w0 * v[e], &sn, &cs);
                            } else {
                                sincosf(g.w0 * v[e], &sn, &cs);
                            }
                            v[e] = sn;
                            d[e] = g.w0 * cs;
                        }
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) d[e] = 1.f;
                    }
                    if (g.Dmul) {
#pragma unroll
                        for (int e = 0; e < 8; ++e) v[e] *= dm[q4][e >> 2][e & 3];
                    }
                    if (g.emu && (g.Dmul ? (g.emu & 2) : (g.emu & 1))) {  // precision study: bf16 rounding
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            v[e] = (float)(bf16)v[e];
                            d[e] = (float)(bf16)d[e];
                        }
                    }
                    if (row < g.M && colok) {
                        if (out16) {
                            *reinterpret_cast<u32x4*>(g.C16 + (int64_t)row * g.ldc + col) = pack8(v);
                            if (g.D16) *reinterpret_cast<u32x4*>(g.D16 + (int64_t)row * g.ld_dout + col) = pack8(d);
                        } else {
                            float* pc = g.C + (int64_t)row * g.ldc + col;
                            st4(pc, f32x4{v[0], v[1], v[2], v[3]});
                            st4(pc + 4, f32x4{v[4], v[5], v[6], v[7]});
                            if (g.Dout && sine_cols) {
                                float* pd = g.Dout + (int64_t)row * g.ld_dout + col;
                                st4(pd, f32x4{d[0], d[1], d[2], d[3]});
                                st4(pd + 4, f32x4{d[4], d[5], d[6], d[7]});
                            }
                        }
                    }
                }
            }
        }
        if (!more) break;  // block-uniform
        __syncthreads();   // every wave is done with its staging slice
        if constexpr (DMA) {
            gissue(tn, 0, 0);
            gissue(tn, min(1, nk - 1) * KS, 1);
        } else {
            sstore(r0, 0);
            if constexpr (P2) gload(r1, tn, min(1, nk - 1) * KS);
            __syncthreads();
        }
        t = tn;
    }
}

// ST = LDS stages (1 or 2); ST = 3: two stages with the operand loads two steps ahead in two
// register sets and the next stage's stores between the halves of the step's MFMAs (as
// k_gemm_nt_w's PIPE 1).
template <int ST>
__global__ __launch_bounds__(256) void k_gemm_tn(TNArgs g) {
    constexpr int LDN = 128;
    constexpr int NSTG = ST == 1 ? 1 : 2;
    __shared__ __attribute__((aligned(16))) float smem[NSTG * 2 * BK * LDN];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // 1-D grid, split-major after the XCD remap: the tiles of one split share one XCD's L2
    // (see k_gemm_tn_bf16)
    const int nK = (g.K + 127) / 128;
    const int ntiles = cdiv(g.N, 128) * nK;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * 128, k0 = (t % nK) * 128;
    const int p_beg = split * g.p_per_split;
    const int p_end = min(g.P, p_beg + g.p_per_split);
    const int lr = tid >> 5, lc = (tid & 31) * 4;

    // Unconditional loads (see k_gemm_nt): features past N / K read a clamped column (outputs
    // never stored); points past the split are zeroed at the LDS write, after the MFMAs.
    struct Regs {
        f32x4 a[4], b[4];
        int p;
    };
    const int nc = min(n0 + lc, g.N - 4);
    const int kc = min(k0 + lc, g.K - 4);
    const float* pb = kc < g.K1 ? g.B + kc : g.B2 + (kc - g.K1);
    const int ldb = kc < g.K1 ? g.ldb : g.ldb2;
    const int lda = g.lda;
    auto gload_r = [&](Regs& r, int p0) {
        r.p = p0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pc = min(p0 + lr + 8 * i, p_end - 1);
            r.a[i] = ld4(g.A + (int64_t)pc * lda + nc);
            r.b[i] = ld4(pb + (int64_t)pc * ldb);
        }
    };
    auto sstore_r = [&](const Regs& r, int stg) {
        float* sA = smem + stg * 2 * BK * LDN;
        float* sB = sA + BK * LDN;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool pin = r.p + lr + 8 * i < p_end;
            *reinterpret_cast<f32x4*>(sA + (lr + 8 * i) * LDN + lc) = pin ? r.a[i] : z;
            *reinterpret_cast<f32x4*>(sB + (lr + 8 * i) * LDN + lc) = pin ? r.b[i] : z;
        }
    };
    Regs r0, r1;
    auto gload = [&](int p0) { gload_r(r0, p0); };
    auto sstore = [&](int stg) { sstore_r(r0, stg); };

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const bool do_bias = g.slab_b != nullptr && k0 == 0 && tid < 128;
    float bsum = 0.f;
    const int wr = wid >> 1, wc = wid & 1, r32 = lane & 31, h = lane >> 5;
    // k-groups [lo, hi) of a stage (8 points each); the bias column sums go with the first half
    auto compute_kg = [&](int stg, auto klo, auto khi) {
        constexpr int lo = decltype(klo)::value, hi = decltype(khi)::value;
        const float* sA = smem + stg * 2 * BK * LDN;
        const float* sB = sA + BK * LDN;
        if (lo == 0 && do_bias) {
#pragma unroll 8
            for (int q = 0; q < BK; ++q) bsum += sA[q * LDN + tid];
        }
#pragma unroll
        for (int kg = lo; kg < hi; ++kg) {
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int q = kg * 8 + 4 * h + s;
                const float a0 = sA[q * LDN + wr * 64 + r32], a1 = sA[q * LDN + wr * 64 + 32 + r32];
                const float b0 = sB[q * LDN + wc * 64 + r32], b1 = sB[q * LDN + wc * 64 + 32 + r32];
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
            }
        }
    };
    auto compute = [&](int stg) {
        compute_kg(stg, std::integral_constant<int, 0>{}, std::integral_constant<int, BK / 8>{});
    };

    if (ST == 3) {
        if (p_beg < p_end) {  // block-uniform
            // step p0: stage stg holds it, rn the next step, rl receives the one after
            gload_r(r0, p_beg);
            sstore_r(r0, 0);
            gload_r(r1, p_beg + BK);
            __syncthreads();
            int stg = 0;
            auto step2 = [&](int p0, Regs& rn, Regs& rl) {
                gload_r(rl, p0 + 2 * BK);  // past the split: clamped rows, zeroed at the store
                __builtin_amdgcn_sched_barrier(0);
                compute_kg(stg, std::integral_constant<int, 0>{}, std::integral_constant<int, BK / 16>{});
                __builtin_amdgcn_sched_barrier(0);
                sstore_r(rn, stg ^ 1);  // that stage was last read in the previous step
                __builtin_amdgcn_sched_barrier(0);
                compute_kg(stg, std::integral_constant<int, BK / 16>{}, std::integral_constant<int, BK / 8>{});
                __syncthreads();
                stg ^= 1;
            };
            int p0 = p_beg;
            for (; p0 + BK < p_end; p0 += 2 * BK) {
                step2(p0, r1, r0);
                step2(p0 + BK, r0, r1);
            }
            if (p0 < p_end) step2(p0, r1, r0);
        }
    } else if (ST == 1) {
        if (p_beg < p_end) gload(p_beg);
        for (int p0 = p_beg; p0 < p_end; p0 += BK) {
            __syncthreads();
            sstore(0);
            __syncthreads();
            if (p0 + BK < p_end) gload(p0 + BK);
            compute(0);
        }
    } else if (p_beg < p_end) {  // block-uniform
        gload(p_beg);
        sstore(0);
        __syncthreads();
        int stg = 0;
        for (int p0 = p_beg; p0 < p_end; p0 += BK) {
            gload(p0 + BK);  // unconditional: past the split the rows clamp and are zeroed
            __builtin_amdgcn_sched_barrier(0);
            compute(stg);
            __builtin_amdgcn_sched_barrier(0);
            sstore(stg ^ 1);
            __syncthreads();
            stg ^= 1;
        }
    }

    float* slab = g.slab + (int64_t)split * g.slab_stride;
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
    if (do_bias && n0 + tid < g.N) g.slab_b[(int64_t)split * g.N + n0 + tid] = bsum;
}

// dst[r][c] (+)= Σ_s slab[s][row0+r][c] for c < ncols; dst_b[r] = Σ_s slab_b[s][row0+r];
// with `transpose`, dst[c][r] instead.  256 threads = 64 columns x 4 split phases, the four
// phase partials combined in a fixed order (deterministic).
__device__ __forceinline__ void reduce_slab_row(const ReduceArgs& g, const int r, f32x4 (*part)[64]) {
    // a block: one row, 256 columns (float4 quads), the splits in 4 phases (waves); per column
    // the phases add their splits in order and combine as (p0 + p1) + (p2 + p3)
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int c = (blockIdx.x * 64 + tx) * 4;  // first column of this thread's quad
    const int n = g.row0 + r;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (c + 3 < g.ncols) {
        // 16 (then 4) splits' quads in flight per thread, the sums in split order either way (a
        // skinny reduction's 512-768 splits were 32 serial rounds of 4 loads: 15-30 us for a few MB)
        const float* src = g.slab + (int64_t)n * g.ld_slab + c;
        const int64_t st = g.slab_stride;
        int k = ty;
        for (; k + 60 < g.splits; k += 64) {
            f32x4 x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = ld4(src + (int64_t)(k + 4 * j) * st);
#pragma unroll
            for (int j = 0; j < 16; ++j) v += x[j];
        }
        for (; k + 12 < g.splits; k += 16) {
            const f32x4 x0 = ld4(src + k * st), x1 = ld4(src + (k + 4) * st), x2 = ld4(src + (k + 8) * st),
                        x3 = ld4(src + (k + 12) * st);
            v += x0;
            v += x1;
            v += x2;
            v += x3;
        }
        for (; k < g.splits; k += 4) v += ld4(src + k * st);
    } else if (c <= g.ncols) {  // the ragged last quad and the bias column
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int cc = c + e;
            float a = 0.f;
            if (cc < g.ncols) {
                const float* src = g.slab + (int64_t)n * g.ld_slab + cc;
#pragma unroll 8
                for (int k = ty; k < g.splits; k += 4) a += src[(int64_t)k * g.slab_stride];
            } else if (cc == g.ncols && g.dst_b) {
#pragma unroll 8
                for (int k = ty; k < g.splits; k += 4) a += g.slab_b[(int64_t)k * g.N + n];
            }
            v[e] = a;
        }
    }
    part[ty][tx] = v;
    __syncthreads();
    if (ty == 0 && c <= g.ncols) {
        const f32x4 s4 = (part[0][tx] + part[1][tx]) + (part[2][tx] + part[3][tx]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int cc = c + e;
            const float s = s4[e];
            if (cc < g.ncols) {
                float* d = g.transpose ? g.dst + (int64_t)cc * g.ld_dst + r : g.dst + (int64_t)r * g.ld_dst + cc;
                *d = g.accumulate ? *d + s : s;
            } else if (cc == g.ncols && g.dst_b) {
                g.dst_b[r] = g.accumulate ? g.dst_b[r] + s : s;
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_reduce_slabs(ReduceArgs g) {
    __shared__ f32x4 part[4][64];
    reduce_slab_row(g, blockIdx.y, part);
}

// several reductions in one launch (the outputs of one weight-gradient GEMM: rows of the
// concatenated heads, the skinny reductions' product and column-sum rows): grid.y runs over the
// segments' rows in order
__global__ __launch_bounds__(256) void k_reduce_slabs_multi(ReduceMulti m) {
    __shared__ f32x4 part[4][64];
    int r = blockIdx.y, i = 0;
    while (i + 1 < m.n && r >= m.seg[i].nrows) r -= m.seg[i++].nrows;
    reduce_slab_row(m.seg[i], r, part);
}

// Skinny weight gradient: slab[chunk][m][k] = Σ_{p in chunk} a_m(p) · B[p][k] for m < Ma
// (a_m(p) = A[p*lda + m], plus a_Ma(p) = 1 when `ones`, i.e. the column sums of B), and
// slab_b[chunk][m] = Σ_{p in chunk} a_m(p).  A thread owns one 16-B column group (4 fp32 or 8
// bf16 values of B) and walks the chunk's rows of its row phase four at a time, the four rows'
// loads issued before their arithmetic (the rows still add in increasing order); the row phases'
// partials are combined through LDS in phase order.
template <int MA, typename TB>
__device__ __forceinline__ void skinny_block(const SkinnyArgs& g, const TB* __restrict__ Bm, const int blk, float* red) {
    constexpr int V = sizeof(TB) == 2 ? 8 : 4;     // B values per 16-B load
    const int tid = threadIdx.x;
    const int kq = g.K / V;                        // column groups (kq <= 256, checked on host)
    const int rph = 256 / kq;                      // row phases
    const int c4 = tid % kq, ph = tid / kq;
    const bool live = ph < rph;
    const int64_t p0 = (int64_t)blk * g.chunk;
    const int64_t p1 = min(g.P, p0 + g.chunk);
    const int Mt = g.Ma + (g.ones ? 1 : 0);
    float acc[MA + 1][V];
    float asum[MA];
#pragma unroll
    for (int m = 0; m <= MA; ++m)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[m][e] = 0.f;
#pragma unroll
    for (int m = 0; m < MA; ++m) asum[m] = 0.f;
    auto load = [&](int64_t p, float (&bv)[V]) {
        if constexpr (V == 8) {
            unpack8(ldg16(reinterpret_cast<const bf16*>(Bm) + p * g.ldb + V * c4), bv);
        } else {
            const f32x4 x = ld4(reinterpret_cast<const float*>(Bm) + p * g.ldb + V * c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) bv[e] = x[e];
        }
    };
    auto add = [&](int64_t p, const float (&bv)[V], const float (&av)[MA]) {
#pragma unroll
        for (int m = 0; m < MA; ++m)
            if (m < g.Ma) {
#pragma unroll
                for (int e = 0; e < V; ++e) acc[m][e] += av[m] * bv[e];
                asum[m] += av[m];
            }
        if (g.ones) {
#pragma unroll
            for (int e = 0; e < V; ++e) acc[MA][e] += bv[e];
        }
    };
    auto loada = [&](int64_t p, float (&av)[MA]) {
        const float* ar = g.A + p * g.lda;
#pragma unroll
        for (int m = 0; m < MA; ++m) av[m] = m < g.Ma ? ar[m] : 0.f;
    };
    if (live) {
        int64_t p = p0 + ph;
        for (; p + 3 * rph < p1; p += 4 * rph) {
            float b0[V], b1[V], b2[V], b3[V], a0[MA], a1[MA], a2[MA], a3[MA];
            load(p, b0); load(p + rph, b1); load(p + 2 * rph, b2); load(p + 3 * rph, b3);
            loada(p, a0); loada(p + rph, a1); loada(p + 2 * rph, a2); loada(p + 3 * rph, a3);
            add(p, b0, a0); add(p + rph, b1, a1); add(p + 2 * rph, b2, a2); add(p + 3 * rph, b3, a3);
        }
        for (; p < p1; p += rph) {
            float b0[V], a0[MA];
            load(p, b0);
            loada(p, a0);
            add(p, b0, a0);
        }
    }
    // combine the row phases (every thread reaches every barrier)
    for (int m = 0; m < Mt; ++m) {
        const int q = m == g.Ma ? MA : m;
        float v[V];
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] = 0.f;
#pragma unroll
        for (int qq = 0; qq <= MA; ++qq)
            if (qq == q)
#pragma unroll
                for (int e = 0; e < V; ++e) v[e] = acc[qq][e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < V; ++e) red[V * tid + e] = v[e];
        __syncthreads();
        if (ph == 0) {
#pragma unroll
            for (int e = 0; e < V; ++e) {
                float sum = v[e];
                for (int r = 1; r < rph; ++r) sum += red[V * (r * kq + c4) + e];
                g.slab[((int64_t)blk * Mt + m) * g.K + V * c4 + e] = sum;
            }
        }
    }
    if (g.slab_b) {
        for (int m = 0; m < g.Ma; ++m) {
            float v = 0.f;
#pragma unroll
            for (int q = 0; q < MA; ++q)
                if (q == m) v = asum[q];
            __syncthreads();
            red[tid] = v;
            __syncthreads();
            if (tid == 0) {
                float sum = 0.f;
                for (int q = 0; q < rph; ++q) sum += red[q * kq];
                g.slab_b[(int64_t)blk * g.Ma + m] = sum;
            }
        }
    }
}

template <int MA, typename TB>
__global__ __launch_bounds__(256) void k_tn_skinny(SkinnyArgs g, const TB* __restrict__ Bm) {
    __shared__ float red[256 * (sizeof(TB) == 2 ? 8 : 4)];
    skinny_block<MA, TB>(g, Bm, blockIdx.x, red);
}

// several skinny reductions in one launch (the per-ray parameter gradients of a backward, the
// narrow heads' weight gradients): blockIdx.y = task, blockIdx.x = chunk (tasks with fewer
// chunks leave the rest idle); every task's B rows of type TB
template <int MA, typename TB>
__global__ __launch_bounds__(256) void k_tn_skinny_multi(SkinnyMulti m) {
    __shared__ float red[256 * (sizeof(TB) == 2 ? 8 : 4)];
    const SkinnyArgs& g = m.t[blockIdx.y];
    if ((int64_t)blockIdx.x * g.chunk >= g.P) return;   // whole block: before any barrier
    if constexpr (sizeof(TB) == 2) skinny_block<MA, bf16>(g, g.B16, blockIdx.x, red);
    else skinny_block<MA, float>(g, g.B, blockIdx.x, red);
}

// 8: 256x128 tiles on 4-wave blocks, two per CU, LDS-DMA K-steps of 16 (k_gemm_nt_w<.., 2, 2, 3>);
// 7: the same DMA pipeline on one 8-wave block per CU; 6: register loads 2 K-steps ahead; 5: 1
// step ahead.  C2: 10.30 (5) -> 10.17 (6) -> 10.04 (7, + reduce) -> 9.89 ms/step (8); s_setprio(1)
// around the MFMA groups measured 0.5% slower.
int g_nt_variant = 8;

int g_emu_bf16 = 0;

int32_t gemm_nt(const NTArgs& a0, hipStream_t s, int variant) {
    NTArgs a = a0;
    a.emu = (a.C16 || g_nt_variant != 8) ? 0 : (g_emu_bf16 & 3);   // the study covers the default kernel
    SPN_ARG(a.M >= 0 && a.N > 0 && a.K > 0, "gemm_nt: bad shape M=%d N=%d K=%d", a.M, a.N, a.K);
    SPN_ARG(a.K % BK == 0 && a.K1 % BK == 0 && a.K1 <= a.K, "gemm_nt: K=%d/K1=%d must be multiples of %d", a.K, a.K1, BK);
    SPN_ARG(a.K1 == a.K || a.A2 != nullptr, "gemm_nt: second A segment missing");
    SPN_ARG(a.lda % 4 == 0 && a.ldb % 4 == 0 && (a.K1 == a.K || a.lda2 % 4 == 0), "gemm_nt: leading dims must be /4");
    SPN_ARG(a.rowbias == nullptr || a.rows_per_ray > 0, "gemm_nt: rows_per_ray");
    SPN_ARG(a.C16 == nullptr || (a.act == 1 && a.n_lin == 0 && a.Dmul == nullptr && a.r1_a == nullptr && a.N % 8 == 0 &&
                                 a.ldc % 8 == 0 && a.ld_dout % 8 == 0),
            "gemm_nt: bf16 output needs the sine epilogue and 8-aligned N / ldc / ld_dout");
    if (a.M == 0) return SPNERF_OK;
    const int nb = cdiv(a.M, BM) * cdiv(a.N, BN);
    ProfScope prof("gemm_nt_f32", s, 2.0 * a.M * a.N * a.K, 4.0 * ((double)a.M * a.K + (double)a.N * a.K + 2.0 * a.M * a.N));
    int v = variant >= 0 ? variant : g_nt_variant;
    if (v >= 4) {  // wide persistent tiles: 8-column epilogue rows need 16-B aligned row segments
        const bool ok = a.N % 8 == 0 && a.n_lin % 8 == 0 && a.ldc % 4 == 0 && (!a.Dout || a.ld_dout % 4 == 0) &&
                        (!a.Dmul || a.ld_dmul % 4 == 0) && (!a.rowbias || a.ld_rb % 4 == 0);
        if (!ok) v = 2;
    }
    if (v >= 4 && v <= 8) {
        const int bm = 256, bn = v == 4 ? 256 : 128;
        const int nt = cdiv(a.M, bm) * cdiv(a.N, bn);
        if (v == 4) hipLaunchKernelGGL((k_gemm_nt_w<256, 256, 2, 4>), dim3(std::min(nt, num_cus())), dim3(512), 0, s, a, nt);
        else if (v == 6) hipLaunchKernelGGL((k_gemm_nt_w<256, 128, 4, 2, 1>), dim3(std::min(nt, num_cus())), dim3(512), 0, s, a, nt);
        else if (v == 7) hipLaunchKernelGGL((k_gemm_nt_w<256, 128, 4, 2, 2>), dim3(std::min(nt, num_cus())), dim3(512), 0, s, a, nt);
        else if (v == 8) hipLaunchKernelGGL((k_gemm_nt_w<256, 128, 2, 2, 3>), dim3(std::min(nt, 512)), dim3(256), 0, s, a, nt);
        else hipLaunchKernelGGL((k_gemm_nt_w<256, 128, 4, 2>), dim3(std::min(nt, num_cus())), dim3(512), 0, s, a, nt);
    } else if (v == 1 && a.K % 64 == 0 && a.K1 % 64 == 0) hipLaunchKernelGGL((k_gemm_nt<64, 1>), dim3(nb), dim3(256), 0, s, a);
    else if (v == 2) hipLaunchKernelGGL((k_gemm_nt<32, 2>), dim3(nb), dim3(256), 0, s, a);
    else if (v == 3 && a.K % 64 == 0 && a.K1 % 64 == 0) hipLaunchKernelGGL((k_gemm_nt<64, 2>), dim3(nb), dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_gemm_nt<32, 1>), dim3(nb), dim3(256), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

// rows per block of a skinny reduction: ≤ 768 chunks, multiples of 64 rows; from 2^16 rows on at
// least 256 (a block's combine and slab writes cost as much as 128 rows' loads: the 512-ray
// step's narrow-head reduction took twice the time per byte of the 4 096-ray one).  Any P' ≤ P
// has at most min(ceil(P / 64), 768) chunks (mlp_layout's slab bound).
int skinny_chunk(int64_t P) {
    int64_t c = (P + 767) / 768;
    c = (c + 63) / 64 * 64;
    if (P >= 65536 && c < 256) c = 256;
    return (int)(c < 64 ? 64 : c);
}

int32_t tn_skinny(const SkinnyArgs& a0, hipStream_t s) {
    SkinnyArgs a = a0;
    SPN_ARG(a.Ma >= 1 && a.Ma <= 8 && a.K % 4 == 0 && a.K <= 1024 && a.ldb % 4 == 0, "tn_skinny: bad shape Ma=%d K=%d",
            a.Ma, a.K);
    SPN_ARG(!a.B16 || (a.K % 8 == 0 && a.K <= 2048 && a.ldb % 8 == 0), "tn_skinny: bf16 rows need K, ldb multiples of 8");
    a.chunk = skinny_chunk(a.P);
    const int nb = cdiv(a.P, a.chunk);
    if (nb == 0) return SPNERF_OK;
    ProfScope prof("tn_skinny", s, 2.0 * a.P * a.K * (a.Ma + a.ones), 4.0 * a.P * (a.K + a.Ma));
    if (a.B16) {
        if (a.Ma <= 1) hipLaunchKernelGGL((k_tn_skinny<1, bf16>), dim3(nb), dim3(256), 0, s, a, a.B16);
        else if (a.Ma <= 3) hipLaunchKernelGGL((k_tn_skinny<3, bf16>), dim3(nb), dim3(256), 0, s, a, a.B16);
        else hipLaunchKernelGGL((k_tn_skinny<8, bf16>), dim3(nb), dim3(256), 0, s, a, a.B16);
    } else {
        if (a.Ma <= 1) hipLaunchKernelGGL((k_tn_skinny<1, float>), dim3(nb), dim3(256), 0, s, a, a.B);
        else if (a.Ma <= 3) hipLaunchKernelGGL((k_tn_skinny<3, float>), dim3(nb), dim3(256), 0, s, a, a.B);
        else hipLaunchKernelGGL((k_tn_skinny<8, float>), dim3(nb), dim3(256), 0, s, a, a.B);
    }
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int32_t tn_skinny_multi(const SkinnyArgs* a, int n, hipStream_t s) {
    SPN_ARG(n >= 0 && n <= kSkinnyMulti, "tn_skinny_multi: %d tasks", n);
    SkinnyMulti m;
    m.n = 0;
    int nb = 0, ma = 1;
    double fl = 0.0, by = 0.0;
    const bool b16 = n > 0 && a[0].B16;
    for (int i = 0; i < n; ++i) {
        SkinnyArgs t = a[i];
        SPN_ARG(t.Ma >= 1 && t.Ma <= 8 && (b16 ? (t.B16 && t.K % 8 == 0 && t.K <= 2048 && t.ldb % 8 == 0)
                                                : (!t.B16 && t.B && t.K % 4 == 0 && t.K <= 1024 && t.ldb % 4 == 0)),
                "tn_skinny_multi: bad task Ma=%d K=%d", t.Ma, t.K);
        if (t.P <= 0) continue;
        t.chunk = skinny_chunk(t.P);
        nb = std::max(nb, cdiv(t.P, t.chunk));
        ma = std::max(ma, t.Ma);
        fl += 2.0 * t.P * t.K * (t.Ma + t.ones);
        by += 4.0 * t.P * (t.K + t.Ma);
        m.t[m.n++] = t;
    }
    if (m.n == 0) return SPNERF_OK;
    ProfScope prof("tn_skinny", s, fl, by);
    if (b16) {
        if (ma <= 1) hipLaunchKernelGGL((k_tn_skinny_multi<1, bf16>), dim3(nb, m.n), dim3(256), 0, s, m);
        else if (ma <= 3) hipLaunchKernelGGL((k_tn_skinny_multi<3, bf16>), dim3(nb, m.n), dim3(256), 0, s, m);
        else hipLaunchKernelGGL((k_tn_skinny_multi<8, bf16>), dim3(nb, m.n), dim3(256), 0, s, m);
    } else if (ma <= 3) {
        hipLaunchKernelGGL((k_tn_skinny_multi<3, float>), dim3(nb, m.n), dim3(256), 0, s, m);
    } else {
        hipLaunchKernelGGL((k_tn_skinny_multi<8, float>), dim3(nb, m.n), dim3(256), 0, s, m);
    }
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int tn_splits(int P, int N, int K) {
    const int tiles = cdiv(N, 128) * cdiv(K, 128);
    // whole rounds of the 512 co-resident blocks: the skip layer's 20 tiles at cdiv(1024, 20) = 52
    // splits made 1 040 blocks, a third round of 16 (434 us against 297 for 1 024 blocks)
    int splits = 1024 / tiles;
    if (splits > 64) splits = 64;
    const int max_splits = cdiv(P, 256);
    if (splits > max_splits) splits = max_splits;
    return splits < 1 ? 1 : splits;
}

int g_tn_variant = 2;  // 2: k_gemm_tn<3> (loads two steps ahead; C2 9.89 -> 9.81 ms/step), 1: <2>, 0: <1>

int32_t gemm_tn(const TNArgs& a0, int splits, hipStream_t s, int variant) {
    TNArgs a = a0;
    SPN_ARG(a.N > 0 && a.K > 0 && a.P >= 0, "gemm_tn: bad shape");
    SPN_ARG(a.N % 4 == 0 && a.K % 4 == 0 && a.K1 % 4 == 0 && a.lda % 4 == 0 && a.ldb % 4 == 0, "gemm_tn: dims must be /4");
    SPN_ARG(a.K1 == a.K || a.B2 != nullptr, "gemm_tn: second B segment missing");
    int pps = cdiv(a.P, splits);
    pps = ((pps + BK - 1) / BK) * BK;
    a.p_per_split = pps < BK ? BK : pps;
    const int nb = cdiv(a.N, 128) * cdiv(a.K, 128);
    ProfScope prof("gemm_tn_f32", s, 2.0 * a.P * a.N * a.K, 4.0 * ((double)a.P * (a.N + a.K) + (double)splits * a.N * a.K));
    const int v = variant >= 0 ? variant : g_tn_variant;
    if (v == 2) hipLaunchKernelGGL(k_gemm_tn<3>, dim3(nb * splits), dim3(256), 0, s, a);
    else if (v == 1) hipLaunchKernelGGL(k_gemm_tn<2>, dim3(nb * splits), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_gemm_tn<1>, dim3(nb * splits), dim3(256), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int32_t reduce_slabs_multi(const ReduceArgs* a, int n, hipStream_t s) {
    ReduceMulti m;
    m.n = 0;
    int rows = 0, cols = 0;
    double bytes = 0.0;
    for (int i = 0; i < n; ++i) {
        if (a[i].nrows <= 0) continue;
        SPN_ARG(m.n < kReduceMulti, "reduce_slabs_multi: too many segments");
        m.seg[m.n++] = a[i];
        rows += a[i].nrows;
        cols = std::max(cols, a[i].ncols + 1);
        bytes += 4.0 * (double)a[i].nrows * (a[i].ncols + 1) * (a[i].splits + (a[i].accumulate ? 2.0 : 1.0));
    }
    if (m.n == 0) return SPNERF_OK;
    if (m.n == 1) return reduce_slabs(m.seg[0], s);
    ProfScope prof("reduce_slabs", s, 0.0, bytes);
    hipLaunchKernelGGL(k_reduce_slabs_multi, dim3(cdiv(cols, 256), rows), dim3(256), 0, s, m);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int32_t reduce_slabs(const ReduceArgs& a, hipStream_t s) {
    if (a.nrows <= 0) return SPNERF_OK;
    const int cols = a.ncols + 1;
    ProfScope prof("reduce_slabs", s, 0.0, 4.0 * (double)a.nrows * cols * (a.splits + (a.accumulate ? 2.0 : 1.0)));
    hipLaunchKernelGGL(k_reduce_slabs, dim3(cdiv(cols, 256), a.nrows), dim3(256), 0, s, a);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

}  // namespace spn
