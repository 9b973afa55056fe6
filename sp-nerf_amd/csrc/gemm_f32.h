// Launch descriptors of the fp32 MFMA GEMMs (gemm_f32.hip).
#pragma once
#include "common.h"

namespace spn {

// C[M,N] = epi(A[M,K] · B[N,K]^T).  A may be split along K into two sources: columns [0,K1)
// from A, [K1,K) from A2 (the skip-layer input [h | x0], spnerf.py:326-327).
struct NTArgs {
    const float* A = nullptr; int lda = 0;
    const float* A2 = nullptr; int lda2 = 0; int K1 = 0;
    const float* B = nullptr; int ldb = 0;
    float* C = nullptr; int ldc = 0;
    int M = 0, N = 0, K = 0;
    // epilogue, in order: + bias[col] + rowbias[row/rows_per_ray][col] + r1_a[row]*r1_v[col];
    // act==1 and col>=n_lin: y = sin(w0*v), Dout = w0*cos(w0*v); linear columns: y = v, Dout not
    // written (nothing reads a linear derivative); y *= Dmul
    const float* bias = nullptr;
    const float* rowbias = nullptr; int ld_rb = 0; int rows_per_ray = 1;
    const float* r1_a = nullptr; int r1_lda = 0; const float* r1_v = nullptr;
    int act = 0; float w0 = 1.f; int n_lin = 0;
    float* Dout = nullptr; int ld_dout = 0;
    const float* Dmul = nullptr; int ld_dmul = 0;
    // bf16 outputs instead of C / Dout (sine epilogue only: layer 0 of the bf16 MLP), same ld
    bf16* C16 = nullptr; bf16* D16 = nullptr;
    // precision study (option "emu_bf16", fp32 MLP only): 1 = outputs of forward layers (C, Dout)
    // rounded to bf16, 2 = the backward dX outputs (Dmul instances) rounded to bf16
    int emu = 0;
};
extern int g_emu_bf16;  // option "emu_bf16": bits 1 / 2 as NTArgs::emu, 4 = GEMM weights packed bf16-rounded

// slab[s][n][k] = Σ_{p in split s} A[p][n] · B[p][k]  (B split along K at K1 like NTArgs.A);
// slab_b[s][n] = Σ_{p in split s} A[p][n]  (bias gradient), if slab_b != nullptr.
struct TNArgs {
    const float* A = nullptr; int lda = 0;
    const float* B = nullptr; int ldb = 0;
    const float* B2 = nullptr; int ldb2 = 0; int K1 = 0;
    float* slab = nullptr; int ld_slab = 0; int64_t slab_stride = 0;
    float* slab_b = nullptr;
    int P = 0, N = 0, K = 0;
    int p_per_split = 0;  // set by gemm_tn
};

// Skinny reduction over points: slab[chunk][m][k] = Σ_p A[p*lda+m]·B[p*ldb+k] (m < Ma ≤ 8,
// plus m = Ma: Σ_p B[p][k] when `ones`), slab_b[chunk][m] = Σ_p A[p*lda+m].
struct SkinnyArgs {
    const float* A = nullptr; int lda = 0; int Ma = 0;
    const float* B = nullptr; int ldb = 0; int K = 0;
    const bf16* B16 = nullptr;  // bf16 B rows instead of B (same ldb)
    int64_t P = 0; int chunk = 0; int ones = 0;
    float* slab = nullptr; float* slab_b = nullptr;
};

struct ReduceArgs {
    const float* slab = nullptr; int ld_slab = 0; int64_t slab_stride = 0; int splits = 0; int N = 0;
    const float* slab_b = nullptr;
    int row0 = 0, nrows = 0, ncols = 0;
    float* dst = nullptr; int ld_dst = 0;
    float* dst_b = nullptr;
    int accumulate = 0;
    int transpose = 0;  // dst[c][r] instead of dst[r][c]
};

// variant: -1 = library default (g_nt_variant); 0 = K-step 32, 1 LDS stage; 1 = 64/1;
// 2 = 32 with double-buffered LDS; 3 = 64 double-buffered; 4 / 5 = persistent k_gemm_nt_w with
// 256x256 / 256x128 tiles of 8 waves (one block per CU; falls back to 2 when N, n_lin or a
// leading dimension is not 8 / 4 aligned)
extern int g_nt_variant;
int32_t gemm_nt(const NTArgs& a, hipStream_t s, int variant = -1);
int tn_splits(int P, int N, int K);
int skinny_chunk(int64_t P);
int32_t tn_skinny(const SkinnyArgs& a, hipStream_t s);
constexpr int kSkinnyMulti = 8;
struct SkinnyMulti {
    SkinnyArgs t[kSkinnyMulti];
    int n = 0;
};
// up to kSkinnyMulti fp32-B skinny reductions (own slabs each) in one launch
int32_t tn_skinny_multi(const SkinnyArgs* a, int n, hipStream_t s);
extern int g_tn_variant;  // 0 = one LDS stage, 1 = double-buffered
int32_t gemm_tn(const TNArgs& a, int splits, hipStream_t s, int variant = -1);
int32_t reduce_slabs(const ReduceArgs& a, hipStream_t s);
constexpr int kReduceMulti = 8;
struct ReduceMulti {
    ReduceArgs seg[kReduceMulti];
    int n = 0;
};
// up to kReduceMulti reductions (empty ones skipped) in one launch; bit-identical to one each
int32_t reduce_slabs_multi(const ReduceArgs* a, int n, hipStream_t s);

}  // namespace spn
