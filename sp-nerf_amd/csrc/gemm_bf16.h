// Launch descriptors of the bf16 MFMA GEMMs (gemm_bf16.hip), the cfg.dtype = 1 path.
#pragma once
#include <climits>
#include "common.h"

namespace spn {

typedef __bf16 bf16;

// Narrow output heads computed in the epilogue of the GEMM producing their input (the training
// forward's G, Q and sun_v.3 layers; models/spnerf.py:345-367): a tile whose 256 columns start at
// col0[i] is head group i's whole input; out[p] = f(Σ_c y[p][c]·w[o][c] + b[o]) over the tile's
// bf16-rounded outputs y, o < nout[i].  kind: 0 = rgb (sigmoid, out cols 0..2 as x·1.002 - 0.001,
// hsave 1..3), 1 = sun (sigmoid, out col 4 / hsave 4; the tile also writes σ = softplus(hsave 0)
// to col 3 and, full, the ray's sky to cols 5..7 — not full: zeros elsewhere), 2 = beta
// (softplus, out col 8, hsave 5 = pre-activation), 3 = semantic logits (out sem_col + o).
constexpr int kNTHeads = 3;
struct NTHeads {
    int n = 0;
    int col0[kNTHeads] = {}, nout[kNTHeads] = {}, kind[kNTHeads] = {};
    const float* w[kNTHeads] = {};   // [nout][256] fp32 (row stride ldw)
    int ldw[kNTHeads] = {};
    const float* b[kNTHeads] = {};
    float* out = nullptr; int NO = 0; int sem_col = 0;
    float* hsave = nullptr;          // [M][8]
    const float* sky = nullptr; int S = 1; int full = 0;
};

// C[M,N] = epi(A[M,K] · B[N,K]^T), bf16 operands, fp32 accumulation, bf16 C.  A may be split
// along K (columns [K1,K) from A2: the skip-layer input [h | x0]).  Epilogue (as NTArgs):
// + bias[col] + rowbias[row/rows_per_ray][col] + r1_a[row]*r1_v[col]; act==1 and col>=n_lin:
// y = sin(w0*v), D = w0*cos(w0*v) (else y = v, D = 1); y *= Dmul.
struct NT16Args {
    const bf16* A = nullptr; int lda = 0;
    const bf16* A2 = nullptr; int lda2 = 0; int K1 = 0;
    const bf16* B = nullptr; int ldb = 0;
    bf16* C = nullptr; int ldc = 0;
    int M = 0, N = 0, K = 0;
    const float* bias = nullptr;
    const float* rowbias = nullptr; int ld_rb = 0; int rows_per_ray = 1;
    const float* r1_a = nullptr; int r1_lda = 0; const float* r1_v = nullptr;
    int act = 0; float w0 = 1.f; int n_lin = 0;
    bf16* Dout = nullptr; int ld_dout = 0;
    const bf16* Dmul = nullptr; int ld_dmul = 0;
    int k_alg = 0;  // algorithmic K for the FLOP count (0 = K; the hi/lo layer-0 GEMM: K0p of its K = 4·K0p)
    // saved-pre-activation trunk layers (w0 = 1; option "zsave"): zround rounds the sine columns'
    // v to fp16 before sin / cos, dout_z stores that v (Z, fp16 bits) in Dout instead of
    // D = cos, and dmul_z reads Dmul as Z (fp16) and multiplies by cos(Z)
    int zround = 0, dout_z = 0, dmul_z = 0;
    int dbg = 0;    // ablations (tools only; variant 8): 1 = no MFMAs, 2 = no epilogue, 4 = no DMA wait
    unsigned long long* stamps = nullptr;  // diagnostic builds (-DND_STAMPS, tools only)
    NTHeads hd;     // narrow output heads folded into the epilogue (k_gemm_nt_bf16d, option heads_epi)
};

// slab[s][n][k] = Σ_{p in split s} A[p][n] · B[p][k] (B split along k at K1),
// slab_b[s][n] = Σ_{p in split s} A[p][n]; reduced by reduce_slabs (gemm_f32.h).
struct TN16Args {
    const bf16* A = nullptr; int lda = 0;
    const bf16* B = nullptr; int ldb = 0;
    const bf16* B2 = nullptr; int ldb2 = 0; int K1 = 0;
    float* slab = nullptr; int ld_slab = 0; int64_t slab_stride = 0;
    float* slab_b = nullptr;
    int P = 0, N = 0, K = 0;
    int p_per_split = 0;  // set by gemm_tn_bf16
    int b_sin = 0;        // B's columns [0, K1) hold a saved Z (fp16): staged as bf16(sin(Z)) (= the layer's H)
    int dbg = 0;          // ablations (tools only; wide tiles): 1 = no MFMAs
    int bias_split = 0;   // k_gemm_tn_bf16d: the bias sums shared by the nK = 2 tiles of a column range (g_tn16_bias_split)
    // Second point segment (one weight gradient over two passes' points, spnerf_mlp_trunk_wgrad):
    // rows p >= P1 read A_s2 / B_s2 / B2_s2 + p * ld — pointers the host shifted back by P1 rows,
    // same leading dimensions.  P1 >= P (the default) = one segment.
    int64_t P1 = INT64_MAX;
    const bf16 *A_s2 = nullptr, *B_s2 = nullptr, *B2_s2 = nullptr;
    unsigned long long* stamps = nullptr;  // diagnostic builds (-DND_STAMPS, tools/tn_lab_stamps only)
};

// variant: prefetch depth in K-steps (1 or 2); <= 0 = library default (g_nt16_variant)
extern int g_nt16_variant;
extern int g_nt16_epi;  // option nt_bf16_epi
extern int g_nt16_ip, g_tn16_ip, g_nt16_ip_gen;
extern int g_tn16_bias_split;  // option tn_bf16_bias_split
extern int g_tn16_k64;         // option tn_bf16_k64: the narrow kernel for N = 512, K = 64 weight gradients
extern int g_tn16_quad;        // option tn_bf16_quad: the quad-wave 128x128-per-wave DMA weight-gradient kernel
extern int g_tn16_m16;         // option tn_bf16_m16: the 16x16x32 weight-gradient kernel (1: 4 stages, 2: 5)
extern int g_tn16_pf;          // option tn_bf16_pf: prefetched LDS fragments in the DMA weight-gradient GEMM
extern int g_tn16_few_tiles;   // option tn_bf16_few_tiles  // DMA kernels: issue placement of the next K-step (options nt_bf16_ip, tn_bf16_ip)
int32_t gemm_nt_bf16(const NT16Args& a, hipStream_t s, int variant = -1);
// variant: 1 = 128x128 tiles, 2 = 256x256 tiles where N, K are multiples of 256, 3 = the same
// tiles fed by LDS-DMA (when P % 32 == 0 as well);
// <= 0 = library default (g_tn16_variant)
extern int g_tn16_variant;
extern int g_tn16_rounds;      // option tn_bf16_rounds: wide weight-gradient blocks per CU (1 or 2)
extern int g_tn16_min_points;  // fewest points per split (option "tn_bf16_min_points")
// few: the tn_bf16_few_tiles choice (-1: the option; the workspace layout takes the larger, 1)
// cus: the CU count to size for (-1: split_cus(); the workspace layout passes kLayoutCus)
int tn_splits_bf16(int P, int N, int K, int variant = -1, int few = -1, int cus = -1);
int32_t gemm_tn_bf16(const TN16Args& a, int splits, hipStream_t s);

// Up to kTnGroup weight-gradient GEMMs (each its own operands, shape and slabs) in ONE launch
// of the DMA kernel, splits[i] point splits for GEMM i (option tn_group in mlp.hip): a 512 x 512
// GEMM has 4 tiles, so alone it fills the CUs with 64 splits and writes 64 MB of partial slabs;
// n of them together need 1/n of the splits each (n x fewer slab bytes, one launch, one tail).
constexpr int kTnGroup = 10;
// most blocks per CU a group launch may take: the product's automatic choice is at most 2; the
// ablation build's option tn_group_rounds reaches 4 (and sizes the slab reservation for it)
#ifdef SPN_ABLATIONS
constexpr int kTnGroupRounds = 4;
#else
constexpr int kTnGroupRounds = 2;
#endif
struct TN16Group {
    TN16Args g[kTnGroup];
    int start[kTnGroup + 1];  // GEMM i's blocks: [start[i], start[i + 1])
    int n = 1;
};
static_assert(sizeof(TN16Group) <= 4096, "a kernel argument: within the 4 KB kernarg segment");
bool tn_group_ok(int P, int N, int K);  // the shape runs on the DMA kernel
int tn_tiles_bf16(int N, int K);        // its 256 x 256 tiles
int32_t gemm_tn_bf16_group(const TN16Args* a, int n, const int* splits, hipStream_t s);
// the same for the narrow N = 512, K = 64 kernel (fc_net.0 and the skip layer's PE tail together)
bool tn_k64_ok(int N, int K);
int32_t gemm_tn_bf16_k64_group(const TN16Args* a, int n, const int* splits, hipStream_t s);

}  // namespace spn
