// Fused bf16 trunk kernel (trunk_bf16.hip): launch descriptor and the MFMA-fragment weight
// layout shared with spnerf_pack_params.
#pragma once
#include "common.h"

namespace spn {

constexpr int kTrunkMaxL = 16;
// The trunk kernels' nt (cache policy of the copy-outs) and dbg (profiling ablations) arguments
// vary only in a -DSPN_ABLATIONS build; the product build folds them to the product defaults, so
// no store or copy-out sits behind a runtime branch (a branch around a store made hipcc's later
// vmcnt waits conservative: they then waited for the stores as well)
constexpr bool kTrunkAbl = kAblBuild;

// fc_net layers 1 .. L-1 over P points: H1 (layer-0 output, [P][512] bf16) in, the output of
// layer i to Hs[i] and its derivative cos(z) (with zround: Z itself) to Ds[i] where non-null
// (the last layer's Hs is required).  The skip layer reads [H | X0b] and adds the per-ray rows rb_skip[p / S].
// With X0 set, layer 0 runs in the same launch instead (H1 unused): its input is the fp32
// encoding X0 [P][K0p], split in LDS into the bf16 planes [hi | lo | hi | lo] against the
// weights' [hi | hi | lo | lo] (Wf[0], K = 4·K0p), w0 = 30, per-ray rows rb0[p / S]; the skip
// layer's PE columns are the hi plane.
// One positional-encoding value (rendering.py:147; spnerf.py:32-37): channel c of point p at
// depth zz on ray `ray` (o at [0, 3), dir at [dir_off, dir_off + 3)); n_freq = 0: xyz itself.
// o + dir*z as two rounded ops like the reference (no FMA contraction: sin(2^9 x) amplifies a
// 1-ulp difference in x by 512).  k_encode and the fused trunk's inline layer-0 staging share it.
__device__ __forceinline__ float pe_value(const float* ray, int dir_off, float zz, int c, int n_freq, int K0) {
    if (c >= K0) return 0.f;
    if (n_freq == 0) return __fadd_rn(ray[c], __fmul_rn(ray[dir_off + c], zz));
    const int k = c / 6, j = c % 6, dim = j % 3;
    const float x = __fadd_rn(ray[dim], __fmul_rn(ray[dir_off + dim], zz));
    const float arg = __fmul_rn((float)(1 << k), x);
    return j < 3 ? sinf(arg) : cosf(arg);
}

// Sum over the wavefront, returned to every lane: DPP adds inside each row of 16 lanes, then
// the four row sums read out as scalars (no LDS traffic, unlike a shuffle butterfly).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_total(float v) {
    v += dpp_f<0xb1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4e>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x124>(v);  // row_ror:4
    v += dpp_f<0x128>(v);  // row_ror:8
    const int b = __float_as_int(v);
    return (__int_as_float(__builtin_amdgcn_readlane(b, 0)) + __int_as_float(__builtin_amdgcn_readlane(b, 16))) +
           (__int_as_float(__builtin_amdgcn_readlane(b, 32)) + __int_as_float(__builtin_amdgcn_readlane(b, 48)));
}

__device__ __forceinline__ f32x4 raw_f32(f32x4 v) { return v; }
__device__ __forceinline__ f32x4 raw_f32(u32x2 v) {
    return f32x4{__uint_as_float(v[0] << 16), __uint_as_float(v[0] & 0xffff0000u), __uint_as_float(v[1] << 16),
                 __uint_as_float(v[1] & 0xffff0000u)};
}
__device__ __forceinline__ float dot4(f32x4 a, f32x4 b) { return (a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3]); }

struct TrunkArgs {
    const bf16* H1 = nullptr;
    const bf16* X0b = nullptr;
    const float* X0 = nullptr;
    const float* rb0 = nullptr;
    const bf16* Wf[kTrunkMaxL] = {};     // fragment-packed weights of layer i (trunk_frag_off)
    const float* bias[kTrunkMaxL] = {};
    bf16* Hs[kTrunkMaxL] = {};
    bf16* Ds[kTrunkMaxL] = {};
    const float* rb_skip = nullptr;
    int64_t P = 0;
    int S = 1, L = 0, skip = -1, K0p = 0;
    int dbg = 0;  // set from g_trunk_dbg by trunk_bf16
    int nt = 0;   // set from g_trunk_nt: 1 = non-temporal copy-out stores of H, 2 = of the register-D stores
    // layers >= 1 (w0 = 1): H = sin(Z), Z = the pre-activation rounded to fp16; when saving, Ds[i]
    // receives Z as fp16 (consumers recompute cos(Z) and sin(Z)) and Hs[i] may be null
    int zround = 0;
    // layer 0 from the rays themselves (inference, option "pe_inline"): with rays set and X0 null
    // the staging computes the encoding of o + dir·z (pe_value) instead of reading X0 rows
    const float* rays = nullptr;
    const float* z = nullptr;
    int rs = 0, dir_off = 0, n_freq = 0, K0 = 0;
    int ldz = 0;  // z's row stride per ray (sample j of ray r at z[r·ldz + j]); 0 = S (contiguous)
    // training with the inline encoding (k_trunk_bf16 only): the staging also writes each point's
    // bf16 PE row (the hi plane = k_encode's X0b) here, for the weight gradients of layer 0 and the
    // skip layer's PE columns
    bf16* X0b_out = nullptr;
    // training (64-point tiles, trunk_sigma_ok): the σ head's pre-activation of every point from the
    // last layer's LDS image, hsave[p·8] = w_σ·H_L + b_σ in k_heads_fwd_v's arithmetic (lane l:
    // features 4l.. and 256 + 4l.., dot4, wave_total), so the heads kernel skips H_L (1 KB / point)
    float* sig_hsave = nullptr;
    const float* wsig = nullptr;  // [512]
    const float* bsig = nullptr;  // [1]
};

// Backward dX chain of the bf16 trunk in one persistent launch (k_trunk_bwd_bf16): from
// dZ_{L-1} (dL/d pre-activation of the last trunk layer, [P][512] bf16) down to dZ_0, each
// dZ_{i-1} = (dZ_i · W_i[:, :512]) ⊙ D_{i-1} with the point tile's dZ resident in LDS between
// layers (models/spnerf.py:323-330 differentiated; the skip layer's PE columns get no gradient).
// Wb[i] = W_i[:, :512]ᵀ in the forward trunk's fragment order (trunk_frag_off, Kp = 512).
// dZ[i] may alias D[i] (a tile reads its D rows before it writes its dZ rows).
struct TrunkBwdArgs {
    const bf16* dZtop = nullptr;
    const bf16* Wb[kTrunkMaxL] = {};
    const bf16* D[kTrunkMaxL] = {};
    bf16* dZ[kTrunkMaxL] = {};
    int64_t P = 0;
    int L = 0;
    int dbg = 0;  // g_trunk_dbg (profiling ablations, outputs invalid): 1 = no dZ copy-outs, 2 = no D loads
    int nt = 3;   // g_trunk_bwd_nt: 1 = non-temporal dZ copy-outs, 2 = non-temporal D loads (3: the default)
    // per-tile column sums of dZ_l for l = rs_layer[k] (-1: none) into Rsum[k][tile][512]: the
    // per-ray sums of layer 0's and the skip layer's dZ (semantic columns) from the LDS image
    // instead of a re-read of dZ (k_ray_rowsum16).  Needs P % 64 == 0; the order is tile_colsum's
    float* Rsum[2] = {nullptr, nullptr};
    int rs_layer[2] = {-1, -1};
};

// Column sums of a 64-row bf16 [64][512] tile in a fixed order shared by the fused backward (LDS
// image) and k_tile_rowsum16 (HBM): wave w adds rows 8w .. 8w+7 of its 8 columns (lane = 16-B
// chunk) in row order, then column c = Σ_w part[w][c] in wave order.
__device__ __forceinline__ void tile_colsum_part(const u32x4 (&rows)[8], float (&a)[8]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        float f[8];
        unpack8(rows[r], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += f[e];
    }
}
__device__ __forceinline__ float tile_colsum_final(const float* part, int c) {
    float s = part[c];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += part[k * 512 + c];
    return s;
}

// Offset (bf16 elements) of W[n][k] of a [512][Kp] layer in MFMA A-fragment order: wave w =
// n / 64 streams k-steps of 16; per k-step its two 32-feature tiles are 1 KB each, lane
// (n % 32) + 32·((k / 8) % 2) holding 8 consecutive k.
#ifndef SPN_TRUNK_KMAJOR
#define SPN_TRUNK_KMAJOR 0
#endif
// With SPN_TRUNK_KMAJOR the 8 waves' 2 KB pieces of one k-step are adjacent (16 KB per k-step)
// instead of each wave's stream being contiguous.
__host__ __device__ inline int64_t trunk_frag_off(int n, int k, int Kp) {
    const int nks = Kp >> 4;
    const int64_t blk = SPN_TRUNK_KMAJOR ? (int64_t)(k >> 4) * 8 + (n >> 6) : (int64_t)(n >> 6) * nks + (k >> 4);
    return ((blk * 2 + ((n >> 5) & 1)) * 64 + (n & 31) + 32 * ((k >> 3) & 1)) * 8 + (k & 7);
}
// wave w's stream of a layer with nks k-steps: the first k-step's offset and the k-step stride
__host__ __device__ inline int64_t trunk_wave_off(int w, int nks) { return SPN_TRUNK_KMAJOR ? w * 1024 : (int64_t)w * nks * 1024; }
constexpr int kTrunkKStride = SPN_TRUNK_KMAJOR ? 8192 : 1024;

// MFMA A-fragment order for a layer whose waves own NA 32-feature tiles each (NA = 2: the trunk's
// layout above; NA = 1: 32 features per wave, for 256-wide layers)
__host__ __device__ inline int64_t frag_off(int n, int k, int Kp, int NA) {
    const int nks = Kp >> 4, per = 32 * NA;
    return ((((int64_t)(n / per) * nks + (k >> 4)) * NA + (n >> 5) % NA) * 64 + (n & 31) + 32 * ((k >> 3) & 1)) * 8 +
           (k & 7);
}

// Fused inference heads (heads_bf16.hip): from the trunk's last activation H_L (bf16 [P][W]) to
// the output rows, one persistent launch, a 128-point tile's activations resident in LDS:
// σ = softplus(w_σ·H + b); semantic hidden = sin(W_m1 H + b) → logits (its C dot products in
// the epilogue); feat = W_f H + b; [sun1 | rgb1] = sin(W_Q feat + b + per-ray sun rows);
// albedo from rgb1; sun2 = sin(W_s2 sun1 + b); sun3 = sin(W_s3 sun2 + b); sun = sigmoid(w_s4
// sun3 + b); sky from the per-ray rows.  W = 512, H = 256, no β head, C ≤ 4
// (models/spnerf.py:332-367).
struct HeadsFusedArgs {
    const bf16* HL = nullptr;
    const float* packed = nullptr;
    const float* rbQ = nullptr;   // per-ray sun-direction rows of Q [B][2H]
    const float* sky = nullptr;   // per-ray sky colour [B][4]
    float* out = nullptr;
    int64_t P = 0;
    int S = 1, NO = 8, C = 0, sem_col = 8, mode = 0;  // mode: 0 all heads, 1 σ only
    int nt = 0;  // non-temporal loads of HL (g_trunk_nt & 2)
    int dbg = 0;  // profiling ablations (g_heads_dbg; outputs invalid): 2 = no H staging loads
    // training (k_heads_train_bf16, hd::heads_tile_train; mode 0 or 2 = the solar pass): every
    // activation the backward reads, at the layer-by-layer GEMMs' addresses —
    // G = [feat | sem hidden] and DG [P][ldG], Q = [sun1 | rgb1] and DQ [P][ldQ], sun_v 2 / 3 and
    // their D [P][H]; hsave[p·8] = the heads' saved gates (σ pre-activation written by the trunk)
    bf16 *G = nullptr, *DG = nullptr, *Q = nullptr, *DQ = nullptr;
    bf16 *S2 = nullptr, *DS2 = nullptr, *S3 = nullptr, *DS3 = nullptr;
    float* hsave = nullptr;
    int ldG = 0, ldQ = 0;
};
struct PackedOffs;
struct Dims;
bool heads_bf16_shape_ok(const Dims& d);   // the packed layout carries the fused heads' weights
bool heads_bf16_supported(const Dims& d);  // ... and the option is on
int32_t heads_bf16(const HeadsFusedArgs& a, const PackedOffs& k, hipStream_t s, double flop, double bytes);
// training heads as their own launch after the saving trunk (option heads_epi 2): H_L from HBM
bool heads_train_bf16_ok(const HeadsFusedArgs& h, const PackedOffs& k);
int32_t heads_train_bf16(const HeadsFusedArgs& a, const PackedOffs& k, hipStream_t s, double flop, double bytes);
// the inference trunk with the fused heads on its last LDS image (k_trunk2_bf16 HEADS): no H_L in HBM
extern int g_trunk_heads;
bool trunk2_heads_ok(const TrunkArgs& a);
// the same fused heads inside the one-workgroup k_trunk_bf16<128> (option trunk_heads 2)
bool trunk1_heads_ok(const TrunkArgs& a);
int32_t trunk1_heads_bf16(const TrunkArgs& a, const HeadsFusedArgs& h, const PackedOffs& k, hipStream_t s, double flop,
                          double bytes);
int32_t trunk2_heads_bf16(const TrunkArgs& a, const HeadsFusedArgs& h, const PackedOffs& k, hipStream_t s, double flop,
                          double bytes);

extern int g_heads_dbg;    // HeadsFusedArgs::dbg
extern int g_fused_heads;  // 1 = bf16 inference runs the fused heads where supported (default)
extern int g_fused_trunk;  // 1 = bf16 forwards use the fused trunk where supported (default)
extern int g_trunk_tile;   // 0 = tile by mode; 64 / 128 = force
extern int g_trunk_dbg;    // profiling ablations (outputs invalid): 1 = no HBM copy-outs
extern int g_trunk_var;    // profiling ablations of the 128-point trunk (outputs invalid)
extern int g_trunk_dreg;   // 64-point training tiles: D stored from the registers in the epilogue
extern int g_trunk_nt;     // 1 = trunk H stores non-temporal, 2 = fused heads' H loads non-temporal, 4 = training D stores
bool trunk_bf16_supported(int W, int L, int skip, int K0p);
// layer 0 inside the launch (TrunkArgs::X0) for this PE width when saving / not saving
bool trunk_l0_supported(int K0p, bool save, bool zround = false);  // zround: the zsave (64-point) tiling
int32_t trunk_bf16(const TrunkArgs& a, hipStream_t s, double flop, double bytes);
// the launch trunk_bf16 would make for a (saving) computes the σ rows (TrunkArgs::sig_hsave)
bool trunk_sigma_ok(const TrunkArgs& a, bool save);
extern int g_trunk_sigma;  // option trunk_sigma
// the two-workgroups-per-CU tiling (trunk2_bf16.hip): D stored from the registers, 76 KB of LDS
extern int g_trunk2;       // 0 = off, 1 = saving (training) launches, 2 = every launch
extern int g_trunk2_tile;  // 64 or 128 points per tile
bool trunk2_supported(const TrunkArgs& a, bool save);
int32_t trunk2_bf16(const TrunkArgs& a, hipStream_t s, bool save, double flop, double bytes);
int32_t trunk_bwd_bf16(const TrunkBwdArgs& a, hipStream_t s, double flop, double bytes);
extern int g_trunk_bwd_nt;    // the dX chain's non-temporal dZ stores (1) / D loads (2)
extern int g_trunk_bwd_dreg;  // the fused dX chain stores dZ from the epilogue's registers
extern int g_fused_bwd;  // 1 = the bf16 training backward runs its dX chain in k_trunk_bwd_bf16

}  // namespace spn
