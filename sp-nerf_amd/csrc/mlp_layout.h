// Parameter, packed-weight and workspace layouts of the SP-NeRF MLP (host side).
#pragma once
#include <string>
#include <vector>

#include "common.h"

namespace spn {

// Derived network dimensions (models/spnerf.py:162-271).
struct Dims {
    int W, H, L, skip;
    int K0, K0p;        // encoded xyz width (60 with PE, 3 without) and its MFMA padding
    int sd, C, td;      // semantic embedding width, classes, t-embedding width
    bool sem, beta;
    int NG;             // H8 consumers  G = [feat (W) | sem hidden (H)]
    int NQ;             // feat consumers Q = [sun hidden 1 (H) | rgb hidden (H) | beta hidden (H)]
    int NO;             // outputs per point: 8 + beta + C
    int sem_col;        // first semantic-logit column of `out`
    int HP;             // per-point head pre-gradient row: [dσ, drgb3, dsun, dβ, dsem C]
    bool bf;            // cfg.dtype == 1: bf16 activations and GEMM operands (layer 0 stays fp32)
};

int32_t make_dims(const spnerf_model_cfg* cfg, Dims* d);

struct PSpec {
    std::string name;
    int64_t rows, cols;  // torch shape (cols = 0 → 1-D)
    int64_t off;         // offset (floats) in the flat gradient buffer
    int64_t numel() const { return cols ? rows * cols : rows; }
    int64_t ld() const { return cols ? cols : rows; }
};

// indices into the canonical parameter list
struct PIdx {
    int emb = -1;
    std::vector<int> fcW, fcb;
    int sigW, sigb, featW, featb, m1W = -1, m1b = -1, m2W = -1, m2b = -1;
    int r1W, r1b, r2W, r2b, s1W, s1b, s2W, s2b, s3W, s3b, s4W, s4b;
    int k1W, k1b, k2W, k2b, b1W = -1, b1b = -1, b2W = -1, b2b = -1;
};

std::vector<PSpec> param_specs(const Dims& d, PIdx* idx);

// Offsets (floats) inside the packed weight buffer.  PackedOffs is the trivially copyable part
// handed to kernels; Packed adds the per-layer vectors (host only).
struct PackedOffs {
    int64_t WG, bG, WGT, WQ, bQ, WQT;
    int64_t Ws2, bs2, Ws2T, Ws3, bs3, Ws3T;
    int64_t wsig, bsig, Wr2, br2, ws4, bs4, Wm2, bm2, wb2, bb2;
    int64_t Wk1, bk1, Wk2, bk2, Wsem0, Wsem4, emb, Wsun, Wtt;
    // bf16 copies (cfg.dtype == 1), offsets in bf16 elements from the packed base: the G, Q and
    // sun_v 2/3 matrices (forward and transposed)
    int64_t WG16 = -1, WGT16 = -1, WQ16 = -1, WQT16 = -1, Ws2_16 = -1, Ws2T16 = -1, Ws3_16 = -1, Ws3T16 = -1;
    // fc_net.0 as four bf16 planes [W][4·K0p] = [hi | hi | lo | lo] for the split layer 0
    int64_t W0s16 = -1;
    // fused inference heads (heads_bf16.hip), MFMA fragment order (frag_off): semantic hidden
    // [H][W] and sun_v 2 / 3 [H][H] with 32 features per wave, feat [W][W] and Q = [sun_v.0 ;
    // rgb.0] [2H][W] with 64 per wave; -1 where the fused heads do not apply
    int64_t Fsem16 = -1, Ffeat16 = -1, FQ16 = -1, Fs2_16 = -1, Fs3_16 = -1;
    // the training heads' solar pass: sun_v.0's rows alone [H][W], 32 features per wave
    int64_t FQs16 = -1;
    // the narrow heads as 32-row MFMA A operands (fragment order, 32 features per wave), each
    // weight row split into a bf16 hi row and a bf16 lo row (hi + lo carries the fp32 weight to
    // ~2^-17): σ [32][W] rows 0/1; albedo [32][H] rows 0/1, 2/3, 8/9 (r, g, b); sun visibility
    // [32][H] rows 0/1; zero elsewhere.  Fnar16 + narrow_off(0 / 1 / 2)
    int64_t Fnar16 = -1;
    // the training heads' fused dX chain (heads_dx_bf16.hip): the TRANSPOSED weights in fragment
    // order, element [n][k] = W[k][n] — sun_v 3 / 2 (32 features per wave, K = H), Q (64 per wave,
    // K = NQ: sun_v.0 rows then rgb.0 rows) and G (64 per wave, K = NG: feat rows then semantic
    // hidden rows); -1 where the fused dX chain does not apply
    int64_t Bs3_16 = -1, Bs2_16 = -1, BQ16 = -1, BG16 = -1;
    int64_t total;
};
struct Packed : PackedOffs {
    std::vector<int64_t> Wt, bt, WTt;   // trunk: forward [W][Kp_i], bias, transposed h-part [W][W]
    std::vector<int> Kp;                // padded K of each trunk layer
    std::vector<int64_t> Wt16, WTt16;   // bf16 trunk layers 1.. (bf16 units), -1 for layer 0
    std::vector<int64_t> Wf16;          // the same in MFMA fragment order for the fused trunk (-1: none);
                                        // layer 0: the split planes [hi | hi | lo | lo], K = 4·K0p
    std::vector<int64_t> Wb16;          // W_i[:, :W]ᵀ in fragment order (Kp = W) for the fused backward
                                        // dX chain (k_trunk_bwd_bf16); -1 for layer 0 / none
};
Packed packed_layout(const Dims& d);

// Workspace offsets (floats).  SAVE keeps every activation + derivative for the backward.
// With Dims::bf the activation / derivative / pre-activation-gradient buffers (Hb, Db, G, DG,
// Q, DQ, S2, DS2, S3, DS3, dZG, dZQ, dS3, dS2, dZa, dZb, dZc, X0b) hold bf16 at the same float offset.
struct WS {
    int64_t P, B;
    int64_t X0, X0b;
    int64_t X0s;                        // bf16 MLP: encoded input as [hi | lo | hi | lo] bf16 planes, [P][4·K0p]
    std::vector<int64_t> Hb, Db;        // H_1..H_L (save) or 3 ping-pong buffers; D_1..D_L
    int64_t G, DG, Q, DQ, S2, DS2, S3, DS3, hsave;
    int64_t rb0, rb4, rbQ, skyh, sky;
    // backward
    int64_t dZG, dZQ, dS3, dS2, dZa, dZb, dZc, hpre, slab, slab_b, RQ, R0, R4, Rp0, Rp4, skyd, skydh, gemb, embr, sk_slab, sk_slab_b;
    int64_t sk_slab_n = 0, sk_slab_b_n = 0;  // their capacities (floats)
    int64_t slab_n = 0, slab_b_n = 0;        // the TN slabs' capacities (floats)
    int64_t total;
};
WS ws_layout(const Dims& d, int64_t n_rays, int32_t n_samples, int32_t flags);
// The forward's buffers of `full` (a layout for n_total rays) restricted to rays [r0, r0 + n): the
// point-major rows from point r0·S on, the per-ray rows from ray r0 on (spnerf_mlp_forward_window;
// the backward buffers are left as laid out — the backward runs over all n_total rays)
WS ws_window(const Dims& d, const WS& full, int64_t r0, int64_t n, int32_t S);

}  // namespace spn
