// The training heads' fused dX chain (heads_dx_bf16.hip): launch descriptor.
#pragma once
#include "common.h"

namespace spn {

// One backward pass's heads dX chain over P points (bf16 MLP, W = 512, H = 256, no β; mode 0 = every
// head, 2 = the solar pass): the narrow heads' gradients (dS3, dZQ's rgb half, dZG's semantic half,
// hpre's dσ column) and the saved derivatives (DS2, DQ, D_L) in; dS2, dZQ's sun half, dZG's feat
// half and dZL = the trunk's top pre-activation gradient out — the four layer-by-layer DMA GEMMs'
// outputs, bit for bit.
struct HeadsDxArgs {
    const bf16 *dS3 = nullptr, *DS2 = nullptr, *DQ = nullptr, *DL = nullptr;
    bf16 *dS2 = nullptr, *dZQ = nullptr, *dZG = nullptr, *dZL = nullptr;
    const float* hpre = nullptr;  // [P][HP], column 0 = dσ (the rank-1 term's point factor)
    const float* wsig = nullptr;  // [W] w_σ
    const bf16* packed16 = nullptr;
    int64_t Bs3 = -1, Bs2 = -1, BQ = -1, BG = -1;  // PackedOffs fragment streams (bf16 units)
    int64_t P = 0;
    int ldQ = 0, ldG = 0, HP = 0;  // dZQ / DQ and dZG row strides (= the layouts' K: NQ, NG)
    int kQ = 0, kG = 0;            // K of the Q / G fragment layouts (NQ, NG)
    int mode = 0, sem = 0;
};

extern int g_heads_dx;
bool heads_dx_bf16_ok(const HeadsDxArgs& a);
int32_t heads_dx_bf16(const HeadsDxArgs& a, hipStream_t s, double flop, double bytes);

}  // namespace spn
