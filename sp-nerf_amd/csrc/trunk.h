// Fused bf16 trunk kernel (trunk_bf16.hip): launch descriptor and the MFMA-fragment weight
// layout shared with spnerf_pack_params.
#pragma once
#include "common.h"

namespace spn {

constexpr int kTrunkMaxL = 16;

// fc_net layers 1 .. L-1 over P points: H1 (layer-0 output, [P][512] bf16) in, the output of
// layer i to Hs[i] and its derivative cos(z) to Ds[i] where non-null (the last layer's Hs is
// required).  The skip layer reads [H | X0b] and adds the per-ray rows rb_skip[p / S].
// With X0 set, layer 0 runs in the same launch instead (H1 unused): its input is the fp32
// encoding X0 [P][K0p], split in LDS into the bf16 planes [hi | lo | hi | lo] against the
// weights' [hi | hi | lo | lo] (Wf[0], K = 4·K0p), w0 = 30, per-ray rows rb0[p / S]; the skip
// layer's PE columns are the hi plane.
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
};

// Offset (bf16 elements) of W[n][k] of a [512][Kp] layer in MFMA A-fragment order: wave w =
// n / 64 streams k-steps of 16; per k-step its two 32-feature tiles are 1 KB each, lane
// (n % 32) + 32·((k / 8) % 2) holding 8 consecutive k.
__host__ __device__ inline int64_t trunk_frag_off(int n, int k, int Kp) {
    const int nks = Kp >> 4;
    return ((((int64_t)(n >> 6) * nks + (k >> 4)) * 2 + ((n >> 5) & 1)) * 64 + (n & 31) + 32 * ((k >> 3) & 1)) * 8 +
           (k & 7);
}

extern int g_fused_trunk;  // 1 = bf16 forwards use the fused trunk where supported (default)
extern int g_trunk_tile;   // 0 = tile by mode; 64 / 128 = force
extern int g_trunk_dbg;    // profiling ablations (outputs invalid): 1 = no HBM copy-outs
bool trunk_bf16_supported(int W, int L, int skip, int K0p);
// layer 0 inside the launch (TrunkArgs::X0) for this PE width when saving / not saving
bool trunk_l0_supported(int K0p, bool save);
int32_t trunk_bf16(const TrunkArgs& a, hipStream_t s, double flop, double bytes);

}  // namespace spn
