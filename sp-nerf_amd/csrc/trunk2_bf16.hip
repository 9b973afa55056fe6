// Fused bf16 SIREN trunk, TWO workgroups per CU (models/spnerf.py:201-209, 323-330): the
// training tiling of the trunk (H_i and D_i = cos of every layer saved for the backward) rebuilt
// so that one workgroup's epilogue (VALU: bias, sin/cos, bf16 packing) runs beside the other
// workgroup's MFMAs on the same SIMDs.
//
// Why: in the one-workgroup 64-point kernel (k_trunk_bf16<64>, trunk_bf16.hip) every layer of a
// tile is k-loop → barrier → epilogue → barrier, and the next layer needs the whole epilogue's
// output, so the MFMA pipe idles through every epilogue and every barrier (PMC: MFMA busy 0.30).
// Its D image, which drained D through LDS, took the second half of the LDS, so a second tile
// could not be resident.  Here D leaves straight from the accumulator registers: pairs of
// 8-byte pieces joined by v_permlane32_swap into one 16-byte store per lane (32 rows × 32 B per
// instruction), so the LDS holds only the [64][512] activation image, the skip layer's PE
// tile, the bias slots and one per-ray row (80 KB), and two workgroups share each CU.
//
// Geometry: 64 points per tile, 4 waves (one per SIMD per workgroup); wave w owns output features
// [128w, 128w + 128) — four 32-feature A tiles — of both 32-point B tiles: 8 MFMAs
// (v_mfma_f32_32x32x16_bf16) per B-fragment pair and k-step.  Weights are the A operand streamed
// from L2 in the fused trunk's fragment order (trunk_frag_off: the wave reads the streams of the
// 64-feature groups 2w and 2w + 1) through a TPD-deep register ring that runs on from one
// layer's stream into the next one's; the image is the B operand.  Epilogue arithmetic and k
// order are those of k_trunk_bf16 (and of the layer-by-layer k_gemm_nt_bf16): outputs equal
// theirs bit for bit.
//
// Memory-counter discipline (vmcnt counts loads and stores together, in order): every store
// goes through a buffer descriptor whose range ends at the last valid row (rows past P are
// dropped by the hardware, no branch), and the next layer's bias and per-ray row are loaded
// right after the k-loop, BEFORE the epilogue's stores — so waiting for them never waits for
// this layer's D stores.
#include <algorithm>
#include <type_traits>

#include "heads_tile.h"
#include "trunk.h"

namespace spn {

// Measured slower than the one-workgroup k_trunk_bf16 since round 4 (comments below): the kernel is
// compiled only into -DSPN_ABLATIONS builds; the product build keeps the option variables, and its
// trunk2_supported / trunk2_heads_ok are false.
int g_trunk2 = 0;
int g_trunk2_tile = 128;
int g_trunk_heads = 2;

#ifdef SPN_ABLATIONS
#if SPN_TRUNK_KMAJOR
#error "trunk2_bf16.hip reads the wave-contiguous fragment streams (SPN_TRUNK_KMAJOR 0)"
#endif

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 0 = the one-workgroup kernels; 1 = this kernel for the saving (training) launches; 2 = for
// every launch; 3 = for the inference (non-saving) launches only — the default: C5 23.41 / 23.42
// against 23.33 / 23.25 ms per step, trunk 16.13 -> 15.92 ms (pairs in one call, 128-point tiles).  Measured on MI355X (tools/gpu_t2ab.sh, tools/pmc_trunk2.sh,
// training forward at 524 288 points): one-workgroup k_trunk_bf16<64> 3.05 ms, this kernel
// 3.08 ms (64-point tiles, two workgroups per CU) and 3.38 ms (128-point tiles); without any HBM
// copy-out it is the faster one (1.84–1.96 against 2.45 ms), but PMC shows the waves waiting on
// s_waitcnt 51–65 % of their cycles (one-workgroup kernel 37 %): vmcnt retires loads and stores
// in order, so the weight refills issued after an epilogue's D stores wait for those stores'
// acknowledgements.  Bit-identical (tests/test_gpu_trunk.py).
// Round 4: 0 is the default again — the one-workgroup k_trunk_bf16<128> is now the faster inference
// trunk (C5 trunk alone, trunk_heads 0: 15.49 against 16.65 ms per step, one call) and carries the
// fused heads itself (trunk_heads 2).
// (g_trunk2 is defined at the top of the namespace)

namespace {
constexpr int TW = 512;
constexpr int TPD = 4;                     // weight prefetch depth (k-steps)
constexpr int NMAIN = TW / 16;             // k-steps over the image
constexpr int ROWB = TW * 2;               // bytes per [512] bf16 row

// Two tilings:
//  * TM = 64: 4 waves, wave w owns features [128w, 128w + 128) (4 A tiles) of the 2 B tiles; two
//    workgroups per CU (80 KB of LDS each), so one's epilogue can run beside the other's MFMAs;
//  * TM = 128: 8 waves, wave w owns features [64w, 64w + 64) (2 A tiles) of the 4 B tiles; one
//    workgroup per CU (152 KB) — every weight byte streamed from L2 serves 128 points instead of
//    64 (at the MFMA peak 32 instead of 64 B/clk/CU of weights, against the ≈55 the L2 delivers).
template <int TM>
struct T2Geo {
    static constexpr int NT = TM == 64 ? 256 : 512;   // threads
    static constexpr int NW = NT / 64;                 // waves
    static constexpr int NA = TW / 32 / NW;            // 32-feature A tiles per wave
    static constexpr int NJ = TM / 32;                 // 32-point B tiles
    static constexpr int WGS = TM == 64 ? 2 : 1;       // resident workgroups per CU
    static constexpr int IMG = TM * TW * 2;            // [TM][512] bf16
    static constexpr int X0_OFF = IMG;                 // [TM][K0p <= 64] bf16 PE tile (skip layer)
    static constexpr int BIAS_OFF = X0_OFF + TM * 64 * 2;
    static constexpr int RB_OFF = BIAS_OFF + 2 * TW * 4;  // two slots of the tile's per-ray row
    static constexpr int LDS = RB_OFF + 2 * TW * 4;    // 81 920 / 155 648 B
    static constexpr int CPT = TM * 64 / NT;           // 16-B chunks of the image per thread (16)
    static constexpr int PT = TW / NT;                 // bias / row values per thread
    static_assert(LDS * WGS <= 160 * 1024, "LDS");
};

__device__ __forceinline__ int act_off(int row, int ch) { return row * 1024 + ((ch ^ (row & 15)) << 4); }
__device__ __forceinline__ int x0_rel(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

// a store descriptor over rows [p0, p0 + nrows) of a [P][512] bf16 tensor (nrows = 0 or a null
// tensor: every store through it is dropped)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(bf16* t, int64_t p0, int nrows) {
    bf16* base = t ? t + p0 * TW : nullptr;
    const int bytes = t ? nrows * ROWB : 0;
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}
}  // namespace

// SAVE: every layer's D out (training; Ds[i] all set); L0: layer 0 in the launch.
// HEADS (inference, TM = 128, option trunk_heads): the fused heads (heads_tile.h) run on the
// last layer's LDS image, so H_L never leaves the chip (≈1 KB per point written and read back
// by k_heads_bf16); their output staging is 8 KB beyond the trunk's LDS, their partials overlay
// the PE tile (restaged by the next tile), and the weight ring is primed per tile instead of
// running on through the heads.
// The HEADS kernel's argument: the trunk's (first, so the kernarg-segment reads of TrunkArgs stay
// valid) and the heads' — read per tile through an opaque kernarg pointer, so the compiler does not
// hoist the heads' ~40 offsets out of the tile loop into registers live through the trunk layers
using Trunk2HeadsArgs = TrunkHeadsArgs;  // (heads_tile.h)

template <int TM, bool L0, bool SAVE, bool HEADS = false>
__global__ __launch_bounds__(T2Geo<TM>::NT, T2Geo<TM>::WGS) void k_trunk2_bf16(
    std::conditional_t<HEADS, Trunk2HeadsArgs, TrunkArgs> g, int ntiles) {
    using Geo = T2Geo<TM>;
    static_assert(!HEADS || (TM == 128 && !SAVE), "the fused heads: 128-point inference tiles");
    constexpr int NT = Geo::NT, NA = Geo::NA, NJ = Geo::NJ, CPT = Geo::CPT, PT = Geo::PT;
    constexpr int X0_OFF = Geo::X0_OFF, BIAS_OFF = Geo::BIAS_OFF, RB_OFF = Geo::RB_OFF;
    constexpr int OST_OFF = Geo::LDS;  // (HEADS) the heads' output staging
    static_assert(!HEADS || (Geo::RB_OFF - Geo::X0_OFF >= hd::PART_BYTES && Geo::LDS + hd::OST_BYTES <= 160 * 1024),
                  "heads LDS");
    __shared__ __attribute__((aligned(16))) char smem[Geo::LDS + (HEADS ? hd::OST_BYTES : 0)];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, h = lane >> 5;
    float* sbias = reinterpret_cast<float*>(smem + BIAS_OFF);
    float* srb = reinterpret_cast<float*>(smem + RB_OFF);
    char* sx0 = smem + X0_OFF;
    const int x0ch = g.K0p >> 3;
    const int ntail = g.K0p >> 4;
    const int first = L0 ? 0 : 1;
    const int nk0 = g.K0p >> 2;  // layer 0's k-steps over the 4·K0p hi/lo planes
    auto nks_of = [&](int i) { return i == 0 ? nk0 : NMAIN + (i == g.skip ? ntail : 0); };
    const int sw = r32 & 15;
    typedef const __attribute__((address_space(4))) TrunkArgs* KArgs;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();
    // the per-ray row of layer i (semantic rows at layer 0 and the skip layer), or null
    auto rb_of = [&](int i) -> const float* { return i == 0 ? (L0 ? g.rb0 : nullptr) : (i == g.skip ? g.rb_skip : nullptr); };
    // Bias and per-ray row of a layer: LDS slot pairs alternating from layer to layer (across
    // tiles too).  The next layer's values are loaded right after a k-loop, unconditionally (a
    // layer without a row loads its bias in its place), and written into the other slot at the
    // end of the epilogue.  A layer without a row gets −0.0 in its row slot: the epilogue adds
    // the row everywhere, (acc + b) + (−0.0) = acc + b exactly, so no layer-dependent branch
    // splits the epilogue (joins of instances made hipcc wait vmcnt(0) on the D stores).
    auto ray_row = [&](int i, int64_t pt) {  // row source of layer i for the tile at point pt
        const float* rb = rb_of(i);
        return rb ? rb + (std::min<int64_t>(pt, g.P - 1) / g.S) * TW : ka->bias[i];
    };

    u32x4 ring[TPD][NA];
    // this wave's stream of layer i: the 64-feature groups (NA / 2)·w + a / 2 (A tiles a of the
    // wave), each k-step 1 KB per A tile; group g + 1's stream starts nks k-steps after group g's
    auto wstream = [&](int i) { return ka->Wf[i] + trunk_wave_off(NA / 2 * w, nks_of(i)) + opaque(lane) * 8; };
    auto load_step = [&](int d, const bf16* src, int nks) {
#pragma unroll
        for (int a = 0; a < NA; ++a) ring[d][a] = ldg16(src + (a >> 1) * nks * kTrunkKStride + (a & 1) * 512);
    };
    // chunks [q0, q0 + n) (per thread) of the image to the rows of descriptor r
    auto copy_out = [&](__amdgpu_buffer_rsrc_t r, int q0, auto kn) {
        constexpr int n = decltype(kn)::value;
        const int ct = opaque(tid);
        u32x4 v[n];
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int c = ct + NT * (q0 + q);
            v[q] = *reinterpret_cast<const u32x4*>(smem + act_off(c >> 6, c & 63));
        }
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int c = ct + NT * (q0 + q);
            if (SAVE && (g.nt & 1))  // block-uniform: non-temporal H copy-outs of training (trunk_nt 1)
                __builtin_amdgcn_raw_buffer_store_b128(v[q], r, (c >> 6) * ROWB + (c & 63) * 16, 0, 3);
            else
                __builtin_amdgcn_raw_buffer_store_b128(v[q], r, (c >> 6) * ROWB + (c & 63) * 16, 0, 0);
        }
    };

    int tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;  // block-uniform
    int sl = 0;  // the slot of the current layer
    {
        const int t = opaque(tid);
        const float* rr = ray_row(first, (int64_t)tile * TM);
        const bool row = rb_of(first) != nullptr;
#pragma unroll
        for (int q = 0; q < PT; ++q) {
            sbias[t + q * NT] = ka->bias[first][t + q * NT];
            srb[t + q * NT] = row ? rr[t + q * NT] : -0.f;
        }
        if constexpr (!HEADS) {
            const bf16* src = wstream(first);
            const int nks = nks_of(first);
#pragma unroll
            for (int d = 0; d < TPD; ++d) load_step(d, src + d * kTrunkKStride, nks);
        }
    }
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TM;
        const int nrows = (int)std::min<int64_t>(TM, g.P - p0);
        const int st = opaque(tid);
        if constexpr (HEADS) {  // the first layer's stream, in flight through the tile's staging
            const bf16* src = wstream(first);
            const int nks = nks_of(first);
#pragma unroll
            for (int d = 0; d < TPD; ++d) load_step(d, src + d * kTrunkKStride, nks);
        }
        // stage the first layer's input and the PE tile; rows past P read a clamped row (their
        // outputs are dropped by the store descriptors)
        if constexpr (L0) {
            // 8 fp32 PE values per unit → hi and lo chunks: image columns [hi | lo | hi | lo]
            // (layer 0's B operand against the weights' [hi | hi | lo | lo]) and the PE tile (= hi)
            for (int u = st; u < TM * x0ch; u += NT) {
                const int row = u / x0ch, q = u % x0ch;
                const int64_t pr = std::min<int64_t>(p0 + row, g.P - 1);
                float xv[8];
                if (g.rays) {  // block-uniform: encode o + dir·z here (pe_value, as k_encode)
                    const int64_t rr = pr / g.S;
                    const float* rp = g.rays + rr * g.rs;
                    const float zz = g.z[rr * g.ldz + (pr - rr * g.S)];
#pragma unroll
                    for (int e = 0; e < 8; ++e) xv[e] = pe_value(rp, g.dir_off, zz, q * 8 + e, g.n_freq, g.K0);
                } else {
                    const float* src = g.X0 + pr * g.K0p + q * 8;
                    const f32x4 v0 = ld4(src), v1 = ld4(src + 4);
#pragma unroll
                    for (int e = 0; e < 8; ++e) xv[e] = e < 4 ? v0[e] : v1[e - 4];
                }
                float hf[8], lf[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    hf[e] = (float)(bf16)xv[e];
                    lf[e] = xv[e] - hf[e];
                }
                const u32x4 hi = pack8(hf), lo = pack8(lf);
                *reinterpret_cast<u32x4*>(smem + act_off(row, q)) = hi;
                *reinterpret_cast<u32x4*>(smem + act_off(row, x0ch + q)) = lo;
                *reinterpret_cast<u32x4*>(smem + act_off(row, 2 * x0ch + q)) = hi;
                *reinterpret_cast<u32x4*>(smem + act_off(row, 3 * x0ch + q)) = lo;
                if (g.skip > 0) *reinterpret_cast<u32x4*>(sx0 + x0_rel(row, q)) = hi;
            }
        } else {
#pragma unroll
            for (int q0 = 0; q0 < CPT; q0 += 8) {
                u32x4 v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int c = st + NT * (q0 + q);
                    v[q] = ldg16(g.H1 + std::min<int64_t>(p0 + (c >> 6), g.P - 1) * TW + (c & 63) * 8);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int c = st + NT * (q0 + q);
                    *reinterpret_cast<u32x4*>(smem + act_off(c >> 6, c & 63)) = v[q];
                }
            }
            if (g.skip > 0) {
                for (int c = st; c < TM * x0ch; c += NT) {
                    const int row = c / x0ch, ch = c % x0ch;
                    *reinterpret_cast<u32x4*>(sx0 + x0_rel(row, ch)) =
                        ldg16(g.X0b + std::min<int64_t>(p0 + row, g.P - 1) * g.K0p + ch * 8);
                }
            }
        }

        // H of the previous layer (copied out during this k-loop; none before the first layer)
        __amdgpu_buffer_rsrc_t hpend = rows_rsrc(nullptr, 0, 0);
        for (int i = first; i < g.L; ++i) {
            const bf16* wsrc = wstream(i);
            const int nks = nks_of(i);
            const bool last = i == g.L - 1;
            const int inext = last ? (!HEADS && tile + (int)gridDim.x < ntiles ? first : -1) : i + 1;
            const bf16* wnxt = inext >= 0 ? wstream(inext) : wsrc;
            const int nks_nxt = inext >= 0 ? nks_of(inext) : nks;
            const int nkm = i == 0 ? nk0 : NMAIN;
            const float* sb = sbias + sl * TW;
            const float* sr = srb + sl * TW;
            f32x16 acc[NA][NJ];
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
            __syncthreads();  // the image, the bias slot and the per-ray row of layer i are complete

            const char* brow = smem + r32 * 1024;
            bf16x8 bc[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) bc[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((h ^ sw) << 4));
#pragma unroll 1
            for (int ks0 = 0; ks0 < nkm; ks0 += TPD) {
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    const int ks = ks0 + d;
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
                    // refill the slot just consumed (TPD - 1 steps of cover); past the stream's
                    // end the next layer's step d (a selected address, not a branch: a load
                    // behind a branch made hipcc drain vmcnt(0))
                    const bool in = ks + TPD < nks;
                    load_step(d, in ? wsrc + (ks + TPD) * kTrunkKStride : wnxt + d * kTrunkKStride, in ? nks : nks_nxt);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, NA, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x020, NA, 0);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) bc[j] = bn[j];
                }
                // drain the previous layer's H: CPT / (NMAIN / TPD) chunks per thread per slice
                constexpr int per = CPT / (NMAIN / TPD);
                static_assert(per * (NMAIN / TPD) == CPT && per >= 1, "copy slices");
                if (!(g.dbg & 1)) copy_out(hpend, (ks0 / TPD) * per, std::integral_constant<int, per>{});
            }
            // the PE columns of the skip layer's input [h | x0]: exactly TPD k-steps (host check)
            if (nks > NMAIN) {  // block-uniform
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    bf16x8 b[NJ];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) b[j] = *reinterpret_cast<const bf16x8*>(sx0 + x0_rel(32 * j + r32, 2 * d + h));
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
#pragma unroll
                        for (int a = 0; a < NA; ++a)
                            acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ring[d][a]), b[j],
                                                                              acc[a][j], 0, 0, 0);
                    load_step(d, wnxt + d * kTrunkKStride, nks_nxt);
                }
            }

            __syncthreads();  // every wave is done reading the image of layer i
            // the next layer's (past the last layer: the next tile's first layer's) bias and
            // per-ray row, loaded before this epilogue's stores
            float nb[PT], nr[PT];
            const int in = last ? first : i + 1;
            const bool nrow = rb_of(in) != nullptr;
            {
                const int t = opaque(tid);
                const float* rr = ray_row(in, last ? p0 + (int64_t)gridDim.x * TM : p0);
#pragma unroll
                for (int q = 0; q < PT; ++q) {
                    nb[q] = ka->bias[in][t + q * NT];
                    nr[q] = rr[t + q * NT];
                }
            }
            // (dbg 2: every D store dropped by the descriptor — the HBM bytes of D ablated)
            const __amdgpu_buffer_rsrc_t dr = rows_rsrc(SAVE && !(g.dbg & 2) ? ka->Ds[i] : nullptr, p0, nrows);
            // sin → the image; with Ds: cos (×w0 at layer 0) → HBM straight from the registers,
            // the 8-byte pieces of groups (0, 1) and (2, 3) joined by permlane32 swaps into 16 B
            auto epilogue = [&](auto ksave, auto kl0) {
                constexpr bool save = decltype(ksave)::value;
                constexpr float w0 = decltype(kl0)::value ? 30.f : 1.f;
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
#pragma unroll
                for (int a = 0; a < NA; ++a) {
                    const int fa = 32 * NA * w + 32 * a + 4 * eh;  // + 8·gq: this lane's 4 features of group gq
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int row = 32 * j + er32;
                        u32x2 cq[4];
#pragma unroll
                        for (int gq = 0; gq < 4; ++gq) {
                            const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + fa + 8 * gq);
                            const f32x4 rv = *reinterpret_cast<const f32x4*>(sr + fa + 8 * gq);
                            float y[4], c[4];
                            if constexpr (w0 == 1.f && SPN_PK_EPI) {
                                // (acc + bias) + row, then · 1/2π (fast_sin's argument in
                                // revolutions) as packed pairs: the same roundings per element,
                                // half the VALU issue slots
#pragma unroll
                                for (int e = 0; e < 4; e += 2) {
                                    const f32x2 v2 = (f32x2{acc[a][j][4 * gq + e], acc[a][j][4 * gq + e + 1]} + f32x2{bv[e], bv[e + 1]}) +
                                                     f32x2{rv[e], rv[e + 1]};
                                    const f32x2 r2 = v2 * f32x2{0.15915494309189535f, 0.15915494309189535f};
#pragma unroll
                                    for (int u = 0; u < 2; ++u) {
                                        y[e + u] = __builtin_amdgcn_sinf(r2[u]);
                                        if constexpr (save) c[e + u] = __builtin_amdgcn_cosf(r2[u]);
                                    }
                                }
                            } else {
#pragma unroll
                                for (int e = 0; e < 4; ++e) {
                                    // (acc + bias) + row, as the layer-by-layer epilogue adds them
                                    const float v = (acc[a][j][4 * gq + e] + bv[e]) + rv[e];
                                    const float x = w0 * v;
                                    if constexpr (save) {
                                        fast_sincos(x, &y[e], &c[e]);
                                        c[e] = w0 * c[e];
                                    } else {
                                        y[e] = fast_sin(x);
                                    }
                                }
                            }
                            *reinterpret_cast<u32x2*>(smem + act_off(row, (fa + 8 * gq) >> 3) + 8 * eh) =
                                u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                            if constexpr (save) cq[gq] = u32x2{pack2(c[0], c[1]), pack2(c[2], c[3])};
                        }
                        if constexpr (save) {
#pragma unroll
                            for (int k = 0; k < 4; k += 2) {
#pragma unroll
                                for (int e = 0; e < 2; ++e) {
                                    const auto r = __builtin_amdgcn_permlane32_swap(cq[k][e], cq[k + 1][e], false, false);
                                    cq[k][e] = r[0];
                                    cq[k + 1][e] = r[1];
                                }
                                // lanes 0..31: features 8k..8k+7 of the group pair, lanes 32..63: 8k+8..8k+15
                                const int fb = 32 * NA * w + 32 * a + 8 * k + 8 * eh;
                                __builtin_amdgcn_raw_buffer_store_b128(u32x4{cq[k][0], cq[k][1], cq[k + 1][0], cq[k + 1][1]}, dr,
                                                                       row * ROWB + fb * 2, 0, 0);
                            }
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted loads
                }
                // the next layer's bias and row into the other slot (last read by the previous
                // layer's epilogue); every instance issues the same stores, so the wait for these
                // loads counts them exactly
                const int t = opaque(tid);
                float* sbn = sbias + (sl ^ 1) * TW;
                float* srn = srb + (sl ^ 1) * TW;
#pragma unroll
                for (int q = 0; q < PT; ++q) {
                    sbn[t + q * NT] = nb[q];
                    srn[t + q * NT] = nrow ? nr[q] : -0.f;
                }
            };
            constexpr std::integral_constant<bool, SAVE> ks{};
            if (L0 && i == 0) epilogue(ks, std::true_type{});  // block-uniform
            else epilogue(ks, std::false_type{});
            sl ^= 1;
            const __amdgpu_buffer_rsrc_t hr = rows_rsrc(ka->Hs[i], p0, nrows);
            if (last) {
                __syncthreads();
                if constexpr (HEADS) {  // H_L stays on chip: the heads on this image
                    typedef const __attribute__((address_space(4))) Trunk2HeadsArgs* KH;
                    KH kh = (KH)__builtin_amdgcn_kernarg_segment_ptr();
                    asm volatile("" : "+s"(kh));  // opaque per tile: the heads' argument loads stay here
                    hd::heads_tile<false>(kh->hg, kh->hk, smem, reinterpret_cast<float*>(smem + OST_OFF),
                                          reinterpret_cast<float*>(smem + X0_OFF), nullptr, p0);
                } else if (!(g.dbg & 1)) {
#pragma unroll
                    for (int q0 = 0; q0 < CPT; q0 += 4) copy_out(hr, q0, std::integral_constant<int, 4>{});
                }
            }
            hpend = hr;
        }
        __syncthreads();  // the next tile restages the image and reuses the bias slots
    }
}

// option "trunk2_tile": 64 (two workgroups per CU) or 128 points per tile (the default); 0 = 128, or
// 64 when per-ray rows are staged per tile and a ray's samples (e.g. 64) do not fill 128 points —
// which puts C4's guided pass 1 on the two-workgroup kernel: measured slower than the one-workgroup
// k_trunk_bf16<128> it otherwise falls back to (0.161 vs 0.145 ms per 512-ray step, 1.17 vs 1.05 at
// 4 096 rays; same call)
// (g_trunk2_tile is defined at the top of the namespace)

static int trunk2_tm(const TrunkArgs& a) {
    if (g_trunk2_tile == 64 || g_trunk2_tile == 128) return g_trunk2_tile;
    const bool rows = ((a.X0 || a.rays) && a.rb0) || a.rb_skip;
    return rows && a.S % 128 != 0 && a.S % 64 == 0 ? 64 : 128;
}

bool trunk2_supported(const TrunkArgs& a, bool save) {
    const bool on = g_trunk2 == 2 || (g_trunk2 == 1 && save) || (g_trunk2 == 3 && !save);
    if (!on || a.zround) return false;
    const int TM = trunk2_tm(a);
    const bool l0 = a.X0 || a.rays;
    if (l0 && !(a.K0p % 4 == 0 && (a.K0p / 4) % TPD == 0)) return false;
    if (a.skip > 0 && a.K0p != 16 * TPD) return false;  // the skip layer's PE tail is one ring round
    // per-ray rows staged once per tile: every tile within one ray
    const bool rows = (l0 && a.rb0) || a.rb_skip;
    if (rows && a.S % TM != 0) return false;
    if (save)
        for (int i = l0 ? 0 : 1; i < a.L; ++i)
            if (!a.Ds[i]) return false;
    return true;
}

template <int TM>
static void launch_trunk2(const TrunkArgs& ad, hipStream_t s, bool l0, bool save, int ntiles) {
    using Geo = T2Geo<TM>;
    const dim3 grid(std::min(ntiles, num_cus() * Geo::WGS)), block(Geo::NT);
    if (l0 && save) hipLaunchKernelGGL((k_trunk2_bf16<TM, true, true>), grid, block, 0, s, ad, ntiles);
    else if (l0) hipLaunchKernelGGL((k_trunk2_bf16<TM, true, false>), grid, block, 0, s, ad, ntiles);
    else if (save) hipLaunchKernelGGL((k_trunk2_bf16<TM, false, true>), grid, block, 0, s, ad, ntiles);
    else hipLaunchKernelGGL((k_trunk2_bf16<TM, false, false>), grid, block, 0, s, ad, ntiles);
}

int32_t trunk2_bf16(const TrunkArgs& a, hipStream_t s, bool save, double flop, double bytes) {
    const int TM = trunk2_tm(a);
    const int ntiles = cdiv(a.P, TM);
    TrunkArgs ad = a;
    if (ad.ldz == 0) ad.ldz = ad.S;  // contiguous z rows
    ad.dbg = g_trunk_dbg;
    ad.nt = save ? (g_trunk_nt & 1) : 0;
    const bool l0 = a.X0 || a.rays;
    if (!l0) ad.rb0 = nullptr;
    ProfScope prof(save ? "trunk_bf16_train" : "trunk_bf16", s, flop, bytes);
    if (TM == 64) launch_trunk2<64>(ad, s, l0, save, ntiles);
    else launch_trunk2<128>(ad, s, l0, save, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

// option trunk_heads: a bf16 inference forward runs the fused heads inside its trunk launch (H_L
// stays in LDS): 2 = in the one-workgroup k_trunk_bf16<128> (trunk_bf16.hip, the default), 1 = in
// the two-workgroup kernel here; 0 = the trunk, then k_heads_bf16
// (g_trunk_heads is defined at the top of the namespace)

bool trunk2_heads_ok(const TrunkArgs& a) {
    return g_trunk_heads == 1 && trunk2_tm(a) == 128 && trunk2_supported(a, false);
}

int32_t trunk2_heads_bf16(const TrunkArgs& a, const HeadsFusedArgs& h, const PackedOffs& k, hipStream_t s, double flop,
                          double bytes) {
    SPN_ARG(trunk2_heads_ok(a), "trunk2_heads_bf16: unsupported shape or option");
    SPN_ARG(h.P == a.P && h.S == a.S && h.NO <= hd::OST_LD && h.C <= 4 && k.Fnar16 >= 0, "trunk2_heads_bf16: bad heads");
    if (a.P == 0) return SPNERF_OK;
    const int ntiles = cdiv(a.P, 128);
    Trunk2HeadsArgs ad;
    static_cast<TrunkArgs&>(ad) = a;
    if (ad.ldz == 0) ad.ldz = ad.S;  // contiguous z rows
    ad.dbg = 0;
    ad.nt = 0;
    const bool l0 = a.X0 || a.rays;
    if (!l0) ad.rb0 = nullptr;
    ad.hg = h;
    ad.hg.nt = 0;
    ad.hg.dbg = 0;
    ad.hk = k;
    const dim3 grid(std::min(ntiles, num_cus())), block(T2Geo<128>::NT);
    ProfScope prof("trunk_heads_bf16", s, flop, bytes);
    if (l0) hipLaunchKernelGGL((k_trunk2_bf16<128, true, false, true>), grid, block, 0, s, ad, ntiles);
    else hipLaunchKernelGGL((k_trunk2_bf16<128, false, false, true>), grid, block, 0, s, ad, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

#else   // product build: the two-workgroup trunk is not compiled
bool trunk2_supported(const TrunkArgs&, bool) { return false; }
int32_t trunk2_bf16(const TrunkArgs&, hipStream_t, bool, double, double) {
    SPN_ARG(false, "trunk2_bf16: the two-workgroup trunk is an ablation-build kernel (-DSPN_ABLATIONS)");
    return SPNERF_OK;
}
bool trunk2_heads_ok(const TrunkArgs&) { return false; }
int32_t trunk2_heads_bf16(const TrunkArgs&, const HeadsFusedArgs&, const PackedOffs&, hipStream_t, double, double) {
    SPN_ARG(false, "trunk2_heads_bf16: the two-workgroup trunk is an ablation-build kernel (-DSPN_ABLATIONS)");
    return SPNERF_OK;
}
#endif  // SPN_ABLATIONS

}  // namespace spn

// resident workgroups per CU of the 64-point tiling (profiling aid: 2 expected; -1 in the product
// build, which does not compile that kernel)
extern "C" int32_t spnerf_debug_trunk2_occupancy(int32_t save) {
    int n = -1;
#ifndef SPN_ABLATIONS
    (void)save;
    return n;
#else
    const void* f = save ? (const void*)spn::k_trunk2_bf16<64, false, true, false> : (const void*)spn::k_trunk2_bf16<64, true, false, false>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, spn::T2Geo<64>::NT, 0) != hipSuccess) return -1;
    return n;
#endif
}
