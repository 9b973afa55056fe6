// Fused SIREN trunk of the bf16 MLP (cfg.dtype = 1, W = 512): fc_net layers 1 .. L-1
// (models/spnerf.py:201-209, 323-330) for a tile of TMt points per workgroup, with the
// activations resident in LDS from layer to layer — the persistent MFMA MLP kernel of DESIGN.md.
//
// Formulation: every layer computes Hᵀ_next = sin(W·Hᵀ + b) with the WEIGHTS as the MFMA A
// operand and the activation tile as B (v_mfma_f32_32x32x16_bf16).  A 32x32 accumulator then
// holds, per lane, 4 runs of 4 consecutive output features of ONE point: each run is an 8-byte
// piece of a row of the next layer's [point][feature] image, written with one ds_write_b64.
//  * LDS: the [TMt][512] bf16 activation image (16-B chunks XOR-swizzled by row & 15:
//    conflict-free ds_read_b128 B fragments and ds_write_b64 epilogue writes), when saving a
//    second image for D = cos, the [TMt][K0p] PE tile of the skip layer, two bias slots.
//  * Weights stream from L2 (every CU walks the same 512 KB per layer), packed by
//    spnerf_pack_params in MFMA fragment order (trunk_frag_off): wave w's A fragments of k-step
//    ks are one contiguous 2 KB, loaded TPD k-steps ahead into a register ring that runs on
//    from one layer's stream into the next one's (and into the next tile's first layer), so the
//    next layer's first k-steps are in flight through the epilogue.
//  * 8 waves; wave w owns output features [64w, 64w + 64) of all TMt points (2 x TMt/32 tiles).
//  * Epilogue = the unfused k_gemm_nt_bf16 arithmetic (fp32 accumulator + bias (+ the per-ray
//    semantic rows at the skip layer), fast_sincos, bf16 rounding) over the same k-order, so the
//    outputs equal the layer-by-layer path's bit for bit.
//  * Outputs leave through the images: a wave writes its 8-byte pieces to LDS, and whole 1-KB
//    rows are copied to HBM (one row per store instruction; scattered 8-byte stores straight
//    from the accumulator layout cost ~2x the whole layer) behind the NEXT layer's MFMAs, which
//    read the same image.
// Two tilings:
//  * TMt = 128 (inference: nothing saved but the last layer's H): 148 KB of LDS, 4 B fragments
//    per weight fragment (32 B/clk/CU of L2 weight traffic at the MFMA peak);
//  * TMt = 64 (training: H_i and D_i of every layer saved for the backward): the H and D images
//    (64 KB each) both drain behind the next layer's k-loop, instead of D leaving between two
//    barriers; twice the weight traffic per point.
#include <algorithm>
#include <type_traits>

#include "heads_tile.h"
#include "trunk.h"

#ifndef SPN_BIAS_HOIST
#define SPN_BIAS_HOIST 1  // register-D epilogue: the biases of a feature tile read once for both point tiles
#endif
#ifndef SPN_TRUNK_EPI_PK
#define SPN_TRUNK_EPI_PK 1  // the 128-point epilogue's bias adds as packed pairs (0: scalar, A/B builds)
#endif
#ifndef SPN_TRUNK_DCOLS
#define SPN_TRUNK_DCOLS 1  // saving 128-point tiles: each wave copies out its own D columns (0: between barriers)
#endif
#ifndef SPN_TRUNK_BUFSTORE
#define SPN_TRUNK_BUFSTORE 1  // copy-outs through buffer descriptors (0: guarded stores, A/B builds)
#endif

namespace spn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

int g_fused_trunk = 1;
int g_trunk_tile = 0;  // 0 = 128 (64 when saving Z, zsave); 64 / 128 force a tiling (A/B runs)
// bit 1: the training trunk's H copy-outs non-temporal (glc slc), the default: C4@512 4.41 -> 4.30 and
// 4.18 / 4.20 -> 4.09 / 4.09 ms, C4 26.63 / 26.64 -> 26.60 / 26.57, C3 7.36 -> 7.26, C5 level (pairs in
// one call each, tools/gpu_r3u.sh, tools/gpu_r3v.sh); bit 4: the register-D
// stores too (slower); bit 2: the fused heads' H loads
int g_trunk_nt = 1;
int g_trunk_var = 0;  // profiling ablations of the 128-point tiling (k_trunk_bf16 VAR)
int g_trunk_dreg = 1;  // 64-point training tiles: D = cos leaves from the accumulators in the epilogue
                       // (VAR 512) instead of through the D image behind the next k-loop.  The same
                       // epilogue on 128-point training tiles (no D image needed: 148 KB of LDS)
                       // measured 3.65 ms per 524 288 points against 2.96 (64) and 3.13 (128 with the
                       // two-barrier cos pass): 128 KB of D stores per epilogue hold up the refills
int g_trunk_dbg = 0;   // profiling ablations, outputs invalid when set: 1 = skip the HBM copy-outs
                       // (4 = only the register-D stores, 8 = only the H copy-outs in the k-loop),
                       // (options trunk_var 16 / 32: no MFMAs in the main k-loop / no sine in the
                       // inference epilogue)

constexpr int TW = 512;  // trunk width of the fused kernel

template <int TMt>
struct TrunkGeo {
    static constexpr int NJ = TMt / 32;                        // point tiles per wave
    static constexpr bool DIMG = TMt == 64;                    // a D image beside the H image
    static constexpr int TPD = TMt == 64 ? 8 : 4;              // weight prefetch depth (k-steps)
    static constexpr int IMG = TMt * TW * 2;                   // one [TMt][512] bf16 image
    static constexpr int X0_OFF = IMG * (DIMG ? 2 : 1);
    static constexpr int BIAS_OFF = X0_OFF + TMt * 64 * 2;     // K0p <= 64
    static constexpr int LDS = BIAS_OFF + 2 * TW * 4;
    static constexpr int CPT = TMt * 64 / 512;                 // 16-B chunks of an image per thread
    // the per-ray rows of a layer with them (layer 0, the skip layer) for the tile's first SRB_RAYS
    // rays, staged by LDS-DMA at the layer's top (kernels without the fused heads: after LDS)
    static constexpr int SRB_RAYS = 4;
    static constexpr int SRB_BYTES = SRB_RAYS * TW * 4;
};

__device__ __forceinline__ int act_off(int row, int ch) { return row * 1024 + ((ch ^ (row & 15)) << 4); }
// PE rows are 8 chunks (128 B): XOR with (row >> 1) & 7 keeps the 16 rows of a ds_read_b128
// lane group on distinct 16-B slots of the bank row
__device__ __forceinline__ int x0_rel(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

// VAR (TMt = 128 only): 0 = the kernel; profiling ablations (outputs invalid; option trunk_var),
// bits: 16 = no MFMAs in the main k-loop, 32 = no sine in the epilogue, 64 = no weight refills
// in the k-loop, 128 = no image (B) reads in the k-loop, 256 = no epilogue (464: all of them)
// HEADS (VAR 4096; inference, TMt = 128, option trunk_heads 2): the fused heads (heads_tile.h) run
// on the last layer's LDS image, so H_L never leaves the chip; their output staging is 8 KB beyond
// the trunk's LDS, their partials overlay the PE tile (restaged by the next tile), and the weight
// ring is primed per tile instead of running on through the heads.  The heads' arguments are read
// per tile through an opaque kernarg pointer (not hoisted into registers live through the layers).
template <int TMt, int VAR = 0>
__global__ __launch_bounds__(512) void k_trunk_bf16(std::conditional_t<(VAR & 4096) != 0, TrunkHeadsArgs, TrunkArgs> g,
                                                    int ntiles) {
    using Geo = TrunkGeo<TMt>;
    constexpr int NJ = Geo::NJ, IMG = Geo::IMG, CPT = Geo::CPT;
    constexpr int TPD = Geo::TPD;
    constexpr bool HEADS = (VAR & 4096) != 0;
    static_assert(!HEADS || (TMt == 128 && Geo::BIAS_OFF - Geo::X0_OFF >= hd::PART_BYTES &&
                             Geo::LDS + hd::OST_BYTES <= 160 * 1024), "the fused heads: 128-point tiles, LDS");
    constexpr bool NOMF = VAR & 16, NOSIN = VAR & 32, NOW = VAR & 64, NOB = VAR & 128, NOEPI = VAR & 256;
    constexpr bool NOPE = VAR & 8192;  // ablation (outputs invalid): the inline encoding's math skipped
    constexpr bool DREG = Geo::DIMG && (VAR & 512);  // D from the registers (see epilogue_dreg)
    // (VAR 2048: the saving launches of the 128-point tiling as their own instance — the same code,
    // so rocprof tells the training launches from the inference ones by name)
    static_assert(!(VAR & 2048) || TMt == 128, "the 128-point training instance");
    constexpr bool SRB = !HEADS;  // per-ray rows staged in LDS (the fused heads' kernel has no room)
    constexpr bool SAVING = (VAR & 2048) != 0;  // the 128-point training instance (every layer saved)
    __shared__ __attribute__((aligned(16))) char smem[Geo::LDS + (HEADS ? hd::OST_BYTES : Geo::SRB_BYTES)];
    float* srb = reinterpret_cast<float*>(smem + Geo::LDS);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, h = lane >> 5;
    // product: the H copy-outs non-temporal (g_trunk_nt's default, bit 1; the fused-heads launch
    // copies nothing out and passes 0), the register-D stores not (bit 2)
    constexpr int kNtDefault = (VAR & 4096) ? 0 : 1;
    const int gnt = kTrunkAbl ? g.nt : kNtDefault;
    const int gdbg = kTrunkAbl ? g.dbg : 0;
    float* sbias = reinterpret_cast<float*>(smem + Geo::BIAS_OFF);
    char* sx0 = smem + Geo::X0_OFF;
    const int x0ch = g.K0p >> 3;
    constexpr int nmain = TW / 16;  // k-steps over the activation image
    const int ntail = g.K0p >> 4;   // extra k-steps over the PE at the skip layer
    const bool l0 = g.X0 != nullptr || g.rays != nullptr;  // layer 0 in this launch (block-uniform)
    const int first = l0 ? 0 : 1;
    const int nk0 = g.K0p >> 2;     // layer 0's k-steps: the 4·K0p split planes
    auto nks_of = [&](int i) { return i == 0 ? nk0 : nmain + (i == g.skip ? ntail : 0); };
    const int sw = r32 & 15;
    // per-layer pointers indexed by the (runtime) layer: scalar loads straight from the kernarg
    // segment (indexing the by-value struct copies its arrays to scratch)
    typedef const __attribute__((address_space(4))) TrunkArgs* KArgs;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();

    u32x4 ring[TPD][2];
    // wave w's fragment stream of layer i: k-step ks at + ks * kTrunkKStride, feature tile a at + 512 * a
    auto wstream = [&](int i) { return ka->Wf[i] + trunk_wave_off(w, nks_of(i)) + lane * 8; };
    // slots [d0, d1) of layer i's first k-steps
    auto prime = [&](int i, auto kd0, auto kd1) {
        constexpr int d0 = decltype(kd0)::value, d1 = decltype(kd1)::value;
        const bf16* src = wstream(i);
#pragma unroll
        for (int d = d0; d < d1; ++d) {
            ring[d][0] = ldg16(src + d * kTrunkKStride);
            ring[d][1] = ldg16(src + d * kTrunkKStride + 512);
        }
    };
    // copy chunks [q0, q0 + n) (per thread) of an image to HBM rows p0 + row.  The stores go
    // through a buffer descriptor over the tile's valid rows (rows past P are dropped by the
    // hardware): a branch around them made every later wait on an older load (the weight ring's
    // refills) hipcc's conservative count, i.e. a wait for these stores as well
    auto copy_out = [&](const char* img, bf16* dst, int64_t p0, int q0, auto kn) {
        constexpr int n = decltype(kn)::value;
        const int ct = opaque(tid);
        const int rows = (int)std::min<int64_t>(TMt, g.P - p0);
        // (dst nullptr: an empty resource, every store dropped — no branch around the stores)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + p0 * TW, 0, dst ? rows * TW * 2 : 0, 0x00020000);
        u32x4 v[n];
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int c = ct + 512 * (q0 + q);
            v[q] = *reinterpret_cast<const u32x4*>(img + act_off(c >> 6, c & 63));
        }
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int c = ct + 512 * (q0 + q);
#if SPN_TRUNK_BUFSTORE
            const int off = ((c >> 6) * TW + (c & 63) * 8) * 2;
            if (gnt & 1) __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 3);  // block-uniform: glc slc
            else __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 0);
#else  // A/B build: the guarded stores
            if (p0 + (c >> 6) < g.P) {
                u32x4* o = reinterpret_cast<u32x4*>(dst + (p0 + (c >> 6)) * TW + (c & 63) * 8);
                if (gnt & 1) __builtin_nontemporal_store(v[q], o);
                else *o = v[q];
            }
#endif
        }
    };

    // a whole image, 4 chunks per thread at a time (the accumulators may still be live)
    auto copy_all = [&](const char* img, bf16* dst, int64_t p0) {
        if (gdbg & 1) return;
#pragma unroll
        for (int q0 = 0; q0 < CPT; q0 += 4) copy_out(img, dst, p0, q0, std::integral_constant<int, 4>{});
    };

    // wave w's own feature columns [64w, 64w + 64) of the image (the chunks its epilogue wrote) to
    // HBM rows p0 + row: lane l takes chunk 8w + (l & 7) of rows 8q + (l >> 3), so 8 lanes store
    // one row's whole 128-B line; 4 chunks per lane at a time (the accumulators are still live)
    auto copy_cols = [&](bf16* dst, int64_t p0) {
        if (gdbg & 1) return;
        const int l = opaque(lane);
        const int rows = (int)std::min<int64_t>(TMt, g.P - p0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + p0 * TW, 0, rows * TW * 2, 0x00020000);
        const int ch = 8 * w + (l & 7), r0 = l >> 3;
        asm volatile("" ::: "memory");  // the epilogue's image writes (other lanes' chunks) stay before
#pragma unroll
        for (int q0 = 0; q0 < TMt / 8; q0 += 4) {
            u32x4 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = *reinterpret_cast<const u32x4*>(smem + act_off(8 * (q0 + q) + r0, ch));
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int off = ((8 * (q0 + q) + r0) * TW + ch * 8) * 2;
                if (gnt & 1) __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 3);  // block-uniform: glc slc
                else __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 0);
            }
        }
        asm volatile("" ::: "memory");  // ... and the next pass's writes after
    };

    // σ pre-activation of the tile's points from the last layer's image (TrunkArgs::sig_hsave):
    // wave w takes rows [TMt/8 · w, +TMt/8); lane l the features 4l.. and 256 + 4l.. — the lane
    // layout, dot4 order and wave_total of k_heads_fwd_v, so hsave[p·8] is bit-identical to it
    auto sigma_rows = [&](int64_t p0) {
        const int l = opaque(lane);
        const f32x4 w0v = ld4(g.wsig + 4 * l), w1v = ld4(g.wsig + 256 + 4 * l);
        const float bs = *g.bsig;
#pragma unroll 1
        for (int r = 0; r < TMt / 8; ++r) {
            const int row = (TMt / 8) * w + r;
            const u32x2 h0 = *reinterpret_cast<const u32x2*>(smem + act_off(row, l >> 1) + 8 * (l & 1));
            const u32x2 h1 = *reinterpret_cast<const u32x2*>(smem + act_off(row, 32 + (l >> 1)) + 8 * (l & 1));
            float ps = 0.f;
            ps += dot4(raw_f32(h0), w0v);
            ps += dot4(raw_f32(h1), w1v);
            const float spre = wave_total(ps) + bs;
            if (l == 0 && p0 + row < g.P) g.sig_hsave[(p0 + row) * 8] = spre;
        }
    };

    int tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;  // block-uniform
    if constexpr (!HEADS) prime(first, std::integral_constant<int, 0>{}, std::integral_constant<int, TPD>{});
    // the next layer's bias, loaded behind a layer's k-loop (before its epilogue's stores, so the
    // wait for it at the next layer's top does not wait for those stores as well)
    float bpre = ka->bias[first][tid];
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TMt;
        const int st = opaque(tid);
        // (HEADS) the first layer's stream, in flight through the tile's staging
        if constexpr (HEADS) prime(first, std::integral_constant<int, 0>{}, std::integral_constant<int, TPD>{});
        // stage the first layer's input and the PE tile; rows past P read a clamped row (their
        // outputs are never stored)
        if (l0) {
            // 8 fp32 PE values per unit → 16-B hi and lo chunks: image columns [hi | lo | hi | lo]
            // (layer 0's B operand) and the skip layer's PE tile (= hi, as X0b)
            for (int u = st; u < TMt * x0ch; u += 512) {
                const int row = u / x0ch, q = u % x0ch;
                const int64_t pr = std::min<int64_t>(p0 + row, g.P - 1);
                float xv[8];
                if (g.rays) {  // block-uniform: encode o + dir·z here (pe_value, as k_encode)
                    const int rr = (int)pr / g.S;
                    const float* ray = g.rays + (int64_t)rr * g.rs;
                    const float zz = g.z[(int64_t)rr * g.ldz + ((int)pr - rr * g.S)];
#pragma unroll
                    for (int e = 0; e < 8; ++e) xv[e] = NOPE ? ray[e & 3] * zz : pe_value(ray, g.dir_off, zz, q * 8 + e, g.n_freq, g.K0);
                } else {
                    const float* src = g.X0 + pr * g.K0p + q * 8;
                    const f32x4 v0 = ld4(src), v1 = ld4(src + 4);
#pragma unroll
                    for (int e = 0; e < 8; ++e) xv[e] = e < 4 ? v0[e] : v1[e - 4];
                }
                float hf[8], lf[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float x = xv[e];
                    hf[e] = (float)(bf16)x;
                    lf[e] = x - hf[e];
                }
                const u32x4 hi = {pack2(hf[0], hf[1]), pack2(hf[2], hf[3]), pack2(hf[4], hf[5]), pack2(hf[6], hf[7])};
                const u32x4 lo = {pack2(lf[0], lf[1]), pack2(lf[2], lf[3]), pack2(lf[4], lf[5]), pack2(lf[6], lf[7])};
                *reinterpret_cast<u32x4*>(smem + act_off(row, q)) = hi;
                *reinterpret_cast<u32x4*>(smem + act_off(row, x0ch + q)) = lo;
                *reinterpret_cast<u32x4*>(smem + act_off(row, 2 * x0ch + q)) = hi;
                *reinterpret_cast<u32x4*>(smem + act_off(row, 3 * x0ch + q)) = lo;
                if (g.skip > 0) *reinterpret_cast<u32x4*>(sx0 + x0_rel(row, q)) = hi;
                // training, inline encoding: the bf16 PE row for the weight gradients (= X0b)
                if (g.X0b_out && p0 + row < g.P) *reinterpret_cast<u32x4*>(g.X0b_out + (p0 + row) * g.K0p + q * 8) = hi;
            }
        } else {
#pragma unroll
        for (int q0 = 0; q0 < CPT; q0 += 8) {
            u32x4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = st + 512 * (q0 + q), row = c >> 6, ch = c & 63;
                v[q] = ldg16(g.H1 + std::min<int64_t>(p0 + row, g.P - 1) * TW + ch * 8);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = st + 512 * (q0 + q), row = c >> 6, ch = c & 63;
                *reinterpret_cast<u32x4*>(smem + act_off(row, ch)) = v[q];
            }
        }
        if (g.skip > 0) {
            for (int c = st; c < TMt * x0ch; c += 512) {
                const int row = c / x0ch, ch = c % x0ch;
                *reinterpret_cast<u32x4*>(sx0 + x0_rel(row, ch)) =
                    ldg16(g.X0b + std::min<int64_t>(p0 + row, g.P - 1) * g.K0p + ch * 8);
            }
        }
        }

        bf16* hpend = nullptr;  // H (and D) of the previous layer: copied out during this k-loop
        bf16* dpend = nullptr;
        for (int i = first; i < g.L; ++i) {
            const bool skip = i == g.skip;
            const bf16* wsrc = wstream(i);
            const int nks = nks_of(i);
            // the ring runs on into the next layer's (or the next tile's first layer's) stream:
            // once slot d has served this layer's last k-step in it, it loads the next layer's
            // k-step d (past the last tile: this layer's step d again, unused).  Priming after the
            // k-loop instead reloaded registers whose refills were still in flight, and hipcc
            // drained vmcnt(0) — every refill and H / D copy-out store — before each epilogue
            const bool last = i == g.L - 1;
            const int inext = last ? (!HEADS && tile + (int)gridDim.x < ntiles ? first : -1) : i + 1;
            const bf16* wnxt = inext >= 0 ? wstream(inext) : wsrc;
            const int nkm = i == 0 ? nk0 : nmain;  // k-steps over the image
            float* sb = sbias + (i & 1) * TW;  // slot (i-1)&1 may still be read by the previous epilogue
            sb[tid] = bpre;
            // this layer's per-ray rows (block-uniform): into LDS by DMA now, the oldest loads of
            // the layer, so the k-loop's refill waits cover them and the epilogue reads LDS (a
            // global load there was waited for with everything in flight: refills and copy-outs)
            const float* rbl = i == 0 ? g.rb0 : (i == g.skip ? g.rb_skip : nullptr);
            const int ray0 = (int)p0 / g.S, rayl = (int)(std::min<int64_t>(p0 + TMt, g.P) - 1) / g.S;
            const bool srb_on = SRB && rbl && rayl - ray0 < Geo::SRB_RAYS;
            if (srb_on) {
                typedef __attribute__((address_space(3))) void* lds_ptr_t;
                typedef __attribute__((address_space(1))) void* gbl_ptr_t;
                // wave w: row w / 2, floats 256·(w % 2) .. +255, 16 B per lane
                const int rr = w >> 1;
                const float* src = rbl + (int64_t)std::min(ray0 + rr, rayl) * TW + 256 * (w & 1) + 4 * opaque(lane);
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)(srb + rr * TW + 256 * (w & 1)), 16, 0, 0);
            }
            f32x16 acc[2][NJ];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
            __syncthreads();  // the image (and the bias slot) of layer i are complete

            // B fragments are double-buffered: step ks+1's image reads are issued between step
            // ks's MFMAs (past the image's last step the read lands in the next LDS region: in
            // bounds, unused)
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
                    for (int j = 0; j < NJ; ++j) bn[j] = NOB ? bc[j] : *reinterpret_cast<const bf16x8*>(brow + j * 32768 + offn);
                    const bf16x8 a0 = __builtin_bit_cast(bf16x8, ring[d][0]);
                    const bf16x8 a1 = __builtin_bit_cast(bf16x8, ring[d][1]);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        if constexpr (NOMF) {  // ablation: no MFMAs (keep the operands live)
                            acc[0][j][0] += __builtin_bit_cast(float, a0[0] != bc[j][0] ? 1 : 0);
                            acc[1][j][0] += __builtin_bit_cast(float, a1[0] != bc[j][0] ? 1 : 0);
                            continue;
                        }
                        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bc[j], acc[0][j], 0, 0, 0);
                        acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bc[j], acc[1][j], 0, 0, 0);
                    }
                    // refill the slot just consumed, right behind its MFMAs (TPD - 1 steps of
                    // cover); past the stream's end: re-read its last step
                    if constexpr (!NOW) {
                        const bf16* src = ks + TPD < nks ? wsrc + (ks + TPD) * kTrunkKStride : wnxt + d * kTrunkKStride;
                        ring[d][0] = ldg16(src);
                        ring[d][1] = ldg16(src + 512);
                    }
                    // order: (1 image read, 2 MFMAs) x NJ, then the 2 weight loads
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) bc[j] = bn[j];
                }
                // drain the previous layer's outputs: CPT / (nmain / TPD) chunks per thread
                constexpr int per = CPT / (nmain / TPD);
                static_assert(per * (nmain / TPD) == CPT && per >= 1, "copy slices");
#if SPN_TRUNK_BUFSTORE
                if constexpr (SAVING) {
                    // (hpend nullptr on a tile's first layer: an empty resource, no branch around the
                    // stores).  Only the saving instance: elsewhere hpend is null on every layer and
                    // the branch skips the copy entirely (inference: no LDS reads, no dropped stores)
                    copy_out(smem, (gdbg & 9) ? nullptr : hpend, p0, (ks0 / TPD) * per, std::integral_constant<int, per>{});
                } else {
                    if (hpend && !(gdbg & 9)) copy_out(smem, hpend, p0, (ks0 / TPD) * per, std::integral_constant<int, per>{});
                    if (Geo::DIMG && dpend && !(gdbg & 1)) copy_out(smem + IMG, dpend, p0, (ks0 / TPD) * per, std::integral_constant<int, per>{});
                }
#else
                if (hpend && !(gdbg & 9)) copy_out(smem, hpend, p0, (ks0 / TPD) * per, std::integral_constant<int, per>{});
                if (Geo::DIMG && dpend && !(gdbg & 1)) copy_out(smem + IMG, dpend, p0, (ks0 / TPD) * per, std::integral_constant<int, per>{});
#endif
            }
            // the x0 columns of the skip layer's input [h | x0] (nks == nmain elsewhere)
#pragma unroll 1
            for (int ks0 = nmain; ks0 < nks; ks0 += TPD) {
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    const int ks = ks0 + d;
                    if (ks < nks) {  // block-uniform
                        bf16x8 b[NJ];
#pragma unroll
                        for (int j = 0; j < NJ; ++j)
                            b[j] = *reinterpret_cast<const bf16x8*>(sx0 + x0_rel(32 * j + r32, 2 * (ks - nmain) + h));
                        const bf16x8 a0 = __builtin_bit_cast(bf16x8, ring[d][0]);
                        const bf16x8 a1 = __builtin_bit_cast(bf16x8, ring[d][1]);
#pragma unroll
                        for (int j = 0; j < NJ; ++j) {
                            acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[j], acc[0][j], 0, 0, 0);
                            acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[j], acc[1][j], 0, 0, 0);
                        }
                        ring[d][0] = ldg16(wnxt + d * kTrunkKStride);  // ks + TPD >= nks here
                        ring[d][1] = ldg16(wnxt + d * kTrunkKStride + 512);
                    }
                }
            }

            bpre = ka->bias[inext >= 0 ? inext : first][tid];
            __syncthreads();  // every wave is done reading the images of layer i
            bf16* Hs = ka->Hs[i];
            bf16* Ds = ka->Ds[i];
            const float* rb = i == 0 ? g.rb0 : (skip ? g.rb_skip : nullptr);
            // block-uniform: Z = fp16(v), the D slot gets Z (saving tiles only: the host keeps
            // zround off the 128-point tiling)
            const bool zr = Geo::DIMG && g.zround && i >= 1;
            // kpass 0: cos (or Z) into the image (TMt = 128 when saving: it leaves between two
            // barriers); 1: sin into the image; 2: sin into the image and cos (or Z) into the D image
            // kl0: layer 0 (SIREN w0 = 30 of fc_net.0; ×1 elsewhere, exact, so not multiplied)
            auto epilogue = [&](auto kpass, auto kl0, auto krb, auto klds) {
                if constexpr (NOEPI) {  // keep the accumulators (and so the MFMAs) live
                    float t = 0.f;
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int j = 0; j < NJ; ++j) t += acc[a][j][0];
                    if (t == 1234.5f) *reinterpret_cast<float*>(smem + 4 * tid) = t;
                    return;
                }
                constexpr int pass = decltype(kpass)::value;
                constexpr float w0 = decltype(kl0)::value ? 30.f : 1.f;
                constexpr bool RB = decltype(krb)::value;  // per-ray rows (layer 0, the skip layer)
                constexpr bool RBL = decltype(klds)::value;  // ... staged in LDS (srb)
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                        const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + f0);
#pragma unroll
                        for (int j = 0; j < NJ; ++j) {
                            const int row = 32 * j + er32;
                            float v[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * gq + e] + bv[e];
                            if constexpr (RB) {
                                const int ray = (int)std::min<int64_t>(p0 + row, g.P - 1) / g.S;  // P < 2^31 / 512
                                const f32x4 rv = RBL ? *reinterpret_cast<const f32x4*>(srb + (ray - ray0) * TW + f0)
                                                     : ld4(rb + (int64_t)ray * TW + f0);
#pragma unroll
                                for (int e = 0; e < 4; ++e) v[e] += rv[e];
                            }
                            const int o = act_off(row, f0 >> 3) + 8 * eh;
                            float y[4], c[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const float z = zr ? zr16(v[e]) : v[e];
                                const float x = w0 == 1.f ? z : w0 * z;
                                if (pass == 2) {
                                    fast_sincos(x, &y[e], &c[e]);
                                    c[e] = zr ? z : (w0 == 1.f ? c[e] : w0 * c[e]);
                                } else if (pass == 1) {
                                    y[e] = NOSIN ? x : fast_sin(x);
                                } else {
                                    y[e] = zr ? z : (w0 == 1.f ? fast_cos(x) : w0 * fast_cos(x));
                                }
                            }
                            // Z (zr: into the D image, or into the image by pass 0) is stored as fp16
                            if (pass == 0 && zr)
                                *reinterpret_cast<u32x2*>(smem + o) = u32x2{pack2_f16(y[0], y[1]), pack2_f16(y[2], y[3])};
                            else
                                *reinterpret_cast<u32x2*>(smem + o) = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                            if (pass == 2) {
                                if (zr) *reinterpret_cast<u32x2*>(smem + IMG + o) = u32x2{pack2_f16(c[0], c[1]), pack2_f16(c[2], c[3])};
                                else *reinterpret_cast<u32x2*>(smem + IMG + o) = u32x2{pack2(c[0], c[1]), pack2(c[2], c[3])};
                            }
                        }
                        __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted loads
                    }
            };
            // The saving 128-point instance: the element arithmetic r = (acc + b [+ row]) [· w0] · 1/2π runs per
            // pair (the bias adds as v_pk_add_f32; the same roundings per element as fast_sin /
            // fast_cos: bit-identical).  (Handing r from the cos pass to the sin pass through the
            // accumulators would save that pass's add / mul, but made the saving kernel spill.)
            auto epilogue_pk = [&](auto kpass, auto kl0, auto krb, auto klds) {
                if constexpr (NOEPI) {  // keep the accumulators (and so the MFMAs) live
                    float t = 0.f;
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int j = 0; j < NJ; ++j) t += acc[a][j][0];
                    if (t == 1234.5f) *reinterpret_cast<float*>(smem + 4 * tid) = t;
                    return;
                }
                constexpr int pass = decltype(kpass)::value;
                constexpr float w0 = decltype(kl0)::value ? 30.f : 1.f;
                constexpr bool RB = decltype(krb)::value;  // per-ray rows (layer 0, the skip layer)
                constexpr bool RBL = decltype(klds)::value;  // ... staged in LDS (srb)
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                        const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + f0);
#pragma unroll
                        for (int j = 0; j < NJ; ++j) {
                            const int row = 32 * j + er32;
                            const int o = act_off(row, f0 >> 3) + 8 * eh;
                            float y[4], c[4];
                            f32x4 rv = f32x4{0.f, 0.f, 0.f, 0.f};
                            if constexpr (RB) {
                                const int ray = (int)std::min<int64_t>(p0 + row, g.P - 1) / g.S;  // P < 2^31 / 512
                                rv = RBL ? *reinterpret_cast<const f32x4*>(srb + (ray - ray0) * TW + f0)
                                         : ld4(rb + (int64_t)ray * TW + f0);
                            }
                            // one pair at a time (fewer live temporaries)
#pragma unroll
                            for (int q = 0; q < 2; ++q) {
                                const int e = 2 * q;
                                f32x2 r2;
                                {
#if SPN_TRUNK_EPI_PK
                                    f32x2 v2 = f32x2{acc[a][j][4 * gq + e], acc[a][j][4 * gq + e + 1]} + f32x2{bv[e], bv[e + 1]};
                                    if constexpr (RB) v2 += f32x2{rv[e], rv[e + 1]};
                                    const f32x2 x2 = w0 == 1.f ? v2 : v2 * f32x2{w0, w0};
                                    r2 = x2 * f32x2{0.15915494309189535f, 0.15915494309189535f};
#else
#pragma unroll
                                    for (int u = 0; u < 2; ++u) {
                                        float v = acc[a][j][4 * gq + e + u] + bv[e + u];
                                        if constexpr (RB) v += rv[e + u];
                                        r2[u] = revs(w0 == 1.f ? v : w0 * v);
                                    }
#endif
                                }
#pragma unroll
                                for (int u = 0; u < 2; ++u) {
                                    if (pass == 2) {
                                        y[e + u] = __builtin_amdgcn_sinf(r2[u]);
                                        c[e + u] = w0 == 1.f ? __builtin_amdgcn_cosf(r2[u]) : w0 * __builtin_amdgcn_cosf(r2[u]);
                                    } else if (pass == 1) {
                                        y[e + u] = NOSIN ? r2[u] : __builtin_amdgcn_sinf(r2[u]);
                                    } else {
                                        y[e + u] = w0 == 1.f ? __builtin_amdgcn_cosf(r2[u]) : w0 * __builtin_amdgcn_cosf(r2[u]);
                                    }
                                }
                            }
                            // Z (zr: into the D image, or into the image by pass 0) is stored as fp16
                            if (pass == 0 && zr)
                                *reinterpret_cast<u32x2*>(smem + o) = u32x2{pack2_f16(y[0], y[1]), pack2_f16(y[2], y[3])};
                            else
                                *reinterpret_cast<u32x2*>(smem + o) = u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                            if (pass == 2) {
                                if (zr) *reinterpret_cast<u32x2*>(smem + IMG + o) = u32x2{pack2_f16(c[0], c[1]), pack2_f16(c[2], c[3])};
                                else *reinterpret_cast<u32x2*>(smem + IMG + o) = u32x2{pack2(c[0], c[1]), pack2(c[2], c[3])};
                            }
                        }
                        __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted loads
                    }
            };
            // block-uniform choices of compile-time instances: a load behind a runtime branch would
            // be waited for with vmcnt(0) — every refill and copy-out store in flight
            auto epi = [&](auto kpass) {
                const std::false_type F{};
                const std::true_type T{};
                auto ep = [&](auto l0, auto rbk, auto lds) {
                    if constexpr (SAVING) epilogue_pk(kpass, l0, rbk, lds);
                    else epilogue(kpass, l0, rbk, lds);
                };
                if (i == 0) {
                    if (rb && srb_on) ep(T, T, T);
                    else if (rb) ep(T, T, F);
                    else ep(T, F, F);
                } else if (rb && srb_on) {
                    ep(F, T, T);
                } else if (rb) {
                    ep(F, T, F);
                } else {
                    ep(F, F, F);
                }
            };
            // DREG: sin → the image as above, D = cos (×w0 at layer 0) straight from the registers
            // to HBM during the epilogue — the 8-byte pieces of feature groups (0, 1) and (2, 3) of
            // a row joined by v_permlane32_swap into one 16-B buffer store per lane (the store of
            // k_trunk2_bf16).  The k-loop then drains only H, and D's HBM writes run while the
            // epilogue's VALU work does (HBM was idle through every epilogue); layers with per-ray
            // rows (whose loads would wait behind the stores) or a saved Z keep the D image.
            auto epilogue_dreg = [&](auto kl0) {
                if constexpr (NOEPI) {  // ablation: keep the accumulators (and so the MFMAs) live
                    float t = 0.f;
#pragma unroll
                    for (int a = 0; a < 2; ++a)
#pragma unroll
                        for (int j = 0; j < NJ; ++j) t += acc[a][j][0];
                    if (t == 1234.5f) *reinterpret_cast<float*>(smem + 4 * tid) = t;
                    return;
                }
                constexpr float w0 = decltype(kl0)::value ? 30.f : 1.f;
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
                const int rows = (int)std::min<int64_t>(TMt, g.P - p0);
                // (dbg 1, no copy-outs: an empty range drops every store — no branch around them)
                const __amdgpu_buffer_rsrc_t dr =
                    __builtin_amdgcn_make_buffer_rsrc(Ds + p0 * TW, 0, (gdbg & 5) ? 0 : rows * TW * 2, 0x00020000);
                // act_off(32j + er32, 8w + 4a + gq) + 8eh without per-piece index math: the row's
                // swizzle (row & 15 = er32 & 15) only touches the chunk's low 4 bits
                char* lbase = smem + er32 * 1024 + 256 * (w >> 1) + 8 * eh;
                const int sw4 = er32 & 15, c8 = 8 * (w & 1);
#pragma unroll
                for (int a = 0; a < 2; ++a) {
#if SPN_BIAS_HOIST
                    // this feature tile's biases once for both point tiles (one LDS read per group)
                    f32x4 bva[4];
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) bva[gq] = *reinterpret_cast<const f32x4*>(sb + 64 * w + 32 * a + 8 * gq + 4 * eh);
#endif
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        u32x2 cq[4];
#pragma unroll
                        for (int gq = 0; gq < 4; ++gq) {
#if SPN_BIAS_HOIST
                            const f32x4 bv = bva[gq];
#else
                            const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + 64 * w + 32 * a + 8 * gq + 4 * eh);
#endif
                            float y[4], c[4];
                            if constexpr (w0 == 1.f && SPN_PK_EPI) {
                                // (acc + b) · 1/2π as packed pairs: the same two roundings per
                                // element as fast_sincos's, half the VALU issue slots
#pragma unroll
                                for (int e = 0; e < 4; e += 2) {
                                    const f32x2 v2 = f32x2{acc[a][j][4 * gq + e], acc[a][j][4 * gq + e + 1]} + f32x2{bv[e], bv[e + 1]};
                                    const f32x2 r2 = v2 * f32x2{0.15915494309189535f, 0.15915494309189535f};
                                    if constexpr (NOSIN) {  // ablation (outputs invalid): no transcendentals
                                        y[e] = r2[0]; y[e + 1] = r2[1]; c[e] = -r2[0]; c[e + 1] = -r2[1];
                                    } else {
                                        y[e] = __builtin_amdgcn_sinf(r2[0]);
                                        y[e + 1] = __builtin_amdgcn_sinf(r2[1]);
                                        c[e] = __builtin_amdgcn_cosf(r2[0]);
                                        c[e + 1] = __builtin_amdgcn_cosf(r2[1]);
                                    }
                                }
                            } else {
#pragma unroll
                                for (int e = 0; e < 4; ++e) {
                                    const float v = acc[a][j][4 * gq + e] + bv[e];
                                    fast_sincos(w0 * v, &y[e], &c[e]);
                                    c[e] = w0 * c[e];
                                }
                            }
                            *reinterpret_cast<u32x2*>(lbase + j * 32768 + (((c8 + 4 * a + gq) ^ sw4) << 4)) =
                                u32x2{pack2(y[0], y[1]), pack2(y[2], y[3])};
                            cq[gq] = u32x2{pack2(c[0], c[1]), pack2(c[2], c[3])};
                        }
#pragma unroll
                        for (int k = 0; k < 4; k += 2) {
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                const auto r = __builtin_amdgcn_permlane32_swap(cq[k][e], cq[k + 1][e], false, false);
                                cq[k][e] = r[0];
                                cq[k + 1][e] = r[1];
                            }
                            // lanes 0..31: features 8k..8k+7 of the pair, lanes 32..63: 8k+8..8k+15
                            const int fb = 64 * w + 32 * a + 8 * k + 8 * eh;
                            // (option trunk_nt bit 4: glc slc — measured 3.50-3.57 against 2.92 ms per
                            // 524 288 points: without L2 write-combining the 32-B row pieces reach HBM
                            // as partial lines.  H non-temporal, bit 1: 2.88 against 2.92, not default)
                            if (gnt & 2)  // block-uniform
                                __builtin_amdgcn_raw_buffer_store_b128(u32x4{cq[k][0], cq[k][1], cq[k + 1][0], cq[k + 1][1]},
                                    dr, ((32 * j + er32) * TW + fb) * 2, 0, 3);
                            else
                                __builtin_amdgcn_raw_buffer_store_b128(u32x4{cq[k][0], cq[k][1], cq[k + 1][0], cq[k + 1][1]},
                                    dr, ((32 * j + er32) * TW + fb) * 2, 0, 0);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted loads
                }
            };
            if constexpr (Geo::DIMG) {
                const bool dreg = DREG && Ds && !rb && !zr;  // block-uniform
                if (dreg) {
                    if (i == 0) epilogue_dreg(std::true_type{});
                    else epilogue_dreg(std::false_type{});
                } else if (Ds) {
                    epi(std::integral_constant<int, 2>{});  // block-uniform
                } else {
                    epi(std::integral_constant<int, 1>{});
                }
                if (last) {
                    __syncthreads();
                    copy_all(smem, Hs, p0);
                    if (Ds && !dreg) copy_all(smem + IMG, Ds, p0);
                    if (g.sig_hsave) sigma_rows(p0);  // block-uniform
                }
                hpend = last ? nullptr : Hs;
                dpend = last || dreg ? nullptr : Ds;
            } else {
                if (Ds) {  // block-uniform
                    epi(std::integral_constant<int, 0>{});
#if SPN_TRUNK_DCOLS
                    if constexpr (SAVING) {
                        // each wave copies out the columns it wrote itself: no barriers (one wave's
                        // LDS accesses run in order), whole 128-B lines per 8 lanes
                        copy_cols(Ds, p0);
                    } else
#endif
                    {
                        __syncthreads();
                        copy_all(smem, Ds, p0);
                        __syncthreads();  // the sin pass overwrites the image
                    }
                }
                epi(std::integral_constant<int, 1>{});
                if (last) {
                    __syncthreads();
                    if constexpr (HEADS) {  // H_L stays on chip: the heads on this image
                        typedef const __attribute__((address_space(4))) TrunkHeadsArgs* KH;
                        KH kh = (KH)__builtin_amdgcn_kernarg_segment_ptr();
                        asm volatile("" : "+s"(kh));  // opaque per tile: the heads' argument loads stay here
                        hd::heads_tile<false>(kh->hg, kh->hk, smem, reinterpret_cast<float*>(smem + Geo::LDS),
                                              reinterpret_cast<float*>(smem + Geo::X0_OFF), nullptr, p0);
                    } else {
                        copy_all(smem, Hs, p0);
                        if (g.sig_hsave) sigma_rows(p0);  // block-uniform
                    }
                }
                hpend = last ? nullptr : Hs;
            }
        }
        __syncthreads();  // the next tile restages the image and reuses the bias slots
    }
}

// Backward dX chain (TrunkBwdArgs): the 64-point tiling of the training forward run top to
// bottom.  The LDS image holds the tile's dZ_i (B operand); the weights Wb[i] = W_iᵀ stream from
// L2 as the A operand through the same register ring; the epilogue multiplies the fp32
// accumulator by D_{i-1} and rounds to bf16 — the ×Dmul epilogue of the layer-by-layer dX GEMMs
// over the same k order, so dZ_{i-1} equals theirs bit for bit.  The tile's D_{i-1} rows load
// (coalesced 1-KB rows, in registers) while layer i's k-loop runs and land in a second LDS image
// before the epilogue; dZ_i leaves for HBM (the weight gradients read it) behind the NEXT
// layer's MFMAs, which read the same image.  Per point and layer: 1 KB of D in, 1 KB of dZ out
// (the layer-by-layer GEMM also re-reads dZ_i: 3 KB).
// DREG (option trunk_bwd_dreg, off: measured slower): dZ_{i-1} also leaves straight from the epilogue's registers
// (permlane32-joined 16-B buffer stores, as the forward's D) instead of from the image behind the
// next layer's k-loop, which then streams only the D rows and the weights.
template <bool DREG>
__global__ __launch_bounds__(512) void k_trunk_bwd_bf16(TrunkBwdArgs g, int ntiles) {
    using Geo = TrunkGeo<64>;
    constexpr int TMt = 64, NJ = Geo::NJ, IMG = Geo::IMG, CPT = Geo::CPT, TPD = Geo::TPD;
    constexpr int nks = TW / 16;
    __shared__ __attribute__((aligned(16))) char smem[2 * IMG + 8 * TW * 4];  // + the column-sum partials
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, h = lane >> 5;
    const int sw = r32 & 15;
    const int gnt = kTrunkAbl ? g.nt : 3;    // product: trunk_bwd_nt 3 (non-temporal D loads and dZ stores)
    const int gdbg = kTrunkAbl ? g.dbg : 0;
    typedef const __attribute__((address_space(4))) TrunkBwdArgs* KArgs;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();

    u32x4 ring[TPD][2];
    auto wstream = [&](int i) { return ka->Wb[i] + trunk_wave_off(w, nks) + lane * 8; };
    auto prime = [&](int i) {
        const bf16* src = wstream(i);
#pragma unroll
        for (int d = 0; d < TPD; ++d) {
            ring[d][0] = ldg16(src + d * kTrunkKStride);
            ring[d][1] = ldg16(src + d * kTrunkKStride + 512);
        }
    };
    // the tile's rows of a [P][512] bf16 tensor as a buffer resource: rows past P are dropped by
    // the hardware (stores) — no branch around the stores, whose conservative vmcnt accounting
    // made later weight-refill waits wait for them too (as in the forward's copy-outs)
    // (base nullptr: an empty resource — every access dropped, no branch)
    auto tile_rsrc = [&](const bf16* base, int64_t p0) {
        const int rows = (int)std::min<int64_t>(TMt, g.P - p0);
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(base) + p0 * TW, 0, base ? rows * TW * 2 : 0, 0x00020000);
    };
    auto copy_out = [&](bf16* dst, int64_t p0, int q0, auto kn) {
        constexpr int n = decltype(kn)::value;
        const int ct = opaque(tid);
        const __amdgpu_buffer_rsrc_t rs = tile_rsrc(dst, p0);
        u32x4 v[n];
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int c = ct + 512 * (q0 + q);
            v[q] = *reinterpret_cast<const u32x4*>(smem + act_off(c >> 6, c & 63));
        }
#pragma unroll
        for (int q = 0; q < n; ++q) {
            const int c = ct + 512 * (q0 + q);
            const int off = ((c >> 6) * TW + (c & 63) * 8) * 2;
            if (gnt & 1) __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 3);  // the product's (glc slc)
            else __builtin_amdgcn_raw_buffer_store_b128(v[q], rs, off, 0, 0);
        }
    };
    // 16 B of row min(p0 + row, P - 1) (rows past P read a clamped row, as before) through a buffer
    // resource over the tile's rows: 32-bit offsets, no 64-bit address per load
    auto tile_load = [&](const __amdgpu_buffer_rsrc_t& rs, int rows, int row, int ch) -> u32x4 {
        const int off = (std::min(row, rows - 1) * TW + ch * 8) * 2;
        return __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    };
    // per-tile column sums of the image (dZ_l, complete: called after a barrier, by every thread)
    // into dst[512]; the partials sit beyond the two images
    auto colsum = [&](float* dst) {
        const int cl = opaque(lane);
        u32x4 rows[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) rows[r] = *reinterpret_cast<const u32x4*>(smem + act_off(8 * w + r, cl));
        float a[8];
        tile_colsum_part(rows, a);
        float* part = reinterpret_cast<float*>(smem + 2 * IMG);
        *reinterpret_cast<f32x4*>(part + w * TW + cl * 8) = f32x4{a[0], a[1], a[2], a[3]};
        *reinterpret_cast<f32x4*>(part + w * TW + cl * 8 + 4) = f32x4{a[4], a[5], a[6], a[7]};
        __syncthreads();
        dst[tid] = tile_colsum_final(part, tid);
    };

    int tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;  // block-uniform
    prime(g.L - 1);
    // a tile's dZ_{L-1} rows in registers: the next tile's load at the end of this tile's layer
    // loop, before its last copy-out (the wait for them at the next tile's top does not wait for
    // those stores as well, and their HBM latency runs under the copy-out)
    u32x4 tv[CPT];
    auto load_top = [&](int64_t q0) {
        const int st = opaque(tid);
        const int rows = (int)std::min<int64_t>(TMt, g.P - q0);
        const __amdgpu_buffer_rsrc_t rs = tile_rsrc(g.dZtop, q0);
#pragma unroll
        for (int q = 0; q < CPT; ++q) {
            const int c = st + 512 * q;
            tv[q] = tile_load(rs, rows, c >> 6, c & 63);
        }
    };
    load_top((int64_t)tile * TMt);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TMt;
        {
            const int st = opaque(tid);
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                const int c = st + 512 * q;
                *reinterpret_cast<u32x4*>(smem + act_off(c >> 6, c & 63)) = tv[q];
            }
        }
        // this tile's D_{l} rows (rows past P: a clamped row), in registers until the k-loop of
        // layer l + 1 has run.  They are issued BEFORE the epilogue that precedes that k-loop:
        // vmcnt retires in order, so the weight refills issued after them are only usable once
        // the D rows are in — the epilogue plus TPD k-steps cover that HBM latency
        u32x4 dv[CPT];
        const int trows = (int)std::min<int64_t>(TMt, g.P - p0);
        auto load_d = [&](int l) {
            const int st = opaque(tid);
            if (gdbg & 2) return;
            const __amdgpu_buffer_rsrc_t rs = tile_rsrc(ka->D[l], p0);
#pragma unroll
            for (int q = 0; q < CPT; ++q) {
                const int c = st + 512 * q;
                if (gnt & 2)  // non-temporal (glc slc): the product's; 0 only in ablation builds
                    dv[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (std::min(c >> 6, trows - 1) * TW + (c & 63) * 8) * 2, 0, 3);
                else
                    dv[q] = tile_load(rs, trows, c >> 6, c & 63);
            }
        };
        load_d(g.L - 2);
        bf16* pend = nullptr;  // dZ_i of the layer whose k-loop runs: copied out during it
        for (int i = g.L - 1; i >= 1; --i) {
            const bf16* wsrc = wstream(i);
            // the next layer's (or the next tile's top layer's) stream: the ring runs on into it
            // during this k-loop's last TPD steps
            const int inext = i > 1 ? i - 1 : (tile + (int)gridDim.x < ntiles ? g.L - 1 : -1);
            f32x16 acc[2][NJ];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
            __syncthreads();  // the dZ_i image is complete; the D image is free
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (i == g.rs_layer[k]) colsum(g.Rsum[k] + tile * TW);  // block-uniform
            const char* brow = smem + r32 * 1024;
            bf16x8 bc[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) bc[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((h ^ sw) << 4));
#pragma unroll 1
            for (int ks0 = 0; ks0 < nks; ks0 += TPD) {
                // refill source of this slice's slots (block-uniform): k-steps ks0 + TPD + d of this
                // layer, past its end the next layer's k-steps d (after the last tile: this
                // layer's last slice again, unused).  A refill issued after the k-loop instead
                // (into registers whose previous loads were still in flight) made hipcc drain
                // vmcnt(0) — every weight refill and dZ store of the layer — before each epilogue
                const bf16* rsrc = ks0 + TPD < nks ? wsrc + (ks0 + TPD) * kTrunkKStride
                                                   : (inext >= 0 ? wstream(inext) : wsrc + (nks - TPD) * kTrunkKStride);
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    const int ks = ks0 + d;
                    const int offn = ((2 * (ks + 1) + h) ^ sw) << 4;
                    bf16x8 bn[NJ];
#pragma unroll
                    for (int j = 0; j < NJ; ++j) bn[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + offn);
                    const bf16x8 a0 = __builtin_bit_cast(bf16x8, ring[d][0]);
                    const bf16x8 a1 = __builtin_bit_cast(bf16x8, ring[d][1]);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bc[j], acc[0][j], 0, 0, 0);
                        acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bc[j], acc[1][j], 0, 0, 0);
                    }
                    ring[d][0] = ldg16(rsrc + d * kTrunkKStride);
                    ring[d][1] = ldg16(rsrc + d * kTrunkKStride + 512);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
#pragma unroll
                    for (int j = 0; j < NJ; ++j) bc[j] = bn[j];
                }
                constexpr int per = CPT / (nks / TPD);
                static_assert(per * (nks / TPD) == CPT && per >= 1, "copy slices");
                // (pend nullptr on a tile's first layer: the stores are dropped, no branch around them)
                copy_out(gdbg & 1 ? nullptr : pend, p0, (ks0 / TPD) * per, std::integral_constant<int, per>{});
            }
            {
                const int st = opaque(tid);
#pragma unroll
                for (int q = 0; q < CPT; ++q) {
                    const int c = st + 512 * q;
                    *reinterpret_cast<u32x4*>(smem + IMG + act_off(c >> 6, c & 63)) = dv[q];
                }
            }
            if (i > 1) load_d(i - 2);  // block-uniform
            __syncthreads();  // every wave is done reading dZ_i; the D image is complete
            if constexpr (DREG) {
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
                const int rows = (int)std::min<int64_t>(TMt, g.P - p0);
                // (dbg 1, no copy-outs: an empty range drops every store)
                const __amdgpu_buffer_rsrc_t dr =
                    __builtin_amdgcn_make_buffer_rsrc(ka->dZ[i - 1] + p0 * TW, 0, (gdbg & 1) ? 0 : rows * TW * 2, 0x00020000);
#pragma unroll
                for (int a = 0; a < 2; ++a) {
#pragma unroll
                    for (int j = 0; j < NJ; ++j) {
                        const int row = 32 * j + er32;
                        u32x2 cq[4];
#pragma unroll
                        for (int gq = 0; gq < 4; ++gq) {
                            const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                            const int o = act_off(row, f0 >> 3) + 8 * eh;
                            const f32x4 dm = ld4(reinterpret_cast<const bf16*>(smem + IMG + o));
                            float v[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * gq + e] * dm[e];
                            cq[gq] = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
                            *reinterpret_cast<u32x2*>(smem + o) = cq[gq];
                        }
#pragma unroll
                        for (int k = 0; k < 4; k += 2) {
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                const auto r = __builtin_amdgcn_permlane32_swap(cq[k][e], cq[k + 1][e], false, false);
                                cq[k][e] = r[0];
                                cq[k + 1][e] = r[1];
                            }
                            const int fb = 64 * w + 32 * a + 8 * k + 8 * eh;
                            __builtin_amdgcn_raw_buffer_store_b128(u32x4{cq[k][0], cq[k][1], cq[k + 1][0], cq[k + 1][1]}, dr,
                                                                   (row * TW + fb) * 2, 0, 0);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            } else {
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
#pragma unroll
                        for (int j = 0; j < NJ; ++j) {
                            const int row = 32 * j + er32;
                            const int o = act_off(row, f0 >> 3) + 8 * eh;
                            const f32x4 dm = ld4(reinterpret_cast<const bf16*>(smem + IMG + o));
                            float v[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * gq + e] * dm[e];
                            *reinterpret_cast<u32x2*>(smem + o) = u32x2{pack2(v[0], v[1]), pack2(v[2], v[3])};
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
            }
            pend = DREG ? nullptr : ka->dZ[i - 1];
        }
        // (past the last tile: this tile's rows again, never used — no branch around the loads)
        load_top((int64_t)std::min(tile + (int)gridDim.x, ntiles - 1) * TMt);
        __syncthreads();  // dZ_0 is complete
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (g.rs_layer[k] == 0) colsum(g.Rsum[k] + tile * TW);  // block-uniform
        if constexpr (!DREG) {
#pragma unroll
            for (int q0 = 0; q0 < CPT; q0 += 4) copy_out(pend, p0, q0, std::integral_constant<int, 4>{});
        }
        __syncthreads();  // the next tile restages the image
    }
}

int g_fused_bwd = 1;
// k_trunk_bwd_bf16<true>: dZ stored from the epilogue's registers — measured SLOWER (C4: dX chain
// 5.05-5.10 -> 5.25-5.27 ms per step, C4@512 4.42 -> 4.47 ms): unlike the forward's sin/cos, the
// x D epilogue is too short to cover the stores, which then hold up the next k-loop's refills
int g_trunk_bwd_dreg = 0;
// dX chain: 1 = non-temporal dZ copy-outs, 2 = non-temporal D loads.  Round 3 (the kernel then): level
// either way (C4 26.27 / 26.27 / 26.22 / 26.23 ms for 0 / 1 / 2 / 3, tools/gpu_r3w.sh).  Round 6 (32-bit
// buffer loads, branch-free copy-outs): 2 is the default — dX chain 5.17 / 5.18 -> 4.96 / 4.99 ms per C4
// step, the same HBM bytes (PMC FETCH_SIZE 5.235 GB per launch either way; without D loads 1.48 GB:
// D is read exactly once, the rest over dZ_top is weight re-fetch; tools/dx_probe.sh); 3 (the dZ
// copy-outs — whole 1-KB rows — non-temporal too) is the default since: dX chain 5.06 / 5.01 -> 4.97 /
// 4.97 ms, C4 24.15 / 24.18 -> 24.05 / 24.07 (ablation build, pairs in one call)
int g_trunk_bwd_nt = 3;

int32_t trunk_bwd_bf16(const TrunkBwdArgs& a, hipStream_t s, double flop, double bytes) {
    SPN_ARG(a.P >= 0 && a.L >= 2 && a.L <= kTrunkMaxL, "trunk_bwd_bf16: bad sizes (P=%lld L=%d)", (long long)a.P, a.L);
    if (a.P == 0) return SPNERF_OK;
    SPN_ARG(a.P < (1ll << 31) / TW, "trunk_bwd_bf16: too many points (%lld)", (long long)a.P);
    SPN_ARG(a.dZtop != nullptr, "trunk_bwd_bf16: NULL dZ_{L-1}");
    for (int i = 1; i < a.L; ++i)
        SPN_ARG(a.Wb[i] && a.D[i - 1] && a.dZ[i - 1], "trunk_bwd_bf16: NULL pointer at layer %d", i);
    for (int k = 0; k < 2; ++k)
        SPN_ARG(a.rs_layer[k] < 0 || (a.rs_layer[k] < a.L && a.Rsum[k] && a.P % 64 == 0),
                "trunk_bwd_bf16: column sums of layer %d need a buffer and whole 64-point tiles", a.rs_layer[k]);
    const int ntiles = cdiv(a.P, 64);
    TrunkBwdArgs ad = a;
    ad.dbg = g_trunk_dbg;
    ad.nt = g_trunk_bwd_nt;
    ProfScope prof("trunk_bwd_bf16", s, flop, bytes);
#ifdef SPN_ABLATIONS
    if (g_trunk_bwd_dreg) hipLaunchKernelGGL(k_trunk_bwd_bf16<true>, dim3(std::min(ntiles, num_cus())), dim3(512), 0, s, ad, ntiles);
    else
#endif
        hipLaunchKernelGGL(k_trunk_bwd_bf16<false>, dim3(std::min(ntiles, num_cus())), dim3(512), 0, s, ad, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

bool trunk_bf16_supported(int W, int L, int skip, int K0p) {
    // skip == 1 is refused: layers 0 and 1 would both stage per-ray rows into srb, and layer 1's
    // DMA is issued at its top with no barrier after layer 0's epilogue, which still reads srb
    // (those shapes run layer by layer; the reference's skips=[4] is unaffected)
    return W == TW && L >= 2 && L <= kTrunkMaxL && K0p <= 64 && K0p % 16 == 0 && skip < L && skip != 1;
}

// 128-point tiles for training too: C4 26.16 / 26.07 -> 25.41 / 25.43 ms, C4@512 3.789 -> 3.656 ms
// (pairs in one call; the 64-point tiling halves the points each weight byte from L2 serves)
static int trunk_tile(bool save) { return g_trunk_tile ? g_trunk_tile : 128; }

bool trunk_l0_supported(int K0p, bool save, bool zround) {
    // the tiling trunk_bf16 runs: the fp16-Z (zsave) path exists on 64-point tiles only
    const int tm = zround ? 64 : trunk_tile(save);
    const int tpd = tm == 64 ? TrunkGeo<64>::TPD : TrunkGeo<128>::TPD;
    return K0p % 4 == 0 && (K0p / 4) % tpd == 0;  // layer 0's k-loop in whole prefetch rounds
}

// σ rows from the training trunk's last image (TrunkArgs::sig_hsave): k_heads_fwd_v 0.66 -> 0.56 ms per
// C4 step (no H_L reads), trunk +0.03 ms, C4 26.83 / 26.77 -> 26.81 / 26.70 ms (tools/gpu_r3zb.sh)
int g_trunk_sigma = 1;

bool trunk_sigma_ok(const TrunkArgs& a, bool save) {
    return g_trunk_sigma && save && !a.zround && !trunk2_supported(a, save);  // either training tiling
}

bool trunk1_heads_ok(const TrunkArgs& a) {
    bool save = false;
    for (int i = 1; i < a.L; ++i) save |= a.Ds[i] != nullptr;
    return g_trunk_heads == 2 && g_fused_trunk && !save && !a.zround && trunk_tile(false) == 128 && !a.X0b_out &&
           trunk_bf16_supported(TW, a.L, a.skip, a.K0p) && (!(a.X0 || a.rays) || (a.Wf[0] && trunk_l0_supported(a.K0p, false)));
}

int32_t trunk1_heads_bf16(const TrunkArgs& a, const HeadsFusedArgs& h, const PackedOffs& k, hipStream_t s, double flop,
                          double bytes) {
    SPN_ARG(trunk1_heads_ok(a), "trunk1_heads_bf16: unsupported shape or option");
    SPN_ARG(h.P == a.P && h.S == a.S && h.NO <= hd::OST_LD && h.C <= 4 && k.Fnar16 >= 0, "trunk1_heads_bf16: bad heads");
    SPN_ARG(!a.rays || (a.z && a.rs > 0 && !a.X0), "trunk1_heads_bf16: inline encoding needs z and rs");
    if (a.P == 0) return SPNERF_OK;
    SPN_ARG(a.P < (1ll << 31) / TW, "trunk1_heads_bf16: too many points (%lld)", (long long)a.P);
    const int ntiles = cdiv(a.P, 128);
    TrunkHeadsArgs ad;
    static_cast<TrunkArgs&>(ad) = a;
    if (ad.ldz == 0) ad.ldz = ad.S;  // contiguous z rows
    ad.dbg = 0;
    ad.nt = 0;
    ad.hg = h;
    ad.hg.nt = 0;
    ad.hg.dbg = 0;
    ad.hk = k;
    ProfScope prof("trunk_heads_bf16", s, flop, bytes);
    hipLaunchKernelGGL((k_trunk_bf16<128, 4096>), dim3(std::min(ntiles, num_cus())), dim3(512), 0, s, ad, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

int32_t trunk_bf16(const TrunkArgs& a, hipStream_t s, double flop, double bytes) {
    SPN_ARG(a.P >= 0 && a.S > 0, "trunk_bf16: bad sizes");
    SPN_ARG(trunk_bf16_supported(TW, a.L, a.skip, a.K0p), "trunk_bf16: unsupported shape L=%d skip=%d K0p=%d", a.L,
            a.skip, a.K0p);
    SPN_ARG(a.Hs[a.L - 1] != nullptr, "trunk_bf16: the last layer's output is required");
    if (a.P == 0) return SPNERF_OK;
    SPN_ARG(a.P < (1ll << 31) / TW, "trunk_bf16: too many points (%lld)", (long long)a.P);
    bool save = false;
    for (int i = 1; i < a.L; ++i) save |= a.Ds[i] != nullptr;
    SPN_ARG(!a.rays || (a.z && a.rs > 0 && !a.X0 && (!save || a.X0b_out)),
            "trunk_bf16: inline encoding needs z, rs, and when saving the X0b output");
    if (!a.X0b_out && trunk2_supported(a, save)) return trunk2_bf16(a, s, save, flop, bytes);
    const int tm = a.zround ? 64 : trunk_tile(save);  // the 128-point tiling has no fp16-Z path
    SPN_ARG(!(a.X0 || a.rays) || (a.Wf[0] && trunk_l0_supported(a.K0p, save, a.zround != 0)), "trunk_bf16: layer 0 unsupported for K0p=%d",
            a.K0p);
    TrunkArgs ad = a;
    if (ad.ldz == 0) ad.ldz = ad.S;  // contiguous z rows
    ad.dbg = g_trunk_dbg;
    ad.nt = (g_trunk_nt & 1) | ((g_trunk_nt & 4) ? 2 : 0);  // H copy-outs / register-D stores non-temporal
    const int ntiles = cdiv(a.P, tm);
    // the saving launches (training) are their own profiling class: their roofline (HBM-heavy,
    // H and D of every layer out) is not the inference launches' (MFMA-bound)
    ProfScope prof(save ? "trunk_bf16_train" : "trunk_bf16", s, flop, bytes);
    const dim3 grid(std::min(ntiles, num_cus())), block(512);
    bool done = false;
#ifdef SPN_ABLATIONS
    // profiling ablations (outputs invalid) and the measured-slower 64-point tiling without the
    // register-D epilogue: compiled only into -DSPN_ABLATIONS builds
    done = true;
    if (tm == 64 && g_trunk_dreg && g_trunk_var == 32)  // ablation: no sin / cos in the epilogue
        hipLaunchKernelGGL((k_trunk_bf16<64, 544>), grid, block, 0, s, ad, ntiles);
    else if (tm == 64 && g_trunk_dreg && g_trunk_var == 256)  // ablation: no epilogue at all
        hipLaunchKernelGGL((k_trunk_bf16<64, 768>), grid, block, 0, s, ad, ntiles);
    else if (tm == 64 && !g_trunk_dreg) hipLaunchKernelGGL(k_trunk_bf16<64>, grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && g_trunk_var == 16) hipLaunchKernelGGL((k_trunk_bf16<128, 16>), grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && g_trunk_var == 32) hipLaunchKernelGGL((k_trunk_bf16<128, 32>), grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && g_trunk_var == 64) hipLaunchKernelGGL((k_trunk_bf16<128, 64>), grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && g_trunk_var == 128) hipLaunchKernelGGL((k_trunk_bf16<128, 128>), grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && g_trunk_var == 256) hipLaunchKernelGGL((k_trunk_bf16<128, 256>), grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && g_trunk_var == 464) hipLaunchKernelGGL((k_trunk_bf16<128, 464>), grid, block, 0, s, ad, ntiles);
    else if (tm == 128 && save && g_trunk_var == 8192) hipLaunchKernelGGL((k_trunk_bf16<128, 2048 | 8192>), grid, block, 0, s, ad, ntiles);
    else done = false;
#endif
    if (!done) {
        if (tm == 64) hipLaunchKernelGGL((k_trunk_bf16<64, 512>), grid, block, 0, s, ad, ntiles);
        else if (save) hipLaunchKernelGGL((k_trunk_bf16<128, 2048>), grid, block, 0, s, ad, ntiles);
        else hipLaunchKernelGGL((k_trunk_bf16<128, 0>), grid, block, 0, s, ad, ntiles);
    }
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

}  // namespace spn
