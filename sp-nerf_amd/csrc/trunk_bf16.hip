// Fused SIREN trunk of the bf16 MLP (cfg.dtype = 1, W = 512): fc_net layers 1 .. L-1
// (models/spnerf.py:201-209, 323-330) for a tile of 128 points per workgroup, with the
// activations resident in LDS from layer to layer — the persistent MFMA MLP kernel of DESIGN.md.
//
// Formulation: every layer computes Hᵀ_next = sin(W·Hᵀ + b) with the WEIGHTS as the MFMA A
// operand and the activation tile as B (v_mfma_f32_32x32x16_bf16).  A 32x32 accumulator then
// holds, per lane, 4 runs of 4 consecutive output features of ONE point: each run is an 8-byte
// piece of a row of the next layer's [point][feature] image, written with one ds_write_b64.
//  * LDS (148 KB): the [128][512] bf16 activation image (16-B chunks XOR-swizzled by row & 15:
//    conflict-free ds_read_b128 B fragments and ds_write_b64 epilogue writes), the [128][K0p]
//    PE tile of the skip layer, and two bias slots (layer parity).
//  * Weights stream from L2 (every CU walks the same 512 KB per layer), packed by
//    spnerf_pack_params in MFMA fragment order (trunk_frag_off): wave w's A fragments of k-step
//    ks are one contiguous 2 KB, loaded TPD k-steps ahead into a register ring.  The next
//    layer's first k-steps load during the current layer's epilogue.
//  * 8 waves; wave w owns output features [64w, 64w + 64) of all 128 points (2 x 4 tiles).
//  * Epilogue = the unfused k_gemm_nt_bf16 arithmetic (fp32 accumulator + bias (+ the per-ray
//    semantic rows at the skip layer), fast_sincos, bf16 rounding) over the same k-order: sin
//    goes to the LDS image and, when saving for the backward, H_i / D_i = cos go to HBM; the
//    last layer's H always goes to HBM (the heads read it).
#include <algorithm>
#include <type_traits>

#include "trunk.h"

namespace spn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

int g_fused_trunk = 1;

constexpr int TW = 512;                      // trunk width of the fused kernel
constexpr int TM = 128;                      // points per tile
constexpr int TPD = 4;                       // weight prefetch depth (k-steps)
constexpr int ACT_BYTES = TM * TW * 2;       // 131072
constexpr int X0_BYTES = TM * 64 * 2;        // 16384 (K0p <= 64)
constexpr int TRUNK_LDS = ACT_BYTES + X0_BYTES + 2 * TW * 4;

__device__ __forceinline__ int act_off(int row, int ch) { return row * 1024 + ((ch ^ (row & 15)) << 4); }
// PE rows are 8 chunks (128 B): XOR with (row >> 1) & 7 keeps the 16 rows of a ds_read_b128
// lane group on distinct 16-B slots of the bank row
__device__ __forceinline__ int x0_off(int row, int ch) { return ACT_BYTES + row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }

// a copy of x the compiler cannot see through: lane-derived addresses are recomputed in each
// region (staging, k-loop, epilogue) instead of being hoisted out of all loops and kept live
// across the k-loop, where the accumulators and the weight ring need the registers
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

__global__ __launch_bounds__(512) void k_trunk_bf16(TrunkArgs g, int ntiles) {
    __shared__ __attribute__((aligned(16))) char smem[TRUNK_LDS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r32 = lane & 31, h = lane >> 5;
    float* sbias = reinterpret_cast<float*>(smem + ACT_BYTES + X0_BYTES);
    const int x0ch = g.K0p >> 3;
    constexpr int nmain = TW / 16;                // k-steps over the activation image
    const int ntail = g.K0p >> 4;                 // extra k-steps over the PE at the skip layer
    const int sw = r32 & 15;
    // per-layer pointers indexed by the (runtime) layer: scalar loads straight from the kernarg
    // segment (indexing the by-value struct copies its arrays to scratch)
    typedef const __attribute__((address_space(4))) TrunkArgs* KArgs;
    const KArgs ka = (KArgs)__builtin_amdgcn_kernarg_segment_ptr();

    u32x4 ring[TPD][2];
    // wave w's fragment stream of layer i: k-step ks at + ks * 1024, feature tile a at + 512 * a
    auto wstream = [&](int i) {
        const int nks = nmain + (i == g.skip ? ntail : 0);
        return ka->Wf[i] + (int64_t)w * nks * 1024 + lane * 8;
    };
    auto prime = [&](int i) {
        const bf16* src = wstream(i);
#pragma unroll
        for (int d = 0; d < TPD; ++d) {
            ring[d][0] = ldg16(src + d * 1024);
            ring[d][1] = ldg16(src + d * 1024 + 512);
        }
    };

    int tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile >= ntiles) return;  // block-uniform
    prime(1);
    for (; tile < ntiles; tile += gridDim.x) {
        const int64_t p0 = (int64_t)tile * TM;
        const int st = opaque(tid);
        // stage the layer-1 input and the PE tile; rows past P read a clamped row (their
        // outputs are never stored)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            u32x4 v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = st + 512 * (8 * half + q), row = c >> 6, ch = c & 63;
                v[q] = ldg16(g.H1 + std::min<int64_t>(p0 + row, g.P - 1) * TW + ch * 8);
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int c = st + 512 * (8 * half + q), row = c >> 6, ch = c & 63;
                *reinterpret_cast<u32x4*>(smem + act_off(row, ch)) = v[q];
            }
        }
        if (g.skip > 0) {
            for (int c = st; c < TM * x0ch; c += 512) {
                const int row = c / x0ch, ch = c % x0ch;
                *reinterpret_cast<u32x4*>(smem + x0_off(row, ch)) =
                    ldg16(g.X0b + std::min<int64_t>(p0 + row, g.P - 1) * g.K0p + ch * 8);
            }
        }

        bf16* hpend = nullptr;  // H of the previous layer: copied to HBM during this layer's k-loop
        for (int i = 1; i < g.L; ++i) {
            const bool skip = i == g.skip;
            const bf16* wsrc = wstream(i);
            const int nks = nmain + (skip ? ntail : 0);
            float* sb = sbias + (i & 1) * TW;  // slot (i-1)&1 may still be read by the previous epilogue
            sb[tid] = ka->bias[i][tid];
            f32x16 acc[2][4];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;
            __syncthreads();  // the image (and the bias slot) of layer i are complete

            // B fragments are double-buffered: step ks+1's image reads are issued between step
            // ks's MFMAs (past the image's last step the read lands in the PE area: in bounds,
            // unused)
            const char* brow = smem + r32 * 1024;
            bf16x8 bc[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) bc[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + ((h ^ sw) << 4));
#pragma unroll 1
            for (int ks0 = 0; ks0 < nmain; ks0 += TPD) {
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    const int ks = ks0 + d;
                    const int offn = ((2 * (ks + 1) + h) ^ sw) << 4;
                    bf16x8 bn[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) bn[j] = *reinterpret_cast<const bf16x8*>(brow + j * 32768 + offn);
                    const bf16x8 a0 = __builtin_bit_cast(bf16x8, ring[d][0]);
                    const bf16x8 a1 = __builtin_bit_cast(bf16x8, ring[d][1]);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bc[j], acc[0][j], 0, 0, 0);
                        acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bc[j], acc[1][j], 0, 0, 0);
                    }
                    // refill the slot just consumed, right behind its MFMAs (TPD - 1 steps of
                    // cover); past the stream's end: re-read its last step
                    const int kn = std::min(ks + TPD, nks - 1);
                    ring[d][0] = ldg16(wsrc + kn * 1024);
                    ring[d][1] = ldg16(wsrc + kn * 1024 + 512);
                    // order: (1 image read, 2 MFMAs) x 4, then the 2 weight loads
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    }
                    __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
#pragma unroll
                    for (int j = 0; j < 4; ++j) bc[j] = bn[j];
                }
                if (hpend) {  // block-uniform: 2 of the image's 16 row chunks per thread
                    const int ct = opaque(tid);
#pragma unroll
                    for (int q = 0; q < 2; ++q) {
                        const int c = ct + 512 * (2 * (ks0 / TPD) + q);
                        const u32x4 v = *reinterpret_cast<const u32x4*>(smem + act_off(c >> 6, c & 63));
                        if (p0 + (c >> 6) < g.P) *reinterpret_cast<u32x4*>(hpend + (p0 + (c >> 6)) * TW + (c & 63) * 8) = v;
                    }
                }
            }
            static_assert(TW / 16 / TPD * 2 == 16, "the k-loop copies the 16 chunks per thread of the image");
            // the x0 columns of the skip layer's input [h | x0] (nks == nmain elsewhere); ntail
            // is a multiple of TPD (K0p is 32 or 64)
#pragma unroll 1
            for (int ks0 = nmain; ks0 < nks; ks0 += TPD) {
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    const int ks = ks0 + d;
                    bf16x8 b[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        b[j] = *reinterpret_cast<const bf16x8*>(smem + x0_off(32 * j + r32, 2 * (ks - nmain) + h));
                    const bf16x8 a0 = __builtin_bit_cast(bf16x8, ring[d][0]);
                    const bf16x8 a1 = __builtin_bit_cast(bf16x8, ring[d][1]);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[j], acc[0][j], 0, 0, 0);
                        acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[j], acc[1][j], 0, 0, 0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    const int kn = std::min(ks + TPD, nks - 1);
                    ring[d][0] = ldg16(wsrc + kn * 1024);
                    ring[d][1] = ldg16(wsrc + kn * 1024 + 512);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // the next layer's (or the next tile's layer-1) first k-steps load during the epilogue
            const bool last = i == g.L - 1;
            if (!last) prime(i + 1);
            else if (tile + (int)gridDim.x < ntiles) prime(1);

            __syncthreads();  // every wave is done reading the image of layer i
            bf16* Hs = ka->Hs[i];
            bf16* Ds = ka->Ds[i];
            const float* rb = skip ? g.rb_skip : nullptr;
            // Outputs leave through the image: a wave writes its 8-byte pieces to LDS, then every
            // wave copies whole 1-KB rows to HBM (one row per store instruction; scattered 8-byte
            // stores from the accumulator layout cost ~2x the whole layer).  Pass 0 (saving only)
            // writes cos = D_i and copies it out between two barriers; pass 1 writes sin, the next
            // layer's input, which that layer's k-loop copies out as H_i behind its MFMAs (the last
            // layer copies its H here).
            auto epilogue = [&](auto kpass) {
                constexpr int pass = decltype(kpass)::value;
                const int el = opaque(lane), er32 = el & 31, eh = el >> 5;
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int gq = 0; gq < 4; ++gq) {
                        const int f0 = 64 * w + 32 * a + 8 * gq + 4 * eh;
                        const f32x4 bv = *reinterpret_cast<const f32x4*>(sb + f0);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int row = 32 * j + er32;
                            float v[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * gq + e] + bv[e];
                            if (rb) {
                                const f32x4 rv = ld4(rb + (std::min<int64_t>(p0 + row, g.P - 1) / g.S) * TW + f0);
#pragma unroll
                                for (int e = 0; e < 4; ++e) v[e] += rv[e];
                            }
                            float y[4];
#pragma unroll
                            for (int e = 0; e < 4; ++e) y[e] = pass ? fast_sin(v[e]) : fast_cos(v[e]);
                            const u32x2 o = {pack2(y[0], y[1]), pack2(y[2], y[3])};
                            *reinterpret_cast<u32x2*>(smem + act_off(row, f0 >> 3) + 8 * eh) = o;
                        }
                        __builtin_amdgcn_sched_barrier(0);  // bound the live range of hoisted loads
                    }
                bf16* dst = pass ? (last ? Hs : nullptr) : Ds;
                if (dst) {  // block-uniform
                    __syncthreads();
                    const int ct = opaque(tid);
#pragma unroll
                    for (int q0 = 0; q0 < 16; q0 += 4) {
                        u32x4 v[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int c = ct + 512 * (q0 + q);
                            v[q] = *reinterpret_cast<const u32x4*>(smem + act_off(c >> 6, c & 63));
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const int c = ct + 512 * (q0 + q);
                            if (p0 + (c >> 6) < g.P) *reinterpret_cast<u32x4*>(dst + (p0 + (c >> 6)) * TW + (c & 63) * 8) = v[q];
                        }
                    }
                    if (pass == 0) __syncthreads();  // the sin pass overwrites the image
                }
            };
            if (Ds) epilogue(std::integral_constant<int, 0>{});  // block-uniform
            epilogue(std::integral_constant<int, 1>{});
            hpend = last ? nullptr : Hs;
        }
        __syncthreads();  // the next tile restages the image and reuses the bias slots
    }
}

bool trunk_bf16_supported(int W, int L, int skip, int K0p) {
    return W == TW && L >= 2 && L <= kTrunkMaxL && K0p <= 64 && K0p % (16 * TPD) == 0 && skip < L;
}

int32_t trunk_bf16(const TrunkArgs& a, hipStream_t s, double flop, double bytes) {
    SPN_ARG(a.P >= 0 && a.S > 0, "trunk_bf16: bad sizes");
    SPN_ARG(trunk_bf16_supported(TW, a.L, a.skip, a.K0p), "trunk_bf16: unsupported shape L=%d skip=%d K0p=%d", a.L,
            a.skip, a.K0p);
    SPN_ARG(a.Hs[a.L - 1] != nullptr, "trunk_bf16: the last layer's output is required");
    if (a.P == 0) return SPNERF_OK;
    SPN_ARG(a.P < (1ll << 31) / TW, "trunk_bf16: too many points (%lld)", (long long)a.P);
    const int ntiles = cdiv(a.P, TM);
    ProfScope prof("trunk_bf16", s, flop, bytes);
    hipLaunchKernelGGL(k_trunk_bf16, dim3(std::min(ntiles, 256)), dim3(512), 0, s, a, ntiles);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

}  // namespace spn
