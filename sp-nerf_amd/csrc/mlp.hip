// SP-NeRF per-point network on gfx950: SPNeRF.forward (models/spnerf.py:273-369) and its
// backward, as a sequence of fp32 MFMA GEMMs (gemm_f32.hip) with fused epilogues plus small
// per-point / per-ray kernels.
//
// Algebraic re-layout (exact up to fp32 summation order):
//  * the semantic embedding, the sun direction and the time embedding are constant along a
//    ray, so their input columns of fc_net.0 / fc_net.<2*skip> / sun_v_net.0 / beta_from_xyz.0
//    become per-RAY bias rows (k_ray_fwd) added in the GEMM epilogue — no repeat_interleave,
//    no K padding for 63/575/515 wide inputs;
//  * sky_color depends only on sun_d → evaluated once per ray, broadcast to the points;
//  * sibling heads that read the same activation are one GEMM: G = H_L·[feat; sem hidden]^T,
//    Q = feat·[sun hidden 1; rgb hidden; beta hidden]^T;
//  * N ≤ C-wide output heads (σ, rgb, sun, β, semantic logits) are per-point dot products.
#include <algorithm>
#include <atomic>
#include <type_traits>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

#include "common.h"
#include "gemm_bf16.h"
#include "gemm_f32.h"
#include "heads_dx.h"
#include "mlp_layout.h"
#include "trunk.h"
#include "wave.h"

namespace spn {

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------

struct PackPiece {
    const float* src;
    // bf: 1 = bf16 destination (dst in bf16 units); 2 = bf16 in the fused trunk's MFMA fragment
    // order (trunk_frag_off, dst_ld = the layer's padded K; transposed: element [c][r]); 5 = the same for 32 features per
    // wave (frag_off NA = 1: the fused heads' 256-wide layers); 7 = frag_off NA = 2 (64 features per wave; the
    // heads' dX chain, transposed only); 3 = split into bf16 planes
    // [hi | hi | lo | lo] of width dst_ld / 4 each (hi = bf16(v), lo = bf16(v − hi)); 4 = the
    // same planes in the fused trunk's fragment order (dst_ld = 4·K0p); 6 = a narrow head's
    // [32][cols] hi/lo-row A operand (PackedOffs::Fnar16; rows = 32, nsrc source rows)
    int src_ld, src_c0, rows, cols, dst_ld, transpose, bf;
    int src_idx;   // the parameter's index (device-resident tables: src comes from PackSrcs)
    int64_t dst;
    int nsrc = 0;  // bf = 6: source rows
    int rnd = 0;   // fp32 destination rounded to bf16 (precision study, option emu_bf16 & 4)
};
static_assert(sizeof(PackPiece) == 56, "PackArgs must stay within the 4 KB kernel-argument segment");
constexpr int kPackParams = 64;
struct PackSrcs {
    const float* p[kPackParams];
};
constexpr int kMaxPieces = 64;
constexpr int kPackTR = 32, kPackTC = 64;  // a block re-lays one 32 x 64 tile of a piece
struct PackArgs {
    PackPiece p[kMaxPieces];
    int tile0[kMaxPieces + 1];  // prefix of the pieces' tile counts (block ranges)
    int n;
    float* packed;
};

// One launch for up to kMaxPieces pieces: block b re-lays tile (b - tile0[piece]) of its piece,
// 8 elements per thread.  Transposed pieces (fp32 or bf16) go through an LDS tile so both the
// read (rows of the source) and the write (rows of the transpose) are coalesced.
// block b re-lays tile t of piece pc into packed
__device__ __forceinline__ void pack_block(const PackPiece pc, int t, float* packed) {
    __shared__ float tileT[kPackTC][kPackTR + 1];
    const int tcols = (pc.cols + kPackTC - 1) / kPackTC;
    const int r0 = (t / tcols) * kPackTR, c0 = (t % tcols) * kPackTC;
    const int tid = threadIdx.x;
    if (pc.transpose && (pc.bf <= 2 || pc.bf == 5 || pc.bf == 7)) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int rr = (tid >> 6) + 4 * e, cc = tid & 63;
            const int r = r0 + rr, c = c0 + cc;
            tileT[cc][rr] = (r < pc.rows && c < pc.cols) ? pc.src[(int64_t)r * pc.src_ld + pc.src_c0 + c] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int rr = tid & 31, cc = (tid >> 5) + 8 * e;
            const int r = r0 + rr, c = c0 + cc;
            if (r < pc.rows && c < pc.cols) {
                const int64_t o = pc.dst + (pc.bf == 2   ? trunk_frag_off(c, r, pc.dst_ld)
                                            : pc.bf == 5 ? frag_off(c, r, pc.dst_ld, 1)
                                            : pc.bf == 7 ? frag_off(c, r, pc.dst_ld, 2)
                                                         : (int64_t)c * pc.dst_ld + r);
                if (pc.bf) reinterpret_cast<bf16*>(packed)[o] = (bf16)tileT[cc][rr];
                else packed[o] = pc.rnd ? (float)(bf16)tileT[cc][rr] : tileT[cc][rr];
            }
        }
        return;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int r = r0 + (tid >> 6) + 4 * e, c = c0 + (tid & 63);
        if (r >= pc.rows || c >= pc.cols) continue;
        if (pc.bf == 6) {  // destination row r: source row sr's hi (r even) or lo (r odd) plane
            const int sr = r < 2 ? 0 : r < 4 ? 1 : (r == 8 || r == 9) ? 2 : -1;
            bf16 o = (bf16)0.f;
            if (sr >= 0 && sr < pc.nsrc) {
                const float v = pc.src[(int64_t)sr * pc.src_ld + pc.src_c0 + c];
                const bf16 hi = (bf16)v;
                o = (r & 1) ? (bf16)(v - (float)hi) : hi;
            }
            reinterpret_cast<bf16*>(packed)[pc.dst + frag_off(r, c, pc.dst_ld, 1)] = o;
            continue;
        }
        const float v = pc.src[(int64_t)r * pc.src_ld + pc.src_c0 + c];
        if (pc.bf == 3 || pc.bf == 4) {
            bf16* dst = reinterpret_cast<bf16*>(packed) + pc.dst;
            const int kp = pc.dst_ld / 4;
            const bf16 hi = (bf16)v, lo = (bf16)(v - (float)hi);
            const bf16 pl[4] = {hi, hi, lo, lo};
            for (int j = 0; j < 4; ++j)
                dst[pc.bf == 4 ? trunk_frag_off(r, c + j * kp, pc.dst_ld) : (int64_t)r * pc.dst_ld + c + j * kp] = pl[j];
            continue;
        }
        const int64_t o = pc.dst + (pc.bf == 2        ? trunk_frag_off(r, c, pc.dst_ld)
                                    : pc.bf == 5   ? frag_off(r, c, pc.dst_ld, 1)
                                    : pc.transpose ? (int64_t)c * pc.dst_ld + r
                                                   : (int64_t)r * pc.dst_ld + c);
        if (pc.bf) reinterpret_cast<bf16*>(packed)[o] = (bf16)v;
        else packed[o] = pc.rnd ? (float)(bf16)v : v;
    }
}

__global__ __launch_bounds__(256) void k_pack(PackArgs a) {
    const int b = blockIdx.x;
    int pi = 0;
    while (pi + 1 < a.n && a.tile0[pi + 1] <= b) ++pi;  // block-uniform
    pack_block(a.p[pi], b - a.tile0[pi], a.packed);
}

// The same for a piece table resident in device memory (pack_table: one launch for any number
// of pieces — the bf16 MLP's ~90 pieces took two kernarg-table launches per re-pack).  blk[b] =
// {piece, tile} of block b, one load (a binary search over the tile prefix was 7 dependent loads
// ahead of every block's work: 24 us per re-pack)
__global__ __launch_bounds__(256) void k_pack_dev(const PackPiece* __restrict__ pcs, const int2* __restrict__ blk,
                                                  float* packed, PackSrcs srcs) {
    const int2 bt = blk[blockIdx.x];
    PackPiece pc = pcs[bt.x];
    pc.src = srcs.p[pc.src_idx];
    pack_block(pc, bt.y, packed);
}

// X0[p][c]: positional encoding of xyz = o + dir*z (rendering.py:147; spnerf.py:32-37), one
// output element per thread.  Each of the fp32 row X0, its bf16 copy X0b and its split planes
// X0s = [hi | lo | hi | lo] (hi = bf16(v), lo = bf16(v − hi), row length 4·K0p) is written when
// non-null.  o + dir*z is evaluated as two rounded ops like the reference
// (no FMA contraction: sin(2^9 x) amplifies a 1-ulp difference in x by 512).
__global__ void k_encode(const float* __restrict__ rays, int rs, int dir_off, const float* __restrict__ z, int S, int ldz,
                         int64_t P, int n_freq, int K0, int K0p, float* __restrict__ X0, bf16* __restrict__ X0b,
                         bf16* __restrict__ X0s) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= P * K0p) return;
    const int64_t p = i / K0p;
    const int c = (int)(i % K0p);
    const int64_t r = p / S;
    const float v = c < K0 ? pe_value(rays + r * rs, dir_off, z[r * ldz + (p - r * S)], c, n_freq, K0) : 0.f;
    if (X0) X0[i] = v;
    const bf16 hi = (bf16)v;
    if (X0b) X0b[i] = hi;
    if (X0s) {
        bf16* r = X0s + p * 4 * K0p + c;
        const bf16 lo = (bf16)(v - (float)hi);
        r[0] = hi;
        r[K0p] = lo;
        r[2 * K0p] = hi;
        r[3 * K0p] = lo;
    }
}

struct RayFwdArgs {
    const float* rays; int rs;
    const int64_t* labels; const float* temb;
    const float* packed; PackedOffs k; Dims d;
    float *rb0, *rb4, *rbQ, *skyh, *sky;
    int sem_on, need_q, need_sky;
};

// Per-ray terms: semantic bias rows of fc_net.0 / fc_net.<skip>, sun / t bias rows of the Q
// GEMM, and the sky_color MLP (spnerf.py:244-249,355).  One 256-thread block per ray.
__global__ __launch_bounds__(256) void k_ray_fwd(RayFwdArgs a) {
    const int64_t ray = blockIdx.x;
    const int tid = threadIdx.x;
    const Dims& d = a.d;
    const float* P = a.packed;
    const float* r = a.rays + ray * a.rs;
    const float s0 = r[8], s1 = r[9], s2 = r[10];
    if (a.sem_on) {
        int64_t lab = a.labels[ray];
        if (lab == -100) lab = d.C;
        const float* e = P + a.k.emb + lab * d.sd;
        for (int n = tid; n < d.W; n += blockDim.x) {
            float v0 = 0.f, v4 = 0.f;
            for (int j = 0; j < d.sd; ++j) {
                v0 += P[a.k.Wsem0 + (int64_t)n * d.sd + j] * e[j];
                v4 += P[a.k.Wsem4 + (int64_t)n * d.sd + j] * e[j];
            }
            a.rb0[ray * d.W + n] = v0;
            a.rb4[ray * d.W + n] = v4;
        }
    }
    if (a.need_q) {
        for (int n = tid; n < d.NQ; n += blockDim.x) {
            float v = 0.f;
            if (n < d.H) {
                const float* w = P + a.k.Wsun + n * 3;
                v = w[0] * s0 + w[1] * s1 + w[2] * s2;
            } else if (n >= 2 * d.H) {
                const float* w = P + a.k.Wtt + (int64_t)(n - 2 * d.H) * d.td;
                const float* t = a.temb + ray * d.td;
                for (int j = 0; j < d.td; ++j) v += w[j] * t[j];
            }
            a.rbQ[ray * d.NQ + n] = v;
        }
    }
    if (a.need_sky) {
        __shared__ float red[3][256];
        float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;
        for (int n = tid; n < d.H; n += blockDim.x) {
            const float* w = P + a.k.Wk1 + n * 3;
            const float hv = fmaxf(P[a.k.bk1 + n] + (w[0] * s0 + w[1] * s1 + w[2] * s2), 0.f);
            a.skyh[ray * d.H + n] = hv;
            acc0 += P[a.k.Wk2 + n] * hv;
            acc1 += P[a.k.Wk2 + d.H + n] * hv;
            acc2 += P[a.k.Wk2 + 2 * d.H + n] * hv;
        }
        red[0][tid] = acc0;
        red[1][tid] = acc1;
        red[2][tid] = acc2;
        __syncthreads();
        for (int st = 128; st > 0; st >>= 1) {
            if (tid < st)
                for (int c = 0; c < 3; ++c) red[c][tid] += red[c][tid + st];
            __syncthreads();
        }
        if (tid < 3) a.sky[ray * 4 + tid] = sigmoidf_(red[tid][0] + P[a.k.bk2 + tid]);
    }
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// lane-partial dot product of a row with a weight vector, columns 4*lane + 256*i
template <typename T>
__device__ __forceinline__ float pdot(const T* __restrict__ x, const float* __restrict__ w, int n, int lane) {
    float s = 0.f;
    for (int k = 4 * lane; k < n; k += 256) {
        const f32x4 a = ld4(x + k);
        const f32x4 b = *reinterpret_cast<const f32x4*>(w + k);
        s += (a[0] * b[0] + a[1] * b[1]) + (a[2] * b[2] + a[3] * b[3]);
    }
    return s;
}

template <typename T>
struct HeadsArgs {
    const float* packed; Dims d;
    const T *HL, *G, *Q, *S3;
    const float* sky;
    float* out; float* hsave;
    int64_t P; int S; int mode;  // mode: 0 full, 1 sigma only, 2 sigma + sun
};

// Narrow output heads (spnerf.py:333-367): σ = softplus, albedo = sigmoid·1.002−0.001,
// sun = sigmoid, β = softplus, semantic logits; sky broadcast per ray.  One wavefront per
// point: every row read is a coalesced 1-KiB sweep, dot products end in a DPP reduction.
template <typename T>
__global__ __launch_bounds__(256) void k_heads_fwd(HeadsArgs<T> a, PackedOffs k) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const Dims& d = a.d;
    const float* Pk = a.packed;
    for (int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < a.P; p += nw) {
        float* o = a.out + p * d.NO;
        float* hs = a.hsave + p * 8;
        const float spre = wsum(pdot(a.HL + p * d.W, Pk + k.wsig, d.W, lane)) + Pk[k.bsig];
        float sun = 0.f, rgb[3] = {0.f, 0.f, 0.f}, bpre = 0.f;
        if (a.mode != 1) sun = sigmoidf_(wsum(pdot(a.S3 + p * d.H, Pk + k.ws4, d.H, lane)) + Pk[k.bs4]);
        if (a.mode == 0) {
            const T* R1 = a.Q + p * d.NQ + d.H;
            for (int c = 0; c < 3; ++c) rgb[c] = sigmoidf_(wsum(pdot(R1, Pk + k.Wr2 + c * d.H, d.H, lane)) + Pk[k.br2 + c]);
            if (d.beta) bpre = wsum(pdot(a.Q + p * d.NQ + 2 * d.H, Pk + k.wb2, d.H, lane)) + Pk[k.bb2];
            if (d.sem) {
                const T* M1 = a.G + p * d.NG + d.W;
                for (int c = 0; c < d.C; ++c) {
                    const float v = wsum(pdot(M1, Pk + k.Wm2 + c * d.H, d.H, lane)) + Pk[k.bm2 + c];
                    if (lane == 0) o[d.sem_col + c] = v;
                }
            }
        }
        if (lane == 0) {
            o[3] = softplusf_(spre);
            hs[0] = spre;
            if (a.mode == 1) continue;
            o[4] = sun;
            hs[4] = sun;
            if (a.mode == 2) {
                o[0] = o[1] = o[2] = o[5] = o[6] = o[7] = 0.f;
                for (int c = 8; c < d.NO; ++c) o[c] = 0.f;
                continue;
            }
            for (int c = 0; c < 3; ++c) {
                hs[1 + c] = rgb[c];
                o[c] = __fsub_rn(__fmul_rn(rgb[c], 1.002f), 0.001f);
            }
            const float* sk = a.sky + (p / a.S) * 4;
            o[5] = sk[0];
            o[6] = sk[1];
            o[7] = sk[2];
            if (d.beta) {
                hs[5] = bpre;
                o[8] = softplusf_(bpre);
            }
        }
    }
}

int g_heads_variant = 1;  // 0 = the one-point-at-a-time k_heads_fwd (ablation)
// backward: 2 = weight gradients on a second stream beside the dX chain; 1 = one stream (default:
// measured on MI355X, the two streams' GEMMs contend for HBM / L2 and the step got 3% slower,
// in eager mode and as a captured graph alike — C4 at 512 rays 4.99 -> 5.15 ms)
int g_bwd_streams = 1;

// The backward's second stream: the weight-gradient GEMMs, their slab reductions and the per-ray
// parameter sums run there, beside the dX chain on the caller's stream, joined by events
// (fork: main → side after an input is produced; join: side → main at the end, so the caller
// sees the usual stream order).  Inside a captured HIP graph the same calls record a fork/join
// graph.  One library-owned non-blocking stream and an event ring per device.
namespace {
struct Side {
    hipStream_t s = nullptr;
    hipEvent_t ev[64] = {};
    int next = 0;
    bool ok = false;
};
Side g_side[64];

Side* side_stream() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    Side& sd = g_side[dev];
    if (!sd.ok) {
        if (hipStreamCreateWithFlags(&sd.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
        for (auto& e : sd.ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        sd.ok = true;
    }
    return &sd;
}

// `to` waits for everything issued so far on `from`
// Gradient readiness marks (spnerf_grad_marks): when armed, a backward records mark k's event
// on the stream that finishes that group of weight gradients — mark 0 after the output heads',
// 1 + (L-1-i) after trunk layer i's, L+1 at the end (per-ray parameters) — so that a data-parallel
// caller can all-reduce each group while the rest of the backward runs.  One event set per device.
// Inside a HIP-graph capture the marks are the graph's own dependency edges: the all-reduces must
// then be captured into the same graph (dp.GradBuckets).
struct Marks {
    hipEvent_t ev[64] = {};
    std::atomic<bool> ok{false};
    std::atomic<uint64_t> recorded{0};   // bit k: mark k recorded at least once since the events were made
};
Marks g_marks[64];
std::mutex g_marks_mu;                   // creation only (a watchdog thread may query concurrently)
int g_marks_armed = 0;
int g_marks_flags = hipEventDisableTiming;  // option "grad_marks_flags": hipEventCreateWithFlags flags (before the first arm)

// The mark events of device `dev`, created on first use when `create` (on that device: the
// calling thread's current device is the caller's, e.g. the rank's own GPU); nullptr when they do
// not exist and `create` is false — a query from another thread never creates them.
static Marks* marks_of(int dev, bool create) {
    if (dev < 0 || dev >= 64) return nullptr;
    Marks& m = g_marks[dev];
    if (m.ok.load(std::memory_order_acquire)) return &m;
    if (!create) return nullptr;
    std::lock_guard<std::mutex> lock(g_marks_mu);
    if (!m.ok.load(std::memory_order_relaxed)) {
        for (auto& e : m.ev)
            if (hipEventCreateWithFlags(&e, (unsigned)g_marks_flags) != hipSuccess) return nullptr;
        m.ok.store(true, std::memory_order_release);
    }
    return &m;
}

static Marks* marks_of_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    return marks_of(dev, true);
}

int g_tile_rowsum = 1;  // 1 = per-ray dZ sums by 64-point tiles (fused into the dX chain); 0 = k_ray_rowsum16

static int32_t grad_mark(int k, hipStream_t s) {
    if (!g_marks_armed) return SPNERF_OK;
    Marks* m = marks_of_device();
    SPN_ARG(m && k >= 0 && k < 64, "grad_mark: no mark events");
    // a plain record: under stream capture it becomes a dependency edge of the graph being
    // captured (a wait on it from another stream of the same capture joins that stream to the
    // graph); this HIP runtime refuses external event-record nodes (hipEventRecordExternal)
    SPN_HIP(hipEventRecord(m->ev[k], s));
    m->recorded.fetch_or(uint64_t(1) << k, std::memory_order_relaxed);
    return SPNERF_OK;
}

int32_t stream_dep(Side* sd, hipStream_t from, hipStream_t to) {
    if (!sd || from == to) return SPNERF_OK;
    hipEvent_t e = sd->ev[sd->next];
    sd->next = (sd->next + 1) % 64;
    SPN_HIP(hipEventRecord(e, from));
    SPN_HIP(hipStreamWaitEvent(to, e, 0));
    return SPNERF_OK;
}
}  // namespace
int g_l0_split = 1;       // bf16 MLP: fc_net.0 on bf16 hi/lo planes (0 = fp32 MFMA GEMM)
int g_trunk_l0 = 2;       // ... and inside the fused trunk launch: 1 = when nothing is saved (inference),
                          // 2 = also when saving (the default since round 4: the 64-point register-D training
                          // trunk with layer 0 against the separate hi/lo-plane GEMM + k_encode's planes:
                          // C4 26.56 / 26.58 -> 26.44 / 26.36 ms, C4@512 4.248 -> 4.202 ms, same call; it had
                          // measured 400 us slower on the round-2 trunk)

template <typename T> struct RawOf;
template <> struct RawOf<float> { using type = f32x4; };
template <> struct RawOf<bf16> { using type = u32x2; };
template <typename T>
__device__ __forceinline__ typename RawOf<T>::type ld_raw(const T* p) {
    return *reinterpret_cast<const typename RawOf<T>::type*>(p);
}

// The rows one point's heads read: its last trunk row (σ), sun_v.3 output, rgb / β hidden
// (Q) and semantic hidden (G); lane `l` holds columns 4l + 256i.
template <typename T, int NC, int NH>
struct HeadRows {
    typename RawOf<T>::type hl[NC], s3[NH], r1[NH], b1[NH], m1[NH];
    float sp;  // k_heads_fwd_v<…, SIGB>: the σ pre-activation from hsave
};

// Narrow output heads (spnerf.py:333-367): σ = softplus, albedo = sigmoid·1.002−0.001,
// sun = sigmoid, β = softplus, semantic logits; sky broadcast per ray.  One wavefront per
// point, W ≤ 256·NC.  HBM-latency bound, so the rows of point p + nw are in flight while
// point p's dot products and DPP reductions run: two register sets in turn (no copies, which
// would wait on the loads), a fixed number of row loads per point (rows a mode does not use
// are re-reads of the σ row, so the wait counts are static), and every other operand in
// registers or LDS (σ / sun / rgb / β weights in VGPRs, semantic weights staged in LDS) so no
// vector-memory load is issued behind the prefetch.  A point's output row leaves as one
// coalesced store.
// SIGB: the σ pre-activation comes from hsave[p·8], written by the fused training trunk with this
// kernel's own arithmetic (TrunkArgs::sig_hsave) — no H_L row is loaded
template <typename T, int NC, bool SIGB = false>
__global__ __launch_bounds__(256) void k_heads_fwd_v(HeadsArgs<T> a, PackedOffs k) {
    constexpr int NH = (NC + 1) / 2;
    extern __shared__ float wsem[];  // [C][H] semantic weights + [C] biases (mode 0, semantic model)
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const Dims& d = a.d;
    const float* Pk = a.packed;
    const int W = d.W, H = d.H;
    const bool sun_on = a.mode != 1, full = a.mode == 0, beta = full && d.beta, sem = full && d.sem;
    if (sem) {
        for (int i = threadIdx.x; i < d.C * H; i += 256) wsem[i] = Pk[k.Wm2 + i];
        if (threadIdx.x < d.C) wsem[d.C * H + threadIdx.x] = Pk[k.bm2 + threadIdx.x];
        __syncthreads();
    }
    int cw[NC], ch[NH];
    bool vw[NC], vh[NH];
#pragma unroll
    for (int i = 0; i < NC; ++i) {
        vw[i] = 4 * lane + 256 * i < W;
        cw[i] = vw[i] ? 4 * lane + 256 * i : 0;
    }
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        vh[i] = 4 * lane + 256 * i < H;
        ch[i] = vh[i] ? 4 * lane + 256 * i : 0;
    }
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    f32x4 wsg[NC], w4[NH], wr[3][NH], wb[NH];
#pragma unroll
    for (int i = 0; i < NC; ++i) wsg[i] = vw[i] ? ld4(Pk + k.wsig + cw[i]) : z4;
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        w4[i] = vh[i] && sun_on ? ld4(Pk + k.ws4 + ch[i]) : z4;
        for (int c = 0; c < 3; ++c) wr[c][i] = vh[i] && full ? ld4(Pk + k.Wr2 + c * H + ch[i]) : z4;
        wb[i] = vh[i] && beta ? ld4(Pk + k.wb2 + ch[i]) : z4;
    }
    const float bsig = Pk[k.bsig];
    const float bs4 = sun_on ? Pk[k.bs4] : 0.f;
    const float br0 = full ? Pk[k.br2] : 0.f, br1 = full ? Pk[k.br2 + 1] : 0.f, br2 = full ? Pk[k.br2 + 2] : 0.f;
    const float bb = beta ? Pk[k.bb2] : 0.f;

    // row bases of point p; unused rows alias the σ row (SIGB: the Q row)
    auto load = [&](int64_t p, HeadRows<T, NC, NH>& r) {
        const T* q = a.Q + p * d.NQ;
        const T* hl = SIGB ? q : a.HL + p * W;
        const T* s3 = sun_on ? a.S3 + p * H : hl;
        const T* r1 = full ? q + H : hl;
        const T* b1 = beta ? q + 2 * H : hl;
        const T* m1 = sem ? a.G + p * d.NG + W : hl;
        if constexpr (SIGB) {
            r.sp = a.hsave[p * 8];
        } else {
#pragma unroll
            for (int i = 0; i < NC; ++i) r.hl[i] = ld_raw(hl + cw[i]);
        }
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            r.s3[i] = ld_raw(s3 + ch[i]);
            r.r1[i] = ld_raw(r1 + ch[i]);
            r.b1[i] = ld_raw(b1 + ch[i]);
            r.m1[i] = ld_raw(m1 + ch[i]);
        }
    };

    auto body = [&](int64_t p, const HeadRows<T, NC, NH>& cur, HeadRows<T, NC, NH>& nxt) {
        // this point's sky colour before the prefetch, so waiting on it leaves the prefetch in flight
        float sky = 0.f;
        if (full && lane >= 5 && lane <= 7) sky = a.sky[(int64_t)((int)p / a.S) * 4 + lane - 5];
        load(std::min(p + nw, a.P - 1), nxt);
        // lane-partial dot products (masked columns carry zero weights)
        float ps = 0.f, pu = 0.f, pr0 = 0.f, pr1 = 0.f, pr2 = 0.f, pb = 0.f;
        if constexpr (!SIGB) {
#pragma unroll
            for (int i = 0; i < NC; ++i) ps += dot4(raw_f32(cur.hl[i]), wsg[i]);
        }
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            pu += dot4(raw_f32(cur.s3[i]), w4[i]);
            const f32x4 r = raw_f32(cur.r1[i]);
            pr0 += dot4(r, wr[0][i]);
            pr1 += dot4(r, wr[1][i]);
            pr2 += dot4(r, wr[2][i]);
            pb += dot4(raw_f32(cur.b1[i]), wb[i]);
        }
        const float spre = SIGB ? cur.sp : wave_total(ps) + bsig;
        float ov = lane == 3 ? softplusf_(spre) : 0.f;  // this lane's output column
        float hv = spre;                                // this lane's hsave column (lane 0: σ pre-activation)
        float* o = a.out + p * d.NO;
        float* hs = a.hsave + p * 8;
        if (!sun_on) {
            if (lane == 3) o[3] = ov;
            if (lane == 0) hs[0] = hv;
            return;
        }
        const float sun = sigmoidf_(wave_total(pu) + bs4);
        if (lane == 4) ov = hv = sun;
        if (full) {
            const float g0 = sigmoidf_(wave_total(pr0) + br0), g1 = sigmoidf_(wave_total(pr1) + br1),
                        g2 = sigmoidf_(wave_total(pr2) + br2);
            const float g = lane == 0 ? g0 : lane == 1 ? g1 : g2;
            if (lane < 3) ov = __fsub_rn(__fmul_rn(g, 1.002f), 0.001f);
            if (lane >= 1 && lane <= 3) hv = lane == 1 ? g0 : lane == 2 ? g1 : g2;  // hsave[1 + c] = rgb c
            if (lane >= 5 && lane <= 7) ov = sky;
            if (beta) {
                const float bpre = wave_total(pb) + bb;
                if (lane == 8) ov = softplusf_(bpre);
                if (lane == 5) hv = bpre;
            }
            if (sem) {
                for (int c = 0; c < d.C; ++c) {
                    float pm = 0.f;
#pragma unroll
                    for (int i = 0; i < NH; ++i)
                        pm += dot4(raw_f32(cur.m1[i]), vh[i] ? *reinterpret_cast<const f32x4*>(wsem + c * H + ch[i]) : z4);
                    const float v = wave_total(pm) + wsem[d.C * H + c];
                    if (lane == d.sem_col + c) ov = v;
                }
            }
        }
        if (lane < d.NO) o[lane] = ov;
        if (lane == 0 || lane == 4 || (full && (lane <= 3 || (lane == 5 && d.beta)))) hs[lane] = hv;
    };

    // the point index is wave-uniform: keep it (and every row address) in scalar registers;
    // P < 2^31 (spnerf_mlp_forward checks it)
    int64_t p = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
    if (p >= a.P) return;
    // two register sets in turn (a third, prefetching two points ahead, measured no faster)
    HeadRows<T, NC, NH> ra, rb;
    load(p, ra);
    for (;;) {
        body(p, ra, rb);
        if ((p += nw) >= a.P) break;
        body(p, rb, ra);
        if ((p += nw) >= a.P) break;
    }
}

template <typename T>
struct HeadsBwdArgs {
    const float* packed; Dims d;
    const float *d_out, *hsave;
    const T *DQ, *DG, *DS3;
    float* hpre;
    T *dZQ, *dZG, *dS3;
    int64_t P; int mode;
    int emu = 0;  // precision study (fp32 only): the dX outputs rounded to bf16
};

// Backward of the narrow heads, one wavefront per point: per-point pre-activation gradients
// (hpre, reduced over points into the head weights by the skinny reduction) and the
// gradients of the hidden layers feeding them (dX = dY·W, × sin' saved in D*), written as
// coalesced rows.
template <typename T>
__global__ __launch_bounds__(256) void k_heads_bwd(HeadsBwdArgs<T> a, PackedOffs k) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const Dims& d = a.d;
    const float* Pk = a.packed;
    const int H = d.H;
    for (int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < a.P; p += nw) {
        const float* g = a.d_out + p * d.NO;
        const float* hs = a.hsave + p * 8;
        float* hp = a.hpre + p * d.HP;
        const float dsig = softplus_grad(g[3], hs[0]);
        float dys = 0.f, dy[3] = {0.f, 0.f, 0.f}, db = 0.f;
        if (a.mode != 1) {
            const float s = hs[4];
            dys = g[4] * (1.f - s) * s;
        }
        if (a.mode == 0) {
            for (int c = 0; c < 3; ++c) {
                const float s = hs[1 + c];
                dy[c] = g[c] * 1.002f * (1.f - s) * s;
            }
            if (d.beta) db = softplus_grad(g[8], hs[5]);
        }
        for (int c = lane; c < d.HP; c += 64) {
            float v = 0.f;
            if (c == 0) v = dsig;
            else if (c <= 3) v = dy[c - 1];
            else if (c == 4) v = dys;
            else if (c == 5) v = db;
            else if (a.mode == 0) v = g[d.sem_col + c - 6];
            hp[c] = v;
        }
        if (a.mode == 1) continue;
        for (int c = 4 * lane; c < H; c += 256) {
            const f32x4 D = ld4(a.DS3 + p * H + c);
            const f32x4 w = *reinterpret_cast<const f32x4*>(Pk + k.ws4 + c);
            st4(a.dS3 + p * H + c, (dys * w) * D);
        }
        if (a.mode == 2) continue;
        for (int c = 4 * lane; c < H; c += 256) {
            const f32x4 D = ld4(a.DQ + p * d.NQ + H + c);
            const f32x4 w0 = *reinterpret_cast<const f32x4*>(Pk + k.Wr2 + c);
            const f32x4 w1 = *reinterpret_cast<const f32x4*>(Pk + k.Wr2 + H + c);
            const f32x4 w2 = *reinterpret_cast<const f32x4*>(Pk + k.Wr2 + 2 * H + c);
            st4(a.dZQ + p * d.NQ + H + c, (dy[0] * w0 + dy[1] * w1 + dy[2] * w2) * D);
            if (d.beta) {
                const f32x4 Db = ld4(a.DQ + p * d.NQ + 2 * H + c);
                const f32x4 wb = *reinterpret_cast<const f32x4*>(Pk + k.wb2 + c);
                st4(a.dZQ + p * d.NQ + 2 * H + c, (db * wb) * Db);
            }
            if (d.sem) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                for (int j = 0; j < d.C; ++j)
                    acc += g[d.sem_col + j] * *reinterpret_cast<const f32x4*>(Pk + k.Wm2 + j * H + c);
                const f32x4 Dm = ld4(a.DG + p * d.NG + d.W + c);
                st4(a.dZG + p * d.NG + d.W + c, acc * Dm);
            }
        }
    }
}

// k_heads_bwd with the latency structure of k_heads_fwd_v: the d_out row, the hsave row and
// the D rows of point p + nw load into a second register set while point p computes (two sets
// in turn), the d_out / hsave values come from one coalesced load each (lane c holds column c,
// read back with readlane), the head weights sit in VGPRs / LDS.  Same arithmetic per element
// as k_heads_bwd (bit-identical).  H ≤ 256·NH.
template <typename T, int NH>
__global__ __launch_bounds__(256) void k_heads_bwd_v(HeadsBwdArgs<T> a, PackedOffs k) {
    extern __shared__ float wsem[];  // [C][H] semantic weights (mode 0, semantic model)
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * 4;
    const Dims& d = a.d;
    const float* Pk = a.packed;
    const int H = d.H;
    const bool sun_on = a.mode != 1, full = a.mode == 0, beta = full && d.beta, sem = full && d.sem;
    if (sem) {
        for (int i = threadIdx.x; i < d.C * H; i += 256) wsem[i] = Pk[k.Wm2 + i];
        __syncthreads();
    }
    int ch[NH];
    bool vh[NH];
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        vh[i] = 4 * lane + 256 * i < H;
        ch[i] = vh[i] ? 4 * lane + 256 * i : 0;
    }
    const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
    f32x4 w4[NH], wr[3][NH], wb[NH];
#pragma unroll
    for (int i = 0; i < NH; ++i) {
        w4[i] = vh[i] && sun_on ? ld4(Pk + k.ws4 + ch[i]) : z4;
        for (int c = 0; c < 3; ++c) wr[c][i] = vh[i] && full ? ld4(Pk + k.Wr2 + c * H + ch[i]) : z4;
        wb[i] = vh[i] && beta ? ld4(Pk + k.wb2 + ch[i]) : z4;
    }
    struct Rows {
        float g, h;  // lane c: d_out[c] (c < NO), hsave[c] (c < 8)
        typename RawOf<T>::type s3[NH], qr[NH], qb[NH], gm[NH];
    };
    auto load = [&](int64_t p, Rows& r) {
        r.g = a.d_out[p * d.NO + min(lane, d.NO - 1)];
        r.h = a.hsave[p * 8 + (lane & 7)];
        if (sun_on) {
#pragma unroll
            for (int i = 0; i < NH; ++i) r.s3[i] = ld_raw(a.DS3 + p * H + ch[i]);
        }
        if (full) {
#pragma unroll
            for (int i = 0; i < NH; ++i) {
                r.qr[i] = ld_raw(a.DQ + p * d.NQ + H + ch[i]);
                if (beta) r.qb[i] = ld_raw(a.DQ + p * d.NQ + 2 * H + ch[i]);
                if (sem) r.gm[i] = ld_raw(a.DG + p * d.NG + d.W + ch[i]);
            }
        }
    };
    auto col = [](float v, int c) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), c)); };
    auto body = [&](int64_t p, const Rows& cur, Rows& nxt) {
        load(std::min(p + nw, a.P - 1), nxt);
        const float dsig = softplus_grad(col(cur.g, 3), col(cur.h, 0));
        float dys = 0.f, dy[3] = {0.f, 0.f, 0.f}, db = 0.f;
        if (sun_on) {
            const float s = col(cur.h, 4);
            dys = col(cur.g, 4) * (1.f - s) * s;
        }
        if (full) {
            for (int c = 0; c < 3; ++c) {
                const float s = col(cur.h, 1 + c);
                dy[c] = col(cur.g, c) * 1.002f * (1.f - s) * s;
            }
            if (d.beta) db = softplus_grad(col(cur.g, 8), col(cur.h, 5));
        }
        // hpre row [dσ, drgb3, dsun, dβ, dsem C]: lane c; the semantic gradients are d_out's
        // columns sem_col + c - 6, shifted across lanes
        const float gs = __shfl(cur.g, min(d.sem_col + lane - 6 + 64, 63 + 64) - 64, 64);
        if (lane < d.HP) {
            float v = 0.f;
            if (lane == 0) v = dsig;
            else if (lane <= 3) v = dy[lane - 1];
            else if (lane == 4) v = dys;
            else if (lane == 5) v = db;
            else if (full) v = gs;
            a.hpre[p * d.HP + lane] = v;
        }
        if (!sun_on) return;
        auto st = [&](T* q, f32x4 v) {
            if (a.emu)
                for (int e = 0; e < 4; ++e) v[e] = (float)(bf16)v[e];
            st4(q, v);
        };
#pragma unroll
        for (int i = 0; i < NH; ++i)
            if (vh[i]) st(a.dS3 + p * H + ch[i], (dys * w4[i]) * raw_f32(cur.s3[i]));
        if (!full) return;
#pragma unroll
        for (int i = 0; i < NH; ++i) {
            if (!vh[i]) continue;
            st(a.dZQ + p * d.NQ + H + ch[i], (dy[0] * wr[0][i] + dy[1] * wr[1][i] + dy[2] * wr[2][i]) * raw_f32(cur.qr[i]));
            if (d.beta) st(a.dZQ + p * d.NQ + 2 * H + ch[i], (db * wb[i]) * raw_f32(cur.qb[i]));
            if (d.sem) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
                for (int j = 0; j < d.C; ++j)
                    acc += col(cur.g, d.sem_col + j) * *reinterpret_cast<const f32x4*>(wsem + j * H + ch[i]);
                st(a.dZG + p * d.NG + d.W + ch[i], acc * raw_f32(cur.gm[i]));
            }
        }
    };
    int64_t p = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6));
    if (p >= a.P) return;
    Rows ra, rb;
    load(p, ra);
    for (;;) {
        body(p, ra, rb);
        if ((p += nw) >= a.P) break;
        body(p, rb, ra);
        if ((p += nw) >= a.P) break;
    }
}

// out[ray][n] = Σ_{s<S} in[(ray*S + s)*ld + c0 + n]
template <typename T>
__global__ void k_ray_rowsum(const T* __restrict__ in, int ld, int c0, int N, int S, float* __restrict__ out,
                             int ldo) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ray = blockIdx.y;
    if (n >= N) return;
    const T* p = in + ray * S * (int64_t)ld + c0 + n;
    float s = 0.f;
    for (int i = 0; i < S; ++i) s += ld1(p + (int64_t)i * ld);
    out[ray * ldo + n] = s;
}

// Same sum for bf16 rows with N, ld, c0 multiples of 8: one block per ray, a thread owns 8
// columns (16-B loads) in one of 256/(N/8) row phases; phases combined in a fixed order.  A
// thread's rows load 8 at a time before they are summed (in the same order): one HBM latency per
// 8 rows instead of one per row (two launches per step: C4 0.138 -> 0.135 ms, C4@512 0.044 ->
// 0.037 ms, bit-identical; the same batching in the skinny reductions measured level)
__global__ __launch_bounds__(256) void k_ray_rowsum16(const bf16* __restrict__ in, int ld, int c0, int N, int S,
                                                      float* __restrict__ out, int ldo) {
    __shared__ float part[256 * 8];
    const int64_t ray = blockIdx.x;
    const int nq = N >> 3;                   // column chunks (<= 256)
    const int ph = threadIdx.x / nq, q = threadIdx.x % nq;
    const int nph = 256 / nq;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ph < nph) {
        const bf16* p = in + ray * S * (int64_t)ld + c0 + 8 * q;
        for (int i0 = ph; i0 < S; i0 += 8 * nph) {
            u32x4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * nph;
                v[u] = i < S ? ldg16(p + (int64_t)i * ld) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (i0 + u * nph < S) {
                    float f[8];
                    unpack8(v[u], f);
#pragma unroll
                    for (int e = 0; e < 8; ++e) acc[e] += f[e];
                }
            }
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[threadIdx.x * 8 + e] = acc[e];
    __syncthreads();
    if (threadIdx.x < nq) {
        float r[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) r[e] = part[threadIdx.x * 8 + e];
        for (int k = 1; k < nph; ++k)
#pragma unroll
            for (int e = 0; e < 8; ++e) r[e] += part[(k * nq + threadIdx.x) * 8 + e];
#pragma unroll
        for (int e = 0; e < 8; ++e) out[ray * ldo + 8 * threadIdx.x + e] = r[e];
    }
}

// The per-ray sums of the 512-wide trunk dZ in the fused backward's order (S % 64 == 0): per
// 64-point tile the column sums of tile_colsum_part / _final (trunk.h), read from HBM here (the
// layer-by-layer backward; k_trunk_bwd_bf16 forms them from its LDS image) ...
__global__ __launch_bounds__(512) void k_tile_rowsum16(const bf16* __restrict__ in, float* __restrict__ part_out) {
    __shared__ float part[8 * 512];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const bf16* src = in + ((int64_t)blockIdx.x * 64 + 8 * w) * 512 + 8 * lane;
    u32x4 rows[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) rows[r] = ldg16(src + r * 512);
    float a[8];
    tile_colsum_part(rows, a);
    *reinterpret_cast<f32x4*>(part + w * 512 + lane * 8) = f32x4{a[0], a[1], a[2], a[3]};
    *reinterpret_cast<f32x4*>(part + w * 512 + lane * 8 + 4) = f32x4{a[4], a[5], a[6], a[7]};
    __syncthreads();
    part_out[(int64_t)blockIdx.x * 512 + tid] = tile_colsum_final(part, tid);
}

// ... and the T tiles of a ray added in tile order: out[ray][c] = Σ_t part[ray·T + t][c]
// (blockIdx.y = 1: the second part / output pair — layer 0 and the skip layer in one launch)
__global__ __launch_bounds__(256) void k_ray_tiles_sum(const float* __restrict__ part0, int T, int64_t n_rays,
                                                       float* __restrict__ out0, const float* __restrict__ part1,
                                                       float* __restrict__ out1) {
    const float* part = blockIdx.y ? part1 : part0;
    float* out = blockIdx.y ? out1 : out0;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n_rays * 512) return;
    const int64_t ray = i >> 9;
    const int c = (int)(i & 511);
    const float* p = part + ray * T * 512 + c;
    float s = p[0];
    for (int t = 1; t < T; ++t) s += p[t * 512];
    out[i] = s;
}

struct RayBwdArgs {
    const float* packed; PackedOffs k; Dims d;
    const float *sky, *skyh, *R0, *R4, *RQ;
    const float* d_out; int NO, S;   // the points' output gradients (sky columns 5..7)
    const int64_t* labels;
    float *skyd, *skydh, *gemb, *embr, *grad_t;
    int sem_on, beta_on, sky_on;
};

// Per-ray backward pieces: sky MLP pre-activation grads, the semantic-embedding input grad
// and the time-embedding input grad.  One 256-thread block per ray.  The sky colour's gradient
// is the sum of d_out's sky columns over the ray's samples (the sky is per ray, broadcast to every
// sample: spnerf.py:244-249): wave c sums column c, its lanes strided over the samples (a separate
// one-thread-per-column launch walked the 128 samples serially: 50 us per C4 step).
__global__ __launch_bounds__(256) void k_ray_bwd(RayBwdArgs a) {
    const int64_t ray = blockIdx.x;
    const int tid = threadIdx.x;
    const Dims& d = a.d;
    const float* P = a.packed;
    if (a.sky_on) {
        __shared__ float dsk[3];
        if ((tid >> 6) < 3) {
            const int c = tid >> 6, lane = tid & 63;
            const float* q = a.d_out + ray * a.S * (int64_t)a.NO + 5 + c;
            float v = 0.f;
            for (int s = lane; s < a.S; s += 64) v += q[(int64_t)s * a.NO];
            v = wave_sum(v);
            if (lane == 0) dsk[c] = v;
        }
        __syncthreads();
        float dp[3];
        for (int c = 0; c < 3; ++c) {
            const float s = a.sky[ray * 4 + c];
            dp[c] = dsk[c] * (1.f - s) * s;
        }
        if (tid < 3) a.skyd[ray * 4 + tid] = dp[tid];
        for (int n = tid; n < d.H; n += blockDim.x) {
            const float hv = a.skyh[ray * d.H + n];
            const float g = dp[0] * P[a.k.Wk2 + n] + dp[1] * P[a.k.Wk2 + d.H + n] + dp[2] * P[a.k.Wk2 + 2 * d.H + n];
            a.skydh[ray * d.H + n] = hv > 0.f ? g : 0.f;
        }
    }
    __shared__ float red[256];
    if (a.sem_on) {
        int64_t lab = a.labels[ray];
        if (lab == -100) lab = d.C;
        for (int j = tid; j < d.sd; j += blockDim.x) a.embr[ray * d.sd + j] = P[a.k.emb + lab * d.sd + j];
        for (int j = 0; j < d.sd; ++j) {
            float acc = 0.f;
            for (int n = tid; n < d.W; n += blockDim.x)
                acc += a.R0[ray * d.W + n] * P[a.k.Wsem0 + (int64_t)n * d.sd + j] +
                       a.R4[ray * d.W + n] * P[a.k.Wsem4 + (int64_t)n * d.sd + j];
            red[tid] = acc;
            __syncthreads();
            for (int st = 128; st > 0; st >>= 1) {
                if (tid < st) red[tid] += red[tid + st];
                __syncthreads();
            }
            if (tid == 0) a.gemb[ray * d.sd + j] = red[0];
            __syncthreads();
        }
    }
    if (a.beta_on && a.grad_t) {
        for (int j = 0; j < d.td; ++j) {
            float acc = 0.f;
            for (int n = tid; n < d.H; n += blockDim.x)
                acc += a.RQ[ray * d.NQ + 2 * d.H + n] * P[a.k.Wtt + (int64_t)n * d.td + j];
            red[tid] = acc;
            __syncthreads();
            for (int st = 128; st > 0; st >>= 1) {
                if (tid < st) red[tid] += red[tid + st];
                __syncthreads();
            }
            if (tid == 0) a.grad_t[ray * d.td + j] = red[0];
            __syncthreads();
        }
    }
}

// d_emb[c][j] = Σ_{rays with label c} gemb[ray][j]; the padding row (−100 → C) gets none
// (nn.Embedding padding_idx, spnerf.py:191-194).
// One block per (class, j): rays strided over 256 threads, then a fixed-order tree in LDS.
__global__ __launch_bounds__(256) void k_class_sum(int64_t B, const float* __restrict__ gemb, int sd,
                                                   const int64_t* __restrict__ labels, int C, float* __restrict__ out,
                                                   int accumulate) {
    __shared__ float red[256];
    const int c = blockIdx.x / sd, j = blockIdx.x % sd;
    float s = 0.f;
    if (c < C)
        for (int64_t r = threadIdx.x; r < B; r += 256)
            if (labels[r] == c) s += gemb[r * sd + j];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = accumulate ? out[blockIdx.x] + red[0] : red[0];
}

// ------------------------------------------------------------------------------------------
// host orchestration
// ------------------------------------------------------------------------------------------

// Device-resident piece tables, one per distinct model layout (the parameters' addresses go in
// the launch's kernarg PackSrcs, so every model of one configuration shares a table), built on
// first use outside a stream capture and never freed (a captured graph may hold one); option
// pack_table 0 = the kernarg tables only
int g_pack_table = 1;
struct PackTable {
    int dev;
    std::vector<PackPiece> key;
    PackPiece* d_pcs;
    int2* d_blk;   // per block: {piece, tile of the piece}
    int tiles;
};
static std::mutex g_pack_mu;
static std::deque<PackTable> g_pack_tables;   // deque: the returned pointers stay valid

static const PackTable* pack_table(const std::vector<PackPiece>& pieces0, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::vector<PackPiece> pieces = pieces0;   // the key: layout only
    for (PackPiece& p : pieces) {
        if (p.src_idx < 0 || p.src_idx >= kPackParams) return nullptr;
        p.src = nullptr;
    }
    std::lock_guard<std::mutex> lk(g_pack_mu);
    for (const PackTable& t : g_pack_tables)
        if (t.dev == dev && t.key.size() == pieces.size() &&
            std::memcmp(t.key.data(), pieces.data(), pieces.size() * sizeof(PackPiece)) == 0)
            return &t;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    if (g_pack_tables.size() >= 64) return nullptr;
    std::vector<int2> blk;
    for (size_t i = 0; i < pieces.size(); ++i) {
        const int nt = cdiv(pieces[i].rows, kPackTR) * cdiv(pieces[i].cols, kPackTC);
        for (int t = 0; t < nt; ++t) blk.push_back(make_int2((int)i, t));
    }
    if (blk.empty()) return nullptr;
    PackTable t{dev, pieces, nullptr, nullptr, (int)blk.size()};
    if (hipMalloc(&t.d_pcs, pieces.size() * sizeof(PackPiece)) != hipSuccess) return nullptr;
    if (hipMalloc(&t.d_blk, blk.size() * sizeof(int2)) != hipSuccess ||
        hipMemcpy(t.d_pcs, pieces.data(), pieces.size() * sizeof(PackPiece), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(t.d_blk, blk.data(), blk.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(t.d_pcs);
        if (t.d_blk) (void)hipFree(t.d_blk);
        return nullptr;
    }
    g_pack_tables.push_back(t);
    return &g_pack_tables.back();
}

static int32_t launch_pack(const std::vector<PackPiece>& pieces, float* packed, hipStream_t s) {
    if (g_pack_table && pieces.size() > (size_t)kMaxPieces) {
        if (const PackTable* t = pack_table(pieces, s)) {
            PackSrcs srcs{};
            for (const PackPiece& p : pieces) srcs.p[p.src_idx] = p.src;
            ProfScope prof("pack", s, 0.0, 0.0);
            hipLaunchKernelGGL(k_pack_dev, dim3(t->tiles), dim3(256), 0, s, t->d_pcs, t->d_blk, packed, srcs);
            SPN_HIP(hipGetLastError());
            return SPNERF_OK;
        }
    }
    for (size_t b = 0; b < pieces.size(); b += kMaxPieces) {
        PackArgs a{};
        a.packed = packed;
        int n = 0, tiles = 0;
        for (size_t i = b; i < pieces.size() && n < kMaxPieces; ++i, ++n) {
            a.p[n] = pieces[i];
            a.tile0[n] = tiles;
            tiles += cdiv(pieces[i].rows, kPackTR) * cdiv(pieces[i].cols, kPackTC);
        }
        a.tile0[n] = tiles;
        a.n = n;
        ProfScope prof("pack", s, 0.0, 0.0);
        hipLaunchKernelGGL(k_pack, dim3(tiles), dim3(256), 0, s, a);
        SPN_HIP(hipGetLastError());
    }
    return SPNERF_OK;
}

static int32_t pack_params(const Dims& d, const float* const* prm, float* packed, hipStream_t s) {
    PIdx x;
    auto specs = param_specs(d, &x);
    const Packed k = packed_layout(d);
    std::vector<PackPiece> v;
    auto piece = [&](int pi, int c0, int rows, int cols, int64_t dst, int dst_ld, int tr, int bf = 0) {
        SPN_ARG(prm[pi] != nullptr, "parameter %s is NULL", specs[pi].name.c_str());
        v.push_back(PackPiece{prm[pi], (int)specs[pi].ld(), c0, rows, cols, dst_ld, tr, bf, pi, dst});
        return SPNERF_OK;
    };
    const int W = d.W, H = d.H;
    // precision study: the fp32 MLP's GEMM weights rounded to bf16 (as the bf16 MLP packs them)
    const bool rnd16 = !d.bf && (g_emu_bf16 & 4);
    auto mark = [&]() { v.back().rnd = rnd16 ? 1 : 0; };
    for (int i = 0; i < d.L; ++i) {
        const int kreal = i == 0 ? d.K0 : (i == d.skip ? W + d.K0 : W);
        SPN_TRY(piece(x.fcW[i], 0, W, kreal, k.Wt[i], k.Kp[i], 0));
        if (i > 0) mark();
        SPN_TRY(piece(x.fcb[i], 0, 1, W, k.bt[i], W, 0));
        if (i > 0) {
            SPN_TRY(piece(x.fcW[i], 0, W, W, k.WTt[i], W, 1));
            mark();
        }
    }
    if (d.sem) {
        SPN_TRY(piece(x.fcW[0], d.K0, W, d.sd, k.Wsem0, d.sd, 0));
        SPN_TRY(piece(x.fcW[d.skip], W + d.K0, W, d.sd, k.Wsem4, d.sd, 0));
        SPN_TRY(piece(x.emb, 0, d.C + 1, d.sd, k.emb, d.sd, 0));
        SPN_TRY(piece(x.m1W, 0, H, W, k.WG + (int64_t)W * W, W, 0));
        mark();
        SPN_TRY(piece(x.m1b, 0, 1, H, k.bG + W, H, 0));
        SPN_TRY(piece(x.m1W, 0, H, W, k.WGT + W, d.NG, 1));
        mark();
        SPN_TRY(piece(x.m2W, 0, d.C, H, k.Wm2, H, 0));
        SPN_TRY(piece(x.m2b, 0, 1, d.C, k.bm2, d.C, 0));
    }
    SPN_TRY(piece(x.featW, 0, W, W, k.WG, W, 0));
    mark();
    SPN_TRY(piece(x.featb, 0, 1, W, k.bG, W, 0));
    SPN_TRY(piece(x.featW, 0, W, W, k.WGT, d.NG, 1));
    mark();
    SPN_TRY(piece(x.s1W, 0, H, W, k.WQ, W, 0));
    mark();
    SPN_TRY(piece(x.r1W, 0, H, W, k.WQ + (int64_t)H * W, W, 0));
    mark();
    SPN_TRY(piece(x.s1b, 0, 1, H, k.bQ, H, 0));
    SPN_TRY(piece(x.r1b, 0, 1, H, k.bQ + H, H, 0));
    SPN_TRY(piece(x.s1W, 0, H, W, k.WQT, d.NQ, 1));
    mark();
    SPN_TRY(piece(x.r1W, 0, H, W, k.WQT + H, d.NQ, 1));
    mark();
    SPN_TRY(piece(x.s1W, W, H, 3, k.Wsun, 3, 0));
    if (d.beta) {
        SPN_TRY(piece(x.b1W, 0, H, W, k.WQ + (int64_t)2 * H * W, W, 0));
        SPN_TRY(piece(x.b1b, 0, 1, H, k.bQ + 2 * H, H, 0));
        SPN_TRY(piece(x.b1W, 0, H, W, k.WQT + 2 * H, d.NQ, 1));
        SPN_TRY(piece(x.b1W, W, H, d.td, k.Wtt, d.td, 0));
        SPN_TRY(piece(x.b2W, 0, 1, H, k.wb2, H, 0));
        SPN_TRY(piece(x.b2b, 0, 1, 1, k.bb2, 1, 0));
    }
    SPN_TRY(piece(x.s2W, 0, H, H, k.Ws2, H, 0));
    mark();
    SPN_TRY(piece(x.s2b, 0, 1, H, k.bs2, H, 0));
    SPN_TRY(piece(x.s2W, 0, H, H, k.Ws2T, H, 1));
    mark();
    SPN_TRY(piece(x.s3W, 0, H, H, k.Ws3, H, 0));
    mark();
    SPN_TRY(piece(x.s3b, 0, 1, H, k.bs3, H, 0));
    SPN_TRY(piece(x.s3W, 0, H, H, k.Ws3T, H, 1));
    mark();
    SPN_TRY(piece(x.sigW, 0, 1, W, k.wsig, W, 0));
    SPN_TRY(piece(x.sigb, 0, 1, 1, k.bsig, 1, 0));
    SPN_TRY(piece(x.r2W, 0, 3, H, k.Wr2, H, 0));
    SPN_TRY(piece(x.r2b, 0, 1, 3, k.br2, 3, 0));
    SPN_TRY(piece(x.s4W, 0, 1, H, k.ws4, H, 0));
    SPN_TRY(piece(x.s4b, 0, 1, 1, k.bs4, 1, 0));
    SPN_TRY(piece(x.k1W, 0, H, 3, k.Wk1, 3, 0));
    SPN_TRY(piece(x.k1b, 0, 1, H, k.bk1, H, 0));
    SPN_TRY(piece(x.k2W, 0, 3, H, k.Wk2, H, 0));
    SPN_TRY(piece(x.k2b, 0, 1, 3, k.bk2, 3, 0));
    if (d.bf) {  // bf16 GEMM operands (same shapes as their fp32 counterparts above)
        SPN_TRY(piece(x.fcW[0], 0, W, d.K0, k.W0s16, 4 * k.Kp[0], 0, 3));
        if (k.Wf16[0] >= 0) SPN_TRY(piece(x.fcW[0], 0, W, d.K0, k.Wf16[0], 4 * k.Kp[0], 0, 4));
        for (int i = 1; i < d.L; ++i) {
            const int kreal = i == d.skip ? W + d.K0 : W;
            SPN_TRY(piece(x.fcW[i], 0, W, kreal, k.Wt16[i], k.Kp[i], 0, 1));
            SPN_TRY(piece(x.fcW[i], 0, W, W, k.WTt16[i], W, 1, 1));
            if (k.Wf16[i] >= 0) SPN_TRY(piece(x.fcW[i], 0, W, kreal, k.Wf16[i], k.Kp[i], 0, 2));
            if (k.Wb16[i] >= 0) SPN_TRY(piece(x.fcW[i], 0, W, W, k.Wb16[i], W, 1, 2));
        }
        if (d.sem) {
            SPN_TRY(piece(x.m1W, 0, H, W, k.WG16 + (int64_t)W * W, W, 0, 1));
            SPN_TRY(piece(x.m1W, 0, H, W, k.WGT16 + W, d.NG, 1, 1));
        }
        SPN_TRY(piece(x.featW, 0, W, W, k.WG16, W, 0, 1));
        SPN_TRY(piece(x.featW, 0, W, W, k.WGT16, d.NG, 1, 1));
        SPN_TRY(piece(x.s1W, 0, H, W, k.WQ16, W, 0, 1));
        SPN_TRY(piece(x.r1W, 0, H, W, k.WQ16 + (int64_t)H * W, W, 0, 1));
        SPN_TRY(piece(x.s1W, 0, H, W, k.WQT16, d.NQ, 1, 1));
        SPN_TRY(piece(x.r1W, 0, H, W, k.WQT16 + H, d.NQ, 1, 1));
        if (d.beta) {
            SPN_TRY(piece(x.b1W, 0, H, W, k.WQ16 + (int64_t)2 * H * W, W, 0, 1));
            SPN_TRY(piece(x.b1W, 0, H, W, k.WQT16 + 2 * H, d.NQ, 1, 1));
        }
        SPN_TRY(piece(x.s2W, 0, H, H, k.Ws2_16, H, 0, 1));
        SPN_TRY(piece(x.s2W, 0, H, H, k.Ws2T16, H, 1, 1));
        SPN_TRY(piece(x.s3W, 0, H, H, k.Ws3_16, H, 0, 1));
        SPN_TRY(piece(x.s3W, 0, H, H, k.Ws3T16, H, 1, 1));
        if (k.Ffeat16 >= 0) {  // the fused inference heads' fragment streams
            if (d.sem) SPN_TRY(piece(x.m1W, 0, H, W, k.Fsem16, W, 0, 5));
            SPN_TRY(piece(x.featW, 0, W, W, k.Ffeat16, W, 0, 2));
            SPN_TRY(piece(x.s1W, 0, H, W, k.FQ16, W, 0, 2));
            SPN_TRY(piece(x.r1W, 0, H, W, k.FQ16 + (int64_t)H * W, W, 0, 2));  // rows H.. of Q (64-row waves)
            SPN_TRY(piece(x.s2W, 0, H, H, k.Fs2_16, H, 0, 5));
            SPN_TRY(piece(x.s3W, 0, H, H, k.Fs3_16, H, 0, 5));
            SPN_TRY(piece(x.s1W, 0, H, W, k.FQs16, W, 0, 5));   // the solar pass's Q (sun_v.0 alone)
            auto narrow = [&](int pi, int nsrc, int K, int64_t dst) {
                SPN_TRY(piece(pi, 0, 32, K, dst, K, 0, 6));
                v.back().nsrc = nsrc;
                return SPNERF_OK;
            };
            SPN_TRY(narrow(x.sigW, 1, W, k.Fnar16));
            SPN_TRY(narrow(x.r2W, 3, H, k.Fnar16 + (int64_t)32 * W));
            SPN_TRY(narrow(x.s4W, 1, H, k.Fnar16 + (int64_t)32 * (W + H)));
        }
        if (k.BG16 >= 0) {  // the heads' fused dX chain: transposed, fragment order
            SPN_TRY(piece(x.s3W, 0, H, H, k.Bs3_16, H, 1, 5));
            SPN_TRY(piece(x.s2W, 0, H, H, k.Bs2_16, H, 1, 5));
            // K index q of Q: sun_v.0 rows, then rgb.0 rows (k += H: (H / 16) k-steps of 2 · 512)
            SPN_TRY(piece(x.s1W, 0, H, W, k.BQ16, d.NQ, 1, 7));
            SPN_TRY(piece(x.r1W, 0, H, W, k.BQ16 + (int64_t)(H / 16) * 2 * 512, d.NQ, 1, 7));
            SPN_TRY(piece(x.featW, 0, W, W, k.BG16, d.NG, 1, 7));
            if (d.sem) SPN_TRY(piece(x.m1W, 0, H, W, k.BG16 + (int64_t)(W / 16) * 2 * 512, d.NG, 1, 7));
        }
    }
    return launch_pack(v, packed, s);
}

namespace {
struct Ctx {
    Dims d;
    Packed k;
    WS w;
    const float* P;  // packed
    float* ws;       // workspace base
    int S;
    int acc = 0;     // backward: gradient reductions add into the flat gradient
    int defer = 0;   // backward: the trunk layers' weight gradients are left to spnerf_mlp_trunk_wgrad
    // the forward's ray inputs (the fused inference trunk encodes layer 0's input itself)
    const float* rays = nullptr;
    const float* z = nullptr;
    int rs = 0, dir_off = 0;
    int ldz = 0;                    // z's row stride per ray (S: contiguous rows)
    float* out = nullptr;           // the forward's output rows (the fused trunk + heads write them)
    bool* heads_done = nullptr;     // set when the trunk launch ran the fused heads too
    bool* heads_epi_done = nullptr;  // set when the head GEMMs' epilogues wrote the narrow heads
    float* at(int64_t off) const { return ws + off; }
    const float* pk(int64_t off) const { return P + off; }
    bf16* hb(int64_t off) const { return reinterpret_cast<bf16*>(ws + off); }          // bf16 workspace buffer
    const bf16* pk16(int64_t off) const { return reinterpret_cast<const bf16*>(P) + off; }  // bf16 packed weights
};
}  // namespace

// dtype dispatch for the GEMM sequence: fp32 (NTArgs / TNArgs) or bf16 (NT16Args / TN16Args,
// same field names); T is the activation element type.
template <typename T>
struct Gemms;
template <>
struct Gemms<float> {
    using NT = NTArgs;
    using TN = TNArgs;
    static float* buf(const Ctx& c, int64_t off) { return c.at(off); }
    static const float* w(const Ctx& c, int64_t off32, int64_t) { return c.pk(off32); }
    static int32_t nt(const NT& a, hipStream_t s) { return gemm_nt(a, s); }
    static int splits(int P, int N, int K) { return tn_splits(P, N, K); }
    static int32_t tn(const TN& a, int sp, hipStream_t s) { return gemm_tn(a, sp, s); }
};
template <>
struct Gemms<bf16> {
    using NT = NT16Args;
    using TN = TN16Args;
    static bf16* buf(const Ctx& c, int64_t off) { return c.hb(off); }
    static const bf16* w(const Ctx& c, int64_t, int64_t off16) { return c.pk16(off16); }
    static int32_t nt(const NT& a, hipStream_t s) { return gemm_nt_bf16(a, s); }
    static int splits(int P, int N, int K) { return tn_splits_bf16(P, N, K); }
    static int32_t tn(const TN& a, int sp, hipStream_t s) { return gemm_tn_bf16(a, sp, s); }
};

int g_tn_split_tail = 1;  // option "tn_split_tail": see tn_grad
// option "tn_group": deferred weight-gradient GEMMs per launch (trunk_wgrad; 1 = one launch each).
// All 9 of a W = 512 model (sun_v_net.4 / .2, trunk layers 7 .. 1) in one launch: C4 at 512 rays
// 4.252 / 4.288 -> 4.033 / 4.036 ms, at 4 096 rays 26.57 / 26.49 -> 26.50 / 26.45 (same call; the
// slab reductions 0.35 -> 0.22 ms per step)
int g_tn_group = 9;
// option "tn_group_rounds": a group launch's blocks per CU (≤ kTnGroupRounds); 0 = 2 when a block
// would otherwise take ≥ 64 K points (C4 at 4 096 rays: 26.29 / 26.32 -> 26.25 / 26.26 ms), else 1
// (at 512 rays 2 rounds measured 3.976 / 3.977 against 3.963 / 3.964 ms)
int g_tn_group_rounds = 0;
int g_tn_group_last = 0;   // option "tn_group_last" (bench.py sets 2 when N > 1): the last group's size cap
// option "defer_heads": under deferred trunk weight gradients the output heads' G / Q weight
// gradients run in trunk_wgrad too (one GEMM over every pass's points, inside the group launch)
// — 1 always, 0 never, 2 (default) for passes of at most 2^18 points: C4 at 512 rays 3.970 / 3.973
// -> 3.926 / 3.917 ms, while at 4 096 rays the per-pass GEMMs overlapping the dX chain on the side
// stream are worth more (26.04 / 26.14 against 26.16 / 26.19 ms deferred; same call)
int g_defer_heads = 2;
int g_tn_k64_pair = 1;  // option "tn_k64_pair": the skip layer's PE tail and fc_net.0 in one narrow launch
// option "heads_epi": the training forward's narrow heads (rgb, sun, beta, semantic logits; σ and the
// sky columns with the sun) in the epilogues of the G / Q / sun_v.3 GEMMs instead of k_heads_fwd_v:
// C4 26.39 / 26.35 -> 26.13 / 26.08 ms (heads_fwd's 0.58 ms for +0.31 ms of epilogue), C4@512
// 3.950 / 3.945 -> 3.919 / 3.921 ms (same call).  2: the whole training heads (G, Q, sun_v 2 / 3
// with their saved activations, and the narrow heads) in one LDS-resident launch after the trunk
// (k_heads_train_bf16, train_heads_on), the epilogue GEMMs where the shape does not fit: the same
// step time (C4 25.34 / 25.39 against 25.32 / 25.37 ms, C4@512 3.712 / 3.709 ms, pairs in one
// call), 2.5 GB fewer HBM bytes per C4 step (PMC 88.3 against 90.8 GB) and 6 fewer launches
int g_heads_epi = 2;
int g_ray_tiles_pair = 1;  // option "ray_tiles_pair": the per-ray dZ sums of layer 0 and the skip layer in one launch
static bool defer_heads_for(int64_t P) { return g_defer_heads == 1 || (g_defer_heads == 2 && P <= (1 << 18)); }

#ifndef SPN_DEFER_SUNV
#define SPN_DEFER_SUNV 1  // sun_v_net.2 / .4's weight gradients deferred with the trunk's (0: A/B builds)
#endif

// A second point segment of a weight gradient: the same operands in another pass's workspace
// (spnerf_mlp_trunk_wgrad: the main and the solar pass of a render in one GEMM per layer)
struct TnSeg {
    const bf16 *A = nullptr, *B = nullptr, *B2 = nullptr;
    int64_t P = 0;
};

template <typename T>
static int32_t tn_grad(const Ctx& c, const T* A, int lda, int N, const T* B, int ldb, const T* B2, int ldb2, int K1,
                       int K, hipStream_t s, const std::vector<ReduceArgs>& outs, bool b_sin = false,
                       const TnSeg* sg = nullptr) {
    using G = Gemms<T>;
    const int P1 = (int)c.w.P;
    const int P = P1 + (sg ? (int)sg->P : 0);
    // bf16 skip layer ([H | x0], K = 512 + K0p): the K = 576 GEMM has no 256-wide tiling and ran
    // on the 128x128 kernel at 710 us per 524 288 points; split into the wide K = 512 part and
    // the K0p tail (two passes over dZ, the tail's slab reduced into columns K1..) it is ≈470.
    // Below 2^18 points the single launch is as fast
    // (with the narrow N = 512, K = 64 kernel for the tail, tn_bf16_k64, splitting below 2^18
    // points measured level too: C4 at 512 rays 4.468 / 4.491 against 4.469 / 4.465 ms)
    bool split = std::is_same<T, bf16>::value && g_tn_split_tail && B2 && K > K1 && P >= (1 << 18) &&
                 N % 256 == 0 && K1 % 256 == 0 && (N / 256) * (K1 / 256) >= 4;
    for (const ReduceArgs& r : outs) split = split && !r.transpose;
    if (split) {
        std::vector<ReduceArgs> head, tail;
        for (ReduceArgs r : outs) {
            ReduceArgs h = r;
            h.ncols = std::min(r.ncols, K1);
            head.push_back(h);
            if (r.ncols > K1) {
                ReduceArgs t = r;
                t.dst = r.dst + K1;
                t.ncols = r.ncols - K1;
                t.dst_b = nullptr;  // the column sums come with the head
                tail.push_back(t);
            }
        }
        TnSeg sh, st;
        if (sg) {
            sh = {sg->A, sg->B, nullptr, sg->P};
            st = {sg->A, sg->B2, nullptr, sg->P};
        }
        SPN_TRY(tn_grad<T>(c, A, lda, N, B, ldb, nullptr, 0, K1, K1, s, head, b_sin, sg ? &sh : nullptr));
        if (!tail.empty())
            SPN_TRY(tn_grad<T>(c, A, lda, N, B2, ldb2, nullptr, 0, K - K1, K - K1, s, tail, false, sg ? &st : nullptr));
        return SPNERF_OK;
    }
    // the slab buffer is sized for this workspace's points: a longer (two-segment) GEMM takes
    // no more splits than that
    const int splits = std::min(G::splits(P, N, K), G::splits(P1, N, K));
    typename G::TN t;
    t.A = A; t.lda = lda;
    t.B = B; t.ldb = ldb; t.B2 = B2; t.ldb2 = ldb2; t.K1 = K1;
    if constexpr (std::is_same<T, bf16>::value) t.b_sin = b_sin ? 1 : 0;  // B[:, :K1] holds a saved Z
    t.slab = c.at(c.w.slab); t.ld_slab = K; t.slab_stride = (int64_t)N * K;
    t.slab_b = c.at(c.w.slab_b);
    t.P = P; t.N = N; t.K = K;
    if (sg) {
        if constexpr (std::is_same<T, bf16>::value) {
            // rows p >= P1 come from the second segment: its pointers shifted back by P1 rows
            t.P1 = P1;
            t.A_s2 = sg->A - (int64_t)P1 * lda;
            t.B_s2 = sg->B - (int64_t)P1 * ldb;
            t.B2_s2 = sg->B2 ? sg->B2 - (int64_t)P1 * ldb2 : nullptr;
        } else {
            SPN_ARG(false, "tn_grad: two point segments need the bf16 MLP");
        }
    }
    SPN_TRY(G::tn(t, splits, s));
    std::vector<ReduceArgs> rs;
    for (ReduceArgs r : outs) {
        r.slab = t.slab; r.ld_slab = K; r.slab_stride = t.slab_stride; r.splits = splits; r.N = N;
        r.slab_b = t.slab_b;
        r.accumulate = c.acc;
        rs.push_back(r);
    }
    for (size_t i = 0; i < rs.size(); i += kReduceMulti)
        SPN_TRY(reduce_slabs_multi(rs.data() + i, (int)std::min<size_t>(kReduceMulti, rs.size() - i), s));
    return SPNERF_OK;
}

static ReduceArgs red(int row0, int nrows, int ncols, float* dst, int ld_dst, float* dst_b) {
    ReduceArgs r;
    r.row0 = row0; r.nrows = nrows; r.ncols = ncols; r.dst = dst; r.ld_dst = ld_dst; r.dst_b = dst_b;
    return r;
}

// out[m][k] = Σ_r A[r*lda+m] · B[r*ldb+k] over `rows` rows (points or rays), written to dst
// (row-major, or dst[k][m] with `transpose`); dst_b[m] = Σ_r A[r][m]; dst_ones[k] = Σ_r B[r][k].
template <typename TB>
static int32_t skinny(const Ctx& c, int64_t rows, const float* A, int lda, int Ma, const TB* B, int ldb, int K,
                      float* dst, int ld_dst, int transpose, float* dst_b, float* dst_ones, hipStream_t s) {
    SkinnyArgs k;
    k.A = A; k.lda = lda; k.Ma = Ma; k.ldb = ldb; k.K = K; k.P = rows; k.ones = dst_ones ? 1 : 0;
    if constexpr (std::is_same<TB, bf16>::value) k.B16 = B;
    else k.B = B;
    k.slab = c.at(c.w.sk_slab); k.slab_b = c.at(c.w.sk_slab_b);
    SPN_TRY(tn_skinny(k, s));
    const int chunks = cdiv(rows, skinny_chunk(rows));
    const int Mt = Ma + k.ones;
    ReduceArgs r = red(0, Ma, K, dst, ld_dst, dst_b);
    r.slab = k.slab; r.ld_slab = K; r.slab_stride = (int64_t)Mt * K; r.splits = chunks; r.N = Mt; r.slab_b = k.slab_b;
    r.transpose = transpose;
    r.accumulate = c.acc;
    ReduceArgs rr[2];
    int n = 0;
    if (dst) rr[n++] = r;
    if (dst_ones) {
        ReduceArgs o = r;
        o.row0 = Ma; o.nrows = 1; o.dst = dst_ones; o.ld_dst = K; o.dst_b = nullptr; o.transpose = 0;
        rr[n++] = o;
    }
    return reduce_slabs_multi(rr, n, s);
}

// Skinny reductions with fp32 rows batched into ONE launch (tn_skinny_multi) plus one reduction
// launch per kReduceMulti outputs — the per-ray parameter gradients of a backward (step 7) were
// a dozen launches of a few microseconds of work each.  Same arithmetic as skinny().
struct SkinnyBatch {
    const Ctx& c;
    std::vector<SkinnyArgs> tasks;
    std::vector<ReduceArgs> reds;
    int64_t off = 0, off_b = 0;
    explicit SkinnyBatch(const Ctx& cc) : c(cc) {}
    template <typename TB>
    int32_t add(int64_t rows, const float* A, int lda, int Ma, const TB* B, int ldb, int K, float* dst, int ld_dst,
                int transpose, float* dst_b, float* dst_ones) {
        SkinnyArgs k;
        k.A = A; k.lda = lda; k.Ma = Ma; k.ldb = ldb; k.K = K; k.P = rows; k.ones = dst_ones ? 1 : 0;
        if constexpr (std::is_same<TB, bf16>::value) k.B16 = B;
        else k.B = B;
        const int64_t chunks = rows > 0 ? cdiv(rows, skinny_chunk(rows)) : 0;
        const int Mt = Ma + k.ones;
        SPN_ARG(off + chunks * Mt * K <= c.w.sk_slab_n && off_b + chunks * Ma <= c.w.sk_slab_b_n &&
                (int)tasks.size() < kSkinnyMulti, "skinny batch: slab capacity");
        k.slab = c.at(c.w.sk_slab) + off;
        k.slab_b = c.at(c.w.sk_slab_b) + off_b;
        off += chunks * Mt * K;
        off_b += chunks * Ma;
        tasks.push_back(k);
        ReduceArgs r = red(0, Ma, K, dst, ld_dst, dst_b);
        r.slab = k.slab; r.ld_slab = K; r.slab_stride = (int64_t)Mt * K; r.splits = (int)chunks; r.N = Mt;
        r.slab_b = k.slab_b;
        r.transpose = transpose;
        r.accumulate = c.acc;
        if (dst) reds.push_back(r);
        if (dst_ones) {
            ReduceArgs o = r;
            o.row0 = Ma; o.nrows = 1; o.dst = dst_ones; o.ld_dst = K; o.dst_b = nullptr; o.transpose = 0;
            reds.push_back(o);
        }
        return SPNERF_OK;
    }
    int32_t run(hipStream_t s) {
        SPN_TRY(tn_skinny_multi(tasks.data(), (int)tasks.size(), s));
        for (size_t i = 0; i < reds.size(); i += kReduceMulti)
            SPN_TRY(reduce_slabs_multi(reds.data() + i, (int)std::min<size_t>(kReduceMulti, reds.size() - i), s));
        return SPNERF_OK;
    }
};

// Trunk + G/Q/sun_v GEMMs of the forward (spnerf.py:323-355).  In the bf16 MLP, layer 0 stays
// an fp32 GEMM (sin(30·x) amplifies operand rounding 30x) that writes bf16 H_1 / D_1.
// bf16 MLP: layer 0 runs inside the fused trunk launch (reading the fp32 PE rows itself)
// bf16 trunk layers 1 .. L-1 (w0 = 1) compute H = sin(Z) with Z = fp16(pre-activation), and the
// training forward saves Z alone for layers 1 .. L-2 (Z and H for the last): the backward stages
// sin(Z) for the weight gradients and multiplies by cos(Z) in the dX epilogues, so the forward
// writes one [P][512] tensor per layer instead of H and D (option "zsave"; must not change
// between a forward and its backward).  Off by default: measured on C4 (tools/gpu_ab_opt.sh) the
// trunk saves 0.9 ms per step but the weight gradients' sin staging costs 1.25 ms (31.3 vs 31.9 ms)
int g_zsave = 0;

static bool fused_trunk_on(const Ctx& c) {
    return c.d.bf && g_fused_trunk && !c.k.Wf16.empty() && c.k.Wf16[1] >= 0;
}
// inference (nothing saved) of the full or the σ-only heads: the fused heads kernel after the trunk
static bool heads_fused_on(const Ctx& c, bool save, int mode) {
    return !save && (mode == 0 || mode == 1) && c.d.bf && c.k.Ffeat16 >= 0 && heads_bf16_supported(c.d);
}
int g_pe_inline = 1;  // option "pe_inline": inference trunk with layer 0 encodes o + dir·z itself (no k_encode)
static bool trunk_l0_on(const Ctx& c, bool save);
// (training too since round 4: the trunk then writes the bf16 PE rows X0b the weight gradients read,
// and no k_encode runs)
static bool pe_inline_on(const Ctx& c, bool save) { return g_pe_inline && trunk_l0_on(c, save); }

static bool trunk_l0_on(const Ctx& c, bool save) {
    return fused_trunk_on(c) && g_l0_split && (g_trunk_l0 == 2 || (g_trunk_l0 == 1 && !save)) && c.k.Wf16[0] >= 0 &&
           trunk_l0_supported(c.d.K0p, save, c.d.bf && g_zsave);
}

// option heads_epi 2: the training forward's heads (k_heads_train_bf16) as one launch after the
// saving trunk, where the shape allows: W = 512, H = 256, no β head, C <= 3
static bool train_heads_shape(const Ctx& c, int mode) {
    const Dims& d = c.d;
    return d.bf && (mode == 0 || mode == 2) && d.W == 512 && d.H == 256 && !d.beta && (!d.sem || d.C <= 3) &&
           c.k.Ffeat16 >= 0 && c.k.Fnar16 >= 0 && c.out && c.heads_done && !g_zsave;
}
static bool train_heads_on(const Ctx& c, int mode) { return g_heads_epi == 2 && train_heads_shape(c, mode); }
static HeadsFusedArgs heads_args(const Ctx& c, int mode, int64_t hl, double* flop, double* bytes);
// the training heads' arguments: what they store, and their counted work (the wide layers as
// computed — the solar pass's Q runs all 2H columns — and the narrow heads; stored: feat (+ the
// semantic hidden and its D), Q and DQ, S2 / S3 and their D, the output rows, the gates)
static HeadsFusedArgs train_heads_args(const Ctx& c, int mode, int64_t hl, double* flop, double* bytes) {
    const Dims& d = c.d;
    const int64_t P = c.w.P;
    const int W = d.W, H = d.H;
    HeadsFusedArgs h = heads_args(c, mode, hl, flop, bytes);
    h.G = c.hb(c.w.G); h.DG = d.sem ? c.hb(c.w.DG) : nullptr; h.ldG = d.NG;
    h.Q = c.hb(c.w.Q); h.DQ = c.hb(c.w.DQ); h.ldQ = d.NQ;
    h.S2 = c.hb(c.w.S2); h.DS2 = c.hb(c.w.DS2); h.S3 = c.hb(c.w.S3); h.DS3 = c.hb(c.w.DS3);
    h.hsave = c.at(c.w.hsave);
    const bool m0 = mode == 0, sm = m0 && d.sem;
    *flop = 2.0 * P * ((double)W * W + 2.0 * H * W + 2.0 * H * H + (sm ? (double)H * W + H * d.C : 0.0) + (m0 ? 3.0 * H : 0.0) + H);
    *bytes = 2.0 * P * (W + (sm ? 2.0 * H : 0.0) + 2.0 * (m0 ? 2 * H : H) + 4.0 * H) + 4.0 * P * (d.NO + (m0 ? 4 : 1));
    return h;
}

// the fused heads' arguments and counted work (k_heads_bf16, or inside the inference trunk)
static HeadsFusedArgs heads_args(const Ctx& c, int mode, int64_t hl, double* flop, double* bytes) {
    const Dims& d = c.d;
    const int64_t P = c.w.P;
    const int W = d.W, H = d.H;
    HeadsFusedArgs a;
    a.HL = hl >= 0 ? c.hb(hl) : nullptr; a.packed = c.P; a.rbQ = c.at(c.w.rbQ); a.sky = c.at(c.w.sky); a.out = c.out;
    a.P = P; a.S = c.S; a.NO = d.NO; a.C = d.sem ? d.C : 0; a.sem_col = d.sem_col; a.mode = mode;
    *flop = mode == 1 ? 2.0 * P * W
                      : 2.0 * P * ((double)W * (W + 2 * H) + 2.0 * H * H + (d.sem ? (double)H * W + H * d.C : 0.0) + W + 4.0 * H);
    *bytes = 2.0 * P * W + 4.0 * P * (mode == 1 ? 1 : d.NO);
    return a;
}

template <typename T>
static int32_t forward_gemms(const Ctx& c, bool save, int mode, hipStream_t s, bool* sig_done) {
    using G = Gemms<T>;
    using NT = typename G::NT;
    const Dims& d = c.d;
    const int64_t P = c.w.P;
    const int W = d.W, H = d.H, S = c.S;
    constexpr bool BF = std::is_same<T, bf16>::value;
    const T* X0 = BF ? G::buf(c, c.w.X0b) : G::buf(c, c.w.X0);
    const T* h = nullptr;
    T* HL = nullptr;
    const bool fused = BF && fused_trunk_on(c);
    const bool zs = BF && g_zsave;
    const int first = fused && trunk_l0_on(c, save) ? 0 : 1;  // first layer of the fused launch
    for (int i = 0; i < d.L; ++i) {
        if (fused && i == first) {
            // layers first .. L-1 in one persistent launch, activations resident in LDS
            TrunkArgs a;
            a.H1 = reinterpret_cast<const bf16*>(h);
            a.X0b = c.hb(c.w.X0b);
            if (first == 0) {
                if (pe_inline_on(c, save)) {
                    a.rays = c.rays; a.rs = c.rs; a.dir_off = c.dir_off; a.z = c.z; a.ldz = c.ldz;
                    a.n_freq = d.K0 == 3 ? 0 : d.K0 / 6; a.K0 = d.K0;
                    if (save) a.X0b_out = c.hb(c.w.X0b);
                } else {
                    a.X0 = c.at(c.w.X0);
                }
                a.rb0 = d.sem ? c.at(c.w.rb0) : nullptr;
            }
            double ksum = 0.0;
            for (int l = first; l < d.L; ++l) {
                a.Wf[l] = c.pk16(c.k.Wf16[l]);
                a.bias[l] = c.pk(c.k.bt[l]);
                const bool zonly = zs && l >= 1 && l < d.L - 1;  // Z alone (in Db) for the backward
                a.Hs[l] = save ? (zonly ? nullptr : c.hb(c.w.Hb[l])) : (l == d.L - 1 ? c.hb(c.w.Hb[l & 1]) : nullptr);
                a.Ds[l] = save ? c.hb(c.w.Db[l]) : nullptr;
                ksum += l == 0 ? d.K0p : c.k.Kp[l];   // algorithmic K (layer 0 runs 4·K0p on hi/lo planes)
            }
            a.rb_skip = d.sem ? c.at(c.w.rb4) : nullptr;
            a.P = P; a.S = S; a.L = d.L; a.skip = d.skip; a.K0p = d.K0p;
            a.zround = zs ? 1 : 0;
            // the σ head's pre-activation from the last layer's LDS image (the wave-per-point
            // heads then skip H_L); option trunk_sigma
            if (sig_done && !heads_fused_on(c, save, mode) && g_heads_variant != 0 && W == 512 && trunk_sigma_ok(a, save)) {
                a.sig_hsave = c.at(c.w.hsave);
                a.wsig = c.pk(c.k.wsig);
                a.bsig = c.pk(c.k.bsig);
                *sig_done = true;
            }
            // algorithmic HBM bytes: the first layer's input (fp32 PE, or H_1 and the bf16 PE)
            // in; out when saving H and D of every layer, or Z of every layer and the last H
            const double in = first == 0 ? (a.rays ? 4.0 * P : 4.0 * P * d.K0p) : 2.0 * P * (W + (d.skip > 0 ? d.K0p : 0));
            const double nout = !save ? 1.0 : (zs ? d.L - first + 1.0 : 2.0 * (d.L - first));
            const double bytes = in + 2.0 * P * W * nout + (a.X0b_out ? 2.0 * P * d.K0p : 0.0);
            if constexpr (BF) {
                // inference: the fused heads on the trunk's last LDS image (no H_L in HBM)
                if (c.heads_done && c.out && heads_fused_on(c, save, mode) && (trunk1_heads_ok(a) || trunk2_heads_ok(a))) {
                    double hflop = 0.0, hbytes = 0.0;
                    const HeadsFusedArgs h = heads_args(c, mode, -1, &hflop, &hbytes);
                    // algorithmic bytes: the trunk's input, the output rows (H_L never leaves)
                    if (trunk1_heads_ok(a))
                        SPN_TRY(trunk1_heads_bf16(a, h, c.k, s, 2.0 * P * W * ksum + hflop, in + (hbytes - 2.0 * P * W)));
                    else
                        SPN_TRY(trunk2_heads_bf16(a, h, c.k, s, 2.0 * P * W * ksum + hflop, in + (hbytes - 2.0 * P * W)));
                    *c.heads_done = true;
                    return SPNERF_OK;
                }
            }
            SPN_TRY(trunk_bf16(a, s, 2.0 * P * W * ksum, bytes));
            HL = reinterpret_cast<T*>(a.Hs[d.L - 1]);
            break;
        }
        T* dst = save ? G::buf(c, c.w.Hb[i]) : G::buf(c, c.w.Hb[i & 1]);
        T* dd = save ? G::buf(c, c.w.Db[i]) : nullptr;
        const float* rb = (d.sem && (i == 0 || i == d.skip)) ? c.at(i == 0 ? c.w.rb0 : c.w.rb4) : nullptr;
        if (i == 0 && BF && g_l0_split) {
            // fc_net.0 on MFMA bf16 as (x_hi + x_lo)·(w_hi + w_lo), K = 4·K0p: relative error
            // ≈ 2^-17 per product (the split's remainder) against the fp32 GEMM's 2^-24, far
            // inside the bf16 output's 2^-9, at bf16 MFMA rates instead of fp32 ones
            NT16Args g;
            g.A = c.hb(c.w.X0s); g.lda = 4 * d.K0p; g.K1 = 4 * d.K0p;
            g.B = c.pk16(c.k.W0s16); g.ldb = 4 * d.K0p;
            g.C = reinterpret_cast<bf16*>(dst); g.ldc = W;
            g.M = (int)P; g.N = W; g.K = 4 * d.K0p;
            g.bias = c.pk(c.k.bt[0]);
            if (rb) { g.rowbias = rb; g.ld_rb = W; g.rows_per_ray = S; }
            g.act = 1; g.w0 = 30.f; g.n_lin = 0;
            if (save) { g.Dout = reinterpret_cast<bf16*>(dd); g.ld_dout = W; }
            g.k_alg = d.K0p;   // FLOPs counted at the layer's own K (the split's 4x MFMA work is overhead)
            SPN_TRY(gemm_nt_bf16(g, s));
        } else if (i == 0) {
            NTArgs g;
            g.A = c.at(c.w.X0); g.lda = d.K0p; g.K1 = d.K0p;
            g.B = c.pk(c.k.Wt[0]); g.ldb = d.K0p;
            g.ldc = W;
            g.M = (int)P; g.N = W; g.K = d.K0p;
            g.bias = c.pk(c.k.bt[0]);
            if (rb) { g.rowbias = rb; g.ld_rb = W; g.rows_per_ray = S; }
            g.act = 1; g.w0 = 30.f; g.n_lin = 0;
            g.ld_dout = W;
            if constexpr (BF) { g.C16 = dst; g.D16 = dd; }
            else { g.C = dst; g.Dout = dd; }
            SPN_TRY(gemm_nt(g, s));
        } else {
            NT g;
            g.A = h; g.lda = W; g.K1 = W;
            if (i == d.skip) { g.A2 = X0; g.lda2 = d.K0p; }
            g.B = G::w(c, c.k.Wt[i], BF ? c.k.Wt16[i] : -1); g.ldb = c.k.Kp[i];
            g.C = dst; g.ldc = W;
            g.M = (int)P; g.N = W; g.K = c.k.Kp[i];
            g.bias = c.pk(c.k.bt[i]);
            if (rb) { g.rowbias = rb; g.ld_rb = W; g.rows_per_ray = S; }
            g.act = 1; g.w0 = 1.f; g.n_lin = 0;
            if (save) { g.Dout = dd; g.ld_dout = W; }
            if constexpr (BF) {
                g.zround = zs ? 1 : 0;
                g.dout_z = zs ? 1 : 0;
            }
            SPN_TRY(G::nt(g, s));
        }
        h = dst;
        HL = dst;
    }
    if (mode == 1) return SPNERF_OK;
    if (BF && heads_fused_on(c, save, mode)) return SPNERF_OK;  // G, Q, sun_v 2/3 inside the fused heads
    if constexpr (BF) {
        // option heads_epi 2: the training heads as one launch after the trunk (H_L from HBM)
        if (save && train_heads_on(c, mode) && sig_done && *sig_done) {
            double hflop = 0.0, hbytes = 0.0;
            const HeadsFusedArgs h = train_heads_args(c, mode, c.w.Hb[d.L - 1], &hflop, &hbytes);
            if (heads_train_bf16_ok(h, c.k)) {
                SPN_TRY(heads_train_bf16(h, c.k, s, hflop, hbytes + 2.0 * P * W));
                *c.heads_done = true;
                return SPNERF_OK;
            }
        }
    }
    T* S2buf = save ? G::buf(c, c.w.S2) : G::buf(c, c.w.Hb[((d.L - 1) & 1) ^ 1]);
    T* S3buf = save ? G::buf(c, c.w.S3) : G::buf(c, c.w.Hb[2]);
    // option heads_epi: the narrow heads in the G / Q / sun_v.3 epilogues (bf16 DMA NT with the
    // bias / per-ray-row epilogue; σ from the trunk's hsave column)
    const bool hepi = BF && g_heads_epi && g_nt16_epi && (g_nt16_ip_gen == 2 || g_nt16_ip_gen == 3) && !zs && g_nt16_variant == 8 && save &&
                      sig_done && *sig_done && c.out && c.heads_epi_done &&
                      W == 512 && H == 256 && (!d.sem || d.C <= 3) && S % 32 == 0 && mode != 1 &&
                      d.NG % 256 == 0 && d.NQ % 256 == 0;
    NTHeads hbase;
    if (hepi) {
        hbase.out = c.out; hbase.NO = d.NO; hbase.sem_col = d.sem_col;
        hbase.hsave = c.at(c.w.hsave); hbase.sky = c.at(c.w.sky); hbase.S = S; hbase.full = mode == 0 ? 1 : 0;
    }
    auto head = [&](NTHeads& hd, int col0, int nout, int kind, int64_t w, int ldw, int64_t b) {
        hd.col0[hd.n] = col0; hd.nout[hd.n] = nout; hd.kind[hd.n] = kind;
        hd.w[hd.n] = c.pk(w); hd.ldw[hd.n] = ldw; hd.b[hd.n] = c.pk(b);
        ++hd.n;
    };
    // G = H_L · [feat ; sem hidden]^T   (feat linear, sem hidden sin)
    NT g;
    g.A = HL; g.lda = W; g.K1 = W;
    g.B = G::w(c, c.k.WG, c.k.WG16); g.ldb = W;
    g.C = G::buf(c, c.w.G); g.ldc = d.NG;
    g.M = (int)P; g.N = mode == 0 ? d.NG : W; g.K = W;
    g.bias = c.pk(c.k.bG);
    g.act = 1; g.w0 = 1.f; g.n_lin = W;
    if (save) { g.Dout = G::buf(c, c.w.DG); g.ld_dout = d.NG; }
    if constexpr (BF)
        if (hepi && mode == 0 && d.sem) {
            g.hd = hbase;
            head(g.hd, W, d.C, 3, c.k.Wm2, H, c.k.bm2);
        }
    SPN_TRY(G::nt(g, s));
    // Q = feat · [sun1 ; rgb1 ; beta1]^T + per-ray (sun_d / t) rows, all sin
    NT q;
    q.A = G::buf(c, c.w.G); q.lda = d.NG; q.K1 = W;
    q.B = G::w(c, c.k.WQ, c.k.WQ16); q.ldb = W;
    q.C = G::buf(c, c.w.Q); q.ldc = d.NQ;
    q.M = (int)P; q.N = mode == 0 ? d.NQ : H; q.K = W;
    q.bias = c.pk(c.k.bQ);
    q.rowbias = c.at(c.w.rbQ); q.ld_rb = d.NQ; q.rows_per_ray = S;
    q.act = 1; q.w0 = 1.f;
    if (save) { q.Dout = G::buf(c, c.w.DQ); q.ld_dout = d.NQ; }
    if constexpr (BF)
        if (hepi && mode == 0) {
            q.hd = hbase;
            head(q.hd, H, 3, 0, c.k.Wr2, H, c.k.br2);
            if (d.beta) head(q.hd, 2 * H, 1, 2, c.k.wb2, H, c.k.bb2);
        }
    SPN_TRY(G::nt(q, s));
    // sun_v_net layers 2 and 3
    NT s2;
    s2.A = G::buf(c, c.w.Q); s2.lda = d.NQ; s2.K1 = H;
    s2.B = G::w(c, c.k.Ws2, c.k.Ws2_16); s2.ldb = H;
    s2.C = S2buf; s2.ldc = H;
    s2.M = (int)P; s2.N = H; s2.K = H;
    s2.bias = c.pk(c.k.bs2); s2.act = 1; s2.w0 = 1.f;
    if (save) { s2.Dout = G::buf(c, c.w.DS2); s2.ld_dout = H; }
    SPN_TRY(G::nt(s2, s));
    NT s3 = s2;
    s3.A = S2buf; s3.lda = H;
    s3.B = G::w(c, c.k.Ws3, c.k.Ws3_16);
    s3.C = S3buf;
    s3.bias = c.pk(c.k.bs3);
    s3.Dout = save ? G::buf(c, c.w.DS3) : nullptr;
    if constexpr (BF)
        if (hepi) {
            s3.hd = hbase;
            head(s3.hd, 0, 1, 1, c.k.ws4, H, c.k.bs4);
        }
    SPN_TRY(G::nt(s3, s));
    if (hepi) *c.heads_epi_done = true;
    return SPNERF_OK;
}

static int32_t mlp_forward(const Dims& d, const float* packed, const float* rays, int rs, int dir_off,
                           int64_t n_rays, int S, const float* z, const int64_t* labels, const float* temb, int flags,
                           float* ws, float* out, hipStream_t s, int64_t n_total = -1, int64_t r0 = 0, int ldz = 0) {
    // n_total >= 0: rays [r0, r0 + n_rays) of a workspace laid out for n_total rays (forward_window)
    Ctx c{d, packed_layout(d),
          n_total < 0 ? ws_layout(d, n_rays, S, flags) : ws_window(d, ws_layout(d, n_total, S, flags), r0, n_rays, S),
          packed, ws, S};
    const bool save = flags & SPNERF_MLP_SAVE;
    const int mode = (flags & SPNERF_MLP_SIGMA_ONLY) ? 1 : ((flags & SPNERF_MLP_SUN_ONLY) ? 2 : 0);
    const int64_t P = n_rays * S;
    const int W = d.W, H = d.H;
    if (P == 0) return SPNERF_OK;
    SPN_ARG(P < (1ll << 31) / std::max(d.NQ, d.NG), "too many points (%lld) for one call", (long long)P);
    SPN_ARG(!d.sem || labels, "semantic model needs labels");
    SPN_ARG(!d.beta || mode != 0 || temb, "beta model needs t_emb");

    // per-ray terms
    {
        RayFwdArgs a{rays, rs, labels, temb, packed, c.k, d, c.at(c.w.rb0), c.at(c.w.rb4), c.at(c.w.rbQ),
                     c.at(c.w.skyh), c.at(c.w.sky), d.sem ? 1 : 0, mode != 1, mode == 0};
        if (d.beta && mode == 0) {
        } else {
            a.d.beta = false;
            a.d.td = 0;
        }
        if (d.sem || mode != 1) {
            ProfScope prof("ray_terms", s, 0.0, 0.0);
            hipLaunchKernelGGL(k_ray_fwd, dim3((unsigned)n_rays), dim3(256), 0, s, a);
            SPN_HIP(hipGetLastError());
        }
    }
    // positional encoding (fp32 for layer 0, plus a bf16 copy for the skip layer / dW_0); the
    // fused inference trunk with layer 0 computes it in its staging instead
    c.rays = rays; c.rs = rs; c.dir_off = dir_off; c.z = z; c.ldz = ldz > 0 ? ldz : S;
    if (!pe_inline_on(c, save)) {
        const int64_t n = P * d.K0p;
        // bf16 MLP, layer 0 on bf16 planes: a separate GEMM reads the planes X0s; inside the
        // fused trunk it splits the fp32 rows itself
        const bool l0t = trunk_l0_on(c, save);
        const bool planes = d.bf && g_l0_split && !l0t;
        ProfScope prof("encode", s, 0.0, (planes ? 10.0 : 4.0 + (d.bf ? 2.0 : 0.0)) * n);
        hipLaunchKernelGGL(k_encode, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rays, rs, dir_off, z, S, c.ldz, P,
                           d.K0 == 3 ? 0 : d.K0 / 6, d.K0, d.K0p, planes ? nullptr : c.at(c.w.X0),
                           d.bf ? c.hb(c.w.X0b) : nullptr, planes ? c.hb(c.w.X0s) : nullptr);
        SPN_HIP(hipGetLastError());
    }
    bool sig_done = false;  // hsave[p·8] (σ pre-activation) written by the fused trunk
    bool heads_done = false;  // the trunk launch ran the fused heads
    bool heads_epi_done = false;  // the head GEMMs' epilogues wrote the narrow heads
    c.out = out;
    c.heads_done = &heads_done;
    c.heads_epi_done = &heads_epi_done;
    if (d.bf) SPN_TRY(forward_gemms<bf16>(c, save, mode, s, &sig_done));
    else SPN_TRY(forward_gemms<float>(c, save, mode, s, nullptr));
    if (heads_done || heads_epi_done) return SPNERF_OK;
    if (heads_fused_on(c, save, mode)) {
        double flop = 0.0, bytes = 0.0;
        const HeadsFusedArgs a = heads_args(c, mode, c.w.Hb[(d.L - 1) & 1], &flop, &bytes);
        SPN_TRY(heads_bf16(a, c.k, s, flop, bytes));
        return SPNERF_OK;
    }
    {
        const int64_t L = d.L - 1;
        const int64_t hl = save ? c.w.Hb[L] : c.w.Hb[L & 1];
        const int64_t s3 = save ? c.w.S3 : c.w.Hb[2];
        const int grid = (int)std::min<int64_t>(cdiv(P, 4), 8192);
        ProfScope prof("heads_fwd", s, 2.0 * P * ((sig_done ? 0 : W) + (mode != 1 ? 4 * H + H * d.C : 0)),
                       (d.bf ? 2.0 : 4.0) * P * ((sig_done ? 0 : W) + 3 * H) + 4.0 * P * (d.NO + (sig_done ? 1 : 0)));
        const int nc = g_heads_variant == 0 ? 0 : cdiv(W, 256);
        const size_t lds = mode == 0 && d.sem ? sizeof(float) * d.C * (H + 1) : 0;  // ≤ 32 × 513 floats when nc ≤ 4
        auto launch = [&](auto a) {
            using T = std::remove_cv_t<std::remove_pointer_t<decltype(a.HL)>>;
            if (sig_done && nc == 2) {  // σ from hsave (W = 512, bf16)
                hipLaunchKernelGGL((k_heads_fwd_v<T, 2, true>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k);
                return;
            }
            switch (nc) {
                case 1: hipLaunchKernelGGL((k_heads_fwd_v<T, 1>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k); break;
                case 2: hipLaunchKernelGGL((k_heads_fwd_v<T, 2>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k); break;
                case 3: hipLaunchKernelGGL((k_heads_fwd_v<T, 3>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k); break;
                case 4: hipLaunchKernelGGL((k_heads_fwd_v<T, 4>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k); break;
                default: hipLaunchKernelGGL(k_heads_fwd<T>, dim3(grid), dim3(256), 0, s, a, (PackedOffs)c.k);
            }
        };
        if (d.bf) launch(HeadsArgs<bf16>{packed, d, c.hb(hl), c.hb(c.w.G), c.hb(c.w.Q), c.hb(s3), c.at(c.w.sky), out, c.at(c.w.hsave), P, S, mode});
        else launch(HeadsArgs<float>{packed, d, c.at(hl), c.at(c.w.G), c.at(c.w.Q), c.at(s3), c.at(c.w.sky), out, c.at(c.w.hsave), P, S, mode});
        SPN_HIP(hipGetLastError());
    }
    return SPNERF_OK;
}

// Zeroing with a kernel of our own instead of hipMemsetAsync: inside a captured HIP graph the
// runtime's memset node (a blit kernel) did not survive later eager memsets on this ROCm —
// replays then left every 4th float of the range stale (tests/test_gpu_graph.py).
__global__ void k_zero(float* __restrict__ p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0.f;
}

static int32_t zero_fill(float* p, int64_t n, hipStream_t s) {
    if (n <= 0) return SPNERF_OK;
    ProfScope prof("zero", s, 0.0, 4.0 * n);
    hipLaunchKernelGGL(k_zero, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 2048)), dim3(256), 0, s, p, n);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

// per-ray sums of a point-major buffer (see k_ray_rowsum)
template <typename T>
static int32_t ray_rowsum(const T* in, int ld, int c0, int N, int S, int64_t n_rays, float* out, int ldo, hipStream_t s) {
    ProfScope prof("ray_rowsum", s, 0.0, (double)n_rays * (S * (double)N * sizeof(T) + 4.0 * N));
    if constexpr (std::is_same<T, bf16>::value) {
        if (N % 8 == 0 && N <= 2048 && ld % 8 == 0 && c0 % 8 == 0) {
            hipLaunchKernelGGL(k_ray_rowsum16, dim3((unsigned)n_rays), dim3(256), 0, s, in, ld, c0, N, S, out, ldo);
            SPN_HIP(hipGetLastError());
            return SPNERF_OK;
        }
    }
    hipLaunchKernelGGL(k_ray_rowsum<T>, dim3(cdiv(N, 256), (unsigned)n_rays), dim3(256), 0, s, in, ld, c0, N, S, out, ldo);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

// Backward of the per-point network (steps 1-6): narrow heads, head / sun_v / feat / trunk
// weight gradients (split-P TN GEMMs + fixed-order slab reduction), dX GEMMs with the saved
// sin' as Dmul, and the per-ray sums R0 / R4 / RQ feeding the per-ray parameters.
template <typename T>
static int32_t backward_points(const Ctx& c, int mode, const float* packed, const float* d_out, int64_t n_rays,
                               float* grad, hipStream_t s, hipStream_t s2, Side* sd) {
    using G = Gemms<T>;
    using NT = typename G::NT;
    constexpr bool BF = std::is_same<T, bf16>::value;
    const bool zs = BF && g_zsave;  // the forward saved Z for the trunk layers >= 1 (forward_gemms)
    const Dims& d = c.d;
    const int64_t P = c.w.P;
    const int W = d.W, H = d.H, S = c.S;
    PIdx x;
    auto specs = param_specs(d, &x);
    auto gp = [&](int pi) { return grad + specs[pi].off; };
    auto ld = [&](int pi) { return (int)specs[pi].ld(); };
    auto buf = [&](int64_t off) { return G::buf(c, off); };

    T* HL = buf(c.w.Hb[d.L - 1]);
    T* Gb = buf(c.w.G);
    T* Qb = buf(c.w.Q);
    T* dZG = buf(c.w.dZG);
    T* dZQ = buf(c.w.dZQ);
    T* dS3 = buf(c.w.dS3);
    T* dS2 = buf(c.w.dS2);
    float* hpre = c.at(c.w.hpre);

    // 1. narrow heads
    {
        HeadsBwdArgs<T> a{packed, d, d_out, c.at(c.w.hsave), buf(c.w.DQ), buf(c.w.DG), buf(c.w.DS3), hpre, dZQ, dZG, dS3,
                          P, mode, (!BF && (g_emu_bf16 & 2)) ? 1 : 0};
        const double eb = BF ? 2.0 : 4.0;
        ProfScope prof("heads_bwd", s, 2.0 * P * 4 * H, 4.0 * P * (d.NO + d.HP) + eb * P * 6 * H);
        const unsigned grid = (unsigned)std::min<int64_t>(cdiv(P, 4), 8192);
        const int nh = g_heads_variant == 0 ? 0 : cdiv(H, 256);
        const size_t lds = mode == 0 && d.sem ? sizeof(float) * d.C * H : 0;
        if (nh == 1) hipLaunchKernelGGL((k_heads_bwd_v<T, 1>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k);
        else if (nh == 2) hipLaunchKernelGGL((k_heads_bwd_v<T, 2>), dim3(grid), dim3(256), lds, s, a, (PackedOffs)c.k);
        else hipLaunchKernelGGL(k_heads_bwd<T>, dim3(grid), dim3(256), 0, s, a, (PackedOffs)c.k);
        SPN_HIP(hipGetLastError());
    }
    // from here on: dX chain on s, weight gradients on s2 (each after a fork from s)
    SPN_TRY(stream_dep(sd, s, s2));
    // 2. narrow-head weights: reductions over points (one launch + one reduction launch)
    {
        SkinnyBatch sb(c);
        SPN_TRY(sb.add(P, hpre + 0, d.HP, 1, HL, W, W, gp(x.sigW), W, 0, gp(x.sigb), nullptr));
        SPN_TRY(sb.add(P, hpre + 4, d.HP, 1, buf(c.w.S3), H, H, gp(x.s4W), H, 0, gp(x.s4b), nullptr));
        if (mode == 0) {
            SPN_TRY(sb.add(P, hpre + 1, d.HP, 3, Qb + H, d.NQ, H, gp(x.r2W), H, 0, gp(x.r2b), nullptr));
            if (d.beta) SPN_TRY(sb.add(P, hpre + 5, d.HP, 1, Qb + 2 * H, d.NQ, H, gp(x.b2W), H, 0, gp(x.b2b), nullptr));
            if (d.sem) SPN_TRY(sb.add(P, hpre + 6, d.HP, d.C, Gb + W, d.NG, H, gp(x.m2W), H, 0, gp(x.m2b), nullptr));
        }
        SPN_TRY(sb.run(s2));
    }
    // 3 - 5 (their dX GEMMs): the training heads' fused dX chain (heads_dx_bf16.hip, option
    // heads_dx) — dS2, dZQ's sun half, dZG's feat half and dZ_{L-1} in ONE launch, bit for bit the
    // four GEMMs below; their weight gradients then follow on s2 as before
    const int NQ = mode == 0 ? d.NQ : H;
    const int NG = mode == 0 ? d.NG : W;
    bool hdx = false;
    if constexpr (BF) {
        HeadsDxArgs h;
        h.dS3 = dS3; h.DS2 = buf(c.w.DS2); h.DQ = buf(c.w.DQ); h.DL = buf(c.w.Db[d.L - 1]);
        h.dS2 = dS2; h.dZQ = dZQ; h.dZG = dZG; h.dZL = buf(c.w.dZa);
        h.hpre = hpre; h.wsig = c.pk(c.k.wsig); h.packed16 = c.pk16(0);
        h.Bs3 = c.k.Bs3_16; h.Bs2 = c.k.Bs2_16; h.BQ = c.k.BQ16; h.BG = c.k.BG16;
        h.P = P; h.ldQ = d.NQ; h.ldG = d.NG; h.HP = d.HP; h.kQ = d.NQ; h.kG = d.NG;
        h.mode = mode; h.sem = d.sem ? 1 : 0;
        hdx = g_heads_dx && !zs && !d.beta && W == 512 && H == 256 && (mode == 0 || mode == 2) && heads_dx_bf16_ok(h);
        if (hdx) {
            const double flop = 2.0 * P * ((double)H * H * 2 + (double)NQ * W + (double)NG * W);
            const double in = 2.0 * P * (3.0 * H + (mode == 0 ? H : 0) + (mode == 0 && d.sem ? H : 0) + W) + 4.0 * P;
            const double out = 2.0 * P * (2.0 * H + 2.0 * W);
            SPN_TRY(heads_dx_bf16(h, s, flop, in + out));
            SPN_TRY(stream_dep(sd, s, s2));
        }
    }
    // 3. sun_v_net chain: dZ_S2 = (dZ_S3 · Ws3) ⊙ DS2 ; dZ_S1 = (dZ_S2 · Ws2) ⊙ DQ[:, :H]
    {
        // deferred (SPNERF_MLP_DEFER_TRUNK_WGRAD): sun_v_net.4 / .2's weight gradients run in
        // spnerf_mlp_trunk_wgrad too — every pass of a render has them
        if (!c.defer || !SPN_DEFER_SUNV)
            SPN_TRY(tn_grad<T>(c, dS3, H, H, buf(c.w.S2), H, nullptr, 0, H, H, s2, {red(0, H, H, gp(x.s3W), H, gp(x.s3b))}));
        NT g;
        g.A = dS3; g.lda = H; g.K1 = H; g.B = G::w(c, c.k.Ws3T, c.k.Ws3T16); g.ldb = H; g.C = dS2; g.ldc = H;
        g.M = (int)P; g.N = H; g.K = H; g.Dmul = buf(c.w.DS2); g.ld_dmul = H;
        if (!hdx) {
            SPN_TRY(G::nt(g, s));
            SPN_TRY(stream_dep(sd, s, s2));
        }
        if (!c.defer || !SPN_DEFER_SUNV)
            SPN_TRY(tn_grad<T>(c, dS2, H, H, Qb, d.NQ, nullptr, 0, H, H, s2, {red(0, H, H, gp(x.s2W), H, gp(x.s2b))}));
        NT g2 = g;
        g2.A = dS2; g2.B = G::w(c, c.k.Ws2T, c.k.Ws2T16); g2.C = dZQ; g2.ldc = d.NQ; g2.Dmul = buf(c.w.DQ); g2.ld_dmul = d.NQ;
        if (!hdx) {
            SPN_TRY(G::nt(g2, s));
            SPN_TRY(stream_dep(sd, s, s2));
        }
    }
    // 4. feat: dF = dZ_Q · WQ → dZG[:, :W];  dWQ = dZ_Q^T · feat
    // deferred (SPNERF_MLP_DEFER_TRUNK_WGRAD, option defer_heads): the G / Q weight gradients run in
    // spnerf_mlp_trunk_wgrad, over every pass's points in one GEMM each
    const bool heads_def = c.defer && defer_heads_for(P);
    {
        if (heads_def) {
        } else if (mode == 0) {
            if (d.beta)
                SPN_TRY(tn_grad<T>(c, dZQ, d.NQ, NQ, Gb, d.NG, nullptr, 0, W, W, s2,
                                   {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b)), red(H, H, W, gp(x.r1W), ld(x.r1W), gp(x.r1b)),
                                    red(2 * H, H, W, gp(x.b1W), ld(x.b1W), gp(x.b1b))}));
            else
                SPN_TRY(tn_grad<T>(c, dZQ, d.NQ, NQ, Gb, d.NG, nullptr, 0, W, W, s2,
                                   {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b)), red(H, H, W, gp(x.r1W), ld(x.r1W), gp(x.r1b))}));
        } else {
            SPN_TRY(tn_grad<T>(c, dZQ, d.NQ, H, Gb, d.NG, nullptr, 0, W, W, s2, {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b))}));
        }
        // per-ray sums of dZ_Q feed the sun-direction / time-embedding columns (sun_v.0's and β.0's
        // blocks of RQ; rgb.0 has no per-ray input, so its block is not summed without β)
        SPN_TRY(ray_rowsum<T>(dZQ, d.NQ, 0, d.beta ? NQ : H, S, n_rays, c.at(c.w.RQ), d.NQ, s2));
        NT g;
        g.A = dZQ; g.lda = d.NQ; g.K1 = NQ; g.B = G::w(c, c.k.WQT, c.k.WQT16); g.ldb = d.NQ; g.C = dZG; g.ldc = d.NG;
        g.M = (int)P; g.N = W; g.K = NQ;
        if (!hdx) {
            SPN_TRY(G::nt(g, s));
            SPN_TRY(stream_dep(sd, s, s2));
        }
    }
    // 5. H_L: dH_L = dZ_G · WG + dσ ⊗ w_σ ;  dZ_{L-1} = dH_L ⊙ D_L ;  dWG = dZ_G^T · H_L
    // trunk dZ buffers in rotation: the dX GEMM of layer i writes the buffer whose dZ_{i+2} the
    // side stream's weight gradient of layer i+2 read (it waits for that, not for layer i+1's)
    T* dzb[3] = {buf(c.w.dZa), buf(c.w.dZb), buf(c.w.dZc)};
    std::vector<hipEvent_t> tn_done(d.L + 2, nullptr);
    int cur = 0;
    T* dZ = dzb[cur];
    {
        if (heads_def) {
        } else if (mode == 0 && d.sem)
            SPN_TRY(tn_grad<T>(c, dZG, d.NG, d.NG, HL, W, nullptr, 0, W, W, s2,
                               {red(0, W, W, gp(x.featW), W, gp(x.featb)), red(W, H, W, gp(x.m1W), W, gp(x.m1b))}));
        else
            SPN_TRY(tn_grad<T>(c, dZG, d.NG, W, HL, W, nullptr, 0, W, W, s2, {red(0, W, W, gp(x.featW), W, gp(x.featb))}));
        // every output head's gradient is final (spnerf_grad_marks) — unless sun_v_net.2 / .4's
        // are deferred: then spnerf_mlp_trunk_wgrad records the mark once they are
        if (!c.defer || (!SPN_DEFER_SUNV && !heads_def)) SPN_TRY(grad_mark(0, s2));
        NT g;
        g.A = dZG; g.lda = d.NG; g.K1 = NG; g.B = G::w(c, c.k.WGT, c.k.WGT16); g.ldb = d.NG; g.C = dZ; g.ldc = W;
        g.M = (int)P; g.N = W; g.K = NG;
        g.r1_a = hpre; g.r1_lda = d.HP; g.r1_v = c.pk(c.k.wsig);
        g.Dmul = buf(c.w.Db[d.L - 1]); g.ld_dmul = W;
        if constexpr (BF) g.dmul_z = zs ? 1 : 0;
        if (!hdx) {
            SPN_TRY(G::nt(g, s));
            SPN_TRY(stream_dep(sd, s, s2));
        }
    }
    // 6. trunk, top to bottom
    const T* X0 = BF ? buf(c.w.X0b) : buf(c.w.X0);
    // the per-ray sums of dZ_0 / dZ_skip (semantic columns) by 64-point tiles: the fused dX chain
    // forms the tiles' column sums from its LDS image (no re-read of dZ), the layer-by-layer chain
    // from HBM in the same order (bit-identical), then one launch adds each ray's tiles
    const bool tsum = BF && g_tile_rowsum && d.sem && W == 512 && S % 64 == 0;
    auto ray_tiles = [&](int i, const T* dZi, bool parts_done) -> int32_t {
        float* part = c.at(i == 0 ? c.w.Rp0 : c.w.Rp4);
        ProfScope prof("ray_rowsum", s2, 0.0, (parts_done ? 0.0 : 2.0 * P * W) + 4.0 * (P / 64 + n_rays) * W);
        if (!parts_done) {
            hipLaunchKernelGGL(k_tile_rowsum16, dim3((unsigned)(P / 64)), dim3(512), 0, s2,
                               reinterpret_cast<const bf16*>(dZi), part);
            SPN_HIP(hipGetLastError());
        }
        hipLaunchKernelGGL(k_ray_tiles_sum, dim3((unsigned)cdiv(n_rays * 512, 256)), dim3(256), 0, s2, part, S / 64,
                           n_rays, c.at(i == 0 ? c.w.R0 : c.w.R4), nullptr, nullptr);
        SPN_HIP(hipGetLastError());
        return SPNERF_OK;
    };
    // both layers' tile sums written by the fused chain: one launch adds both, after the chain
    bool pair_tiles = false;
    auto ray_tiles_pair = [&]() -> int32_t {
        ProfScope prof("ray_rowsum", s2, 0.0, 2.0 * 4.0 * (P / 64 + n_rays) * W);
        hipLaunchKernelGGL(k_ray_tiles_sum, dim3((unsigned)cdiv(n_rays * 512, 256), 2), dim3(256), 0, s2, c.at(c.w.Rp0),
                           S / 64, n_rays, c.at(c.w.R0), c.at(c.w.Rp4), c.at(c.w.R4));
        SPN_HIP(hipGetLastError());
        return SPNERF_OK;
    };
    bool parts_in_bwd = false;  // the fused chain wrote the tile sums
    // layer i's weight gradient (and the per-ray sums of its dZ at layer 0 / the skip layer)
    auto layer_grads = [&](int i, const T* dZi) -> int32_t {
        // dZi holds dL/d(pre-activation of layer i).  The input of layer i >= 2 is saved as Z
        // (option zsave): staged as sin(Z) by the TN
        const bool zin = zs && i >= 2;
        const T* In = i == 0 ? X0 : buf(zin ? c.w.Db[i - 1] : c.w.Hb[i - 1]);
        const int ldin = i == 0 ? d.K0p : W;
        const int kreal = i == 0 ? d.K0 : (i == d.skip ? W + d.K0 : W);
        if (c.defer) {   // spnerf_mlp_trunk_wgrad computes it later, over this and other passes' points
        } else if (i == d.skip)
            SPN_TRY(tn_grad<T>(c, dZi, W, W, In, W, X0, d.K0p, W, W + d.K0p, s2,
                               {red(0, W, kreal, gp(x.fcW[i]), ld(x.fcW[i]), gp(x.fcb[i]))}, zin));
        else
            SPN_TRY(tn_grad<T>(c, dZi, W, W, In, ldin, nullptr, 0, c.k.Kp[i], c.k.Kp[i], s2,
                               {red(0, W, kreal, gp(x.fcW[i]), ld(x.fcW[i]), gp(x.fcb[i]))}, zin));
        if (d.sem && (i == 0 || i == d.skip)) {
            if (pair_tiles) {
            } else if (tsum) SPN_TRY(ray_tiles(i, dZi, parts_in_bwd));
            else SPN_TRY(ray_rowsum<T>(dZi, W, 0, W, S, n_rays, c.at(i == 0 ? c.w.R0 : c.w.R4), W, s2));
        }
        // a mark is recorded only once its gradients are final: deferred layers get theirs from
        // spnerf_mlp_trunk_wgrad
        return c.defer ? SPNERF_OK : grad_mark(1 + (d.L - 1 - i), s2);
    };
    if (BF && !zs && g_fused_bwd && !c.k.Wb16.empty() && c.k.Wb16[1] >= 0) {
        // the whole dX chain in one launch (k_trunk_bwd_bf16): dZ_{i-1} overwrites D_{i-1} in
        // place (the workspace serves one backward: spnerf_mlp_backward consumes it), then the
        // weight gradients of every layer
        TrunkBwdArgs a;
        a.dZtop = reinterpret_cast<const bf16*>(dZ);
        for (int i = 1; i < d.L; ++i) {
            a.Wb[i] = c.pk16(c.k.Wb16[i]);
            a.D[i - 1] = c.hb(c.w.Db[i - 1]);
            a.dZ[i - 1] = c.hb(c.w.Db[i - 1]);
        }
        a.P = P; a.L = d.L;
        if (tsum && d.skip > 0 && d.skip < d.L) {
            a.Rsum[0] = c.at(c.w.Rp0); a.rs_layer[0] = 0;
            a.Rsum[1] = c.at(c.w.Rp4); a.rs_layer[1] = d.skip;
            parts_in_bwd = true;
        }
        // algorithmic HBM bytes: dZ_{L-1} in, per layer D_{i-1} in and dZ_{i-1} out
        SPN_TRY(trunk_bwd_bf16(a, s, 2.0 * P * W * W * (d.L - 1), 2.0 * P * W * (1.0 + 2.0 * (d.L - 1))));
        SPN_TRY(stream_dep(sd, s, s2));
        pair_tiles = parts_in_bwd && g_ray_tiles_pair;
        if (pair_tiles) SPN_TRY(ray_tiles_pair());
        for (int i = d.L - 1; i >= 0; --i) SPN_TRY(layer_grads(i, i == d.L - 1 ? dZ : buf(c.w.Db[i])));
        return SPNERF_OK;
    }
    for (int i = d.L - 1; i >= 0; --i) {
        // dZ (buffer cur) holds dL/d(pre-activation of layer i); the side stream has it
        SPN_TRY(layer_grads(i, dZ));
        if (sd && s2 != s) {   // this layer's reads of buffer `cur` are issued on s2
            tn_done[i] = sd->ev[sd->next];
            sd->next = (sd->next + 1) % 64;
            SPN_HIP(hipEventRecord(tn_done[i], s2));
        }
        if (i > 0) {
            const int nxt = (cur + 1) % 3;
            // buffer nxt last held dZ_{i+2}: its weight gradient (layer i+2) must be done
            if (i + 2 <= d.L - 1 && tn_done[i + 2]) SPN_HIP(hipStreamWaitEvent(s, tn_done[i + 2], 0));
            NT g;
            g.A = dZ; g.lda = W; g.K1 = W; g.B = G::w(c, c.k.WTt[i], BF ? c.k.WTt16[i] : -1); g.ldb = W; g.C = dzb[nxt];
            g.ldc = W; g.M = (int)P; g.N = W; g.K = W; g.Dmul = buf(c.w.Db[i - 1]); g.ld_dmul = W;
            if constexpr (BF) g.dmul_z = zs && i >= 2;   // Db[i - 1] holds Z for layers >= 1
            SPN_TRY(G::nt(g, s));
            SPN_TRY(stream_dep(sd, s, s2));
            cur = nxt;
            dZ = dzb[cur];
        }
    }
    return SPNERF_OK;
}

// Deferred trunk weight gradients need every layer's dZ to outlive the backward: the fused dX
// chain of the bf16 MLP leaves dZ_i in Db[i] (and dZ_{L-1} in dZa) — the layer-by-layer chain
// rotates three buffers.
static bool trunk_wgrad_ok(const Ctx& c) {
    return c.d.bf && !g_zsave && g_fused_bwd && !c.k.Wb16.empty() && c.k.Wb16[1] >= 0;
}

// The trunk layers' weight gradients (fc_net.2i weight / bias, without the per-ray semantic
// columns, which each backward adds itself) and sun_v_net.2 / .4's over the points of up to two
// deferred backwards' workspaces per GEMM, added into grad (spnerf_mlp_trunk_wgrad).
static int32_t trunk_wgrad(const Dims& d, int n_seg, void* const* wss, const int64_t* n_rays, const int32_t* S,
                           const int32_t* flags, float* grad, hipStream_t s) {
    PIdx x;
    auto specs = param_specs(d, &x);
    auto gp = [&](int pi) { return grad + specs[pi].off; };
    auto ld = [&](int pi) { return (int)specs[pi].ld(); };
    const int W = d.W;
    for (int j = 0; j < n_seg; j += 2) {
        auto ctx = [&](int k) {
            const int fl = flags[k] & ~(SPNERF_MLP_ACCUMULATE | SPNERF_MLP_DEFER_TRUNK_WGRAD);
            Ctx c{d, packed_layout(d), ws_layout(d, n_rays[k], S[k], fl), nullptr, static_cast<float*>(wss[k]), S[k]};
            c.acc = 1;
            return c;
        };
        const Ctx c = ctx(j);
        SPN_ARG(wss[j] && (flags[j] & SPNERF_MLP_SAVE) && trunk_wgrad_ok(c), "spnerf_mlp_trunk_wgrad: bad segment");
        const bool two = j + 1 < n_seg;
        Ctx c2 = two ? ctx(j + 1) : c;
        if (two) SPN_ARG(wss[j + 1] && (flags[j + 1] & SPNERF_MLP_SAVE), "spnerf_mlp_trunk_wgrad: bad segment");
        if (c.w.P + (two ? c2.w.P : 0) == 0) continue;
        auto dzl = [&](const Ctx& q, int i) { return q.hb(i == d.L - 1 ? q.w.dZa : q.w.Db[i]); };
        const int64_t Pt = c.w.P + (two ? c2.w.P : 0);
        const int H = d.H;
        // option tn_group (> 1): the output heads' G / Q weight gradients (defer_heads), sun_v_net.4
        // / .2 and the trunk layers L-1 .. 1 (the skip layer's H part; its PE tail on the narrow
        // kernel) run g_tn_group GEMMs per launch of the DMA kernel, splits in proportion to each
        // GEMM's points (equal points per block), the slab shared out among them
        struct Item {
            TN16Args t;
            ReduceArgs r[3];
            int nr, mark, layer;
        };
        std::vector<Item> items;
        bool sunv_grouped = false, heads_grouped = false, grouped[16] = {};
        const int mode_a = (flags[j] & SPNERF_MLP_SUN_ONLY) ? 2 : 0;
        const int mode_b = two ? ((flags[j + 1] & SPNERF_MLP_SUN_ONLY) ? 2 : 0) : -1;
        // segment a (c) and / or b (c2) of one GEMM: A / B pointers of each, nullptr = not in it
        struct Seg2 {
            const bf16 *A1, *B1;
            int64_t P1;
            const bf16 *A2, *B2;
            int64_t P2;
        };
        auto seg2 = [&](const bf16* Aa, const bf16* Ba, bool in_a, const bf16* Ab, const bf16* Bb, bool in_b) {
            Seg2 g{nullptr, nullptr, 0, nullptr, nullptr, 0};
            if (in_a) g = {Aa, Ba, c.w.P, nullptr, nullptr, 0};
            if (in_b) {
                if (in_a) g.A2 = Ab, g.B2 = Bb, g.P2 = c2.w.P;
                else g = {Ab, Bb, c2.w.P, nullptr, nullptr, 0};
            }
            return g;
        };
        auto item_ok = [&](const Seg2& g, int N, int K) {
            return g.P1 + g.P2 > 0 && tn_group_ok((int)(g.P1 + g.P2), N, K) && (g.P2 == 0 || g.P1 % 32 == 0);
        };
        auto add = [&](const Seg2& g, int lda, int N, int ldb, int K, std::initializer_list<ReduceArgs> reds, int mark,
                       int layer) {
            Item it;
            it.t.A = g.A1; it.t.lda = lda; it.t.B = g.B1; it.t.ldb = ldb; it.t.K1 = K;
            it.t.P = (int)(g.P1 + g.P2); it.t.N = N; it.t.K = K;
            it.t.ld_slab = K; it.t.slab_stride = (int64_t)N * K;
            if (g.P2) {
                it.t.P1 = g.P1;
                it.t.A_s2 = g.A2 - g.P1 * lda;
                it.t.B_s2 = g.B2 - g.P1 * ldb;
            }
            it.nr = 0;
            for (const ReduceArgs& r : reds) it.r[it.nr++] = r;
            it.mark = mark;
            it.layer = layer;
            items.push_back(it);
        };
        const bool grp = g_tn_group > 1;
        const bool hda = defer_heads_for(c.w.P), hdb = two && defer_heads_for(c2.w.P), hd = hda || hdb;
        if (grp && hda && (!two || hdb)) {
            // feat (+ the semantic hidden rows) = dZ_Gᵀ · H_L; sun_v_net.0 (+ rgb / beta rows) = dZ_Qᵀ · G[:, :W]
            const bool m0a = mode_a == 0, m0b = mode_b == 0;
            const Seg2 gf = seg2(c.hb(c.w.dZG), c.hb(c.w.Hb[d.L - 1]), true, c2.hb(c2.w.dZG), c2.hb(c2.w.Hb[d.L - 1]), two);
            const Seg2 gm = seg2(c.hb(c.w.dZG) + W, c.hb(c.w.Hb[d.L - 1]), m0a, c2.hb(c2.w.dZG) + W, c2.hb(c2.w.Hb[d.L - 1]),
                                 m0b);
            const Seg2 qs = seg2(c.hb(c.w.dZQ), c.hb(c.w.G), true, c2.hb(c2.w.dZQ), c2.hb(c2.w.G), two);
            const Seg2 qr = seg2(c.hb(c.w.dZQ) + H, c.hb(c.w.G), m0a, c2.hb(c2.w.dZQ) + H, c2.hb(c2.w.G), m0b);
            const int nqr = d.beta ? 2 * H : H;
            const bool any0 = m0a || m0b;
            if (item_ok(gf, W, W) && item_ok(qs, H, W) && (!any0 || ((!d.sem || item_ok(gm, H, W)) && item_ok(qr, nqr, W)))) {
                add(gf, d.NG, W, W, W, {red(0, W, W, gp(x.featW), W, gp(x.featb))}, 0, -1);
                add(qs, d.NQ, H, d.NG, W, {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b))}, 0, -1);
                if (any0) {
                    if (d.sem) add(gm, d.NG, H, W, W, {red(0, H, W, gp(x.m1W), W, gp(x.m1b))}, 0, -1);
                    if (d.beta)
                        add(qr, d.NQ, nqr, d.NG, W,
                            {red(0, H, W, gp(x.r1W), ld(x.r1W), gp(x.r1b)), red(H, H, W, gp(x.b1W), ld(x.b1W), gp(x.b1b))}, 0, -1);
                    else
                        add(qr, d.NQ, nqr, d.NG, W, {red(0, H, W, gp(x.r1W), ld(x.r1W), gp(x.r1b))}, 0, -1);
                }
                heads_grouped = true;
            }
        }
        if (grp && SPN_DEFER_SUNV) {
            const Seg2 g3 = seg2(c.hb(c.w.dS3), c.hb(c.w.S2), true, c2.hb(c2.w.dS3), c2.hb(c2.w.S2), two);
            const Seg2 g2 = seg2(c.hb(c.w.dS2), c.hb(c.w.Q), true, c2.hb(c2.w.dS2), c2.hb(c2.w.Q), two);
            if (item_ok(g3, H, H) && item_ok(g2, H, H)) {
                add(g3, H, H, H, H, {red(0, H, H, gp(x.s3W), H, gp(x.s3b))}, 0, -1);
                add(g2, H, H, d.NQ, H, {red(0, H, H, gp(x.s2W), H, gp(x.s2b))}, 0, -1);
                sunv_grouped = true;
            }
        }
        if (grp)
            for (int i = d.L - 1; i >= 1; --i) {
                const Seg2 g = seg2(dzl(c, i), c.hb(c.w.Hb[i - 1]), true, dzl(c2, i), c2.hb(c2.w.Hb[i - 1]), two);
                if ((c.k.Kp[i] == W || i == d.skip) && i < 16 && item_ok(g, W, W)) {
                    add(g, W, W, W, W, {red(0, W, W, gp(x.fcW[i]), ld(x.fcW[i]), gp(x.fcb[i]))}, 1 + (d.L - 1 - i), i);
                    grouped[i] = true;
                }
            }
        // the skip layer's PE tail and fc_net.0 (both N = W, K = K0p over the PE rows X0b) share one
        // launch of the narrow kernel at the end, with half the splits each
        // (not with tn_group_last: the skip layer's tail then runs right after its group, so its mark
        // fires a launch earlier instead of with fc_net.0's at the very end)
        const bool pair_tail = g_tn_k64_pair && g_tn_group_last == 0 && tn_k64_ok(W, d.K0p) && d.skip >= 1 && d.skip < 16 &&
                               grouped[d.skip] && c.k.Kp[0] == d.K0p;
        bool tail_pending = false;
        for (size_t g0 = 0; g0 < items.size();) {
            size_t g1 = std::min(items.size(), g0 + (size_t)std::min(g_tn_group, kTnGroup));
            // option tn_group_last: the final group at most that many GEMMs (the ones before it one
            // launch more), so the marks of all but the lowest layers fire a group earlier and their
            // all-reduce overlaps the last group (data parallelism: a smaller exposed last bucket)
            if (g_tn_group_last > 0 && g1 == items.size() && g1 - g0 > (size_t)g_tn_group_last)
                g1 = items.size() - (size_t)g_tn_group_last;
            // one split count per point: GEMM q takes sp · P_q / Pt splits, rounds x the CUs' worth
            // of blocks, within the workspace's slab capacity
            double tiles = 0, nk = 0, nn = 0;
            for (size_t q = g0; q < g1; ++q) {
                const double w = (double)items[q].t.P / (double)Pt;
                tiles += w * tn_tiles_bf16(items[q].t.N, items[q].t.K);
                nk += w * items[q].t.N * items[q].t.K;
                nn += w * items[q].t.N;
            }
            const int64_t sp1 = std::max<int64_t>(1, (int64_t)(split_cus() / tiles));
            const int rounds = g_tn_group_rounds > 0 ? std::min(g_tn_group_rounds, kTnGroupRounds)
                                                     : (Pt / sp1 >= 65536 ? 2 : 1);
            const int64_t sp = std::max<int64_t>(1, std::min({(int64_t)(rounds * split_cus() / tiles), (int64_t)cdiv(Pt, g_tn16_min_points),
                                                             (int64_t)(c.w.slab_n / nk), (int64_t)(c.w.slab_b_n / nn)}));
            TN16Args t[kTnGroup];
            int spl[kTnGroup];
            std::vector<ReduceArgs> r;
            int64_t off = 0, off_b = 0;
            bool skip_in = false, mark0 = false;
            for (size_t q = g0; q < g1; ++q) {
                Item& it = items[q];
                const int sq = (int)std::max<int64_t>(1, sp * it.t.P / Pt);
                it.t.slab = c.at(c.w.slab) + off;
                it.t.slab_b = c.at(c.w.slab_b) + off_b;
                off += sq * it.t.slab_stride;
                off_b += (int64_t)sq * it.t.N;
                for (int k = 0; k < it.nr; ++k) {
                    ReduceArgs& rr = it.r[k];
                    rr.slab = it.t.slab; rr.ld_slab = it.t.K; rr.slab_stride = it.t.slab_stride; rr.splits = sq;
                    rr.N = it.t.N; rr.slab_b = it.t.slab_b; rr.accumulate = c.acc;
                    r.push_back(rr);
                }
                t[q - g0] = it.t;
                spl[q - g0] = sq;
                skip_in = skip_in || it.layer == d.skip;
                mark0 = mark0 || it.layer < 0;
            }
            SPN_ARG(off <= c.w.slab_n && off_b <= c.w.slab_b_n, "trunk_wgrad: slab capacity for a group of %d GEMMs",
                    (int)(g1 - g0));
            SPN_TRY(gemm_tn_bf16_group(t, (int)(g1 - g0), spl, s));
            for (size_t q = 0; q < r.size(); q += kReduceMulti)
                SPN_TRY(reduce_slabs_multi(r.data() + q, (int)std::min<size_t>(kReduceMulti, r.size() - q), s));
            if (skip_in && pair_tail) {
                tail_pending = true;   // with fc_net.0's, one launch of the narrow kernel (below)
            } else if (skip_in) {  // the skip layer's PE columns: N = W, K = K0p (the narrow kernel)
                const int l = d.skip;
                const TnSeg st{dzl(c2, l), c2.hb(c2.w.X0b), nullptr, c2.w.P};
                SPN_TRY(tn_grad<bf16>(c, dzl(c, l), W, W, c.hb(c.w.X0b), d.K0p, nullptr, 0, d.K0p, d.K0p, s,
                                      {red(0, W, d.K0, gp(x.fcW[l]) + W, ld(x.fcW[l]), nullptr)}, false, two ? &st : nullptr));
            }
            // mark 0 (the output heads) once the last group holding one of them is done
            bool later0 = false;
            for (size_t q = g1; q < items.size(); ++q) later0 = later0 || items[q].layer < 0;
            if (mark0 && !later0 && (sunv_grouped || !SPN_DEFER_SUNV) && (heads_grouped || !hd))
                SPN_TRY(grad_mark(0, s));
            for (size_t q = g0; q < g1; ++q)
                if (items[q].layer >= 0 && !(tail_pending && items[q].layer == d.skip)) SPN_TRY(grad_mark(items[q].mark, s));
            g0 = g1;
        }
        // the heads' G / Q weight gradients not grouped: per segment, as the backward computes them
        if (hd && !heads_grouped) {
            for (int k = 0; k < (two ? 2 : 1); ++k) {
                const Ctx& q = k ? c2 : c;
                if (!(k ? hdb : hda)) continue;
                const int mode = k ? mode_b : mode_a;
                const bf16 *dZQ = q.hb(q.w.dZQ), *dZG = q.hb(q.w.dZG), *Gb = q.hb(q.w.G), *HL = q.hb(q.w.Hb[d.L - 1]);
                if (mode == 0 && d.beta)
                    SPN_TRY(tn_grad<bf16>(q, dZQ, d.NQ, d.NQ, Gb, d.NG, nullptr, 0, W, W, s,
                                          {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b)), red(H, H, W, gp(x.r1W), ld(x.r1W), gp(x.r1b)),
                                           red(2 * H, H, W, gp(x.b1W), ld(x.b1W), gp(x.b1b))}));
                else if (mode == 0)
                    SPN_TRY(tn_grad<bf16>(q, dZQ, d.NQ, d.NQ, Gb, d.NG, nullptr, 0, W, W, s,
                                          {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b)), red(H, H, W, gp(x.r1W), ld(x.r1W), gp(x.r1b))}));
                else
                    SPN_TRY(tn_grad<bf16>(q, dZQ, d.NQ, H, Gb, d.NG, nullptr, 0, W, W, s, {red(0, H, W, gp(x.s1W), ld(x.s1W), gp(x.s1b))}));
                if (mode == 0 && d.sem)
                    SPN_TRY(tn_grad<bf16>(q, dZG, d.NG, d.NG, HL, W, nullptr, 0, W, W, s,
                                          {red(0, W, W, gp(x.featW), W, gp(x.featb)), red(W, H, W, gp(x.m1W), W, gp(x.m1b))}));
                else
                    SPN_TRY(tn_grad<bf16>(q, dZG, d.NG, W, HL, W, nullptr, 0, W, W, s, {red(0, W, W, gp(x.featW), W, gp(x.featb))}));
            }
            if (sunv_grouped || !SPN_DEFER_SUNV) SPN_TRY(grad_mark(0, s));
        }
        // sun_v_net.4 and .2 (sun-visibility head, in every pass): dW = dZᵀ · input over all points
        if (SPN_DEFER_SUNV && !sunv_grouped) {
            const TnSeg s3{c2.hb(c2.w.dS3), c2.hb(c2.w.S2), nullptr, c2.w.P};
            SPN_TRY(tn_grad<bf16>(c, c.hb(c.w.dS3), H, H, c.hb(c.w.S2), H, nullptr, 0, H, H, s,
                                  {red(0, H, H, gp(x.s3W), H, gp(x.s3b))}, false, two ? &s3 : nullptr));
            const TnSeg s2g{c2.hb(c2.w.dS2), c2.hb(c2.w.Q), nullptr, c2.w.P};
            SPN_TRY(tn_grad<bf16>(c, c.hb(c.w.dS2), H, H, c.hb(c.w.Q), d.NQ, nullptr, 0, H, H, s,
                                  {red(0, H, H, gp(x.s2W), H, gp(x.s2b))}, false, two ? &s2g : nullptr));
            SPN_TRY(grad_mark(0, s));   // the heads' gradients are final again
        }
        for (int i = d.L - 1; i >= 0; --i) {
            if (i < 16 && grouped[i]) continue;
            if (i == 0 && tail_pending) {
                const int l = d.skip;
                TN16Args t[2];
                int spl[2];
                ReduceArgs r[2];
                const int sp = std::max(1, tn_splits_bf16((int)Pt, W, d.K0p) / 2);
                for (int q = 0; q < 2; ++q) {
                    TN16Args& a = t[q];
                    const int li = q ? l : 0;
                    a.A = dzl(c, li); a.lda = W; a.B = c.hb(c.w.X0b); a.ldb = d.K0p; a.K1 = d.K0p;
                    a.P = (int)Pt; a.N = W; a.K = d.K0p;
                    a.slab = c.at(c.w.slab) + (int64_t)q * sp * W * d.K0p; a.ld_slab = d.K0p; a.slab_stride = (int64_t)W * d.K0p;
                    a.slab_b = q ? nullptr : c.at(c.w.slab_b);
                    if (two) {
                        a.P1 = c.w.P;
                        a.A_s2 = dzl(c2, li) - c.w.P * W;
                        a.B_s2 = c2.hb(c2.w.X0b) - c.w.P * d.K0p;
                    }
                    spl[q] = sp;
                    r[q] = q ? red(0, W, d.K0, gp(x.fcW[l]) + W, ld(x.fcW[l]), nullptr)
                             : red(0, W, d.K0, gp(x.fcW[0]), ld(x.fcW[0]), gp(x.fcb[0]));
                    r[q].slab = a.slab; r[q].ld_slab = d.K0p; r[q].slab_stride = a.slab_stride; r[q].splits = sp; r[q].N = W;
                    r[q].slab_b = a.slab_b; r[q].accumulate = c.acc;
                }
                SPN_ARG(2 * sp * (int64_t)W * d.K0p <= c.w.slab_n && sp * (int64_t)W <= c.w.slab_b_n, "trunk_wgrad: slab capacity");
                SPN_TRY(gemm_tn_bf16_k64_group(t, 2, spl, s));
                SPN_TRY(reduce_slabs_multi(r, 2, s));
                SPN_TRY(grad_mark(1 + (d.L - 1 - l), s));
                SPN_TRY(grad_mark(d.L, s));
                continue;
            }
            auto dz = [&](const Ctx& q) { return dzl(q, i); };
            auto in = [&](const Ctx& q) { return q.hb(i == 0 ? q.w.X0b : q.w.Hb[i - 1]); };
            const int ldin = i == 0 ? d.K0p : W;
            const int kreal = i == 0 ? d.K0 : (i == d.skip ? W + d.K0 : W);
            const TnSeg sg{dz(c2), in(c2), c2.hb(c2.w.X0b), c2.w.P};
            const TnSeg* psg = two ? &sg : nullptr;
            if (i == d.skip)
                SPN_TRY(tn_grad<bf16>(c, dz(c), W, W, in(c), W, c.hb(c.w.X0b), d.K0p, W, W + d.K0p, s,
                                      {red(0, W, kreal, gp(x.fcW[i]), ld(x.fcW[i]), gp(x.fcb[i]))}, false, psg));
            else
                SPN_TRY(tn_grad<bf16>(c, dz(c), W, W, in(c), ldin, nullptr, 0, c.k.Kp[i], c.k.Kp[i], s,
                                      {red(0, W, kreal, gp(x.fcW[i]), ld(x.fcW[i]), gp(x.fcb[i]))}, false, psg));
            SPN_TRY(grad_mark(1 + (d.L - 1 - i), s));
        }
    }
    return grad_mark(d.L + 1, s);
}

static int32_t mlp_backward(const Dims& d, const float* packed, const float* rays, int rs, int64_t n_rays, int S,
                            const int64_t* labels, const float* temb, int flags, float* ws, const float* d_out,
                            float* grad, float* grad_t, hipStream_t s) {
    SPN_ARG(flags & SPNERF_MLP_SAVE, "backward needs a workspace written with SPNERF_MLP_SAVE");
    SPN_ARG(!(flags & SPNERF_MLP_SIGMA_ONLY), "backward of a sigma-only pass is not supported");
    Ctx c{d, packed_layout(d), ws_layout(d, n_rays, S, flags & ~(SPNERF_MLP_ACCUMULATE | SPNERF_MLP_DEFER_TRUNK_WGRAD)),
          packed, ws, S};
    c.acc = (flags & SPNERF_MLP_ACCUMULATE) ? 1 : 0;
    c.defer = (flags & SPNERF_MLP_DEFER_TRUNK_WGRAD) ? 1 : 0;
    SPN_ARG(!c.defer || trunk_wgrad_ok(c), "backward: SPNERF_MLP_DEFER_TRUNK_WGRAD needs the bf16 MLP's fused dX chain "
                                           "(spnerf_mlp_trunk_wgrad with n_seg = 0 tells)");
    const int mode = (flags & SPNERF_MLP_SUN_ONLY) ? 2 : 0;
    const int64_t P = n_rays * S;
    const int W = d.W, H = d.H;
    PIdx x;
    auto specs = param_specs(d, &x);
    const int64_t total = specs.back().off + specs.back().numel();
    if (!c.acc) SPN_TRY(zero_fill(grad, total, s));
    if (grad_t && d.beta) SPN_TRY(zero_fill(grad_t, n_rays * d.td, s));
    if (P == 0) return SPNERF_OK;
    auto gp = [&](int pi) { return grad + specs[pi].off; };
    auto ld = [&](int pi) { return (int)specs[pi].ld(); };
    Side* sd = g_bwd_streams >= 2 ? side_stream() : nullptr;
    hipStream_t s2 = sd ? sd->s : s;
    if (d.bf) SPN_TRY(backward_points<bf16>(c, mode, packed, d_out, n_rays, grad, s, s2, sd));
    else SPN_TRY(backward_points<float>(c, mode, packed, d_out, n_rays, grad, s, s2, sd));
    SPN_TRY(stream_dep(sd, s, s2));   // step 7 reads d_out and the workspace written on s
    const hipStream_t s_main = s;
    s = s2;                           // step 7 (per-ray parameters) runs on the side stream
    // 7. per-ray parameters: sun-direction columns, t columns, sky MLP, semantic embedding
    {
        const int sky_on = mode == 0;
        RayBwdArgs a{packed, c.k, d, c.at(c.w.sky), c.at(c.w.skyh), c.at(c.w.R0), c.at(c.w.R4),
                     c.at(c.w.RQ), d_out, (int)d.NO, (int)S, labels, c.at(c.w.skyd), c.at(c.w.skydh), c.at(c.w.gemb), c.at(c.w.embr), grad_t,
                     d.sem ? 1 : 0, (d.beta && mode == 0) ? 1 : 0, sky_on};
        {
            ProfScope prof("ray_terms", s, 0.0, 0.0);
            hipLaunchKernelGGL(k_ray_bwd, dim3((unsigned)n_rays), dim3(256), 0, s, a);
            SPN_HIP(hipGetLastError());
        }
        const float* sun = rays + 8;
        const int64_t B = n_rays;
        SkinnyBatch sb(c);
        // sun_v_net.0 sun-direction columns: dW[n][W+j] = Σ_ray RQ[ray][n] sun[ray][j]
        SPN_TRY(sb.add(B, sun, rs, 3, c.at(c.w.RQ), d.NQ, H, gp(x.s1W) + W, ld(x.s1W), 1, nullptr, nullptr));
        if (sky_on) {
            SPN_TRY(sb.add(B, sun, rs, 3, c.at(c.w.skydh), H, H, gp(x.k1W), 3, 1, nullptr, gp(x.k1b)));
            SPN_TRY(sb.add(B, c.at(c.w.skyd), 4, 3, c.at(c.w.skyh), H, H, gp(x.k2W), H, 0, gp(x.k2b), nullptr));
        }
        if (d.beta && mode == 0) {
            if (d.td <= 8)
                SPN_TRY(sb.add(B, temb, d.td, d.td, c.at(c.w.RQ) + 2 * H, d.NQ, H, gp(x.b1W) + W, ld(x.b1W), 1, nullptr,
                               nullptr));
            else
                SPN_TRY(skinny(c, B, temb, d.td, d.td, c.at(c.w.RQ) + 2 * H, d.NQ, H, gp(x.b1W) + W, ld(x.b1W), 1,
                               nullptr, nullptr, s));
        }
        if (d.sem) {
            SPN_TRY(sb.add(B, c.at(c.w.embr), d.sd, d.sd, c.at(c.w.R0), W, W, gp(x.fcW[0]) + d.K0, ld(x.fcW[0]), 1,
                           nullptr, nullptr));
            SPN_TRY(sb.add(B, c.at(c.w.embr), d.sd, d.sd, c.at(c.w.R4), W, W, gp(x.fcW[d.skip]) + W + d.K0,
                           ld(x.fcW[d.skip]), 1, nullptr, nullptr));
        }
        SPN_TRY(sb.run(s));
        if (d.sem) {
            ProfScope prof("ray_terms", s, 0.0, 0.0);
            hipLaunchKernelGGL(k_class_sum, dim3((d.C + 1) * d.sd), dim3(256), 0, s, n_rays, c.at(c.w.gemb), d.sd, labels,
                               d.C, gp(x.emb), c.acc);
            SPN_HIP(hipGetLastError());
        }
    }
    SPN_TRY(stream_dep(sd, s2, s_main));  // join: the caller's stream sees every gradient
    return grad_mark(d.L + 1, s_main);
}

}  // namespace spn

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
using namespace spn;

static int* option_slot(const char* name) {
    const std::string n(name);
    // The product library's switches (at most 15): the default kernels and their one documented
    // alternate each (INTEGRATION.md §Kernel selection).
    if (n == "fused_trunk") return &g_fused_trunk;        // 0: layer-by-layer trunk GEMMs
    if (n == "trunk_tile") return &g_trunk_tile;          // 64 / 128-point training tiles
    if (n == "trunk_heads") return &g_trunk_heads;        // 0: inference heads in their own launch
    if (n == "heads_epi") return &g_heads_epi;            // 0: narrow training heads wave-per-point
    if (n == "trunk_l0") return &g_trunk_l0;              // layer 0 inside the fused trunk (1: inference only)
    if (n == "pe_inline") return &g_pe_inline;            // 0: k_encode writes the PE rows
    if (n == "tn_group") return &g_tn_group;              // weight-gradient GEMMs per group launch (1: none)
    if (n == "tn_group_last") return &g_tn_group_last;    // cap of the last group (bench.py: 2 when N > 1)
    if (n == "defer_heads") return &g_defer_heads;        // the heads' weight gradients in the group launch
    if (n == "fused_bwd") return &g_fused_bwd;            // 0: the dX chain layer by layer
    if (n == "tn_bf16_variant") return &g_tn16_variant;   // 1: 128x128 TN tiles, 2: register-staged 256x256
    if (n == "tn_bf16_k64") return &g_tn16_k64;           // 0: N = 512, K = 64 weight gradients on 128x128 tiles
    if (n == "nt_f32_variant") return &g_nt_variant;      // the fp32 (parity) NT GEMM tilings
    if (n == "pack_table") return &g_pack_table;          // 0: one re-pack launch per parameter group
    if (n == "prof_shapes") return &g_prof_shapes;        // in-library timer keyed by launch shape
#ifdef SPN_ABLATIONS
    // A/B switches of kernels measured slower than the defaults and
    // profiling ablations whose outputs are INVALID: only in a -DSPN_ABLATIONS build
    // (make -C sp-nerf_amd variant VDEF=-DSPN_ABLATIONS VLIB=libspnerf_amd_abl.so)
    if (n == "trunk_dbg") return &g_trunk_dbg;
    if (n == "trunk_var") return &g_trunk_var;
    if (n == "heads_dbg") return &g_heads_dbg;
    if (n == "trunk_nt") return &g_trunk_nt;
    if (n == "trunk_dreg") return &g_trunk_dreg;
    if (n == "trunk_bwd_dreg") return &g_trunk_bwd_dreg;
    if (n == "trunk_bwd_nt") return &g_trunk_bwd_nt;
    if (n == "trunk_sigma") return &g_trunk_sigma;
    if (n == "tn_f32_variant") return &g_tn_variant;
    if (n == "nt_bf16_variant") return &g_nt16_variant;
    if (n == "nt_bf16_ip") return &g_nt16_ip;
    if (n == "tn_bf16_ip") return &g_tn16_ip;
    if (n == "tn_bf16_bias_split") return &g_tn16_bias_split;
    if (n == "tn_bf16_few_tiles") return &g_tn16_few_tiles;
    if (n == "tn_bf16_pf") return &g_tn16_pf;
    if (n == "tn_bf16_quad") return &g_tn16_quad;
    if (n == "tn_bf16_m16") return &g_tn16_m16;
    if (n == "tn_bf16_rounds") return &g_tn16_rounds;
    if (n == "tn_group_rounds") return &g_tn_group_rounds;
    if (n == "tn_k64_pair") return &g_tn_k64_pair;
    if (n == "ray_tiles_pair") return &g_ray_tiles_pair;
    if (n == "nt_bf16_ip_gen") return &g_nt16_ip_gen;
    if (n == "nt_bf16_epi") return &g_nt16_epi;
    if (n == "grad_marks_flags") return &g_marks_flags;
    if (n == "heads_variant") return &g_heads_variant;
    if (n == "l0_split") return &g_l0_split;
    if (n == "bwd_streams") return &g_bwd_streams;
    if (n == "tn_bf16_min_points") return &g_tn16_min_points;
    if (n == "fused_heads") return &g_fused_heads;
    if (n == "zsave") return &g_zsave;
    if (n == "tn_split_tail") return &g_tn_split_tail;
    if (n == "tile_rowsum") return &g_tile_rowsum;
    if (n == "trunk2") return &g_trunk2;
    if (n == "trunk2_tile") return &g_trunk2_tile;
    if (n == "emu_bf16") return &g_emu_bf16;
    if (n == "heads_dx") return &g_heads_dx;
#endif
    return nullptr;
}

extern "C" int32_t spnerf_set_option(const char* name, int32_t value) {
    SPN_ARG(name != nullptr, "set_option: NULL name");
    int* slot = option_slot(name);
    SPN_ARG(slot != nullptr, "set_option: unknown option '%s'", name);
    *slot = value;
    return SPNERF_OK;
}

extern "C" int32_t spnerf_get_option(const char* name, int32_t* value) {
    SPN_ARG(name != nullptr && value != nullptr, "get_option: NULL pointer");
    int* slot = option_slot(name);
    SPN_ARG(slot != nullptr, "get_option: unknown option '%s'", name);
    *value = *slot;
    return SPNERF_OK;
}

extern "C" int32_t spnerf_mlp_trunk_wgrad(const spnerf_model_cfg* cfg, int32_t n_seg, void* const* workspaces,
                                          const int64_t* n_rays, const int32_t* n_samples, const int32_t* flags,
                                          float* grad_flat, void* stream) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    if (n_seg == 0) {   // capability query: may a backward defer under the current options?
        Ctx c{d, packed_layout(d), WS{}, nullptr, nullptr, 0};
        return trunk_wgrad_ok(c) ? 1 : 0;
    }
    SPN_ARG(n_seg > 0 && workspaces && n_rays && n_samples && flags && grad_flat, "spnerf_mlp_trunk_wgrad: NULL argument");
    return trunk_wgrad(d, n_seg, workspaces, n_rays, n_samples, flags, grad_flat, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int32_t spnerf_grad_marks(const spnerf_model_cfg* cfg, int32_t* mark_of_param, int32_t n_params) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    PIdx x;
    auto specs = param_specs(d, &x);
    SPN_ARG(mark_of_param && n_params == (int32_t)specs.size(), "spnerf_grad_marks: need one slot per parameter");
    SPN_ARG(d.L + 2 <= 64, "spnerf_grad_marks: too many layers");
    const int end = d.L + 1;
    for (size_t i = 0; i < specs.size(); ++i) mark_of_param[i] = 0;  // output heads (mark 0)
    for (int i = 0; i < d.L; ++i) {
        const int m = 1 + (d.L - 1 - i);
        mark_of_param[x.fcb[i]] = m;
        // the semantic columns of layer 0 / the skip layer come from per-ray sums at the end
        mark_of_param[x.fcW[i]] = (d.sem && (i == 0 || i == d.skip)) ? end : m;
    }
    // per-ray parameters and columns (step 7 of the backward)
    for (int pi : {x.emb, x.s1W, x.k1W, x.k1b, x.k2W, x.k2b, x.b1W})
        if (pi >= 0) mark_of_param[pi] = end;
    return d.L + 2;
}

extern "C" int32_t spnerf_grad_marks_arm(int32_t on) {
    if (on) SPN_ARG(marks_of_device() != nullptr, "spnerf_grad_marks_arm: cannot create the mark events");
    g_marks_armed = on ? 1 : 0;
    return SPNERF_OK;
}

extern "C" int32_t spnerf_grad_mark_wait(int32_t mark, void* stream) {
    Marks* m = marks_of_device();
    SPN_ARG(m && mark >= 0 && mark < 64, "spnerf_grad_mark_wait: bad mark");
    SPN_HIP(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream), m->ev[mark], 0));
    return SPNERF_OK;
}

extern "C" int32_t spnerf_grad_mark_query(int32_t device, int32_t mark) {
    SPN_ARG(device >= 0 && device < 64 && mark >= 0 && mark < 64, "spnerf_grad_mark_query: bad device or mark");
    Marks* m = marks_of(device, false);
    if (!m || !(m->recorded.load(std::memory_order_relaxed) & (uint64_t(1) << mark))) return 2;   // never recorded
    int cur = -1;
    SPN_HIP(hipGetDevice(&cur));
    if (cur != device) SPN_HIP(hipSetDevice(device));
    const hipError_t e = hipEventQuery(m->ev[mark]);
    if (cur != device) SPN_HIP(hipSetDevice(cur));
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    SPN_HIP(e);
    return 0;
}

extern "C" int32_t spnerf_param_count(const spnerf_model_cfg* cfg) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    return (int32_t)param_specs(d, nullptr).size();
}

extern "C" int32_t spnerf_param_info(const spnerf_model_cfg* cfg, int32_t idx, char* name, int32_t cap, int64_t* rows,
                                     int64_t* cols) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    auto v = param_specs(d, nullptr);
    SPN_ARG(idx >= 0 && idx < (int)v.size(), "param index %d out of range", idx);
    if (name && cap > 0) {
        snprintf(name, cap, "%s", v[idx].name.c_str());
    }
    if (rows) *rows = v[idx].rows;
    if (cols) *cols = v[idx].cols;
    return SPNERF_OK;
}

extern "C" int64_t spnerf_packed_bytes(const spnerf_model_cfg* cfg) {
    Dims d;
    if (make_dims(cfg, &d) != SPNERF_OK) return -1;
    return packed_layout(d).total * (int64_t)sizeof(float);
}

extern "C" int32_t spnerf_pack_params(const spnerf_model_cfg* cfg, const float* const* params, void* packed, void* stream) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    SPN_ARG(params && packed, "pack: NULL pointer");
    return pack_params(d, params, (float*)packed, (hipStream_t)stream);
}

extern "C" int64_t spnerf_mlp_workspace_bytes(const spnerf_model_cfg* cfg, int64_t n_rays, int32_t n_samples, int32_t flags) {
    Dims d;
    if (make_dims(cfg, &d) != SPNERF_OK || n_rays < 0 || n_samples <= 0) return -1;
    return ws_layout(d, n_rays, n_samples, flags).total * (int64_t)sizeof(float);
}

extern "C" int32_t spnerf_mlp_forward(const spnerf_model_cfg* cfg, const void* packed, const float* rays, int32_t ray_stride,
                                      int32_t dir_offset, int64_t n_rays, int32_t n_samples, const float* z,
                                      const int64_t* labels, const float* t_emb, int32_t flags, void* workspace, float* out,
                                      void* stream) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    SPN_ARG(packed && rays && z && workspace && out, "mlp_forward: NULL pointer");
    SPN_ARG(n_rays >= 0 && n_samples > 0 && ray_stride >= 11, "mlp_forward: bad sizes");
    SPN_ARG(dir_offset == 3 || dir_offset == 8, "mlp_forward: dir_offset must be 3 (view) or 8 (sun)");
    return mlp_forward(d, (const float*)packed, rays, ray_stride, dir_offset, n_rays, n_samples, z, labels, t_emb, flags,
                       (float*)workspace, out, (hipStream_t)stream);
}

extern "C" int32_t spnerf_mlp_forward_window(const spnerf_model_cfg* cfg, const void* packed, const float* rays,
                                             int32_t ray_stride, int32_t dir_offset, int64_t n_rays_total,
                                             int64_t ray_begin, int64_t n_rays, int32_t n_samples, const float* z,
                                             int32_t z_stride, const int64_t* labels, const float* t_emb, int32_t flags,
                                             void* workspace, float* out, void* stream) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    SPN_ARG(packed && rays && z && workspace && out, "mlp_forward_window: NULL pointer");
    SPN_ARG(n_rays >= 0 && n_samples > 0 && ray_stride >= 11, "mlp_forward_window: bad sizes");
    SPN_ARG(ray_begin >= 0 && n_rays_total >= ray_begin + n_rays, "mlp_forward_window: rays [%lld, %lld) outside %lld",
            (long long)ray_begin, (long long)(ray_begin + n_rays), (long long)n_rays_total);
    SPN_ARG(n_rays_total * n_samples < (1ll << 31) / std::max(d.NQ, d.NG), "mlp_forward_window: too many points");
    SPN_ARG(dir_offset == 3 || dir_offset == 8, "mlp_forward_window: dir_offset must be 3 (view) or 8 (sun)");
    SPN_ARG(z_stride == 0 || z_stride >= n_samples, "mlp_forward_window: z_stride %d < n_samples %d", z_stride, n_samples);
    return mlp_forward(d, (const float*)packed, rays, ray_stride, dir_offset, n_rays, n_samples, z, labels, t_emb, flags,
                       (float*)workspace, out, (hipStream_t)stream, n_rays_total, ray_begin, z_stride);
}

extern "C" int32_t spnerf_mlp_backward(const spnerf_model_cfg* cfg, const void* packed, const float* rays,
                                       int32_t ray_stride, int64_t n_rays, int32_t n_samples, const int64_t* labels,
                                       const float* t_emb, int32_t flags, void* workspace, const float* d_out,
                                       float* grad_flat, float* grad_t_emb, void* stream) {
    Dims d;
    SPN_TRY(make_dims(cfg, &d));
    SPN_ARG(packed && rays && workspace && d_out && grad_flat, "mlp_backward: NULL pointer");
    SPN_ARG(!d.sem || labels, "mlp_backward: semantic model needs labels");
    SPN_ARG(!d.beta || (flags & SPNERF_MLP_SUN_ONLY) || t_emb, "mlp_backward: beta model needs t_emb");
    return mlp_backward(d, (const float*)packed, rays, ray_stride, n_rays, n_samples, labels, t_emb, flags,
                        (float*)workspace, d_out, grad_flat, grad_t_emb, (hipStream_t)stream);
}
