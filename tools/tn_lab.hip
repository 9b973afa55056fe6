// Weight-gradient GEMM lab (tools only): slab[s][n][k] = Σ_p A[p][n]·B[p][k] over P points
// (N = K = 512, bf16 operands, fp32 sums) — the library's LDS-DMA kernel (gemm_tn_bf16, row
// layout [P][F]) against a kernel with NO LDS that loads its MFMA fragments straight from a
// point-interleaved layout [P/8][F][8] (8 consecutive points of one feature = one 16-B lane
// load, a wave's 64 lanes = 2 point groups x 32 features = two 512-B runs).
//   make -C tools tn_lab && ./tools/tn_lab [P] [iters]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../sp-nerf_amd/csrc/common.h"
#include "../sp-nerf_amd/csrc/gemm_bf16.h"

using namespace spn;

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// 256 x 256 tile per block, 8 waves of 128 x 64 (4 x 2 32x32 accumulators), one block per CU;
// per 16-point k-step a wave loads its 4 A and 2 B fragments (16 B per lane each) from the
// interleaved operands, DEPTH k-steps ahead in registers.
template <int DEPTH>
__global__ __launch_bounds__(512) void k_tn_direct(const bf16* __restrict__ A, const bf16* __restrict__ B, int P, int N,
                                                   int K, int pps, float* slab, int resident) {
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nK = K / 256, ntiles = (N / 256) * nK;
    const int w = xcd_remap(blockIdx.x, gridDim.x);
    const int split = w / ntiles, t = w % ntiles;
    const int n0 = (t / nK) * 256, k0 = (t % nK) * 256;
    const int p_beg = resident ? 0 : split * pps, p_end = min(P, p_beg + pps);
    const int nks = (p_end - p_beg) / 16;
    const int wa = wid >> 2, wb = wid & 3, h = lane >> 5, m = lane & 31;
    // lane bases: point group (p / 8 + h), feature n0 + 128 wa + m (+ 32 i) / k0 + 64 wb + m (+ 32 j)
    const bf16* pa = A + ((int64_t)(p_beg / 8 + h) * N + n0 + 128 * wa + m) * 8;
    const bf16* pb = B + ((int64_t)(p_beg / 8 + h) * K + k0 + 64 * wb + m) * 8;
    const int64_t sa = (int64_t)2 * N * 8, sb = (int64_t)2 * K * 8;  // one k-step = 2 point groups
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    u32x4 ra[DEPTH][4], rb[DEPTH][2];
    auto load = [&](int d, int ks) {
        const int kc = min(ks, nks - 1);
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[d][i] = ldg16(pa + kc * sa + 32 * 8 * i);
#pragma unroll
        for (int j = 0; j < 2; ++j) rb[d][j] = ldg16(pb + kc * sb + 32 * 8 * j);
    };
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) load(d, d);
    for (int ks0 = 0; ks0 < nks; ks0 += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            if (ks0 + d < nks) {  // block-uniform
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, ra[d][i]),
                                                                          __builtin_bit_cast(bf16x8, rb[d][j]), acc[i][j], 0, 0, 0);
                load(d, ks0 + d + DEPTH);
            }
        }
    }
    float* out = slab + (int64_t)split * N * K;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = k0 + wb * 64 + j * 32 + m;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int n = n0 + wa * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                out[(int64_t)n * K + k] = acc[i][j][r];
            }
    }
}

__global__ void k_reduce(const float* slab, int splits, int64_t nk, float* out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nk) return;
    float s = 0.f;
    for (int q = 0; q < splits; ++q) s += slab[q * nk + e];
    out[e] = s;
}

int main(int argc, char** argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 1 << 20;
    const int iters = argc > 2 ? atoi(argv[2]) : 20;
    const int N = 512, K = 512;
    std::vector<uint16_t> a((size_t)P * N), b((size_t)P * K), ai(a.size()), bi(b.size());
    srand(1);
    auto rnd = [] {
        float x = 2.f * (float)rand() / (float)RAND_MAX - 1.f;
        uint32_t u;
        memcpy(&u, &x, 4);
        return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    };
    // TN_ASCALE: scale of A (the bench's A is a gradient dZ, orders of magnitude below B = H)
    const float ascale = getenv("TN_ASCALE") ? (float)atof(getenv("TN_ASCALE")) : 1.f;
    for (auto& v : a) {
        const uint16_t r = rnd();
        uint32_t u = (uint32_t)r << 16;
        float x;
        memcpy(&x, &u, 4);
        x *= ascale;
        memcpy(&u, &x, 4);
        v = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
    for (auto& v : b) v = rnd();
    for (int p = 0; p < P; ++p) {
        for (int f = 0; f < N; ++f) ai[((size_t)(p / 8) * N + f) * 8 + p % 8] = a[(size_t)p * N + f];
        for (int f = 0; f < K; ++f) bi[((size_t)(p / 8) * K + f) * 8 + p % 8] = b[(size_t)p * K + f];
    }
    bf16 *dA, *dB, *dAi, *dBi;
    CK(hipMalloc(&dA, a.size() * 2));
    CK(hipMalloc(&dB, b.size() * 2));
    CK(hipMalloc(&dAi, a.size() * 2));
    CK(hipMalloc(&dBi, b.size() * 2));
    CK(hipMemcpy(dA, a.data(), a.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, b.data(), b.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dAi, ai.data(), ai.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dBi, bi.data(), bi.size() * 2, hipMemcpyHostToDevice));
    const int splits = tn_splits_bf16(P, N, K);
    float *slab, *slab_b, *ref, *got;
    CK(hipMalloc(&slab, (size_t)4 * splits * N * K * 4));   // (room for the 4x-splits runs)
    CK(hipMalloc(&slab_b, (size_t)4 * splits * N * 4));
    CK(hipMalloc(&ref, (size_t)N * K * 4));
    CK(hipMalloc(&got, (size_t)N * K * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto f) {
        for (int i = 0; i < 3; ++i) f();
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < iters; ++i) f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return 1e3 * ms / iters;
    };
    const double flop = 2.0 * P * N * K, bytes = 2.0 * P * (N + K);
#ifdef ND_STAMPS
    {   // phase stamps of the library kernel's main loop (tools/tn_lab_stamps): lane 0 of waves 0 / 4
        // of blocks 0 / 128; per phase transition the mean s_memtime cycles over the stages
        unsigned long long* st;
        CK(hipMalloc(&st, 4 * 4096 * 8));
        CK(hipMemset(st, 0, 4 * 4096 * 8));
        TN16Args t;
        t.A = dA; t.lda = N; t.B = dB; t.ldb = K; t.K1 = K;
        t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K; t.slab_b = slab_b;
        t.P = P; t.N = N; t.K = K;
        for (int rep = 0; rep < 5; ++rep) gemm_tn_bf16(t, splits, 0);   // warm clocks
        t.stamps = st;
        gemm_tn_bf16(t, splits, 0);
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> h(4 * 4096);
        CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        for (int w = 0; w < 4; ++w) {
            const unsigned long long* r = h.data() + w * 4096;
            const int n = (int)r[4095];
            double sum[16][16] = {};
            int cnt[16][16] = {};
            double total = 0;
            for (int i = 1; i < n && i < 4095; ++i) {
                const int a = (int)(r[i - 1] & 15), b = (int)(r[i] & 15);
                const double d = (double)((r[i] >> 4) - (r[i - 1] >> 4));
                sum[a][b] += d;
                cnt[a][b] += 1;
                total += d;
            }
            printf("stream %d (block %d wave %d): %d stamps, %.0f cycles\n", w, w >= 2 ? 128 : 0, (w & 1) * 4, n, total);
            for (int a = 0; a < 16; ++a)
                for (int b = 0; b < 16; ++b)
                    if (cnt[a][b]) printf("   %2d -> %2d: n=%4d mean %7.1f cyc  share %5.1f%%\n", a, b, cnt[a][b], sum[a][b] / cnt[a][b],
                                          100.0 * sum[a][b] / total);
        }
        return 0;
    }
#endif
    // profiling mode (argv[3]): one configuration only, for PMC passes — 1 DMA one-row, 2 quad
    // one-row, 3 DMA, 4 quad, 5 prefetched one-row, 6 16x16x32 one-row, 7 16x16x32; 8 / 9: the
    // library kernel with / without the bias sums, alternating (what the bias rows cost)
    const int mode = argc > 3 ? atoi(argv[3]) : 0;
    if (mode == 8) {
        TN16Args t;
        t.A = dA; t.lda = N; t.B = dB; t.ldb = K; t.K1 = K;
        t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K;
        t.P = P; t.N = N; t.K = K;
        for (int r = 0; r < 3; ++r)
            for (int b : {1, 0}) {
                t.slab_b = b ? slab_b : nullptr;
                const double u = timeit([&] { gemm_tn_bf16(t, splits, 0); });
                printf("library DMA TN %s bias sums: %8.1f us  %7.1f TF/s\n", b ? "with" : "without", u, flop / u * 1e-6);
            }
        return 0;
    }
    if (mode) {
        TN16Args t;
        t.A = dA; t.lda = (mode == 1 || mode == 2 || mode == 5 || mode == 6) ? 0 : N; t.B = dB; t.ldb = t.lda ? K : 0; t.K1 = K;
        t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K; t.slab_b = slab_b;
        t.P = P; t.N = N; t.K = K;
        g_tn16_quad = mode == 2 || mode == 4;
        g_tn16_pf = mode == 5;
        g_tn16_m16 = mode == 6 || mode == 7 ? 1 : 0;
        if (mode == 7) { t.lda = N; t.ldb = K; }
        const double u = timeit([&] { gemm_tn_bf16(t, splits, 0); });
        printf("mode %d: %8.1f us  %7.1f TF/s\n", mode, u, flop / u * 1e-6);
        return 0;
    }
    // library kernel (row layout), its slab reduction on the side
    TN16Args t;
    t.A = dA; t.lda = N; t.B = dB; t.ldb = K; t.K1 = K;
    t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K; t.slab_b = slab_b;
    t.P = P; t.N = N; t.K = K;
    const double ul = timeit([&] { gemm_tn_bf16(t, splits, 0); });
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_reduce, dim3(N * K / 256), dim3(256), 0, 0, slab, splits, (int64_t)N * K, ref);
    printf("P=%d splits=%d  library DMA TN: %8.1f us  %7.1f TF/s  %6.2f TB/s (operands)\n", P, splits, ul, flop / ul * 1e-6,
           bytes / ul * 1e-6);
    for (int variant : {2, 1}) {   // 2: option tn_bf16_quad (4 waves of 128x128); 1: tn_bf16_pf
        g_tn16_quad = variant == 2;
        g_tn16_pf = variant == 1;
        const char* name = variant == 2 ? "quad-wave" : "prefetched fragments";
        const double up = timeit([&] { gemm_tn_bf16(t, splits, 0); });
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_reduce, dim3(N * K / 256), dim3(256), 0, 0, slab, splits, (int64_t)N * K, got);
        std::vector<float> hr((size_t)N * K), hg(hr.size());
        CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hg.data(), got, hg.size() * 4, hipMemcpyDeviceToHost));
        printf("library DMA TN, %s: %8.1f us  %7.1f TF/s  %6.2f TB/s  bitwise %s\n", name, up, flop / up * 1e-6,
               bytes / up * 1e-6, memcmp(hr.data(), hg.data(), hr.size() * 4) == 0 ? "equal" : "DIFFERENT");
        TN16Args t0 = t;
        t0.lda = 0;
        t0.ldb = 0;
        const double u0 = timeit([&] { gemm_tn_bf16(t0, splits, 0); });
        printf("  ... one row (on-chip): %8.1f us  %7.1f TF/s\n", u0, flop / u0 * 1e-6);
        const double u2 = timeit([&] { gemm_tn_bf16(t, 2 * splits, 0); });
        printf("  ... %3d splits: %8.1f us  %7.1f TF/s\n", 2 * splits, u2, flop / u2 * 1e-6);
        g_tn16_pf = 0;
        g_tn16_quad = 0;
    }
    for (int ip : {3, 4, 5, 1}) {   // option tn_bf16_ip: 3 = DMAs spread over the MFMAs, 4 = the two waves of a SIMD a k-step apart, 5 = bias in registers
        g_tn16_ip = ip;
        const double up = timeit([&] { gemm_tn_bf16(t, splits, 0); });
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_reduce, dim3(N * K / 256), dim3(256), 0, 0, slab, splits, (int64_t)N * K, got);
        std::vector<float> hr((size_t)N * K), hg(hr.size());
        CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hg.data(), got, hg.size() * 4, hipMemcpyDeviceToHost));
        const double u2 = timeit([&] { gemm_tn_bf16(t, 2 * splits, 0); });
        printf("library DMA TN, IP %d: %8.1f us  %7.1f TF/s  %6.2f TB/s  bitwise %s;  %d splits: %8.1f us\n", ip, up,
               flop / up * 1e-6, bytes / up * 1e-6, memcmp(hr.data(), hg.data(), hr.size() * 4) == 0 ? "equal" : "DIFFERENT",
               2 * splits, u2);
    }
    g_tn16_ip = 1;
    for (int m16 : {1, 2, 3, 4}) {   // option tn_bf16_m16: 16x16x32 kernels (1/2: 8 waves, 3/4: 16 waves; 4 / 5 DMA stages)
        g_tn16_m16 = m16;
        const double up = timeit([&] { gemm_tn_bf16(t, splits, 0); });
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_reduce, dim3(N * K / 256), dim3(256), 0, 0, slab, splits, (int64_t)N * K, got);
        std::vector<float> hr((size_t)N * K), hg(hr.size()), br((size_t)N), bg((size_t)N);
        CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hg.data(), got, hg.size() * 4, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (size_t i = 0; i < hr.size(); ++i) {
            md = fmax(md, fabs((double)hr[i] - hg[i]));
            mx = fmax(mx, fabs((double)hr[i]));
        }
        // bias sums of split 0 against the 32x32x16 kernel's (same row order: bitwise)
        CK(hipMemcpy(bg.data(), slab_b, bg.size() * 4, hipMemcpyDeviceToHost));
        g_tn16_m16 = 0;
        gemm_tn_bf16(t, splits, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(br.data(), slab_b, br.size() * 4, hipMemcpyDeviceToHost));
        g_tn16_m16 = m16;
        printf("16x16x32 TN m16=%d, %d stages: %8.1f us  %7.1f TF/s  %6.2f TB/s  max|diff|/max|ref| %.2e  bias %s\n", m16, m16 % 2 == 0 ? 5 : 4,
               up, flop / up * 1e-6, bytes / up * 1e-6, md / mx,
               memcmp(br.data(), bg.data(), br.size() * 4) == 0 ? "bitwise" : "DIFFERENT");
        TN16Args t0 = t;
        t0.lda = 0;
        t0.ldb = 0;
        const double u0 = timeit([&] { gemm_tn_bf16(t0, splits, 0); });
        printf("  ... one row (on-chip): %8.1f us  %7.1f TF/s\n", u0, flop / u0 * 1e-6);
        const double u2 = timeit([&] { gemm_tn_bf16(t, 2 * splits, 0); });
        printf("  ... %3d splits: %8.1f us  %7.1f TF/s\n", 2 * splits, u2, flop / u2 * 1e-6);
        g_tn16_m16 = 0;
    }
    {   // the register-staged 256x256 kernel (tn_bf16_variant 2), normal and one-row operands
        g_tn16_variant = 2;
        const double u = timeit([&] { gemm_tn_bf16(t, splits, 0); });
        TN16Args t0 = t;
        t0.lda = 0;
        t0.ldb = 0;
        const double u0 = timeit([&] { gemm_tn_bf16(t0, splits, 0); });
        printf("register-staged TN (variant 2): %8.1f us  %7.1f TF/s; one row (on-chip): %8.1f us  %7.1f TF/s\n", u,
               flop / u * 1e-6, u0, flop / u0 * 1e-6);
        g_tn16_variant = 3;
    }
    {   // the same kernel with every point row the same row (lda = ldb = 0): operands from L2 / L1,
        // the on-chip ceiling of the DMA pipeline
        TN16Args t0 = t;
        t0.lda = 0;
        t0.ldb = 0;
        const double u0 = timeit([&] { gemm_tn_bf16(t0, splits, 0); });
        printf("library DMA TN, one row (on-chip): %8.1f us  %7.1f TF/s\n", u0, flop / u0 * 1e-6);
        for (int sp : {splits / 2, splits * 2, splits * 4}) {
            const double u1 = timeit([&] { gemm_tn_bf16(t, sp, 0); });
            printf("library DMA TN, %3d splits: %8.1f us  %7.1f TF/s  %6.2f TB/s\n", sp, u1, flop / u1 * 1e-6, bytes / u1 * 1e-6);
        }
    }
    const int pps = (P + splits - 1) / splits;
    auto run = [&](auto kern, const char* name, int resident = 0) {
        const double us = timeit([&] { hipLaunchKernelGGL(kern, dim3(4 * splits), dim3(512), 0, 0, dAi, dBi, P, N, K, pps, slab, resident); });
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_reduce, dim3(N * K / 256), dim3(256), 0, 0, slab, splits, (int64_t)N * K, got);
        std::vector<float> hr((size_t)N * K), hg(hr.size());
        CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hg.data(), got, hg.size() * 4, hipMemcpyDeviceToHost));
        double md = 0, mx = 0;
        for (size_t i = 0; i < hr.size(); ++i) {
            md = fmax(md, fabs((double)hr[i] - hg[i]));
            mx = fmax(mx, fabs((double)hr[i]));
        }
        printf("%-24s %8.1f us  %7.1f TF/s  %6.2f TB/s  max|diff|/max|ref| %.2e\n", name, us, flop / us * 1e-6, bytes / us * 1e-6,
               md / mx);
    };
    run(k_tn_direct<2>, "direct, 2 steps ahead");
    run(k_tn_direct<3>, "direct, 3 steps ahead");
    run(k_tn_direct<4>, "direct, 4 steps ahead");
    run(k_tn_direct<2>, "direct 2, L2-resident", 1);
    run(k_tn_direct<4>, "direct 4, L2-resident", 1);
    CK(hipMemset(dAi, 0, a.size() * 2));
    CK(hipMemset(dBi, 0, b.size() * 2));
    run(k_tn_direct<2>, "direct 2, zero operands");
    run(k_tn_direct<2>, "direct 2, zero + resident", 1);
    return 0;
}
