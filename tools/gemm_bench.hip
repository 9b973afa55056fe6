// Standalone timing of the fp32 MFMA GEMM kernels (tools only; not part of the library ABI).
//   make -C tools gemm_bench && ./tools/gemm_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../sp-nerf_amd/csrc/gemm_f32.h"

using namespace spn;

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

static float* rnd(size_t n, float scale, unsigned seed) {
    std::vector<float> h(n);
    srand(seed);
    for (auto& v : h) v = scale * (2.f * rand() / RAND_MAX - 1.f);
    float* d;
    CK(hipMalloc(&d, n * 4));
    CK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
    return d;
}

template <typename F>
static double time_it(F f, int iters = 20) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return 1e3 * ms / iters;  // us
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 65536, N = 512, K = argc > 2 ? atoi(argv[2]) : 512;
    float* A = rnd((size_t)M * K, 1.f, 1);
    float* B = rnd((size_t)N * K, 0.1f, 2);
    float* bias = rnd(N, 0.1f, 3);
    float *C, *D, *slab, *slab_b;
    CK(hipMalloc(&C, (size_t)M * N * 4));
    CK(hipMalloc(&D, (size_t)M * N * 4));
    CK(hipMalloc(&slab, (size_t)64 * N * K * 4));
    CK(hipMalloc(&slab_b, (size_t)64 * N * 4));
    const double flop = 2.0 * M * N * K;
    auto report = [&](const char* name, double us) { printf("%-34s %9.1f us  %6.1f TF/s\n", name, us, flop / us * 1e-6); };

    NTArgs g;
    g.A = A; g.lda = K; g.K1 = K; g.B = B; g.ldb = K; g.C = C; g.ldc = N; g.M = M; g.N = N; g.K = K;
    // correctness cross-check of every variant against variant 0 (fwd epilogue incl. Dout)
    {
        std::vector<float> ref((size_t)M * N), got((size_t)M * N), refD((size_t)M * N), gotD((size_t)M * N);
        NTArgs f = g;
        f.bias = bias; f.act = 1; f.w0 = 1.f; f.Dout = D; f.ld_dout = N;
        gemm_nt(f, 0, 0);
        CK(hipMemcpy(ref.data(), C, ref.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(refD.data(), D, ref.size() * 4, hipMemcpyDeviceToHost));
        for (int v = 1; v < 9; ++v) {
            CK(hipMemset(C, 0, ref.size() * 4));
            CK(hipMemset(D, 0, ref.size() * 4));
            gemm_nt(f, 0, v);
            CK(hipMemcpy(got.data(), C, ref.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(gotD.data(), D, ref.size() * 4, hipMemcpyDeviceToHost));
            double md = 0, mdd = 0;
            for (size_t i = 0; i < ref.size(); ++i) {
                md = std::max(md, (double)std::fabs(ref[i] - got[i]));
                mdd = std::max(mdd, (double)std::fabs(refD[i] - gotD[i]));
            }
            printf("variant %d max|diff| vs variant 0: C %.3g D %.3g\n", v, md, mdd);
        }
    }
    for (int v = 0; v < 9; ++v) {
        char nm[64];
        snprintf(nm, 64, "nt plain variant %d", v);
        report(nm, time_it([&] { gemm_nt(g, 0, v); }));
    }
    for (int v = 0; v < 9; ++v) {
        NTArgs f = g;
        f.bias = bias; f.act = 1; f.w0 = 1.f; f.Dout = D; f.ld_dout = N;
        char nm[64];
        snprintf(nm, 64, "nt fwd variant %d", v);
        report(nm, time_it([&] { gemm_nt(f, 0, v); }));
    }
    NTArgs f = g;
    f.bias = bias; f.act = 1; f.w0 = 1.f; f.Dout = D; f.ld_dout = N;
    report("nt fwd: bias+sincos+Dout", time_it([&] { gemm_nt(f, 0); }));
    NTArgs f2 = f;
    f2.Dout = nullptr;
    report("nt fwd: bias+sin, no Dout", time_it([&] { gemm_nt(f2, 0); }));
    NTArgs b = g;
    b.Dmul = D; b.ld_dmul = N;
    report("nt bwd: Dmul", time_it([&] { gemm_nt(b, 0); }));
    TNArgs t;
    t.A = C; t.lda = N; t.B = A; t.ldb = K; t.K1 = K; t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K;
    t.slab_b = slab_b; t.P = M; t.N = N; t.K = K;
    const int sp = tn_splits(M, N, K);
    report("tn (dW) 1 stage", time_it([&] { gemm_tn(t, sp, 0, 0); }));
    report("tn (dW) 2 stages", time_it([&] { gemm_tn(t, sp, 0, 1); }));
    report("tn (dW) 2 stages, 2 ahead", time_it([&] { gemm_tn(t, sp, 0, 2); }));
    {  // slabs of variants 0 and 2 vs variant 1 (same k-order: bit-identical)
        const size_t ns = (size_t)sp * N * K;
        std::vector<float> ref(ns), got(ns);
        gemm_tn(t, sp, 0, 1);
        CK(hipMemcpy(ref.data(), slab, ns * 4, hipMemcpyDeviceToHost));
        for (int v : {0, 2}) {
            CK(hipMemset(slab, 0, ns * 4));
            gemm_tn(t, sp, 0, v);
            CK(hipMemcpy(got.data(), slab, ns * 4, hipMemcpyDeviceToHost));
            double md = 0;
            for (size_t i = 0; i < ns; ++i) md = std::max(md, (double)std::fabs(ref[i] - got[i]));
            printf("tn variant %d max|diff| vs variant 1: %.3g\n", v, md);
        }
    }
    for (int v = 0; v < 9; ++v) {
        NTArgs bb = b;
        char nm[64];
        snprintf(nm, 64, "nt bwd Dmul variant %d", v);
        report(nm, time_it([&] { gemm_nt(bb, 0, v); }));
    }
    printf("tn splits=%d\n", sp);
    {  // point-split sweep of the default TN variant (timing only)
        float *big, *big_b;
        CK(hipMalloc(&big, (size_t)256 * N * K * 4));
        CK(hipMalloc(&big_b, (size_t)256 * N * 4));
        TNArgs ts = t;
        ts.slab = big;
        ts.slab_b = big_b;
        for (int s2 : {16, 32, 64, 128, 256}) {
            if (s2 * 256 > M) continue;
            char nm[64];
            snprintf(nm, 64, "tn variant 2, %d splits", s2);
            report(nm, time_it([&] { gemm_tn(ts, s2, 0, 2); }));
        }
        CK(hipFree(big));
        CK(hipFree(big_b));
    }
    return 0;
}
