// Correctness + timing of the bf16 MFMA GEMMs (tools only; not part of the library ABI).
//   make -C tools gemm_bench_bf16 && ./tools/gemm_bench_bf16 [P]
// Every shape is checked against an fp64 host product of the same bf16-rounded operands on a
// sample of rows / entries; the first block of shapes covers the MLP's edge cases (split A / B
// segments, N and K not multiples of the 128 tile, P not a multiple of the 64-point step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../sp-nerf_amd/csrc/gemm_bf16.h"
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

static float bfr(float x) {  // round to bf16 (RNE), back to float
    uint32_t u;
    memcpy(&u, &x, 4);
    u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
    float y;
    memcpy(&y, &u, 4);
    return y;
}

struct HMat {
    int rows, cols;
    std::vector<float> h;  // bf16-rounded values
    bf16* d = nullptr;
    HMat(int r, int c, float scale, unsigned seed) : rows(r), cols(c), h((size_t)r * c) {
        srand(seed);
        std::vector<uint16_t> raw(h.size());
        for (size_t i = 0; i < h.size(); ++i) {
            h[i] = bfr(scale * (2.f * (float)rand() / (float)RAND_MAX - 1.f));
            uint32_t u;
            memcpy(&u, &h[i], 4);
            raw[i] = (uint16_t)(u >> 16);
        }
        CK(hipMalloc(&d, raw.size() * 2));
        CK(hipMemcpy(d, raw.data(), raw.size() * 2, hipMemcpyHostToDevice));
    }
    float at(int r, int c) const { return h[(size_t)r * cols + c]; }
};

static std::vector<float> dl16(const bf16* d, size_t n) {
    std::vector<uint16_t> raw(n);
    CK(hipMemcpy(raw.data(), d, n * 2, hipMemcpyDeviceToHost));
    std::vector<float> f(n);
    for (size_t i = 0; i < n; ++i) {
        uint32_t u = (uint32_t)raw[i] << 16;
        memcpy(&f[i], &u, 4);
    }
    return f;
}

static int g_iters = 20;

template <typename F>
static double time_it(F f, int iters = g_iters) {
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

static int fails = 0;

// C[M,N] = sin(A·B^T + bias) (act) or (A·B^T)·Dmul, A = [A1 | A2] split at K1
static void check_nt(int M, int N, int K, int K1, bool sine, bool timing) {
    HMat A1(M, K1, 1.f, 1), A2(M, std::max(8, K - K1), 1.f, 2), B(N, K, 0.1f, 3), Dm(M, N, 1.f, 4);
    std::vector<float> bias(N);
    for (int i = 0; i < N; ++i) bias[i] = 0.01f * (i % 17);
    float* dbias;
    CK(hipMalloc(&dbias, N * 4));
    CK(hipMemcpy(dbias, bias.data(), N * 4, hipMemcpyHostToDevice));
    bf16 *C, *D;
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&D, (size_t)M * N * 2));
    NT16Args g;
    g.A = A1.d; g.lda = K1; g.A2 = A2.d; g.lda2 = A2.cols; g.K1 = K1;
    g.B = B.d; g.ldb = K; g.C = C; g.ldc = N; g.M = M; g.N = N; g.K = K;
    if (sine) { g.bias = dbias; g.act = 1; g.w0 = 1.f; g.Dout = D; g.ld_dout = N; }
    else { g.Dmul = Dm.d; g.ld_dmul = N; }
    std::vector<uint16_t> c5;
    for (int v : {1, 3, 5, 6, 7, 8}) {
    CK(hipMemset(C, 0, (size_t)M * N * 2));
    if (gemm_nt_bf16(g, 0, v) != 0) { printf("launch refused\n"); fails++; return; }
    CK(hipDeviceSynchronize());
    auto c = dl16(C, (size_t)M * N), dd = dl16(D, (size_t)M * N);
    double worst = 0, worstd = 0;
    for (int s = 0; s < 256; ++s) {
        const int r = (int)((int64_t)s * 7919 % M);
        for (int n = 0; n < N; ++n) {
            double acc = 0;
            for (int k = 0; k < K; ++k) acc += (double)(k < K1 ? A1.at(r, k) : A2.at(r, k - K1)) * B.at(n, k);
            double ref, refd = 1;
            if (sine) { ref = std::sin(acc + bias[n]); refd = std::cos(acc + bias[n]); }
            else ref = acc * Dm.at(r, n);
            worst = std::max(worst, std::fabs(ref - c[(size_t)r * N + n]));
            if (sine) worstd = std::max(worstd, std::fabs(refd - dd[(size_t)r * N + n]));
        }
    }
    bool ok = worst < 2e-2 && worstd < 2e-2;  // bf16 output rounding: |y| <= ~2, ulp 2^-8
    {   // variants 5 and 8 accumulate in the same k order: bit-identical C
        std::vector<uint16_t> raw((size_t)M * N);
        CK(hipMemcpy(raw.data(), C, raw.size() * 2, hipMemcpyDeviceToHost));
        if (v == 5) c5 = raw;
        if (v == 8 && raw != c5) { printf("[v8 != v5 bitwise] "); ok = false; }
    }
    if (!ok) fails++;
    printf("nt%d M=%-7d N=%-4d K=%-4d K1=%-4d %s  max|err| C %.2e D %.2e  %s", v, M, N, K, K1, sine ? "sine" : "dmul", worst,
           worstd, ok ? "ok" : "FAIL");
    if (timing) {
        const double us = time_it([&] { gemm_nt_bf16(g, 0, v); });
        printf("   %8.1f us %7.1f TF/s", us, 2.0 * M * N * K / us * 1e-6);
    }
    printf("\n");
    }
    CK(hipFree(C)); CK(hipFree(D)); CK(hipFree(dbias));
}

// saved-Z trunk layers (option zsave): Z stored as fp16 bits; forward zround + dout_z, backward
// dmul_z (x cos(Z)) and TN b_sin (B staged as bf16(sin(Z)))
struct ZMat {
    int rows, cols;
    std::vector<float> h;  // fp16-rounded values
    bf16* d = nullptr;     // fp16 bits
    ZMat(int r, int c, float scale, unsigned seed) : rows(r), cols(c), h((size_t)r * c) {
        srand(seed);
        std::vector<uint16_t> raw(h.size());
        for (size_t i = 0; i < h.size(); ++i) {
            const _Float16 z = (_Float16)(scale * (2.f * (float)rand() / (float)RAND_MAX - 1.f));
            h[i] = (float)z;
            raw[i] = __builtin_bit_cast(uint16_t, z);
        }
        CK(hipMalloc(&d, raw.size() * 2));
        CK(hipMemcpy(d, raw.data(), raw.size() * 2, hipMemcpyHostToDevice));
    }
    float at(int r, int c) const { return h[(size_t)r * cols + c]; }
};

static void check_z(int M) {
    const int N = 512, K = 512;
    HMat A(M, K, 1.f, 11), B(N, K, 0.1f, 12);
    ZMat Z(M, N, 3.f, 13);
    bf16 *C, *D;
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&D, (size_t)M * N * 2));
    for (int v : {1, 5, 8}) {
        NT16Args g;
        g.A = A.d; g.lda = K; g.K1 = K; g.B = B.d; g.ldb = K; g.C = C; g.ldc = N; g.M = M; g.N = N; g.K = K;
        g.Dmul = Z.d; g.ld_dmul = N; g.dmul_z = 1;
        if (gemm_nt_bf16(g, 0, v) != 0) { printf("launch refused\n"); fails++; return; }
        CK(hipDeviceSynchronize());
        auto c = dl16(C, (size_t)M * N);
        double worst = 0;
        for (int s = 0; s < 128; ++s) {
            const int r = (int)((int64_t)s * 7919 % M);
            for (int n = 0; n < N; ++n) {
                double acc = 0;
                for (int k = 0; k < K; ++k) acc += (double)A.at(r, k) * B.at(n, k);
                worst = std::max(worst, std::fabs(acc * std::cos((double)Z.at(r, n)) - c[(size_t)r * N + n]));
            }
        }
        const bool ok = worst < 2e-2;
        if (!ok) fails++;
        printf("nt%d dmul_z  M=%d max|err| %.2e  %s\n", v, M, worst, ok ? "ok" : "FAIL");
        // forward: zround + dout_z (w0 = 1)
        NT16Args f;
        f.A = A.d; f.lda = K; f.K1 = K; f.B = B.d; f.ldb = K; f.C = C; f.ldc = N; f.M = M; f.N = N; f.K = K;
        f.act = 1; f.w0 = 1.f; f.Dout = D; f.ld_dout = N; f.zround = 1; f.dout_z = 1;
        if (gemm_nt_bf16(f, 0, v) != 0) { printf("launch refused\n"); fails++; return; }
        CK(hipDeviceSynchronize());
        auto cc = dl16(C, (size_t)M * N);
        std::vector<uint16_t> dz((size_t)M * N);
        CK(hipMemcpy(dz.data(), D, dz.size() * 2, hipMemcpyDeviceToHost));
        double wc = 0, wz = 0;
        for (int s = 0; s < 128; ++s) {
            const int r = (int)((int64_t)s * 7919 % M);
            for (int n = 0; n < N; ++n) {
                double acc = 0;
                for (int k = 0; k < K; ++k) acc += (double)A.at(r, k) * B.at(n, k);
                const float zf = (float)(_Float16)(float)acc;
                const float got = (float)__builtin_bit_cast(_Float16, dz[(size_t)r * N + n]);
                wz = std::max(wz, std::fabs((double)zf - got) / std::max(1.0, std::fabs(acc)));
                wc = std::max(wc, std::fabs(std::sin((double)got) - cc[(size_t)r * N + n]));
            }
        }
        const bool okf = wz < 2e-3 && wc < 8e-3;
        if (!okf) fails++;
        printf("nt%d zround  M=%d max|err| Z %.2e  sin(Z) %.2e  %s\n", v, M, wz, wc, okf ? "ok" : "FAIL");
    }
    CK(hipFree(C)); CK(hipFree(D));
    // TN with B = Z (b_sin)
    const int P = M;
    HMat Ad(P, N, 1.f, 14);
    ZMat Zb(P, K, 3.f, 15);
    for (int tv : {1, 2}) {
        g_tn16_variant = tv;
        const int sp = tn_splits_bf16(P, N, K);
        float *slab, *slab_b, *dW;
        CK(hipMalloc(&slab, (size_t)sp * N * K * 4));
        CK(hipMalloc(&slab_b, (size_t)sp * N * 4));
        CK(hipMalloc(&dW, (size_t)N * K * 4));
        TN16Args t;
        t.A = Ad.d; t.lda = N; t.B = Zb.d; t.ldb = K; t.K1 = K; t.b_sin = 1;
        t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K; t.slab_b = slab_b; t.P = P; t.N = N; t.K = K;
        ReduceArgs r;
        r.slab = slab; r.ld_slab = K; r.slab_stride = t.slab_stride; r.splits = sp; r.N = N; r.slab_b = slab_b;
        r.row0 = 0; r.nrows = N; r.ncols = K; r.dst = dW; r.ld_dst = K; r.dst_b = nullptr;
        if (gemm_tn_bf16(t, sp, 0) != 0 || reduce_slabs(r, 0) != 0) { printf("launch refused\n"); fails++; return; }
        CK(hipDeviceSynchronize());
        std::vector<float> w((size_t)N * K);
        CK(hipMemcpy(w.data(), dW, w.size() * 4, hipMemcpyDeviceToHost));
        double worst = 0, scale = std::sqrt((double)P);
        for (int s = 0; s < 512; ++s) {
            const int n = (int)((int64_t)s * 131 % N), k = (int)((int64_t)s * 977 % K);
            double acc = 0;
            for (int p = 0; p < P; ++p) acc += (double)Ad.at(p, n) * bfr(std::sin(Zb.at(p, k)));
            worst = std::max(worst, std::fabs(acc - w[(size_t)n * K + k]) / scale);
        }
        const bool ok = worst < 2e-3;  // bf16(sin) on the device's v_sin vs libm: ulp-level differences
        if (!ok) fails++;
        printf("tn%d b_sin  P=%d max|err|/sqrt(P) %.2e  %s\n", tv, P, worst, ok ? "ok" : "FAIL");
        CK(hipFree(slab)); CK(hipFree(slab_b)); CK(hipFree(dW));
    }
    g_tn16_variant = 2;
}

// dW[n][k] = Σ_p A[p][n] B[p][k], B = [B1 | B2] split at K1; bias[n] = Σ_p A[p][n]
static void check_tn(int P, int N, int K, int K1, bool timing) {
    HMat A(P, N, 1.f, 5), B1(P, K1, 1.f, 6), B2(P, std::max(8, K - K1), 1.f, 7);
    const int sp = tn_splits_bf16(P, N, K);
    float *slab, *slab_b, *dW, *db;
    CK(hipMalloc(&slab, (size_t)sp * N * K * 4));
    CK(hipMalloc(&slab_b, (size_t)sp * N * 4));
    CK(hipMalloc(&dW, (size_t)N * K * 4));
    CK(hipMalloc(&db, (size_t)N * 4));
    TN16Args t;
    t.A = A.d; t.lda = N; t.B = B1.d; t.ldb = K1; t.B2 = B2.d; t.ldb2 = B2.cols; t.K1 = K1;
    t.slab = slab; t.ld_slab = K; t.slab_stride = (int64_t)N * K; t.slab_b = slab_b; t.P = P; t.N = N; t.K = K;
    ReduceArgs r;
    r.slab = slab; r.ld_slab = K; r.slab_stride = t.slab_stride; r.splits = sp; r.N = N; r.slab_b = slab_b;
    r.row0 = 0; r.nrows = N; r.ncols = K; r.dst = dW; r.ld_dst = K; r.dst_b = db;
    if (gemm_tn_bf16(t, sp, 0) != 0 || reduce_slabs(r, 0) != 0) { printf("launch refused\n"); fails++; return; }
    CK(hipDeviceSynchronize());
    std::vector<float> w((size_t)N * K), b(N);
    CK(hipMemcpy(w.data(), dW, w.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), db, N * 4, hipMemcpyDeviceToHost));
    double worst = 0, worstb = 0, scale = std::sqrt((double)P);
    for (int s = 0; s < 1024; ++s) {
        const int n = (int)((int64_t)s * 131 % N), k = (int)((int64_t)s * 977 % K);
        double acc = 0;
        for (int p = 0; p < P; ++p) acc += (double)A.at(p, n) * (k < K1 ? B1.at(p, k) : B2.at(p, k - K1));
        worst = std::max(worst, std::fabs(acc - w[(size_t)n * K + k]) / scale);
    }
    for (int n = 0; n < N; ++n) {
        double acc = 0;
        for (int p = 0; p < P; ++p) acc += A.at(p, n);
        worstb = std::max(worstb, std::fabs(acc - b[n]) / scale);
    }
    const bool ok = worst < 1e-4 && worstb < 1e-4;  // fp32 accumulation of exact bf16 products
    if (!ok) fails++;
    printf("tn  P=%-7d N=%-4d K=%-4d K1=%-4d splits=%-2d max|err|/sqrt(P) W %.2e b %.2e  %s", P, N, K, K1, sp, worst,
           worstb, ok ? "ok" : "FAIL");
    if (timing) {
        const double us = time_it([&] { gemm_tn_bf16(t, sp, 0); });
        const double usr = time_it([&] { reduce_slabs(r, 0); });
        printf("   %8.1f us %7.1f TF/s (+ reduce %.1f us)", us, 2.0 * P * N * K / us * 1e-6, usr);
        t.dbg = 1;
        const double un = time_it([&] { gemm_tn_bf16(t, sp, 0); });
        t.dbg = 2;
        const double ua = time_it([&] { gemm_tn_bf16(t, sp, 0); });
        t.dbg = 4;
        const double um = time_it([&] { gemm_tn_bf16(t, sp, 0); });
        t.dbg = 0;
        printf("  [no MFMA %.1f us, DMA after %.1f, mid %.1f]", un, ua, um);
    }
    printf("\n");
    CK(hipFree(slab)); CK(hipFree(slab_b)); CK(hipFree(dW)); CK(hipFree(db));
}

int main(int argc, char** argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 131072;
    if (argc > 2) g_iters = atoi(argv[2]);
    if (argc > 3 && !strcmp(argv[3], "tn")) {  // TN tilings only: checks, then timings per variant
        const int vs = argc > 4 ? atoi(argv[4]) : 0;  // 0 = all
        for (int v = 1; v <= 3; ++v) {
            if (vs && v != vs) continue;
            g_tn16_variant = v;
            printf("tn_bf16_variant %d\n", v);
            check_tn(4100, 512, 512, 512, false);
            check_tn(4096 + 96, 512, 768, 512, false);
            check_tn(8192, 768, 512, 512, false);
            check_tn(4100, 512, 584, 520, false);  // wide + tail, the tail straddling B / B2
            check_tn(4100, 512, 800, 640, false);  // wide + tail, the tail in B2
            check_tn(P, 512, 512, 512, true);
            check_tn(P, 768, 512, 512, true);
            check_tn(P, 256, 256, 256, true);
            check_tn(P, 512, 576, 512, true);
        }
        printf("%s\n", fails ? "SOME CHECKS FAILED" : "all checks ok");
        return fails ? 1 : 0;
    }
    if (argc > 3 && !strcmp(argv[3], "epi")) {  // forward sine epilogue share: full vs no epilogue (dbg 2)
        const int shapes[][3] = {{512, 512, 0}, {768, 512, 512}, {512, 512, 512}, {256, 256, 0}};
        for (auto& sh : shapes) {
            const int N = sh[0], K = sh[1];
            HMat A(P, K, 1.f, 1), B(N, K, 0.1f, 3);
            bf16 *C, *D;
            CK(hipMalloc(&C, (size_t)P * N * 2));
            CK(hipMalloc(&D, (size_t)P * N * 2));
            std::vector<float> bias(N, 0.01f);
            float* dbias;
            CK(hipMalloc(&dbias, N * 4));
            CK(hipMemcpy(dbias, bias.data(), N * 4, hipMemcpyHostToDevice));
            NT16Args g;
            g.A = A.d; g.lda = K; g.K1 = K; g.B = B.d; g.ldb = K; g.C = C; g.ldc = N; g.M = P; g.N = N; g.K = K;
            g.bias = dbias; g.act = 1; g.w0 = 1.f; g.n_lin = sh[2]; g.Dout = D; g.ld_dout = N;
            const double full = time_it([&] { gemm_nt_bf16(g, 0, 8); });
            g.dbg = 2;
            const double noepi = time_it([&] { gemm_nt_bf16(g, 0, 8); });
            g.dbg = 0;
            g.act = 0; g.Dout = nullptr;
            const double lin = time_it([&] { gemm_nt_bf16(g, 0, 8); });
            const double gb = ((double)P * K + 2.0 * P * N) * 2 / 1e9;
            printf("nt8 P=%d N=%d K=%d n_lin=%d: full %.1f us (%.2f TB/s alg), no epilogue %.1f us, linear (C only) %.1f us\n",
                   P, N, K, sh[2], full, gb / full * 1e3, noepi, lin);
            CK(hipFree(C)); CK(hipFree(D)); CK(hipFree(dbias));
        }
        return 0;
    }
    if (argc > 3 && !strcmp(argv[3], "z")) {  // saved-Z epilogues / staging only
        check_z(4100);
        check_z(20000);
        printf("%s\n", fails ? "SOME CHECKS FAILED" : "all checks ok");
        return fails ? 1 : 0;
    }
    // edge shapes (MLP at W=64 / nomap / skip layer)
    check_nt(1000, 64, 64, 64, true, false);
    check_nt(1000, 64, 128, 64, true, false);
    check_nt(777, 96, 32, 32, false, false);
    check_nt(4100, 512, 576, 512, true, false);
    check_nt(4100, 512, 544, 512, true, false);
    check_tn(1000, 64, 64, 64, false);
    check_tn(1000, 64, 128, 64, false);
    check_tn(4100, 512, 576, 512, false);
    check_tn(2049, 96, 544, 512, false);
    check_tn(300, 32, 64, 64, false);
    // C3 shapes
    check_nt(P, 512, 512, 512, true, true);
    check_nt(P, 512, 512, 512, false, true);
    check_nt(P, 512, 576, 512, true, true);
    check_nt(P, 768, 512, 512, true, true);
    {   // timing-only ablations of the NT kernel (outputs not checked)
        HMat A(P, 512, 1.f, 1), B(512, 512, 0.1f, 3);
        bf16 *C, *D;
        CK(hipMalloc(&C, (size_t)P * 512 * 2));
        CK(hipMalloc(&D, (size_t)P * 512 * 2));
        std::vector<float> bias(512, 0.01f);
        float* dbias;
        CK(hipMalloc(&dbias, 512 * 4));
        CK(hipMemcpy(dbias, bias.data(), 512 * 4, hipMemcpyHostToDevice));
        NT16Args g;
        g.A = A.d; g.lda = 512; g.K1 = 512; g.B = B.d; g.ldb = 512; g.C = C; g.ldc = 512; g.M = P; g.N = 512; g.K = 512;
        g.bias = dbias; g.act = 1; g.Dout = D; g.ld_dout = 512;
        const char* names[] = {"128x128 persistent", "256x256 8 waves", "256x128 8 waves", "128x256 4 waves",
                               "256x256 DMA ring"};
        const int vs[] = {3, 5, 6, 7, 8};
        for (int i = 0; i < 5; ++i) {
            const double us = time_it([&] { gemm_nt_bf16(g, 0, vs[i]); });
            printf("variant %-20s %8.1f us %7.1f TF/s\n", names[i], us, 2.0 * P * 512 * 512 / us * 1e-6);
        }
        // variant 8 ablations on the backward (xDmul) shape
        HMat Dm(P, 512, 1.f, 4);
        NT16Args gd = g;
        gd.bias = nullptr; gd.act = 0; gd.Dout = nullptr; gd.Dmul = Dm.d; gd.ld_dmul = 512;
        const char* an[] = {"dmul full", "no MFMA", "no epilogue", "no MFMA+epi", "no DMA wait", "no wait+MFMA+epi",
                            "A only", "A only no MFMA+epi", "A only no epi", "A only no MFMA", "DMA after MFMAs",
                            "DMA mid MFMAs"};
        const int ad[] = {0, 1, 2, 3, 4, 7, 16, 19, 18, 17, 32, 64};
        for (int i = 0; i < 12; ++i) {
            gd.dbg = ad[i];
            const double us = time_it([&] { gemm_nt_bf16(gd, 0, 8); });
            printf("nt8 ablation %-18s %8.1f us\n", an[i], us);
        }
#ifdef ND_STAMPS
        {   // phase shares of one block's waves 0 and 4 (diagnostic build: read shares, not lengths)
            unsigned long long* st;
            CK(hipMalloc(&st, 8192 * 8));
            CK(hipMemset(st, 0, 8192 * 8));
            gd.dbg = 0;
            gd.stamps = st;
            gemm_nt_bf16(gd, 0, 8);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(8192);
            CK(hipMemcpy(h.data(), st, 8192 * 8, hipMemcpyDeviceToHost));
            const char* ph[] = {"top->waited", "waited->barrier", "barrier->issued", "issued->next top (compute)",
                                "loop end->epi barrier", "epi barrier", "epi->piece 0", "piece i->i+1"};
            for (int w = 0; w < 2; ++w) {
                const unsigned long long* v = h.data() + 4096 * w;
                const int n = (int)v[4095];
                double sum[9] = {0};
                for (int k = 1; k < n; ++k) {
                    const int from = (int)(v[k - 1] & 15);
                    const double dt = (double)((v[k] >> 4) - (v[k - 1] >> 4));
                    int cls = from <= 2 ? from : (from == 3 ? 3 : (from == 4 ? 4 : (from == 5 ? 5 : (from == 6 ? 6 : 7))));
                    if (from == 8 && (v[k] & 15) == 0) cls = 8;  // last piece -> next tile's loop
                    sum[cls] += dt;
                }
                double tot = 0;
                for (double x : sum) tot += x;
                printf("stamps wave %d: %d stamps, %.0f cycles\n", w * 4, n, tot);
                for (int c = 0; c < 8; ++c) printf("   %-28s %5.1f%%\n", ph[c], 100 * sum[c] / tot);
                printf("   %-28s %5.1f%%\n", "last piece->next tile", 100 * sum[8] / tot);
            }
            gd.stamps = nullptr;
            CK(hipFree(st));
        }
#endif
        CK(hipFree(C)); CK(hipFree(D));
    }
    check_tn(P, 512, 512, 512, true);
    check_tn(P, 512, 576, 512, true);
    check_tn(P, 768, 512, 512, true);
    check_tn(P, 256, 256, 256, true);
    printf("%s\n", fails ? "SOME CHECKS FAILED" : "all checks ok");
    return fails ? 1 : 0;
}
