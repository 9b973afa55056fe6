// HBM rates by traffic mix on one MI355X: read-only, write-only, copy (1:1) and the training
// trunk's mix (1 byte read per 16 written), 16-B vector accesses, grid-stride over 2 GiB
// buffers — the ceiling a store-heavy kernel (the training trunk writes H and D, the dX chain
// reads D and writes dZ) can reach, against the 8 TB/s read peak the rooflines quote.
//     hipcc -O3 --offload-arch=gfx950 tools/hbm_mix.hip -o tools/hbm_mix && tools/hbm_mix
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e = (x);                                                         \
        if (e != hipSuccess) {                                                      \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));        \
            return 1;                                                               \
        }                                                                           \
    } while (0)

// rd: 16-B loads per thread-iteration, wr: 16-B stores; out[] receives a checksum so loads stay
__global__ __launch_bounds__(256) void k_mix(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n,
                                             int rd, int wr, u32x4* sink) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        u32x4 v = {(unsigned)i, 1u, 2u, 3u};
        if (rd) {
            v = src[i];
            acc += v;
        }
        if (wr) dst[i] = v;
    }
    if (rd && acc.x == 0xFFFFFFFFu && acc.y == 0x12345u) sink[0] = acc;  // never true in practice
}

// the trunk's mix: every thread writes 16 x 16 B for each 16 B it reads (writes contiguous too)
__global__ __launch_bounds__(256) void k_mix16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n_out,
                                               u32x4* sink) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_out / 16; i += stride) {
        const u32x4 v = src[i];
        acc += v;
#pragma unroll
        for (int j = 0; j < 16; ++j) dst[i + j * (n_out / 16)] = v;
    }
    if (acc.x == 0xFFFFFFFFu && acc.y == 0x12345u) sink[0] = acc;
}

int main() {
    const int64_t bytes = 2LL << 30, n = bytes / 16;
    u32x4 *a, *b, *sink;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 1, bytes));
    CHECK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int bpc : {4, 8, 16}) {
        const int grid = cus * bpc;
        struct Case { const char* name; int rd, wr; double mult; } cases[] = {
            {"read only", 1, 0, 1.0}, {"write only", 0, 1, 1.0}, {"copy 1:1", 1, 1, 2.0}};
        for (const Case& c : cases) {
            float best = 1e30f;
            for (int it = 0; it < 6; ++it) {
                CHECK(hipEventRecord(e0));
                hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, a, b, n, c.rd, c.wr, sink);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0.f;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                if (it > 0 && ms < best) best = ms;
            }
            printf("blocks/CU %2d  %-12s %7.1f us  %6.2f TB/s\n", bpc, c.name, best * 1e3, c.mult * bytes / (best * 1e-3) / 1e12);
        }
        float best = 1e30f;
        for (int it = 0; it < 6; ++it) {
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_mix16, dim3(grid), dim3(256), 0, 0, a, b, n, sink);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (it > 0 && ms < best) best = ms;
        }
        printf("blocks/CU %2d  %-12s %7.1f us  %6.2f TB/s (reads + writes)\n", bpc, "1:16 r:w", best * 1e3,
               (bytes + bytes / 16.0) / (best * 1e-3) / 1e12);
    }
    CHECK(hipFree(a));
    CHECK(hipFree(b));
    CHECK(hipFree(sink));
    return 0;
}
