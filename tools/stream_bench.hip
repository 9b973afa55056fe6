// HBM read rate by access shape (tools only): a 256-row x 1-KB tile walked in K-slices of
// SEG bytes per row, the way a GEMM's K-loop sweeps its A operand, against whole-row sweeps.
//   make -C tools stream_bench && ./tools/stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// persistent: block b walks tiles b, b + G, ...; a tile = 256 rows x 1024 B; per K-slice every
// thread loads 16 B; a slice covers 256 rows x SEG bytes = 256 * SEG / 16 loads over 512 threads
template <int SEG>
__global__ __launch_bounds__(512) void k_stream(const char* __restrict__ src, int ntiles, u32x4* out) {
    constexpr int CPR = SEG / 16;               // 16-B chunks per row per slice
    constexpr int LPS = 256 * CPR / 512;        // loads per thread per slice
    constexpr int NS = 1024 / SEG;              // slices per tile
    const int tid = threadIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const char* base = src + (size_t)t * 256 * 1024;
        for (int s = 0; s < NS; ++s) {
            u32x4 v[LPS > 0 ? LPS : 1];
#pragma unroll
            for (int i = 0; i < LPS; ++i) {
                const int q = tid + 512 * i;
                const int row = q / CPR, c = q % CPR;
                v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)row * 1024 + s * SEG + c * 16);
            }
#pragma unroll
            for (int i = 0; i < LPS; ++i) acc ^= v[i];
        }
    }
    if (acc[0] == 0x12345678u) out[tid] = acc;
}

// the same walk landing in LDS by global_load_lds_dwordx4 (one 1-KB wave-instruction = 16 rows x
// 64 B when SEG = 64, 4 rows x 256 B, or one 1-KB row), four slices in flight per wave, no
// consumer; tiles taken modulo tmod (tmod = 8: a 2 MB footprint, L2-resident)
template <int SEG, bool BAR = false>
__global__ __launch_bounds__(512) void k_stream_dma(const char* __restrict__ src, int ntiles, int tmod, u32x4* out) {
    __shared__ __attribute__((aligned(16))) char smem[4 * 32768];
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    typedef __attribute__((address_space(1))) void* gbl_ptr_t;
    constexpr int RPI = 1024 / SEG;             // rows per wave-instruction
    constexpr int NS = 1024 / SEG;              // slices per tile
    constexpr int IPS = 256 / RPI / 8;          // instructions per wave per slice (8 waves)
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int n = 0;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const char* base = src + (size_t)(t % tmod) * 256 * 1024;
        for (int s = 0; s < NS; ++s, ++n) {
#pragma unroll
            for (int i = 0; i < IPS; ++i) {
                const int q = wid * IPS + i;
                const int row = q * RPI + lane / (SEG / 16), c = lane % (SEG / 16);
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(base + (size_t)row * 1024 + s * SEG + c * 16),
                                                 (lds_ptr_t)(smem + (n & 3) * 32768 + q * 1024), 16, 0, 0);
            }
            if (IPS == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            else if (IPS == 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
            if constexpr (BAR) __builtin_amdgcn_s_barrier();  // a GEMM K-loop's per-step block barrier
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (smem[tid * 7] == 123) out[tid] = u32x4{1u, 1u, 1u, 1u};
}

template <int SEG>
__global__ __launch_bounds__(512) void k_stream_mod(const char* __restrict__ src, int ntiles, int tmod, u32x4* out) {
    constexpr int CPR = SEG / 16;
    constexpr int LPS = 256 * CPR / 512;
    constexpr int NS = 1024 / SEG;
    const int tid = threadIdx.x;
    u32x4 acc = {0u, 0u, 0u, 0u};
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const char* base = src + (size_t)(t % tmod) * 256 * 1024;
        for (int s = 0; s < NS; ++s) {
            u32x4 v[LPS];
#pragma unroll
            for (int i = 0; i < LPS; ++i) {
                const int q = tid + 512 * i;
                const int row = q / CPR, c = q % CPR;
                v[i] = *reinterpret_cast<const u32x4*>(base + (size_t)row * 1024 + s * SEG + c * 16);
            }
#pragma unroll
            for (int i = 0; i < LPS; ++i) acc ^= v[i];
        }
    }
    if (acc[0] == 0x12345678u) out[tid] = acc;
}


// The fused trunk's weight stream without its MFMAs: every block (one per CU, 8 waves) walks
// ntl tiles x 8 layers x 32 k-steps; per k-step each wave loads its 2 KB (two 16-B loads per
// lane) of a 4 MB weight set through a TPD-deep register ring.  Layouts: 0 = each wave's stream
// contiguous (64 KB per wave per layer), 1 = k-step-major (the 8 waves' pieces of a k-step
// adjacent), 2 = k-step-major with the k order rotated per block.
template <int TPD, int LAYOUT>
__global__ __launch_bounds__(512) void k_wstream(const char* __restrict__ wts, int ntl, u32x4* out) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    u32x4 ring[TPD][2];
    u32x4 acc = {0u, 0u, 0u, 0u};
    const int rot = LAYOUT == 2 ? (blockIdx.x * 5) & 31 : 0;
    auto addr = [&](int layer, int ks) -> const u32x4* {
        ks = (ks + rot) & 31;
        const size_t blk = LAYOUT == 0 ? (size_t)w * 32 + ks : (size_t)ks * 8 + w;
        return reinterpret_cast<const u32x4*>(wts + (size_t)layer * 524288 + blk * 2048) + lane;
    };
    for (int t = 0; t < ntl; ++t)
        for (int layer = 0; layer < 8; ++layer) {
#pragma unroll
            for (int d = 0; d < TPD; ++d) {
                ring[d][0] = addr(layer, d)[0];
                ring[d][1] = addr(layer, d)[64];
            }
            for (int ks0 = 0; ks0 < 32; ks0 += TPD) {
#pragma unroll
                for (int d = 0; d < TPD; ++d) {
                    acc ^= ring[d][0] ^ ring[d][1];
                    const int kn = min(ks0 + d + TPD, 31);  // past the end: re-read (as the trunk)
                    ring[d][0] = addr(layer, kn)[0];
                    ring[d][1] = addr(layer, kn)[64];
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            __syncthreads();
        }
    if (acc[0] == 0x12345678u) out[tid] = acc;
}

int main() {
    const size_t bytes = (size_t)524288 * 1024;  // 512 MiB: 524 288 rows of 1 KB (bf16 x 512)
    char* src;
    u32x4* out;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&out, 4096 * 16));
    CK(hipMemset(src, 1, bytes));
    const int ntiles = (int)(bytes / (256 * 1024));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](auto kern, const char* name, int grid) {
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, src, ntiles, out);
        CK(hipEventRecord(a));
        const int it = 10;
        for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, 0, src, ntiles, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = 1e3 * ms / it;
        printf("%-28s grid %5d  %8.1f us  %6.2f TB/s\n", name, grid, us, bytes / us * 1e-6);
    };
    auto run2 = [&](auto kern, const char* name, int tmod) {
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, src, ntiles, tmod, out);
        CK(hipEventRecord(a));
        const int it = 10;
        for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, src, ntiles, tmod, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = 1e3 * ms / it;
        printf("%-34s %-9s %8.1f us  %6.2f TB/s  %5.1f B/clk/CU at 2.4 GHz\n", name, tmod < ntiles ? "L2" : "HBM", us,
               bytes / us * 1e-6, bytes / us * 1e-6 * 1e12 / 256 / 2.4e9);
    };
    for (int tmod : {ntiles, 8}) {
        run2(k_stream_mod<64>, "regs, 64 B of each row", tmod);
        run2(k_stream_mod<256>, "regs, 256 B of each row", tmod);
        run2(k_stream_mod<1024>, "regs, whole rows", tmod);
        run2(k_stream_dma<64>, "LDS-DMA, 16 rows x 64 B / instr", tmod);
        run2(k_stream_dma<256>, "LDS-DMA, 4 rows x 256 B / instr", tmod);
        run2(k_stream_dma<1024>, "LDS-DMA, 1 row x 1 KB / instr", tmod);
        run2(k_stream_dma<64, true>, "LDS-DMA 64 B + barrier per slice", tmod);
    }
    {
        const int ntl = 64;
        auto runw = [&](auto kern, const char* name) {
            for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, src, ntl, out);
            CK(hipEventRecord(a));
            const int it = 10;
            for (int i = 0; i < it; ++i) hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, src, ntl, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double us = 1e3 * ms / it, per_cu = (double)ntl * 8 * 524288;
            printf("%-40s %8.1f us  %5.1f B/clk/CU at 2.4 GHz\n", name, us, per_cu / (us * 1e-6) / 2.4e9);
        };
        runw(k_wstream<4, 0>, "weights TPD 4, wave-major");
        runw(k_wstream<4, 1>, "weights TPD 4, k-major");
        runw(k_wstream<4, 2>, "weights TPD 4, k-major rotated");
        runw(k_wstream<8, 0>, "weights TPD 8, wave-major");
        runw(k_wstream<8, 1>, "weights TPD 8, k-major");
        runw(k_wstream<8, 2>, "weights TPD 8, k-major rotated");
        runw(k_wstream<16, 1>, "weights TPD 16, k-major");
    }
    for (int grid : {256}) {
        run(k_stream<64>, "slices of 64 B per row", grid);
        run(k_stream<128>, "slices of 128 B per row", grid);
        run(k_stream<256>, "slices of 256 B per row", grid);
        run(k_stream<512>, "slices of 512 B per row", grid);
        run(k_stream<1024>, "whole 1-KB rows", grid);
    }
    return 0;
}
