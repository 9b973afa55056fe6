// Batch gather of the training loop's per-ray fields (reference main.py:108-115 with
// satellite_scene.py:577-592: the DataLoader hands the trainer rays, targets, depth priors and
// labels row by row).  Here every field stays resident in HBM and one launch copies the rows of a
// sampled batch into the step's static buffers — the bench step's six gathers (rays, rgb, depth,
// depth validity, depth std, semantic label) in one kernel instead of six index kernels.
#include <algorithm>

#include "common.h"

namespace spn {

constexpr int kGatherFields = 8;

struct GatherArgs {
    const int64_t* idx = nullptr;
    int64_t n = 0;
    int nf = 0;
    const uint32_t* src[kGatherFields] = {};
    uint32_t* dst[kGatherFields] = {};
    int64_t src_rows[kGatherFields] = {};
    int words[kGatherFields] = {};  // 4-byte words per row
};

// blockIdx.y = field; a thread copies one word of one row (rows in order, words of a row
// adjacent, so a wave's loads and stores are contiguous runs of rows).  An index outside the source
// rows (torch indexing would raise; the launch cannot without a host sync) POISONS its destination
// row with all-one bits — NaN in a float field, -1 in an integer one — so a sampler or offset bug
// shows up as a non-finite loss at once instead of training on the previous batch's rows
__global__ __launch_bounds__(256) void k_gather_rows(GatherArgs g) {
    const int f = blockIdx.y;
    const int wpr = g.words[f];
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= g.n * wpr) return;
    const int64_t row = t / wpr;
    const int w = (int)(t - row * wpr);
    const int64_t r = g.idx[row];
    g.dst[f][row * wpr + w] = (r < 0 || r >= g.src_rows[f]) ? 0xFFFFFFFFu : g.src[f][r * wpr + w];
}

// one thread: the render's step advanced and snapshotted (spnerf_rng_begin)
__global__ void k_rng_begin(int64_t* state, int64_t* snap) {
    const int64_t step = state[1] + 1;
    state[1] = step;
    snap[0] = state[0];
    snap[1] = step;
}

}  // namespace spn

using namespace spn;

extern "C" int32_t spnerf_rng_begin(int64_t* state, int64_t* snap, void* stream) {
    SPN_ARG(state && snap && state != snap, "rng_begin: null or aliased state / snapshot");
    hipLaunchKernelGGL(k_rng_begin, dim3(1), dim3(1), 0, (hipStream_t)stream, state, snap);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}

extern "C" int32_t spnerf_gather_rows(const int64_t* idx, int64_t n, int32_t nfields, const void* const* src,
                                      const int64_t* src_rows, const int32_t* row_bytes, void* const* dst,
                                      void* stream) {
    SPN_ARG(n >= 0 && nfields >= 0 && nfields <= kGatherFields, "gather_rows: bad sizes (n=%lld, fields=%d)",
            (long long)n, nfields);
    if (n == 0 || nfields == 0) return SPNERF_OK;
    SPN_ARG(idx && src && src_rows && row_bytes && dst, "gather_rows: null list");
    GatherArgs g;
    g.idx = idx;
    g.n = n;
    g.nf = nfields;
    int64_t maxw = 0;
    for (int f = 0; f < nfields; ++f) {
        SPN_ARG(src[f] && dst[f] && src_rows[f] >= 0, "gather_rows: field %d: null tensor or negative rows", f);
        SPN_ARG(row_bytes[f] > 0 && row_bytes[f] % 4 == 0, "gather_rows: field %d: row bytes %d not a positive multiple of 4",
                f, row_bytes[f]);
        SPN_ARG((reinterpret_cast<uintptr_t>(src[f]) | reinterpret_cast<uintptr_t>(dst[f])) % 4 == 0,
                "gather_rows: field %d: pointers not 4-byte aligned", f);
        g.src[f] = static_cast<const uint32_t*>(src[f]);
        g.dst[f] = static_cast<uint32_t*>(dst[f]);
        g.src_rows[f] = src_rows[f];
        g.words[f] = row_bytes[f] / 4;
        maxw = std::max<int64_t>(maxw, g.words[f]);
    }
    const int64_t blocks = (n * maxw + 255) / 256;
    SPN_ARG(blocks < (1ll << 31), "gather_rows: too many rows");
    hipStream_t s = (hipStream_t)stream;
    ProfScope prof("gather_rows", s, 0.0, 0.0);
    hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)blocks, (unsigned)nfields), dim3(256), 0, s, g);
    SPN_HIP(hipGetLastError());
    return SPNERF_OK;
}
