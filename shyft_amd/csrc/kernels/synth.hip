// Deterministic synthetic forcing generator for the bench and
// the parity tests. Integer hashing (SplitMix64) plus IEEE-exact + - * / only,
// with FP contraction off, so numpy (shyft_amd/synthetic.py) reproduces every
// value bit for bit on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../include_internal/kernels.h"
#include "../include_internal/synth_hash.h"

namespace {

// the prefetch variant (a few CUs, beside a running kernel): few long-lived workgroups striding over cells and rows,
// so the side stream does not flood the workgroup dispatcher, and streaming (non-temporal) stores, so the 29 GB of
// a window do not evict the running kernel's working set from L2
__global__ __launch_bounds__(256) void synthetic_forcing_stream_kernel(double* __restrict__ forcing, size_t win_len,
                                                                       size_t row0, size_t n_rows, size_t n_cells,
                                                                       uint64_t seed, uint64_t cell_offset,
                                                                       uint64_t step0, const double* __restrict__ zc,
                                                                       const int64_t* __restrict__ ids) {
#pragma clang fp contract(off)
    for (size_t cell = blockIdx.x * (size_t)blockDim.x + threadIdx.x; cell < n_cells;
         cell += (size_t)gridDim.x * blockDim.x) {
        const double z = zc[cell];
        const uint64_t gcell = cell_offset + (ids ? (uint64_t)ids[cell] : cell);
        const uint64_t ck = synth_cell_key(seed, gcell);
        for (size_t r = 0; r < n_rows; ++r) {
            double v[5];
            synth_values_ck(ck, step0 + r, z, v);
            const size_t o = (row0 + r) * n_cells + cell;
            for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(v[k], &forcing[(size_t)k * win_len * n_cells + o]);
        }
    }
}

__global__ __launch_bounds__(256) void synthetic_forcing_kernel(double* __restrict__ forcing, size_t win_len, size_t row0,
                                                                size_t n_rows, size_t n_cells, uint64_t seed,
                                                                uint64_t cell_offset, uint64_t step0,
                                                                const double* __restrict__ zc,
                                                                const int64_t* __restrict__ ids) {
#pragma clang fp contract(off)
    const size_t cell = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (cell >= n_cells) return;
    const double z = zc[cell];
    const uint64_t gcell = cell_offset + (ids ? (uint64_t)ids[cell] : cell);
    const uint64_t ck = synth_cell_key(seed, gcell);  // once per lane, not per row
    for (size_t r = blockIdx.y; r < n_rows; r += gridDim.y) {
        const uint64_t step = step0 + r;
        double v[5];
        synth_values_ck(ck, step, z, v);
        const size_t o = (row0 + r) * n_cells + cell;
        // streaming stores: a window (17.5 GB at 1M cells x 438 steps) is far larger than L2 / MALL
        // (59.4 -> 59.2 ms per bench step, r05)
        for (int k = 0; k < 5; ++k) __builtin_nontemporal_store(v[k], &forcing[(size_t)k * win_len * n_cells + o]);
    }
}

}  // namespace

hipError_t launch_synthetic_forcing(double* forcing, size_t win_len, size_t row0, size_t n_rows, size_t n_cells,
                                    uint64_t seed, uint64_t cell_offset, uint64_t step0, const double* z,
                                    hipStream_t stream, const int64_t* ids) {
    if (n_rows == 0 || n_cells == 0) return hipSuccess;
    const unsigned gx = (unsigned)((n_cells + 255) / 256);
    unsigned gy = (unsigned)(n_rows < 64 ? n_rows : 64);
    hipLaunchKernelGGL(synthetic_forcing_kernel, dim3(gx, gy), dim3(256), 0, stream, forcing, win_len, row0, n_rows,
                       n_cells, seed, cell_offset, step0, z, ids);
    return hipGetLastError();
}

hipError_t launch_synthetic_forcing_stream(double* forcing, size_t win_len, size_t row0, size_t n_rows, size_t n_cells,
                                           uint64_t seed, uint64_t cell_offset, uint64_t step0, const double* z,
                                           int n_blocks, hipStream_t stream, const int64_t* ids) {
    if (n_rows == 0 || n_cells == 0) return hipSuccess;
    const size_t need = (n_cells + 255) / 256;
    const unsigned gx = (unsigned)(need < (size_t)n_blocks ? need : (size_t)n_blocks);
    hipLaunchKernelGGL(synthetic_forcing_stream_kernel, dim3(gx), dim3(256), 0, stream, forcing, win_len, row0, n_rows,
                       n_cells, seed, cell_offset, step0, z, ids);
    return hipGetLastError();
}
