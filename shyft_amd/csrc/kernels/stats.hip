// Catchment statistics kernels (gfx950): the reductions behind
// cell_statistics::sum_catchment_feature / average_catchment_feature
// (core/cell_model.h:228-333) and region_model::catchment_discharges
// (core/region_model.h:873-885).
//
// Series are [step][cell]. One workgroup reduces one step (and, for segment
// sums, one catchment): lanes stride over the selected cells in a fixed order,
// then a fixed-shape wavefront shuffle tree + LDS combine, so results are
// bitwise reproducible run to run (no float atomics).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>

#include "../include_internal/kernels.h"

namespace {

constexpr int RB = 256;  // 4 wavefronts

__device__ inline double wave_sum(double v) {
    // fixed butterfly over 64 lanes
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ inline double block_sum(double v) {
    __shared__ double part[RB / 64];
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) part[wid] = v;
    __syncthreads();
    double r = 0.0;
    if (threadIdx.x == 0) {
        r = part[0];
        for (int w = 1; w < RB / 64; ++w) r += part[w];
    }
    return r;
}

__global__ __launch_bounds__(RB) void select_sum_kernel(const double* __restrict__ series, size_t n_cells,
                                                        const int32_t* __restrict__ cells, size_t n_sel,
                                                        const double* __restrict__ w, double* __restrict__ out) {
    const size_t t = blockIdx.x;
    const double* __restrict__ row = series + t * n_cells;
    double acc = 0.0;
    if (w) {
        for (size_t k = threadIdx.x; k < n_sel; k += RB) acc += row[cells[k]] * w[k];
    } else {
        for (size_t k = threadIdx.x; k < n_sel; k += RB) acc += row[cells[k]];
    }
    const double r = block_sum(acc);
    if (threadIdx.x == 0) out[t] = r;
}

// ID: the segments' cells are the identity permutation (seg_cells[k] == k: catchments as contiguous cell ranges in
// cell order), so the index array is not read (8 instead of 12 B per cell-step). Each lane loads four of its terms
// ahead and adds them in its own order: the same sum as one term at a time, with four loads in flight.
template <bool ID, bool W>
__global__ __launch_bounds__(RB) void segment_sum_kernel(const double* __restrict__ series, size_t n_cells, size_t n_steps,
                                                         const int32_t* __restrict__ seg_cells,
                                                         const int32_t* __restrict__ seg_off, double* __restrict__ out,
                                                         const double* __restrict__ w) {
    const size_t t = blockIdx.x;
    const size_t c = blockIdx.y;
    const double* __restrict__ row = series + t * n_cells;
    const int32_t b = seg_off[c], e = seg_off[c + 1];
    double acc = 0.0;
    int32_t k = b + (int32_t)threadIdx.x;
    for (; k + 3 * RB < e; k += 4 * RB) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int32_t i = ID ? k + u * RB : seg_cells[k + u * RB];
            v[u] = W ? row[i] * w[i] : row[i];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += v[u];
    }
    for (; k < e; k += RB) {
        const int32_t i = ID ? k : seg_cells[k];
        acc += W ? row[i] * w[i] : row[i];
    }
    const double r = block_sum(acc);
    if (threadIdx.x == 0) out[c * n_steps + t] = r;
}

// region_model::is_cell_env_ts_ok (region_model.h:954-962): any NaN in the forcing of a calculated cell.
// One flag word, set with a plain store by any lane that sees a NaN (all writers store the same value).
__global__ void nan_scan_kernel(const double* __restrict__ f, size_t n_rows, size_t n_cells,
                                const uint8_t* __restrict__ active, int32_t* __restrict__ flag) {
    const size_t total = n_rows * n_cells;
    bool bad = false;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const double v = f[i];
        if (v != v && (!active || active[i % n_cells])) bad = true;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) *flag = 1;
}

// Lowest cell index whose run error code is non-zero (errors are rare: one atomic per failing lane).
__global__ void first_error_kernel(const int32_t* __restrict__ err, size_t n, int32_t* __restrict__ first) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (err[i]) atomicMin(first, (int32_t)i);
}

__global__ void fill_kernel(double* __restrict__ p, size_t n, double v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// dst[r][l] = src[r][idx[l]]: replicate cell columns into parameter-ensemble lanes
__global__ void gather_columns_kernel(double* __restrict__ dst, const double* __restrict__ src, size_t n_rows,
                                      size_t src_cols, const int32_t* __restrict__ idx, size_t n_lanes) {
    const size_t total = n_rows * n_lanes;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / n_lanes, l = i - r * n_lanes;
        dst[i] = src[r * src_cols + (size_t)idx[l]];
    }
}

}  // namespace

hipError_t launch_gather_columns(double* dst, const double* src, size_t n_rows, size_t src_cols, const int32_t* idx,
                                 size_t n_lanes, hipStream_t stream) {
    const size_t total = n_rows * n_lanes;
    if (total == 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<size_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(gather_columns_kernel, dim3(grid), dim3(256), 0, stream, dst, src, n_rows, src_cols, idx, n_lanes);
    return hipGetLastError();
}

hipError_t launch_select_sum(const double* series, size_t n_cells, size_t n_steps, const int32_t* cells, size_t n_sel,
                             const double* w, double* out, hipStream_t stream) {
    if (n_steps == 0) return hipSuccess;
    hipLaunchKernelGGL(select_sum_kernel, dim3((unsigned)n_steps), dim3(RB), 0, stream, series, n_cells, cells, n_sel, w,
                       out);
    return hipGetLastError();
}

hipError_t launch_segment_sums(const double* series, size_t n_cells, size_t n_steps, const int32_t* seg_cells,
                               const int32_t* seg_off, size_t n_seg, double* out, hipStream_t stream, const double* w) {
    if (n_steps == 0 || n_seg == 0) return hipSuccess;
    const dim3 grid((unsigned)n_steps, (unsigned)n_seg);
    if (!seg_cells) {
        if (w) hipLaunchKernelGGL((segment_sum_kernel<true, true>), grid, dim3(RB), 0, stream, series, n_cells, n_steps, seg_cells, seg_off, out, w);
        else hipLaunchKernelGGL((segment_sum_kernel<true, false>), grid, dim3(RB), 0, stream, series, n_cells, n_steps, seg_cells, seg_off, out, w);
    } else {
        if (w) hipLaunchKernelGGL((segment_sum_kernel<false, true>), grid, dim3(RB), 0, stream, series, n_cells, n_steps, seg_cells, seg_off, out, w);
        else hipLaunchKernelGGL((segment_sum_kernel<false, false>), grid, dim3(RB), 0, stream, series, n_cells, n_steps, seg_cells, seg_off, out, w);
    }
    return hipGetLastError();
}

hipError_t launch_fill(double* p, size_t n, double v, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, p, n, v);
    return hipGetLastError();
}

hipError_t launch_first_error(const int32_t* err, size_t n, int32_t* first, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(first_error_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, err, n, first);
    return hipGetLastError();
}

hipError_t launch_nan_scan(const double* f, size_t n_rows, size_t n_cells, const uint8_t* active, int32_t* flag,
                           hipStream_t stream) {
    const size_t n = n_rows * n_cells;
    if (n == 0) return hipSuccess;
    size_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(nan_scan_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, f, n_rows, n_cells, active, flag);
    return hipGetLastError();
}

// ---------------------------------------------------------------- sharded regions (shards.hip)
namespace {
// dst[rows[r]][t] = src[r][t]: a shard's partial sums into the region's row order
__global__ __launch_bounds__(256) void scatter_rows_kernel(const double* __restrict__ src, const int32_t* __restrict__ rows,
                                                           size_t n_rows, size_t n, double* __restrict__ dst) {
    const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n_rows * n) return;
    const size_t r = i / n, t = i - r * n;
    dst[size_t(rows[r]) * n + t] = src[i];
}
// out[j] = ((g[0][j] + g[1][j]) + g[2][j]) + ...: the shards' partials added in shard order (deterministic)
__global__ __launch_bounds__(256) void ordered_sum_kernel(const double* __restrict__ g, size_t S, size_t M,
                                                          double* __restrict__ out) {
    const size_t j = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (j >= M) return;
    double v = g[j];
    for (size_t k = 1; k < S; ++k) v += g[k * M + j];
    out[j] = v;
}
}  // namespace

hipError_t launch_scatter_rows(const double* src, const int32_t* rows, size_t n_rows, size_t n, double* dst,
                               hipStream_t stream) {
    const size_t m = n_rows * n;
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_rows_kernel, dim3(unsigned((m + 255) / 256)), dim3(256), 0, stream, src, rows, n_rows, n,
                       dst);
    return hipGetLastError();
}

hipError_t launch_ordered_sum(const double* g, size_t S, size_t M, double* out, hipStream_t stream) {
    if (M == 0) return hipSuccess;
    hipLaunchKernelGGL(ordered_sum_kernel, dim3(unsigned((M + 255) / 256)), dim3(256), 0, stream, g, S, M, out);
    return hipGetLastError();
}
