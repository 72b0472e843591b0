// routing::uhg river aggregation on gfx950 (core/routing.h:326-387, region_model.h:909-949).
//
// The reference convolves every routed cell's avg_discharge with the cell's
// unit hydrograph and sums the results per river (local_inflow), adds the
// outputs of the upstream rivers (upstream_inflow, recursive) and convolves the
// total with the river's own UHG (output_m3s). Convolution is linear, so cells
// that share (river, UHG) are first reduced to one discharge sum per group
// (segment_sums over the group's cells: the HBM-bound pass, 8 B per cell-step),
// and only the [groups][T] sums are convolved:
//
//   route_local_kernel : local[r][t]  = sum_{g in r} sum_{j < L_g, j <= t} w_g[j] S[g][t-j]
//   route_in_kernel    : in[r][t]     = local[r][t] + sum_{u upstream of r} out[u][t]   (one network level)
//   route_out_kernel   : out[r][t]    = sum_{j < L_r, j <= t} w_r[j] in[r][t-j]         (one network level)
//
// Rivers are processed level by level (a river's level is above all of its
// upstream rivers), two launches per level. Additions follow the reference's
// order within a river (groups ascending, taps ascending, upstream rivers in
// ascending id), so results are deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../include_internal/kernels.h"

namespace {

constexpr int RT = 256;

__global__ __launch_bounds__(RT) void route_local_kernel(const routing_args a) {
    const size_t t = blockIdx.x * (size_t)RT + threadIdx.x;
    const int r = blockIdx.y;
    if (t >= (size_t)a.n_steps) return;
    double acc = 0.0;
    for (int k = a.river_group_off[r]; k < a.river_group_off[r + 1]; ++k) {
        const int g = a.river_groups[k];
        const double* __restrict__ w = a.group_w + (size_t)g * a.max_len;
        const double* __restrict__ s = a.group_sums + (size_t)g * a.n_steps;
        const int L = a.group_len[g];
        double v = 0.0;
        for (int j = 0; j < L; ++j) v += (size_t)j <= t ? w[j] * s[t - j] : 0.0;
        acc += v;
    }
    a.local[(size_t)r * a.n_steps + t] = acc;
}

__global__ __launch_bounds__(RT) void route_in_kernel(const routing_args a, int level_begin, int level_end) {
    const size_t t = blockIdx.x * (size_t)RT + threadIdx.x;
    const int r = a.level_rivers[level_begin + blockIdx.y];
    if (t >= (size_t)a.n_steps) return;
    double up = 0.0;
    for (int k = a.river_up_off[r]; k < a.river_up_off[r + 1]; ++k) up += a.output[(size_t)a.river_up[k] * a.n_steps + t];
    a.upstream[(size_t)r * a.n_steps + t] = up;
    a.inflow[(size_t)r * a.n_steps + t] = a.local[(size_t)r * a.n_steps + t] + up;
    (void)level_end;
}

__global__ __launch_bounds__(RT) void route_out_kernel(const routing_args a, int level_begin, int level_end) {
    const size_t t = blockIdx.x * (size_t)RT + threadIdx.x;
    const int r = a.level_rivers[level_begin + blockIdx.y];
    if (t >= (size_t)a.n_steps) return;
    const double* __restrict__ w = a.river_w + (size_t)r * a.max_len;
    const double* __restrict__ in = a.inflow + (size_t)r * a.n_steps;
    const int L = a.river_len[r];
    double v = 0.0;
    for (int j = 0; j < L; ++j) v += (size_t)j <= t ? w[j] * in[t - j] : 0.0;
    a.output[(size_t)r * a.n_steps + t] = v;
    (void)level_end;
}

}  // namespace

hipError_t launch_route(const routing_args& a, const int* level_off, int n_levels, hipStream_t stream) {
    if (a.n_steps == 0 || a.n_rivers == 0) return hipSuccess;
    const unsigned tb = (unsigned)((a.n_steps + RT - 1) / RT);
    hipLaunchKernelGGL(route_local_kernel, dim3(tb, (unsigned)a.n_rivers), dim3(RT), 0, stream, a);
    for (int l = 0; l < n_levels; ++l) {
        const int b = level_off[l], e = level_off[l + 1];
        if (e == b) continue;
        hipLaunchKernelGGL(route_in_kernel, dim3(tb, (unsigned)(e - b)), dim3(RT), 0, stream, a, b, e);
        hipLaunchKernelGGL(route_out_kernel, dim3(tb, (unsigned)(e - b)), dim3(RT), 0, stream, a, b, e);
    }
    return hipGetLastError();
}
