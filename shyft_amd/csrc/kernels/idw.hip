// Inverse-distance forcing interpolation for gfx950
// (core/inverse_distance.h:142-250 run_interpolation, models :265-472, driven by
// region_model::interpolate, core/region_model.h:397-527).
//
// Two kernels:
//  - idw_neighbours_kernel, once per (source geometry, parameters): lane = cell,
//    weights to every source, keeps the max_members best in registers (sorted
//    insertion, ties after the earlier source) -> neighbour table [K][N]:
//    source index, weight, and the time-invariant part of the transform
//    (temperature: d.z - s.z; precipitation: pow(scale, (d.z - s.z)/100)).
//  - idw_gather_kernel, per batch of steps: lane = cell, the neighbour list in
//    registers, per step a gather of K source values (the [step][source] row is
//    a few KB and stays in L1/L2), the temperature gradient from the valid
//    neighbours, and the weighted mean written straight into the forcing window.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device/special.h"
#include "../include_internal/kernels.h"

using namespace shyft_dev;

namespace {

constexpr int KMAX = IDW_KMAX;

__global__ __launch_bounds__(128) void idw_neighbours_kernel(idw_nb_args a) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n_cells) return;
    const double dx = a.dst_xyz[3 * (size_t)j], dy = a.dst_xyz[3 * (size_t)j + 1], dz = a.dst_xyz[3 * (size_t)j + 2];
    const double f = a.distance_measure_factor, zs = a.zscale;
    // min_weight = 1/distance_measure(geo_point(0), geo_point(max_distance), f, zscale)
    const double min_weight = 1.0 / dpow(a.max_distance * a.max_distance + 0.0 * 0.0 + 0.0 * 0.0 * zs * zs, f / 2.0);
    double lw[KMAX];
    int ls[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) { lw[k] = -1.0; ls[k] = -1; }
    int count = 0;
    for (int s = 0; s < a.n_sources; ++s) {
        const double sx = a.src_xyz[3 * s], sy = a.src_xyz[3 * s + 1], sz = a.src_xyz[3 * s + 2];
        // geo_point::distance_measure (geo_point.h:41-43)
        const double dm = dpow((dx - sx) * (dx - sx) + (dy - sy) * (dy - sy) + (dz - sz) * (dz - sz) * zs * zs, f / 2.0);
        const double w = smin(1.0, 1.0 / dm);
        if (!(w >= min_weight)) continue;
        ++count;
        // sorted insertion (descending weight, equal weights keep source order)
#pragma unroll
        for (int k = KMAX - 1; k >= 0; --k) {
            if (k > 0 && lw[k - 1] < w) {
                lw[k] = lw[k - 1];
                ls[k] = ls[k - 1];
            } else if (lw[k] < w) {
                lw[k] = w;
                ls[k] = s;
            }
        }
    }
    const int K = a.max_members;
    const int kept = count < K ? count : K;
    if (count <= K) {
        // all candidates kept: the reference keeps them in source order (no partial_sort)
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
#pragma unroll
            for (int k = KMAX - 1; k > 0; --k) {
                const bool swap = (ls[k - 1] > ls[k]) && ls[k] >= 0;
                const int ts = swap ? ls[k - 1] : ls[k];
                const double tw = swap ? lw[k - 1] : lw[k];
                ls[k - 1] = swap ? ls[k] : ls[k - 1];
                lw[k - 1] = swap ? lw[k] : lw[k - 1];
                ls[k] = ts;
                lw[k] = tw;
            }
        }
    }
    const size_t N = (size_t)a.n_cells;
    a.count[j] = kept;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        if (k >= K) break;
        const int s = k < kept ? ls[k] : 0;
        a.idx[k * N + j] = k < kept ? s : -1;
        a.w[k * N + j] = k < kept ? lw[k] : 0.0;
        double aux = 0.0;
        if (k < kept) {
            const double ddz = dz - a.src_xyz[3 * s + 2];
            if (a.kind == IDW_TEMPERATURE) aux = ddz;
            else if (a.kind == IDW_PRECIPITATION) aux = dpow(a.scale_factor, ddz / 100.0);
        }
        a.aux[k * N + j] = aux;
    }
}

// The lane's neighbour list (source index, weight, transform constant and the
// source z for the gradient) is loaded ONCE into registers (KT >= count, a
// compile-time bound so the arrays stay in VGPRs) and reused for every row; only
// the [row][source] values (a few KB per row, L1/L2 resident) are gathered per step.
template <int KT>
__global__ __launch_bounds__(256) void idw_gather_kernel(idw_gather_args a) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n_cells) return;
    if (a.active && !a.active[j]) return;
    const size_t N = (size_t)a.n_cells;
    const int kept = a.count[j];
    const int S = a.n_sources;
    const double slope = a.slope ? a.slope[j] : 0.9;
    const bool temp = a.kind == IDW_TEMPERATURE;
    int nidx[KT];
    double nw[KT], naux[KT], nx[KT], ny[KT], nz[KT];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        const bool in = k < kept;
        const int s = in ? a.idx[k * N + j] : 0;
        nidx[k] = s;
        nw[k] = in ? a.w[k * N + j] : 0.0;
        naux[k] = in ? a.aux[k * N + j] : 0.0;
        nz[k] = (in && temp) ? a.src_xyz[3 * s + 2] : 0.0;
        nx[k] = (in && temp && a.by_equation) ? a.src_xyz[3 * s] : 0.0;
        ny[k] = (in && temp && a.by_equation) ? a.src_xyz[3 * s + 1] : 0.0;
    }
    double* __restrict__ out = a.out;
    for (int r = 0; r < a.n_rows; ++r) {
        const double* __restrict__ row = a.src_values + (size_t)r * S;
        double v[KT];
#pragma unroll
        for (int k = 0; k < KT; ++k) v[k] = k < kept ? row[nidx[k]] : 0.0;
        double scale = 1.0;
        if (temp) {
            // temperature_gradient_scale_computer::compute over the valid neighbours in
            // neighbour order (inverse_distance.h:305-330)
            int n = 0;
            double z_mn = 0, z_mx = 0, t_mn = 0, t_mx = 0;
            double p0x = 0, p0y = 0, p0z = 0, t0 = 0;
            double A[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, b[3] = {0, 0, 0};
#pragma unroll
            for (int k = 0; k < KT; ++k) {
                if (k >= kept || !__builtin_isfinite(v[k])) continue;
                const double sz = nz[k];
                if (n == 0) {
                    z_mn = z_mx = sz;
                    t_mn = t_mx = v[k];
                } else if (sz < z_mn) {
                    z_mn = sz; t_mn = v[k];
                } else if (sz > z_mx) {
                    z_mx = sz; t_mx = v[k];
                }
                if (a.by_equation) {
                    if (n == 0) { p0x = nx[k]; p0y = ny[k]; p0z = sz; t0 = v[k]; }
                    else if (n == 1) { A[0][0] = nx[k] - p0x; A[0][1] = ny[k] - p0y; A[0][2] = sz - p0z; b[0] = v[k] - t0; }
                    else if (n == 2) { A[1][0] = nx[k] - p0x; A[1][1] = ny[k] - p0y; A[1][2] = sz - p0z; b[1] = v[k] - t0; }
                    else if (n == 3) { A[2][0] = nx[k] - p0x; A[2][1] = ny[k] - p0y; A[2][2] = sz - p0z; b[2] = v[k] - t0; }
                }
                ++n;
            }
            bool solved = false;
            if (a.by_equation && n > 3) {
                // arma::solve on the 3x3 system of the first four valid points: determinant + cofactors
                const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
                                   A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                                   A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
                if (fabs(det) > 0.0 && __builtin_isfinite(det)) {
                    const double i00 = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
                    const double i01 = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
                    const double i02 = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
                    const double i10 = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
                    const double i11 = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
                    const double i12 = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
                    const double i20 = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
                    const double i21 = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
                    const double i22 = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
                    const double x0 = i00 * b[0] + i01 * b[1] + i02 * b[2];
                    const double x1 = i10 * b[0] + i11 * b[1] + i12 * b[2];
                    const double x2 = i20 * b[0] + i21 * b[1] + i22 * b[2];
                    if (__builtin_isfinite(x0) && __builtin_isfinite(x1) && __builtin_isfinite(x2)) {
                        scale = x2;
                        solved = true;
                    }
                }
            }
            if (!solved) {
                if (n > 1) {
                    const double dzm = z_mx - z_mn;
                    scale = dzm > 50.0 ? (t_mx - t_mn) / dzm : a.default_gradient;
                } else {
                    scale = a.default_gradient;
                }
            }
        }
        double sum_weights = 0.0, sum_weight_value = 0.0;
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            if (k >= kept || !__builtin_isfinite(v[k])) continue;
            double tr;
            switch (a.kind) {
                case IDW_TEMPERATURE: tr = v[k] + scale * naux[k]; break;
                case IDW_PRECIPITATION: tr = v[k] * naux[k]; break;
                case IDW_RADIATION: tr = v[k] * slope; break;
                default: tr = v[k]; break;
            }
            sum_weight_value += nw[k] * tr;
            sum_weights += nw[k];
        }
        out[(size_t)r * N + j] = sum_weight_value / sum_weights;
    }
}

// single temperature source: copied to every calculated cell (region_model.h:470-481)
__global__ void copy_source_kernel(const double* __restrict__ v, int n_rows, int n_cells, const uint8_t* __restrict__ active,
                                   double* __restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_cells) return;
    if (active && !active[j]) return;
    for (int r = 0; r < n_rows; ++r) out[(size_t)r * n_cells + j] = v[r];
}

}  // namespace

hipError_t launch_idw_neighbours(const idw_nb_args& a, hipStream_t stream) {
    if (a.n_cells == 0) return hipSuccess;
    hipLaunchKernelGGL(idw_neighbours_kernel, dim3((a.n_cells + 127) / 128), dim3(128), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_idw_gather(const idw_gather_args& a, hipStream_t stream) {
    if (a.n_cells == 0 || a.n_rows == 0) return hipSuccess;
    const dim3 grid((a.n_cells + 255) / 256), block(256);
    // smallest register-resident list that holds max_members
    if (a.max_members <= 8) hipLaunchKernelGGL(idw_gather_kernel<8>, grid, block, 0, stream, a);
    else if (a.max_members <= 12) hipLaunchKernelGGL(idw_gather_kernel<12>, grid, block, 0, stream, a);
    else if (a.max_members <= 20) hipLaunchKernelGGL(idw_gather_kernel<20>, grid, block, 0, stream, a);
    else hipLaunchKernelGGL(idw_gather_kernel<IDW_KMAX>, grid, block, 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_copy_source(const double* v, int n_rows, int n_cells, const uint8_t* active, double* out,
                              hipStream_t stream) {
    if (n_cells == 0 || n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(copy_source_kernel, dim3((n_cells + 255) / 256), dim3(256), 0, stream, v, n_rows, n_cells, active,
                       out);
    return hipGetLastError();
}
