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

// the temperature gather (without gradient_by_equation) keeps each neighbour's d.z - s.z in a register (the
// neighbour table's aux column), not the station coordinates in LDS
constexpr bool DZREG = true;
// LDS budget of the row-tile gather's source tiles (60 KB measured slower)
constexpr size_t LDS_KB = 32;

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

// Per lane (cell) the neighbour list -- source index and weight, plus the
// precipitation factor pow(scale, dz/100) -- is loaded ONCE into registers and
// reused for every row. The [row][source] values are staged through LDS a tile
// of rows at a time (loaded cooperatively, coalesced), together with the source
// coordinates, so a neighbour lookup is an LDS read instead of a scattered
// 8-byte L2 gather, and the temperature transform's d.z - s.z is formed from the
// LDS copy of s.z (the expression the neighbour kernel evaluates, so the bits are
// the same). The kernel is specialised on the model (KIND) and on
// gradient_by_equation so each variant keeps only the registers it needs
// (occupancy). The temperature gradient pass re-reads the LDS row instead of
// holding the K values in registers. When the source table is too large for the
// LDS budget the rows and coordinates are read from global memory (LDS = false).
template <int KT, int KIND, bool BYEQ, bool LDS>
__device__ inline void idw_gather_body(const idw_gather_args& a, int j, bool lane_on, double* smem, int lds_rows) {
    const size_t N = (size_t)a.n_cells;
    if (!lane_on) j = 0;  // an idle lane still joins the tile loads, computes on cell 0 and stores nothing
    const int S = a.n_sources;
    const int kept = a.count[j];
    const double slope = KIND == IDW_RADIATION ? (a.slope ? a.slope[j] : 0.9) : 0.0;
    // LDS layout: [src x | src y | src z] (temperature with gradient_by_equation, or without DZREG) then
    // the row tile; otherwise the coordinates are read from global memory where they are still needed (once per
    // lane, and by the general scan of a row with a non-finite value)
    constexpr bool COORDS = KIND == IDW_TEMPERATURE && (BYEQ || !DZREG);
    double* sxyz = smem;
    double* tile = smem + (COORDS ? 3 * S : 0);
    if (LDS && COORDS) {
        for (int i = threadIdx.x; i < S; i += blockDim.x) {
            sxyz[i] = a.src_xyz[3 * i];
            sxyz[S + i] = a.src_xyz[3 * i + 1];
            sxyz[2 * S + i] = a.src_xyz[3 * i + 2];
        }
    }
    auto src_x = [&](int s) { return LDS && COORDS ? sxyz[s] : a.src_xyz[3 * s]; };
    auto src_y = [&](int s) { return LDS && COORDS ? sxyz[S + s] : a.src_xyz[3 * s + 1]; };
    auto src_z = [&](int s) { return LDS && COORDS ? sxyz[2 * S + s] : a.src_xyz[3 * s + 2]; };
    const double dst_z = KIND == IDW_TEMPERATURE ? a.dst_xyz[3 * (size_t)j + 2] : 0.0;
    int nidx[KT];
    double nw[KT];
    // naux: precipitation pow(scale, dz/100); temperature (DZREG) d.z - s.z of each neighbour, the
    // neighbour table's aux (the same subtraction of the same coordinates), held in registers instead of the
    // per-row LDS read of s.z: K fewer LDS reads per cell-row (not with gradient_by_equation, whose instance has
    // no VGPRs left for it at 2 waves per SIMD)
    double naux[KIND == IDW_PRECIPITATION || (KIND == IDW_TEMPERATURE && DZREG && !BYEQ) ? KT : 1];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        const bool in = k < kept;
        nidx[k] = in ? a.idx[k * N + j] : 0;
        nw[k] = in ? a.w[k * N + j] : 0.0;
        if (KIND == IDW_PRECIPITATION || (KIND == IDW_TEMPERATURE && DZREG && !BYEQ)) naux[k] = in ? a.aux[k * N + j] : 0.0;
    }
    double* __restrict__ out = a.out;
    // Temperature fast path: when every source value of a row is finite (the common case) the gradient
    // scan's outcome depends only on the neighbours' fixed geometry -- which neighbour holds the lowest and
    // the highest z, and (gradient_by_equation) the 3x3 system of the first four neighbours. Both are
    // resolved once per lane here with the scan's own comparisons and expressions; a row with a non-finite
    // source takes the general scan below. Results are bit-identical either way.
    __shared__ int row_finite[64];
    int kmin = 0, kmax = 0;
    double inv[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    bool inv_ok = false;
    double dz_fast = 0.0;  // src_z(nidx[kmax]) - src_z(nidx[kmin]): the fast path's gradient denominator per lane
    if (KIND == IDW_TEMPERATURE && LDS) {
        if (COORDS) __syncthreads();  // coordinates stored
        double z_mn = 0, z_mx = 0;
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            if (k >= kept) continue;
            const double sz = src_z(nidx[k]);
            if (k == 0) { z_mn = z_mx = sz; kmin = kmax = 0; }
            else if (sz < z_mn) { z_mn = sz; kmin = k; }
            else if (sz > z_mx) { z_mx = sz; kmax = k; }
        }
        dz_fast = src_z(nidx[kmax]) - src_z(nidx[kmin]);
        if (BYEQ && kept > 3) {
            double A[3][3];
            const double p0x = src_x(nidx[0]), p0y = src_y(nidx[0]), p0z = src_z(nidx[0]);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                A[q][0] = src_x(nidx[q + 1]) - p0x; A[q][1] = src_y(nidx[q + 1]) - p0y; A[q][2] = src_z(nidx[q + 1]) - p0z;
            }
            const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
                               A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                               A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
            if (fabs(det) > 0.0 && __builtin_isfinite(det)) {
                inv_ok = true;
                inv[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
                inv[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
                inv[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
                inv[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
                inv[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
                inv[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
                inv[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
                inv[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
                inv[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
            }
        }
    }
    double sw_all = 0.0;  // the weight sum of a row whose values are all finite
#pragma unroll
    for (int k = 0; k < KT; ++k)
        if (k < kept) sw_all += nw[k];
    const int step = LDS ? lds_rows : a.n_rows;
    for (int r0 = 0; r0 < a.n_rows; r0 += step) {
        const int r1 = r0 + step < a.n_rows ? r0 + step : a.n_rows;
        if (LDS) {
            __syncthreads();  // the previous tile is consumed (and the coordinates are stored)
            if ((int)threadIdx.x < r1 - r0) row_finite[threadIdx.x] = 1;
            __syncthreads();
            const int n = (r1 - r0) * S;
            const double* __restrict__ src = a.src_values + (size_t)r0 * S;
            // all of a lane's loads are issued before the first use: the tile fill is L2-latency bound otherwise
            constexpr int U = 8;  // 16 deep measured slower (VGPRs of the 20-member variants)
            for (int i0 = threadIdx.x; i0 < n; i0 += U * blockDim.x) {
                double v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = i0 + u * blockDim.x;
                    v[u] = i < n ? src[i] : 0.0;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = i0 + u * blockDim.x;
                    if (i < n) {
                        tile[i] = v[u];
                        if (!__builtin_isfinite(v[u])) row_finite[i / S] = 0;
                    }
                }
            }
            __syncthreads();
        }
        for (int r = r0; r < r1; ++r) {
            const double* __restrict__ row = LDS ? tile + (size_t)(r - r0) * S : a.src_values + (size_t)r * S;
            double scale = 1.0;
            if (KIND == IDW_TEMPERATURE && LDS && row_finite[r - r0]) {
                bool solved = false;
                if (BYEQ && inv_ok) {
                    const double t0 = row[nidx[0]];
                    const double b0 = row[nidx[1]] - t0, b1 = row[nidx[2]] - t0, b2 = row[nidx[3]] - t0;
                    const double x0 = inv[0][0] * b0 + inv[0][1] * b1 + inv[0][2] * b2;
                    const double x1 = inv[1][0] * b0 + inv[1][1] * b1 + inv[1][2] * b2;
                    const double x2 = inv[2][0] * b0 + inv[2][1] * b1 + inv[2][2] * b2;
                    if (__builtin_isfinite(x0) && __builtin_isfinite(x1) && __builtin_isfinite(x2)) {
                        scale = x2;
                        solved = true;
                    }
                }
                if (!solved) {
                    if (kept > 1) {
                        const double dzm = dz_fast;
                        scale = dzm > 50.0 ? (row[nidx[kmax]] - row[nidx[kmin]]) / dzm : a.default_gradient;
                    } else {
                        scale = a.default_gradient;
                    }
                }
            } else if (KIND == IDW_TEMPERATURE) {
                // temperature_gradient_scale_computer over the valid neighbours in neighbour order
                // (inverse_distance.h:305-330)
                int n = 0;
                double z_mn = 0, z_mx = 0, t_mn = 0, t_mx = 0;
                double p0x = 0, p0y = 0, p0z = 0, t0 = 0;
                double A[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, b[3] = {0, 0, 0};
#pragma unroll
                for (int k = 0; k < KT; ++k) {
                    if (k >= kept) continue;
                    const double v = row[nidx[k]];
                    if (!__builtin_isfinite(v)) continue;
                    const double sz = src_z(nidx[k]);
                    if (n == 0) {
                        z_mn = z_mx = sz;
                        t_mn = t_mx = v;
                    } else if (sz < z_mn) {
                        z_mn = sz; t_mn = v;
                    } else if (sz > z_mx) {
                        z_mx = sz; t_mx = v;
                    }
                    if (BYEQ) {
                        const double sx = src_x(nidx[k]), sy = src_y(nidx[k]);
                        if (n == 0) { p0x = sx; p0y = sy; p0z = sz; t0 = v; }
                        else if (n == 1) { A[0][0] = sx - p0x; A[0][1] = sy - p0y; A[0][2] = sz - p0z; b[0] = v - t0; }
                        else if (n == 2) { A[1][0] = sx - p0x; A[1][1] = sy - p0y; A[1][2] = sz - p0z; b[1] = v - t0; }
                        else if (n == 3) { A[2][0] = sx - p0x; A[2][1] = sy - p0y; A[2][2] = sz - p0z; b[2] = v - t0; }
                    }
                    ++n;
                }
                bool solved = false;
                if (BYEQ && n > 3) {
                    // arma::solve on the 3x3 system of the first four valid points: determinant + cofactors
                    const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
                                       A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                                       A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
                    if (fabs(det) > 0.0 && __builtin_isfinite(det)) {
                        const double i20 = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
                        const double i21 = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
                        const double i22 = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
                        const double i00 = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
                        const double i01 = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
                        const double i02 = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
                        const double i10 = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
                        const double i11 = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
                        const double i12 = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
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
            // second pass over the row: hide the pointer from the optimiser so the K values of the gradient
            // pass are re-read from LDS rather than kept live in VGPRs (occupancy)
            const double* rowp = row;
            if (KIND == IDW_TEMPERATURE && LDS) asm volatile("" : "+v"(rowp));
            if (LDS && row_finite[r - r0]) {
                // every value finite: no neighbour is skipped, so the weight sum is the per-lane constant
                // (same additions in the same order) and only the weighted values are accumulated
#pragma unroll
                for (int k = 0; k < KT; ++k) {
                    if (k >= kept) continue;
                    const double v = rowp[nidx[k]];
                    double tr;
                    if (KIND == IDW_TEMPERATURE) tr = v + scale * (DZREG && !BYEQ ? naux[k] : dst_z - src_z(nidx[k]));
                    else if (KIND == IDW_PRECIPITATION) tr = v * naux[k];
                    else if (KIND == IDW_RADIATION) tr = v * slope;
                    else tr = v;
                    sum_weight_value += nw[k] * tr;
                }
                if (lane_on) out[(size_t)r * N + j] = sum_weight_value / sw_all;
                continue;
            }
#pragma unroll
            for (int k = 0; k < KT; ++k) {
                if (k >= kept) continue;
                const double v = rowp[nidx[k]];
                if (!__builtin_isfinite(v)) continue;
                double tr;
                if (KIND == IDW_TEMPERATURE) tr = v + scale * (DZREG && !BYEQ ? naux[k] : dst_z - src_z(nidx[k]));
                else if (KIND == IDW_PRECIPITATION) tr = v * naux[k];
                else if (KIND == IDW_RADIATION) tr = v * slope;
                else tr = v;
                sum_weight_value += nw[k] * tr;
                sum_weights += nw[k];
            }
            if (lane_on) out[(size_t)r * N + j] = sum_weight_value / sum_weights;
        }
    }
}

template <int KT, int KIND, bool BYEQ>
__global__ __launch_bounds__(256) void idw_gather_kernel(idw_gather_args a, int lds_rows) {
    extern __shared__ double smem[];
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const bool lane_on = j < a.n_cells && !(a.active && !a.active[j]);
    if (lds_rows > 0) {
        // every lane of the workgroup takes part in the tile loads and barriers
        idw_gather_body<KT, KIND, BYEQ, true>(a, j, lane_on, smem, lds_rows);
    } else if (lane_on) {
        idw_gather_body<KT, KIND, BYEQ, false>(a, j, true, smem, 0);
    }
}


// ------------------------------------------------------------------ wavefront-union gathers
// A wavefront's 64 cells are neighbours on the ground, so their neighbour lists draw on a few dozen stations. The
// union kernel lists those stations once per wavefront (<= 64) and stores each neighbour as its position in that
// list (one byte). The gather then has lane u fetch station u's value of a row (one gathered load from L2 per lane
// and row, prefetched several rows ahead) into a 64-entry LDS slot of its wavefront, and every neighbour read is an
// LDS read of that slot: a few dozen distinct addresses in 128 consecutive dwords, where the row tile spread them
// over every source's 8 bytes (bank conflicts bound the tile kernel). No workgroup barriers: the wavefronts are
// independent. Values, weights and the order of every sum are the tile kernel's, so the results are the same bits.
__global__ __launch_bounds__(64) void idw_wave_union_kernel(idw_union_args a) {
    const int N = a.n_cells;
    const int lane = threadIdx.x;
    const int j = blockIdx.x * 64 + lane;
    const int kept = j < N ? a.count[j] : 0;
    int nid[IDW_KMAX];
    int loc[IDW_KMAX];
#pragma unroll
    for (int k = 0; k < IDW_KMAX; ++k) {
        nid[k] = k < kept ? a.idx[(size_t)k * N + j] : -1;
        loc[k] = 255;
    }
    int cnt = 0, mine = 0;
    bool over = false;
    for (;;) {
        int cand = -1;
#pragma unroll
        for (int k = IDW_KMAX - 1; k >= 0; --k)
            if (nid[k] >= 0 && loc[k] == 255) cand = nid[k];
        const unsigned long long b = __ballot(cand >= 0);
        if (b == 0ull) break;
        if (cnt == 64) {
            over = true;
            break;
        }
        const int s = __shfl(cand, __ffsll((long long)b) - 1, 64);
#pragma unroll
        for (int k = 0; k < IDW_KMAX; ++k)
            if (nid[k] == s) loc[k] = cnt;
        if (lane == cnt) mine = s;
        ++cnt;
    }
    a.wu[(size_t)blockIdx.x * 64 + lane] = (!over && lane < cnt) ? mine : 0;
    if (lane == 0) {
        a.wn[blockIdx.x] = over ? -1 : cnt;
        if (over) atomicMax(a.overflow, 1);
    }
    if (j < N) {
        const int nq = (a.max_members + 3) / 4;
#pragma unroll
        for (int q = 0; q < IDW_KMAX / 4; ++q)
            if (q < nq)
                a.lidx[(size_t)q * N + j] = (uint32_t)loc[4 * q] | ((uint32_t)loc[4 * q + 1] << 8) |
                                            ((uint32_t)loc[4 * q + 2] << 16) | ((uint32_t)loc[4 * q + 3] << 24);
    }
}

template <int KT, int KIND, bool BYEQ>
__global__ __launch_bounds__(256) void idw_wave_gather_kernel(idw_gather_args a) {
    constexpr int P = 4;  // source rows in flight per lane
    constexpr bool TEMP = KIND == IDW_TEMPERATURE;
    // row pairs through one neighbour pass for the temperature gather (5.33 -> 5.25 ms per 730-row chunk, 1M
    // cells, vs 6.20 single-row); the 20-member precipitation pass measured slower with pairs (more VGPRs, 3 -> 2
    // waves per SIMD), so it keeps single rows
    constexpr bool PAIR = TEMP;
    __shared__ double vslot[4][4][64];                 // each wavefront's union values of a row pair (double-buffered)
    __shared__ double zslot[TEMP ? 4 : 1][64];         // the union's z
    __shared__ double xslot[BYEQ ? 4 : 1][64], yslot[BYEQ ? 4 : 1][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int wave = j >> 6;
    const int NC = a.n_cells;
    if (wave * 64 >= NC) return;  // a whole wavefront past the cells (wave-uniform; no barriers below)
    const size_t N = (size_t)NC;
    const bool in_range = j < NC;
    const bool lane_on = in_range && !(a.active && !a.active[j]);
    const int S = a.n_sources;
    const int un = a.wn[wave];
    const int su = lane < un ? a.wu[(size_t)wave * 64 + lane] : 0;
    if (TEMP) zslot[wv][lane] = a.src_xyz[3 * (size_t)su + 2];
    if (BYEQ) {
        xslot[BYEQ ? wv : 0][lane] = a.src_xyz[3 * (size_t)su];
        yslot[BYEQ ? wv : 0][lane] = a.src_xyz[3 * (size_t)su + 1];
    }
    const int kept = in_range ? a.count[j] : 0;
    const double slope = KIND == IDW_RADIATION ? (in_range ? (a.slope ? a.slope[j] : 0.9) : 0.0) : 0.0;
    const double dst_z = TEMP && in_range ? a.dst_xyz[3 * (size_t)j + 2] : 0.0;
    uint32_t lw[(KT + 3) / 4];
#pragma unroll
    for (int q = 0; q < (KT + 3) / 4; ++q) lw[q] = 4 * q < kept ? a.lidx[(size_t)q * N + j] : 0u;
    auto L = [&](int k) { return (int)((lw[k >> 2] >> (8 * (k & 3))) & 0xffu); };
    double nw[KT];
    double naux[KIND == IDW_PRECIPITATION || (TEMP && DZREG && !BYEQ) ? KT : 1];
#pragma unroll
    for (int k = 0; k < KT; ++k) {
        const bool in = k < kept;
        nw[k] = in ? a.w[k * N + j] : 0.0;
        if (KIND == IDW_PRECIPITATION || (TEMP && DZREG && !BYEQ)) naux[k] = in ? a.aux[k * N + j] : 0.0;
    }
    const double* zs = zslot[TEMP ? wv : 0];
    const double* xs = xslot[BYEQ ? wv : 0];
    const double* ys = yslot[BYEQ ? wv : 0];
    __builtin_amdgcn_wave_barrier();
    // the gradient's fixed geometry (idw_gather_body's fast path, from the union's coordinates)
    int kmin = 0, kmax = 0;
    double inv[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    bool inv_ok = false;
    double dz_fast = 0.0;
    if (TEMP) {
        double z_mn = 0, z_mx = 0;
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            if (k >= kept) continue;
            const double sz = zs[L(k)];
            if (k == 0) { z_mn = z_mx = sz; kmin = kmax = 0; }
            else if (sz < z_mn) { z_mn = sz; kmin = k; }
            else if (sz > z_mx) { z_mx = sz; kmax = k; }
        }
        if (kept > 0) dz_fast = zs[L(kmax)] - zs[L(kmin)];
        if (BYEQ && kept > 3) {
            double A[3][3];
            const double p0x = xs[L(0)], p0y = ys[L(0)], p0z = zs[L(0)];
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                A[q][0] = xs[L(q + 1)] - p0x; A[q][1] = ys[L(q + 1)] - p0y; A[q][2] = zs[L(q + 1)] - p0z;
            }
            const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
                               A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                               A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
            if (fabs(det) > 0.0 && __builtin_isfinite(det)) {
                inv_ok = true;
                inv[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
                inv[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
                inv[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
                inv[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
                inv[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
                inv[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
                inv[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
                inv[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
                inv[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
            }
        }
    }
    double sw_all = 0.0;
#pragma unroll
    for (int k = 0; k < KT; ++k)
        if (k < kept) sw_all += nw[k];
    // every cell of the wavefront has KT neighbours (lanes past the cells read slot 0 with weight 0, unused)
    const bool full = __ballot(in_range && kept != KT) == 0ull;
    const double* __restrict__ src = a.src_values;
    const int R = a.n_rows;
    double pv[P];
#pragma unroll
    for (int p = 0; p < P; ++p) pv[p] = (lane < un && p < R) ? src[(size_t)p * S + su] : 0.0;
    double* __restrict__ out = a.out;
    // the gradient of one row (temperature_gradient_scale_computer, inverse_distance.h:305-330) from its LDS slot
    auto row_scale = [&](const double* row, bool fin) -> double {
        double scale = 1.0;
        if (TEMP && fin) {
            bool solved = false;
            if (BYEQ && inv_ok) {
                const double t0 = row[L(0)];
                const double b0 = row[L(1)] - t0, b1 = row[L(2)] - t0, b2 = row[L(3)] - t0;
                const double x0 = inv[0][0] * b0 + inv[0][1] * b1 + inv[0][2] * b2;
                const double x1 = inv[1][0] * b0 + inv[1][1] * b1 + inv[1][2] * b2;
                const double x2 = inv[2][0] * b0 + inv[2][1] * b1 + inv[2][2] * b2;
                if (__builtin_isfinite(x0) && __builtin_isfinite(x1) && __builtin_isfinite(x2)) {
                    scale = x2;
                    solved = true;
                }
            }
            if (!solved) {
                if (kept > 1) scale = dz_fast > 50.0 ? (row[L(kmax)] - row[L(kmin)]) / dz_fast : a.default_gradient;
                else scale = a.default_gradient;
            }
        } else if (TEMP) {
            // over the valid neighbours only
            int n = 0;
            double z_mn = 0, z_mx = 0, t_mn = 0, t_mx = 0;
            double p0x = 0, p0y = 0, p0z = 0, t0 = 0;
            double A[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, b[3] = {0, 0, 0};
#pragma unroll
            for (int k = 0; k < KT; ++k) {
                if (k >= kept) continue;
                const double v = row[L(k)];
                if (!__builtin_isfinite(v)) continue;
                const double sz = zs[L(k)];
                if (n == 0) {
                    z_mn = z_mx = sz;
                    t_mn = t_mx = v;
                } else if (sz < z_mn) {
                    z_mn = sz; t_mn = v;
                } else if (sz > z_mx) {
                    z_mx = sz; t_mx = v;
                }
                if (BYEQ) {
                    const double sx = xs[L(k)], sy = ys[L(k)];
                    if (n == 0) { p0x = sx; p0y = sy; p0z = sz; t0 = v; }
                    else if (n == 1) { A[0][0] = sx - p0x; A[0][1] = sy - p0y; A[0][2] = sz - p0z; b[0] = v - t0; }
                    else if (n == 2) { A[1][0] = sx - p0x; A[1][1] = sy - p0y; A[1][2] = sz - p0z; b[1] = v - t0; }
                    else if (n == 3) { A[2][0] = sx - p0x; A[2][1] = sy - p0y; A[2][2] = sz - p0z; b[2] = v - t0; }
                }
                ++n;
            }
            bool solved = false;
            if (BYEQ && n > 3) {
                const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
                                   A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                                   A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
                if (fabs(det) > 0.0 && __builtin_isfinite(det)) {
                    const double i20 = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
                    const double i21 = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
                    const double i22 = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
                    const double i00 = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
                    const double i01 = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
                    const double i02 = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
                    const double i10 = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
                    const double i11 = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
                    const double i12 = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
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
        return scale;
    };
    // neighbour k's transformed value (inverse_distance.h:390-472)
    auto transform = [&](double v, double scale, int k, int l) -> double {
        if (TEMP) return v + scale * (DZREG && !BYEQ ? naux[k] : dst_z - zs[l]);
        if (KIND == IDW_PRECIPITATION) return v * naux[k];
        if (KIND == IDW_RADIATION) return v * slope;
        return v;
    };
    // one row by the general paths (a lane with fewer than KT neighbours, or missing source values)
    auto one_row = [&](int r, const double* row, bool fin) {
        const double scale = row_scale(row, fin);
        double sum_weights = 0.0, sum_weight_value = 0.0;
        if (fin) {
            // branch-free over the KT slots (a slot past the lane's count reads a valid LDS word and is not added):
            // the LDS reads issue back to back instead of one read-and-wait per neighbour
#pragma unroll
            for (int k = 0; k < KT; ++k) {
                const int l = L(k) & 63;
                const double acc = sum_weight_value + nw[k] * transform(row[l], scale, k, l);
                sum_weight_value = k < kept ? acc : sum_weight_value;
            }
            if (lane_on) out[(size_t)r * N + j] = sum_weight_value / sw_all;
            return;
        }
#pragma unroll
        for (int k = 0; k < KT; ++k) {
            if (k >= kept) continue;
            const double v = row[L(k)];
            if (!__builtin_isfinite(v)) continue;
            sum_weight_value += nw[k] * transform(v, scale, k, L(k));
            sum_weights += nw[k];
        }
        if (lane_on) out[(size_t)r * N + j] = sum_weight_value / sum_weights;
    };
    // Rows go in pairs: both rows' values into the wavefront's slots, then -- when every lane of the wavefront has
    // its KT neighbours and both rows are finite -- one pass over the neighbours feeds two independent sums (each
    // in the reference's order: the same bits as two single-row passes), so one neighbour-slot decode and one
    // weight register serve two rows and the two add chains overlap.
    for (int r = 0; r < R; r += 2) {
        const bool two = r + 1 < R;
        const double v0 = pv[0], v1 = pv[1];
#pragma unroll
        for (int p = 0; p + 2 < P; ++p) pv[p] = pv[p + 2];
        pv[P - 2] = (lane < un && r + P < R) ? src[(size_t)(r + P) * S + su] : 0.0;
        pv[P - 1] = (lane < un && r + P + 1 < R) ? src[(size_t)(r + P + 1) * S + su] : 0.0;
        double* row0 = vslot[wv][((r >> 1) & 1) * 2];
        double* row1 = row0 + 64;
        row0[lane] = v0;
        row1[lane] = v1;
        const bool fin0 = __ballot(lane < un && !__builtin_isfinite(v0)) == 0ull;
        const bool fin1 = !two || __ballot(lane < un && !__builtin_isfinite(v1)) == 0ull;
        __builtin_amdgcn_wave_barrier();
        if (PAIR && full && fin0 && fin1 && two) {
            const double scale0 = row_scale(row0, true), scale1 = row_scale(row1, true);
            double s0 = 0.0, s1 = 0.0;
#pragma unroll
            for (int k = 0; k < KT; ++k) {
                const int l = L(k);
                s0 += nw[k] * transform(row0[l], scale0, k, l);
                s1 += nw[k] * transform(row1[l], scale1, k, l);
            }
            if (lane_on) {
                out[(size_t)r * N + j] = s0 / sw_all;
                out[(size_t)(r + 1) * N + j] = s1 / sw_all;
            }
            continue;
        }
        if (full && fin0) {  // the single-row straight-line sum
            const double scale0 = row_scale(row0, true);
            double s0 = 0.0;
#pragma unroll
            for (int k = 0; k < KT; ++k) {
                const int l = L(k);
                s0 += nw[k] * transform(row0[l], scale0, k, l);
            }
            if (lane_on) out[(size_t)r * N + j] = s0 / sw_all;
        } else {
            one_row(r, row0, fin0);
        }
        if (two) one_row(r + 1, row1, fin1);
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
    // LDS: the source coordinates (temperature) + a tile of source rows, up to 32 KB per workgroup
    // (the kernels run at 2 waves per SIMD, 2 workgroups per CU: 60 KB each fits the 160 KB)
    constexpr size_t LDS_BUDGET = LDS_KB * 1024;
    const size_t row_bytes = (size_t)a.n_sources * sizeof(double);
    const size_t coord_bytes = a.kind == IDW_TEMPERATURE && (a.by_equation || !DZREG) ? 3 * row_bytes : 0;
    int lds_rows = row_bytes + coord_bytes <= LDS_BUDGET ? (int)((LDS_BUDGET - coord_bytes) / row_bytes) : 0;
    if (lds_rows > 64) lds_rows = 64;  // row_finite[] flags per tile
    if (lds_rows > a.n_rows) lds_rows = a.n_rows;
    const size_t shm = lds_rows > 0 ? coord_bytes + (size_t)lds_rows * row_bytes : 0;
    // smallest register-resident list that holds max_members, per model
#define IDW_LAUNCH(KIND_, BYEQ_)                                                                               \
    do {                                                                                                             \
        if (a.max_members <= 8)                                                                                      \
            hipLaunchKernelGGL((idw_gather_kernel<8, KIND_, BYEQ_>), grid, block, shm, stream, a, lds_rows);         \
        else if (a.max_members <= 12)                                                                                \
            hipLaunchKernelGGL((idw_gather_kernel<12, KIND_, BYEQ_>), grid, block, shm, stream, a, lds_rows);        \
        else if (a.max_members <= 20)                                                                                \
            hipLaunchKernelGGL((idw_gather_kernel<20, KIND_, BYEQ_>), grid, block, shm, stream, a, lds_rows);        \
        else                                                                                                         \
            hipLaunchKernelGGL((idw_gather_kernel<IDW_KMAX, KIND_, BYEQ_>), grid, block, shm, stream, a, lds_rows);  \
    } while (0)
    // gathers through the wavefront's union of neighbour stations when every wavefront's union fits 64
    if (a.wu && a.wn && a.lidx) {
        const dim3 wgrid((a.n_cells + 255) / 256);
#define IDW_WLAUNCH(KIND_, BYEQ_)                                                                              \
    do {                                                                                                             \
        if (a.max_members <= 8)                                                                                      \
            hipLaunchKernelGGL((idw_wave_gather_kernel<8, KIND_, BYEQ_>), wgrid, block, 0, stream, a);               \
        else if (a.max_members <= 12)                                                                                \
            hipLaunchKernelGGL((idw_wave_gather_kernel<12, KIND_, BYEQ_>), wgrid, block, 0, stream, a);              \
        else if (a.max_members <= 20)                                                                                \
            hipLaunchKernelGGL((idw_wave_gather_kernel<20, KIND_, BYEQ_>), wgrid, block, 0, stream, a);              \
        else                                                                                                         \
            hipLaunchKernelGGL((idw_wave_gather_kernel<IDW_KMAX, KIND_, BYEQ_>), wgrid, block, 0, stream, a);        \
    } while (0)
        switch (a.kind) {
            case IDW_TEMPERATURE:
                if (a.by_equation) IDW_WLAUNCH(IDW_TEMPERATURE, true);
                else IDW_WLAUNCH(IDW_TEMPERATURE, false);
                break;
            case IDW_PRECIPITATION: IDW_WLAUNCH(IDW_PRECIPITATION, false); break;
            case IDW_RADIATION: IDW_WLAUNCH(IDW_RADIATION, false); break;
            default: IDW_WLAUNCH(IDW_WIND_SPEED, false); break;
        }
#undef IDW_WLAUNCH
        return hipGetLastError();
    }
    switch (a.kind) {
        case IDW_TEMPERATURE:
            if (a.by_equation) IDW_LAUNCH(IDW_TEMPERATURE, true);
            else IDW_LAUNCH(IDW_TEMPERATURE, false);
            break;
        case IDW_PRECIPITATION: IDW_LAUNCH(IDW_PRECIPITATION, false); break;
        case IDW_RADIATION: IDW_LAUNCH(IDW_RADIATION, false); break;
        default: IDW_LAUNCH(IDW_WIND_SPEED, false); break;  // wind speed and rel_hum: plain mean
    }
#undef IDW_LAUNCH
    return hipGetLastError();
}

hipError_t launch_idw_wave_union(const idw_union_args& a, hipStream_t stream) {
    if (a.n_cells == 0) return hipSuccess;
    if (a.max_members < 1 || a.max_members > IDW_KMAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(idw_wave_union_kernel, dim3((a.n_cells + 63) / 64), dim3(64), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_copy_source(const double* v, int n_rows, int n_cells, const uint8_t* active, double* out,
                              hipStream_t stream) {
    if (n_cells == 0 || n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(copy_source_kernel, dim3((n_cells + 255) / 256), dim3(256), 0, stream, v, n_rows, n_cells, active,
                       out);
    return hipGetLastError();
}
