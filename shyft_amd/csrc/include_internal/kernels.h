// Kernel argument structs and launch entry points (internal to libshyft_hip.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

struct ptgsk_kargs {
    int n_cells;      // lanes (cells) in the launch
    int step0;        // first absolute step to run
    int n_steps;      // number of steps
    int win0;         // absolute step of window row 0
    int win_len;      // window rows (forcing/response stride)
    int collect;      // collect_mode
    int uniform_params;  // 1: every cell uses parameter set 0 (n_sets == 1)
    double dt_s;      // to_seconds(dt)
    double dt_us;     // dt in microseconds (as double)
    double t1_hours;  // kirchner integration end: to_seconds(dt)/3600
    const int32_t* doy;            // [T] day of year of period start
    const int64_t* t_rel_year_us;  // [T] period start - trim(start, YEAR)
    const double* params;          // [n_sets][PTGSK_NP]
    const int32_t* set_ix;         // [N]
    const double* cellc;           // [PTGSK_NC][N]
    double* state;                 // [PTGSK_NS][N]
    const double* forcing;         // [N_FORCING][win_len][f_cols]
    const int32_t* fcol;           // [N] forcing column of each lane (parameter ensembles), null = lane
    int f_cols;                    // forcing columns (== n_cells unless fcol is set)
    double* resp;                  // [n_series][win_len][N]
    double* state_series;          // [PTGSK_NS][win_len+1][N] or null
    const uint8_t* active;         // [N] catchment filter or null
    int32_t* err;                  // [N]
    // test knobs (shyft_hip_set_test_knob; 0 in production): instance 2 / 4 forces the 64-lane 2-wave or the 256-lane
    // 4-wave instance; read_delay > 0 makes every wavefront but the first sleep read_delay x s_sleep(127) after the
    // Brent phase's second barrier, before reading its lanes' results (forces the job-queue interleaving)
    int instance;
    int read_delay;
};

hipError_t launch_ptgsk_run(const ptgsk_kargs& a, hipStream_t stream);

struct hbv_kargs {
    int n_cells, step0, n_steps, win0, win_len, collect;
    double step_in_days;     // to_seconds(dt)/86400
    double dt_hours;         // to_seconds(dt)/3600
    const double* params;    // [n_sets][HBV_NP]
    const int32_t* set_ix;   // [N]
    const double* cellc;     // [HBV_NC][N]
    double* state;           // [HBV_NS][N]
    const double* forcing;   // [N_FORCING][win_len][f_cols]
    const int32_t* fcol;     // [N] forcing column of each lane, null = lane
    int f_cols;              // forcing columns
    double* resp;            // [n_series][win_len][N]
    double* state_series;    // [HBV_NS][win_len+1][N] or null
    const uint8_t* active;   // [N] or null
    int32_t* err;            // [N]
    int uniform_params;      // 1: every cell uses parameter set 0 (n_sets == 1)
    int nb_max;              // the largest snow bin count of the parameter sets
};

hipError_t launch_hbv_run(const hbv_kargs& a, hipStream_t stream);

struct ptssk_kargs {
    int n_cells, step0, n_steps, win0, win_len, collect;
    double step_in_days;     // to_seconds(dt)/86400 (skaugen.h:160)
    double dt_hours;         // to_seconds(dt)/3600 (skaugen.h:161)
    double t1_hours;         // kirchner integration end: to_seconds(dt)/to_seconds(1h)
    double dt_us;            // dt in microseconds (exact integer value)
    const double* params;    // [n_sets][PTSSK_NP]
    const int32_t* set_ix;   // [N]
    const double* cellc;     // [PTGSK_NC][N]
    double* state;           // [PTSSK_NS][N]
    const double* forcing;   // [N_FORCING][win_len][f_cols]
    const int32_t* fcol;     // [N] forcing column of each lane, null = lane
    int f_cols;              // forcing columns
    double* resp;            // [n_series][win_len][N]
    double* state_series;    // [PTSSK_NSC][win_len+1][N] or null
    const uint8_t* active;   // [N] or null
    int32_t* err;            // [N]
    int uniform_params;      // 1: every cell uses parameter set 0 (n_sets == 1)
    int nb_max;              // pt_hs_k: the largest snow bin count of the parameter sets
};

hipError_t launch_ptssk_run(const ptssk_kargs& a, hipStream_t stream);

// pt_hs_k (kernels/pthsk.hip): same arguments; params [n_sets][PTHSK_NP], state [PTHSK_NS][N],
// state_series [PTHSK_NSC][win_len+1][N]
using pthsk_kargs = ptssk_kargs;
hipError_t launch_pthsk_run(const pthsk_kargs& a, hipStream_t stream);

// pt_hps_k (kernels/pthpsk.hip): same arguments; params [n_sets][PTHPSK_NP], state [PTHPSK_NS][N],
// state_series [PTHPSK_NSC][win_len+1][N]
using pthpsk_kargs = ptssk_kargs;
hipError_t launch_pthpsk_run(const pthpsk_kargs& a, hipStream_t stream);

// routing (kernels/routing.hip): river aggregation of (river, UHG) group discharge sums
struct routing_args {
    int n_steps, n_rivers, max_len;
    const double* group_sums;       // [G][n_steps]
    const double* group_w;          // [G][max_len] UHG taps (zero padded)
    const int32_t* group_len;       // [G]
    const int32_t* river_group_off; // [R+1] CSR of the groups of each river (ascending group index)
    const int32_t* river_groups;
    const double* river_w;          // [R][max_len]
    const int32_t* river_len;       // [R]
    const int32_t* river_up_off;    // [R+1] CSR of upstream rivers (ascending river id)
    const int32_t* river_up;
    const int32_t* level_rivers;    // rivers ordered by network level (upstream levels first)
    double* local;                  // [R][n_steps] local_inflow
    double* upstream;               // [R][n_steps] upstream_inflow
    double* inflow;                 // [R][n_steps] local + upstream (scratch)
    double* output;                 // [R][n_steps] output_m3s
};
hipError_t launch_route(const routing_args& a, const int* level_off, int n_levels, hipStream_t stream);

// synthetic workload generator, fills [5][n][N] window rows; cell i is generator cell
// cell_offset + (ids ? ids[i] : i) (ids: a z-balanced shard's region cells, shards.hip)
// few-workgroup, non-temporal-store variant for generating beside a running kernel (n_blocks workgroups)
hipError_t launch_synthetic_forcing_stream(double* forcing, size_t win_len, size_t row0, size_t n_rows, size_t n_cells,
                                           uint64_t seed, uint64_t cell_offset, uint64_t step0, const double* z,
                                           int n_blocks, hipStream_t stream, const int64_t* ids = nullptr);
hipError_t launch_synthetic_forcing(double* forcing, size_t win_len, size_t row0, size_t n_rows, size_t n_cells,
                                    uint64_t seed, uint64_t cell_offset, uint64_t step0, const double* z,
                                    hipStream_t stream, const int64_t* ids = nullptr);

// sums over selected cells: out[t] = sum_k w[k]*series[t][cells[k]] for t in [0,n)
// (w == null -> plain sum), deterministic fixed-order tree per step
hipError_t launch_select_sum(const double* series, size_t n_cells, size_t n_steps, const int32_t* cells, size_t n_sel,
                             const double* w, double* out, hipStream_t stream);

// per-catchment sums: out[c][t] = sum over cells of segment c (seg_cells[seg_off[c]..seg_off[c+1]))
// (w != null: sum of series * w[cell], the area-weighted sums of model_calibration.h:765-776; seg_cells == null: the
// identity, seg_cells[k] == k)
hipError_t launch_segment_sums(const double* series, size_t n_cells, size_t n_steps, const int32_t* seg_cells,
                               const int32_t* seg_off, size_t n_seg, double* out, hipStream_t stream,
                               const double* w = nullptr);
// sharded regions: a shard's [n_rows][n] partials into rows[r] of the region's [R][n]; S partials [S][M] added in
// shard order
hipError_t launch_scatter_rows(const double* src, const int32_t* rows, size_t n_rows, size_t n, double* dst,
                               hipStream_t stream);
hipError_t launch_ordered_sum(const double* g, size_t S, size_t M, double* out, hipStream_t stream);

// dst[r][l] = src[r][idx[l]] for r < n_rows, l < n_lanes (parameter-ensemble lane replication)
hipError_t launch_gather_columns(double* dst, const double* src, size_t n_rows, size_t src_cols, const int32_t* idx,
                                 size_t n_lanes, hipStream_t stream);

// flag = 1 if any of rows x cells (restricted to active cells when active != null) is NaN
// first[0] = min(first[0], lowest i with err[i] != 0); caller initialises first[0] to a value >= n
hipError_t launch_first_error(const int32_t* err, size_t n, int32_t* first, hipStream_t stream);
hipError_t launch_nan_scan(const double* f, size_t n_rows, size_t n_cells, const uint8_t* active, int32_t* flag,
                           hipStream_t stream);

// fill with a constant
hipError_t launch_fill(double* p, size_t n, double v, hipStream_t stream);

// inverse-distance interpolation (kernels/idw.hip)
#define IDW_KMAX 32
enum idw_kind { IDW_TEMPERATURE = 0, IDW_PRECIPITATION = 1, IDW_RADIATION = 2, IDW_WIND_SPEED = 3, IDW_REL_HUM = 4 };

struct idw_nb_args {
    int n_cells, n_sources, kind, max_members;
    double max_distance, distance_measure_factor, zscale, scale_factor;
    const double* src_xyz;  // [S][3]
    const double* dst_xyz;  // [N][3]
    int32_t* idx;           // [K][N] source index, -1 beyond count
    double* w;              // [K][N] weight
    double* aux;            // [K][N] temperature: d.z - s.z; precipitation: pow(scale, (d.z - s.z)/100)
    int32_t* count;         // [N]
};

struct idw_gather_args {
    int n_cells, n_sources, n_rows, kind, by_equation, max_members;
    double default_gradient;
    const double* src_xyz;     // [S][3]
    const double* src_values;  // [n_rows][S]
    const double* dst_xyz;     // [N][3] cell mid points (temperature: d.z - s.z)
    const double* slope;       // [N] radiation slope factor (geo_cell_data)
    const int32_t* idx;
    const double* w;
    const double* aux;
    const int32_t* count;
    const uint8_t* active;     // catchment calculation filter or null
    double* out;               // [n_rows][N] (a forcing window slice)
    // wave-union tables (idw_wave_union): when set, the gather reads each neighbour through its wavefront's
    // compacted station list instead of a row tile of every source
    const int32_t* wu;         // [ceil(N/64)][64] stations of the wavefront's union (lanes >= union size: 0)
    const int32_t* wn;         // [ceil(N/64)] union size
    const uint32_t* lidx;      // [ceil(K/4)][N] the neighbours' positions in the union, 4 bytes per word
};

// per wavefront of 64 cells: the union of their neighbour lists (<= 64 stations) and every neighbour's position in
// it; *overflow = 1 if some wavefront needs more than 64 stations (the gather then keeps the row-tile path)
struct idw_union_args {
    int n_cells, max_members;
    const int32_t* idx;
    const int32_t* count;
    int32_t* wu;
    int32_t* wn;
    uint32_t* lidx;
    int32_t* overflow;
};
hipError_t launch_idw_wave_union(const idw_union_args& a, hipStream_t stream);

hipError_t launch_idw_neighbours(const idw_nb_args& a, hipStream_t stream);
hipError_t launch_idw_gather(const idw_gather_args& a, hipStream_t stream);
hipError_t launch_copy_source(const double* v, int n_rows, int n_cells, const uint8_t* active, double* out,
                              hipStream_t stream);

// Bayesian temperature kriging engine (kernels/btk.hip, core/bayesian_kriging.h:280-402). Host inputs are
// read synchronously; the result is complete on `stream` when btk_run returns. Throws std::runtime_error
// with the reference's messages.
struct btk_cache;  // full-set operators + device A of the last call (kernels/btk.hip)
btk_cache* btk_cache_create();
void btk_cache_destroy(btk_cache* c);

struct btk_args {
    btk_cache* cache;              // or null (no reuse)
    uint64_t dst_version;          // identifies the destination set for the cache; 0 = never reuse
    size_t n_sources;
    const double* src_xyz;         // host [S][3]
    const double* src_values;      // host [n_steps][S], NaN = missing
    size_t n_steps;
    const double* prior_gradient;  // host [n_steps]: parameter.temperature_gradient(period) per step
    double gradient_sd, sill, nug, range, zscale;  // gradient_sd already /100 (bayesian_kriging.h:213-217)
    size_t n_dst;
    const double* d_dst_xyz;       // device [D][3]
    const int32_t* d_dst_index;    // device [D] output column of each destination, or null (= d)
    double* d_out;                 // device: step j, destination d -> d_out[j * ld_out + column]
    size_t ld_out;
};
void btk_run(const btk_args& a, hipStream_t stream);
