/* shyft_hip.h — C ABI of the MI355X (gfx950) region engine.
 *
 * This is the drop-in boundary for Shyft's distributed-cell hot path:
 * region_model::run_interpolation / run_cells (core/region_model.h:546-597)
 * and the catchment statistics that consume run_cells' output
 * (core/cell_model.h:228-368, api/api.h:289-318). The C++ host class that
 * keeps the reference's region_model<cell_t> API (shyft_amd/csrc/host/) and
 * the Python surface (shyft_amd.api) call nothing but these functions.
 *
 * Conventions
 *  - Every function returns 0 on success, non-zero on error; the message is
 *    available from shyft_hip_last_error(h) (or shyft_hip_last_error(NULL) for
 *    errors raised before a handle exists). This replaces the std::runtime_error
 *    the reference throws (region_model.h:583-592, cell_model.h:198-211).
 *  - Cells are indexed 0..n_cells-1 in the caller's order. Host arrays are
 *    borrowed for the duration of the call; device memory is owned by the handle.
 *  - Time is int64 microseconds since 1970-01-01Z, as the reference's utctime
 *    (core/utctime_utilities.h:29-34). The time axis is fixed_dt
 *    (core/time_axis.h:74-115).
 *  - Arrays marked [A][B] are row-major: element (a, b) at a*B + b.
 */
#ifndef SHYFT_HIP_H
#define SHYFT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shyft_hip_region shyft_hip_region;

/* method stacks (core/pt_gs_k.h, core/hbv_stack.h, core/pt_ss_k.h, core/pt_hs_k.h, core/pt_hps_k.h) */
enum shyft_hip_stack {
    SHYFT_HIP_PT_GS_K = 1, SHYFT_HIP_HBV_STACK = 2, SHYFT_HIP_PT_SS_K = 3, SHYFT_HIP_PT_HS_K = 4, SHYFT_HIP_PT_HPS_K = 5
};

/* forcing variables, the cell env_ts of core/cell_model.h:47-81 */
enum shyft_hip_forcing {
    SHYFT_HIP_TEMPERATURE = 0, SHYFT_HIP_PRECIPITATION = 1, SHYFT_HIP_WIND_SPEED = 2,
    SHYFT_HIP_REL_HUM = 3, SHYFT_HIP_RADIATION = 4
};

/* response collection (core/pt_gs_k_cell_model.h:41-150):
 *  DISCHARGE      = discharge_collector (avg_discharge, charge_m3s)
 *  DISCHARGE_SNOW = discharge_collector with collect_snow (+ snow_sca, snow_swe)
 *  ALL            = all_response_collector (8 series) */
enum shyft_hip_collect { SHYFT_HIP_COLLECT_DISCHARGE = 0, SHYFT_HIP_COLLECT_DISCHARGE_SNOW = 1, SHYFT_HIP_COLLECT_ALL = 2 };

/* pt_gs_k response series ids (all_response_collector member order) */
enum shyft_hip_ptgsk_series {
    SHYFT_HIP_AVG_DISCHARGE = 0, SHYFT_HIP_CHARGE_M3S = 1, SHYFT_HIP_SNOW_SCA = 2, SHYFT_HIP_SNOW_SWE = 3,
    SHYFT_HIP_SNOW_OUTFLOW = 4, SHYFT_HIP_GLACIER_MELT = 5, SHYFT_HIP_AE_OUTPUT = 6, SHYFT_HIP_PE_OUTPUT = 7
};

/* series ids accepted by the statistics / cell-series entry points besides the response ids above:
 * the cell environment (forcing) variable v as SHYFT_HIP_SERIES_FORCING + v, and state-collector
 * field f (T+1 instant axis) as SHYFT_HIP_SERIES_STATE + f. */
enum shyft_hip_series_base { SHYFT_HIP_SERIES_FORCING = 100, SHYFT_HIP_SERIES_STATE = 200 };

/* statistics scope (core/cell_model.h:183-186 stat_scope) */
enum shyft_hip_stat_scope { SHYFT_HIP_SCOPE_CELL_IX = 0, SHYFT_HIP_SCOPE_CATCHMENT = 1 };

const char* shyft_hip_last_error(const shyft_hip_region* h);

/* Replaces region_model(const vector<geo_cell_data>&, const parameter_t&) — core/region_model.h:285-293.
 * device < 0 selects the current HIP device. */
int shyft_hip_region_create(int stack, size_t n_cells, int device, shyft_hip_region** out);
void shyft_hip_region_destroy(shyft_hip_region* h);
/* One region whose cells are split into n_shards contiguous shards, shard k (cells [n*k/S, n*(k+1)/S)) on device
 * devices[k] -- devices may repeat (several shards on one device). Every entry point below works on the whole
 * region as on an unsharded one (cell indexes, catchment ids and series are the region's); the shards run
 * concurrently, one host thread per shard. This is region_model over all of a node's GPUs from one process
 * (core/region_model.h:972-1021 runs the whole region in one process). Catchment / routing-group / ensemble sums
 * add per-shard partial sums in shard order after an all-gather: RCCL (ncclAllGather over xGMI) when every shard
 * has its own device, device-to-device copies when shards share one; a catchment whose cells lie in one shard sums
 * exactly as on the unsharded region. Forcing and series move between host memory and the shards (no device
 * pointers: each shard's memory is on its own device). */
int shyft_hip_region_create_sharded(int stack, size_t n_cells, const int* devices, size_t n_shards,
                                    shyft_hip_region** out);
/* create_sharded with options. The combine path is chosen once, at creation: RCCL when every shard has its own
 * device (or with SHYFT_HIP_SHARD_RCCL_ALWAYS: also one shard, a one-rank communicator), then a self-check before any
 * data uses it -- an all-gather of known partials must arrive bit for bit on every device and their shard-order sum
 * must equal the device-copy path's bitwise. A failed communicator initialisation, a failed self-check, or an RCCL error
 * at run time switches the region to device copies (same results; shyft_hip_region_combine_report says why). Every
 * RCCL step has a deadline (SHYFT_HIP_RCCL_DEADLINE_MS, default 120 s; non-blocking communicators, polled): one that
 * stalls is aborted (ncclCommAbort) and handled like one that fails. No reference
 * counterpart: the reference's one-process region has no exchange (core/region_model.h:972-1021).
 * SHYFT_HIP_SHARD_NO_RCCL: device copies only. The TEST_ flags inject the failures for the fallback tests:
 * ncclCommInitAll failing, the first all-gather after the self-check failing, the self-check comparing unequal, the
 * self-check's all-gather not seen to complete before the deadline (TEST_STALL_CHECK).
 * SHYFT_HIP_SHARD_BALANCE_Z: instead of contiguous cell ranges, the first shyft_hip_set_geo ranks the cells by
 * elevation and deals rank r to shard r % n_shards (each shard keeps its cells in region order), so every shard holds
 * the same mix of elevations and so of snow-season work. Every entry point still takes the region's cell indexes;
 * results per cell are unchanged, catchment sums are partial sums added in shard order (each catchment now spans the
 * shards, so they are reassociated), and shyft_hip_region_shards reports shard k's cell count (cell0 is then only its
 * position in the deal). */
enum shyft_hip_shard_flags {
    SHYFT_HIP_SHARD_RCCL_ALWAYS = 1, SHYFT_HIP_SHARD_NO_RCCL = 2, SHYFT_HIP_SHARD_TEST_FAIL_INIT = 4,
    SHYFT_HIP_SHARD_TEST_FAIL_GATHER = 8, SHYFT_HIP_SHARD_TEST_CORRUPT_CHECK = 16, SHYFT_HIP_SHARD_BALANCE_Z = 32,
    SHYFT_HIP_SHARD_TEST_STALL_CHECK = 64
};
int shyft_hip_region_create_sharded_ex(int stack, size_t n_cells, const int* devices, size_t n_shards, unsigned flags,
                                       shyft_hip_region** out);
/* One line: the combine path, why it was chosen, the self-check result and any run-time fallback ("" unsharded). */
const char* shyft_hip_region_combine_report(const shyft_hip_region* h);
/* Number of shards (1 for an unsharded region); for k below it, shard k's device, first cell and cell count. */
size_t shyft_hip_region_shards(const shyft_hip_region* h, size_t k, int* device, size_t* cell0, size_t* n_cells);
/* How the shards' partial sums are combined: SHYFT_HIP_COMBINE_NONE (unsharded), _COPY (device copies), _RCCL. */
enum shyft_hip_combine { SHYFT_HIP_COMBINE_NONE = 0, SHYFT_HIP_COMBINE_COPY = 1, SHYFT_HIP_COMBINE_RCCL = 2 };
int shyft_hip_region_combine_path(const shyft_hip_region* h);
size_t shyft_hip_region_size(const shyft_hip_region* h);

/* Cell geometry, n_cells x 11 doubles in the geo_cell_data_io layout
 * (api/api.h:1598-1621): x y z area cid slope glacier lake reservoir forest unspecified.
 * routing_id / routing_distance (geo_cell_data.routing, core/geo_cell_data.h:83-92) may be NULL. */
int shyft_hip_set_geo(shyft_hip_region* h, const double* geo11, const int64_t* routing_id, const double* routing_distance);

/* Parameters: n_sets rows of the stack's calibration vector in the reference's
 * get/set order (pt_gs_k: 31 values, core/pt_gs_k.h:77-112; hbv_stack 22, hbv_stack.h:82-109;
 * pt_ss_k 21, pt_ss_k.h:78-101; pt_hs_k 18, pt_hs_k.h:66-88; pt_hps_k 24, pt_hps_k.h:64-90). hbv_stack and
 * pt_hs_k rows may carry 17 more values, the hbv_snow distribution: n_bins (2..8), s[8], intervals[8]; pt_hps_k
 * rows may carry 18 more: gm.direct_response, then that distribution; set_ix[n_cells]
 * selects the row of each cell (region parameter + catchment overrides,
 * region_model.h:287-319). set_ix == NULL means row 0 for every cell. */
int shyft_hip_set_parameters(shyft_hip_region* h, const double* params, size_t n_sets, size_t n_per_set,
                             const int32_t* set_ix);

/* Time axis (fixed_dt). Allocates forcing/response storage for a resident
 * window of window_steps steps starting at step 0 (window_steps == 0: whole axis).
 * Replaces initialize_cell_environment (region_model.h:359-364): forcing is NaN-filled. */
int shyft_hip_set_time_axis(shyft_hip_region* h, int64_t t0_us, int64_t dt_us, size_t n_steps, size_t window_steps);
/* Move the resident window to start at step w0 (window length unchanged). Forcing
 * in the window becomes NaN, responses NaN. Used to stream long horizons in chunks. */
int shyft_hip_set_window(shyft_hip_region* h, size_t w0);
/* set_window with control over the NaN fill: fill_mask bit 0 forcing, bit 1 responses, bit 2 state series
 * (set_window == fill_mask 7). A caller that rewrites the whole window (a device forcing generator, a full
 * run_cells over the window) passes 0 and saves a pass over the window's HBM. */
int shyft_hip_move_window(shyft_hip_region* h, size_t w0, int fill_mask);

/* Collection mode (shyft_hip_collect) and state collection on/off
 * (set_state_collection / set_snow_sca_swe_collection, region_model.h:784-818). */
int shyft_hip_set_collection(shyft_hip_region* h, int collect, int collect_state);

/* Catchment calculation filter (region_model.h:715-779): cids[n] or n == 0 to clear. */
int shyft_hip_set_catchment_filter(shyft_hip_region* h, const int64_t* cids, size_t n);

/* State, n_cells x n_fields (pt_gs_k: 9 = gs albedo lwc surface_heat alpha sdc_melt_mean acc_melt
 * iso_pot_energy temp_swe, kirchner q; hbv_stack: 22 = swe sca sm uz lz n_bins sp[8] sw[8];
 * pt_ss_k: 8 = nu alpha sca swe free_water residual num_units q; pt_hs_k: 20 = swe sca n_bins sp[8]
 * sw[8] q; pt_hps_k: 37 = swe sca surface_heat n_bins sp[8] sw[8] albedo[8] iso_pot_energy[8] q).
 * get/set_states (region_model.h:784-805). */
int shyft_hip_set_state(shyft_hip_region* h, const double* state, size_t n_fields);
int shyft_hip_get_state(const shyft_hip_region* h, double* state, size_t n_fields);
/* dst's state := src's state, device to device (the same method stack and cell count, one device).
 * Replaces dst.set_states(src.get_states()) (region_model.h:784-805) without the host round trip: waits for
 * src's queued work, then copies on dst's stream. Used to pipeline two regions over consecutive windows. */
int shyft_hip_copy_state(shyft_hip_region* dst, const shyft_hip_region* src);

/* Forcing for steps [step0, step0+n) of one variable, [n][n_cells].
 * src_on_device != 0: src is a device pointer on the region's device. */
int shyft_hip_set_forcing(shyft_hip_region* h, int var, size_t step0, size_t n, const double* src, int src_on_device);
int shyft_hip_get_forcing(const shyft_hip_region* h, int var, size_t step0, size_t n, double* dst, int dst_on_device);

/* Inverse-distance interpolation of one forcing variable from n_sources geo-located sources
 * into the cells (region_model::interpolate's per-variable idw::run_interpolation,
 * core/region_model.h:456-515, core/inverse_distance.h:142-250), for steps [step0, step0+n)
 * of the resident window. Only cells passing the catchment calculation filter are written.
 *  src_xyz    : n_sources x 3 (geo_point x y z)
 *  src_values : [n][n_sources], the sources already averaged onto the model time axis
 *               (the average_accessor step, region_model.h:135-145, is the caller's)
 *  idw_param  : max_members (<= 32), max_distance, distance_measure_factor, zscale,
 *               default_temp_gradient, gradient_by_equation (0/1), precipitation scale_factor
 *               (inverse_distance.h:38-74)
 * Model by variable: temperature (gradient transform), precipitation (scale^(dz/100)),
 * radiation (x slope factor), wind_speed and rel_hum (plain). A single temperature source is
 * copied to every cell as the reference does (region_model.h:470-481). The neighbour table is
 * built on the first call and reused while sources and parameters are unchanged. */
int shyft_hip_interpolate(shyft_hip_region* h, int var, size_t n_sources, const double* src_xyz,
                          const double* src_values, size_t step0, size_t n, const double* idw_param);
/* Which gather the last shyft_hip_interpolate of variable var ran (no reference counterpart: a test and
 * measurement aid): SHYFT_HIP_IDW_WAVE (every wavefront's neighbour union fits 64 stations: the compacted
 * wavefront-union gather), SHYFT_HIP_IDW_TILE (the row-tile gather), SHYFT_HIP_IDW_COPY (one temperature source
 * copied), SHYFT_HIP_IDW_NONE (no interpolation of var yet). Returns -1 on a bad handle or variable. */
enum shyft_hip_idw_path { SHYFT_HIP_IDW_NONE = 0, SHYFT_HIP_IDW_TILE = 1, SHYFT_HIP_IDW_WAVE = 2, SHYFT_HIP_IDW_COPY = 3 };
int shyft_hip_interpolation_path(const shyft_hip_region* h, int var);

/* Bayesian temperature kriging of the temperature forcing into the calculated cells, steps [step0, step0+n)
 * of the resident window: region_model::interpolate's default temperature method
 * (core/region_model.h:460-468 -> bayesian_kriging::btk_interpolation, core/bayesian_kriging.h:280-402).
 *  src_xyz        : n_sources x 3
 *  src_values     : [n][n_sources] on the model axis (average_accessor is the caller's); NaN = missing, and
 *                   a step whose valid-source set differs from the full set uses the reference's reduced
 *                   operators for that set
 *  prior_gradient : [n] the prior temperature gradient per step (parameter.temperature_gradient(period)), or
 *                   NULL for bayesian_kriging::parameter's day-of-year formula on the region's time axis
 *                   (bayesian_kriging.h:220-223)
 *  btk_param      : temperature_gradient_sd (C/m, i.e. already /100), sill, nugget, range, zscale
 * One source is copied to the cells (region_model.h:470-481). Errors carry the reference's texts ("needs at
 * least two sources at different heights", "No valid sources for time period"). */
int shyft_hip_interpolate_btk(shyft_hip_region* h, size_t n_sources, const double* src_xyz, const double* src_values,
                              size_t step0, size_t n, const double* prior_gradient, const double* btk_param);
/* Stateless bayesian_kriging_temperature (api/boostpython/api_interpolation.cpp:54-71) on a device (device < 0 =
 * current): dst_xyz [n_dst][3], prior_gradient [n] (required), out [n][n_dst] host. */
int shyft_hip_btk(int device, size_t n_sources, const double* src_xyz, const double* src_values, size_t n,
                  const double* prior_gradient, const double* btk_param, size_t n_dst, const double* dst_xyz,
                  double* out);

/* Deterministic synthetic forcing for steps [step0, step0+n) of the resident window,
 * generated on device (bench/test workload; SURVEY.md §8d generator). */
int shyft_hip_synthetic_forcing(shyft_hip_region* h, uint64_t seed, uint64_t cell_offset, size_t step0, size_t n);
/* The synthetic region's cell elevations z[i] = 2000*u(seed, 7, cell_offset+i, 0) (same generator), n_cells values. */
int shyft_hip_synthetic_elevation(uint64_t seed, uint64_t cell_offset, size_t n_cells, double* z_host);

/* region_model::run_cells(use_ncore, start_step, n_steps) — region_model.h:578-597.
 * use_ncore is validated like the reference and otherwise ignored. Blocks until done. */
int shyft_hip_run_cells(shyft_hip_region* h, size_t use_ncore, int start_step, int n_steps);
/* Asynchronous variant on the region's stream (no argument re-validation of state). */
int shyft_hip_run_cells_async(shyft_hip_region* h, int start_step, int n_steps);
int shyft_hip_synchronize(shyft_hip_region* h);
/* Double-buffered forcing window (measurement / pipelining aid, no reference counterpart): generate the synthetic
   forcing of the window starting at w0_next into a second buffer on a side stream restricted to n_cus CUs (0: no
   restriction; < 0: the whole device at the lowest stream priority) while the current window runs (it waits only
   for the run that last read that buffer); shyft_hip_swap_forcing_window(h, w0_next) then makes it the
   region's window (the next run waits for the generator on the device). The swap does not NaN-fill the response
   and state-series rows: a run over the new window must follow before they are read. A pending prefetch is
   dropped when the time axis or window length changes (shyft_hip_set_time_axis). */
int shyft_hip_prefetch_synthetic_forcing(shyft_hip_region* h, uint64_t seed, uint64_t cell_offset, size_t w0_next,
                                         int n_cus);
int shyft_hip_swap_forcing_window(shyft_hip_region* h, size_t w0_next);
/* Milliseconds of the last run_cells kernel launch(es), timed with HIP events on the region's stream. */
double shyft_hip_last_run_ms(const shyft_hip_region* h);
/* The last run's kernels separately: every stack runs one kernel per run_cells, so parts is 1 (ms[0] = the kernel;
   a sharded region: the slowest running shard's). Fills ms[0..min(n, parts)) and returns the number of parts.
   (No reference counterpart: measurement only.) */
int shyft_hip_last_run_kernel_ms(const shyft_hip_region* h, double* ms, int n);
/* Milliseconds of the last shyft_hip_interpolate's gather kernel (HIP events on the region's stream; the neighbour
   table build of a new source geometry is not included). A sharded region: the slowest interpolating shard's.
   (No reference counterpart: measurement only.) */
double shyft_hip_last_interpolate_ms(const shyft_hip_region* h);
/* Kernel milliseconds of the last run_cells of every shard (0 for a shard idle under the catchment filter) into
   ms[0..min(n, shards)); returns the number of shards (1 and the region's own time when unsharded). */
size_t shyft_hip_shard_run_ms(const shyft_hip_region* h, double* ms, size_t n);

/* Response series for steps [step0, step0+n), [n][n_cells]. */
int shyft_hip_get_series(const shyft_hip_region* h, int series, size_t step0, size_t n, double* dst, int dst_on_device);
/* State-collector series (instant, T+1 axis), field f in state order, steps [step0, step0+n). */
int shyft_hip_get_state_series(const shyft_hip_region* h, int field, size_t step0, size_t n, double* dst,
                               int dst_on_device);

/* Catchment statistics (cell_statistics::sum_catchment_feature / average_catchment_feature,
 * core/cell_model.h:228-333): sum (weighted == 0) or area-weighted average (weighted != 0)
 * of series `series` (response id, SHYFT_HIP_SERIES_FORCING + v or SHYFT_HIP_SERIES_STATE + f) over the cells selected by ids[n_ids] (scope: cell index or catchment id;
 * n_ids == 0 selects all cells), for steps [step0, step0+n). dst[n]. Throws (returns error)
 * on unknown ids like verify_cids_exist (cell_model.h:198-211). */
int shyft_hip_statistics(const shyft_hip_region* h, int series, const int64_t* ids, size_t n_ids, int scope,
                         int weighted, size_t step0, size_t n, double* dst);
/* Per-catchment sums of a series for all catchments at once (region_model::catchment_discharges,
 * region_model.h:873-885): dst[n_catchments][n] in catchment_ids() order, device or host. */
int shyft_hip_catchment_sums(const shyft_hip_region* h, int series, size_t step0, size_t n, double* dst,
                             int dst_on_device);
/* Per-catchment sums of value x cell area (calculated catchments, cell order, same reduction as
 * shyft_hip_catchment_sums): the area-weighted snow sca/swe sums of the calibration goal function
 * (optimizer::extract_area_ts_property, core/model_calibration.h:759-776). dst[n_catchments][n]. */
int shyft_hip_catchment_area_sums(const shyft_hip_region* h, int series, size_t step0, size_t n, double* dst,
                                  int dst_on_device);
size_t shyft_hip_number_of_catchments(const shyft_hip_region* h);
int shyft_hip_catchment_ids(const shyft_hip_region* h, int64_t* cids);

/* Deep copy of a region (cells, parameters, time axis, forcing, state, collected series) on the
 * same device: the region_model copy constructor / clone (core/region_model.h:297-301, expose.h:147),
 * used for create_opt_model_clone / create_full_model_clone. */
int shyft_hip_region_clone(const shyft_hip_region* src, shyft_hip_region** out);

/* One cell's view of a series (cell.env_ts.<var>, cell.rc.<series>, cell.sc.<field>,
 * core/cell_model.h:47-81,112-160): steps [step0, step0+n) copied to/from buf[n].
 * write != 0 is allowed for forcing only (env_ts.<var>.set(i, v)). series uses the ids above. */
int shyft_hip_cell_series(shyft_hip_region* h, int series, size_t cell, size_t step0, size_t n, double* buf, int write);
/* Many cells' views at once (the per-cell collector series of region_model::get_cells(), read in bulk): columns
 * cells[n_cells] of series `series` (ids as above), steps [step0, step0+n) of the resident window, into host
 * dst[n][n_cells]. One gather on the device (per shard for a sharded region). */
int shyft_hip_sample_cells(const shyft_hip_region* h, int series, const int64_t* cells, size_t n_cells, size_t step0,
                           size_t n, double* dst);

/* Test knobs (no reference counterpart; every knob is 0 in production). SHYFT_HIP_KNOB_PTGSK_INSTANCE: 0 = the
 * launcher picks the pt_gs_k kernel instance by region size, 2 = the 64-lane 2-wave instance, 4 = the 256-lane 4-wave
 * instance. SHYFT_HIP_KNOB_BRENT_READ_DELAY: n > 0 makes every wavefront of a 256-lane pt_gs_k workgroup except the
 * first sleep n x s_sleep(127) between the Brent phase and reading its results, so the first wavefront runs ahead
 * into the next step's job queue (the interleaving the queue's double buffering must survive). */
enum shyft_hip_knob {
    SHYFT_HIP_KNOB_PTGSK_INSTANCE = 1, SHYFT_HIP_KNOB_BRENT_READ_DELAY = 2,
    /* sharded regions: 1 = run_cells runs the shards one after another (per-shard kernel times without contention,
     * shyft_hip_shard_run_ms); 0 = concurrently (the default) */
    SHYFT_HIP_KNOB_SERIAL_SHARDS = 3,
    /* sharded regions: k >= 0 makes the next shyft_hip_region_clone of this region fail when it reaches shard k (the
     * shards before it already cloned, with their streams), so the clean-up of a partly built clone is exercised;
     * the failure is reported like any other and disarms the knob; < 0 = off (the default) */
    SHYFT_HIP_KNOB_CLONE_FAIL_AT = 4
};
int shyft_hip_set_test_knob(shyft_hip_region* h, int knob, int64_t value);

/* region_model::is_cell_env_ts_ok (core/region_model.h:954-962): *ok = 1 when no forcing value of a
 * calculated cell (catchment filter) in the resident window is NaN. */
int shyft_hip_forcing_ok(const shyft_hip_region* h, int* ok);

/* ---- routing::uhg river aggregation (core/routing.h:239-421; region_model.h:909-949) ----
 * Convolution is linear, so the engine reduces the avg_discharge of all cells that share a river
 * and a unit hydrograph ("routing group") to one sum per group on the device, and convolves only
 * those sums. */

/* group_of_cell[n_cells]: the routing group of each cell, -1 = not routed (routing.id <= 0). */
int shyft_hip_set_routing_groups(shyft_hip_region* h, const int32_t* group_of_cell, size_t n_groups);
/* dst[n_groups][n]: sum over each group's cells (cell order) of avg_discharge, steps [step0, step0+n). */
int shyft_hip_routing_group_sums(const shyft_hip_region* h, size_t step0, size_t n, double* dst, int dst_on_device);
/* River network evaluation on a device (stateless; device < 0 = current): rivers are indexed 0..R-1 in
 * ascending river id. group_sums[G][T] (host or device), group_uhg[G][max_len] / group_len[G] the cell UHG
 * of each group (make_uhg_from_gamma, routing.h:399-421), group_river[G] its river, river_uhg[R][max_len] /
 * river_len[R], river_downstream[R] (index, -1 = none). Outputs [R][T]: local_inflow, upstream_inflow,
 * output_m3s (routing::model::local_inflow / upstream_inflow / output_m3s, routing.h:347-387). */
int shyft_hip_route(int device, size_t n_groups, size_t T, const double* group_sums, int src_on_device,
                    const double* group_uhg, const int32_t* group_len, const int32_t* group_river, size_t n_rivers,
                    const double* river_uhg, const int32_t* river_len, const int32_t* river_downstream, size_t max_len,
                    double* local, double* upstream, double* output, int dst_on_device);

/* ---- parameter ensembles for calibration (core/model_calibration.h:830-899) ----
 * The reference optimizer evaluates one parameter vector per region run: set parameters, revert to the
 * initial state, run_cells over the calculated catchments, sum catchment discharge, score against the
 * targets. shyft_hip_ensemble_run evaluates n_members parameter vectors in ONE launch: its lanes are
 * (calculated cell, member) pairs, member-fastest, each starting from the region's current state and
 * reading the region's forcing in place (shared, not copied). The region's own state and responses are
 * not modified. params[n_members][n_per_set] in the reference get/set order (as shyft_hip_set_parameters).
 * collect: SHYFT_HIP_COLLECT_DISCHARGE or SHYFT_HIP_COLLECT_DISCHARGE_SNOW (adds snow sca / swe). */
int shyft_hip_ensemble_run(shyft_hip_region* h, const double* params, size_t n_members, size_t n_per_set,
                           int start_step, int n_steps, int collect);
/* Sums of response `series` of the last ensemble run per member and catchment, steps [step0, step0+n)
 * inside its run range: dst[n_members][n_catchments][n], catchments in shyft_hip_catchment_ids order
 * (uncalculated catchments sum to 0). area_weighted != 0: sum of value x cell area (the area-weighted
 * snow sums of model_calibration.h:765-776). */
int shyft_hip_ensemble_sums(const shyft_hip_region* h, int series, int area_weighted, size_t step0, size_t n,
                            double* dst, int dst_on_device);
/* Milliseconds of the last ensemble launch (HIP events on its stream). */
double shyft_hip_ensemble_last_ms(const shyft_hip_region* h);

/* Diagnostic: evaluate one device elementary function (0 exp, 1 log, 2 pow(x, y), 3 lgamma,
 * 4 gamma_p(x, y)) on n host inputs on the current device; out[n] host. Used by the parity
 * tests to show device math == host math bit for bit. */
int shyft_hip_math_selftest(int fn, const double* x, const double* y, size_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* SHYFT_HIP_H */
