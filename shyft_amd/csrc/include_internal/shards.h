// Internal: the sharded-region layer (shards.hip) behind the C ABI entry points of region.hip.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "region_impl.h"

namespace shyft_hip_impl {

shard_set* shard_set_create(int stack, size_t n_cells, const int* devices, size_t n_shards,
                            unsigned flags);  // throws
void shard_set_destroy(shard_set* s);

// region.hip: the generator keys of a region's cells (null: 0..n-1), for a z-balanced shard
void region_set_cell_ids(shyft_hip_region* h, const int64_t* ids);  // throws

// region.hip: sum over the selected cells of one region (select_cells semantics), value x cell area when weighted;
// *sum_area = the selected cells' area sum (weighted only). dst[n] host. No selection match: dst = 0.
int region_selected_sums(shyft_hip_region* h, int series, const int64_t* ids, size_t n_ids, int scope, int weighted,
                         size_t step0, size_t n, double* dst, double* sum_area, size_t* n_selected);

namespace shards {
size_t info(const shard_set* s, size_t k, int* device, size_t* cell0, size_t* n_cells);
int combine_path(const shard_set* s);
const char* combine_report(const shard_set* s);
void set_test_knob(shard_set* s, int knob, int64_t value);
size_t shard_run_ms(const shard_set* s, double* ms, size_t n);
void sample_cells(shard_set* s, int series, const int64_t* cells, size_t n_cells, size_t step0, size_t n, double* dst);
void set_geo(shard_set* s, const double* geo11, const int64_t* rid, const double* rdist);
void set_parameters(shard_set* s, const double* params, size_t n_sets, size_t n_per_set, const int32_t* set_ix);
void set_time_axis(shard_set* s, int64_t t0, int64_t dt, size_t n_steps, size_t window);
void move_window(shard_set* s, size_t w0, int fill_mask);
void set_collection(shard_set* s, int collect, int collect_state);
void set_catchment_filter(shard_set* s, const int64_t* cids, size_t n);
void set_state(shard_set* s, const double* state, size_t n_fields);
void get_state(shard_set* s, double* state, size_t n_fields);
void copy_state(shard_set* d, const shard_set* src);
void set_forcing(shard_set* s, int var, size_t step0, size_t n, const double* src, int on_device);
void get_rows(shard_set* s, int what, int id, size_t step0, size_t n, double* dst, int on_device);
void interpolate(shard_set* s, int var, size_t n_sources, const double* xyz, const double* vals, size_t step0, size_t n,
                 const double* prm);
int interpolation_path(const shard_set* s, int var);
void interpolate_btk(shard_set* s, size_t n_sources, const double* xyz, const double* vals, size_t step0, size_t n,
                     const double* prior, const double* prm);
void synthetic_forcing(shard_set* s, uint64_t seed, uint64_t cell_offset, size_t step0, size_t n);
void prefetch_synthetic_forcing(shard_set* s, uint64_t seed, uint64_t cell_offset, size_t w0_next, int n_cus);
void swap_forcing_window(shard_set* s, size_t w0_next);
void run_cells(shard_set* s, size_t use_ncore, int start_step, int n_steps);
void run_cells_async(shard_set* s, int start_step, int n_steps);
void synchronize(shard_set* s);
double last_run_ms(const shard_set* s);
double last_interpolate_ms(const shard_set* s);
int last_run_kernel_ms(const shard_set* s, double* ms, int n);
void cell_series(shard_set* s, int series, size_t cell, size_t step0, size_t n, double* buf, int write);
void forcing_ok(shard_set* s, int* ok);
void statistics(shard_set* s, int series, const int64_t* ids, size_t n_ids, int scope, int weighted, size_t step0,
                size_t n, double* dst);
void catchment_sums(shard_set* s, int series, size_t step0, size_t n, double* dst, int on_device, bool area);
size_t number_of_catchments(const shard_set* s);
void catchment_ids(const shard_set* s, int64_t* cids);
void set_routing_groups(shard_set* s, const int32_t* group_of_cell, size_t n_groups);
void routing_group_sums(shard_set* s, size_t step0, size_t n, double* dst, int on_device);
void ensemble_run(shard_set* s, const double* params, size_t n_members, size_t n_per_set, int start_step, int n_steps,
                  int collect);
void ensemble_sums(shard_set* s, int series, int area_weighted, size_t step0, size_t n, double* dst, int on_device);
double ensemble_last_ms(const shard_set* s);
shard_set* clone(const shard_set* src);
}  // namespace shards

}  // namespace shyft_hip_impl
