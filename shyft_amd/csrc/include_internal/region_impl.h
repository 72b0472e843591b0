// Internal: the region handle behind the C ABI (include/shyft_hip.h), shared by region.hip (one region on one
// device) and shards.hip (a region whose cells are split over several regions / devices).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/shyft_hip.h"
#include "kernels.h"
#include "layout.h"

namespace shyft_hip_impl {

extern thread_local std::string g_last_error;  // region.hip

struct hip_error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw hip_error(std::string(what) + ": " + hipGetErrorString(e));
}

template <class T>
struct dbuf {
    T* p = nullptr;
    size_t n = 0;
    dbuf() = default;
    dbuf(const dbuf&) = delete;
    dbuf& operator=(const dbuf&) = delete;
    ~dbuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t count) {
        if (count == n && p) return;
        release();
        if (count == 0) return;
        hip_check(hipMalloc(&p, count * sizeof(T)), "hipMalloc");
        n = count;
    }
};

struct shard_set;  // shards.hip: the shards of a sharded region

}  // namespace shyft_hip_impl

using shyft_hip_impl::dbuf;

struct shyft_hip_region {
    // a sharded region (shyft_hip_region_create_sharded) owns its shards here and no device buffers of its own;
    // every entry point forwards to shards.hip
    shyft_hip_impl::shard_set* sh = nullptr;
    int stack = 0;
    size_t n = 0;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_copy = nullptr;  // shyft_hip_copy_state: the copy out of this region's state has finished
    std::string err;
    double last_ms = 0.0;
    double last_interp_ms = 0.0;  // the last interpolate's gather kernel
    int knob_instance = 0, knob_read_delay = 0;  // shyft_hip_set_test_knob (pt_gs_k launches)

    // host mirrors
    std::vector<double> geo;  // n x 11
    std::vector<int64_t> routing_id;
    std::vector<double> routing_distance;
    std::vector<int64_t> cid;          // per cell
    std::vector<size_t> cix;           // per cell
    std::vector<int64_t> cix_to_cid;   // region_model::cix_to_cid
    std::map<int64_t, size_t> cid_to_cix;
    std::vector<double> params;        // n_sets x param_width()
    size_t n_sets = 0;
    std::vector<int32_t> set_ix;
    std::vector<uint8_t> active;       // empty = no filter
    int64_t t0 = 0, dt = 0;
    size_t T = 0, w0 = 0, TW = 0;
    int collect = COLLECT_DISCHARGE;
    int collect_state = 0;
    bool derived_dirty = true;
    bool has_geo = false, has_params = false, has_state = false;

    // device
    dbuf<double> d_params, d_cellc, d_state, d_forcing, d_resp, d_state_series;
    // double-buffered forcing window (shyft_hip_prefetch_synthetic_forcing / shyft_hip_swap_forcing_window): the
    // next window is generated on gen_stream (restricted to a few CUs) while the current one runs
    dbuf<double> d_forcing_next;
    hipStream_t gen_stream = nullptr;
    int gen_cus = -1;
    hipEvent_t ev_gen = nullptr;
    hipEvent_t ev_free = nullptr;  // recorded at the last swap: the swapped-out buffer's last reader has finished
    bool free_pending = false;
    size_t gen_w0 = SIZE_MAX;
    dbuf<int32_t> d_set_ix, d_err, d_doy, d_seg_cells, d_seg_off, d_sel;
    dbuf<int64_t> d_trel;
    dbuf<uint8_t> d_active;
    dbuf<double> d_tmp, d_w, d_alt;
    dbuf<int64_t> d_cell_ids;  // a z-balanced shard: the region cell of each of its cells (synthetic forcing keys)
    dbuf<int32_t> d_flag;

    // inverse-distance neighbour tables, one per forcing variable, cached by
    // (model, parameters, source geometry)
    struct idw_table {
        std::vector<double> key;
        dbuf<int32_t> idx, cnt;
        dbuf<double> w, aux;
        dbuf<int32_t> wu, wn, ovf;  // wavefront unions of the neighbour lists (idw_wave_union)
        dbuf<uint32_t> lidx;
        bool wave_ok = false;
        int K = 0;
        int last_path = SHYFT_HIP_IDW_NONE;  // the gather the last interpolate of this variable ran
    } idw[N_FORCING];
    dbuf<double> d_dst_xyz, d_slope, d_src_xyz, d_src_vals;
    bool dst_dirty = true;
    // Bayesian temperature kriging destinations (calculated cells) and their window columns
    dbuf<double> d_btk_xyz;
    dbuf<int32_t> d_btk_index;
    std::vector<double> btk_xyz_host;
    std::vector<int32_t> btk_index_host;
    uint64_t btk_dst_version = 0;
    std::unique_ptr<btk_cache, void (*)(btk_cache*)> btk{nullptr, btk_cache_destroy};

    // routing groups (cells sharing river + UHG): segment tables for the group discharge sums
    dbuf<int32_t> d_rseg_cells, d_rseg_off;
    // the catchment / routing-group segments are the identity permutation of the cells (contiguous ranges in cell
    // order): the segment sums do not read the index arrays
    bool seg_identity = false, rseg_identity = false;
    size_t n_route_groups = 0;

    // parameter ensemble (calibration): a lane region of calculated cells x members that reads this
    // region's forcing through d_fcol (see shyft_hip_ensemble_run)
    shyft_hip_region* ens = nullptr;
    const shyft_hip_region* forcing_src = nullptr;  // set on an ensemble lane region: whose forcing it reads
    dbuf<int32_t> d_fcol;                            // [lanes] forcing column (cell of the parent region)
    size_t ens_members = 0, ens_cells = 0, ens_groups = 0, ens_b = 0, ens_e = 0;

    bool hbv() const { return stack == SHYFT_HIP_HBV_STACK; }
    bool ptssk() const { return stack == SHYFT_HIP_PT_SS_K; }
    bool pthsk() const { return stack == SHYFT_HIP_PT_HS_K; }
    bool pthpsk() const { return stack == SHYFT_HIP_PT_HPS_K; }
    size_t n_series() const {
        if (collect == COLLECT_ALL) return hbv() ? HBV_NR : PTGSK_NR;
        return collect == COLLECT_DISCHARGE_SNOW ? 4 : 2;
    }
    size_t n_state_fields() const {
        return hbv() ? HBV_NS : (ptssk() ? PTSSK_NS : (pthsk() ? PTHSK_NS : (pthpsk() ? PTHPSK_NS : PTGSK_NS)));
    }
    // state-collector series per cell (pt_ss_k collects 7 series from its 8 state values)
    size_t n_state_series() const {
        return ptssk() ? PTSSK_NSC : (pthsk() ? PTHSK_NSC : (pthpsk() ? PTHPSK_NSC : n_state_fields()));
    }
    size_t n_ref_params() const {
        return hbv() ? HBV_NP_REF
                     : (ptssk() ? PTSSK_NP : (pthsk() ? PTHSK_NP_REF : (pthpsk() ? PTHPSK_NP_REF : PTGSK_NP_REF)));
    }
    size_t param_width() const {
        return hbv() ? HBV_NP : (ptssk() ? PTSSK_NP : (pthsk() ? PTHSK_NP : (pthpsk() ? PTHPSK_NP : PTGSK_NP_REF)));
    }
    // hbv_snow quantile distribution (n_bins, s[], intervals[]) in the parameter row, or -1
    int snow_dist_index() const { return hbv() ? HK_NB : (pthsk() ? PH_NB : (pthpsk() ? PP_NB : -1)); }
};

namespace shyft_hip_impl {

int fail(shyft_hip_region* h, const std::string& msg);

template <class F>
inline int guarded(shyft_hip_region* h, F&& f) {
    try {
        if (h) hip_check(hipSetDevice(h->device), "hipSetDevice");
        f();
        return 0;
    } catch (const std::exception& e) {
        return fail(h, e.what());
    } catch (...) {
        return fail(h, "unknown error");
    }
}

}  // namespace shyft_hip_impl
