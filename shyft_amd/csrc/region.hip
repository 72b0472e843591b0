// C-ABI implementation (include/shyft_hip.h): one region handle owns the
// SoA device buffers of its cells on one device and one HIP stream.
//
// Mirrors the state machine of region_model (core/region_model.h:211-1049):
// cells + parameters + time axis + cell environment (forcing) + state +
// collectors; run_cells launches one kernel over every cell of the region.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/shyft_hip.h"
#include "include_internal/kernels.h"
#include "include_internal/layout.h"
#include "include_internal/region_impl.h"
#include "include_internal/shards.h"
#include "include_internal/synth_hash.h"
#include "../../detmath/detmath.h"

namespace shyft_hip_impl {
thread_local std::string g_last_error;
int fail(shyft_hip_region* h, const std::string& msg) {
    if (h) h->err = msg;
    g_last_error = msg;
    return 1;
}
}  // namespace shyft_hip_impl

using namespace shyft_hip_impl;

namespace {

// UTC civil calendar (core/utctime_utilities.cpp:230-253)
int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}
void civil_from_days(int64_t z, int64_t& y, int& m, int& d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    d = int(doy - (153 * mp + 2) / 5 + 1);
    m = int(mp < 10 ? mp + 3 : mp - 9);
    y += (m <= 2);
}
int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
constexpr int64_t DAY_US = 86400LL * 1000000LL;

// calendar::day_of_year (UTC, core/utctime_utilities.cpp:230-235)
int day_of_year(int64_t t_us) {
    const int64_t days = floor_div(t_us, DAY_US);
    int64_t y;
    int m, d;
    civil_from_days(days, y, m, d);
    return int(1 + days - days_from_civil(y, 1, 1));
}

// bayesian_kriging::parameter::temperature_gradient(period) (core/bayesian_kriging.h:220-223): the prior
// gradient from the day of year of the period's midpoint
double btk_prior_gradient(int64_t start_us, int64_t dt_us) {
    const double doy = double(day_of_year(start_us + dt_us / 2));
    return 1.18e-3 * std::sin(6.2831 / 365 * (doy + 79.0)) - 5.48e-3;
}

}  // namespace


namespace {


// host <-> region copies are ordered on the region's stream (created non-blocking, so a null-stream copy would
// not wait for a run or copy_state still queued there) and complete before returning, like hipMemcpy
hipError_t region_copy(shyft_hip_region* h, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, h->stream);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(h->stream);
}


// region_model::update_ix_to_id_mapping (region_model.h:236-252)
void update_ix_to_id_mapping(shyft_hip_region* h) {
    h->cid_to_cix.clear();
    h->cix_to_cid.clear();
    h->cid.resize(h->n);
    h->cix.resize(h->n);
    for (size_t i = 0; i < h->n; ++i) {
        const int64_t c = int64_t(int(h->geo[i * 11 + 4]));
        h->cid[i] = c;
        auto f = h->cid_to_cix.find(c);
        if (f == h->cid_to_cix.end()) {
            h->cid_to_cix[c] = h->cix_to_cid.size();
            h->cix[i] = h->cix_to_cid.size();
            h->cix_to_cid.push_back(c);
        } else {
            h->cix[i] = f->second;
        }
    }
    // catchment segments: cells of each catchment in cell order
    const size_t C = h->cix_to_cid.size();
    std::vector<int32_t> off(C + 1, 0), cells(h->n);
    for (size_t i = 0; i < h->n; ++i) off[h->cix[i] + 1]++;
    for (size_t c = 0; c < C; ++c) off[c + 1] += off[c];
    std::vector<int32_t> pos(off.begin(), off.end() - 1);
    for (size_t i = 0; i < h->n; ++i) cells[pos[h->cix[i]]++] = int32_t(i);
    h->seg_identity = true;
    for (size_t i = 0; i < h->n && h->seg_identity; ++i) h->seg_identity = cells[i] == int32_t(i);
    h->d_seg_cells.alloc(h->n);
    h->d_seg_off.alloc(C + 1);
    hip_check(region_copy(h, h->d_seg_cells.p, cells.data(), h->n * sizeof(int32_t), hipMemcpyHostToDevice), "upload seg");
    hip_check(region_copy(h, h->d_seg_off.p, off.data(), (C + 1) * sizeof(int32_t), hipMemcpyHostToDevice), "upload seg");
}

// derived per-set parameter rows and per-cell constants (pt_gs_k.h:347-357,
// gamma_snow.h:85-87, :188, :340-343). Evaluated with the same expressions
// the reference evaluates, on the host.
void update_derived_hbv(shyft_hip_region* h) {
    const size_t N = h->n;
    std::vector<double> cc(HBV_NC * N);
    for (size_t i = 0; i < N; ++i) {
        const double* g = &h->geo[i * 11];
        const double* p = &h->params[size_t(h->set_ix[i]) * HBV_NP];
        const double glacier = g[6], reservoir = g[8];
        const double direct = glacier * p[HK_GM_DIRECT] + reservoir * p[HK_RSV_DRF];
        cc[HC_GLACIER * N + i] = glacier;
        cc[HC_DIRECT_RESPONSE * N + i] = direct;
        cc[HC_LAND_FRACTION * N + i] = 1 - direct;
        cc[HC_AREA * N + i] = g[3];
        cc[HC_GLACIER_AREA * N + i] = g[3] * glacier;
    }
    h->d_params.alloc(h->params.size());
    h->d_cellc.alloc(cc.size());
    h->d_set_ix.alloc(N);
    hip_check(region_copy(h, h->d_params.p, h->params.data(), h->params.size() * sizeof(double), hipMemcpyHostToDevice),
              "upload params");
    hip_check(region_copy(h, h->d_cellc.p, cc.data(), cc.size() * sizeof(double), hipMemcpyHostToDevice), "upload cellc");
    hip_check(region_copy(h, h->d_set_ix.p, h->set_ix.data(), N * sizeof(int32_t), hipMemcpyHostToDevice), "upload set_ix");
    h->derived_dirty = false;
}

// pt_ss_k / pt_hs_k: parameter rows as given, per-cell constants of pt_ss_k.h:237-245 (pt_hs_k.h:233-242,
// the same expressions) in the pt_gs_k PC_* rows
void update_derived_ptssk(shyft_hip_region* h) {
    const size_t N = h->n;
    const size_t width = h->param_width();
    const int k_gm = h->pthsk() ? PH_GM_DIRECT : (h->pthpsk() ? PP_GM_DIRECT : SK_GM_DIRECT);
    const int k_rsv = h->pthsk() ? PH_RSV_DRF : (h->pthpsk() ? PP_RSV_DRF : SK_RSV_DRF);
    std::vector<double> cc(PTGSK_NC * N, 0.0);
    for (size_t i = 0; i < N; ++i) {
        const double* g = &h->geo[i * 11];
        const double* p = &h->params[size_t(h->set_ix[i]) * width];
        const double glacier = g[6], lake = g[7], reservoir = g[8];
        const double gm_direct = p[k_gm];
        const double rdrf = p[k_rsv];
        const double direct = glacier * gm_direct + reservoir * rdrf;
        cc[PC_GLACIER * N + i] = glacier;
        cc[PC_SNOW_STORAGE * N + i] = 1.0 - lake - reservoir;
        cc[PC_KIRCHNER_ROUTED_PREC * N + i] = reservoir * (1.0 - rdrf) + lake;
        cc[PC_DIRECT_RESPONSE * N + i] = direct;
        cc[PC_KIRCHNER_FRACTION * N + i] = 1 - direct;
        cc[PC_AREA * N + i] = g[3];
        cc[PC_GLACIER_AREA * N + i] = g[3] * glacier;
    }
    h->d_params.alloc(h->params.size());
    h->d_cellc.alloc(cc.size());
    h->d_set_ix.alloc(N);
    hip_check(region_copy(h, h->d_params.p, h->params.data(), h->params.size() * sizeof(double), hipMemcpyHostToDevice),
              "upload params");
    hip_check(region_copy(h, h->d_cellc.p, cc.data(), cc.size() * sizeof(double), hipMemcpyHostToDevice), "upload cellc");
    hip_check(region_copy(h, h->d_set_ix.p, h->set_ix.data(), N * sizeof(int32_t), hipMemcpyHostToDevice), "upload set_ix");
    h->derived_dirty = false;
}

void update_derived(shyft_hip_region* h) {
    if (!h->derived_dirty) return;
    if (!h->has_geo) throw std::runtime_error("region: geo_cell_data not set");
    if (!h->has_params) throw std::runtime_error("region: parameters not set");
    if (h->dt <= 0) throw std::runtime_error("region_model::run with invalid time_axis invoked");
    if (h->hbv()) return update_derived_hbv(h);
    if (h->ptssk() || h->pthsk() || h->pthpsk()) return update_derived_ptssk(h);
    const size_t N = h->n;
    const double dt_s = double(h->dt) / 1e6;
    const double dt_in_days = dt_s / 86400.0;
    std::vector<double> P(h->n_sets * PTGSK_NP, 0.0);
    for (size_t k = 0; k < h->n_sets; ++k) {
        const double* p = &h->params[k * PTGSK_NP_REF];
        double* q = &P[k * PTGSK_NP];
        for (int j = 0; j < PTGSK_NP_REF; ++j) q[j] = p[j];
        q[PK_WED] = double(size_t(p[PK_WED]));   // size_t(p[i]) (pt_gs_k.h:103)
        q[PK_NWD] = double(size_t(p[PK_NWD]));   // implicit size_t conversion (pt_gs_k.h:109)
        q[PK_ISO] = p[PK_ISO] != 0.0 ? 1.0 : 0.0;
        const double albedo_range = p[PK_MAX_ALBEDO] - p[PK_MIN_ALBEDO];
        q[PK_ALBEDO_RANGE] = albedo_range;
        q[PK_SLOW_DECAY] = 0.5 * albedo_range * dt_in_days / p[PK_SLOW_DECAY_RATE];
        q[PK_FAST_DECAY] = detmath::pow(2.0, -dt_in_days / p[PK_FAST_DECAY_RATE]);
        q[PK_BB0] = 0.98 * 5.670373e-8 * detmath::pow(273.15, 4.0);
        q[PK_INV_CV2_PARAM] = 1.0 / (p[PK_SNOW_CV] * p[PK_SNOW_CV]);
    }
    std::vector<double> cc(PTGSK_NC * N);
    for (size_t i = 0; i < N; ++i) {
        const double* g = &h->geo[i * 11];
        const double* p = &h->params[size_t(h->set_ix[i]) * PTGSK_NP_REF];
        const double glacier = g[6], lake = g[7], reservoir = g[8], forest = g[9];
        const double gm_direct = p[PK_GM_DIRECT];
        const double rdrf = p[PK_RSV_DRF];
        const double direct = glacier * gm_direct + reservoir * rdrf;
        const double cv = p[PK_SNOW_CV] + forest * p[PK_CV_FOREST] + g[2] * p[PK_CV_ALT];
        cc[PC_FOREST * N + i] = forest;
        cc[PC_GLACIER * N + i] = glacier;
        cc[PC_SNOW_STORAGE * N + i] = 1.0 - lake - reservoir;
        cc[PC_KIRCHNER_ROUTED_PREC * N + i] = reservoir * (1.0 - rdrf) + lake;
        cc[PC_DIRECT_RESPONSE * N + i] = direct;
        cc[PC_KIRCHNER_FRACTION * N + i] = 1 - direct;
        cc[PC_AREA * N + i] = g[3];
        cc[PC_GLACIER_AREA * N + i] = g[3] * glacier;
        cc[PC_ALTITUDE * N + i] = g[2];
        cc[PC_CV2 * N + i] = cv * cv;
        cc[PC_INV_CV2 * N + i] = 1.0 / (cv * cv);
    }
    h->d_params.alloc(P.size());
    h->d_cellc.alloc(cc.size());
    h->d_set_ix.alloc(N);
    hip_check(region_copy(h, h->d_params.p, P.data(), P.size() * sizeof(double), hipMemcpyHostToDevice), "upload params");
    hip_check(region_copy(h, h->d_cellc.p, cc.data(), cc.size() * sizeof(double), hipMemcpyHostToDevice), "upload cellc");
    hip_check(region_copy(h, h->d_set_ix.p, h->set_ix.data(), N * sizeof(int32_t), hipMemcpyHostToDevice), "upload set_ix");
    h->derived_dirty = false;
}

// a pending shyft_hip_prefetch_synthetic_forcing is dropped: its buffer has the old window's shape
void cancel_prefetch(shyft_hip_region* h) {
    if (h->gen_stream) hip_check(hipStreamSynchronize(h->gen_stream), "sync generator");
    h->gen_w0 = SIZE_MAX;
    h->free_pending = false;
    h->d_forcing_next.release();
}

void alloc_window(shyft_hip_region* h) {
    const size_t N = h->n;
    cancel_prefetch(h);
    h->d_forcing.alloc(N_FORCING * h->TW * N);
    hip_check(launch_fill(h->d_forcing.p, h->d_forcing.n, NAN, h->stream), "fill forcing");
    h->d_resp.alloc(h->n_series() * h->TW * N);
    hip_check(launch_fill(h->d_resp.p, h->d_resp.n, NAN, h->stream), "fill resp");
    if (h->collect_state) {
        h->d_state_series.alloc(h->n_state_series() * (h->TW + 1) * N);
        hip_check(launch_fill(h->d_state_series.p, h->d_state_series.n, NAN, h->stream), "fill state series");
    } else {
        h->d_state_series.release();
    }
    hip_check(hipStreamSynchronize(h->stream), "sync");
}

void check_window(const shyft_hip_region* h, size_t step0, size_t n, const char* what) {
    if (step0 < h->w0 || step0 + n > h->w0 + h->TW)
        throw std::runtime_error(std::string(what) + ": steps [" + std::to_string(step0) + "," + std::to_string(step0 + n) +
                                 ") outside the resident window [" + std::to_string(h->w0) + "," +
                                 std::to_string(h->w0 + h->TW) + ")");
}

void copy_rows(hipStream_t s, double* dst, const double* src, size_t bytes, int dst_dev, int src_dev) {
    hipMemcpyKind k = src_dev ? (dst_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost)
                              : (dst_dev ? hipMemcpyHostToDevice : hipMemcpyHostToHost);
    hip_check(hipMemcpyAsync(dst, src, bytes, k, s), "hipMemcpyAsync");
    hip_check(hipStreamSynchronize(s), "sync");
}

// cell_statistics::verify_cids_exist (cell_model.h:198-211) + is_match selection
std::vector<int32_t> select_cells(const shyft_hip_region* h, const int64_t* ids, size_t n_ids, int scope) {
    std::vector<int32_t> sel;
    if (n_ids == 0) {
        sel.resize(h->n);
        for (size_t i = 0; i < h->n; ++i) sel[i] = int32_t(i);
        return sel;
    }
    if (scope == SHYFT_HIP_SCOPE_CELL_IX) {
        for (size_t k = 0; k < n_ids; ++k)
            if (ids[k] < 0 || ids[k] > int64_t(h->n))
                throw std::runtime_error("Supplied cell index reference " + std::to_string(ids[k]) +
                                         " is ouside valid range 0 .." + std::to_string(h->n));
        for (size_t i = 0; i < h->n; ++i)
            for (size_t k = 0; k < n_ids; ++k)
                if (ids[k] == int64_t(i)) { sel.push_back(int32_t(i)); break; }
    } else {
        for (size_t k = 0; k < n_ids; ++k)
            if (h->cid_to_cix.count(ids[k]) == 0)
                throw std::runtime_error("one or more supplied catchment_indexes does not exist:" + std::to_string(ids[k]));
        for (size_t i = 0; i < h->n; ++i)
            for (size_t k = 0; k < n_ids; ++k)
                if (h->cid[i] == ids[k]) { sel.push_back(int32_t(i)); break; }
    }
    return sel;
}

// device rows [step0, step0+n) of a series id (shyft_hip.h: response ids, SHYFT_HIP_SERIES_FORCING + var,
// SHYFT_HIP_SERIES_STATE + field on the T+1 state axis)
const double* series_rows(const shyft_hip_region* h, int series, size_t step0, size_t n, const char* what) {
    const size_t N = h->n;
    if (series >= SHYFT_HIP_SERIES_STATE) {
        const int f = series - SHYFT_HIP_SERIES_STATE;
        if (!h->collect_state || !h->d_state_series.p)
            throw std::runtime_error(std::string(what) + ": state collection is off");
        if (f < 0 || size_t(f) >= h->n_state_series()) throw std::runtime_error(std::string(what) + ": invalid state field");
        if (step0 < h->w0 || step0 + n > h->w0 + h->TW + 1)
            throw std::runtime_error(std::string(what) + ": steps outside the resident window");
        return h->d_state_series.p + (size_t(f) * (h->TW + 1) + (step0 - h->w0)) * N;
    }
    check_window(h, step0, n, what);
    if (series >= SHYFT_HIP_SERIES_FORCING) {
        const int v = series - SHYFT_HIP_SERIES_FORCING;
        if (v < 0 || v >= N_FORCING) throw std::runtime_error(std::string(what) + ": invalid forcing variable");
        return h->d_forcing.p + (size_t(v) * h->TW + (step0 - h->w0)) * N;
    }
    if (series < 0 || size_t(series) >= h->n_series())
        throw std::runtime_error(std::string(what) + ": series not collected in this collection mode");
    return h->d_resp.p + (size_t(series) * h->TW + (step0 - h->w0)) * N;
}

template <class T>
void clone_buf(dbuf<T>& dst, const dbuf<T>& src) {
    dst.release();
    if (!src.p) return;
    dst.alloc(src.n);
    hip_check(hipMemcpy(dst.p, src.p, src.n * sizeof(T), hipMemcpyDeviceToDevice), "clone");
}

}  // namespace

extern "C" {

const char* shyft_hip_last_error(const shyft_hip_region* h) { return h ? h->err.c_str() : g_last_error.c_str(); }

int shyft_hip_region_create(int stack, size_t n_cells, int device, shyft_hip_region** out) {
    if (!out) return fail(nullptr, "shyft_hip_region_create: out is null");
    *out = nullptr;
    if (stack != SHYFT_HIP_PT_GS_K && stack != SHYFT_HIP_HBV_STACK && stack != SHYFT_HIP_PT_SS_K &&
        stack != SHYFT_HIP_PT_HS_K && stack != SHYFT_HIP_PT_HPS_K)
        return fail(nullptr, "shyft_hip_region_create: unsupported method stack");
    if (n_cells == 0 || n_cells > (size_t)INT32_MAX) return fail(nullptr, "shyft_hip_region_create: invalid n_cells");
    std::unique_ptr<shyft_hip_region> h(new shyft_hip_region());
    h->stack = stack;
    h->n = n_cells;
    try {
        if (device < 0) hip_check(hipGetDevice(&device), "hipGetDevice");
        h->device = device;
        hip_check(hipSetDevice(device), "hipSetDevice");
        hip_check(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking), "hipStreamCreate");
        hip_check(hipEventCreate(&h->ev0), "hipEventCreate");
        hip_check(hipEventCreate(&h->ev1), "hipEventCreate");
        hip_check(hipEventCreateWithFlags(&h->ev_copy, hipEventDisableTiming), "hipEventCreate");
        h->d_state.alloc(h->n_state_fields() * n_cells);
        h->d_err.alloc(n_cells);
        h->d_flag.alloc(1);
        hip_check(hipMemset(h->d_err.p, 0, n_cells * sizeof(int32_t)), "memset");
        h->set_ix.assign(n_cells, 0);
    } catch (const std::exception& e) {
        return fail(nullptr, e.what());
    }
    *out = h.release();
    return 0;
}

int shyft_hip_region_create_sharded(int stack, size_t n_cells, const int* devices, size_t n_shards,
                                    shyft_hip_region** out) {
    return shyft_hip_region_create_sharded_ex(stack, n_cells, devices, n_shards, 0u, out);
}

const char* shyft_hip_region_combine_report(const shyft_hip_region* h) {
    return h && h->sh ? shards::combine_report(h->sh) : "";
}

int shyft_hip_region_create_sharded_ex(int stack, size_t n_cells, const int* devices, size_t n_shards, unsigned flags,
                                       shyft_hip_region** out) {
    if (!out) return fail(nullptr, "shyft_hip_region_create_sharded: out is null");
    *out = nullptr;
    if (stack != SHYFT_HIP_PT_GS_K && stack != SHYFT_HIP_HBV_STACK && stack != SHYFT_HIP_PT_SS_K &&
        stack != SHYFT_HIP_PT_HS_K && stack != SHYFT_HIP_PT_HPS_K)
        return fail(nullptr, "shyft_hip_region_create: unsupported method stack");
    if (n_cells == 0 || n_cells > (size_t)INT32_MAX) return fail(nullptr, "shyft_hip_region_create: invalid n_cells");
    try {
        std::unique_ptr<shyft_hip_region> h(new shyft_hip_region());
        h->stack = stack;
        h->n = n_cells;
        h->device = devices && n_shards ? devices[0] : 0;
        h->sh = shard_set_create(stack, n_cells, devices, n_shards, flags);
        *out = h.release();
        return 0;
    } catch (const std::exception& e) {
        return fail(nullptr, e.what());
    }
}

size_t shyft_hip_region_shards(const shyft_hip_region* h, size_t k, int* device, size_t* cell0, size_t* n_cells) {
    if (!h) return 0;
    if (h->sh) return shards::info(h->sh, k, device, cell0, n_cells);
    if (k == 0) {
        if (device) *device = h->device;
        if (cell0) *cell0 = 0;
        if (n_cells) *n_cells = h->n;
    }
    return 1;
}

int shyft_hip_region_combine_path(const shyft_hip_region* h) {
    return h && h->sh ? shards::combine_path(h->sh) : SHYFT_HIP_COMBINE_NONE;
}

void shyft_hip_region_destroy(shyft_hip_region* h) {
    if (!h) return;
    if (h->sh) shard_set_destroy(h->sh);
    if (h->ens) shyft_hip_region_destroy(h->ens);
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->gen_stream) (void)hipStreamSynchronize(h->gen_stream);  // a prefetch may still write d_forcing_next
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->ev_gen) (void)hipEventDestroy(h->ev_gen);
    if (h->ev_free) (void)hipEventDestroy(h->ev_free);
    if (h->gen_stream) (void)hipStreamDestroy(h->gen_stream);
    if (h->ev_copy) (void)hipEventDestroy(h->ev_copy);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

size_t shyft_hip_region_size(const shyft_hip_region* h) { return h ? h->n : 0; }

int shyft_hip_set_geo(shyft_hip_region* h, const double* geo11, const int64_t* routing_id, const double* routing_distance) {
    if (!h || !geo11) return fail(h, "shyft_hip_set_geo: null argument");
    if (h->sh) return guarded(h, [&] { shards::set_geo(h->sh, geo11, routing_id, routing_distance); });
    return guarded(h, [&] {
        for (size_t i = 0; i < h->n; ++i) {
            const double* g = geo11 + i * 11;
            // land_type_fractions::set_fractions validation (geo_cell_data.h:67-79)
            const double sum = g[6] + g[7] + g[8] + g[9];
            if (!(sum > 1.0 && sum < 1.0 + 1.0e-3) && (sum > 1.0 || g[6] < 0 || g[7] < 0 || g[8] < 0 || g[9] < 0))
                throw std::invalid_argument("LandTypeFractions:: must be >=0.0 and sum <= 1.0");
        }
        h->geo.assign(geo11, geo11 + 11 * h->n);
        for (size_t i = 0; i < h->n; ++i) {  // normalise like set_fractions
            double* g = &h->geo[i * 11];
            const double sum = g[6] + g[7] + g[8] + g[9];
            if (sum > 1.0 && sum < 1.0 + 1.0e-3)
                for (int k = 6; k < 10; ++k) g[k] /= sum;
        }
        h->routing_id.assign(h->n, 0);
        h->routing_distance.assign(h->n, 0.0);
        if (routing_id) h->routing_id.assign(routing_id, routing_id + h->n);
        if (routing_distance) h->routing_distance.assign(routing_distance, routing_distance + h->n);
        update_ix_to_id_mapping(h);
        std::vector<double> z(h->n);
        for (size_t i = 0; i < h->n; ++i) z[i] = h->geo[i * 11 + 2];
        h->d_alt.alloc(h->n);
        hip_check(region_copy(h, h->d_alt.p, z.data(), h->n * sizeof(double), hipMemcpyHostToDevice), "upload z");
        h->has_geo = true;
        h->derived_dirty = true;
        h->dst_dirty = true;
        for (auto& t : h->idw) t.key.clear();
    });
}

int shyft_hip_set_parameters(shyft_hip_region* h, const double* params, size_t n_sets, size_t n_per_set,
                             const int32_t* set_ix) {
    if (!h || !params) return fail(h, "shyft_hip_set_parameters: null argument");
    if (h->sh) return guarded(h, [&] { shards::set_parameters(h->sh, params, n_sets, n_per_set, set_ix); });
    return guarded(h, [&] {
        const size_t width = h->param_width();
        if (h->hbv()) {
            if (n_per_set != HBV_NP_REF && n_per_set != HBV_NP)
                throw std::runtime_error("HBV_Stack Parameter Accessor: .set size missmatch");
        } else if (h->ptssk()) {
            if (n_per_set != PTSSK_NP) throw std::runtime_error("pt_ss_k parameter accessor: .set size mismatch");
        } else if (h->pthsk()) {
            if (n_per_set != PTHSK_NP_REF && n_per_set != PTHSK_NP)
                throw std::runtime_error("pt_ss_k parameter accessor: .set size missmatch");  // pt_hs_k.h:68 text
        } else if (h->pthpsk()) {
            if (n_per_set != PTHPSK_NP_REF && n_per_set != PTHPSK_NP)
                throw std::runtime_error("pt_ss_k parameter accessor: .set size missmatch");  // pt_hps_k.h:70 text
        } else if (n_per_set != h->n_ref_params()) {
            throw std::runtime_error("PTGSK Parameter Accessor: .set size missmatch");
        }
        if (n_sets == 0) throw std::runtime_error("shyft_hip_set_parameters: n_sets == 0");
        std::vector<int32_t> ix(h->n, 0);
        if (set_ix) {
            for (size_t i = 0; i < h->n; ++i) {
                if (set_ix[i] < 0 || size_t(set_ix[i]) >= n_sets)
                    throw std::runtime_error("shyft_hip_set_parameters: set index out of range");
                ix[i] = set_ix[i];
            }
        }
        h->params.assign(n_sets * width, 0.0);
        for (size_t k = 0; k < n_sets; ++k) {
            double* q = &h->params[k * width];
            for (size_t j = 0; j < n_per_set; ++j) q[j] = params[k * n_per_set + j];
            const int kd = h->snow_dist_index();  // HK_NB / PH_NB: n_bins, s[HBV_MAX_BINS], intervals[HBV_MAX_BINS]
            if (kd >= 0 && n_per_set == h->n_ref_params()) {
                // hbv_snow::parameter() default distribution: s = 1 (normalised mean of ones is exactly 1),
                // quantiles 0, .25, .5, .75, 1 (hbv_snow.h:29-41)
                static const double I5[5] = {0.0, 0.25, 0.5, 0.75, 1.0};
                q[kd] = 5.0;
                for (int b = 0; b < 5; ++b) {
                    q[kd + 1 + b] = 1.0;
                    q[kd + 1 + HBV_MAX_BINS + b] = I5[b];
                }
            }
            if (kd >= 0) {
                const double nb = q[kd];
                if (!(nb >= 2.0 && nb <= double(HBV_MAX_BINS)) || nb != double(int(nb)))
                    throw std::runtime_error("hbv_snow: number of snow bins must be in [2, " +
                                             std::to_string(HBV_MAX_BINS) + "]");
            }
        }
        h->n_sets = n_sets;
        h->set_ix.swap(ix);
        h->has_params = true;
        h->derived_dirty = true;
    });
}

int shyft_hip_set_time_axis(shyft_hip_region* h, int64_t t0_us, int64_t dt_us, size_t n_steps, size_t window_steps) {
    if (!h) return fail(h, "shyft_hip_set_time_axis: null handle");
    if (h->sh) return guarded(h, [&] { shards::set_time_axis(h->sh, t0_us, dt_us, n_steps, window_steps); });
    return guarded(h, [&] {
        if (dt_us <= 0 || n_steps == 0) throw std::runtime_error("region_model::run with invalid time_axis invoked");
        if (n_steps > (size_t)INT32_MAX) throw std::runtime_error("time axis too long");
        h->t0 = t0_us;
        h->dt = dt_us;
        h->T = n_steps;
        h->w0 = 0;
        h->TW = (window_steps == 0 || window_steps > n_steps) ? n_steps : window_steps;
        std::vector<int32_t> doy(n_steps);
        std::vector<int64_t> trel(n_steps);
        for (size_t i = 0; i < n_steps; ++i) {
            const int64_t t = t0_us + int64_t(i) * dt_us;
            const int64_t days = floor_div(t, DAY_US);
            int64_t y; int m, d;
            civil_from_days(days, y, m, d);
            const int64_t jan1 = days_from_civil(y, 1, 1);
            doy[i] = int32_t(1 + days - jan1);  // calendar::day_of_year
            trel[i] = t - jan1 * DAY_US;        // t - calendar::trim(t, YEAR)
        }
        h->d_doy.alloc(n_steps);
        h->d_trel.alloc(n_steps);
        hip_check(region_copy(h, h->d_doy.p, doy.data(), n_steps * sizeof(int32_t), hipMemcpyHostToDevice), "upload doy");
        hip_check(region_copy(h, h->d_trel.p, trel.data(), n_steps * sizeof(int64_t), hipMemcpyHostToDevice), "upload trel");
        alloc_window(h);
        h->derived_dirty = true;
    });
}

int shyft_hip_set_window(shyft_hip_region* h, size_t w0) { return shyft_hip_move_window(h, w0, 7); }

int shyft_hip_move_window(shyft_hip_region* h, size_t w0, int fill_mask) {
    if (!h) return fail(h, "shyft_hip_set_window: null handle");
    if (h->sh) return guarded(h, [&] { shards::move_window(h->sh, w0, fill_mask); });
    return guarded(h, [&] {
        if (h->T == 0) throw std::runtime_error("set_window: no time axis");
        if (w0 + h->TW > h->T) throw std::runtime_error("set_window: window beyond the time axis");
        h->w0 = w0;
        if (fill_mask & 1) hip_check(launch_fill(h->d_forcing.p, h->d_forcing.n, NAN, h->stream), "fill");
        if (fill_mask & 2) hip_check(launch_fill(h->d_resp.p, h->d_resp.n, NAN, h->stream), "fill");
        if ((fill_mask & 4) && h->d_state_series.p)
            hip_check(launch_fill(h->d_state_series.p, h->d_state_series.n, NAN, h->stream), "fill");
        hip_check(hipStreamSynchronize(h->stream), "sync");
    });
}

int shyft_hip_set_collection(shyft_hip_region* h, int collect, int collect_state) {
    if (!h) return fail(h, "shyft_hip_set_collection: null handle");
    if (h->sh) return guarded(h, [&] { shards::set_collection(h->sh, collect, collect_state); });
    return guarded(h, [&] {
        if (collect < 0 || collect > 2) throw std::runtime_error("set_collection: invalid mode");
        const bool changed = collect != h->collect || (collect_state != 0) != (h->collect_state != 0);
        h->collect = collect;
        h->collect_state = collect_state != 0;
        if (changed && h->TW) {
            const size_t N = h->n;
            h->d_resp.alloc(h->n_series() * h->TW * N);
            hip_check(launch_fill(h->d_resp.p, h->d_resp.n, NAN, h->stream), "fill resp");
            if (h->collect_state) {
                h->d_state_series.alloc(h->n_state_series() * (h->TW + 1) * N);
                hip_check(launch_fill(h->d_state_series.p, h->d_state_series.n, NAN, h->stream), "fill");
            } else {
                h->d_state_series.release();
            }
            hip_check(hipStreamSynchronize(h->stream), "sync");
        }
    });
}

int shyft_hip_set_catchment_filter(shyft_hip_region* h, const int64_t* cids, size_t n) {
    if (!h) return fail(h, "shyft_hip_set_catchment_filter: null handle");
    if (h->sh) return guarded(h, [&] { shards::set_catchment_filter(h->sh, cids, n); });
    return guarded(h, [&] {
        if (n == 0) {
            h->active.clear();
            h->d_active.release();
            return;
        }
        // region_model::set_catchment_calculation_filter (region_model.h:356-370)
        if (n > h->cix_to_cid.size())
            throw std::runtime_error("set_catchment_calculation_filter: supplied list > available catchments");
        for (size_t k = 0; k < n; ++k)
            if (h->cid_to_cix.find(cids[k]) == h->cid_to_cix.end())
                throw std::runtime_error("set_catchment_calculation_filter: no cells have supplied cid");
        std::vector<bool> cf(h->cix_to_cid.size(), false);
        for (size_t k = 0; k < n; ++k) cf[h->cid_to_cix[cids[k]]] = true;
        h->active.assign(h->n, 0);
        for (size_t i = 0; i < h->n; ++i) h->active[i] = cf[h->cix[i]] ? 1 : 0;
        h->d_active.alloc(h->n);
        hip_check(region_copy(h, h->d_active.p, h->active.data(), h->n, hipMemcpyHostToDevice), "upload filter");
    });
}

int shyft_hip_set_state(shyft_hip_region* h, const double* state, size_t n_fields) {
    if (!h || !state) return fail(h, "shyft_hip_set_state: null argument");
    if (h->sh) return guarded(h, [&] { shards::set_state(h->sh, state, n_fields); });
    return guarded(h, [&] {
        if (n_fields != h->n_state_fields()) throw std::runtime_error("set_state: wrong number of state fields");
        const size_t N = h->n;
        std::vector<double> soa(n_fields * N);
        for (size_t i = 0; i < N; ++i)
            for (size_t f = 0; f < n_fields; ++f) soa[f * N + i] = state[i * n_fields + f];
        hip_check(region_copy(h, h->d_state.p, soa.data(), soa.size() * sizeof(double), hipMemcpyHostToDevice), "upload state");
        h->has_state = true;
    });
}

int shyft_hip_copy_state(shyft_hip_region* dst, const shyft_hip_region* src) {
    if (!dst || !src) return fail(dst, "shyft_hip_copy_state: null argument");
    if (dst->sh || src->sh)
        return guarded(dst, [&] {
            if (!dst->sh || !src->sh) throw std::runtime_error("copy_state: one region is sharded, the other is not");
            shards::copy_state(dst->sh, src->sh);
        });
    return guarded(dst, [&] {
        if (src->stack != dst->stack || src->n != dst->n)
            throw std::runtime_error("copy_state: regions differ in method stack or number of cells");
        if (!src->has_state) throw std::runtime_error("copy_state: source region has no state");
        // ordered after everything already queued on the source stream; the copy itself runs on the
        // destination stream, so the destination's next run starts after it without a host wait
        hip_check(hipStreamSynchronize(src->stream), "copy_state: source stream");
        hip_check(hipMemcpyAsync(dst->d_state.p, src->d_state.p, dst->n_state_fields() * dst->n * sizeof(double),
                                 hipMemcpyDeviceToDevice, dst->stream), "copy_state");
        // anything later queued on the source stream (a run, set_state's upload) must not overwrite the source
        // state while the destination stream still reads it
        // (set_state / get_state copy on the region stream too, region_copy). The event lives on the source
        // region's device; a copy between two devices completes before returning instead.
        shyft_hip_region* s = const_cast<shyft_hip_region*>(src);
        if (src->device == dst->device) {
            hip_check(hipEventRecord(s->ev_copy, dst->stream), "copy_state: record");
            hip_check(hipStreamWaitEvent(s->stream, s->ev_copy, 0), "copy_state: order source stream");
        } else {
            hip_check(hipStreamSynchronize(dst->stream), "copy_state: cross-device copy");
        }
        dst->has_state = true;
    });
}

int shyft_hip_get_state(const shyft_hip_region* hc, double* state, size_t n_fields) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !state) return fail(h, "shyft_hip_get_state: null argument");
    if (h->sh) return guarded(h, [&] { shards::get_state(h->sh, state, n_fields); });
    return guarded(h, [&] {
        if (n_fields != h->n_state_fields()) throw std::runtime_error("get_state: wrong number of state fields");
        const size_t N = h->n;
        std::vector<double> soa(n_fields * N);
        hip_check(region_copy(h, soa.data(), h->d_state.p, soa.size() * sizeof(double), hipMemcpyDeviceToHost), "download state");
        for (size_t i = 0; i < N; ++i)
            for (size_t f = 0; f < n_fields; ++f) state[i * n_fields + f] = soa[f * N + i];
    });
}

int shyft_hip_set_forcing(shyft_hip_region* h, int var, size_t step0, size_t n, const double* src, int src_on_device) {
    if (!h || !src) return fail(h, "shyft_hip_set_forcing: null argument");
    if (h->sh) return guarded(h, [&] { shards::set_forcing(h->sh, var, step0, n, src, src_on_device); });
    return guarded(h, [&] {
        if (var < 0 || var >= N_FORCING) throw std::runtime_error("set_forcing: invalid variable");
        check_window(h, step0, n, "set_forcing");
        double* dst = h->d_forcing.p + (size_t(var) * h->TW + (step0 - h->w0)) * h->n;
        copy_rows(h->stream, dst, src, n * h->n * sizeof(double), 1, src_on_device);
    });
}

int shyft_hip_get_forcing(const shyft_hip_region* hc, int var, size_t step0, size_t n, double* dst, int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_get_forcing: null argument");
    if (h->sh) return guarded(h, [&] { shards::get_rows(h->sh, 0, var, step0, n, dst, dst_on_device); });
    return guarded(h, [&] {
        if (var < 0 || var >= N_FORCING) throw std::runtime_error("get_forcing: invalid variable");
        check_window(h, step0, n, "get_forcing");
        const double* src = h->d_forcing.p + (size_t(var) * h->TW + (step0 - h->w0)) * h->n;
        copy_rows(h->stream, dst, src, n * h->n * sizeof(double), dst_on_device, 1);
    });
}

int shyft_hip_synthetic_forcing(shyft_hip_region* h, uint64_t seed, uint64_t cell_offset, size_t step0, size_t n) {
    if (!h) return fail(h, "shyft_hip_synthetic_forcing: null handle");
    if (h->sh) return guarded(h, [&] { shards::synthetic_forcing(h->sh, seed, cell_offset, step0, n); });
    return guarded(h, [&] {
        check_window(h, step0, n, "synthetic_forcing");
        if (!h->has_geo) throw std::runtime_error("synthetic_forcing: geo_cell_data not set");
        const double* z = h->d_alt.p;
        hip_check(launch_synthetic_forcing(h->d_forcing.p, h->TW, step0 - h->w0, n, h->n, seed, cell_offset, step0, z,
                                           h->stream, h->d_cell_ids.p),
                  "synthetic_forcing");
        hip_check(hipStreamSynchronize(h->stream), "sync");
    });
}

int shyft_hip_prefetch_synthetic_forcing(shyft_hip_region* h, uint64_t seed, uint64_t cell_offset, size_t w0_next,
                                         int n_cus) {
    if (!h) return fail(h, "shyft_hip_prefetch_synthetic_forcing: null handle");
    if (h->sh) return guarded(h, [&] { shards::prefetch_synthetic_forcing(h->sh, seed, cell_offset, w0_next, n_cus); });
    return guarded(h, [&] {
        if (h->T == 0 || h->TW == 0) throw std::runtime_error("prefetch_synthetic_forcing: no time axis");
        if (w0_next + h->TW > h->T) throw std::runtime_error("prefetch_synthetic_forcing: window beyond the time axis");
        if (!h->has_geo) throw std::runtime_error("prefetch_synthetic_forcing: geo_cell_data not set");
        if (h->gen_w0 != SIZE_MAX) throw std::runtime_error("prefetch_synthetic_forcing: a prefetched window is pending");
        if (!h->gen_stream || h->gen_cus != n_cus) {
            if (h->gen_stream) {
                hip_check(hipStreamSynchronize(h->gen_stream), "sync");
                hip_check(hipStreamDestroy(h->gen_stream), "hipStreamDestroy");
                h->gen_stream = nullptr;
            }
            int total = 0;
            hip_check(hipDeviceGetAttribute(&total, hipDeviceAttributeMultiprocessorCount, h->device), "CU count");
            if (n_cus > 0 && n_cus < total) {
                // n_cus CUs spread evenly over the device (every XCD keeps most of its CUs for the run kernel)
                std::vector<uint32_t> mask((size_t(total) + 31) / 32, 0u);
                for (int k = 0; k < n_cus; ++k) {
                    const int cu = int((long long)k * total / n_cus);
                    mask[size_t(cu) / 32] |= 1u << (cu % 32);
                }
                hip_check(hipExtStreamCreateWithCUMask(&h->gen_stream, uint32_t(mask.size()), mask.data()),
                          "hipExtStreamCreateWithCUMask");
            } else if (n_cus < 0) {
                // the whole device at the lowest stream priority: the run kernel's workgroups (normal priority,
                // launched first) are dispatched before the generator's, which fill the CUs its tail leaves idle
                int least = 0, greatest = 0;
                hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
                hip_check(hipStreamCreateWithPriority(&h->gen_stream, hipStreamNonBlocking, least),
                          "hipStreamCreateWithPriority");
            } else {
                hip_check(hipStreamCreateWithFlags(&h->gen_stream, hipStreamNonBlocking), "hipStreamCreate");
            }
            h->gen_cus = n_cus;
        }
        if (!h->ev_gen) hip_check(hipEventCreateWithFlags(&h->ev_gen, hipEventDisableTiming), "hipEventCreate");
        h->d_forcing_next.alloc(h->d_forcing.n);
        // the buffer was last read by a run on the region stream: the generator waits for that run -- the event the
        // last swap recorded behind it, or else everything on the region stream so far
        if (h->free_pending) {
            hip_check(hipStreamWaitEvent(h->gen_stream, h->ev_free, 0), "wait");
        } else {
            hip_check(hipEventRecord(h->ev_gen, h->stream), "record");
            hip_check(hipStreamWaitEvent(h->gen_stream, h->ev_gen, 0), "wait");
        }
        const int blocks = 4 * (n_cus > 0 ? n_cus : 256);  // 4 workgroups of 4 waves per CU (grid-stride over cells)
        hip_check(launch_synthetic_forcing_stream(h->d_forcing_next.p, h->TW, 0, h->TW, h->n, seed, cell_offset,
                                                  w0_next, h->d_alt.p, blocks, h->gen_stream, h->d_cell_ids.p),
                  "synthetic_forcing (prefetch)");
        hip_check(hipEventRecord(h->ev_gen, h->gen_stream), "record");
        h->gen_w0 = w0_next;
    });
}

int shyft_hip_swap_forcing_window(shyft_hip_region* h, size_t w0_next) {
    if (!h) return fail(h, "shyft_hip_swap_forcing_window: null handle");
    if (h->sh) return guarded(h, [&] { shards::swap_forcing_window(h->sh, w0_next); });
    return guarded(h, [&] {
        if (h->gen_w0 != w0_next) throw std::runtime_error("swap_forcing_window: no prefetched window at this step");
        if (h->d_forcing_next.n != h->d_forcing.n || w0_next + h->TW > h->T)
            throw std::runtime_error("swap_forcing_window: the prefetched window does not match the region's window");
        // the response / state-series rows still hold the previous window's values (no NaN fill, unlike
        // set_window): the run that follows the swap rewrites them, and reading them before it is the caller's
        // error (shyft_hip.h)
        // later work on the region stream (the next run) waits for the generator, without a host wait
        hip_check(hipStreamWaitEvent(h->stream, h->ev_gen, 0), "wait generator");
        // the buffer swapped out was read by the runs enqueued so far: the next prefetch into it waits for them only
        // (not for the run enqueued after this swap, which reads the other buffer)
        if (!h->ev_free) hip_check(hipEventCreateWithFlags(&h->ev_free, hipEventDisableTiming), "hipEventCreate");
        hip_check(hipEventRecord(h->ev_free, h->stream), "record");
        h->free_pending = true;
        std::swap(h->d_forcing.p, h->d_forcing_next.p);
        std::swap(h->d_forcing.n, h->d_forcing_next.n);
        h->w0 = w0_next;
        h->gen_w0 = SIZE_MAX;
    });
}

int shyft_hip_interpolate(shyft_hip_region* h, int var, size_t n_sources, const double* src_xyz, const double* src_values,
                          size_t step0, size_t n, const double* idw_param) {
    if (!h || !src_xyz || !src_values || !idw_param) return fail(h, "shyft_hip_interpolate: null argument");
    if (h->sh) return guarded(h, [&] { shards::interpolate(h->sh, var, n_sources, src_xyz, src_values, step0, n, idw_param); });
    return guarded(h, [&] {
        if (var < 0 || var >= N_FORCING) throw std::runtime_error("interpolate: invalid variable");
        if (!h->has_geo) throw std::runtime_error("interpolate: geo_cell_data not set");
        if (n_sources == 0) throw std::runtime_error("interpolate: no sources");
        check_window(h, step0, n, "interpolate");
        const size_t N = h->n;
        double* out = h->d_forcing.p + (size_t(var) * h->TW + (step0 - h->w0)) * N;
        const uint8_t* active = h->active.empty() ? nullptr : h->d_active.p;
        h->d_src_vals.alloc(std::max(h->d_src_vals.n, n * n_sources));
        hip_check(hipMemcpyAsync(h->d_src_vals.p, src_values, n * n_sources * sizeof(double), hipMemcpyHostToDevice,
                                 h->stream),
                  "upload source values");
        if (var == FV_TEMPERATURE && n_sources == 1) {
            // one temperature source: copied to the cells (region_model.h:470-481)
            hip_check(launch_copy_source(h->d_src_vals.p, int(n), int(N), active, out, h->stream), "copy_source");
            hip_check(hipStreamSynchronize(h->stream), "sync");
            h->idw[var].last_path = SHYFT_HIP_IDW_COPY;
            return;
        }
        static const int kind_of_var[N_FORCING] = {IDW_TEMPERATURE, IDW_PRECIPITATION, IDW_WIND_SPEED, IDW_REL_HUM,
                                                    IDW_RADIATION};
        const int kind = kind_of_var[var];
        const int K = int(idw_param[0]);
        if (K < 1 || K > IDW_KMAX)
            throw std::runtime_error("interpolate: max_members must be in [1, " + std::to_string(IDW_KMAX) + "]");
        if (h->dst_dirty) {
            std::vector<double> xyz(3 * N), slope(N);
            for (size_t i = 0; i < N; ++i) {
                for (int k = 0; k < 3; ++k) xyz[3 * i + k] = h->geo[i * 11 + k];
                slope[i] = h->geo[i * 11 + 5];
            }
            h->d_dst_xyz.alloc(3 * N);
            h->d_slope.alloc(N);
            hip_check(region_copy(h, h->d_dst_xyz.p, xyz.data(), 3 * N * sizeof(double), hipMemcpyHostToDevice), "upload dst");
            hip_check(region_copy(h, h->d_slope.p, slope.data(), N * sizeof(double), hipMemcpyHostToDevice), "upload slope");
            h->dst_dirty = false;
        }
        auto& tab = h->idw[var];
        std::vector<double> key = {double(kind), double(n_sources), idw_param[0], idw_param[1], idw_param[2],
                                   idw_param[3], idw_param[6]};
        key.insert(key.end(), src_xyz, src_xyz + 3 * n_sources);
        h->d_src_xyz.alloc(std::max(h->d_src_xyz.n, 3 * n_sources));
        hip_check(hipMemcpyAsync(h->d_src_xyz.p, src_xyz, 3 * n_sources * sizeof(double), hipMemcpyHostToDevice, h->stream),
                  "upload source xyz");
        if (key != tab.key) {
            tab.idx.alloc(size_t(K) * N);
            tab.w.alloc(size_t(K) * N);
            tab.aux.alloc(size_t(K) * N);
            tab.cnt.alloc(N);
            tab.K = K;
            idw_nb_args nb;
            nb.n_cells = int(N);
            nb.n_sources = int(n_sources);
            nb.kind = kind;
            nb.max_members = K;
            nb.max_distance = idw_param[1];
            nb.distance_measure_factor = idw_param[2];
            nb.zscale = idw_param[3];
            nb.scale_factor = idw_param[6];
            nb.src_xyz = h->d_src_xyz.p;
            nb.dst_xyz = h->d_dst_xyz.p;
            nb.idx = tab.idx.p;
            nb.w = tab.w.p;
            nb.aux = tab.aux.p;
            nb.count = tab.cnt.p;
            hip_check(launch_idw_neighbours(nb, h->stream), "idw_neighbours");
            // each wavefront's union of neighbour stations (the gather's compacted path when every union fits 64)
            const size_t n_waves = (N + 63) / 64;
            tab.wu.alloc(n_waves * 64);
            tab.wn.alloc(n_waves);
            tab.lidx.alloc(size_t((K + 3) / 4) * N);
            tab.ovf.alloc(1);
            hip_check(hipMemsetAsync(tab.ovf.p, 0, sizeof(int32_t), h->stream), "memset overflow");
            idw_union_args ua;
            ua.n_cells = int(N);
            ua.max_members = K;
            ua.idx = tab.idx.p;
            ua.count = tab.cnt.p;
            ua.wu = tab.wu.p;
            ua.wn = tab.wn.p;
            ua.lidx = tab.lidx.p;
            ua.overflow = tab.ovf.p;
            hip_check(launch_idw_wave_union(ua, h->stream), "idw_wave_union");
            int32_t ovf = 1;
            hip_check(region_copy(h, &ovf, tab.ovf.p, sizeof(int32_t), hipMemcpyDeviceToHost), "read overflow");
            tab.wave_ok = ovf == 0;
            tab.key.swap(key);
        }
        idw_gather_args g;
        g.n_cells = int(N);
        g.n_sources = int(n_sources);
        g.n_rows = int(n);
        g.kind = kind;
        g.by_equation = idw_param[5] != 0.0;
        g.max_members = tab.K;
        g.default_gradient = idw_param[4];
        g.src_xyz = h->d_src_xyz.p;
        g.src_values = h->d_src_vals.p;
        g.dst_xyz = h->d_dst_xyz.p;
        g.slope = h->d_slope.p;
        g.idx = tab.idx.p;
        g.w = tab.w.p;
        g.aux = tab.aux.p;
        g.count = tab.cnt.p;
        g.active = active;
        g.out = out;
        // SHYFT_IDW_TILE=1: the row-tile gather even where the wavefront unions fit (tests cover both paths)
        const bool wave = tab.wave_ok && !getenv("SHYFT_IDW_TILE");
        g.wu = wave ? tab.wu.p : nullptr;
        g.wn = wave ? tab.wn.p : nullptr;
        g.lidx = wave ? tab.lidx.p : nullptr;
        hip_check(hipEventRecord(h->ev0, h->stream), "hipEventRecord");
        hip_check(launch_idw_gather(g, h->stream), "idw_gather");
        hip_check(hipEventRecord(h->ev1, h->stream), "hipEventRecord");
        hip_check(hipStreamSynchronize(h->stream), "idw");
        float ms = 0.0f;
        hip_check(hipEventElapsedTime(&ms, h->ev0, h->ev1), "hipEventElapsedTime");
        h->last_interp_ms = ms;
        tab.last_path = wave ? SHYFT_HIP_IDW_WAVE : SHYFT_HIP_IDW_TILE;
    });
}

int shyft_hip_interpolation_path(const shyft_hip_region* h, int var) {
    if (!h || var < 0 || var >= N_FORCING) return -1;
    if (h->sh) return shards::interpolation_path(h->sh, var);
    return h->idw[var].last_path;
}

namespace {
void check_btk_param(const double* p) {
    if (!(p[0] > 0.0) || !std::isfinite(p[0])) throw std::runtime_error("btk: temperature_gradient_sd must be > 0");
    if (!(p[3] > 0.0)) throw std::runtime_error("btk: range must be > 0");
}
}  // namespace

int shyft_hip_interpolate_btk(shyft_hip_region* h, size_t n_sources, const double* src_xyz, const double* src_values,
                              size_t step0, size_t n, const double* prior_gradient, const double* btk_param) {
    if (!h || !src_xyz || !src_values || !btk_param) return fail(h, "shyft_hip_interpolate_btk: null argument");
    if (h->sh) return guarded(h, [&] { shards::interpolate_btk(h->sh, n_sources, src_xyz, src_values, step0, n, prior_gradient, btk_param); });
    return guarded(h, [&] {
        if (!h->has_geo) throw std::runtime_error("interpolate: geo_cell_data not set");
        if (n_sources == 0) throw std::runtime_error("interpolate: no sources");
        check_window(h, step0, n, "interpolate_btk");
        check_btk_param(btk_param);
        const size_t N = h->n;
        double* out = h->d_forcing.p + (size_t(FV_TEMPERATURE) * h->TW + (step0 - h->w0)) * N;
        if (n_sources == 1) {  // one temperature source: copied to the cells (region_model.h:470-481)
            const uint8_t* active = h->active.empty() ? nullptr : h->d_active.p;
            h->d_src_vals.alloc(std::max(h->d_src_vals.n, n));
            hip_check(hipMemcpyAsync(h->d_src_vals.p, src_values, n * sizeof(double), hipMemcpyHostToDevice, h->stream),
                      "upload source values");
            hip_check(launch_copy_source(h->d_src_vals.p, int(n), int(N), active, out, h->stream), "copy_source");
            hip_check(hipStreamSynchronize(h->stream), "sync");
            return;
        }
        std::vector<double> prior;
        if (!prior_gradient) {
            prior.resize(n);
            for (size_t i = 0; i < n; ++i) prior[i] = btk_prior_gradient(h->t0 + int64_t(step0 + i) * h->dt, h->dt);
            prior_gradient = prior.data();
        }
        // destinations: the calculated cells (region_model.h:420-423), written in place of the window
        std::vector<double> xyz;
        std::vector<int32_t> index;
        xyz.reserve(3 * N);
        for (size_t i = 0; i < N; ++i) {
            if (!h->active.empty() && !h->active[i]) continue;
            for (int k = 0; k < 3; ++k) xyz.push_back(h->geo[i * 11 + k]);
            index.push_back(int32_t(i));
        }
        const size_t D = index.size();
        if (D == 0) return;
        const bool all = D == N;
        if (xyz != h->btk_xyz_host || index != h->btk_index_host || h->btk_dst_version == 0) {
            h->d_btk_xyz.alloc(3 * D);
            hip_check(region_copy(h, h->d_btk_xyz.p, xyz.data(), 3 * D * sizeof(double), hipMemcpyHostToDevice),
                      "upload btk destinations");
            if (!all) {
                h->d_btk_index.alloc(D);
                hip_check(region_copy(h, h->d_btk_index.p, index.data(), D * sizeof(int32_t), hipMemcpyHostToDevice),
                          "upload btk index");
            }
            h->btk_xyz_host.swap(xyz);
            h->btk_index_host.swap(index);
            ++h->btk_dst_version;
        }
        if (!h->btk) h->btk.reset(btk_cache_create());
        btk_args a{};
        a.cache = h->btk.get();
        a.dst_version = h->btk_dst_version;
        a.n_sources = n_sources;
        a.src_xyz = src_xyz;
        a.src_values = src_values;
        a.n_steps = n;
        a.prior_gradient = prior_gradient;
        a.gradient_sd = btk_param[0];
        a.sill = btk_param[1];
        a.nug = btk_param[2];
        a.range = btk_param[3];
        a.zscale = btk_param[4];
        a.n_dst = D;
        a.d_dst_xyz = h->d_btk_xyz.p;
        a.d_dst_index = all ? nullptr : h->d_btk_index.p;
        a.d_out = out;
        a.ld_out = N;
        btk_run(a, h->stream);
        hip_check(hipStreamSynchronize(h->stream), "btk");
    });
}

int shyft_hip_btk(int device, size_t n_sources, const double* src_xyz, const double* src_values, size_t n,
                  const double* prior_gradient, const double* btk_param, size_t n_dst, const double* dst_xyz,
                  double* out) {
    if (!src_xyz || !src_values || !prior_gradient || !btk_param || !dst_xyz || !out)
        return fail(nullptr, "shyft_hip_btk: null argument");
    try {
        if (n_sources == 0) throw std::runtime_error("bayesian_kriging_temperature: no sources");
        check_btk_param(btk_param);
        if (n == 0 || n_dst == 0) return 0;
        if (n_sources == 1) {  // api_interpolation.cpp:63-69: a clean copy to the destinations
            for (size_t t = 0; t < n; ++t)
                for (size_t d = 0; d < n_dst; ++d) out[t * n_dst + d] = src_values[t];
            return 0;
        }
        if (device >= 0) hip_check(hipSetDevice(device), "hipSetDevice");
        hipStream_t s = nullptr;
        hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
        std::unique_ptr<std::remove_pointer<hipStream_t>::type, void (*)(hipStream_t)> stream(
            s, [](hipStream_t x) { (void)hipStreamDestroy(x); });
        dbuf<double> d_xyz, d_out;
        d_xyz.alloc(3 * n_dst);
        d_out.alloc(n * n_dst);
        hip_check(hipMemcpyAsync(d_xyz.p, dst_xyz, 3 * n_dst * sizeof(double), hipMemcpyHostToDevice, s), "upload");
        btk_args a{};
        a.n_sources = n_sources;
        a.src_xyz = src_xyz;
        a.src_values = src_values;
        a.n_steps = n;
        a.prior_gradient = prior_gradient;
        a.gradient_sd = btk_param[0];
        a.sill = btk_param[1];
        a.nug = btk_param[2];
        a.range = btk_param[3];
        a.zscale = btk_param[4];
        a.n_dst = n_dst;
        a.d_dst_xyz = d_xyz.p;
        a.d_dst_index = nullptr;
        a.d_out = d_out.p;
        a.ld_out = n_dst;
        btk_run(a, s);
        hip_check(hipMemcpyAsync(out, d_out.p, n * n_dst * sizeof(double), hipMemcpyDeviceToHost, s), "download");
        hip_check(hipStreamSynchronize(s), "sync");
        return 0;
    } catch (const std::exception& e) {
        return fail(nullptr, e.what());
    }
}

int shyft_hip_synthetic_elevation(uint64_t seed, uint64_t cell_offset, size_t n_cells, double* z_host) {
    if (!z_host) return fail(nullptr, "shyft_hip_synthetic_elevation: null argument");
    for (size_t i = 0; i < n_cells; ++i) z_host[i] = synth_elevation(seed, cell_offset + i);
    return 0;
}

static void launch_run(shyft_hip_region* h, int start_step, int n_steps) {
    update_derived(h);
    size_t b = n_steps > 0 ? size_t(start_step) : 0;
    size_t e = n_steps > 0 ? size_t(start_step + n_steps) : h->T;
    check_window(h, b, e - b, "run_cells");
    if (h->ptssk() || h->pthsk() || h->pthpsk()) {
        ptssk_kargs a;
        a.n_cells = int(h->n);
        a.step0 = int(b);
        a.n_steps = int(e - b);
        a.win0 = int(h->w0);
        a.win_len = int(h->TW);
        a.collect = h->collect;
        const double dt_s = double(h->dt) / 1e6;  // to_seconds(period.timespan())
        a.step_in_days = dt_s / 86400.0;
        a.dt_hours = dt_s / 3600.0;
        a.t1_hours = dt_s / 3600.0;
        a.dt_us = double(h->dt);
        a.params = h->d_params.p;
        a.set_ix = h->d_set_ix.p;
        a.cellc = h->d_cellc.p;
        a.state = h->d_state.p;
        a.forcing = h->forcing_src ? h->forcing_src->d_forcing.p : h->d_forcing.p;
        a.fcol = h->forcing_src ? h->d_fcol.p : nullptr;
        a.f_cols = int(h->forcing_src ? h->forcing_src->n : h->n);
        a.resp = h->d_resp.p;
        a.state_series = h->collect_state ? h->d_state_series.p : nullptr;
        a.active = h->active.empty() ? nullptr : h->d_active.p;
        a.err = h->d_err.p;
        a.uniform_params = h->n_sets == 1 ? 1 : 0;
        a.nb_max = HBV_MAX_BINS;
        if (h->pthsk()) {
            a.nb_max = 0;
            for (size_t k = 0; k < h->n_sets; ++k) a.nb_max = std::max(a.nb_max, int(h->params[k * PTHSK_NP + PH_NB]));
        }
        hip_check(hipEventRecord(h->ev0, h->stream), "hipEventRecord");
        if (h->pthpsk())
            hip_check(launch_pthpsk_run(a, h->stream), "pthpsk_run_kernel launch");
        else if (h->pthsk())
            hip_check(launch_pthsk_run(a, h->stream), "pthsk_run_kernel launch");
        else
            hip_check(launch_ptssk_run(a, h->stream), "ptssk_run_kernel launch");
        hip_check(hipEventRecord(h->ev1, h->stream), "hipEventRecord");
        return;
    }
    if (h->hbv()) {
        hbv_kargs a;
        a.n_cells = int(h->n);
        a.step0 = int(b);
        a.n_steps = int(e - b);
        a.win0 = int(h->w0);
        a.win_len = int(h->TW);
        a.collect = h->collect;
        const double dt_s = double(h->dt) / 1e6;  // to_seconds(t1 - t0)
        a.step_in_days = dt_s / 86400.0;
        a.dt_hours = dt_s / 3600.0;
        a.params = h->d_params.p;
        a.set_ix = h->d_set_ix.p;
        a.cellc = h->d_cellc.p;
        a.state = h->d_state.p;
        a.forcing = h->forcing_src ? h->forcing_src->d_forcing.p : h->d_forcing.p;
        a.fcol = h->forcing_src ? h->d_fcol.p : nullptr;
        a.f_cols = int(h->forcing_src ? h->forcing_src->n : h->n);
        a.resp = h->d_resp.p;
        a.state_series = h->collect_state ? h->d_state_series.p : nullptr;
        a.active = h->active.empty() ? nullptr : h->d_active.p;
        a.err = h->d_err.p;
        a.uniform_params = h->n_sets == 1 ? 1 : 0;
        a.nb_max = 0;
        for (size_t k = 0; k < h->n_sets; ++k) {
            const int nb = int(h->params[k * HBV_NP + HK_NB]);
            if (nb > a.nb_max) a.nb_max = nb;
        }
        hip_check(hipEventRecord(h->ev0, h->stream), "hipEventRecord");
        hip_check(launch_hbv_run(a, h->stream), "hbv_run_kernel launch");
        hip_check(hipEventRecord(h->ev1, h->stream), "hipEventRecord");
        return;
    }
    ptgsk_kargs a;
    a.n_cells = int(h->n);
    a.step0 = int(b);
    a.n_steps = int(e - b);
    a.win0 = int(h->w0);
    a.win_len = int(h->TW);
    a.collect = h->collect;
    a.uniform_params = h->n_sets == 1 ? 1 : 0;
    a.dt_s = double(h->dt) / 1e6;
    a.dt_us = double(h->dt);
    a.t1_hours = a.dt_s / 3600.0;  // to_seconds(T1-T0)/to_seconds(deltahours(1))
    a.doy = h->d_doy.p;
    a.t_rel_year_us = h->d_trel.p;
    a.params = h->d_params.p;
    a.set_ix = h->d_set_ix.p;
    a.cellc = h->d_cellc.p;
    a.state = h->d_state.p;
    a.forcing = h->forcing_src ? h->forcing_src->d_forcing.p : h->d_forcing.p;
    a.fcol = h->forcing_src ? h->d_fcol.p : nullptr;
    a.f_cols = int(h->forcing_src ? h->forcing_src->n : h->n);
    a.resp = h->d_resp.p;
    a.state_series = h->collect_state ? h->d_state_series.p : nullptr;
    a.active = h->active.empty() ? nullptr : h->d_active.p;
    a.err = h->d_err.p;
    a.instance = h->knob_instance;
    a.read_delay = h->knob_read_delay;
    hip_check(hipEventRecord(h->ev0, h->stream), "hipEventRecord");
    hip_check(launch_ptgsk_run(a, h->stream), "ptgsk_run_kernel launch");
    hip_check(hipEventRecord(h->ev1, h->stream), "hipEventRecord");
}

static void finish_run(shyft_hip_region* h) {
    hip_check(hipStreamSynchronize(h->stream), h->hbv() ? "hbv_run_kernel"
                                               : h->ptssk() ? "ptssk_run_kernel"
                                               : h->pthsk() ? "pthsk_run_kernel"
                                               : h->pthpsk() ? "pthpsk_run_kernel" : "ptgsk_run_kernel");
    float ms = 0.f;
    hip_check(hipEventElapsedTime(&ms, h->ev0, h->ev1), "hipEventElapsedTime");
    h->last_ms = ms;
    // the per-cell error codes stay on the device: one reduction to the lowest failing cell, 8 bytes back
    const int32_t none = INT32_MAX;
    hip_check(hipMemcpyAsync(h->d_flag.p, &none, sizeof(int32_t), hipMemcpyHostToDevice, h->stream), "upload flag");
    hip_check(launch_first_error(h->d_err.p, h->n, h->d_flag.p, h->stream), "first_error");
    int32_t first = none;
    hip_check(hipMemcpyAsync(&first, h->d_flag.p, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream), "download flag");
    hip_check(hipStreamSynchronize(h->stream), "first_error");
    if (first == none) return;
    const size_t i = size_t(first);
    int32_t code = 0;
    hip_check(region_copy(h, &code, h->d_err.p + i, sizeof(int32_t), hipMemcpyDeviceToHost), "download err");
    hip_check(hipMemsetAsync(h->d_err.p, 0, h->n * sizeof(int32_t), h->stream), "memset");
    hip_check(hipStreamSynchronize(h->stream), "memset");
    if (code == ERR_NEGATIVE_OUTFLOW)
        throw std::runtime_error("Negative outflow: total_water - swe < -1e-6 in hbv_snow (cell " + std::to_string(i) + ")");
    if (code == ERR_SKAUGEN_BISECT)
        throw std::runtime_error("No change of sign in boost::math::tools::bisect, either there is no root to "
                                 "find, or there are multiple roots in the interval (skaugen sca_rel_red, cell " +
                                 std::to_string(i) + ")");
    if (code == ERR_SKAUGEN_PDF)
        throw std::runtime_error("boost::math::pdf(gamma_distribution): overflow at x = 0 (skaugen sca_rel_red, "
                                 "cell " + std::to_string(i) + ")");
    throw std::runtime_error("kirchner: Max number of iterations exceeded (500). A new step size was not found. (cell " +
                             std::to_string(i) + ")");
}

// argument checks of region_model::run_cells (region_model.h:579-592), shared by the synchronous and the
// asynchronous entry
static void check_run_args(const shyft_hip_region* h, size_t use_ncore, int start_step, int n_steps) {
    // the reference's ncore is the host's hardware_concurrency (region_model.h:280); its "reasonable minimum" of 4
    // is substituted only on the use_ncore == 0 branch (region_model.h:579-584), so with ncore == 0 any
    // use_ncore > 0 is rejected, as there
    const size_t ncore = std::thread::hardware_concurrency();
    if (use_ncore != 0 && use_ncore > 100 * ncore)
        throw std::runtime_error("illegal parameter value: use_ncore(" + std::to_string(use_ncore) +
                                 " is more than 100 time available physical cores: " + std::to_string(ncore));
    if (!(h->T > 0)) throw std::runtime_error("region_model::run with invalid time_axis invoked");
    if (start_step < 0 || size_t(start_step + 1) > h->T)
        throw std::runtime_error("region_model::run start_step must in range[0..n_steps-1>");
    if (n_steps < 0) throw std::runtime_error("region_model::run n_steps must be range[0..time-axis-steps]");
    if (size_t(start_step + n_steps) > h->T)
        throw std::runtime_error("region_model::run start_step+n_steps must be within time-axis range");
    if (!h->has_state) throw std::runtime_error("region_model::run: no state set");
}

int shyft_hip_run_cells(shyft_hip_region* h, size_t use_ncore, int start_step, int n_steps) {
    if (!h) return fail(h, "shyft_hip_run_cells: null handle");
    if (h->sh) return guarded(h, [&] { shards::run_cells(h->sh, use_ncore, start_step, n_steps); });
    return guarded(h, [&] {
        check_run_args(h, use_ncore, start_step, n_steps);
        launch_run(h, start_step, n_steps);
        finish_run(h);
    });
}

int shyft_hip_run_cells_async(shyft_hip_region* h, int start_step, int n_steps) {
    if (!h) return fail(h, "shyft_hip_run_cells_async: null handle");
    if (h->sh) return guarded(h, [&] { shards::run_cells_async(h->sh, start_step, n_steps); });
    return guarded(h, [&] {
        check_run_args(h, 0, start_step, n_steps);
        launch_run(h, start_step, n_steps);
    });
}

int shyft_hip_synchronize(shyft_hip_region* h) {
    if (!h) return fail(h, "shyft_hip_synchronize: null handle");
    if (h->sh) return guarded(h, [&] { shards::synchronize(h->sh); });
    return guarded(h, [&] { finish_run(h); });
}

double shyft_hip_last_run_ms(const shyft_hip_region* h) { return h ? (h->sh ? shards::last_run_ms(h->sh) : h->last_ms) : 0.0; }
double shyft_hip_last_interpolate_ms(const shyft_hip_region* h) {
    return h ? (h->sh ? shards::last_interpolate_ms(h->sh) : h->last_interp_ms) : 0.0;
}

size_t shyft_hip_shard_run_ms(const shyft_hip_region* h, double* ms, size_t n) {
    if (!h) return 0;
    if (h->sh) return shards::shard_run_ms(h->sh, ms, n);
    if (n > 0 && ms) ms[0] = h->last_ms;
    return 1;
}

int shyft_hip_last_run_kernel_ms(const shyft_hip_region* h, double* ms, int n) {
    if (!h) return 0;
    if (h->sh) return shards::last_run_kernel_ms(h->sh, ms, n);
    if (n > 0) ms[0] = h->last_ms;  // every stack runs one kernel per run_cells
    return 1;
}

int shyft_hip_get_series(const shyft_hip_region* hc, int series, size_t step0, size_t n, double* dst, int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_get_series: null argument");
    if (h->sh) return guarded(h, [&] { shards::get_rows(h->sh, 1, series, step0, n, dst, dst_on_device); });
    return guarded(h, [&] {
        if (series < 0 || size_t(series) >= h->n_series())
            throw std::runtime_error("get_series: series not collected in this collection mode");
        check_window(h, step0, n, "get_series");
        const double* src = h->d_resp.p + (size_t(series) * h->TW + (step0 - h->w0)) * h->n;
        copy_rows(h->stream, dst, src, n * h->n * sizeof(double), dst_on_device, 1);
    });
}

int shyft_hip_get_state_series(const shyft_hip_region* hc, int field, size_t step0, size_t n, double* dst,
                               int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_get_state_series: null argument");
    if (h->sh) return guarded(h, [&] { shards::get_rows(h->sh, 2, field, step0, n, dst, dst_on_device); });
    return guarded(h, [&] {
        if (!h->collect_state) throw std::runtime_error("get_state_series: state collection is off");
        if (field < 0 || size_t(field) >= h->n_state_series()) throw std::runtime_error("get_state_series: invalid field");
        if (step0 < h->w0 || step0 + n > h->w0 + h->TW + 1) throw std::runtime_error("get_state_series: outside window");
        const double* src = h->d_state_series.p + (size_t(field) * (h->TW + 1) + (step0 - h->w0)) * h->n;
        copy_rows(h->stream, dst, src, n * h->n * sizeof(double), dst_on_device, 1);
    });
}

}  // extern "C"
namespace shyft_hip_impl {
void region_set_cell_ids(shyft_hip_region* h, const int64_t* ids) {
    if (!ids) {
        h->d_cell_ids.release();
        return;
    }
    hip_check(hipSetDevice(h->device), "hipSetDevice");
    h->d_cell_ids.alloc(h->n);
    hip_check(region_copy(h, h->d_cell_ids.p, ids, h->n * sizeof(int64_t), hipMemcpyHostToDevice), "upload cell ids");
}

int region_selected_sums(shyft_hip_region* h, int series, const int64_t* ids, size_t n_ids, int scope, int weighted,
                         size_t step0, size_t n, double* dst, double* sum_area_out, size_t* n_selected) {
    return guarded(h, [&] {
        const double* src = series_rows(h, series, step0, n, "statistics");
        std::vector<int32_t> sel = select_cells(h, ids, n_ids, scope);
        if (n_selected) *n_selected = sel.size();
        double sum_area = 0.0;
        if (sel.empty()) {
            for (size_t t = 0; t < n; ++t) dst[t] = 0.0;
            if (sum_area_out) *sum_area_out = 0.0;
            return;
        }
        h->d_sel.alloc(std::max(h->d_sel.n, sel.size()));
        hip_check(region_copy(h, h->d_sel.p, sel.data(), sel.size() * sizeof(int32_t), hipMemcpyHostToDevice), "upload sel");
        const double* w = nullptr;
        if (weighted) {
            std::vector<double> a(sel.size());
            for (size_t k = 0; k < sel.size(); ++k) {
                a[k] = h->geo[size_t(sel[k]) * 11 + 3];
                sum_area += a[k];
            }
            h->d_w.alloc(std::max(h->d_w.n, a.size()));
            hip_check(region_copy(h, h->d_w.p, a.data(), a.size() * sizeof(double), hipMemcpyHostToDevice), "upload w");
            w = h->d_w.p;
        }
        h->d_tmp.alloc(std::max(h->d_tmp.n, n));
        hip_check(launch_select_sum(src, h->n, n, h->d_sel.p, sel.size(), w, h->d_tmp.p, h->stream), "select_sum");
        copy_rows(h->stream, dst, h->d_tmp.p, n * sizeof(double), 0, 1);
        if (sum_area_out) *sum_area_out = sum_area;
    });
}
}  // namespace shyft_hip_impl
extern "C" {

int shyft_hip_statistics(const shyft_hip_region* hc, int series, const int64_t* ids, size_t n_ids, int scope, int weighted,
                         size_t step0, size_t n, double* dst) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_statistics: null argument");
    if (h->sh) return guarded(h, [&] { shards::statistics(h->sh, series, ids, n_ids, scope, weighted, step0, n, dst); });
    double sum_area = 0.0;
    size_t n_sel = 0;
    const int rc = region_selected_sums(h, series, ids, n_ids, scope, weighted, step0, n, dst, &sum_area, &n_sel);
    if (rc || !weighted) return rc;
    if (n_sel == 0) {  // no match: sum -> empty ts in the reference (0 here); average -> nan
        for (size_t t = 0; t < n; ++t) dst[t] = NAN;
        return 0;
    }
    const double s = 1 / sum_area;  // scale_by(1/sum_area) (cell_model.h:252)
    for (size_t t = 0; t < n; ++t) dst[t] *= s;
    return 0;
}

int shyft_hip_catchment_sums(const shyft_hip_region* hc, int series, size_t step0, size_t n, double* dst,
                             int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_catchment_sums: null argument");
    if (h->sh) return guarded(h, [&] { shards::catchment_sums(h->sh, series, step0, n, dst, dst_on_device, false); });
    return guarded(h, [&] {
        const double* src = series_rows(h, series, step0, n, "catchment_sums");
        const size_t C = h->cix_to_cid.size();
        double* out = dst;
        if (!dst_on_device) {
            h->d_tmp.alloc(std::max(h->d_tmp.n, C * n));
            out = h->d_tmp.p;
        }
        hip_check(launch_segment_sums(src, h->n, n, h->seg_identity ? nullptr : h->d_seg_cells.p, h->d_seg_off.p, C, out, h->stream), "segment_sums");
        if (!dst_on_device) copy_rows(h->stream, dst, out, C * n * sizeof(double), 0, 1);
        else hip_check(hipStreamSynchronize(h->stream), "sync");
    });
}

int shyft_hip_catchment_area_sums(const shyft_hip_region* hc, int series, size_t step0, size_t n, double* dst,
                                  int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_catchment_area_sums: null argument");
    if (h->sh) return guarded(h, [&] { shards::catchment_sums(h->sh, series, step0, n, dst, dst_on_device, true); });
    return guarded(h, [&] {
        const double* src = series_rows(h, series, step0, n, "catchment_area_sums");
        update_derived(h);  // per-cell constants (cell area) are current
        const size_t C = h->cix_to_cid.size();
        const double* w = h->d_cellc.p + size_t(h->hbv() ? HC_AREA : PC_AREA) * h->n;
        double* out = dst;
        if (!dst_on_device) {
            h->d_tmp.alloc(std::max(h->d_tmp.n, C * n));
            out = h->d_tmp.p;
        }
        hip_check(launch_segment_sums(src, h->n, n, h->seg_identity ? nullptr : h->d_seg_cells.p, h->d_seg_off.p, C, out, h->stream, w),
                  "segment_sums");
        if (!dst_on_device) copy_rows(h->stream, dst, out, C * n * sizeof(double), 0, 1);
        else hip_check(hipStreamSynchronize(h->stream), "sync");
    });
}

size_t shyft_hip_number_of_catchments(const shyft_hip_region* h) {
    return h ? (h->sh ? shards::number_of_catchments(h->sh) : h->cix_to_cid.size()) : 0;
}

int shyft_hip_catchment_ids(const shyft_hip_region* h, int64_t* cids) {
    if (!h || !cids) return fail(const_cast<shyft_hip_region*>(h), "shyft_hip_catchment_ids: null argument");
    if (h->sh) {
        shards::catchment_ids(h->sh, cids);
        return 0;
    }
    for (size_t c = 0; c < h->cix_to_cid.size(); ++c) cids[c] = h->cix_to_cid[c];
    return 0;
}

int shyft_hip_region_clone(const shyft_hip_region* src, shyft_hip_region** out) {
    if (!src || !out) return fail(nullptr, "shyft_hip_region_clone: null argument");
    *out = nullptr;
    if (src->sh) {
        try {
            std::unique_ptr<shyft_hip_region> c(new shyft_hip_region());
            c->stack = src->stack;
            c->n = src->n;
            c->device = src->device;
            c->sh = shards::clone(src->sh);
            *out = c.release();
            return 0;
        } catch (const std::exception& e) {
            return fail(nullptr, e.what());
        }
    }
    shyft_hip_region* c = nullptr;
    if (shyft_hip_region_create(src->stack, src->n, src->device, &c)) return 1;
    std::unique_ptr<shyft_hip_region, void (*)(shyft_hip_region*)> h(c, shyft_hip_region_destroy);
    const int rc = guarded(h.get(), [&] {
        hip_check(hipDeviceSynchronize(), "sync");
        // host mirrors (every member that is not a device buffer, stream or event)
        h->err.clear();
        h->geo = src->geo; h->routing_id = src->routing_id; h->routing_distance = src->routing_distance;
        h->cid = src->cid; h->cix = src->cix; h->cix_to_cid = src->cix_to_cid; h->cid_to_cix = src->cid_to_cix;
        h->params = src->params; h->n_sets = src->n_sets; h->set_ix = src->set_ix; h->active = src->active;
        h->t0 = src->t0; h->dt = src->dt; h->T = src->T; h->w0 = src->w0; h->TW = src->TW;
        h->collect = src->collect; h->collect_state = src->collect_state;
        h->derived_dirty = true; h->has_geo = src->has_geo; h->has_params = src->has_params; h->has_state = src->has_state;
        h->dst_dirty = true;
        clone_buf(h->d_state, src->d_state);
        clone_buf(h->d_forcing, src->d_forcing);
        clone_buf(h->d_resp, src->d_resp);
        clone_buf(h->d_state_series, src->d_state_series);
        clone_buf(h->d_doy, src->d_doy);
        clone_buf(h->d_trel, src->d_trel);
        clone_buf(h->d_seg_cells, src->d_seg_cells);
        h->seg_identity = src->seg_identity;
        clone_buf(h->d_seg_off, src->d_seg_off);
        clone_buf(h->d_active, src->d_active);
        clone_buf(h->d_alt, src->d_alt);
        clone_buf(h->d_cell_ids, src->d_cell_ids);
    });
    if (rc) {
        g_last_error = h->err;
        return rc;
    }
    *out = h.release();
    return 0;
}

int shyft_hip_cell_series(shyft_hip_region* h, int series, size_t cell, size_t step0, size_t n, double* buf, int write) {
    if (!h || !buf) return fail(h, "shyft_hip_cell_series: null argument");
    if (h->sh) return guarded(h, [&] { shards::cell_series(h->sh, series, cell, step0, n, buf, write); });
    return guarded(h, [&] {
        if (cell >= h->n) throw std::runtime_error("cell_series: cell index out of range");
        if (write && series < SHYFT_HIP_SERIES_FORCING)
            throw std::runtime_error("cell_series: only forcing (cell env_ts) is writable");
        const double* rows = series_rows(h, series, step0, n, "cell_series");
        double* p = const_cast<double*>(rows) + cell;
        const size_t pitch = h->n * sizeof(double);
        if (write)
            hip_check(hipMemcpy2DAsync(p, pitch, buf, sizeof(double), sizeof(double), n, hipMemcpyHostToDevice, h->stream),
                      "cell_series write");
        else
            hip_check(hipMemcpy2DAsync(buf, sizeof(double), p, pitch, sizeof(double), n, hipMemcpyDeviceToHost, h->stream),
                      "cell_series read");
        hip_check(hipStreamSynchronize(h->stream), "sync");
    });
}

int shyft_hip_sample_cells(const shyft_hip_region* hc, int series, const int64_t* cells, size_t n_cells, size_t step0,
                           size_t n, double* dst) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || (n_cells && (!cells || !dst))) return fail(h, "shyft_hip_sample_cells: null argument");
    if (n_cells == 0 || n == 0) return 0;
    if (h->sh) return guarded(h, [&] { shards::sample_cells(h->sh, series, cells, n_cells, step0, n, dst); });
    return guarded(h, [&] {
        const double* rows = series_rows(h, series, step0, n, "sample_cells");
        std::vector<int32_t> idx(n_cells);
        for (size_t j = 0; j < n_cells; ++j) {
            if (cells[j] < 0 || size_t(cells[j]) >= h->n) throw std::runtime_error("sample_cells: cell index out of range");
            idx[j] = int32_t(cells[j]);
        }
        h->d_sel.alloc(std::max(h->d_sel.n, n_cells));
        hip_check(region_copy(h, h->d_sel.p, idx.data(), n_cells * sizeof(int32_t), hipMemcpyHostToDevice), "upload cells");
        h->d_tmp.alloc(std::max(h->d_tmp.n, n * n_cells));
        hip_check(launch_gather_columns(h->d_tmp.p, rows, n, h->n, h->d_sel.p, n_cells, h->stream), "gather_columns");
        copy_rows(h->stream, dst, h->d_tmp.p, n * n_cells * sizeof(double), 0, 1);
    });
}

int shyft_hip_set_test_knob(shyft_hip_region* h, int knob, int64_t value) {
    if (!h) return fail(h, "shyft_hip_set_test_knob: null handle");
    if (h->sh) return guarded(h, [&] { shards::set_test_knob(h->sh, knob, value); });
    return guarded(h, [&] {
        if (knob == SHYFT_HIP_KNOB_PTGSK_INSTANCE) {
            if (value != 0 && value != 2 && value != 4)
                throw std::runtime_error("set_test_knob: pt_gs_k instance must be 0 (auto), 2 or 4");
            h->knob_instance = int(value);
        } else if (knob == SHYFT_HIP_KNOB_SERIAL_SHARDS || knob == SHYFT_HIP_KNOB_CLONE_FAIL_AT) {
            throw std::runtime_error("set_test_knob: this knob needs a sharded region");
        } else if (knob == SHYFT_HIP_KNOB_BRENT_READ_DELAY) {
            if (value < 0 || value > 1000) throw std::runtime_error("set_test_knob: read delay must be in [0, 1000]");
            h->knob_read_delay = int(value);
        } else {
            throw std::runtime_error("set_test_knob: unknown knob");
        }
    });
}

int shyft_hip_forcing_ok(const shyft_hip_region* hc, int* ok) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !ok) return fail(h, "shyft_hip_forcing_ok: null argument");
    if (h->sh) return guarded(h, [&] { shards::forcing_ok(h->sh, ok); });
    return guarded(h, [&] {
        *ok = 0;
        if (h->T == 0) throw std::runtime_error("is_cell_env_ts_ok: no time axis (initialize_cell_environment)");
        hip_check(hipMemsetAsync(h->d_flag.p, 0, sizeof(int32_t), h->stream), "memset");
        const uint8_t* active = h->active.empty() ? nullptr : h->d_active.p;
        hip_check(launch_nan_scan(h->d_forcing.p, N_FORCING * h->TW, h->n, active, h->d_flag.p, h->stream), "nan_scan");
        int32_t flag = 0;
        hip_check(hipMemcpyAsync(&flag, h->d_flag.p, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream), "download");
        hip_check(hipStreamSynchronize(h->stream), "sync");
        *ok = flag ? 0 : 1;
    });
}

}  // extern "C"

// ---------------------------------------------------------------- routing (core/routing.h:239-421)
extern "C" {

int shyft_hip_set_routing_groups(shyft_hip_region* h, const int32_t* group_of_cell, size_t n_groups) {
    if (!h) return fail(h, "shyft_hip_set_routing_groups: null handle");
    if (h->sh) return guarded(h, [&] { shards::set_routing_groups(h->sh, group_of_cell, n_groups); });
    return guarded(h, [&] {
        if (n_groups > 0 && !group_of_cell) throw std::runtime_error("set_routing_groups: group_of_cell is null");
        std::vector<int32_t> off(n_groups + 1, 0), cells;
        for (size_t i = 0; i < h->n && n_groups; ++i) {
            const int32_t g = group_of_cell[i];
            if (g < -1 || g >= int32_t(n_groups)) throw std::runtime_error("set_routing_groups: group index out of range");
            if (g >= 0) off[size_t(g) + 1]++;
        }
        for (size_t g = 0; g < n_groups; ++g) off[g + 1] += off[g];
        cells.resize(size_t(off[n_groups]));
        std::vector<int32_t> pos(off.begin(), off.end() - 1);
        for (size_t i = 0; i < h->n && n_groups; ++i)
            if (group_of_cell[i] >= 0) cells[size_t(pos[size_t(group_of_cell[i])]++)] = int32_t(i);
        h->rseg_identity = cells.size() == h->n;
        for (size_t i = 0; i < cells.size() && h->rseg_identity; ++i) h->rseg_identity = cells[i] == int32_t(i);
        h->d_rseg_off.alloc(n_groups + 1);
        h->d_rseg_cells.alloc(std::max<size_t>(1, cells.size()));
        hip_check(region_copy(h, h->d_rseg_off.p, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice), "upload");
        if (!cells.empty())
            hip_check(region_copy(h, h->d_rseg_cells.p, cells.data(), cells.size() * sizeof(int32_t), hipMemcpyHostToDevice),
                      "upload");
        h->n_route_groups = n_groups;
    });
}

int shyft_hip_routing_group_sums(const shyft_hip_region* hc, size_t step0, size_t n, double* dst, int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_routing_group_sums: null argument");
    if (h->sh) return guarded(h, [&] { shards::routing_group_sums(h->sh, step0, n, dst, dst_on_device); });
    return guarded(h, [&] {
        const size_t G = h->n_route_groups;
        if (G == 0) return;
        const double* src = series_rows(h, SHYFT_HIP_AVG_DISCHARGE, step0, n, "routing_group_sums");
        double* out = dst;
        if (!dst_on_device) {
            h->d_tmp.alloc(std::max(h->d_tmp.n, G * n));
            out = h->d_tmp.p;
        }
        hip_check(launch_segment_sums(src, h->n, n, h->rseg_identity ? nullptr : h->d_rseg_cells.p, h->d_rseg_off.p, G, out, h->stream),
                  "routing group sums");
        if (!dst_on_device) copy_rows(h->stream, dst, out, G * n * sizeof(double), 0, 1);
        else hip_check(hipStreamSynchronize(h->stream), "sync");
    });
}

int shyft_hip_route(int device, size_t n_groups, size_t T, const double* group_sums, int src_on_device,
                    const double* group_uhg, const int32_t* group_len, const int32_t* group_river, size_t n_rivers,
                    const double* river_uhg, const int32_t* river_len, const int32_t* river_downstream, size_t max_len,
                    double* local, double* upstream, double* output, int dst_on_device) {
    if (!group_sums || !group_uhg || !group_len || !group_river || !river_uhg || !river_len || !river_downstream ||
        !local || !upstream || !output)
        return fail(nullptr, "shyft_hip_route: null argument");
    try {
        if (device < 0) hip_check(hipGetDevice(&device), "hipGetDevice");
        hip_check(hipSetDevice(device), "hipSetDevice");
        const size_t R = n_rivers, G = n_groups;
        if (R == 0 || T == 0) return 0;
        if (max_len == 0) throw std::runtime_error("route: max_len == 0");
        for (size_t g = 0; g < G; ++g) {
            if (group_river[g] < 0 || size_t(group_river[g]) >= R) throw std::runtime_error("route: group river out of range");
            if (group_len[g] < 1 || size_t(group_len[g]) > max_len) throw std::runtime_error("route: group UHG length");
        }
        // river CSR tables: groups of each river (ascending g), upstream rivers (ascending index = ascending id)
        std::vector<int32_t> gro(R + 1, 0), grs(G), upo(R + 1, 0), ups;
        for (size_t g = 0; g < G; ++g) gro[size_t(group_river[g]) + 1]++;
        for (size_t r = 0; r < R; ++r) gro[r + 1] += gro[r];
        {
            std::vector<int32_t> pos(gro.begin(), gro.end() - 1);
            for (size_t g = 0; g < G; ++g) grs[size_t(pos[size_t(group_river[g])]++)] = int32_t(g);
        }
        for (size_t r = 0; r < R; ++r) {
            if (river_len[r] < 1 || size_t(river_len[r]) > max_len) throw std::runtime_error("route: river UHG length");
            if (river_downstream[r] >= int32_t(R) || river_downstream[r] == int32_t(r))
                throw std::runtime_error("route: invalid downstream river");
        }
        for (size_t r = 0; r < R; ++r) {
            for (size_t u = 0; u < R; ++u)
                if (river_downstream[u] == int32_t(r)) ups.push_back(int32_t(u));
            upo[r + 1] = int32_t(ups.size());
        }
        // network levels: level(r) = 1 + max level of its upstream rivers (sources are level 0)
        std::vector<int32_t> level(R, -1);
        for (size_t pass = 0; pass <= R; ++pass) {
            bool changed = false;
            for (size_t r = 0; r < R; ++r) {
                int32_t lv = 0;
                bool ready = true;
                for (int32_t k = upo[r]; k < upo[r + 1]; ++k) {
                    if (level[size_t(ups[size_t(k)])] < 0) { ready = false; break; }
                    lv = std::max(lv, level[size_t(ups[size_t(k)])] + 1);
                }
                if (ready && level[r] != lv) { level[r] = lv; changed = true; }
            }
            if (!changed) break;
        }
        int32_t n_levels = 0;
        for (size_t r = 0; r < R; ++r) {
            if (level[r] < 0) throw std::runtime_error("adding this river caused circular reference");
            n_levels = std::max(n_levels, level[r] + 1);
        }
        std::vector<int32_t> lvl_off(size_t(n_levels) + 1, 0), lvl_rivers;
        for (int32_t l = 0; l < n_levels; ++l) {
            for (size_t r = 0; r < R; ++r)
                if (level[r] == l) lvl_rivers.push_back(int32_t(r));
            lvl_off[size_t(l) + 1] = int32_t(lvl_rivers.size());
        }
        hipStream_t s = nullptr;
        hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
        struct stream_guard { hipStream_t s; ~stream_guard() { (void)hipStreamDestroy(s); } } sg{s};
        dbuf<double> d_sums, d_gw, d_rw, d_local, d_up, d_in, d_out;
        dbuf<int32_t> d_glen, d_gro, d_grs, d_rlen, d_upo, d_ups, d_lvl;
        auto up_d = [&](dbuf<double>& b, const double* src, size_t n, int on_dev) {
            b.alloc(std::max<size_t>(1, n));
            if (n) hip_check(hipMemcpy(b.p, src, n * sizeof(double), on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice), "upload");
        };
        auto up_i = [&](dbuf<int32_t>& b, const int32_t* src, size_t n) {
            b.alloc(std::max<size_t>(1, n));
            if (n) hip_check(hipMemcpy(b.p, src, n * sizeof(int32_t), hipMemcpyHostToDevice), "upload");
        };
        up_d(d_sums, group_sums, G * T, src_on_device);
        up_d(d_gw, group_uhg, G * max_len, 0);
        up_d(d_rw, river_uhg, R * max_len, 0);
        up_i(d_glen, group_len, G);
        up_i(d_gro, gro.data(), gro.size());
        up_i(d_grs, grs.data(), grs.size());
        up_i(d_rlen, river_len, R);
        up_i(d_upo, upo.data(), upo.size());
        up_i(d_ups, ups.data(), ups.size());
        up_i(d_lvl, lvl_rivers.data(), lvl_rivers.size());
        double* o_local = local;
        double* o_up = upstream;
        double* o_out = output;
        if (!dst_on_device) {
            d_local.alloc(R * T); d_up.alloc(R * T); d_out.alloc(R * T);
            o_local = d_local.p; o_up = d_up.p; o_out = d_out.p;
        }
        d_in.alloc(R * T);
        routing_args a;
        a.n_steps = int(T);
        a.n_rivers = int(R);
        a.max_len = int(max_len);
        a.group_sums = d_sums.p; a.group_w = d_gw.p; a.group_len = d_glen.p;
        a.river_group_off = d_gro.p; a.river_groups = d_grs.p;
        a.river_w = d_rw.p; a.river_len = d_rlen.p;
        a.river_up_off = d_upo.p; a.river_up = d_ups.p; a.level_rivers = d_lvl.p;
        a.local = o_local; a.upstream = o_up; a.inflow = d_in.p; a.output = o_out;
        hip_check(launch_route(a, lvl_off.data(), n_levels, s), "route");
        hip_check(hipStreamSynchronize(s), "route sync");
        if (!dst_on_device) {
            hip_check(hipMemcpy(local, o_local, R * T * sizeof(double), hipMemcpyDeviceToHost), "download");
            hip_check(hipMemcpy(upstream, o_up, R * T * sizeof(double), hipMemcpyDeviceToHost), "download");
            hip_check(hipMemcpy(output, o_out, R * T * sizeof(double), hipMemcpyDeviceToHost), "download");
        }
    } catch (const std::exception& e) {
        return fail(nullptr, e.what());
    }
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- parameter ensembles (core/model_calibration.h:830-899)
extern "C" {

int shyft_hip_ensemble_run(shyft_hip_region* h, const double* params, size_t n_members, size_t n_per_set,
                           int start_step, int n_steps, int collect) {
    if (!h || !params) return fail(h, "shyft_hip_ensemble_run: null argument");
    if (h->sh) return guarded(h, [&] { shards::ensemble_run(h->sh, params, n_members, n_per_set, start_step, n_steps, collect); });
    return guarded(h, [&] {
        if (n_members == 0) throw std::runtime_error("ensemble_run: n_members must be > 0");
        if (collect != COLLECT_DISCHARGE && collect != COLLECT_DISCHARGE_SNOW)
            throw std::runtime_error("ensemble_run: collect must be discharge or discharge+snow");
        if (!h->has_geo) throw std::runtime_error("region: geo_cell_data not set");
        if (!h->has_state) throw std::runtime_error("region_model::run: no state set");
        if (!(h->T > 0)) throw std::runtime_error("region_model::run with invalid time_axis invoked");
        if (start_step < 0 || n_steps < 0 || size_t(start_step) + size_t(n_steps) > h->T)
            throw std::runtime_error("ensemble_run: steps outside the time axis");
        const size_t b = n_steps > 0 ? size_t(start_step) : 0;
        const size_t e = n_steps > 0 ? size_t(start_step + n_steps) : h->T;
        check_window(h, b, e - b, "ensemble_run");
        // calculated cells (catchment filter), cell order
        std::vector<int32_t> cells;
        for (size_t i = 0; i < h->n; ++i)
            if (h->active.empty() || h->active[i]) cells.push_back(int32_t(i));
        if (cells.empty()) throw std::runtime_error("ensemble_run: no calculated cells");
        const size_t P = n_members, K = cells.size(), L = K * P;
        if (L > size_t(INT32_MAX)) throw std::runtime_error("ensemble_run: cells x members exceeds 2^31 lanes");
        hip_check(hipStreamSynchronize(h->stream), "sync");  // forcing/state writes of the region are complete

        if (h->ens && (h->ens->n != L || h->ens->stack != h->stack)) {
            shyft_hip_region_destroy(h->ens);
            h->ens = nullptr;
        }
        if (!h->ens) {
            shyft_hip_region* c = nullptr;
            if (shyft_hip_region_create(h->stack, L, h->device, &c)) throw std::runtime_error(g_last_error);
            h->ens = c;
        }
        shyft_hip_region* x = h->ens;
        x->forcing_src = h;
        x->geo.resize(L * 11);
        std::vector<int32_t> fcol(L), lane_set(L);
        for (size_t k = 0; k < K; ++k)
            for (size_t m = 0; m < P; ++m) {
                const size_t l = k * P + m;
                fcol[l] = cells[k];
                std::copy(h->geo.begin() + size_t(cells[k]) * 11, h->geo.begin() + size_t(cells[k]) * 11 + 11,
                          x->geo.begin() + l * 11);
                lane_set[l] = int32_t(m);
            }
        if (shyft_hip_set_parameters(x, params, P, n_per_set, lane_set.data())) throw std::runtime_error(x->err);
        x->active.clear();
        x->t0 = h->t0; x->dt = h->dt; x->T = h->T; x->w0 = h->w0; x->TW = h->TW;
        x->collect = collect;
        x->collect_state = 0;
        x->has_geo = x->has_params = x->has_state = true;
        x->derived_dirty = true;
        update_derived(x);  // per-member parameter rows and per-lane constants
        x->d_fcol.alloc(L);
        hip_check(hipMemcpy(x->d_fcol.p, fcol.data(), L * sizeof(int32_t), hipMemcpyHostToDevice), "upload fcol");
        clone_buf(x->d_doy, h->d_doy);
        clone_buf(x->d_trel, h->d_trel);
        // every member starts from the region's current state
        hip_check(launch_gather_columns(x->d_state.p, h->d_state.p, h->n_state_fields(), h->n, x->d_fcol.p, L, x->stream),
                  "gather state");
        x->d_resp.alloc(x->n_series() * x->TW * L);
        x->d_state_series.release();
        // (member, catchment) segments, lanes in cell order: group m*C + cix
        const size_t C = h->cix_to_cid.size();
        std::vector<int32_t> off(P * C + 1, 0), seg(L);
        for (size_t k = 0; k < K; ++k)
            for (size_t m = 0; m < P; ++m) off[m * C + h->cix[size_t(cells[k])] + 1]++;
        for (size_t g = 0; g < P * C; ++g) off[g + 1] += off[g];
        std::vector<int32_t> pos(off.begin(), off.end() - 1);
        for (size_t k = 0; k < K; ++k)
            for (size_t m = 0; m < P; ++m) seg[size_t(pos[m * C + h->cix[size_t(cells[k])]]++)] = int32_t(k * P + m);
        x->d_seg_off.alloc(off.size());
        x->d_seg_cells.alloc(L);
        hip_check(hipMemcpy(x->d_seg_off.p, off.data(), off.size() * sizeof(int32_t), hipMemcpyHostToDevice), "upload");
        hip_check(hipMemcpy(x->d_seg_cells.p, seg.data(), L * sizeof(int32_t), hipMemcpyHostToDevice), "upload");
        x->ens_groups = P * C;
        h->ens_members = P;
        h->ens_cells = K;
        h->ens_b = b;
        h->ens_e = e;
        launch_run(x, int(b), int(e - b));
        finish_run(x);
    });
}

int shyft_hip_ensemble_sums(const shyft_hip_region* hc, int series, int area_weighted, size_t step0, size_t n,
                            double* dst, int dst_on_device) {
    shyft_hip_region* h = const_cast<shyft_hip_region*>(hc);
    if (!h || !dst) return fail(h, "shyft_hip_ensemble_sums: null argument");
    if (h->sh) return guarded(h, [&] { shards::ensemble_sums(h->sh, series, area_weighted, step0, n, dst, dst_on_device); });
    return guarded(h, [&] {
        shyft_hip_region* x = h->ens;
        if (!x || h->ens_members == 0) throw std::runtime_error("ensemble_sums: no ensemble run");
        if (series < 0 || size_t(series) >= x->n_series())
            throw std::runtime_error("ensemble_sums: series not collected by the ensemble run");
        if (step0 < h->ens_b || step0 + n > h->ens_e)
            throw std::runtime_error("ensemble_sums: steps outside the last ensemble run");
        const size_t L = x->n, G = x->ens_groups;
        const double* src = x->d_resp.p + (size_t(series) * x->TW + (step0 - x->w0)) * L;
        const double* w = nullptr;
        if (area_weighted) w = x->d_cellc.p + size_t(x->hbv() ? HC_AREA : PC_AREA) * L;
        double* out = dst;
        if (!dst_on_device) {
            x->d_tmp.alloc(std::max(x->d_tmp.n, G * n));
            out = x->d_tmp.p;
        }
        hip_check(launch_segment_sums(src, L, n, x->d_seg_cells.p, x->d_seg_off.p, G, out, x->stream, w),
                  "ensemble sums");
        if (!dst_on_device) copy_rows(x->stream, dst, out, G * n * sizeof(double), 0, 1);
        else hip_check(hipStreamSynchronize(x->stream), "sync");
    });
}

double shyft_hip_ensemble_last_ms(const shyft_hip_region* h) {
    if (h && h->sh) return shards::ensemble_last_ms(h->sh);
    return h && h->ens ? h->ens->last_ms : 0.0;
}

}  // extern "C"
