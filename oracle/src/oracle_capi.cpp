// ORACLE — test infrastructure only (see common.hpp header).
//
// C entry points of the CPU restatement, loaded by tests/ (ctypes) and by
// bench.py's cpu_baseline leg. Not linked by the product library.
#include <chrono>
#include <cstring>
#include <exception>
#include <thread>

#include "common.hpp"
#include "idw.hpp"
#include "methods.hpp"
#include "ptgsk.hpp"
#include "region.hpp"

using namespace oracle;

namespace {
int fail(char* err, size_t errlen, const char* msg) {
    if (err && errlen) {
        std::strncpy(err, msg, errlen - 1);
        err[errlen - 1] = 0;
    }
    return 1;
}
}  // namespace

extern "C" {

double oracle_gamma_p(double a, double x) { return special::gamma_p(a, x); }
// the elementary functions this build uses (detmath, or libm with -DORACLE_LIBM)
double oracle_exp(double x) { return OEXP(x); }
double oracle_log(double x) { return OLOG(x); }
double oracle_pow(double x, double y) { return OPOW(x, y); }
double oracle_lgamma_fn(double x) { return OLGAMMA(x); }
double oracle_lgamma(double a) { return special::lgamma_(a); }

void oracle_gs_calc_snow_state(double shape, double scale, double y0, double lambda, double lwd, double max_water_frac,
                               double temp_swe, double* swe, double* sca) {
    gamma_snow::calculator gs;
    gs.calc_snow_state(shape, scale, y0, lambda, lwd, max_water_frac, temp_swe, *swe, *sca);
}

double oracle_gs_corr_lwc(double z1, double a1, double b1, double z2, double a2, double b2) {
    gamma_snow::calculator gs;
    return gs.corr_lwc(z1, a1, b1, z2, a2, b2);
}

// state: 8 doubles (gamma_snow::state order), resp: sca, storage, outflow
// gsp: the gamma_snow part given as a full 31-element pt_gs_k parameter vector
int oracle_gs_step(double* st, double* resp, int64_t t_us, int64_t dt_us, const double* p31, double T, double rad,
                   double prec, double ws, double rh, double forest, double altitude) {
    pt_gs_k::parameter p;
    p.set(p31);
    gamma_snow::state s{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7]};
    gamma_snow::response r;
    try {
        gamma_snow::calculator().step(s, r, t_us, dt_us, p.gs, T, rad, prec, ws, rh, forest, altitude);
    } catch (...) {
        return 1;
    }
    st[0] = s.albedo; st[1] = s.lwc; st[2] = s.surface_heat; st[3] = s.alpha; st[4] = s.sdc_melt_mean;
    st[5] = s.acc_melt; st[6] = s.iso_pot_energy; st[7] = s.temp_swe;
    resp[0] = r.sca; resp[1] = r.storage; resp[2] = r.outflow;
    return 0;
}

int oracle_kirchner_step(double c1, double c2, double c3, double abs_err, double rel_err, int64_t T0_us, int64_t T1_us,
                         double* q, double* q_avg, double p, double e) {
    kirchner::parameter kp{c1, c2, c3};
    kirchner::calculator k(abs_err, rel_err, kp);
    try {
        k.step(T0_us, T1_us, *q, *q_avg, p, e);
    } catch (...) {
        return 1;
    }
    return 0;
}

double oracle_pt_pot_evap(double albedo, double alpha, double T, double rad, double rh) {
    return priestley_taylor::calculator(albedo, alpha).potential_evapotranspiration(T, rad, rh);
}

int oracle_day_of_year(int64_t t_us) { return day_of_year(t_us); }
int64_t oracle_trim_year(int64_t t_us) { return trim_year(t_us); }

// Run the pt_gs_k region model on the CPU with the reference scheduler.
//  geo11     : n_cells x 11 (geo_cell_data_io layout, api/api.h:1598-1621)
//  params    : n_sets x 31 (pt_gs_k.h:77-112 order); set_ix[n_cells] selects a set per cell
//  state     : n_cells x 9 in/out (pt_gs_k::state order, ptgsk.hpp)
//  forcing   : five [T][n_cells] arrays (temperature, precipitation, wind_speed, rel_hum, radiation)
//  out_main  : [2][T][n_cells] avg_discharge, charge_m3s (may be null)
//  out_full  : [8][T][n_cells] all_response_collector series (may be null)
//  out_state : [9][T+1][n_cells] state_collector series (may be null)
//  elapsed_s : wall seconds spent in run_cells only
int oracle_ptgsk_run(size_t n_cells, const double* geo11, const double* params, size_t n_sets, const int32_t* set_ix,
                     double* state, int64_t t0_us, int64_t dt_us, size_t T, int start_step, int n_steps, const double* temp,
                     const double* prec, const double* ws, const double* rh, const double* rad, double* out_main,
                     double* out_full, double* out_state, int ncore, double* elapsed_s, char* err, size_t errlen) {
    try {
        ptgsk_region rm;
        rm.time_axis = fixed_dt(t0_us, dt_us, T);
        rm.params.resize(n_sets);
        for (size_t k = 0; k < n_sets; ++k) rm.params[k].set(params + k * 31);
        rm.cells.resize(n_cells);
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.geo = geo_cell_data::from_raw(geo11 + i * 11);
            int32_t k = set_ix ? set_ix[i] : 0;
            if (k < 0 || size_t(k) >= n_sets) return fail(err, errlen, "oracle_ptgsk_run: parameter set index out of range");
            c.parameter = &rm.params[k];
            c.state.set(state + i * 9);
            c.temp.resize(T); c.prec.resize(T); c.ws.resize(T); c.rh.resize(T); c.rad.resize(T);
            for (size_t t = 0; t < T; ++t) {
                c.temp[t] = temp[t * n_cells + i];
                c.prec[t] = prec[t * n_cells + i];
                c.ws[t] = ws[t * n_cells + i];
                c.rh[t] = rh[t * n_cells + i];
                c.rad[t] = rad[t * n_cells + i];
            }
            c.col.full = out_full != nullptr;
            c.col.collect_state = out_state != nullptr;
        }
        auto t_begin = std::chrono::steady_clock::now();
        rm.run_cells(size_t(ncore < 0 ? 0 : ncore), start_step, n_steps);
        auto t_end = std::chrono::steady_clock::now();
        if (elapsed_s) *elapsed_s = std::chrono::duration<double>(t_end - t_begin).count();
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.state.get(state + i * 9);
            for (size_t t = 0; t < T; ++t) {
                if (out_main) {
                    out_main[t * n_cells + i] = c.col.rc[pt_gs_k::AVG_DISCHARGE][t];
                    out_main[(T + t) * n_cells + i] = c.col.rc[pt_gs_k::CHARGE_M3S][t];
                }
                if (out_full)
                    for (int k = 0; k < pt_gs_k::N_ALL; ++k) out_full[(size_t(k) * T + t) * n_cells + i] = c.col.rc[k][t];
            }
            if (out_state)
                for (int k = 0; k < 9; ++k)
                    for (size_t t = 0; t <= T; ++t) out_state[(size_t(k) * (T + 1) + t) * n_cells + i] = c.col.sc[k][t];
        }
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

// ---------------------------------------------------------------- pt_ss_k / skaugen
// skaugen::calculator::step on one state: st = nu alpha sca swe free_water residual num_units (7 doubles),
// p8 = alpha_0 d_range unit_size max_water_fraction tx cx ts cfr; resp = outflow sca swe. Returns 1 on a throw.
int oracle_skaugen_step(double* st, double* resp, int64_t dt_us, const double* p8, double T, double prec_mm_h) {
    skaugen::parameter p{p8[0], p8[1], p8[2], p8[3], p8[4], p8[5], p8[6], p8[7]};
    skaugen::state s;
    s.nu = st[0]; s.alpha = st[1]; s.sca = st[2]; s.swe = st[3]; s.free_water = st[4]; s.residual = st[5];
    s.num_units = size_t(st[6]);
    skaugen::response r;
    try {
        skaugen::step(dt_us, p, T, prec_mm_h, s, r);
    } catch (...) {
        return 1;
    }
    st[0] = s.nu; st[1] = s.alpha; st[2] = s.sca; st[3] = s.swe; st[4] = s.free_water; st[5] = s.residual;
    st[6] = double(s.num_units);
    resp[0] = r.outflow; resp[1] = r.sca; resp[2] = r.swe;
    return 0;
}

double oracle_skaugen_sca_rel_red(uint64_t u, uint64_t n, double nu_a, double alpha) {
    return skaugen::statistics::sca_rel_red(u, n, 0.0, nu_a, alpha);
}

// Run the pt_ss_k region model on the CPU with the reference scheduler.
//  params : n_sets x 21 (pt_ss_k.h:78-101 order); state : n_cells x 8 in/out
//  out_main : [2][T][N]; out_full : [8][T][N] (series-id order); out_state : [7][T+1][N]
int oracle_ptssk_run(size_t n_cells, const double* geo11, const double* params, size_t n_sets, const int32_t* set_ix,
                     double* state, int64_t t0_us, int64_t dt_us, size_t T, int start_step, int n_steps, const double* temp,
                     const double* prec, const double* ws, const double* rh, const double* rad, double* out_main,
                     double* out_full, double* out_state, int ncore, double* elapsed_s, char* err, size_t errlen) {
    try {
        ptssk_region rm;
        rm.time_axis = fixed_dt(t0_us, dt_us, T);
        rm.params.resize(n_sets);
        for (size_t k = 0; k < n_sets; ++k) rm.params[k].set(params + k * pt_ss_k::parameter::size());
        rm.cells.resize(n_cells);
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.geo = geo_cell_data::from_raw(geo11 + i * 11);
            int32_t k = set_ix ? set_ix[i] : 0;
            if (k < 0 || size_t(k) >= n_sets) return fail(err, errlen, "oracle_ptssk_run: parameter set index out of range");
            c.parameter = &rm.params[k];
            c.state.set(state + i * pt_ss_k::state::size());
            c.temp.resize(T); c.prec.resize(T); c.ws.resize(T); c.rh.resize(T); c.rad.resize(T);
            for (size_t t = 0; t < T; ++t) {
                c.temp[t] = temp[t * n_cells + i];
                c.prec[t] = prec[t * n_cells + i];
                c.ws[t] = ws[t * n_cells + i];
                c.rh[t] = rh[t * n_cells + i];
                c.rad[t] = rad[t * n_cells + i];
            }
            c.col.full = out_full != nullptr;
            c.col.collect_state = out_state != nullptr;
        }
        auto t_begin = std::chrono::steady_clock::now();
        rm.run_cells(size_t(ncore < 0 ? 0 : ncore), start_step, n_steps);
        auto t_end = std::chrono::steady_clock::now();
        if (elapsed_s) *elapsed_s = std::chrono::duration<double>(t_end - t_begin).count();
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.state.get(state + i * pt_ss_k::state::size());
            for (size_t t = 0; t < T; ++t) {
                if (out_main) {
                    out_main[t * n_cells + i] = c.col.rc[pt_ss_k::AVG_DISCHARGE][t];
                    out_main[(T + t) * n_cells + i] = c.col.rc[pt_ss_k::CHARGE_M3S][t];
                }
                if (out_full)
                    for (int k = 0; k < pt_ss_k::N_ALL; ++k) out_full[(size_t(k) * T + t) * n_cells + i] = c.col.rc[k][t];
            }
            if (out_state)
                for (int k = 0; k < pt_ss_k::N_SC; ++k)
                    for (size_t t = 0; t <= T; ++t) out_state[(size_t(k) * (T + 1) + t) * n_cells + i] = c.col.sc[k][t];
        }
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

}  // extern "C"

// Inverse-distance interpolation of one variable (kind: 0 temperature, 1 precipitation,
// 2 radiation, 3 wind_speed, 4 rel_hum). src_values [T][S], out [T][N].
// param: max_members, max_distance, distance_measure_factor, zscale, default_temp_gradient,
//        gradient_by_equation, precipitation scale_factor
extern "C" int oracle_idw_run(int kind, size_t S, const double* src_xyz, const double* src_values, size_t N,
                              const double* dst_xyz, const double* dst_slope, size_t T, const double* param, double* out) {
    idw::parameter p;
    p.max_members = size_t(param[0]);
    p.max_distance = param[1];
    p.distance_measure_factor = param[2];
    p.zscale = param[3];
    p.default_temp_gradient = param[4];
    p.gradient_by_equation = param[5] != 0.0;
    p.scale_factor = param[6];
    std::vector<std::vector<double>> vals(S, std::vector<double>(T));
    std::vector<idw::source> src(S);
    for (size_t s = 0; s < S; ++s) {
        for (size_t t = 0; t < T; ++t) vals[s][t] = src_values[t * S + s];
        src[s] = idw::source{geo_point(src_xyz[3 * s], src_xyz[3 * s + 1], src_xyz[3 * s + 2]), vals[s].data()};
    }
    std::vector<idw::destination> dst(N);
    for (size_t j = 0; j < N; ++j)
        dst[j] = idw::destination{geo_point(dst_xyz[3 * j], dst_xyz[3 * j + 1], dst_xyz[3 * j + 2]), dst_slope ? dst_slope[j] : 0.9};
    // destinations are independent: split over up to 16 threads (each writes its own columns of out)
    const size_t n_thr = std::min<size_t>({16, std::max(1u, std::thread::hardware_concurrency()), (N + 255) / 256});
    if (n_thr <= 1) {
        idw::run(idw::model_kind(kind), src, dst, T, p, out);
        return 0;
    }
    std::vector<std::thread> pool;
    for (size_t k = 0; k < n_thr; ++k)
        pool.emplace_back([&, k] { idw::run(idw::model_kind(kind), src, dst, T, p, out, N * k / n_thr, N * (k + 1) / n_thr); });
    for (auto& t : pool) t.join();
    return 0;
}

extern "C" double oracle_idw_temperature_gradient(size_t n, const double* xyz, const double* t, double default_gradient,
                                                  int by_equation) {
    std::vector<geo_point> pts;
    std::vector<double> tv;
    for (size_t i = 0; i < n; ++i) {
        pts.emplace_back(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
        tv.push_back(t[i]);
    }
    return idw::temperature_gradient(pts, tv, default_gradient, by_equation != 0);
}

extern "C" void oracle_gamma_pq(double a, double x, double* p, double* p1, double* prefix) {
    const auto r = special::gamma_pq(a, x);
    *p = r.p;
    *p1 = r.p1;
    *prefix = r.prefix;
}

// gamma_pq at gamma_snow's boost precision policy (digits10<10> for a < 2, digits10<5> otherwise,
// gamma_snow.h:189-197): the evaluation calc_snow_state and calc_q make
extern "C" void oracle_gamma_pq_policy(double a, double x, double* p, double* p1, double* prefix) {
    const auto r = special::gamma_pq(a, x, detmath::gamma_snow_policy_eps(a));
    *p = r.p;
    *p1 = r.p1;
    *prefix = r.prefix;
}

// ---------------------------------------------------------------- hbv_stack
// Snow distribution row per parameter set: n_bins, s[8], intervals[8] (17 doubles).
namespace {
hbv_snow::parameter snow_param(const double* tx_cx_ts_lw_cfr, const double* dist17) {
    hbv_snow::parameter p;
    if (dist17) {
        const size_t nb = size_t(dist17[0]);
        p.s.assign(dist17 + 1, dist17 + 1 + nb);
        p.intervals.assign(dist17 + 1 + hbv_stack::MAX_BINS, dist17 + 1 + hbv_stack::MAX_BINS + nb);
    }
    if (tx_cx_ts_lw_cfr) {
        p.tx = tx_cx_ts_lw_cfr[0]; p.cx = tx_cx_ts_lw_cfr[1]; p.ts = tx_cx_ts_lw_cfr[2];
        p.lw = tx_cx_ts_lw_cfr[3]; p.cfr = tx_cx_ts_lw_cfr[4];
    }
    return p;
}
}  // namespace

extern "C" {

double oracle_hbv_integrate(const double* f, const double* x, size_t n, double a, double b, int f_b_is_zero) {
    return hbv_snow::integrate(f, x, n, a, b, f_b_is_zero != 0);
}

// hbv_snow::calculator::step on one flat state (hbv_stack::FLAT order, snow part only used).
// distribute: 0 none, 1 state.distribute(p) (force), 2 distribute(p, false) (size mismatch only)
int oracle_hbv_snow_step(const double* tx_cx_ts_lw_cfr, const double* dist17, double* flat_state, int64_t t0_us,
                         int64_t t1_us, double prec, double temp, int distribute, double* outflow, char* err,
                         size_t errlen) {
    try {
        auto p = snow_param(tx_cx_ts_lw_cfr, dist17);
        hbv_stack::state s;
        s.set(flat_state);
        if (distribute) s.snow.distribute(p, distribute == 1);
        hbv_snow::response r;
        hbv_snow::calculator(p).step(s.snow, r, t0_us, t1_us, prec, temp);
        s.get(flat_state);
        *outflow = r.outflow;
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

void oracle_hbv_soil_step(double fc, double beta, double* sm, double insoil, double act_evap, double* outflow) {
    hbv_soil::parameter p{fc, beta};
    hbv_soil::state s{*sm};
    hbv_soil::response r;
    hbv_soil::step(p, s, r, insoil, act_evap);
    *sm = s.sm;
    *outflow = r.outflow;
}

void oracle_hbv_tank_step(const double* uz1_kuz2_kuz1_perc_klz, double* uz, double* lz, double soil_outflow,
                          double* outflow) {
    const double* q = uz1_kuz2_kuz1_perc_klz;
    hbv_tank::parameter p{q[0], q[1], q[2], q[3], q[4]};
    hbv_tank::state s{*uz, *lz};
    hbv_tank::response r;
    hbv_tank::step(p, s, r, soil_outflow);
    *uz = s.uz;
    *lz = s.lz;
    *outflow = r.outflow;
}

double oracle_hbv_ae(double sm, double pot, double lp, double snow_fraction) {
    return hbv_actual_evapotranspiration::calculate_step(sm, pot, lp, snow_fraction);
}

// Run the hbv_stack region model on the CPU with the reference scheduler.
//  params    : n_sets x 22 (hbv_stack.h:82-109 order)
//  snow_dist : n_sets x 17 (n_bins, s[8], intervals[8]) or null = default 5-bin distribution
//  state     : n_cells x 22 in/out (hbv_stack::FLAT order)
//  out_main  : [2][T][n_cells]; out_full : [9][T][n_cells]; out_state : [22][T+1][n_cells]
int oracle_hbv_run(size_t n_cells, const double* geo11, const double* params, const double* snow_dist, size_t n_sets,
                   const int32_t* set_ix, double* state, int64_t t0_us, int64_t dt_us, size_t T, int start_step,
                   int n_steps, const double* temp, const double* prec, const double* ws, const double* rh,
                   const double* rad, double* out_main, double* out_full, double* out_state, int ncore,
                   double* elapsed_s, char* err, size_t errlen) {
    try {
        hbv_region rm;
        rm.time_axis = fixed_dt(t0_us, dt_us, T);
        rm.params.resize(n_sets);
        for (size_t k = 0; k < n_sets; ++k) {
            rm.params[k].set(params + k * 22);
            auto sp = snow_param(nullptr, snow_dist ? snow_dist + k * 17 : nullptr);
            rm.params[k].snow.s = sp.s;
            rm.params[k].snow.intervals = sp.intervals;
        }
        rm.cells.resize(n_cells);
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.geo = geo_cell_data::from_raw(geo11 + i * 11);
            int32_t k = set_ix ? set_ix[i] : 0;
            if (k < 0 || size_t(k) >= n_sets) return fail(err, errlen, "oracle_hbv_run: parameter set index out of range");
            c.parameter = &rm.params[k];
            c.state.set(state + i * hbv_stack::FLAT);
            c.temp.resize(T); c.prec.resize(T); c.ws.resize(T); c.rh.resize(T); c.rad.resize(T);
            for (size_t t = 0; t < T; ++t) {
                c.temp[t] = temp[t * n_cells + i];
                c.prec[t] = prec[t * n_cells + i];
                c.ws[t] = ws[t * n_cells + i];
                c.rh[t] = rh[t * n_cells + i];
                c.rad[t] = rad[t * n_cells + i];
            }
            c.col.full = out_full != nullptr;
            c.col.collect_state = out_state != nullptr;
        }
        auto t_begin = std::chrono::steady_clock::now();
        rm.run_cells(size_t(ncore < 0 ? 0 : ncore), start_step, n_steps);
        auto t_end = std::chrono::steady_clock::now();
        if (elapsed_s) *elapsed_s = std::chrono::duration<double>(t_end - t_begin).count();
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.state.get(state + i * hbv_stack::FLAT);
            for (size_t t = 0; t < T; ++t) {
                if (out_main) {
                    out_main[t * n_cells + i] = c.col.rc[hbv_stack::AVG_DISCHARGE][t];
                    out_main[(T + t) * n_cells + i] = c.col.rc[hbv_stack::CHARGE_M3S][t];
                }
                if (out_full)
                    for (int k = 0; k < hbv_stack::N_ALL; ++k) out_full[(size_t(k) * T + t) * n_cells + i] = c.col.rc[k][t];
            }
            if (out_state)
                for (size_t k = 0; k < hbv_stack::FLAT; ++k)
                    for (size_t t = 0; t <= T; ++t) out_state[(k * (T + 1) + t) * n_cells + i] = c.col.sc[k][t];
        }
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

// Run the pt_hs_k region model on the CPU with the reference scheduler.
//  params    : n_sets x 18 (pt_hs_k.h:66-88 order); snow_dist : n_sets x 17 or null (default 5 bins)
//  state     : n_cells x 20 in/out (pt_hs_k::FLAT order)
//  out_main  : [2][T][n_cells]; out_full : [8][T][n_cells]; out_state : [19][T+1][n_cells]
int oracle_pthsk_run(size_t n_cells, const double* geo11, const double* params, const double* snow_dist, size_t n_sets,
                     const int32_t* set_ix, double* state, int64_t t0_us, int64_t dt_us, size_t T, int start_step,
                     int n_steps, const double* temp, const double* prec, const double* ws, const double* rh,
                     const double* rad, double* out_main, double* out_full, double* out_state, int ncore,
                     double* elapsed_s, char* err, size_t errlen) {
    try {
        pthsk_region rm;
        rm.time_axis = fixed_dt(t0_us, dt_us, T);
        rm.params.resize(n_sets);
        for (size_t k = 0; k < n_sets; ++k) {
            rm.params[k].set(params + k * pt_hs_k::parameter::size());
            auto sp = snow_param(nullptr, snow_dist ? snow_dist + k * 17 : nullptr);
            rm.params[k].hs.s = sp.s;
            rm.params[k].hs.intervals = sp.intervals;
        }
        rm.cells.resize(n_cells);
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.geo = geo_cell_data::from_raw(geo11 + i * 11);
            int32_t k = set_ix ? set_ix[i] : 0;
            if (k < 0 || size_t(k) >= n_sets) return fail(err, errlen, "oracle_pthsk_run: parameter set index out of range");
            c.parameter = &rm.params[k];
            c.state.set(state + i * pt_hs_k::FLAT);
            c.temp.resize(T); c.prec.resize(T); c.ws.resize(T); c.rh.resize(T); c.rad.resize(T);
            for (size_t t = 0; t < T; ++t) {
                c.temp[t] = temp[t * n_cells + i];
                c.prec[t] = prec[t * n_cells + i];
                c.ws[t] = ws[t * n_cells + i];
                c.rh[t] = rh[t * n_cells + i];
                c.rad[t] = rad[t * n_cells + i];
            }
            c.col.full = out_full != nullptr;
            c.col.collect_state = out_state != nullptr;
        }
        auto t_begin = std::chrono::steady_clock::now();
        rm.run_cells(size_t(ncore < 0 ? 0 : ncore), start_step, n_steps);
        auto t_end = std::chrono::steady_clock::now();
        if (elapsed_s) *elapsed_s = std::chrono::duration<double>(t_end - t_begin).count();
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.state.get(state + i * pt_hs_k::FLAT);
            for (size_t t = 0; t < T; ++t) {
                if (out_main) {
                    out_main[t * n_cells + i] = c.col.rc[pt_hs_k::AVG_DISCHARGE][t];
                    out_main[(T + t) * n_cells + i] = c.col.rc[pt_hs_k::CHARGE_M3S][t];
                }
                if (out_full)
                    for (int k = 0; k < pt_hs_k::N_ALL; ++k) out_full[(size_t(k) * T + t) * n_cells + i] = c.col.rc[k][t];
            }
            if (out_state)
                for (size_t k = 0; k < pt_hs_k::N_SC; ++k)
                    for (size_t t = 0; t <= T; ++t) out_state[(k * (T + 1) + t) * n_cells + i] = c.col.sc[k][t];
        }
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

// ---- hbv_physical_snow / pt_hps_k ----
// One hbv_physical_snow::calculator::step (hbv_physical_snow.h:291-553) on a flat hps state
// st36 = swe sca surface_heat n_bins sp[8] sw[8] albedo[8] iso_pot_energy[8]; p12 = tx lw cfr wind_scale wind_const
// surface_magnitude max_albedo min_albedo fast_decay slow_decay snowfall_reset_depth calculate_iso_pot_energy;
// dist17 = n_bins s[8] intervals[8] (normalised by the caller). distribute: 0 none, 1 force, 2 only on a size mismatch.
// resp = outflow sca storage. Returns 1 and the message on a throw.
int oracle_hps_step(double* st36, double* resp, const double* p12, const double* dist17, int distribute, int64_t dt_us,
                    double T, double rad, double prec_mm_h, double wind_speed, double rel_hum, char* err, size_t errlen) {
    hbv_physical_snow::parameter p;
    const size_t nb = size_t(dist17[0]);
    p.s.assign(dist17 + 1, dist17 + 1 + nb);
    p.intervals.assign(dist17 + 1 + pt_hps_k::MB, dist17 + 1 + pt_hps_k::MB + nb);
    p.tx = p12[0]; p.lw = p12[1]; p.cfr = p12[2]; p.wind_scale = p12[3]; p.wind_const = p12[4];
    p.surface_magnitude = p12[5]; p.max_albedo = p12[6]; p.min_albedo = p12[7]; p.fast_albedo_decay_rate = p12[8];
    p.slow_albedo_decay_rate = p12[9]; p.snowfall_reset_depth = p12[10]; p.calculate_iso_pot_energy = p12[11] != 0.0;
    pt_hps_k::state s;
    std::vector<double> flat(pt_hps_k::FLAT, 0.0);
    std::copy(st36, st36 + pt_hps_k::FLAT - 1, flat.begin());
    s.set(flat.data());
    try {
        if (distribute) s.hps.distribute(p, distribute == 1);
        hbv_physical_snow::calculator c(p);
        hbv_physical_snow::response r;
        c.step(s.hps, r, dt_us, T, rad, prec_mm_h, wind_speed, rel_hum);
        resp[0] = r.outflow; resp[1] = r.sca; resp[2] = r.storage;
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    s.get(flat.data());
    std::copy(flat.begin(), flat.end() - 1, st36);
    return 0;
}

// Run the pt_hps_k region model on the CPU with the reference scheduler.
//  params : n_sets x 24 (pt_hps_k.h:64-90 order); gm_direct : n_sets or null (glacier_melt::parameter default 0);
//  snow_dist : n_sets x 17 or null (default 5 bins); state : n_cells x 37 in/out (pt_hps_k::FLAT order)
//  out_main : [2][T][N]; out_full : [8][T][N]; out_state : [36][T+1][N]
int oracle_pthpsk_run(size_t n_cells, const double* geo11, const double* params, const double* gm_direct,
                      const double* snow_dist, size_t n_sets, const int32_t* set_ix, double* state, int64_t t0_us,
                      int64_t dt_us, size_t T, int start_step, int n_steps, const double* temp, const double* prec,
                      const double* ws, const double* rh, const double* rad, double* out_main, double* out_full,
                      double* out_state, int ncore, double* elapsed_s, char* err, size_t errlen) {
    try {
        pthpsk_region rm;
        rm.time_axis = fixed_dt(t0_us, dt_us, T);
        rm.params.resize(n_sets);
        for (size_t k = 0; k < n_sets; ++k) {
            rm.params[k].set(params + k * pt_hps_k::parameter::size());
            if (gm_direct) rm.params[k].gm.direct_response = gm_direct[k];
            if (snow_dist) {
                const double* d = snow_dist + k * 17;
                const size_t nb = size_t(d[0]);
                rm.params[k].hps.s.assign(d + 1, d + 1 + nb);
                rm.params[k].hps.intervals.assign(d + 1 + pt_hps_k::MB, d + 1 + pt_hps_k::MB + nb);
            }
        }
        rm.cells.resize(n_cells);
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.geo = geo_cell_data::from_raw(geo11 + i * 11);
            int32_t k = set_ix ? set_ix[i] : 0;
            if (k < 0 || size_t(k) >= n_sets) return fail(err, errlen, "oracle_pthpsk_run: parameter set index out of range");
            c.parameter = &rm.params[k];
            c.state.set(state + i * pt_hps_k::FLAT);
            c.temp.resize(T); c.prec.resize(T); c.ws.resize(T); c.rh.resize(T); c.rad.resize(T);
            for (size_t t = 0; t < T; ++t) {
                c.temp[t] = temp[t * n_cells + i];
                c.prec[t] = prec[t * n_cells + i];
                c.ws[t] = ws[t * n_cells + i];
                c.rh[t] = rh[t * n_cells + i];
                c.rad[t] = rad[t * n_cells + i];
            }
            c.col.full = out_full != nullptr;
            c.col.collect_state = out_state != nullptr;
        }
        auto t_begin = std::chrono::steady_clock::now();
        rm.run_cells(size_t(ncore < 0 ? 0 : ncore), start_step, n_steps);
        auto t_end = std::chrono::steady_clock::now();
        if (elapsed_s) *elapsed_s = std::chrono::duration<double>(t_end - t_begin).count();
        for (size_t i = 0; i < n_cells; ++i) {
            auto& c = rm.cells[i];
            c.state.get(state + i * pt_hps_k::FLAT);
            for (size_t t = 0; t < T; ++t) {
                if (out_main) {
                    out_main[t * n_cells + i] = c.col.rc[pt_hps_k::AVG_DISCHARGE][t];
                    out_main[(T + t) * n_cells + i] = c.col.rc[pt_hps_k::CHARGE_M3S][t];
                }
                if (out_full)
                    for (int k = 0; k < pt_hps_k::N_ALL; ++k) out_full[(size_t(k) * T + t) * n_cells + i] = c.col.rc[k][t];
            }
            if (out_state)
                for (size_t k = 0; k < pt_hps_k::N_SC; ++k)
                    for (size_t t = 0; t <= T; ++t) out_state[(k * (T + 1) + t) * n_cells + i] = c.col.sc[k][t];
        }
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

}  // extern "C"

// routing::model query (core/routing.h:347-387) for river `query`: local, upstream, output [T].
//  q [T][N] avg_discharge; per cell: routing id, distance, (velocity, alpha, beta) of its parameter;
//  per river: id, downstream id, downstream distance, (velocity, alpha, beta).
#include "routing.hpp"
extern "C" int oracle_route(size_t n_cells, size_t T, int64_t dt_us, const double* q, const int64_t* cell_rid,
                            const double* cell_dist, const double* cell_vab, size_t n_rivers, const int64_t* rid,
                            const int64_t* ds, const double* rdist, const double* rvab, int64_t query, double* local,
                            double* upstream, double* output) {
    try {
        routing::model m;
        m.T = T;
        m.dt_us = dt_us;
        for (size_t r = 0; r < n_rivers; ++r)
            m.rivers[rid[r]] = routing::river{rid[r], ds[r], rdist[r], rvab[3 * r], rvab[3 * r + 1], rvab[3 * r + 2]};
        for (size_t i = 0; i < n_cells; ++i)
            if (cell_rid[i] > 0)
                m.cells.push_back(routing::cell_route{cell_rid[i], cell_dist[i], cell_vab[3 * i], cell_vab[3 * i + 1],
                                                      cell_vab[3 * i + 2], q + i, n_cells});
        auto a = m.local_inflow(query);
        auto b = m.upstream_inflow(query);
        auto c = m.output(query);
        std::copy(a.begin(), a.end(), local);
        std::copy(b.begin(), b.end(), upstream);
        std::copy(c.begin(), c.end(), output);
    } catch (...) {
        return 1;
    }
    return 0;
}

extern "C" void oracle_make_uhg(int n_steps, double alpha, double beta, double* out, int* len) {
    auto w = routing::make_uhg_from_gamma(n_steps, alpha, beta);
    std::copy(w.begin(), w.end(), out);
    *len = int(w.size());
}

// ---- Bayesian temperature kriging (core/bayesian_kriging.h:280-402) -------------------------------------------------
#include "btk.hpp"

// param: gradient_sd (already /100), sill, nugget, range, zscale. src_values [T][S], prior_gradient [T], out [T][D].
extern "C" int oracle_btk_run(size_t S, const double* src_xyz, const double* src_values, size_t T,
                              const double* prior_gradient, const double* param, size_t D, const double* dst_xyz,
                              double* out, char* err, size_t errlen) {
    btk::parameter p;
    p.gradient_sd = param[0];
    p.sill = param[1];
    p.nug = param[2];
    p.range = param[3];
    p.zscale = param[4];
    try {
        btk::run(S, src_xyz, src_values, T, prior_gradient, p, D, dst_xyz, out);
    } catch (const std::exception& e) {
        return fail(err, errlen, e.what());
    }
    return 0;
}

// the source-source covariance matrix K (utils::build_covariance_matrices, bayesian_kriging.h:93-113), out [S][S]
extern "C" void oracle_btk_source_covariance(size_t S, const double* xyz, const double* param, double* out) {
    btk::parameter p;
    p.gradient_sd = param[0];
    p.sill = param[1];
    p.nug = param[2];
    p.range = param[3];
    p.zscale = param[4];
    const auto K = btk::source_covariance(S, xyz, p);
    std::copy(K.a.begin(), K.a.end(), out);
}
