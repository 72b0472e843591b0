// ORACLE — test infrastructure only (see common.hpp header).
//
// ptgsk.hpp: the pt_gs_k method stack (core/pt_gs_k.h) and its collectors
// (core/pt_gs_k_cell_model.h).
#pragma once
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "methods.hpp"

namespace oracle {
namespace pt_gs_k {

// routing::uhg_parameter (core/routing.h:75-80) and mstack_parameter (core/mstack_param.h)
struct uhg_parameter { double velocity = 1.0, alpha = 7.0, beta = 0.0; };
struct mstack_parameter { double reservoir_direct_response_fraction = 1.0; };

// core/pt_gs_k.h:39-194
struct parameter {
    priestley_taylor::parameter pt;
    gamma_snow::parameter gs;
    actual_evapotranspiration::parameter ae;
    kirchner::parameter kirchner;
    precipitation_correction::parameter p_corr;
    glacier_melt::parameter gm;
    uhg_parameter routing;
    mstack_parameter msp;
    static constexpr size_t size() { return 31; }
    // get/set order: pt_gs_k.h:77-112
    void set(const double* p) {
        int i = 0;
        kirchner.c1 = p[i++]; kirchner.c2 = p[i++]; kirchner.c3 = p[i++];
        ae.ae_scale_factor = p[i++];
        gs.tx = p[i++]; gs.wind_scale = p[i++]; gs.max_water = p[i++]; gs.wind_const = p[i++];
        gs.fast_albedo_decay_rate = p[i++]; gs.slow_albedo_decay_rate = p[i++]; gs.surface_magnitude = p[i++];
        gs.max_albedo = p[i++]; gs.min_albedo = p[i++]; gs.snowfall_reset_depth = p[i++]; gs.snow_cv = p[i++];
        gs.glacier_albedo = p[i++];
        p_corr.scale_factor = p[i++];
        gs.snow_cv_forest_factor = p[i++]; gs.snow_cv_altitude_factor = p[i++];
        pt.albedo = p[i++]; pt.alpha = p[i++];
        gs.initial_bare_ground_fraction = p[i++];
        gs.winter_end_day_of_year = int64_t(size_t(p[i++]));
        gs.calculate_iso_pot_energy = p[i++] != 0.0;
        gm.dtf = p[i++];
        routing.velocity = p[i++]; routing.alpha = p[i++]; routing.beta = p[i++];
        gs.n_winter_days = int64_t(p[i++]);
        gm.direct_response = p[i++];
        msp.reservoir_direct_response_fraction = p[i++];
    }
    void get(double* p) const {
        int i = 0;
        p[i++] = kirchner.c1; p[i++] = kirchner.c2; p[i++] = kirchner.c3;
        p[i++] = ae.ae_scale_factor;
        p[i++] = gs.tx; p[i++] = gs.wind_scale; p[i++] = gs.max_water; p[i++] = gs.wind_const;
        p[i++] = gs.fast_albedo_decay_rate; p[i++] = gs.slow_albedo_decay_rate; p[i++] = gs.surface_magnitude;
        p[i++] = gs.max_albedo; p[i++] = gs.min_albedo; p[i++] = gs.snowfall_reset_depth; p[i++] = gs.snow_cv;
        p[i++] = gs.glacier_albedo;
        p[i++] = p_corr.scale_factor;
        p[i++] = gs.snow_cv_forest_factor; p[i++] = gs.snow_cv_altitude_factor;
        p[i++] = pt.albedo; p[i++] = pt.alpha;
        p[i++] = gs.initial_bare_ground_fraction;
        p[i++] = double(gs.winter_end_day_of_year);
        p[i++] = gs.calculate_iso_pot_energy ? 1.0 : 0.0;
        p[i++] = gm.dtf;
        p[i++] = routing.velocity; p[i++] = routing.alpha; p[i++] = routing.beta;
        p[i++] = double(gs.n_winter_days);
        p[i++] = gm.direct_response;
        p[i++] = msp.reservoir_direct_response_fraction;
    }
};

// core/pt_gs_k.h:204-226; SoA field order used by every C-ABI in this repo
struct state {
    gamma_snow::state gs;
    kirchner::state kirchner;
    static constexpr size_t size() { return 9; }
    void set(const double* v) {
        gs.albedo = v[0]; gs.lwc = v[1]; gs.surface_heat = v[2]; gs.alpha = v[3]; gs.sdc_melt_mean = v[4];
        gs.acc_melt = v[5]; gs.iso_pot_energy = v[6]; gs.temp_swe = v[7]; kirchner.q = v[8];
    }
    void get(double* v) const {
        v[0] = gs.albedo; v[1] = gs.lwc; v[2] = gs.surface_heat; v[3] = gs.alpha; v[4] = gs.sdc_melt_mean;
        v[5] = gs.acc_melt; v[6] = gs.iso_pot_energy; v[7] = gs.temp_swe; v[8] = kirchner.q;
    }
    state scale_snow(double f) const {
        state c{*this};
        c.gs.temp_swe *= f;
        c.gs.lwc *= f;
        return c;
    }
};

// core/pt_gs_k.h:233-255
struct response {
    double pot_evapotranspiration = 0;
    gamma_snow::response gs;
    double ae = 0;
    double q_avg = 0;
    double gm_melt_m3s = 0;
    double total_discharge = 0;
    double charge_m3s = 0;
    response scale_snow(double f) const {
        response c{*this};
        c.gs.storage *= f;
        c.gs.outflow *= f;
        return c;
    }
};

// Collector outputs, [T] series per cell. Layout of the full ("all") collector
// (pt_gs_k_cell_model.h:41-98): avg_discharge, charge_m3s, snow_sca, snow_swe,
// snow_outflow, glacier_melt, ae_output, pe_output.
enum all_series { AVG_DISCHARGE = 0, CHARGE_M3S, SNOW_SCA, SNOW_SWE, SNOW_OUTFLOW, GLACIER_MELT, AE_OUTPUT, PE_OUTPUT, N_ALL };

struct collectors {
    bool full = true;            // all_response_collector vs discharge_collector
    bool collect_snow = false;   // discharge_collector::collect_snow
    bool collect_state = false;  // state_collector::collect_state
    double area = 0;
    std::vector<double> rc[N_ALL];
    std::vector<double> sc[9];   // state collector (T+1): kirchner_discharge (m3/s), gs_* (pt_gs_k_cell_model.h:125-196)
    response end_response;

    static void ts_init(std::vector<double>& v, size_t n, int start, int n_steps) {
        if (v.size() != n || n == 0) v.assign(n, nan);
        else {
            size_t e = n_steps > 0 ? size_t(start + n_steps) : n;
            for (size_t i = size_t(n_steps > 0 ? start : 0); i < e && i < n; ++i) v[i] = nan;
        }
    }
    // begin_run (cell_model.h:135-138)
    void initialize(size_t T, int start, int n, double a) {
        area = a;
        for (int k = 0; k < N_ALL; ++k) {
            bool on = full || k == AVG_DISCHARGE || k == CHARGE_M3S || (collect_snow && (k == SNOW_SCA || k == SNOW_SWE));
            ts_init(rc[k], on ? T : 0, start, n);
        }
        for (int k = 0; k < 9; ++k) ts_init(sc[k], collect_state ? T + 1 : 0, start, n > 0 ? n + 1 : 0);
    }
    void collect_response(size_t i, const response& r) {
        rc[AVG_DISCHARGE][i] = mmh_to_m3s(r.total_discharge, area);
        rc[CHARGE_M3S][i] = r.charge_m3s;
        if (full || collect_snow) {
            rc[SNOW_SCA][i] = r.gs.sca;
            rc[SNOW_SWE][i] = r.gs.storage;
        }
        if (full) {
            rc[SNOW_OUTFLOW][i] = mmh_to_m3s(r.gs.outflow, area);
            rc[GLACIER_MELT][i] = r.gm_melt_m3s;
            rc[AE_OUTPUT][i] = r.ae;
            rc[PE_OUTPUT][i] = r.pot_evapotranspiration;
        }
    }
    void collect_state_(size_t i, const state& s) {
        if (!collect_state) return;
        sc[0][i] = mmh_to_m3s(s.kirchner.q, area);
        sc[1][i] = s.gs.albedo; sc[2][i] = s.gs.lwc; sc[3][i] = s.gs.surface_heat; sc[4][i] = s.gs.alpha;
        sc[5][i] = s.gs.sdc_melt_mean; sc[6][i] = s.gs.acc_melt; sc[7][i] = s.gs.iso_pot_energy; sc[8][i] = s.gs.temp_swe;
    }
};

// forcing accessor: direct_accessor over the cell env_ts (time_series.h:2137-2196)
struct forcing_view {
    const double* temp; const double* prec; const double* ws; const double* rh; const double* rad;
    size_t stride;  // element i of the series is at [i*stride]
};

// core/pt_gs_k.h:312-398
inline void run_pt_gs_k(const geo_cell_data& geo, const parameter& parameter, const fixed_dt& time_axis, int start_step,
                        int n_steps, const forcing_view& fv, state& state, collectors& col) {
    priestley_taylor::calculator pt(parameter.pt.albedo, parameter.pt.alpha);
    gamma_snow::calculator gs;
    kirchner::calculator kirchner(parameter.kirchner);
    response response;
    const auto& ltf = geo.fractions;
    const double forest_fraction = ltf.forest();
    const double glacier_fraction = ltf.glacier();
    const double gm_direct = parameter.gm.direct_response;
    const double gm_routed = 1 - gm_direct;
    const double snow_storage_fraction = ltf.snow_storage();
    const double kirchner_routed_prec = ltf.reservoir() * (1.0 - parameter.msp.reservoir_direct_response_fraction) + ltf.lake();
    const double direct_response_fraction = glacier_fraction * gm_direct + ltf.reservoir() * parameter.msp.reservoir_direct_response_fraction;
    const double kirchner_fraction = 1 - direct_response_fraction;
    const double cell_area_m2 = geo.area;
    const double glacier_area_m2 = geo.area * glacier_fraction;
    const double altitude = geo.mid_point.z;
    size_t i_begin = n_steps > 0 ? size_t(start_step) : 0;
    size_t i_end = n_steps > 0 ? size_t(start_step + n_steps) : time_axis.size();
    for (size_t i = i_begin; i < i_end; ++i) {
        const utctime t0 = time_axis.time(i), t1 = t0 + time_axis.dt;
        const int64_t dt = t1 - t0;
        double temp = fv.temp[i * fv.stride];
        double rad = fv.rad[i * fv.stride];
        double rel_hum = fv.rh[i * fv.stride];
        double prec = fv.prec[i * fv.stride] * parameter.p_corr.scale_factor;
        col.collect_state_(i, state.scale_snow(snow_storage_fraction));
        gs.step(state.gs, response.gs, t0, dt, parameter.gs, temp, rad, prec, fv.ws[i * fv.stride], rel_hum, forest_fraction,
                altitude);
        response.gm_melt_m3s = glacier_melt::step(parameter.gm.dtf, temp, cell_area_m2 * response.gs.sca, glacier_area_m2);
        response.pot_evapotranspiration = pt.potential_evapotranspiration(temp, rad, rel_hum) * to_seconds(HOUR_US);
        response.ae = actual_evapotranspiration::calculate_step(state.kirchner.q, response.pot_evapotranspiration,
                                                                parameter.ae.ae_scale_factor,
                                                                std::max(response.gs.sca, glacier_fraction));
        double gm_mmh = m3s_to_mmh(response.gm_melt_m3s, cell_area_m2);
        kirchner.step(t0, t1, state.kirchner.q, response.q_avg,
                      response.gs.outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh, response.ae);
        response.total_discharge = std::max(0.0, prec - response.ae) * direct_response_fraction + gm_direct * gm_mmh +
                                   response.q_avg * kirchner_fraction;
        response.charge_m3s = +mmh_to_m3s(prec, cell_area_m2) - mmh_to_m3s(response.ae, cell_area_m2) + response.gm_melt_m3s -
                              mmh_to_m3s(response.total_discharge, cell_area_m2);
        col.collect_response(i, response.scale_snow(snow_storage_fraction));
        if (i + 1 == i_end) col.collect_state_(i + 1, state.scale_snow(snow_storage_fraction));
    }
    col.end_response = response.scale_snow(snow_storage_fraction);
}

}  // namespace pt_gs_k
}  // namespace oracle
