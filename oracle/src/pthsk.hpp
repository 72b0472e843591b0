// ORACLE — test infrastructure only (see common.hpp header).
//
// pthsk.hpp: the pt_hs_k method stack (core/pt_hs_k.h:199-283) and its collectors
// (core/pt_hs_k_cell_model.h:41-210): Priestley-Taylor, hbv_snow (hbv.hpp), actual
// evapotranspiration and kirchner (methods.hpp / ptgsk.hpp). Every arithmetic expression
// keeps the reference's operand order.
#pragma once
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "hbv.hpp"
#include "methods.hpp"
#include "ptgsk.hpp"

namespace oracle {
namespace pt_hs_k {

// core/pt_hs_k.h:29-145 (18 calibration values)
struct parameter {
    priestley_taylor::parameter pt;
    hbv_snow::parameter hs;
    actual_evapotranspiration::parameter ae;
    kirchner::parameter kirchner;
    precipitation_correction::parameter p_corr;
    glacier_melt::parameter gm;
    pt_gs_k::uhg_parameter routing;
    pt_gs_k::mstack_parameter msp;
    static constexpr size_t size() { return 18; }
    void set(const double* p) {  // pt_hs_k.h:66-88
        int i = 0;
        kirchner.c1 = p[i++]; kirchner.c2 = p[i++]; kirchner.c3 = p[i++];
        ae.ae_scale_factor = p[i++];
        hs.lw = p[i++]; hs.tx = p[i++]; hs.cx = p[i++]; hs.ts = p[i++]; hs.cfr = p[i++];
        gm.dtf = p[i++];
        p_corr.scale_factor = p[i++];
        pt.albedo = p[i++]; pt.alpha = p[i++];
        routing.velocity = p[i++]; routing.alpha = p[i++]; routing.beta = p[i++];
        gm.direct_response = p[i++];
        msp.reservoir_direct_response_fraction = p[i++];
    }
};

// core/pt_hs_k.h:148-172; flat order swe sca n_bins sp[8] sw[8] kirchner.q
constexpr size_t MAX_BINS = hbv_stack::MAX_BINS;
constexpr size_t FLAT = 3 + 2 * MAX_BINS + 1;
struct state {
    hbv_snow::state snow;
    kirchner::state kirchner;
    void set(const double* v) {
        snow.swe = v[0]; snow.sca = v[1];
        const size_t nb = size_t(v[2]);
        snow.sp.assign(v + 3, v + 3 + nb);
        snow.sw.assign(v + 3 + MAX_BINS, v + 3 + MAX_BINS + nb);
        kirchner.q = v[3 + 2 * MAX_BINS];
    }
    void get(double* v) const {
        v[0] = snow.swe; v[1] = snow.sca; v[2] = double(snow.sp.size());
        for (size_t i = 0; i < MAX_BINS; ++i) {
            v[3 + i] = i < snow.sp.size() ? snow.sp[i] : 0.0;
            v[3 + MAX_BINS + i] = i < snow.sw.size() ? snow.sw[i] : 0.0;
        }
        v[3 + 2 * MAX_BINS] = kirchner.q;
    }
    state scale_snow(double f) const {  // pt_hs_k.h:165-169
        state c{*this};
        c.snow.swe *= f;
        return c;
    }
};

// core/pt_hs_k.h:174-195
struct response {
    double pot_evapotranspiration = 0;
    hbv_snow::response snow;
    double ae = 0, q_avg = 0, gm_melt_m3s = 0, total_discharge = 0, charge_m3s = 0;
    response scale_snow(double f) const {
        response c{*this};
        c.snow.snow_state.swe *= f;
        c.snow.outflow *= f;
        return c;
    }
};

// Collector series in this repo's series-id order (the discharge collector is the prefix):
// avg_discharge, charge_m3s, snow_sca, snow_swe, snow_outflow, glacier_melt, ae_output, pe_output
enum all_series { AVG_DISCHARGE = 0, CHARGE_M3S, SNOW_SCA, SNOW_SWE, SNOW_OUTFLOW, GLACIER_MELT, AE_OUTPUT, PE_OUTPUT, N_ALL };
// state collector (pt_hs_k_cell_model.h:148-210): kirchner_discharge, snow_sca, snow_swe, sp[8], sw[8]
constexpr size_t N_SC = 3 + 2 * MAX_BINS;

struct collectors {
    bool full = true, collect_snow = false, collect_state = false;
    double area = 0;
    std::vector<double> rc[N_ALL];
    std::vector<double> sc[N_SC];
    void initialize(size_t T, int start, int n, double a) {
        area = a;
        for (int k = 0; k < N_ALL; ++k) {
            bool on = full || k == AVG_DISCHARGE || k == CHARGE_M3S || (collect_snow && (k == SNOW_SCA || k == SNOW_SWE));
            pt_gs_k::collectors::ts_init(rc[k], on ? T : 0, start, n);
        }
        for (size_t k = 0; k < N_SC; ++k) pt_gs_k::collectors::ts_init(sc[k], collect_state ? T + 1 : 0, start, n > 0 ? n + 1 : 0);
    }
    void collect_response(size_t i, const response& r) {
        rc[AVG_DISCHARGE][i] = mmh_to_m3s(r.total_discharge, area);
        rc[CHARGE_M3S][i] = r.charge_m3s;
        if (full || collect_snow) {
            rc[SNOW_SCA][i] = r.snow.snow_state.sca;
            rc[SNOW_SWE][i] = r.snow.snow_state.swe;
        }
        if (full) {
            rc[SNOW_OUTFLOW][i] = mmh_to_m3s(r.snow.outflow, area);
            rc[GLACIER_MELT][i] = r.gm_melt_m3s;
            rc[AE_OUTPUT][i] = r.ae;
            rc[PE_OUTPUT][i] = r.pot_evapotranspiration;
        }
    }
    void collect_state_(size_t i, const state& s) {
        if (!collect_state) return;
        sc[0][i] = mmh_to_m3s(s.kirchner.q, area);
        sc[1][i] = s.snow.sca;
        sc[2][i] = s.snow.swe;
        for (size_t k = 0; k < MAX_BINS; ++k) {  // the bins beyond n_bins are collected as 0 here
            sc[3 + k][i] = k < s.snow.sp.size() ? s.snow.sp[k] : 0.0;
            sc[3 + MAX_BINS + k][i] = k < s.snow.sw.size() ? s.snow.sw[k] : 0.0;
        }
    }
};

// core/pt_hs_k.h:199-283
inline void run_pt_hs_k(const geo_cell_data& geo, const parameter& parameter, const fixed_dt& time_axis, int start_step,
                        int n_steps, const pt_gs_k::forcing_view& fv, state& state, collectors& col) {
    priestley_taylor::calculator pt(parameter.pt.albedo, parameter.pt.alpha);
    hbv_snow::calculator hbv_snow(parameter.hs);
    kirchner::calculator kirchner(parameter.kirchner);
    state.snow.distribute(parameter.hs, false);
    response response;
    const auto& ltf = geo.fractions;
    const double glacier_fraction = ltf.glacier();
    const double gm_direct = parameter.gm.direct_response;
    const double gm_routed = 1 - gm_direct;
    const double snow_storage_fraction = ltf.snow_storage();
    const double kirchner_routed_prec = ltf.reservoir() * (1.0 - parameter.msp.reservoir_direct_response_fraction) + ltf.lake();
    const double direct_response_fraction = glacier_fraction * gm_direct + ltf.reservoir() * parameter.msp.reservoir_direct_response_fraction;
    const double kirchner_fraction = 1 - direct_response_fraction;
    const double cell_area_m2 = geo.area;
    const double glacier_area_m2 = geo.area * glacier_fraction;
    size_t i_begin = n_steps > 0 ? size_t(start_step) : 0;
    size_t i_end = n_steps > 0 ? size_t(start_step + n_steps) : time_axis.size();
    for (size_t i = i_begin; i < i_end; ++i) {
        const utctime t0 = time_axis.time(i), t1 = t0 + time_axis.dt;
        double temp = fv.temp[i * fv.stride];
        double rad = fv.rad[i * fv.stride];
        double rel_hum = fv.rh[i * fv.stride];
        double prec = fv.prec[i * fv.stride] * parameter.p_corr.scale_factor;
        col.collect_state_(i, state.scale_snow(snow_storage_fraction));
        hbv_snow.step(state.snow, response.snow, t0, t1, prec, temp);
        response.gm_melt_m3s = glacier_melt::step(parameter.gm.dtf, temp, cell_area_m2 * state.snow.sca, glacier_area_m2);
        response.pot_evapotranspiration = pt.potential_evapotranspiration(temp, rad, rel_hum) * to_seconds(HOUR_US);
        response.ae = actual_evapotranspiration::calculate_step(state.kirchner.q, response.pot_evapotranspiration,
                                                                parameter.ae.ae_scale_factor,
                                                                std::max(state.snow.sca, glacier_fraction));
        double gm_mmh = m3s_to_mmh(response.gm_melt_m3s, cell_area_m2);
        kirchner.step(t0, t1, state.kirchner.q, response.q_avg,
                      response.snow.outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                      response.ae);
        response.total_discharge = std::max(0.0, prec - response.ae) * direct_response_fraction + gm_direct * gm_mmh +
                                   response.q_avg * kirchner_fraction;
        response.charge_m3s = +mmh_to_m3s(prec, cell_area_m2) - mmh_to_m3s(response.ae, cell_area_m2) + response.gm_melt_m3s -
                              mmh_to_m3s(response.total_discharge, cell_area_m2);
        response.snow.snow_state = state.snow;  // pt_hs_k.h:274
        col.collect_response(i, response.scale_snow(snow_storage_fraction));
        if (i + 1 == i_end) col.collect_state_(i + 1, state.scale_snow(snow_storage_fraction));
    }
}

}  // namespace pt_hs_k
}  // namespace oracle
