// ORACLE — test infrastructure only (see common.hpp header).
//
// pthpsk.hpp: hbv_physical_snow (core/hbv_physical_snow.h:41-554) and the pt_hps_k method stack
// (core/pt_hps_k.h:199-300) with the collectors of core/pt_hps_k_cell_model.h. Every arithmetic
// expression keeps the reference's operand order, including its quirks: the step works on a local copy
// of albedo and surface_heat that is never written back (only the no-snow reset changes them), the
// snowfall branch sets sca from the redistribution factors s[], and the melt-front interpolation assigns
// sp[idx-1] = sp[idx] inside its denominator (hbv_physical_snow.h:511-513).
#pragma once
#include <algorithm>
#include <cmath>
#include <sstream>
#include <stdexcept>
#include <vector>

#include "common.hpp"
#include "hbv.hpp"
#include "methods.hpp"
#include "ptgsk.hpp"

namespace oracle {
namespace hbv_physical_snow {

constexpr double tol = 1.0e-10;  // hbv_physical_snow.h:39

// hbv_physical_snow.h:41-132
struct parameter {
    std::vector<double> s, intervals;
    double tx = 0.0, lw = 0.1, cfr = 0.5, wind_scale = 2.0, wind_const = 1.0, surface_magnitude = 30.0,
           max_albedo = 0.9, min_albedo = 0.6, fast_albedo_decay_rate = 5.0, slow_albedo_decay_rate = 5.0,
           snowfall_reset_depth = 5.0;
    bool calculate_iso_pot_energy = false;
    parameter() {
        s = {1.0, 1.0, 1.0, 1.0, 1.0};
        intervals = {0, 0.25, 0.5, 0.75, 1.0};
        const double mean = hbv_snow::integrate(s, intervals, intervals.size(), intervals[0], intervals.back());
        for (auto& v : s) v /= mean;
    }
};

// hbv_physical_snow.h:135-190
struct state {
    std::vector<double> sp, sw, albedo, iso_pot_energy;
    double surface_heat = 30000.0, swe = 0.0, sca = 0.0;
    void distribute(const parameter& p, bool force = true) {
        if (force || sp.size() != p.s.size() || sw.size() != p.s.size()) {
            hbv_snow::parameter hp(p.s, p.intervals);
            hp.lw = p.lw;
            hbv_snow::state hs;
            hs.sp = sp; hs.sw = sw; hs.swe = swe; hs.sca = sca;
            hs.distribute(hp, true);  // distribute_snow (hbv_snow_common.h:47-66)
            sp = hs.sp; sw = hs.sw; swe = hs.swe; sca = hs.sca;
        }
        if (sp.size() != albedo.size()) {
            albedo.assign(sp.size(), 0.4);
            iso_pot_energy.assign(sp.size(), 0.0);
        }
    }
};

struct response {
    double sca = 0.0, storage = 0.0, outflow = 0.0;
};

// hbv_physical_snow.h:227-553
struct calculator {
    const parameter& p;
    const double melt_heat = 333660.0, water_heat = 4180.0, ice_heat = 2050.0, sigma = 5.670373e-8;
    const double BB0 = 0.98 * sigma * OPOW(273.15, 4);
    explicit calculator(const parameter& p_) : p(p_) {}

    static void refreeze(double& sp, double& sw, double rain, double potmelt, double lw) {
        if (sp > 0.0) {
            if (sw + rain > -potmelt) {
                sp -= potmelt;
                sw += potmelt + rain;
                if (sw > sp * lw) sw = sp * lw;
            } else {
                sp += sw + rain;
                sw = 0.0;
            }
        }
    }
    static void update_state(double& sp, double& sw, double rain, double potmelt, double lw) {
        if (sp > potmelt) {
            sw += potmelt + rain;
            sp -= potmelt;
            sw = std::min(sw, sp * lw);
        } else if (sp > 0.0) {
            sp = sw = 0.0;
        }
    }
    size_t sca_index(double sca) const {
        for (size_t i = 0; i < p.intervals.size() - 1; ++i)
            if (sca >= p.intervals[i] && sca < p.intervals[i + 1]) return i;
        return p.intervals.size() - 1;
    }

    void step(state& s, response& r, int64_t dt_us, double T, double rad, double prec_mm_h, double wind_speed,
              double rel_hum) const {
        const auto& I = p.intervals;
        const size_t n = I.size();
        const double dts = double(dt_us) / 1e6;  // to_seconds(dt)
        const double prec = prec_mm_h * double(dt_us) / 3600000000.0;  // prec_mm_h*dt/calendar::HOUR
        const double total_water = prec + s.swe;
        double snow, rain;
        if (T < p.tx) { snow = prec; rain = 0.0; }
        else          { snow = 0.0; rain = prec; }
        s.swe += snow + s.sca * rain;
        if (s.swe < tol) {
            r.outflow = total_water;
            std::fill(s.sp.begin(), s.sp.end(), 0.0);
            std::fill(s.sw.begin(), s.sw.end(), 0.0);
            s.swe = 0.0;
            s.sca = 0.0;
            r.sca = 0.0;
            r.storage = 0.0;
            std::fill(s.albedo.begin(), s.albedo.end(), p.max_albedo);
            s.surface_heat = 0.0;
            std::fill(s.iso_pot_energy.begin(), s.iso_pot_energy.end(), 0.0);
            return;
        }
        std::vector<double> albedo = s.albedo;  // a local copy: never written back (hbv_physical_snow.h:332)
        double surface_heat = s.surface_heat;   // likewise (:333)
        const double min_albedo = p.min_albedo, max_albedo = p.max_albedo;
        const double albedo_range = max_albedo - min_albedo;
        const double dt_in_days = dts / 86400.0;
        const double slow_albedo_decay_rate = (0.5 * albedo_range * dt_in_days / p.slow_albedo_decay_rate);
        const double fast_albedo_decay_rate = OPOW(2.0, -dt_in_days / p.fast_albedo_decay_rate);
        const double T_k = T + 273.15;
        const double turb = p.wind_scale * wind_speed + p.wind_const;
        double vapour_pressure = (33.864 * (OPOW8(7.38e-3 * T + 0.8072) - 1.9e-5 * std::fabs(1.8 * T + 48.0) + 1.316e-3) *
                                  rel_hum);
        if (T < 0.0) vapour_pressure *= 1.0 + 9.72e-3 * T + 4.2e-5 * T * T;
        if (snow > tol) {
            auto idx = sca_index(s.sca);
            if (s.sca > 1.0e-5 && s.sca < 1.0 - 1.0e-5) {
                if (idx == 0) {
                    s.sp[0] *= s.sca / (I[1] - I[0]);
                    s.sw[0] *= s.sca / (I[1] - I[0]);
                } else {
                    s.sp[idx] *= (1.0 + (s.sca - I[idx]) / (I[idx] - I[idx - 1])) / (1.0 + (I[idx + 1] - I[idx]) / (I[idx] - I[idx - 1]));
                    s.sw[idx] *= (1.0 + (s.sca - I[idx]) / (I[idx] - I[idx - 1])) / (1.0 + (I[idx + 1] - I[idx]) / (I[idx] - I[idx - 1]));
                }
            }
            for (size_t i = 0; i < n; ++i) {
                double currsnow = snow * p.s[i];
                s.sp[i] += currsnow;
                albedo[i] += (currsnow * albedo_range / p.snowfall_reset_depth);
            }
            for (size_t i = n - 2; i > 0; --i)
                if (p.s[i] > 0.0) {
                    s.sca = p.s[i + 1];
                    break;
                } else
                    s.sca = p.s[1];
        } else {
            if (T < 0.0) {
                for (auto& alb : albedo) alb -= slow_albedo_decay_rate;
            } else {
                for (auto& alb : albedo) alb = (min_albedo + fast_albedo_decay_rate * (alb - min_albedo));
            }
        }
        for (auto& alb : albedo) alb = std::max(std::min(alb, max_albedo), min_albedo);
        std::vector<double> effect;
        for (auto alb : albedo) effect.push_back(rad * (1.0 - alb));
        for (auto& eff : effect) eff += (0.98 * sigma * OPOWR(vapour_pressure / T_k, 6.87e-2) * OPOW4(T_k));
        if (T > 0.0 && snow < tol)
            for (auto& eff : effect) eff += rain * T * water_heat / dts;
        if (T <= 0.0 && rain < tol)
            for (size_t i = 0; i < n; ++i) effect[i] += snow * p.s[i] * T * ice_heat / dts;
        if (p.calculate_iso_pot_energy) {
            for (size_t i = 0; i < n; ++i) {
                double iso_effect = (effect[i] - BB0 + turb * (T + 1.7 * (vapour_pressure - 6.12)));
                s.iso_pot_energy[i] += (iso_effect * dts / melt_heat);
            }
        }
        double sst = std::min(0.0, 1.16 * T - 2.09);
        if (sst > -tol) {
            for (auto& eff : effect) eff += turb * (T + 1.7 * (vapour_pressure - 6.12)) - BB0;
        } else {
            for (auto& eff : effect)
                eff += (turb * (T - sst + 1.7 * (vapour_pressure - 6.132 * OEXP(0.103 * T - 0.186))) -
                        0.98 * sigma * OPOW4(sst + 273.15));
        }
        double delta_sh = -surface_heat;
        surface_heat = p.surface_magnitude * ice_heat * sst * 0.5;
        delta_sh += surface_heat;
        std::vector<double> energy;
        for (auto eff : effect) energy.push_back(eff * dts);
        if (delta_sh > 0.0)
            for (auto& en : energy) en -= delta_sh;
        std::vector<double> potential_melt;
        for (auto en : energy) potential_melt.push_back(en / melt_heat);
        const double lw = p.lw;
        size_t idx = n;
        bool any_melt = false;
        for (size_t i = 0; i < n; ++i) {
            if (potential_melt[i] >= tol) {
                any_melt = true;
                if (s.sp[i] < potential_melt[i]) {
                    idx = i;
                    break;
                }
            }
        }
        if (any_melt) {
            if (idx == 0) s.sca = 0.0;
            else if (idx == n) s.sca = 1.0;
            else {
                if (s.sp[idx] > 0.0) {
                    s.sca = (I[idx] - (I[idx] - I[idx - 1]) * (potential_melt[idx] - s.sp[idx]) / (s.sp[idx - 1] = s.sp[idx]));
                } else {
                    s.sca = (1.0 - potential_melt[idx] / s.sp[idx - 1]) * (s.sca - I[idx - 1]) + I[idx - 1];
                }
            }
        }
        for (size_t i = 0; i < n; ++i) {
            if (potential_melt[i] < tol) refreeze(s.sp[i], s.sw[i], rain, p.cfr * potential_melt[i], lw);
            else update_state(s.sp[i], s.sw[i], rain, potential_melt[i], lw);
        }
        if (s.sca < tol) s.swe = 0.0;
        else {
            bool f_is_zero = s.sca >= 1.0 ? false : true;
            s.swe = hbv_snow::integrate(s.sp, I, n, 0, s.sca, f_is_zero);
            s.swe += hbv_snow::integrate(s.sw, I, n, 0, s.sca, f_is_zero);
        }
        if (total_water < s.swe) {
            if (total_water - s.swe < -tol) {
                std::ostringstream buff;
                buff << "Negative outflow: total_water (" << total_water << ") - s.swe (" << s.swe << ") = " << total_water - s.swe;
                throw std::runtime_error(buff.str());
            } else
                s.swe = total_water;
        }
        r.outflow = total_water - s.swe;
        r.sca = s.sca;
        r.storage = s.swe;
    }
};

}  // namespace hbv_physical_snow

namespace pt_hps_k {

// core/pt_hps_k.h:25-159 (24 calibration values); gm.direct_response is not one of them (default 0)
struct parameter {
    priestley_taylor::parameter pt;
    hbv_physical_snow::parameter hps;
    actual_evapotranspiration::parameter ae;
    kirchner::parameter kirchner;
    precipitation_correction::parameter p_corr;
    glacier_melt::parameter gm;
    pt_gs_k::uhg_parameter routing;
    pt_gs_k::mstack_parameter msp;
    static constexpr size_t size() { return 24; }
    void set(const double* p) {  // pt_hps_k.h:64-90
        int i = 0;
        kirchner.c1 = p[i++]; kirchner.c2 = p[i++]; kirchner.c3 = p[i++];
        ae.ae_scale_factor = p[i++];
        hps.lw = p[i++]; hps.tx = p[i++]; hps.cfr = p[i++]; hps.wind_scale = p[i++]; hps.wind_const = p[i++];
        hps.surface_magnitude = p[i++]; hps.max_albedo = p[i++]; hps.min_albedo = p[i++];
        hps.fast_albedo_decay_rate = p[i++]; hps.slow_albedo_decay_rate = p[i++]; hps.snowfall_reset_depth = p[i++];
        hps.calculate_iso_pot_energy = std::fabs(p[i++]) < 0.0001 ? false : true;
        gm.dtf = p[i++];
        p_corr.scale_factor = p[i++];
        pt.albedo = p[i++]; pt.alpha = p[i++];
        routing.velocity = p[i++]; routing.alpha = p[i++]; routing.beta = p[i++];
        msp.reservoir_direct_response_fraction = p[i++];
    }
};

// flat state: swe sca surface_heat n_bins sp[8] sw[8] albedo[8] iso_pot_energy[8] kirchner.q
constexpr size_t MB = hbv_stack::MAX_BINS;
constexpr size_t FLAT = 4 + 4 * MB + 1;
struct state {
    hbv_physical_snow::state hps;
    kirchner::state kirchner;
    void set(const double* v) {
        hps.swe = v[0]; hps.sca = v[1]; hps.surface_heat = v[2];
        const size_t nb = size_t(v[3]);
        hps.sp.assign(v + 4, v + 4 + nb);
        hps.sw.assign(v + 4 + MB, v + 4 + MB + nb);
        hps.albedo.assign(v + 4 + 2 * MB, v + 4 + 2 * MB + nb);
        hps.iso_pot_energy.assign(v + 4 + 3 * MB, v + 4 + 3 * MB + nb);
        kirchner.q = v[4 + 4 * MB];
    }
    void get(double* v) const {
        v[0] = hps.swe; v[1] = hps.sca; v[2] = hps.surface_heat; v[3] = double(hps.sp.size());
        for (size_t i = 0; i < MB; ++i) {
            v[4 + i] = i < hps.sp.size() ? hps.sp[i] : 0.0;
            v[4 + MB + i] = i < hps.sw.size() ? hps.sw[i] : 0.0;
            v[4 + 2 * MB + i] = i < hps.albedo.size() ? hps.albedo[i] : 0.0;
            v[4 + 3 * MB + i] = i < hps.iso_pot_energy.size() ? hps.iso_pot_energy[i] : 0.0;
        }
        v[4 + 4 * MB] = kirchner.q;
    }
    state scale_snow(double f) const {  // pt_hps_k.h:178-182
        state c{*this};
        c.hps.swe *= f;
        return c;
    }
};

struct response {
    double pot_evapotranspiration = 0;
    hbv_physical_snow::response hps;
    double ae = 0, q_avg = 0, gm_melt_m3s = 0, total_discharge = 0, charge_m3s = 0;
    response scale_snow(double f) const {  // pt_hps_k.h:196-202
        response c{*this};
        c.hps.storage *= f;
        c.hps.outflow *= f;
        return c;
    }
};

// all_response_collector (pt_hps_k_cell_model.h:41-93) in this repo's series-id order: avg_discharge, charge_m3s,
// hps_sca, hps_swe, hps_outflow (mm/h, as the reference collects it), glacier_melt, ae_output, pe_output
enum all_series { AVG_DISCHARGE = 0, CHARGE_M3S, SNOW_SCA, SNOW_SWE, SNOW_OUTFLOW, GLACIER_MELT, AE_OUTPUT, PE_OUTPUT, N_ALL };
// state collector (pt_hps_k_cell_model.h:160-232): kirchner_discharge, hps_sca, hps_swe, hps_surface_heat,
// sp[8], sw[8], albedo[8], iso_pot_energy[8]
constexpr size_t N_SC = 4 + 4 * MB;

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
            rc[SNOW_SCA][i] = r.hps.sca;
            rc[SNOW_SWE][i] = r.hps.storage;
        }
        if (full) {
            rc[SNOW_OUTFLOW][i] = r.hps.outflow;
            rc[GLACIER_MELT][i] = r.gm_melt_m3s;
            rc[AE_OUTPUT][i] = r.ae;
            rc[PE_OUTPUT][i] = r.pot_evapotranspiration;
        }
    }
    void collect_state_(size_t i, const state& s) {
        if (!collect_state) return;
        sc[0][i] = mmh_to_m3s(s.kirchner.q, area);
        sc[1][i] = s.hps.sca;
        sc[2][i] = s.hps.swe;
        sc[3][i] = s.hps.surface_heat;
        for (size_t k = 0; k < MB; ++k) {  // bins beyond n_bins are collected as 0 here
            sc[4 + k][i] = k < s.hps.sp.size() ? s.hps.sp[k] : 0.0;
            sc[4 + MB + k][i] = k < s.hps.sw.size() ? s.hps.sw[k] : 0.0;
            sc[4 + 2 * MB + k][i] = k < s.hps.albedo.size() ? s.hps.albedo[k] : 0.0;
            sc[4 + 3 * MB + k][i] = k < s.hps.iso_pot_energy.size() ? s.hps.iso_pot_energy[k] : 0.0;
        }
    }
};

// core/pt_hps_k.h:203-300
inline void run_pt_hps_k(const geo_cell_data& geo, const parameter& parameter, const fixed_dt& time_axis, int start_step,
                         int n_steps, const pt_gs_k::forcing_view& fv, state& state, collectors& col) {
    priestley_taylor::calculator pt(parameter.pt.albedo, parameter.pt.alpha);
    const hbv_physical_snow::calculator hps(parameter.hps);
    kirchner::calculator kirchner(parameter.kirchner);
    state.hps.distribute(parameter.hps, false);
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
        double wind_speed = fv.ws[i * fv.stride];
        col.collect_state_(i, state.scale_snow(snow_storage_fraction));
        hps.step(state.hps, response.hps, t1 - t0, temp, rad, prec, wind_speed, rel_hum);
        response.gm_melt_m3s = glacier_melt::step(parameter.gm.dtf, temp, geo.area * state.hps.sca, glacier_area_m2);
        response.pot_evapotranspiration = pt.potential_evapotranspiration(temp, rad, rel_hum) * to_seconds(HOUR_US);
        response.ae = actual_evapotranspiration::calculate_step(state.kirchner.q, response.pot_evapotranspiration,
                                                                parameter.ae.ae_scale_factor,
                                                                std::max(state.hps.sca, glacier_fraction));
        double gm_mmh = m3s_to_mmh(response.gm_melt_m3s, cell_area_m2);
        kirchner.step(t0, t1, state.kirchner.q, response.q_avg,
                      response.hps.outflow * snow_storage_fraction + prec * kirchner_routed_prec + gm_routed * gm_mmh,
                      response.ae);
        response.total_discharge = std::max(0.0, prec - response.ae) * direct_response_fraction + gm_direct * gm_mmh +
                                   response.q_avg * kirchner_fraction;
        response.charge_m3s = +mmh_to_m3s(prec, cell_area_m2) - mmh_to_m3s(response.ae, cell_area_m2) + response.gm_melt_m3s -
                              mmh_to_m3s(response.total_discharge, cell_area_m2);
        col.collect_response(i, response.scale_snow(snow_storage_fraction));
        if (i + 1 == i_end) col.collect_state_(i + 1, state.scale_snow(snow_storage_fraction));
    }
}

}  // namespace pt_hps_k
}  // namespace oracle
