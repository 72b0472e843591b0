// ORACLE — test infrastructure only (see common.hpp header).
//
// hbv.hpp: the hbv_stack method stack (core/hbv_stack.h:278-361) with its
// methods hbv_snow (core/hbv_snow.h, core/hbv_snow_common.h), hbv_soil
// (core/hbv_soil.h), hbv_tank (core/hbv_tank.h), hbv_actual_evapotranspiration
// (core/hbv_actual_evapotranspiration.h) and the collectors of
// core/hbv_stack_cell_model.h. Restated in plain C++; every arithmetic
// expression keeps the reference's operand order.
#pragma once
#include <algorithm>
#include <cmath>
#include <sstream>
#include <stdexcept>
#include <vector>

#include "common.hpp"
#include "methods.hpp"
#include "ptgsk.hpp"  // uhg_parameter, mstack_parameter

namespace oracle {

namespace hbv_snow {

// hbv_snow_common::integrate (hbv_snow_common.h:14-44): integral of the
// piecewise-linear f(x) from a to b; f(b) = 0 when f_b_is_zero (unless b hits a knot).
inline double integrate(const double* f, const double* x, size_t n, double a, double b, bool f_b_is_zero = false) {
    size_t left = 0;
    double area = 0.0;
    double f_l = 0.0;
    double x_l = a;
    while (a > x[left]) ++left;
    if (std::fabs(a - x[left]) > 1.0e-8 && left > 0) {
        --left;
        f_l = (f[left + 1] - f[left]) / (x[left + 1] - x[left]) * (a - x[left]) + f[left];
    } else {
        f_l = f[left];
    }
    while (left < n - 1) {
        if (b >= x[left + 1]) {
            area += 0.5 * (f_l + f[left + 1]) * (x[left + 1] - x_l);
            x_l = x[left + 1];
            f_l = f[left + 1];
            ++left;
        } else {
            if (!f_b_is_zero)
                area += (f_l + 0.5 * (f[left + 1] - f_l) / (x[left + 1] - x_l) * (b - x_l)) * (b - x_l);
            else
                area += 0.5 * f_l * (b - x_l);
            break;
        }
    }
    return area;
}
inline double integrate(const std::vector<double>& f, const std::vector<double>& x, size_t n, double a, double b,
                        bool f_b_is_zero = false) {
    return integrate(f.data(), x.data(), n, a, b, f_b_is_zero);
}

// hbv_snow.h:21-72
struct parameter {
    std::vector<double> s;          // snow redistribution factors
    std::vector<double> intervals;  // snow quantiles, 0 .. 1
    double tx = 0.0, cx = 1.0, ts = 0.0, lw = 0.1, cfr = 0.5;
    parameter() { set_std_distribution_and_quantiles(); }
    parameter(const std::vector<double>& s_, const std::vector<double>& i_) : s(s_), intervals(i_) {}  // no normalisation (:49-51)
    void set_std_distribution_and_quantiles() {
        s = {1.0, 1.0, 1.0, 1.0, 1.0};
        intervals = {0, 0.25, 0.5, 0.75, 1.0};
        normalize_snow_distribution();
    }
    void normalize_snow_distribution() {
        const double mean = integrate(s, intervals, intervals.size(), intervals[0], intervals.back());
        for (auto& v : s) v /= mean;
    }
};

// hbv_snow.h:74-112 (+ distribute_snow, hbv_snow_common.h:47-66)
struct state {
    std::vector<double> sp, sw;
    double swe = 0.0, sca = 0.0;
    void distribute(const parameter& p, bool force = true) {
        if (force || sp.size() != p.s.size() || sw.size() != p.s.size()) {
            const size_t n = p.intervals.size();
            sp.assign(n, 0.0);
            sw.assign(n, 0.0);
            if (swe <= 1.0e-3 || sca <= 1.0e-3) {
                swe = sca = 0.0;
            } else {
                for (size_t i = 0; i < n; ++i) sp[i] = sca < p.intervals[i] ? 0.0 : p.s[i] * swe;
                auto temp_swe = integrate(sp, p.intervals, n, 0.0, sca, true);
                if (temp_swe < swe) {
                    const double corr1 = swe / temp_swe * p.lw;
                    const double corr2 = swe / temp_swe * (1.0 - p.lw);
                    for (size_t i = 0; i < n; ++i) {
                        sw[i] = corr1 * sp[i];
                        sp[i] *= corr2;
                    }
                } else {
                    sw.assign(n, 0.0);
                }
            }
        }
    }
};

struct response {
    double outflow = 0.0;
    state snow_state;  // never written by step (hbv_snow.h:121-124, 195-272): collected as 0
};

// hbv_snow.h:139-272
struct calculator {
    const parameter& p;
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
    size_t melt_index(double potmelt, const state& s) const {
        for (size_t i = 0; i < p.intervals.size(); ++i)
            if (s.sp[i] < potmelt) return i;
        return p.intervals.size();
    }
    void step(state& s, response& r, utctime t0, utctime t1, double prec_mm_h, double temp) const {
        double swe = s.swe;
        double sca = s.sca;
        const auto& I = p.intervals;
        double step_in_days = to_seconds(t1 - t0) / 86400.0;
        const double dt_hours = to_seconds(t1 - t0) / 3600.0;
        const double prec = prec_mm_h * dt_hours;
        const double total_water = prec + swe;
        double snow, rain;
        if (temp < p.tx) { snow = prec; rain = 0.0; }
        else             { snow = 0.0; rain = prec; }
        swe += snow + sca * rain;
        if (swe < 0.1) {
            r.outflow = total_water / dt_hours;
            std::fill(s.sp.begin(), s.sp.end(), 0.0);
            std::fill(s.sw.begin(), s.sw.end(), 0.0);
            s.swe = 0.0;
            s.sca = 0.0;
            return;
        }
        if (snow > 0.0) {
            auto idx = sca_index(sca);
            if (sca > 1.0e-5 && sca < 1.0 - 1.0e-5) {
                if (idx == 0) {
                    s.sp[0] *= sca / (I[1] - I[0]);
                    s.sw[0] *= sca / (I[1] - I[0]);
                } else {
                    s.sp[idx] *= (1.0 + (sca - I[idx]) / (I[idx] - I[idx - 1])) / (1.0 + (I[idx + 1] - I[idx]) / (I[idx] - I[idx - 1]));
                    s.sw[idx] *= (1.0 + (sca - I[idx]) / (I[idx] - I[idx - 1])) / (1.0 + (I[idx + 1] - I[idx]) / (I[idx] - I[idx - 1]));
                }
            }
            for (size_t i = 0; i < p.s.size(); ++i) s.sp[i] += snow * p.s[i];
            sca = I[1];
            for (size_t i = I.size() - 2; i > 0; --i)
                if (p.s[i] > 0.0) {
                    sca = I[i + 1];
                    break;
                }
        }
        double potmelt = p.cx * step_in_days * (temp - p.ts);
        const double lw = p.lw;
        if (potmelt < 0.0) {
            potmelt *= p.cfr;
            for (size_t i = 0; i < I.size(); ++i) refreeze(s.sp[i], s.sw[i], rain, potmelt, lw);
        } else {
            size_t idx = melt_index(potmelt, s);
            if (idx == 0) sca = 0.0;
            else if (idx == I.size()) sca = 1.0;
            else {
                if (s.sp[idx] > 0.0) sca = I[idx] - (I[idx] - I[idx - 1]) * (potmelt - s.sp[idx]) / (s.sp[idx - 1] - s.sp[idx]);
                else sca = (1.0 - potmelt / s.sp[idx - 1]) * (sca - I[idx - 1]) + I[idx - 1];
            }
            for (size_t i = 0; i < I.size(); ++i) update_state(s.sp[i], s.sw[i], rain, potmelt, lw);
        }
        if (sca < 1.0e-6) swe = 0.0;
        else {
            bool f_is_zero = sca >= 1.0 ? false : true;
            swe = integrate(s.sp, I, I.size(), 0, sca, f_is_zero);
            swe += integrate(s.sw, I, I.size(), 0, sca, f_is_zero);
        }
        if (total_water < swe) {
            if (total_water - swe < -1.0e-6) {
                std::ostringstream buff;
                buff << "Negative outflow: total_water (" << total_water << ") - swe (" << swe << ") = " << total_water - swe;
                throw std::runtime_error(buff.str());
            } else {
                swe = total_water;
            }
        }
        r.outflow = (total_water - swe) / dt_hours;
        s.swe = swe;
        s.sca = sca;
    }
};

}  // namespace hbv_snow

// hbv_soil.h:17-64
namespace hbv_soil {
struct parameter { double fc = 300.0, beta = 2.0; };
struct state { double sm = 0.0; };  // explicit state(double sm = 0.0) (:33)
struct response { double outflow = 0.0; };
inline void step(const parameter& param, state& s, response& r, double insoil, double act_evap) {
    double temp = s.sm + insoil;
    double outflow = insoil * OPOW(temp / param.fc, param.beta);
    r.outflow = outflow > temp ? temp : outflow;
    s.sm = std::max(0.0, s.sm + insoil - r.outflow - act_evap);
}
}  // namespace hbv_soil

// hbv_tank.h:17-80
namespace hbv_tank {
struct parameter { double uz1 = 25.0, kuz2 = 0.5, kuz1 = 0.3, perc = 0.8, klz = 0.02; };
struct state { double uz = 20.0, lz = 10.0; };
struct response { double outflow = 0.0; };
inline void step(const parameter& param, state& s, response& r, double soil_outflow) {
    double temp = s.uz + soil_outflow;
    double q12 = std::max(0.0, (temp - param.uz1) * param.kuz2);
    double q11 = std::min(temp, param.uz1) * param.kuz1;
    s.uz = s.uz + soil_outflow - param.perc - (q12 + q11);
    double q2 = (s.lz + param.perc) * param.klz;
    s.lz = s.lz + param.perc - q2;
    r.outflow = q12 + q11 + q2;
}
}  // namespace hbv_tank

// hbv_actual_evapotranspiration.h:12-38
namespace hbv_actual_evapotranspiration {
struct parameter { double lp = 150.0; };
inline double calculate_step(double soil_moisture, double pot_evapo, double lp, double snow_fraction) {
    return (1.0 - snow_fraction) * (soil_moisture < lp ? pot_evapo * (soil_moisture / lp) : pot_evapo);
}
}  // namespace hbv_actual_evapotranspiration

namespace hbv_stack {

// hbv_stack.h:32-176
struct parameter {
    priestley_taylor::parameter pt;
    hbv_snow::parameter snow;
    hbv_actual_evapotranspiration::parameter ae;
    hbv_soil::parameter soil;
    hbv_tank::parameter tank;
    precipitation_correction::parameter p_corr;
    glacier_melt::parameter gm;
    pt_gs_k::uhg_parameter routing;
    pt_gs_k::mstack_parameter msp;
    static constexpr size_t size() { return 22; }
    // get/set order: hbv_stack.h:82-109
    void set(const double* p) {
        int i = 0;
        soil.fc = p[i++]; soil.beta = p[i++];
        ae.lp = p[i++];
        tank.uz1 = p[i++]; tank.kuz2 = p[i++]; tank.kuz1 = p[i++]; tank.perc = p[i++]; tank.klz = p[i++];
        snow.lw = p[i++]; snow.tx = p[i++]; snow.cx = p[i++]; snow.ts = p[i++]; snow.cfr = p[i++];
        p_corr.scale_factor = p[i++];
        pt.albedo = p[i++]; pt.alpha = p[i++];
        gm.dtf = p[i++];
        routing.velocity = p[i++]; routing.alpha = p[i++]; routing.beta = p[i++];
        gm.direct_response = p[i++];
        msp.reservoir_direct_response_fraction = p[i++];
    }
};

// hbv_stack.h:181-201; flat order used by the C-ABIs: swe sca sm uz lz n_bins sp[8] sw[8]
constexpr size_t MAX_BINS = 8;
constexpr size_t FLAT = 6 + 2 * MAX_BINS;
struct state {
    hbv_snow::state snow;
    hbv_soil::state soil;
    hbv_tank::state tank;
    void set(const double* v) {
        snow.swe = v[0]; snow.sca = v[1]; soil.sm = v[2]; tank.uz = v[3]; tank.lz = v[4];
        const size_t nb = size_t(v[5]);
        snow.sp.assign(v + 6, v + 6 + nb);
        snow.sw.assign(v + 6 + MAX_BINS, v + 6 + MAX_BINS + nb);
    }
    void get(double* v) const {
        v[0] = snow.swe; v[1] = snow.sca; v[2] = soil.sm; v[3] = tank.uz; v[4] = tank.lz;
        v[5] = double(snow.sp.size());
        for (size_t i = 0; i < MAX_BINS; ++i) {
            v[6 + i] = i < snow.sp.size() ? snow.sp[i] : 0.0;
            v[6 + MAX_BINS + i] = i < snow.sw.size() ? snow.sw[i] : 0.0;
        }
    }
};

// hbv_stack.h:203-220
struct response {
    double pot_evapotranspiration = 0;
    hbv_snow::response snow;
    double ae = 0;
    hbv_soil::response soil;
    hbv_tank::response tank;
    double gm_melt_m3s = 0;
    double total_discharge = 0;
    double charge_m3s = 0;
};

// Collector series (hbv_stack_cell_model.h:40-136), in this repo's series-id order:
// avg_discharge, charge_m3s, snow_sca, snow_swe, snow_outflow, glacier_melt, ae_output, pe_output, soil_outflow
enum all_series { AVG_DISCHARGE = 0, CHARGE_M3S, SNOW_SCA, SNOW_SWE, SNOW_OUTFLOW, GLACIER_MELT, AE_OUTPUT, PE_OUTPUT,
                  SOIL_OUTFLOW, N_ALL };

struct collectors {
    bool full = true, collect_snow = false, collect_state = false;
    double area = 0;
    std::vector<double> rc[N_ALL];
    std::vector<double> sc[FLAT];  // state collector (T+1), flat state order (n_bins row unused)
    response end_response;
    void initialize(size_t T, int start, int n, double a) {
        area = a;
        for (int k = 0; k < N_ALL; ++k) {
            bool on = full || k == AVG_DISCHARGE || k == CHARGE_M3S || (collect_snow && (k == SNOW_SCA || k == SNOW_SWE));
            pt_gs_k::collectors::ts_init(rc[k], on ? T : 0, start, n);
        }
        for (size_t k = 0; k < FLAT; ++k) pt_gs_k::collectors::ts_init(sc[k], collect_state ? T + 1 : 0, start, n > 0 ? n + 1 : 0);
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
            rc[SOIL_OUTFLOW][i] = r.soil.outflow;
        }
    }
    void collect_state_(size_t i, const state& s) {
        if (!collect_state) return;
        double v[FLAT];
        s.get(v);
        for (size_t k = 0; k < FLAT; ++k) sc[k][i] = v[k];
    }
};

// core/hbv_stack.h:278-361 (wind speed is not read, :295-301)
inline void run_hbv_stack(const geo_cell_data& geo, const parameter& parameter, const fixed_dt& time_axis, int start_step,
                          int n_steps, const pt_gs_k::forcing_view& fv, state& state, collectors& col) {
    priestley_taylor::calculator pt(parameter.pt.albedo, parameter.pt.alpha);
    hbv_snow::calculator snow(parameter.snow);
    response response;
    state.snow.distribute(parameter.snow, false);
    const double glacier_fraction = geo.fractions.glacier();
    const double gm_direct = parameter.gm.direct_response;
    const double gm_routed = 1 - gm_direct;
    const double direct_response_fraction =
        glacier_fraction * gm_direct + geo.fractions.reservoir() * parameter.msp.reservoir_direct_response_fraction;
    const double land_fraction = 1 - direct_response_fraction;
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
        col.collect_state_(i, state);
        snow.step(state.snow, response.snow, t0, t1, prec, temp);
        response.gm_melt_m3s = glacier_melt::step(parameter.gm.dtf, temp, geo.area * state.snow.sca, glacier_area_m2);
        response.pot_evapotranspiration = pt.potential_evapotranspiration(temp, rad, rel_hum) * to_seconds(HOUR_US);
        response.ae = hbv_actual_evapotranspiration::calculate_step(state.soil.sm, response.pot_evapotranspiration,
                                                                    parameter.ae.lp, std::max(state.snow.sca, glacier_fraction));
        double gm_mmh = m3s_to_mmh(response.gm_melt_m3s, cell_area_m2);
        hbv_soil::step(parameter.soil, state.soil, response.soil, response.snow.outflow, response.ae);
        hbv_tank::step(parameter.tank, state.tank, response.tank, response.soil.outflow + gm_routed * gm_mmh);
        response.total_discharge = std::max(0.0, prec - response.ae) * direct_response_fraction + gm_direct * gm_mmh +
                                   response.tank.outflow * land_fraction;
        response.charge_m3s = +mmh_to_m3s(prec, cell_area_m2) - mmh_to_m3s(response.ae, cell_area_m2) + response.gm_melt_m3s -
                              mmh_to_m3s(response.total_discharge, cell_area_m2);
        col.collect_response(i, response);
        if (i + 1 == i_end) col.collect_state_(i + 1, state);
    }
    col.end_response = response;
}

}  // namespace hbv_stack
}  // namespace oracle
