// ORACLE — test infrastructure only (see common.hpp header).
//
// ptssk.hpp: Skaugen's snow routine (core/skaugen.h) and the pt_ss_k method
// stack (core/pt_ss_k.h) with its collectors (core/pt_ss_k_cell_model.h).
//
// Third-party arithmetic restated (boost 1.68, not under /root/reference):
//  - gamma_distribution<double, digits10<16>> pdf / cdf / mean
//    (boost/math/distributions/gamma.hpp): pdf = gamma_p_derivative(k, x/theta)/theta
//    with gamma_p_derivative(a, z) = regularised_gamma_prefix(a, z)/z, cdf = gamma_p(k, x/theta),
//    mean = k*theta. The prefix z^a e^-z / Gamma(a) is evaluated as exp(a log z - z - lgamma a)
//    with this build's elementary functions (detmath, or libm with -DORACLE_LIBM);
//  - brent_find_minima (tools/minima.hpp), shared with gamma_snow (methods.hpp);
//  - bisect with eps_tolerance<double>(10) (tools/roots.hpp): eps = max(2^-9, 4*DBL_EPSILON),
//    converged when |a-b| <= eps*min(|a|,|b|); 100 evaluations; "no change of sign" raises
//    boost's evaluation_error (here std::runtime_error).
// Integer semantics follow the reference: unit counts are unsigned long (uint64 wrap-around
// included) and lrint rounds half to even.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <vector>

#include "common.hpp"
#include "methods.hpp"
#include "ptgsk.hpp"

namespace oracle {
namespace skaugen {

using ulong = unsigned long;  // the reference's unit-count type (LP64: 64 bit)

// gamma_distribution(shape k, scale theta) with boost's full-precision policy
struct gamma_dist {
    double k, theta;
    double mean() const { return k * theta; }
    double pdf(double x) const {
        if (x == 0) {
            if (k == 1) return 1 / theta;
            if (k < 1) throw std::overflow_error("boost::math::pdf(gamma_distribution): overflow at x = 0");
            return 0.0;
        }
        const double z = x / theta;
        const double prefix = OEXP(k * OLOG(z) - z - OLGAMMA(k));
        return prefix / z / theta;
    }
    double cdf(double x) const { return special::gamma_pq(k, x / theta).p; }
};

// boost::math::tools::bisect with eps_tolerance(bits) (tools/roots.hpp)
template <class F>
std::pair<double, double> bisect(F f, double min, double max, int bits, uintmax_t& max_iter) {
    double fmin = f(min);
    double fmax = f(max);
    if (fmin == 0) { max_iter = 2; return {min, min}; }
    if (fmax == 0) { max_iter = 2; return {max, max}; }
    if (min >= max) throw std::runtime_error("Arguments in wrong order in boost::math::tools::bisect");
    if (fmin * fmax >= 0)
        throw std::runtime_error("No change of sign in boost::math::tools::bisect, either there is no root to find, "
                                 "or there are multiple roots in the interval");
    const double eps = std::max(std::ldexp(1.0, 1 - bits), 4 * DBL_EPSILON);
    auto tol = [eps](double a, double b) { return std::fabs(a - b) <= eps * std::min(std::fabs(a), std::fabs(b)); };
    auto sign = [](double z) { return z > 0 ? 1 : (z < 0 ? -1 : 0); };
    uintmax_t count = max_iter;
    if (count < 3) count = 0; else count -= 3;
    while (count && !tol(min, max)) {
        const double mid = (min + max) / 2;
        const double fmid = f(mid);
        if ((mid == max) || (mid == min)) break;
        if (fmid == 0) { min = max = mid; break; }
        else if (sign(fmid) * sign(fmin) < 0) { max = mid; fmax = fmid; }
        else { min = mid; fmin = fmid; }
        --count;
    }
    max_iter -= count;
    return {min, max};
}

// core/skaugen.h:43-87
struct statistics {
    const double alpha_0, d_range, unit_size;
    statistics(double a0, double dr, double us) : alpha_0(a0), d_range(dr), unit_size(us) {}
    static double c(ulong n, double d_range) { return OEXP(-(double)n / d_range); }
    double c(ulong n) const { return c(n, d_range); }

    static double sca_rel_red(ulong u, ulong n, double /*unit_size*/, double nu_a, double alpha) {
        const double nu_m = ((double)u / n) * nu_a;
        const gamma_dist g_m{nu_m, 1.0 / alpha};
        const gamma_dist g_a{nu_a, 1.0 / alpha};
        const double g_a_mean = g_a.mean();
        auto zero_func = [&](const double& x) { return g_m.pdf(x) - g_a.pdf(x); };
        double lower = g_m.mean();
        uintmax_t brent_iter = std::numeric_limits<uintmax_t>::max();
        double upper = special::brent_find_minima(zero_func, 0.0, g_a_mean, 2, brent_iter).first;
        while (g_m.pdf(lower) < g_a.pdf(lower)) lower *= 0.9;
        uintmax_t max_iter = 100;
        auto res = bisect(zero_func, lower, upper, 10, max_iter);
        const double x = (res.first + res.second) * 0.5;
        const double m = g_m.cdf(x);
        const double a = g_a.cdf(x);
        return a + 1.0 - m;
    }
    double sca_rel_red(ulong u, ulong n, double nu_a, double alpha) const {
        return sca_rel_red(u, n, unit_size, nu_a, alpha);
    }
};

// core/skaugen.h:89-112
struct parameter {
    double alpha_0 = 40.77, d_range = 113.0, unit_size = 0.1, max_water_fraction = 0.1;
    double tx = 0.16, cx = 2.5, ts = 0.14, cfr = 0.01;
};

// core/skaugen.h:115-139
struct state {
    double nu = 4.077, alpha = 40.77, sca = 0.0, swe = 0.0, free_water = 0.0, residual = 0.0;
    size_t num_units = 0;
    double swe_for_cell_area() const { return (free_water + swe) * sca; }
    double free_water_for_cell_area() const { return free_water * sca; }
};

struct response {
    double outflow = 0.0, sca = 0.0, swe = 0.0;
};

inline long lrint_(double x) { return std::lrint(x); }

// compute_shape_vars (core/skaugen.h:338-380)
inline void compute_shape_vars(const statistics& stat, ulong nnn, ulong n, ulong u, double sca, double rel_red_sca,
                               double& alpha, double& nu) {
    const double alpha_0 = stat.alpha_0;
    const double nu_0 = stat.alpha_0 * stat.unit_size;
    const double dyn_var = nu / (alpha * alpha);
    const double init_var = nu_0 / (alpha_0 * alpha_0);
    double tot_var = 0.0;
    double tot_mean = 0.0;
    if (n > 0) {
        if (nnn == 0) {
            tot_var = n * init_var * (1 + (n - 1) * stat.c(n));
            tot_mean = n * nu_0 / alpha_0;
        } else {
            const double old_var_cov = (nnn + n) * init_var * (1 + ((nnn + n) - 1) * stat.c(nnn + n));
            const double new_var_cov = n * init_var * (1 + (n - 1) * stat.c(n));
            tot_var = old_var_cov * sca * sca + new_var_cov * (1.0 - sca) * (1.0 - sca);
            tot_mean = (sca * (nnn + n) + (1.0 - sca) * n) * stat.unit_size;
        }
    }
    if (u > 0) {
        const double factor = (dyn_var / (nnn * init_var) + 1.0 + (nnn - 1) * stat.c(nnn)) / (2 * nnn);
        const double non_cond_mean = (nnn - u) * stat.unit_size;
        tot_mean = non_cond_mean / (1.0 - rel_red_sca);
        const ulong cond_u = (ulong)lrint_((1.0 - rel_red_sca) * nnn - (nnn - u));
        const double auto_var = cond_u > 0 ? init_var * cond_u * (1.0 + (cond_u - 1.0) * stat.c(cond_u)) : 0.0;
        const double cross_var = cond_u > 0 ? init_var * cond_u * 2.0 * factor * cond_u : 0.0;
        tot_var = dyn_var + auto_var - cross_var;
    }
    if (std::fabs(tot_mean) < 1.0e-7) {
        nu = nu_0;
        alpha = alpha_0;
        return;
    }
    nu = tot_mean * tot_mean / tot_var;
    alpha = nu / (stat.unit_size * lrint_(tot_mean / stat.unit_size));
}

// calculator::step (core/skaugen.h:151-336)
inline void step(int64_t dt_us, const parameter& p, const double T, const double prec_mm_h, state& s, response& r) {
    const double snow_tol = 1.0e-10;
    const double unit_size = p.unit_size;
    const double step_in_days = to_seconds(dt_us) / 86400.0;
    const double dt_hours = to_seconds(dt_us) / 3600.0;
    const double prec = prec_mm_h * dt_hours;
    const double corr_prec = std::max(0.0, prec + s.residual);
    s.residual = std::min(0.0, prec + s.residual);
    const double snow = T < p.tx ? corr_prec : 0.0;
    const double rain = T < p.tx ? 0.0 : corr_prec;

    if (s.sca * s.swe < unit_size && snow < snow_tol) {
        r.outflow = (rain + s.sca * (s.swe + s.free_water) + s.residual) / dt_hours;
        r.swe = 0.0;
        s.residual = 0.0;
        if (r.outflow < 0.0) {
            s.residual = r.outflow;
            r.outflow = 0.0;
        }
        s.nu = p.alpha_0 * unit_size;
        s.alpha = p.alpha_0;
        s.sca = 0.0;
        s.swe = 0.0;
        s.free_water = 0.0;
        s.num_units = 0;
        r.sca = s.sca;
        r.swe = s.swe;
        return;
    }

    const double alpha_0 = p.alpha_0;
    double swe = s.swe;
    ulong nnn = s.num_units;
    double sca = s.sca;
    double nu = s.nu;
    double alpha = s.alpha;
    if (nnn > 0)
        nu *= nnn;
    else {
        nu = alpha_0 * p.unit_size;
        alpha = alpha_0;
    }

    double total_new_snow = snow;
    double lwc = s.free_water;
    const double total_storage = swe + lwc;
    double pot_melt = p.cx * step_in_days * (T - p.ts);
    const double refreeze = std::min(std::max(0.0, -pot_melt * p.cfr), lwc);
    total_new_snow += sca * refreeze;
    lwc -= refreeze;
    pot_melt = std::max(0.0, pot_melt);
    const double new_snow_reduction = std::min(pot_melt, total_new_snow);
    pot_melt -= new_snow_reduction;
    total_new_snow -= new_snow_reduction;

    statistics stat(alpha_0, p.d_range, unit_size);
    ulong n = 0;

    // 1. accumulation
    if (total_new_snow > unit_size) {
        n = (ulong)lrint_(total_new_snow / unit_size);
        compute_shape_vars(stat, nnn, n, 0, sca, 0.0, alpha, nu);
        nnn = (ulong)lrint_(nnn * sca) + n;
        sca = 1.0;
        swe = nnn * unit_size;
    }

    // 2. melting
    if (pot_melt > unit_size) {
        ulong u = (ulong)lrint_(pot_melt / unit_size);
        if (nnn < u + 2) {
            nnn = 0;
            alpha = alpha_0;
            nu = alpha_0 * unit_size;
            swe = 0.0;
            lwc = 0.0;
            sca = 0.0;
        } else {
            const double rel_red_sca = stat.sca_rel_red(u, nnn, nu, alpha);
            const double sca_scale_factor = 1.0 - rel_red_sca;
            sca = s.sca * sca_scale_factor;
            swe = (nnn - u) / sca_scale_factor * unit_size;
            if (swe >= nnn * unit_size) {
                u = (ulong)(long(nnn * rel_red_sca) + 1);
                swe = (nnn - u) / sca_scale_factor * unit_size;
                if (nnn == u) sca = 0.0;
            }
            if (sca < 0.005) {
                nnn = 0;
                alpha = alpha_0;
                nu = alpha_0 * unit_size;
                swe = 0.0;
                lwc = 0.0;
                sca = 0.0;
            } else {
                compute_shape_vars(stat, nnn, n, u, sca, rel_red_sca, alpha, nu);
                nnn = (ulong)lrint_(swe / unit_size);
                swe = nnn * unit_size;
            }
        }
    }

    // 3. lwc from the swe*sca change
    if (s.sca * s.swe > sca * swe) lwc += std::max(0.0, s.swe - swe);
    lwc *= std::min(1.0, s.sca / sca);
    lwc = std::min(lwc, swe * p.max_water_fraction);
    double discharge = s.sca * total_storage + snow - sca * (swe + lwc);
    if (discharge < 0.0) {
        s.residual += discharge;
        discharge = 0.0;
    }

    // 4. rain into lwc and/or discharge
    if (rain > swe * p.max_water_fraction - lwc) {
        discharge += sca * (rain - (swe * p.max_water_fraction - lwc)) + rain * (1.0 - sca);
        lwc = swe * p.max_water_fraction;
    } else {
        lwc += rain;
        discharge += rain * (1.0 - sca);
    }
    if (discharge >= -s.residual) {
        discharge += s.residual;
        s.residual = 0.0;
    }

    // 5. state and response
    if (nnn > 0) nu /= nnn;
    r.outflow = discharge / dt_hours;
    r.swe = sca * (swe + lwc);
    r.sca = sca;
    s.nu = nu;
    s.alpha = alpha;
    s.sca = sca;
    s.swe = swe;
    s.free_water = lwc;
    s.num_units = nnn;
}

}  // namespace skaugen

namespace pt_ss_k {

// core/pt_ss_k.h:24-151 (21 calibration values)
struct parameter {
    priestley_taylor::parameter pt;
    skaugen::parameter ss;
    actual_evapotranspiration::parameter ae;
    kirchner::parameter kirchner;
    precipitation_correction::parameter p_corr;
    glacier_melt::parameter gm;
    pt_gs_k::uhg_parameter routing;
    pt_gs_k::mstack_parameter msp;
    static constexpr size_t size() { return 21; }
    void set(const double* p) {  // pt_ss_k.h:78-101
        int i = 0;
        kirchner.c1 = p[i++]; kirchner.c2 = p[i++]; kirchner.c3 = p[i++];
        ae.ae_scale_factor = p[i++];
        ss.alpha_0 = p[i++]; ss.d_range = p[i++]; ss.unit_size = p[i++]; ss.max_water_fraction = p[i++];
        ss.tx = p[i++]; ss.cx = p[i++]; ss.ts = p[i++]; ss.cfr = p[i++];
        p_corr.scale_factor = p[i++];
        pt.albedo = p[i++]; pt.alpha = p[i++];
        gm.dtf = p[i++];
        routing.velocity = p[i++]; routing.alpha = p[i++]; routing.beta = p[i++];
        gm.direct_response = p[i++];
        msp.reservoir_direct_response_fraction = p[i++];
    }
};

// core/pt_ss_k.h:154-181; flat order nu alpha sca swe free_water residual num_units kirchner.q
struct state {
    skaugen::state snow;
    kirchner::state kirchner;
    static constexpr size_t size() { return 8; }
    void set(const double* v) {
        snow.nu = v[0]; snow.alpha = v[1]; snow.sca = v[2]; snow.swe = v[3]; snow.free_water = v[4];
        snow.residual = v[5]; snow.num_units = size_t(v[6]); kirchner.q = v[7];
    }
    void get(double* v) const {
        v[0] = snow.nu; v[1] = snow.alpha; v[2] = snow.sca; v[3] = snow.swe; v[4] = snow.free_water;
        v[5] = snow.residual; v[6] = double(snow.num_units); v[7] = kirchner.q;
    }
    state scale_snow(double f) const {
        state c{*this};
        c.snow.swe *= f;
        c.snow.free_water *= f;
        c.snow.num_units = size_t(c.snow.num_units * f);
        return c;
    }
};

// core/pt_ss_k.h:184-204
struct response {
    double pot_evapotranspiration = 0;
    skaugen::response snow;
    double ae = 0, q_avg = 0, gm_melt_m3s = 0, total_discharge = 0, charge_m3s = 0;
    response scale_snow(double f) const {
        response c{*this};
        c.snow.outflow *= f;
        c.snow.swe *= f;
        return c;
    }
};

// Collector series in this repo's series-id order (the discharge collector is the prefix):
// avg_discharge, charge_m3s, snow_sca, snow_swe (= snow_total_stored_water of the all-collector),
// snow_outflow, glacier_melt, ae_output, pe_output (pt_ss_k_cell_model.h:38-130)
enum all_series { AVG_DISCHARGE = 0, CHARGE_M3S, SNOW_SCA, SNOW_SWE, SNOW_OUTFLOW, GLACIER_MELT, AE_OUTPUT, PE_OUTPUT, N_ALL };
// state collector (pt_ss_k_cell_model.h:150-205): kirchner_discharge (m3/s), snow_sca, snow_swe (swe_for_cell_area),
// snow_alpha, snow_nu, snow_lwc (free_water_for_cell_area), snow_residual
enum state_series { SC_KIRCHNER = 0, SC_SCA, SC_SWE, SC_ALPHA, SC_NU, SC_LWC, SC_RESIDUAL, N_SC };

struct collectors {
    bool full = true, collect_snow = false, collect_state = false;
    double area = 0;
    std::vector<double> rc[N_ALL];
    std::vector<double> sc[N_SC];
    static void ts_init(std::vector<double>& v, size_t n, int start, int n_steps) {
        pt_gs_k::collectors::ts_init(v, n, start, n_steps);
    }
    void initialize(size_t T, int start, int n, double a) {
        area = a;
        for (int k = 0; k < N_ALL; ++k) {
            bool on = full || k == AVG_DISCHARGE || k == CHARGE_M3S || (collect_snow && (k == SNOW_SCA || k == SNOW_SWE));
            ts_init(rc[k], on ? T : 0, start, n);
        }
        for (int k = 0; k < N_SC; ++k) ts_init(sc[k], collect_state ? T + 1 : 0, start, n > 0 ? n + 1 : 0);
    }
    void collect_response(size_t i, const response& r) {
        rc[AVG_DISCHARGE][i] = mmh_to_m3s(r.total_discharge, area);
        rc[CHARGE_M3S][i] = r.charge_m3s;
        if (full || collect_snow) {
            rc[SNOW_SCA][i] = r.snow.sca;
            rc[SNOW_SWE][i] = r.snow.swe;
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
        sc[SC_KIRCHNER][i] = mmh_to_m3s(s.kirchner.q, area);
        sc[SC_SCA][i] = s.snow.sca;
        sc[SC_SWE][i] = s.snow.swe_for_cell_area();
        sc[SC_ALPHA][i] = s.snow.alpha;
        sc[SC_NU][i] = s.snow.nu;
        sc[SC_LWC][i] = s.snow.free_water_for_cell_area();
        sc[SC_RESIDUAL][i] = s.snow.residual;
    }
};

// core/pt_ss_k.h:210-291
inline void run_pt_ss_k(const geo_cell_data& geo, const parameter& parameter, const fixed_dt& time_axis, int start_step,
                        int n_steps, const pt_gs_k::forcing_view& fv, state& state, collectors& col) {
    priestley_taylor::calculator pt(parameter.pt.albedo, parameter.pt.alpha);
    kirchner::calculator kirchner(parameter.kirchner);
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
        skaugen::step(t1 - t0, parameter.ss, temp, prec, state.snow, response.snow);
        response.gm_melt_m3s = glacier_melt::step(parameter.gm.dtf, temp, geo.area * state.snow.sca, glacier_area_m2);
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
        col.collect_response(i, response.scale_snow(snow_storage_fraction));
        if (i + 1 == i_end) col.collect_state_(i + 1, state.scale_snow(snow_storage_fraction));
    }
}

}  // namespace pt_ss_k
}  // namespace oracle
