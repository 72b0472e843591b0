// ORACLE — test infrastructure only (see common.hpp header).
//
// methods.hpp: the per-step method library used by pt_gs_k (and pt_ss_k):
// priestley_taylor, actual_evapotranspiration, precipitation_correction,
// glacier_melt, gamma_snow (with gamma_p / lgamma / Brent) and kirchner
// (Dormand-Prince 5(4) dense output + trapezoidal average).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <utility>

#include "common.hpp"
#include "mathlib.hpp"

namespace oracle {

// ---------------------------------------------------------------- priestley_taylor
// core/priestley_taylor.h:12-18 (parameter), :56-102 (calculator)
namespace priestley_taylor {
struct parameter {
    double albedo = 0.2;
    double alpha = 1.26;
};
struct calculator {
    double land_albedo, alpha;
    static constexpr double bolz = 0.0000000567;
    static constexpr double psycr = 0.066;
    static constexpr double ck1 = 0.610780;
    static constexpr double ck2[2] = {17.84362, 17.08085};
    static constexpr double ck3[2] = {245.425, 234.175};
    calculator(double land_albedo, double alpha) : land_albedo(land_albedo), alpha(alpha) {}
    // priestley_taylor.h:75-86, result in mm/s
    double potential_evapotranspiration(double temperature, double global_radiation, double rhumidity) const {
        int i = temperature < 0 ? 0 : 1;
        double ctt_inv = 1 / (ck3[i] + temperature);
        double sat_pressure = ck1 * OEXP(ck2[i] * temperature * ctt_inv);
        double delta = sat_pressure * ck2[i] * ck3[i] * ctt_inv * ctt_inv;
        double vapour_pressure = sat_pressure * rhumidity;
        double epot = alpha * delta * net_radiation(temperature, global_radiation, rhumidity, vapour_pressure) / (delta + psycr);
        if (epot < 0.0) return 0.0;
        return epot / (2500780 - 2361 * temperature);
    }
    // priestley_taylor.h:97-102
    double net_radiation(double temperature, double global_radiation, double rhumidity, double vapour_pressure) const {
        double k_temp = temperature + 273.15;
        double e_atm = 1.24 * OPOWR(10 * vapour_pressure / k_temp, 0.143) * (0.85 + 0.5 * rhumidity);
        return bolz * OPOW4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - land_albedo);
    }
};
}  // namespace priestley_taylor

// ---------------------------------------------------------------- actual_evapotranspiration
// core/actual_evapotranspiration.h:28-62
namespace actual_evapotranspiration {
struct parameter { double ae_scale_factor = 1.5; };
inline double calc_pot_ratio(double water_level, double scale_factor) {
    return 1.0 - OEXP(-water_level * 3.0 / scale_factor);
}
inline double calculate_step(double water_level, double potential_evapotranspiration, double scale_factor,
                             double snow_fraction) {
    return potential_evapotranspiration * calc_pot_ratio(water_level, scale_factor) * (1.0 - snow_fraction);
}
}  // namespace actual_evapotranspiration

// core/precipitation_correction.h:24-41
namespace precipitation_correction {
struct parameter { double scale_factor = 1.0; };
}

// core/glacier_melt.h:26-52
namespace glacier_melt {
struct parameter { double dtf = 6.0; double direct_response = 0.0; };
inline double step(double dtf, double t, double snow_covered_area_m2, double glacier_area_m2) {
    if (glacier_area_m2 <= snow_covered_area_m2 || t <= 0.0) return 0.0;
    const double convert_m2_x_mm_d_to_m3_s = 0.001 / 86400.0;
    return dtf * t * (glacier_area_m2 - snow_covered_area_m2) * convert_m2_x_mm_d_to_m3_s;
}
}  // namespace glacier_melt

// ---------------------------------------------------------------- special functions
// The reference calls boost 1.68 boost::math::gamma_p / lgamma with reduced
// precision policies (gamma_snow.h:189-201: digits10<10> for a<2, digits10<5>
// otherwise). boost is not in /root/reference; the restatement takes the
// incomplete gamma from detmath (detmath/detmath.h: full double precision
// series / continued fraction, the same implementation the kernels use, with
// this build's elementary functions), so it agrees with the reference to the
// reference's own ~1e-5 relative precision. The known-answer tests
// (gamma_snow_test.cpp:76-115) pin it; tests/test_detmath.py checks it against
// scipy.special.gammainc.
namespace special {
struct math_policy {
    static double exp(double x) { return OEXP(x); }
    static double log(double x) { return OLOG(x); }
};
inline double lgamma_(double a) { return OLGAMMA(a); }
inline detmath::gamma_pq_result gamma_pq(double a, double x, double eps = 2.220446049250313e-16) {
    return detmath::gamma_pq<math_policy>(a, x, lgamma_(a), eps);
}
inline double gamma_p(double a, double x) { return gamma_pq(a, x).p; }

// boost::math::tools::brent_find_minima (boost 1.68, tools/minima.hpp), restated:
// bracket [min,max], start at max, golden constant 0.3819660f (a float literal),
// tolerance ldexp(1, 1-bits), bits clamped to digits<double>/2 = 26.
template <class F>
std::pair<double, double> brent_find_minima(F f, double min, double max, int bits, uintmax_t& max_iter) {
    bits = std::min(26, bits);
    const double tolerance = std::ldexp(1.0, 1 - bits);
    double x, w, v, u, delta, delta2, fu, fv, fw, fx, mid, fract1, fract2;
    static const double golden = 0.3819660f;
    x = w = v = max;
    fw = fv = fx = f(x);
    delta2 = delta = 0;
    uintmax_t count = max_iter;
    do {
        mid = (min + max) / 2;
        fract1 = tolerance * std::fabs(x) + tolerance / 4;
        fract2 = 2 * fract1;
        if (std::fabs(x - mid) <= (fract2 - (max - min) / 2)) break;
        if (std::fabs(delta2) > fract1) {
            double r = (x - w) * (fx - fv);
            double q = (x - v) * (fx - fw);
            double p = (x - v) * q - (x - w) * r;
            q = 2 * (q - r);
            if (q > 0) p = -p;
            q = std::fabs(q);
            double td = delta2;
            delta2 = delta;
            if ((std::fabs(p) >= std::fabs(q * td / 2)) || (p <= q * (min - x)) || (p >= q * (max - x))) {
                delta2 = (x >= mid) ? min - x : max - x;
                delta = golden * delta2;
            } else {
                delta = p / q;
                u = x + delta;
                if (((u - min) < fract2) || ((max - u) < fract2))
                    delta = (mid - x) < 0 ? -std::fabs(fract1) : std::fabs(fract1);
            }
        } else {
            delta2 = (x >= mid) ? min - x : max - x;
            delta = golden * delta2;
        }
        u = (std::fabs(delta) >= fract1) ? (x + delta) : (delta > 0 ? x + std::fabs(fract1) : x - std::fabs(fract1));
        fu = f(u);
        if (fu <= fx) {
            if (u >= x) min = x; else max = x;
            v = w; w = x; x = u;
            fv = fw; fw = fx; fx = fu;
        } else {
            if (u < x) min = u; else max = u;
            if ((fu <= fw) || (w == x)) {
                v = w; w = u; fv = fw; fw = fu;
            } else if ((fu <= fv) || (v == x) || (v == w)) {
                v = u; fv = fu;
            }
        }
    } while (--count);
    max_iter -= count;
    return std::make_pair(x, fx);
}
}  // namespace special

// ---------------------------------------------------------------- gamma_snow
// core/gamma_snow.h:46-98 (parameter), :101-137 (state/response), :177-494 (calculator)
namespace gamma_snow {
constexpr double tol = 1.0e-10;

struct parameter {
    int64_t winter_end_day_of_year = 100;
    double initial_bare_ground_fraction = 0.04;
    double snow_cv = 0.4;
    double tx = -0.5;
    double wind_scale = 2.0;
    double wind_const = 1.0;
    double max_water = 0.1;
    double surface_magnitude = 30.0;
    double max_albedo = 0.9;
    double min_albedo = 0.6;
    double fast_albedo_decay_rate = 5.0;
    double slow_albedo_decay_rate = 5.0;
    double snowfall_reset_depth = 5.0;
    double glacier_albedo = 0.4;
    bool calculate_iso_pot_energy = false;
    double snow_cv_forest_factor = 0.0;
    double snow_cv_altitude_factor = 0.0;
    int64_t n_winter_days = 221;
    double effective_snow_cv(double forest_fraction, double altitude) const {
        return snow_cv + forest_fraction * snow_cv_forest_factor + altitude * snow_cv_altitude_factor;
    }
    // gamma_snow.h:89-93; t_w_end = trim(t,YEAR) + deltahours(wed*24)
    bool is_snow_season(utctime t) const {
        utctime t_w_end = trim_year(t) + HOUR_US * int64_t(int(winter_end_day_of_year * 24));
        utctime start = t_w_end - HOUR_US * int64_t(int(n_winter_days * 24));
        return t >= start && t < t_w_end;
    }
    bool is_start_melt_season(utctime t) const { return int64_t(day_of_year(t)) == winter_end_day_of_year; }
};

struct state {
    double albedo = 0.4, lwc = 0.1, surface_heat = 30000.0, alpha = 1.26, sdc_melt_mean = 0.0, acc_melt = 0.0,
           iso_pot_energy = 0.0, temp_swe = 0.0;
};
struct response { double sca = 0.0, storage = 0.0, outflow = 0.0; };

struct calculator {
    static constexpr double melt_heat = 333660.0;
    static constexpr double water_heat = 4180.0;
    static constexpr double ice_heat = 2050.0;
    static constexpr double sigma = 5.670373e-8;
    const double BB0 = 0.98 * sigma * OPOW(273.15, 4);

    // gamma_snow.h:195-197: digits10<10> policy for a < 2, digits10<5> otherwise
    double gamma_p(double a, double b) const { return special::gamma_pq(a, b, detmath::gamma_snow_policy_eps(a)).p; }
    double lgamma(double a) const { return special::lgamma_(a); }

    // gamma_snow.h:209-212
    // gamma_p(a+1, z/b) and gamma_p(a, z/b) come from one evaluation (detmath::gamma_pq),
    // at the stricter of the two policies (that of a)
    double calc_q(double a, double b, double z) const {
        const auto g = special::gamma_pq(a, z / b, detmath::gamma_snow_policy_eps(a));
        return a * b * g.p1 + z * (1.0 - g.p);
    }

    // gamma_snow.h:214-227 (Brent, 12 bits, 60 iterations, bracket [0, z1])
    double corr_lwc(double z1, double a1, double b1, double /*z2*/, double a2, double b2) const {
        uintmax_t iterations = 60;
        int digits = 12;
        double Q1 = calc_q(a1, b1, z1);
        auto result = special::brent_find_minima(
            [Q1, a2, b2, this](const double& z) -> double {
                double f = this->calc_q(a2, b2, z) - Q1;
                return f * f;
            },
            0.0, z1, digits, iterations);
        return result.first;
    }

    // gamma_snow.h:230-260
    void calc_snow_state(double shape, double scale, double y0, double lambda, double lwd, double max_water_frac,
                         double temp_swe, double& swe, double& sca) const {
        double y = 0.0, y1 = 0.0;
        const double m = shape * scale;
        if (lambda <= 0.0) {
            swe = m;
            sca = 1.0 - y0;
        } else if (lambda / scale > 1.3 * shape + 20.0) {
            swe = sca = 0.0;
            return;
        } else {
            const double x = lambda / scale;
            y = gamma_p(shape, x);
            y1 = y - OEXP(shape * OLOG(x) - x - lgamma(shape)) / shape;
            swe = m * (1.0 - y1) - lambda * (1 - y);
            sca = (1.0 - y) * (1.0 - y0);
        }
        if (lwd > m)
            swe *= 1.0 + max_water_frac;
        else if (lwd > 0.0) {
            const double sat = lwd / max_water_frac;
            const double x = sat / scale;
            const double ssa = gamma_p(shape, x);
            const double ssa1 = ssa - OEXP(shape * OLOG(x) - x - lgamma(shape)) / shape;
            const double liqwat = max_water_frac * (m * (ssa1 - y1) + sat * (1.0 - ssa) - lambda * (1.0 - y));
            swe += liqwat;
        }
        swe += temp_swe;
        swe *= 1.0 - y0;
    }

    // gamma_snow.h:262-274
    void reset_snow_pack(double& sca, double& lwc, double& alpha, double& sdc_melt_mean, double& acc_melt, double& temp_swe,
                         double storage, const parameter& p) const {
        if (storage > tol) {
            sca = 1.0 - p.initial_bare_ground_fraction;
            sdc_melt_mean = storage / sca;
        } else {
            sca = sdc_melt_mean = 0.0;
        }
        alpha = 1.0 / (p.snow_cv * p.snow_cv);
        temp_swe = lwc = 0.0;
        acc_melt = -1.0;
    }

    // gamma_snow.h:291-493. t, dt in microseconds. chrono arithmetic of the
    // reference (prec_mm_h*dt/calendar::HOUR, outflow*calendar::HOUR/dt) is
    // restated as double arithmetic on the microsecond counts.
    void step(state& s, response& r, utctime t, int64_t dt, const parameter& p, double T, double rad, double prec_mm_h,
              double wind_speed, double rel_hum, double forest_fraction, double altitude) const {
        double sdc_melt_mean = s.sdc_melt_mean;
        double acc_melt = s.acc_melt;
        double iso_pot_energy = s.iso_pot_energy;
        const double prec = (prec_mm_h * double(dt)) / double(HOUR_US);

        if (p.is_start_melt_season(t)) acc_melt = iso_pot_energy = 0.0;

        double snow, rain;
        if (T < p.tx) { snow = prec; rain = 0.0; }
        else { snow = 0.0; rain = prec; }
        if (std::fabs(snow + rain - prec) > 1.0e-8) throw std::runtime_error("Mass balance violation!!!!");

        if (snow < tol && sdc_melt_mean < tol && acc_melt < 0.0) {
            s.albedo = p.max_albedo;
            s.surface_heat = 0.0;
            s.iso_pot_energy = 0.0;
            r.sca = 0.0;
            r.storage = 0.0;
            r.outflow = prec_mm_h;
            return;
        }
        double albedo = s.albedo;
        double lwc = s.lwc;
        double surface_heat = s.surface_heat;
        double alpha = s.alpha;
        double temp_swe = s.temp_swe;
        double sca = 0.0, storage = 0.0, outflow = 0.0;

        const double min_albedo = p.min_albedo;
        const double max_albedo = p.max_albedo;
        const double snow_cv = p.effective_snow_cv(forest_fraction, altitude);
        const double albedo_range = max_albedo - min_albedo;
        const double dt_s = to_seconds(dt);
        const double dt_in_days = dt_s / to_seconds(DAY_US);
        const double slow_albedo_decay_rate = 0.5 * albedo_range * dt_in_days / p.slow_albedo_decay_rate;
        const double fast_albedo_decay_rate = OPOW(2.0, -dt_in_days / p.fast_albedo_decay_rate);

        const double T_k = T + 273.15;
        const double turb = p.wind_scale * wind_speed + p.wind_const;
        double vapour_pressure = 33.864 * (OPOW8(7.38e-3 * T + 0.8072) - 1.9e-5 * std::fabs(1.8 * T + 48.0) + 1.316e-3) * rel_hum;
        if (T < 0.0) vapour_pressure *= 1.0 + 9.72e-3 * T + 4.2e-5 * T * T;

        if (snow > tol)
            albedo += snow * albedo_range / p.snowfall_reset_depth;
        else {
            if (T < 0.0) albedo -= slow_albedo_decay_rate;
            else albedo = min_albedo + fast_albedo_decay_rate * (albedo - min_albedo);
        }
        albedo = std::max(std::min(albedo, max_albedo), min_albedo);

        double effect = rad * (1.0 - albedo);
        effect += 0.98 * sigma * OPOWR(vapour_pressure / T_k, 6.87e-2) * OPOW4(T_k);
        if (T > 0.0 && snow < tol) effect += rain * T * water_heat / dt_s;
        if (T <= 0.0 && rain < tol) effect += snow * T * ice_heat / dt_s;

        if (p.calculate_iso_pot_energy) {
            double iso_effect = effect - BB0 + turb * (T + 1.7 * (vapour_pressure - 6.12));
            iso_pot_energy += iso_effect * dt_s / melt_heat;
        }

        double sst = std::min(0.0, 1.16 * T - 2.09);
        if (sst > -tol)
            effect += turb * (T + 1.7 * (vapour_pressure - 6.12)) - BB0;
        else
            effect += turb * (T - sst + 1.7 * (vapour_pressure - 6.132 * OEXP(0.103 * T - 0.186)))
                      - 0.98 * sigma * OPOW4(sst + 273.15);

        double delta_sh = -surface_heat;
        surface_heat = p.surface_magnitude * ice_heat * sst * 0.5;
        delta_sh += surface_heat;

        double energy = effect * dt_s;
        if (delta_sh > 0.0) energy -= delta_sh;
        double potential_melt = std::max(0.0, energy / melt_heat);

        double sdc_scale = sdc_melt_mean / alpha;
        calc_snow_state(alpha, sdc_scale, p.initial_bare_ground_fraction, acc_melt, lwc, p.max_water, temp_swe, storage, sca);
        double start_storage_value = storage;

        if (acc_melt < 0.0) {
            if (snow < tol) snow = 0.0;
            else {
                double alpha_prev = alpha;
                double sdc_scale_prev = sdc_scale;
                double sdc_snow = snow / (1.0 - p.initial_bare_ground_fraction);
                alpha = (sdc_melt_mean * alpha + sdc_snow / (snow_cv * snow_cv)) / (sdc_snow + sdc_melt_mean);
                sdc_melt_mean += sdc_snow;
                sdc_scale = sdc_melt_mean / alpha;
                if (lwc > 0.0 && sdc_snow > 0.01 * sdc_melt_mean) {
                    double z1 = lwc / p.max_water;
                    double z1_guess = z1 * (1.0 - sdc_snow / sdc_melt_mean);
                    if (z1_guess < tol) z1_guess = z1 * 0.5;
                    z1 = corr_lwc(z1, alpha_prev, sdc_scale_prev > 0.0 ? sdc_scale_prev : sdc_scale, z1_guess, alpha, sdc_scale);
                    lwc = z1 * p.max_water;
#ifndef ORACLE_SKIP_DEAD_CSS  // the HIP kernel omits this call: its outputs are dead (tests/test_oracle_variants.py)
                    calc_snow_state(alpha, sdc_scale, p.initial_bare_ground_fraction, acc_melt, lwc, p.max_water, temp_swe,
                                    storage, sca);
#endif
                }
            }
            lwc += rain;
            if (sdc_melt_mean <= potential_melt) {
                storage = 0.0;
                reset_snow_pack(sca, lwc, alpha, sdc_melt_mean, acc_melt, temp_swe, storage, p);
                sdc_scale = 0.0;
            } else if (potential_melt > 0.0) {
                sdc_melt_mean -= potential_melt;
                lwc += potential_melt;
                alpha = std::max(0.1, sdc_melt_mean / sdc_scale);
                if (alpha > 1.0 / (snow_cv * snow_cv)) alpha = 1.0 / (snow_cv * snow_cv);
                sdc_scale = sdc_melt_mean / alpha;
            }
        } else {
            temp_swe += snow / (1.0 - p.initial_bare_ground_fraction);
            if (temp_swe > 0.0) {
                double melt = std::min(temp_swe, potential_melt);
                temp_swe -= melt;
                potential_melt -= melt;
                lwc += melt;
                if (temp_swe < tol) temp_swe = 0.0;
            }
            acc_melt += potential_melt;
            lwc += rain + potential_melt;
            if (!p.calculate_iso_pot_energy || p.is_snow_season(t)) {
                if (storage < std::max(0.2, 2 * temp_swe) || storage < 0.2 * rain) {
                    storage += snow;
                    reset_snow_pack(sca, lwc, alpha, sdc_melt_mean, acc_melt, temp_swe, storage, p);
                    sdc_scale = sdc_melt_mean / alpha;
                }
            }
        }
        calc_snow_state(alpha, sdc_scale, p.initial_bare_ground_fraction, acc_melt, lwc, p.max_water, temp_swe, storage, sca);
        outflow = prec + start_storage_value - storage;
        if (outflow < 0.0) outflow = 0.0;

        s.albedo = albedo;
        s.lwc = lwc;
        s.surface_heat = surface_heat;
        s.alpha = alpha;
        s.sdc_melt_mean = sdc_melt_mean;
        s.acc_melt = acc_melt;
        s.iso_pot_energy = iso_pot_energy;
        s.temp_swe = temp_swe;
        r.sca = sca;
        r.storage = storage;
        r.outflow = (outflow * double(HOUR_US)) / double(dt);
    }
};
}  // namespace gamma_snow

// ---------------------------------------------------------------- kirchner
// core/kirchner.h:120-237. The ODE integrator is boost 1.68 odeint
// make_dense_output(1e-7, 1e-8, runge_kutta_dopri5<double>) (kirchner.h:171-176),
// restated here: Dormand-Prince 5(4) FSAL tableau, default_error_checker
// (err = |xerr| / (eps_abs + eps_rel*(|x_old| + dt*|dxdt_old|))),
// default_step_adjuster (reject: dt *= max(0.9*err^(-1/3), 0.2);
// accept: if err < 0.5 { err = max(5^-5, err); dt *= 0.9*err^(-1/5) }),
// failed_step_checker (500 attempts per do_step) and the dopri5 continuous
// extension for calc_state.
namespace kirchner {
struct parameter { double c1 = -2.439, c2 = 0.966, c3 = -0.10; };
struct state { double q = 0.1; };
struct response { double q_avg = 0.0; };

struct calculator {
    parameter param;
    double abs_err = 1.0e-7, rel_err = 1.0e-8;
    explicit calculator(const parameter& p) : param(p) {}
    calculator(double abs_err, double rel_err, const parameter& p) : param(p), abs_err(abs_err), rel_err(rel_err) {}

    double g(double ln_q) const { return OEXP(param.c1 + param.c2 * ln_q + param.c3 * ln_q * ln_q); }
    double f(double ln_q, double p, double e) const {
        const double gln_q = g(ln_q);
        return gln_q >= 1.e-30 ? gln_q * ((p - e) * OEXP(-ln_q) - 1.0) : 0.0;
    }

    // state of the dense-output stepper between do_step calls
    struct dopri5 {
        double x_cur, dxdt_cur, x_old, dxdt_old, t, t_old, dt;
        double k3, k4, k5, k6;
    };

    // one successful dense-output do_step (odeint dense_output_runge_kutta<..., fsal>::do_step)
    void do_step(dopri5& s, double p, double e) const {
        const double a2 = 1.0 / 5, a3 = 3.0 / 10, a4 = 4.0 / 5, a5 = 8.0 / 9;
        (void)a2; (void)a3; (void)a4; (void)a5;  // autonomous system: stage times unused
        const double b21 = 1.0 / 5;
        const double b31 = 3.0 / 40, b32 = 9.0 / 40;
        const double b41 = 44.0 / 45, b42 = -56.0 / 15, b43 = 32.0 / 9;
        const double b51 = 19372.0 / 6561, b52 = -25360.0 / 2187, b53 = 64448.0 / 6561, b54 = -212.0 / 729;
        const double b61 = 9017.0 / 3168, b62 = -355.0 / 33, b63 = 46732.0 / 5247, b64 = 49.0 / 176,
                     b65 = -5103.0 / 18656;
        const double c1 = 35.0 / 384, c3 = 500.0 / 1113, c4 = 125.0 / 192, c5 = -2187.0 / 6784, c6 = 11.0 / 84;
        const double dc1 = c1 - 5179.0 / 57600, dc3 = c3 - 7571.0 / 16695, dc4 = c4 - 393.0 / 640,
                     dc5 = c5 - -92097.0 / 339200, dc6 = c6 - 187.0 / 2100, dc7 = -1.0 / 40;
        int attempts = 0;
        s.t_old = s.t;
        for (;;) {
            const double dt = s.dt;
            const double x = s.x_cur, dxdt = s.dxdt_cur;
            double xt = 1.0 * x + dt * b21 * dxdt;
            const double k2 = f(xt, p, e);
            xt = 1.0 * x + dt * b31 * dxdt + dt * b32 * k2;
            const double k3 = f(xt, p, e);
            xt = 1.0 * x + dt * b41 * dxdt + dt * b42 * k2 + dt * b43 * k3;
            const double k4 = f(xt, p, e);
            xt = 1.0 * x + dt * b51 * dxdt + dt * b52 * k2 + dt * b53 * k3 + dt * b54 * k4;
            const double k5 = f(xt, p, e);
            xt = 1.0 * x + dt * b61 * dxdt + dt * b62 * k2 + dt * b63 * k3 + dt * b64 * k4 + dt * b65 * k5;
            const double k6 = f(xt, p, e);
            const double xo = 1.0 * x + dt * c1 * dxdt + dt * c3 * k3 + dt * c4 * k4 + dt * c5 * k5 + dt * c6 * k6;
            const double dxdt_o = f(xo, p, e);
            double xerr = dt * dc1 * dxdt + dt * dc3 * k3 + dt * dc4 * k4 + dt * dc5 * k5 + dt * dc6 * k6 + dt * dc7 * dxdt_o;
            const double err = std::fabs(xerr) / (abs_err + rel_err * (1.0 * std::fabs(x) + 1.0 * dt * std::fabs(dxdt)));
            s.k3 = k3; s.k4 = k4; s.k5 = k5; s.k6 = k6;
            if (err > 1.0) {
                s.dt = dt * std::max(0.9 * OPOWR(err, -1.0 / 3.0), 1.0 / 5.0);
                if (++attempts >= 500) throw std::runtime_error("kirchner: odeint max number of iterations exceeded (500)");
                continue;
            }
            s.t = s.t + dt;
            double ndt = dt;
            if (err < 0.5) {
                const double e2 = std::max(0.00032, err);  // pow(5.0,-5.0), correctly rounded
                ndt = dt * (9.0 / 10.0 * OPOWR(e2, -1.0 / 5.0));
            }
            s.dt = ndt;
            s.x_old = x; s.dxdt_old = dxdt;
            s.x_cur = xo; s.dxdt_cur = dxdt_o;
            return;
        }
    }

    // odeint runge_kutta_dopri5::calc_state (continuous extension)
    double calc_state(const dopri5& s, double t) const {
        const double b1 = 35.0 / 384, b3 = 500.0 / 1113, b4 = 125.0 / 192, b5 = -2187.0 / 6784, b6 = 11.0 / 84;
        const double dt = s.t - s.t_old;
        const double theta = (t - s.t_old) / dt;
        const double X1 = 5.0 * (2558722523.0 - 31403016.0 * theta) / 11282082432.0;
        const double X3 = 100.0 * (882725551.0 - 15701508.0 * theta) / 32700410799.0;
        const double X4 = 25.0 * (443332067.0 - 31403016.0 * theta) / 1880347072.0;
        const double X5 = 32805.0 * (23143187.0 - 3489224.0 * theta) / 199316789632.0;
        const double X6 = 55.0 * (29972135.0 - 7076736.0 * theta) / 822651844.0;
        const double X7 = 10.0 * (7414447.0 - 829305.0 * theta) / 29380423.0;
        const double theta_m_1 = theta - 1.0;
        const double theta_sq = theta * theta;
        const double A = theta_sq * (3.0 - 2.0 * theta);
        const double B = theta_sq * theta_m_1;
        const double C = theta_sq * theta_m_1 * theta_m_1;
        const double D = theta * theta_m_1 * theta_m_1;
        const double b1_theta = A * b1 - C * X1 + D;
        const double b3_theta = A * b3 + C * X3;
        const double b4_theta = A * b4 - C * X4;
        const double b5_theta = A * b5 + C * X5;
        const double b6_theta = A * b6 - C * X6;
        const double b7_theta = B + C * X7;
        return 1.0 * s.x_old + dt * b1_theta * s.dxdt_old + dt * b3_theta * s.k3 + dt * b4_theta * s.k4 +
               dt * b5_theta * s.k5 + dt * b6_theta * s.k6 + dt * b7_theta * s.dxdt_cur;
    }

    // kirchner.h:213-235 with trapezoidal_average (kirchner.h:23-53)
    void step(utctime T0, utctime T1, double& q, double& q_avg, double p, double e) const {
        const double min_q = 0.00001;
        if (q < min_q) q = min_q;
        double x_tmp = OLOG(q);
        const double t0 = 0.0;
        const double t1 = to_seconds(T1 - T0) / to_seconds(HOUR_US);
        dopri5 s{};
        s.x_cur = x_tmp; s.t = t0; s.dt = t1 - t0;
        s.dxdt_cur = f(s.x_cur, p, e);  // deriv initialised on the first do_step
        // trapezoidal_average::initialize(q, t0)
        double area = 0.0, f_a = q, t_start = t0, t_a = t0;
        double current_time = s.t;
        while (current_time < t1) {
            do_step(s, p, e);
            current_time = s.t;
            if (current_time < t1) {
                const double fv = OEXP(s.x_cur);
                area += 0.5 * (f_a + fv) * (current_time - t_a);
                f_a = fv; t_a = current_time;
            }
        }
        x_tmp = calc_state(s, t1);
        q = OEXP(x_tmp);
        area += 0.5 * (f_a + q) * (t1 - t_a);
        t_a = t1;
        q_avg = area / (t_a - t_start);
    }
};
}  // namespace kirchner

}  // namespace oracle
