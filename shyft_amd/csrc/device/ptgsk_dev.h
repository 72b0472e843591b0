// pt_gs_k per-cell, per-step device physics (gfx950, fp64).
//
// One lane owns one cell; state lives in registers across the time loop.
// Follows core/pt_gs_k.h:312-398 and the methods it calls:
//   priestley_taylor   core/priestley_taylor.h:75-102
//   gamma_snow         core/gamma_snow.h:209-493
//   glacier_melt       core/glacier_melt.h:47-52
//   actual_evap        core/actual_evapotranspiration.h:40-62
//   kirchner           core/kirchner.h:167-237 (boost odeint dopri5 dense output)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_dev.h"
#include "special.h"
#include "gamma_lean.h"
#include "../include_internal/layout.h"


namespace shyft_dev {

constexpr double GS_TOL = 1.0e-10;  // gamma_snow::tol (gamma_snow.h:44)

// ------------------------------------------------------------------ gamma snow
struct gs_state {
    double albedo, lwc, surface_heat, alpha, sdc_melt_mean, acc_melt, iso_pot_energy, temp_swe;
};

// dlgamma(shape) cache: shape (the SDC alpha state) changes only on snowfall,
// melt or reset, so most calls of calc_snow_state within a cell reuse it. The functions below take any cache
// type with this get(): the kernel keeps the cache in its lane's LDS slots (lgamma_cache_lds) rather than in
// registers that the step loop would spill around every call.
struct lgamma_cache {
    double a = -1.0, v = 0.0;
    __device__ inline double get(double shape) {
        if (shape != a) { a = shape; v = dlgamma(shape); }
        return v;
    }
};
// a[threadIdx.x], v[threadIdx.x] of two workgroup arrays (the slot address is formed from threadIdx.x at each
// use, not held in a register)
struct lgamma_cache_lds {
    double* a;
    double* v;
    __device__ inline double get(double shape) {
        const int t = threadIdx.x;
        if (shape != a[t]) { a[t] = shape; v[t] = dlgamma(shape); }
        return v[t];
    }
};

// P(shape, x) and P(shape+1, x) of calc_snow_state's liquid-water evaluation, x = (lwd / max_water) / scale,
// or NaN when the call did not make it. corr_lwc's Q1 = calc_q(alpha_prev, scale_prev, lwc / max_water)
// (gamma_snow.h:225) is the same gamma_p pair at the same point when the step's first calc_snow_state made it.
struct gs_lw {
    double p = __builtin_nan(""), p1 = __builtin_nan("");
};

// calc_snow_state's incomplete gamma: the lean evaluation (device/gamma_lean.h) inline, the general one out of line
// for the lanes it does not cover. 1M cells, the year in 730-step chunks (r05 variants, bit-exact): 92.7 -> 91.6 ms
// per chunk out of line, 85.2 -> 84.0 inline (after the gs_mid slimming)
__device__ __forceinline__ gamma_p_result gs_gamma_pq_cs(double a, double x, double lga) {
    const gsb_k k = gsb_load();
    bool ok;
    gamma_p_result r = gsb_gamma_pq(a, x, lga, detmath::gamma_snow_policy_eps(a), a + 1.0, k, ok);
    if (!ok) r = gs_gamma_pq_general(a, x, lga);
    return r;
}

// gamma_snow.h:230-260
template <class LGC>
__device__ inline void calc_snow_state(double shape, double scale, double y0, double lambda, double lwd,
                                       double max_water_frac, double temp_swe, double& swe, double& sca,
                                       LGC& lgc, gs_lw& lw) {
    lw.p = lw.p1 = __builtin_nan("");
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
        const gamma_p_result g = gs_gamma_pq_cs(shape, x, lgc.get(shape));
        y = g.p;
        y1 = y - g.prefix / shape;
        swe = m * (1.0 - y1) - lambda * (1 - y);
        sca = (1.0 - y) * (1.0 - y0);
    }
    if (lwd > m)
        swe *= 1.0 + max_water_frac;
    else if (lwd > 0.0) {
        const double sat = lwd / max_water_frac;
        const double x = sat / scale;
        const gamma_p_result g = gs_gamma_pq_cs(shape, x, lgc.get(shape));
        lw.p = g.p;
        lw.p1 = g.p1;
        const double ssa = g.p;
        const double ssa1 = ssa - g.prefix / shape;
        const double liqwat = max_water_frac * (m * (ssa1 - y1) + sat * (1.0 - ssa) - lambda * (1.0 - y));
        swe += liqwat;
    }
    swe += temp_swe;
    swe *= 1.0 - y0;
}

// calc_q (gamma_snow.h:209-212); gamma_p(a+1, z/b) and gamma_p(a, z/b) from one gamma_pq
__device__ inline double gs_calc_q(double a, double b, double z, double lga) {
    const gamma_p_result g = gs_gamma_pq(a, z / b, lga);
    return a * b * g.p1 + z * (1.0 - g.p);
}


// corr_lwc (gamma_snow.h:214-227): boost brent_find_minima over [0, z1],
// 12 bits, 60 iterations; golden constant is the float literal 0.3819660f.
#ifdef SHYFT_PROF
#define SHYFT_PROF_NF , int& nf_evals
#else
#define SHYFT_PROF_NF
#endif
// q1: Q1 = calc_q(a1, b1, z1) when the caller already has it (from the step's first calc_snow_state, gs_lw),
// else NaN
// lga2 = lgamma(a2): the job's lane evaluates it (its lgamma cache needs it for the step's calc_snow_state after
// the solve anyway), so the solving wavefront does not
__device__ __noinline__ double gs_corr_lwc(double z1, double a1, double b1, double a2, double b2,
                                           double q1, double lga2 SHYFT_PROF_NF) {
#ifdef SHYFT_ABLATE_BRENT
    return z1 * 0.5;  // timing ablation only (wrong results)
#endif
    const double Q1 = q1 == q1 ? q1 : gs_calc_q(a1, b1, z1, dlgamma(a1));
    auto f = [&](double z) {
#ifdef SHYFT_PROF
        ++nf_evals;
#endif
        const double v = gs_calc_q(a2, b2, z, lga2) - Q1;
        return v * v;
    };
    double min = 0.0, max = z1;
    const double tolerance = 0x1p-11;  // ldexp(1, 1-12)
    const double golden = (double)0.3819660f;
    double x, w, v, u, delta, delta2, fu, fv, fw, fx, mid, fract1, fract2;
    x = w = v = max;
    fw = fv = fx = f(x);
    delta2 = delta = 0;
    int count = 60;
    do {
        mid = (min + max) / 2;
        fract1 = tolerance * fabs(x) + tolerance / 4;
        fract2 = 2 * fract1;
        if (fabs(x - mid) <= (fract2 - (max - min) / 2)) break;
        if (fabs(delta2) > fract1) {
            double r = (x - w) * (fx - fv);
            double q = (x - v) * (fx - fw);
            double p = (x - v) * q - (x - w) * r;
            q = 2 * (q - r);
            if (q > 0) p = -p;
            q = fabs(q);
            double td = delta2;
            delta2 = delta;
            if ((fabs(p) >= fabs(q * td / 2)) || (p <= q * (min - x)) || (p >= q * (max - x))) {
                delta2 = (x >= mid) ? min - x : max - x;
                delta = golden * delta2;
            } else {
                delta = p / q;
                u = x + delta;
                if (((u - min) < fract2) || ((max - u) < fract2)) delta = (mid - x) < 0 ? -fabs(fract1) : fabs(fract1);
            }
        } else {
            delta2 = (x >= mid) ? min - x : max - x;
            delta = golden * delta2;
        }
        u = (fabs(delta) >= fract1) ? (x + delta) : (delta > 0 ? x + fabs(fract1) : x - fabs(fract1));
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
    return x;
}

// per-cell constants of the snow routine
struct gs_cell {
    double forest_fraction, altitude;
    double cv2;       // effective_snow_cv(forest, altitude)^2 (gamma_snow.h:85-87)
    double inv_cv2;   // 1.0/cv2
};

// gamma_snow::calculator::step (gamma_snow.h:291-493), split at its only
// expensive, rarely taken call -- corr_lwc's Brent minimisation
// (gamma_snow.h:425-435) -- so a workgroup can hand the Brent jobs of its lanes
// to as few wavefronts as possible (see the kernel). gs_front runs everything up
// to that point and says whether a Brent job is needed; gs_back finishes the
// step given the Brent result. gs_step = front + Brent + back.
// P is the per-set parameter row (layout.h); dt_s = to_seconds(dt), dt_us the
// microsecond count (prec = prec_mm_h*dt/HOUR, outflow*HOUR/dt as the reference
// evaluates them).
// gs_front writes the state fields it has finished (albedo, surface_heat, iso_pot_energy, and alpha,
// sdc_melt_mean, acc_melt as gs_back starts from them) straight into the state; gs_mid carries only what gs_back
// needs besides the state, so fewer values stay live across the workgroup's Brent phase (r05: 16 -> 5 doubles;
// the same values in the same operations; 1M cells, 730-step chunks: 92.0 -> 85.0 ms per chunk). Recomputing
// snow / rain / sdc_scale in gs_back instead of carrying them measured no better.
struct gs_mid {
    bool done;  // the early "no snow" path was taken (gamma_snow.h:313-322)
    bool need;  // a corr_lwc job was handed to the caller's enqueue
    double snow, rain, potential_melt, start_storage, sdc_scale;  // (gs_front leaves storage == start_storage)
};

// The snow storage of the state as it leaves a step: gs_back's final calc_snow_state(alpha, sdc_melt_mean/alpha,
// ibgf, acc_melt, lwc, ...) -- exactly the call gs_front opens the next step with (same state fields, and
// gs_back always leaves sdc_scale == sdc_melt_mean / alpha), unless the winter-end day resets acc_melt in between
// or the step took the early no-snow path. gs_front then reuses the value instead of evaluating the incomplete
// gamma functions again: same function of the same arguments, so the same bits (gamma_snow.h:359 vs :459).
struct gs_carry {
    double storage = 0.0;
    gs_lw lw;
    bool ok = false;
};

// enqueue(z1, a1, b1, a2, b2, q1, lga2) receives the step's corr_lwc job where it arises (q1 = calc_q(a1, b1, z1)
// or NaN, lga2 = lgamma(a2)): the kernel writes it straight into its workgroup's LDS job queue, so the seven job
// values are not held in registers (or scratch) until a later queue pass
template <class LGC, class Enqueue>
__device__ inline void gs_front(gs_state& s, gs_mid& m, bool start_melt, double dt_s, double dt_us,
                                      const double* __restrict__ P, const gs_cell& cc, double T, double rad,
                                      double prec_mm_h, double wind_speed, double rel_hum, LGC& lgc,
                                      const gs_carry& carry, Enqueue&& enqueue) {
    m.need = false;
    m.done = false;
    double sdc_melt_mean = s.sdc_melt_mean;
    double acc_melt = s.acc_melt;
    double iso_pot_energy = s.iso_pot_energy;
    const double prec = (prec_mm_h * dt_us) / 3600000000.0;
    if (start_melt) acc_melt = iso_pot_energy = 0.0;
    double snow, rain;
    if (T < P[PK_TX]) { snow = prec; rain = 0.0; }
    else { snow = 0.0; rain = prec; }
    if (snow < GS_TOL && sdc_melt_mean < GS_TOL && acc_melt < 0.0) {
        m.done = true;  // (acc_melt was not reset here: the early path needs acc_melt < 0)
        return;
    }
    double albedo = s.albedo;
    double lwc = s.lwc;
    double surface_heat = s.surface_heat;
    double alpha = s.alpha;
    const double temp_swe = s.temp_swe;
    double sca = 0.0, storage = 0.0;
    const double min_albedo = P[PK_MIN_ALBEDO];
    const double max_albedo = P[PK_MAX_ALBEDO];
    const double ibgf = P[PK_IBGF];
    const double max_water = P[PK_MAX_WATER];

    const double T_k = T + 273.15;
    const double turb = P[PK_WIND_SCALE] * wind_speed + P[PK_WIND_CONST];
    double vapour_pressure = 33.864 * (dpow8(7.38e-3 * T + 0.8072) - 1.9e-5 * fabs(1.8 * T + 48.0) + 1.316e-3) * rel_hum;
    if (T < 0.0) vapour_pressure *= 1.0 + 9.72e-3 * T + 4.2e-5 * T * T;

    if (snow > GS_TOL)
        albedo += snow * P[PK_ALBEDO_RANGE] / P[PK_SNOWFALL_RESET];
    else {
        if (T < 0.0) albedo -= P[PK_SLOW_DECAY];
        else albedo = min_albedo + P[PK_FAST_DECAY] * (albedo - min_albedo);
    }
    albedo = smax(smin(albedo, max_albedo), min_albedo);

    const double sigma = 5.670373e-8;
    double effect = rad * (1.0 - albedo);
    // dpowr(vapour_pressure / T_k, 6.87e-2)'s exp and the sub-zero surface branch's exp in one dexp2 call (inline
    // gamma_lean.h exp / log here measured 1 % slower over the year, r05)
    const dexp_pair gse = dexp2(6.87e-2 * dlog(vapour_pressure / T_k), 0.103 * T - 0.186);
    effect += 0.98 * sigma * gse.a * dpow4(T_k);
    if (T > 0.0 && snow < GS_TOL) effect += rain * T * 4180.0 / dt_s;
    if (T <= 0.0 && rain < GS_TOL) effect += snow * T * 2050.0 / dt_s;

    if (P[PK_ISO] != 0.0) {
        const double iso_effect = effect - P[PK_BB0] + turb * (T + 1.7 * (vapour_pressure - 6.12));
        iso_pot_energy += iso_effect * dt_s / 333660.0;
    }
    const double sst = smin(0.0, 1.16 * T - 2.09);
    if (sst > -GS_TOL)
        effect += turb * (T + 1.7 * (vapour_pressure - 6.12)) - P[PK_BB0];
    else
        effect += turb * (T - sst + 1.7 * (vapour_pressure - 6.132 * gse.b)) -
                  0.98 * sigma * dpow4(sst + 273.15);

    double delta_sh = -surface_heat;
    surface_heat = P[PK_SURFACE_MAG] * 2050.0 * sst * 0.5;
    delta_sh += surface_heat;
    double energy = effect * dt_s;
    if (delta_sh > 0.0) energy -= delta_sh;
    const double potential_melt = smax(0.0, energy / 333660.0);

    double sdc_scale = sdc_melt_mean / alpha;
    gs_lw lw;
    if (carry.ok && !start_melt) {
        storage = carry.storage;  // sca of this call is not used by gs_back
        lw = carry.lw;
    } else {
        calc_snow_state(alpha, sdc_scale, ibgf, acc_melt, lwc, max_water, temp_swe, storage, sca, lgc, lw);
    }
    m.start_storage = storage;

    if (acc_melt < 0.0) {
        if (snow < GS_TOL) snow = 0.0;
        else {
            const double alpha_prev = alpha;
            const double sdc_scale_prev = sdc_scale;
            const double sdc_snow = snow / (1.0 - ibgf);
            alpha = (sdc_melt_mean * alpha + sdc_snow / cc.cv2) / (sdc_snow + sdc_melt_mean);
            sdc_melt_mean += sdc_snow;
            sdc_scale = sdc_melt_mean / alpha;
            if (lwc > 0.0 && sdc_snow > 0.01 * sdc_melt_mean) {
                // z1_guess (gamma_snow.h:427-430) is computed by the reference but unused by corr_lwc
                m.need = true;
                const double z1 = lwc / max_water;
                const double a1 = alpha_prev;
                const double b1 = sdc_scale_prev > 0.0 ? sdc_scale_prev : sdc_scale;
                // calc_q(a1, b1, z1) = a1 b1 P(a1+1, z1/b1) + z1 (1 - P(a1, z1/b1)) (gamma_snow.h:209-212) from the
                // opening calc_snow_state's liquid-water pair (same shape, scale and point, z1 / b1 = sat / scale)
                const double q1 = (sdc_scale_prev > 0.0 && lw.p == lw.p) ? a1 * b1 * lw.p1 + z1 * (1.0 - lw.p)
                                                                          : __builtin_nan("");
                enqueue(z1, a1, b1, alpha, sdc_scale, q1, lgc.get(alpha));
            }
        }
    }
    (void)sca;  // (its value is dead: gs_back's final calc_snow_state assigns sca)
    m.snow = snow;
    m.rain = rain;
    m.potential_melt = potential_melt;
    m.sdc_scale = sdc_scale;
    s.albedo = albedo;
    s.surface_heat = surface_heat;
    s.iso_pot_energy = iso_pot_energy;
    s.alpha = alpha;
    s.sdc_melt_mean = sdc_melt_mean;
    s.acc_melt = acc_melt;
    // (lwc and temp_swe are unchanged until gs_back)
}

template <class LGC>
__device__ inline void gs_back(gs_state& s, const gs_mid& m, double z, double& r_sca, double& r_storage,
                                     double& r_outflow, bool snow_season, double dt_us, const double* __restrict__ P,
                                     const gs_cell& cc, double prec_mm_h, LGC& lgc, gs_carry& carry) {
    if (m.done) {
        carry.ok = false;
        carry.storage = 0.0;  // (never read while ok is false: defined here so that the carry is dead across the
        carry.lw = gs_lw();   // workgroup's Brent phase; r05: VGPR spills 49 -> 26, 83.4 -> 82.9 ms per chunk)
        s.albedo = P[PK_MAX_ALBEDO];
        s.surface_heat = 0.0;
        s.iso_pot_energy = 0.0;
        // (s.acc_melt as it was: the early path only triggers when it was not reset)
        r_sca = 0.0;
        r_storage = 0.0;
        r_outflow = prec_mm_h;
        return;
    }
    const double ibgf = P[PK_IBGF];
    const double max_water = P[PK_MAX_WATER];
    const double prec = (prec_mm_h * dt_us) / 3600000000.0;  // gs_front's expression
    double snow = m.snow;
    const double rain = m.rain;
    double lwc = s.lwc, alpha = s.alpha, temp_swe = s.temp_swe, sca = 0.0;
    double storage = m.start_storage;
    double sdc_melt_mean = s.sdc_melt_mean, acc_melt = s.acc_melt, potential_melt = m.potential_melt;
    double sdc_scale = m.sdc_scale;
    if (acc_melt < 0.0) {
        // the reference follows corr_lwc with calc_snow_state(alpha, sdc_scale, ..., lwc, ..., storage, sca)
        // (gamma_snow.h:433-434), whose two outputs are dead: this branch only overwrites storage and sca (or
        // leaves them alone) before the step's final calc_snow_state assigns both (gamma_snow.h:472, below), and
        // calc_snow_state reads neither. Skipping it changes no bit of the step (its incomplete-gamma evaluation,
        // run by every wavefront holding a job lane, was ~6 % of the kernel's static code).
        if (m.need) lwc = z * max_water;
        lwc += rain;
        if (sdc_melt_mean <= potential_melt) {
            storage = 0.0;
            // reset_snow_pack (gamma_snow.h:262-274) with storage == 0
            sca = sdc_melt_mean = 0.0;
            alpha = P[PK_INV_CV2_PARAM];
            temp_swe = lwc = 0.0;
            acc_melt = -1.0;
            sdc_scale = 0.0;
        } else if (potential_melt > 0.0) {
            sdc_melt_mean -= potential_melt;
            lwc += potential_melt;
            alpha = smax(0.1, sdc_melt_mean / sdc_scale);
            if (alpha > cc.inv_cv2) alpha = cc.inv_cv2;
            sdc_scale = sdc_melt_mean / alpha;
        }
    } else {
        temp_swe += snow / (1.0 - ibgf);
        if (temp_swe > 0.0) {
            const double melt = smin(temp_swe, potential_melt);
            temp_swe -= melt;
            potential_melt -= melt;
            lwc += melt;
            if (temp_swe < GS_TOL) temp_swe = 0.0;
        }
        acc_melt += potential_melt;
        lwc += rain + potential_melt;
        if (P[PK_ISO] == 0.0 || snow_season) {
            if (storage < smax(0.2, 2 * temp_swe) || storage < 0.2 * rain) {
                storage += snow;
                // reset_snow_pack (gamma_snow.h:262-274)
                if (storage > GS_TOL) {
                    sca = 1.0 - ibgf;
                    sdc_melt_mean = storage / sca;
                } else {
                    sca = sdc_melt_mean = 0.0;
                }
                alpha = P[PK_INV_CV2_PARAM];
                temp_swe = lwc = 0.0;
                acc_melt = -1.0;
                sdc_scale = sdc_melt_mean / alpha;
            }
        }
    }
    calc_snow_state(alpha, sdc_scale, ibgf, acc_melt, lwc, max_water, temp_swe, storage, sca, lgc, carry.lw);
    carry.storage = storage;
    carry.ok = true;
    double outflow = prec + m.start_storage - storage;
    if (outflow < 0.0) outflow = 0.0;

    s.lwc = lwc;
    s.alpha = alpha;
    s.sdc_melt_mean = sdc_melt_mean;
    s.acc_melt = acc_melt;
    s.temp_swe = temp_swe;
    r_sca = sca;
    r_storage = storage;
    r_outflow = (outflow * 3600000000.0) / dt_us;
}

// ------------------------------------------------------------------ kirchner
// kirchner.h:186-198
// both of kirchner_f's exps in one dexp2 call (exp(-ln_q) is evaluated even when g < 1e-30 does not use it; the
// value is the same either way)
__device__ inline double kirchner_f(double ln_q, double p_minus_e, double c1, double c2, double c3) {
    const dexp_pair ge = dexp2(c1 + c2 * ln_q + c3 * ln_q * ln_q, -ln_q);
    return ge.a >= 1.e-30 ? ge.a * (p_minus_e * ge.b - 1.0) : 0.0;
}

// kirchner::calculator::step with trapezoidal_average (kirchner.h:23-53, 213-235).
// The odeint dense-output dopri5 loop (one do_step = repeated try_step until
// accepted) is flattened into one loop of try_steps so lanes of a wave that
// need different numbers of attempts stay in one convergent loop.
// Returns false if a do_step needed 500 attempts (odeint failed_step_checker).
// INL: the step's exps and logs inline by the gamma_lean.h fast paths (one SGPR constant table per call, the general
// out-of-line functions only beyond them) instead of out-of-line dexp2 / dexp / dlog calls -- the same bits (pt_gs_k:
// 90.8 -> 89.7 ms per 730-step chunk; the other stacks keep the calls, device/pt_dev.h)
template <bool INL = false>
__device__ inline bool kirchner_step(double& q, double& q_avg, double p, double e, double t1, double c1, double c2,
                                     double c3) {
    const double abs_err = 1.0e-7, rel_err = 1.0e-8;
    if (q < 0.00001) q = 0.00001;
#ifdef SHYFT_ABLATE_KIRCHNER
    q_avg = q; q = q + 0.01 * (p - e); return true;  // timing ablation only (wrong results)
#endif
    const double pe = p - e;
    const kmath<INL> km;
    auto kirchner_f = [&](double ln_q, double p_minus_e, double c1_, double c2_, double c3_) {
        const dexp_pair ge = km.exp2(c1_ + c2_ * ln_q + c3_ * ln_q * ln_q, -ln_q);
        return ge.a >= 1.e-30 ? ge.a * (p_minus_e * ge.b - 1.0) : 0.0;
    };
    auto dexp = [&](double v) { return km.exp(v); };
    auto dlog = [&](double v) { return km.log(v); };
    double x = dlog(q);
    double dxdt = kirchner_f(x, pe, c1, c2, c3);
    double t = 0.0, dt = t1;
    double x_old = x, dxdt_old = dxdt, t_old = 0.0;
    double k3 = 0, k4 = 0, k5 = 0, k6 = 0;
    double area = 0.0, f_a = q, t_a = 0.0;
    int attempts = 0;
    bool ok = true;
    // dopri5 tableau (odeint runge_kutta_dopri5)
    const double b21 = 1.0 / 5;
    const double b31 = 3.0 / 40, b32 = 9.0 / 40;
    const double b41 = 44.0 / 45, b42 = -56.0 / 15, b43 = 32.0 / 9;
    const double b51 = 19372.0 / 6561, b52 = -25360.0 / 2187, b53 = 64448.0 / 6561, b54 = -212.0 / 729;
    const double b61 = 9017.0 / 3168, b62 = -355.0 / 33, b63 = 46732.0 / 5247, b64 = 49.0 / 176, b65 = -5103.0 / 18656;
    const double c1_ = 35.0 / 384, c3_ = 500.0 / 1113, c4_ = 125.0 / 192, c5_ = -2187.0 / 6784, c6_ = 11.0 / 84;
    const double dc1 = c1_ - 5179.0 / 57600, dc3 = c3_ - 7571.0 / 16695, dc4 = c4_ - 393.0 / 640,
                 dc5 = c5_ - -92097.0 / 339200, dc6 = c6_ - 187.0 / 2100, dc7 = -1.0 / 40;
    // one try_step of size h (the loop's dt): the same expressions with h in dt's place; returns false when the
    // step failed 500 times
    auto attempt = [&](const double h) -> bool {
        double xt = 1.0 * x + h * b21 * dxdt;
        const double k2 = kirchner_f(xt, pe, c1, c2, c3);
        xt = 1.0 * x + h * b31 * dxdt + h * b32 * k2;
        const double s3 = kirchner_f(xt, pe, c1, c2, c3);
        xt = 1.0 * x + h * b41 * dxdt + h * b42 * k2 + h * b43 * s3;
        const double s4 = kirchner_f(xt, pe, c1, c2, c3);
        xt = 1.0 * x + h * b51 * dxdt + h * b52 * k2 + h * b53 * s3 + h * b54 * s4;
        const double s5 = kirchner_f(xt, pe, c1, c2, c3);
        xt = 1.0 * x + h * b61 * dxdt + h * b62 * k2 + h * b63 * s3 + h * b64 * s4 + h * b65 * s5;
        const double s6 = kirchner_f(xt, pe, c1, c2, c3);
        const double xo = 1.0 * x + h * c1_ * dxdt + h * c3_ * s3 + h * c4_ * s4 + h * c5_ * s5 + h * c6_ * s6;
        const double dxdt_o = kirchner_f(xo, pe, c1, c2, c3);
        const double xerr = h * dc1 * dxdt + h * dc3 * s3 + h * dc4 * s4 + h * dc5 * s5 + h * dc6 * s6 + h * dc7 * dxdt_o;
        const double err = fabs(xerr) / (abs_err + rel_err * (1.0 * fabs(x) + 1.0 * h * fabs(dxdt)));
        if (err > 1.0) {
            dt = h * smax(0.9 * dexp(-1.0 / 3.0 * dlog(err)), 1.0 / 5.0);  // dpowr(err, -1/3)
            return ++attempts < 500;
        }
        attempts = 0;
        t_old = t;
        t = t + h;
        dt = h;
        // the grown step size only matters if the loop goes on (dt is dead once t reaches t1: every call starts
        // from dt = t1), so the log + exp of the controller are skipped on the call's last step
        if (err < 0.5 && t < t1) {
            const double e2 = smax(0.00032, err);  // dpow(5.0, -5.0)
            dt = h * (9.0 / 10.0 * dexp(-1.0 / 5.0 * dlog(e2)));  // dpowr(e2, -1/5)
        }
        x_old = x; dxdt_old = dxdt;
        x = xo; dxdt = dxdt_o;
        k3 = s3; k4 = s4; k5 = s5; k6 = s6;
        if (t < t1) {
            const double fv = dexp(x);
            area += 0.5 * (f_a + fv) * (t - t_a);
            f_a = fv;
            t_a = t;
        }
        return true;
    };
    // the call's first attempt has dt = t1 on every lane; for hourly steps (t1 == 1.0, wave-uniform) it runs with the
    // constant 1.0, so the 27 products with the step size fold away (1.0 * v == v: the same bits). r06, 1M cells, the
    // year in 730-step chunks: pt_gs_k 70.9 -> 70.0 ms, pt_ss_k 70.8 -> 69.5, pt_hs_k 28.8 -> 27.8, bit-exact
    // (profiles/r06/kirchner_peel_variants.txt)
    if (t1 == 1.0) ok = attempt(1.0);
    while (ok && t < t1) ok = attempt(dt);
    // calc_state(t1): dopri5 continuous extension
    struct ext_coeffs {
        double b1, b3, b4, b5, b6, b7;
    };
    auto coeffs = [](double theta) {
        const double b1 = 35.0 / 384, b3 = 500.0 / 1113, b4 = 125.0 / 192, b5 = -2187.0 / 6784, b6 = 11.0 / 84;
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
        ext_coeffs c;
        c.b1 = A * b1 - C * X1 + D;
        c.b3 = A * b3 + C * X3;
        c.b4 = A * b4 - C * X4;
        c.b5 = A * b5 + C * X5;
        c.b6 = A * b6 - C * X6;
        c.b7 = B + C * X7;
        return c;
    };
    const double h = t - t_old;
    // the usual hour: one accepted step from 0 to t1, so theta = (t1 - 0) / t1 = 1 exactly, and the coefficients are
    // the same IEEE operations on the constant 1.0 -- folded at compile time: six divisions and the rest of the
    // polynomial algebra fewer per call (the oracle evaluates them at run time, with the same bits). The weighted sum
    // is written out in each branch (one value joins, not six coefficients: fewer registers live at the join).
    // r06, 1M cells, the year in 730-step chunks: pt_gs_k 72.9 -> 70.8 ms, pt_ss_k 72.6 -> 70.3 (with the coefficients
    // joined instead: 71.5 / 70.9; profiles/r06/kirchner_extension_variants.txt)
    auto sum = [&](const ext_coeffs& c) {
        return 1.0 * x_old + h * c.b1 * dxdt_old + h * c.b3 * k3 + h * c.b4 * k4 + h * c.b5 * k5 + h * c.b6 * k6 +
               h * c.b7 * dxdt;
    };
    if (t_old == 0.0 && h == t1 && t1 > 0.0 && t1 <= 1.7976931348623157e308)
        x = sum(coeffs(1.0));
    else
        x = sum(coeffs((t1 - t_old) / h));
    q = dexp(x);
    area += 0.5 * (f_a + q) * (t1 - t_a);
    q_avg = t1 == 1.0 ? area : area / (t1 - 0.0);  // x / 1.0 == x exactly (hourly steps)
    return ok;
}

}  // namespace shyft_dev
