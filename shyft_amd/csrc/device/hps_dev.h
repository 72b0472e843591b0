// hbv_physical_snow device step (core/hbv_physical_snow.h:227-553) for gfx950, fp64, one lane per cell.
//
// The same expressions in the same order as the oracle (oracle/src/pthpsk.hpp), with the quantile bins
// in fixed register arrays of HBV_MAX_BINS and runtime-indexed reads by hsel (hbv_dev.h). Quirks of the
// reference are kept: the albedo / surface_heat the step works on are local copies never written back
// (only the no-snow reset changes the state's), after snowfall sca is read from the redistribution
// factors s[] (not the quantiles), and the melt-front interpolation sets sp[idx-1] = sp[idx].
#pragma once
#include "hbv_dev.h"
#include "pt_dev.h"

namespace shyft_dev {

constexpr double HPS_TOL = 1.0e-10;  // hbv_physical_snow.h:39

struct hps_par {
    int nb;
    double s[MB], I[MB];
    double tx, lw, cfr, wind_scale, wind_const, surface_magnitude, max_albedo, min_albedo, snowfall_reset_depth;
    bool iso;
    // per launch (depend on the parameters and dt only): slow/fast albedo decay (:344-347), BB0 (:236)
    double slow_decay, fast_decay, BB0;
};

// returns r.outflow (mm over the step, hbv_physical_snow.h:550); r_sca, r_storage as the response
__device__ inline double hps_step(const hps_par& p, double (&sp)[MB], double (&sw)[MB], double (&alb)[MB],
                                  double (&iso)[MB], double& s_swe, double& s_sca, double& s_surface_heat, double dt_us,
                                  double dts, double T, double rad, double prec_mm_h, double wind_speed, double rel_hum,
                                  double& r_sca, double& r_storage, int32_t& err) {
    const double melt_heat = 333660.0, water_heat = 4180.0, ice_heat = 2050.0, sigma = 5.670373e-8;
    const int nb = p.nb;
    const double prec = prec_mm_h * dt_us / 3600000000.0;
    const double total_water = prec + s_swe;
    double snow, rain;
    if (T < p.tx) {
        snow = prec;
        rain = 0.0;
    } else {
        snow = 0.0;
        rain = prec;
    }
    s_swe += snow + s_sca * rain;
    if (s_swe < HPS_TOL) {  // reset (:310-327)
#pragma unroll
        for (int i = 0; i < MB; ++i) {
            sp[i] = sw[i] = 0.0;
            if (i < nb) {
                alb[i] = p.max_albedo;
                iso[i] = 0.0;
            }
        }
        s_swe = 0.0;
        s_sca = 0.0;
        r_sca = 0.0;
        r_storage = 0.0;
        s_surface_heat = 0.0;
        return total_water;
    }
    double albedo[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i) albedo[i] = alb[i];
    const double surface_heat = s_surface_heat;
    const double min_albedo = p.min_albedo, max_albedo = p.max_albedo;
    const double albedo_range = max_albedo - min_albedo;
    const double T_k = T + 273.15;
    const double turb = p.wind_scale * wind_speed + p.wind_const;
    double vapour_pressure = (33.864 * (dpow8(7.38e-3 * T + 0.8072) - 1.9e-5 * fabs(1.8 * T + 48.0) + 1.316e-3) * rel_hum);
    if (T < 0.0) vapour_pressure *= 1.0 + 9.72e-3 * T + 4.2e-5 * T * T;
    double sca = s_sca;
    if (snow > HPS_TOL) {
        int idx = nb - 1;  // sca_index (:266-271)
#pragma unroll
        for (int i = MB - 2; i >= 0; --i)
            if (i < nb - 1 && sca >= p.I[i] && sca < p.I[i + 1]) idx = i;
        if (sca > 1.0e-5 && sca < 1.0 - 1.0e-5) {
            double f;
            if (idx == 0) {
                f = sca / (p.I[1] - p.I[0]);
            } else {
                const double Ii = hsel(p.I, idx), Im = hsel(p.I, idx - 1), Ip = hsel(p.I, idx + 1);
                f = (1.0 + (sca - Ii) / (Ii - Im)) / (1.0 + (Ip - Ii) / (Ii - Im));
            }
#pragma unroll
            for (int i = 0; i < MB; ++i) {  // sp[idx] *= f, sw[idx] *= f (x * 1.0 == x elsewhere)
                const double fi = (i == idx) ? f : 1.0;
                sp[i] *= fi;
                sw[i] *= fi;
            }
        }
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (i < nb) {
                const double currsnow = snow * p.s[i];
                sp[i] += currsnow;
                albedo[i] += (currsnow * albedo_range / p.snowfall_reset_depth);
            }
        bool found = false;  // for (i = n-2; i > 0; --i) if (s[i] > 0) {sca = s[i+1]; break;} else sca = s[1];
#pragma unroll
        for (int i = MB - 2; i > 0; --i)
            if (!found && i <= nb - 2) {
                if (p.s[i] > 0.0) {
                    sca = p.s[i + 1];
                    found = true;
                } else {
                    sca = p.s[1];
                }
            }
    } else {
#pragma unroll
        for (int i = 0; i < MB; ++i)
            if (i < nb) {
                if (T < 0.0) albedo[i] -= p.slow_decay;
                else albedo[i] = (min_albedo + p.fast_decay * (albedo[i] - min_albedo));
            }
    }
    // dpowr and dexp by the inline fast paths (device/pt_dev.h kmath<true>; the same bits): 63.35 -> 62.8 ms per
    // 730-step chunk (r05)
    const kmath<true> hkm;
    const double lw_in = (0.98 * sigma * hkm.exp(6.87e-2 * hkm.log(vapour_pressure / T_k)) * dpow4(T_k));
    const double sst = smin(0.0, 1.16 * T - 2.09);
    double turb_term;
    if (sst > -HPS_TOL) turb_term = turb * (T + 1.7 * (vapour_pressure - 6.12)) - p.BB0;
    else
        turb_term = (turb * (T - sst + 1.7 * (vapour_pressure - 6.132 * hkm.exp(0.103 * T - 0.186))) -
                     0.98 * sigma * dpow4(sst + 273.15));
    double delta_sh = -surface_heat;
    const double new_surface_heat = p.surface_magnitude * ice_heat * sst * 0.5;
    delta_sh += new_surface_heat;
    double pm[MB];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
        double a = albedo[i];
        a = smax(smin(a, max_albedo), min_albedo);
        double eff = rad * (1.0 - a);
        eff += lw_in;
        if (T > 0.0 && snow < HPS_TOL) eff += rain * T * water_heat / dts;
        if (T <= 0.0 && rain < HPS_TOL) eff += snow * p.s[i] * T * ice_heat / dts;
        if (p.iso && i < nb) iso[i] += ((eff - p.BB0 + turb * (T + 1.7 * (vapour_pressure - 6.12))) * dts / melt_heat);
        eff += turb_term;
        double en = eff * dts;
        if (delta_sh > 0.0) en -= delta_sh;
        pm[i] = en / melt_heat;
    }
    int idx = nb;
    bool any_melt = false, stop = false;
#pragma unroll
    for (int i = 0; i < MB; ++i)
        if (i < nb && !stop && pm[i] >= HPS_TOL) {
            any_melt = true;
            if (sp[i] < pm[i]) {
                idx = i;
                stop = true;
            }
        }
    if (any_melt) {
        if (idx == 0) sca = 0.0;
        else if (idx == nb) sca = 1.0;
        else {
            const double spi = hsel(sp, idx), spm = hsel(sp, idx - 1), Ii = hsel(p.I, idx), Im = hsel(p.I, idx - 1);
            const double pmi = hsel(pm, idx);
            if (spi > 0.0) {
                sca = (Ii - (Ii - Im) * (pmi - spi) / spi);
#pragma unroll
                for (int i = 0; i < MB; ++i)  // the reference's sp[idx-1] = sp[idx] inside the denominator
                    if (i == idx - 1) sp[i] = spi;
            } else {
                sca = (1.0 - pmi / spm) * (sca - Im) + Im;
            }
        }
    }
    const double lw = p.lw;
#pragma unroll
    for (int i = 0; i < MB; ++i)
        if (i < nb) {
            if (pm[i] < HPS_TOL) {  // refreeze (:238-253) with potmelt = cfr * potential_melt
                const double potmelt = p.cfr * pm[i];
                if (sp[i] > 0.0) {
                    if (sw[i] + rain > -potmelt) {
                        sp[i] -= potmelt;
                        sw[i] += potmelt + rain;
                        if (sw[i] > sp[i] * lw) sw[i] = sp[i] * lw;
                    } else {
                        sp[i] += sw[i] + rain;
                        sw[i] = 0.0;
                    }
                }
            } else {  // update_state (:256-263)
                const double potmelt = pm[i];
                if (sp[i] > potmelt) {
                    sw[i] += potmelt + rain;
                    sp[i] -= potmelt;
                    sw[i] = smin(sw[i], sp[i] * lw);
                } else if (sp[i] > 0.0) {
                    sp[i] = sw[i] = 0.0;
                }
            }
        }
    double swe;
    if (sca < HPS_TOL) swe = 0.0;
    else {
        const bool f_is_zero = sca >= 1.0 ? false : true;
        swe = hbv_integrate0(sp, p.I, nb, sca, f_is_zero);
        swe += hbv_integrate0(sw, p.I, nb, sca, f_is_zero);
    }
    if (total_water < swe) {
        if (total_water - swe < -HPS_TOL) err = ERR_NEGATIVE_OUTFLOW;  // the reference throws (:540-546)
        else swe = total_water;
    }
    s_swe = swe;
    s_sca = sca;
    r_sca = sca;
    r_storage = swe;
    return total_water - swe;
}

}  // namespace shyft_dev
