// hbv_stack per-cell, per-step device physics (gfx950, fp64).
//
// hbv_snow (core/hbv_snow.h:139-272, core/hbv_snow_common.h:14-66), hbv_soil
// (core/hbv_soil.h:55-64), hbv_tank (core/hbv_tank.h:64-80) and
// hbv_actual_evapotranspiration (core/hbv_actual_evapotranspiration.h:32-38).
//
// The snow quantile bins live in registers: every bin array has the compile-time
// size HBV_MAX_BINS and every loop over bins is fully unrolled with a runtime
// bound nb, so "bin idx" accesses become selects instead of scratch memory.
// Arithmetic keeps the reference's operand order (contraction is off), which
// makes the kernel bit-identical to the oracle restatement.
#pragma once
#include <hip/hip_runtime.h>

#include "special.h"
#include "../include_internal/layout.h"


namespace shyft_dev {

#ifndef HBV_MB_OVERRIDE
constexpr int MB = HBV_MAX_BINS;
#else
constexpr int MB = HBV_MB_OVERRIDE;
#endif

// The functions below are templates on the register capacity NB of the bin arrays (deduced from the arrays):
// HBV_MAX_BINS in general, 5 for the kernel variant that serves parameter sets of at most 5 bins (the
// reference's default distribution): 2 x 3 fewer state doubles in registers, and the per-bin loops are shorter.

// a[idx] for a runtime idx over a register array. Written as a bit-mask OR so the
// compiler cannot fold it back into a dynamically indexed (scratch) access, which it
// does with an equivalent chain of selects. Exact: one mask is all-ones.
template <int NB>
__device__ __forceinline__ double hsel(const double (&a)[NB], int idx) {
    unsigned long long v = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) v |= (unsigned long long)__double_as_longlong(a[i]) & (0ULL - (unsigned long long)(idx == i));
    return __longlong_as_double((long long)v);
}

template <int NB>
struct hbv_snow_par_t {
    int nb;
    double s[NB], I[NB];
    double tx, cx, ts, lw, cfr;
};
using hbv_snow_par = hbv_snow_par_t<MB>;

// hbv_snow_common::integrate (hbv_snow_common.h:14-44) for a = 0 (every call in
// the stack integrates from 0)
template <int NB>
__device__ __forceinline__ double hbv_integrate0(const double (&f)[NB], const double (&x)[NB], int n, double b,
                                                 bool f_b_is_zero) {
    const double a = 0.0;
    int left = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i)  // while (a > x[left]) ++left;
        if (i < n && left == i && a > x[i]) left = i + 1;
    double f_l;
    if (fabs(a - hsel(x, left)) > 1.0e-8 && left > 0) {
        --left;
        const double fl = hsel(f, left), fr = hsel(f, left + 1), xl = hsel(x, left), xr = hsel(x, left + 1);
        f_l = (fr - fl) / (xr - xl) * (a - xl) + fl;
    } else {
        f_l = hsel(f, left);
    }
    double area = 0.0, x_l = a;
    bool done = false;
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) {
        if (!done && i >= left && i < n - 1) {
            if (b >= x[i + 1]) {
                area += 0.5 * (f_l + f[i + 1]) * (x[i + 1] - x_l);
                x_l = x[i + 1];
                f_l = f[i + 1];
            } else {
                if (!f_b_is_zero)
                    area += (f_l + 0.5 * (f[i + 1] - f_l) / (x[i + 1] - x_l) * (b - x_l)) * (b - x_l);
                else
                    area += 0.5 * f_l * (b - x_l);
                done = true;
            }
        }
    }
    return area;
}

// hbv_integrate0 of two functions over the same abscissae and limits (the snow step's swe = integral of sp + integral
// of sw): one walk over the bins; each area is accumulated exactly as its own hbv_integrate0 call would
template <int NB>
__device__ __forceinline__ void hbv_integrate0_2(const double (&f)[NB], const double (&g)[NB], const double (&x)[NB],
                                                 int n, double b, bool f_b_is_zero, double& area_f, double& area_g) {
    const double a = 0.0;
    int left = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i)
        if (i < n && left == i && a > x[i]) left = i + 1;
    double f_l, g_l;
    if (fabs(a - hsel(x, left)) > 1.0e-8 && left > 0) {
        --left;
        const double xl = hsel(x, left), xr = hsel(x, left + 1);
        const double fl = hsel(f, left), fr = hsel(f, left + 1);
        const double gl = hsel(g, left), gr = hsel(g, left + 1);
        f_l = (fr - fl) / (xr - xl) * (a - xl) + fl;
        g_l = (gr - gl) / (xr - xl) * (a - xl) + gl;
    } else {
        f_l = hsel(f, left);
        g_l = hsel(g, left);
    }
    double af = 0.0, ag = 0.0, x_l = a;
    bool done = false;
#pragma unroll
    for (int i = 0; i < NB - 1; ++i) {
        if (!done && i >= left && i < n - 1) {
            if (b >= x[i + 1]) {
                af += 0.5 * (f_l + f[i + 1]) * (x[i + 1] - x_l);
                ag += 0.5 * (g_l + g[i + 1]) * (x[i + 1] - x_l);
                x_l = x[i + 1];
                f_l = f[i + 1];
                g_l = g[i + 1];
            } else {
                if (!f_b_is_zero) {
                    af += (f_l + 0.5 * (f[i + 1] - f_l) / (x[i + 1] - x_l) * (b - x_l)) * (b - x_l);
                    ag += (g_l + 0.5 * (g[i + 1] - g_l) / (x[i + 1] - x_l) * (b - x_l)) * (b - x_l);
                } else {
                    af += 0.5 * f_l * (b - x_l);
                    ag += 0.5 * g_l * (b - x_l);
                }
                done = true;
            }
        }
    }
    area_f = af;
    area_g = ag;
}

// hbv_snow::state::distribute -> distribute_snow (hbv_snow.h:95-99, hbv_snow_common.h:47-66)
template <int NB>
__device__ inline void hbv_distribute(const hbv_snow_par_t<NB>& p, double (&sp)[NB], double (&sw)[NB], double& swe,
                                      double& sca) {
#pragma unroll
    for (int i = 0; i < NB; ++i) sp[i] = sw[i] = 0.0;
    if (swe <= 1.0e-3 || sca <= 1.0e-3) {
        swe = sca = 0.0;
        return;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
        if (i < p.nb) sp[i] = sca < p.I[i] ? 0.0 : p.s[i] * swe;
    const double temp_swe = hbv_integrate0(sp, p.I, p.nb, sca, true);
    if (temp_swe < swe) {
        const double corr1 = swe / temp_swe * p.lw;
        const double corr2 = swe / temp_swe * (1.0 - p.lw);
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (i < p.nb) {
                sw[i] = corr1 * sp[i];
                sp[i] *= corr2;
            }
    }
}

// hbv_snow::calculator::step (hbv_snow.h:195-272); returns the outflow in mm/h
template <int NB>
__device__ inline double hbv_snow_step(const hbv_snow_par_t<NB>& p, double (&sp)[NB], double (&sw)[NB], double& s_swe,
                                       double& s_sca, double step_in_days, double dt_hours, double prec_mm_h,
                                       double temp, int32_t& err) {
    double swe = s_swe;
    double sca = s_sca;
    const int nb = p.nb;
    const double prec = prec_mm_h * dt_hours;
    const double total_water = prec + swe;
    double snow, rain;
    if (temp < p.tx) {
        snow = prec;
        rain = 0.0;
    } else {
        snow = 0.0;
        rain = prec;
    }
    swe += snow + sca * rain;
    if (swe < 0.1) {
#pragma unroll
        for (int i = 0; i < NB; ++i) sp[i] = sw[i] = 0.0;
        s_swe = 0.0;
        s_sca = 0.0;
        return dt_hours == 1.0 ? total_water : total_water / dt_hours;  // x / 1.0 == x exactly (hourly steps)
    }
    if (snow > 0.0) {
        int idx = nb - 1;  // sca_index (hbv_snow.h:175-180)
#pragma unroll
        for (int i = NB - 2; i >= 0; --i)
            if (i < nb - 1 && sca >= p.I[i] && sca < p.I[i + 1]) idx = i;
        if (sca > 1.0e-5 && sca < 1.0 - 1.0e-5) {
            double f;
            if (idx == 0) {
                f = sca / (p.I[1] - p.I[0]);
            } else {
                const double Ii = hsel(p.I, idx), Im = hsel(p.I, idx - 1), Ip = hsel(p.I, idx + 1);
                f = (1.0 + (sca - Ii) / (Ii - Im)) / (1.0 + (Ip - Ii) / (Ii - Im));
            }
            // sp[idx] *= f, sw[idx] *= f as a multiply of every bin by f or 1.0 (x * 1.0 == x
            // exactly): the compiler turns a guarded per-bin update back into a scratch access
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const double fi = (i == idx) ? f : 1.0;
                sp[i] *= fi;
                sw[i] *= fi;
            }
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
            if (i < nb) sp[i] += snow * p.s[i];
        sca = p.I[1];  // at least one bin filled after snowfall
        bool found = false;
#pragma unroll
        for (int i = NB - 2; i > 0; --i)
            if (!found && i <= nb - 2 && p.s[i] > 0.0) {
                sca = p.I[i + 1];
                found = true;
            }
    }
    double potmelt = p.cx * step_in_days * (temp - p.ts);
    const double lw = p.lw;
    if (potmelt < 0.0) {
        potmelt *= p.cfr;
#pragma unroll
        for (int i = 0; i < NB; ++i)  // refreeze (hbv_snow.h:146-158)
            if (i < nb && sp[i] > 0.0) {
                if (sw[i] + rain > -potmelt) {
                    sp[i] -= potmelt;
                    sw[i] += potmelt + rain;
                    if (sw[i] > sp[i] * lw) sw[i] = sp[i] * lw;
                } else {
                    sp[i] += sw[i] + rain;
                    sw[i] = 0.0;
                }
            }
    } else {
        int idx = nb;  // melt_index (hbv_snow.h:182-187)
#pragma unroll
        for (int i = NB - 1; i >= 0; --i)
            if (i < nb && sp[i] < potmelt) idx = i;
        if (idx == 0) sca = 0.0;
        else if (idx == nb) sca = 1.0;
        else {
            const double spi = hsel(sp, idx), spm = hsel(sp, idx - 1), Ii = hsel(p.I, idx), Im = hsel(p.I, idx - 1);
            if (spi > 0.0) sca = Ii - (Ii - Im) * (potmelt - spi) / (spm - spi);
            else sca = (1.0 - potmelt / spm) * (sca - Im) + Im;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)  // update_state (hbv_snow.h:160-168)
            if (i < nb) {
                if (sp[i] > potmelt) {
                    sw[i] += potmelt + rain;
                    sp[i] -= potmelt;
                    sw[i] = smin(sw[i], sp[i] * lw);
                } else if (sp[i] > 0.0) {
                    sp[i] = sw[i] = 0.0;
                }
            }
    }
    if (sca < 1.0e-6) {
        swe = 0.0;
    } else {
        const bool f_is_zero = sca >= 1.0 ? false : true;
        // the two integrals (swe = int sp + int sw over the same bins and limits) in one walk (hbv_integrate0_2)
        double a_sp, a_sw;
        hbv_integrate0_2(sp, sw, p.I, nb, sca, f_is_zero, a_sp, a_sw);
        swe = a_sp;
        swe += a_sw;
    }
    if (total_water < swe) {
        if (total_water - swe < -1.0e-6) err = ERR_NEGATIVE_OUTFLOW;  // the reference throws (hbv_snow.h:259-263)
        else swe = total_water;
    }
    s_swe = swe;
    s_sca = sca;
    return dt_hours == 1.0 ? total_water - swe : (total_water - swe) / dt_hours;  // as above
}

}  // namespace shyft_dev
