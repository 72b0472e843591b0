// Priestley-Taylor potential evapotranspiration (core/priestley_taylor.h:75-102),
// shared by the pt_gs_k, pt_ss_k and hbv_stack kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "special.h"
#include "gamma_lean.h"

namespace shyft_dev {

// Priestley-Taylor's exp / log inline by the gamma_lean.h fast paths (SGPR constant table), the out-of-line general
// function only beyond them -- the same bits as dexp / dlog. Measured (r05, year mean per 730-step chunk):
// hbv_stack 512K cells 7.6 -> 7.5 ms, pt_gs_k 1M cells 91.7 -> 90.8 ms, bit-exact
__device__ __forceinline__ double exp_fast(double x, const gsb_k& k) {
    double r = gsb_exp(x, k);
    if (!(__builtin_fabs(x) <= 708.0)) r = dexp(x);
    return r;
}
__device__ __forceinline__ double log_fast(double x, const gsb_k& k) {
    double r = gsb_log(x, k);
    if (!(x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308)) r = dlog(x);
    return r;
}

// returns potential evapotranspiration in mm/s (priestley_taylor.h:75-102)
__device__ inline double pt_pot_evap(double albedo, double alpha, double temperature, double global_radiation,
                                     double rhumidity) {
    const bool neg = temperature < 0;
    const double ck2 = neg ? 17.84362 : 17.08085;
    const double ck3 = neg ? 245.425 : 234.175;
    const double ctt_inv = 1 / (ck3 + temperature);
    const gsb_k k = gsb_load();
    const double sat_pressure = 0.610780 * exp_fast(ck2 * temperature * ctt_inv, k);
    const double delta = sat_pressure * ck2 * ck3 * ctt_inv * ctt_inv;
    const double vapour_pressure = sat_pressure * rhumidity;
    const double k_temp = temperature + 273.15;
    const double e_atm = 1.24 * exp_fast(0.143 * log_fast(10 * vapour_pressure / k_temp, k), k) * (0.85 + 0.5 * rhumidity);
    const double net_rad = 0.0000000567 * dpow4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - albedo);
    const double epot = alpha * delta * net_rad / (delta + 0.066);
    if (epot < 0.0) return 0.0;
    return epot / (2500780 - 2361 * temperature);
}

// the same, plus exp(ae_arg) for the caller's actual_evapotranspiration (inline beside the saturation
// pressure's exp (two independent exps side by side instead of back to back); the same bits as the two calls
__device__ inline double pt_pot_evap_exp(double albedo, double alpha, double temperature, double global_radiation,
                                         double rhumidity, double ae_arg, double& ae_exp) {
    const bool neg = temperature < 0;
    const double ck2 = neg ? 17.84362 : 17.08085;
    const double ck3 = neg ? 245.425 : 234.175;
    const double ctt_inv = 1 / (ck3 + temperature);
    const gsb_k k = gsb_load();
    const double sat_pressure = 0.610780 * exp_fast(ck2 * temperature * ctt_inv, k);
    ae_exp = exp_fast(ae_arg, k);
    const double delta = sat_pressure * ck2 * ck3 * ctt_inv * ctt_inv;
    const double vapour_pressure = sat_pressure * rhumidity;
    const double k_temp = temperature + 273.15;
    const double e_atm = 1.24 * exp_fast(0.143 * log_fast(10 * vapour_pressure / k_temp, k), k) * (0.85 + 0.5 * rhumidity);
    const double net_rad = 0.0000000567 * dpow4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - albedo);
    const double epot = alpha * delta * net_rad / (delta + 0.066);
    if (epot < 0.0) return 0.0;
    return epot / (2500780 - 2361 * temperature);
}

}  // namespace shyft_dev
