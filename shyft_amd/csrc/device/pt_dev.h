// Priestley-Taylor potential evapotranspiration (core/priestley_taylor.h:75-102),
// shared by the pt_gs_k, pt_ss_k and hbv_stack kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "special.h"

namespace shyft_dev {

// returns potential evapotranspiration in mm/s (priestley_taylor.h:75-102)
__device__ inline double pt_pot_evap(double albedo, double alpha, double temperature, double global_radiation,
                                     double rhumidity) {
    const bool neg = temperature < 0;
    const double ck2 = neg ? 17.84362 : 17.08085;
    const double ck3 = neg ? 245.425 : 234.175;
    const double ctt_inv = 1 / (ck3 + temperature);
    const double sat_pressure = 0.610780 * dexp(ck2 * temperature * ctt_inv);
    const double delta = sat_pressure * ck2 * ck3 * ctt_inv * ctt_inv;
    const double vapour_pressure = sat_pressure * rhumidity;
    const double k_temp = temperature + 273.15;
    const double e_atm = 1.24 * dpowr(10 * vapour_pressure / k_temp, 0.143) * (0.85 + 0.5 * rhumidity);
    const double net_rad = 0.0000000567 * dpow4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - albedo);
    const double epot = alpha * delta * net_rad / (delta + 0.066);
    if (epot < 0.0) return 0.0;
    return epot / (2500780 - 2361 * temperature);
}

// the same, plus exp(ae_arg) for the caller's actual_evapotranspiration in one dexp2 call with the saturation
// pressure's exp (two independent exps side by side instead of back to back); the same bits as the two calls
__device__ inline double pt_pot_evap_exp(double albedo, double alpha, double temperature, double global_radiation,
                                         double rhumidity, double ae_arg, double& ae_exp) {
    const bool neg = temperature < 0;
    const double ck2 = neg ? 17.84362 : 17.08085;
    const double ck3 = neg ? 245.425 : 234.175;
    const double ctt_inv = 1 / (ck3 + temperature);
    const dexp_pair e2 = dexp2(ck2 * temperature * ctt_inv, ae_arg);
    ae_exp = e2.b;
    const double sat_pressure = 0.610780 * e2.a;
    const double delta = sat_pressure * ck2 * ck3 * ctt_inv * ctt_inv;
    const double vapour_pressure = sat_pressure * rhumidity;
    const double k_temp = temperature + 273.15;
    const double e_atm = 1.24 * dpowr(10 * vapour_pressure / k_temp, 0.143) * (0.85 + 0.5 * rhumidity);
    const double net_rad = 0.0000000567 * dpow4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - albedo);
    const double epot = alpha * delta * net_rad / (delta + 0.066);
    if (epot < 0.0) return 0.0;
    return epot / (2500780 - 2361 * temperature);
}

}  // namespace shyft_dev
