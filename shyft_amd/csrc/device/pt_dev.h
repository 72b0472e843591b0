// Priestley-Taylor potential evapotranspiration (core/priestley_taylor.h:75-102),
// shared by the pt_gs_k, pt_ss_k and hbv_stack kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "special.h"
#include "gamma_lean.h"

namespace shyft_dev {

// exp / log by the device/fastmath.h fast paths inline (SGPR constant table), the out-of-line general function only
// beyond them -- the same bits as dexp / dlog. The stacks take them inline (template argument INL = true) since the
// constants are loaded per call (kmath<true> below) and pt_gs_k's parameter row moved to LDS; measured r05 (ms per
// 730-step chunk, year mean, same box): hbv_stack 7.45 -> 7.25, pt_hs_k 33.95 -> 32.95, pt_hps_k 67.65 -> 63.05.
// pt_ss_k keeps the calls: inline measured 87.1 -> 86.65 but its VGPR spills 19 -> 23 raised the C5 line's HBM
// traffic from 1.06x to 1.56x the algorithmic bytes. (With one table held across the whole call, hbv_stack and
// pt_hs_k had measured 3-10 % slower: 54 SGPRs live beside the step loop's uniform values.)
// mathematics of a kernel: out-of-line calls (INL = false) or inline fast paths (INL = true: exp_fast / log_fast)
template <bool INL>
struct kmath {
    __device__ kmath() {}
    __device__ double exp(double x) const { return dexp(x); }
    __device__ double log(double x) const { return dlog(x); }
    __device__ dexp_pair exp2(double x, double y) const { return dexp2(x, y); }
};
// every call loads its own constants (one scalar-cache read per call): short SGPR live ranges instead of 54 SGPRs
// held across the caller (r05, pt_gs_k: v_readlane 270 -> 224 in the kernel's code, 78.85 -> 78.45 ms per chunk)
template <>
struct kmath<true> {
    __device__ kmath() {}
    __device__ double exp(double x) const { return exp_fast(x, gsb_load()); }
    __device__ double log(double x) const { return log_fast(x, gsb_load()); }
    __device__ dexp_pair exp2(double x, double y) const {
        const gsb_k k = gsb_load();
        dexp_pair r;
        r.a = exp_fast(x, k);
        r.b = exp_fast(y, k);
        return r;
    }
};

// returns potential evapotranspiration in mm/s (priestley_taylor.h:75-102)
template <bool INL = false>
__device__ inline double pt_pot_evap(double albedo, double alpha, double temperature, double global_radiation,
                                     double rhumidity) {
    const bool neg = temperature < 0;
    const double ck2 = neg ? 17.84362 : 17.08085;
    const double ck3 = neg ? 245.425 : 234.175;
    const double ctt_inv = 1 / (ck3 + temperature);
    const kmath<INL> km;
    const double sat_pressure = 0.610780 * km.exp(ck2 * temperature * ctt_inv);
    const double delta = sat_pressure * ck2 * ck3 * ctt_inv * ctt_inv;
    const double vapour_pressure = sat_pressure * rhumidity;
    const double k_temp = temperature + 273.15;
    const double e_atm = 1.24 * km.exp(0.143 * km.log(10 * vapour_pressure / k_temp)) * (0.85 + 0.5 * rhumidity);
    const double net_rad = 0.0000000567 * dpow4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - albedo);
    const double epot = alpha * delta * net_rad / (delta + 0.066);
    if (epot < 0.0) return 0.0;
    return epot / (2500780 - 2361 * temperature);
}

// the same, plus exp(ae_arg) for the caller's actual_evapotranspiration (inline beside the saturation
// pressure's exp (two independent exps side by side instead of back to back); the same bits as the two calls
template <bool INL = false>
__device__ inline double pt_pot_evap_exp(double albedo, double alpha, double temperature, double global_radiation,
                                         double rhumidity, double ae_arg, double& ae_exp) {
    const bool neg = temperature < 0;
    const double ck2 = neg ? 17.84362 : 17.08085;
    const double ck3 = neg ? 245.425 : 234.175;
    const double ctt_inv = 1 / (ck3 + temperature);
    const kmath<INL> km;
    const dexp_pair e2 = km.exp2(ck2 * temperature * ctt_inv, ae_arg);
    ae_exp = e2.b;
    const double sat_pressure = 0.610780 * e2.a;
    const double delta = sat_pressure * ck2 * ck3 * ctt_inv * ctt_inv;
    const double vapour_pressure = sat_pressure * rhumidity;
    const double k_temp = temperature + 273.15;
    const double e_atm = 1.24 * km.exp(0.143 * km.log(10 * vapour_pressure / k_temp)) * (0.85 + 0.5 * rhumidity);
    const double net_rad = 0.0000000567 * dpow4(k_temp) * (e_atm - 0.98) + global_radiation * (1.0 - albedo);
    const double epot = alpha * delta * net_rad / (delta + 0.066);
    if (epot < 0.0) return 0.0;
    return epot / (2500780 - 2361 * temperature);
}

}  // namespace shyft_dev
