// Device special functions for the method stacks (gfx950, fp64).
//
// Elementary functions come from detmath (detmath/detmath.h), the
// deterministic fp64 library the CPU oracle uses too, so kernel and oracle
// produce bit-identical results. min/max follow std::min/std::max semantics
// ((b < a) ? b : a and (a < b) ? b : a), which differ from fmin/fmax on
// signed zeros and NaN.
//
// gamma_p: regularized lower incomplete gamma P(a,x), evaluated to full double
// precision (series for x < a+1, modified-Lentz continued fraction otherwise).
// The reference calls boost::math::gamma_p with a digits10<5>/<10> policy
// (core/gamma_snow.h:189-201); this is at least as precise. The prefix
// exp(a*log(x) - x - lgamma(a)) is returned as well, because calc_snow_state
// (core/gamma_snow.h:244-245) needs exactly that term a second time.
#pragma once
#include <hip/hip_runtime.h>

#include "../../../detmath/detmath.h"
#include "fastmath.h"

namespace shyft_dev {

__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }
// the elementary functions are out-of-line device functions (one copy each: I-cache and register pressure of the
// step loops), the physics around them is inlined
#ifndef SHYFT_TABLE_CALLS
#define SHYFT_TABLE_CALLS 0
#endif
#if SHYFT_TABLE_CALLS
// (per kernel file) the fast paths with SGPR-table constants (device/fastmath.h): fewer VALU instructions per call
// (no v_mov_b32 pair per constant), more SGPRs clobbered across it; detmath's general functions beyond them
__device__ __noinline__ double dexp(double x) {
    if (__builtin_fabs(x) <= 708.0) return gsb_exp(x, gsb_load());
    return detmath::exp(x);
}
__device__ __noinline__ double dlog(double x) {
    if (x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308) return gsb_log(x, gsb_load());
    return detmath::log(x);
}
#else
__device__ __noinline__ double dexp(double x) { return detmath::exp(x); }
__device__ __noinline__ double dlog(double x) { return detmath::log(x); }
#endif
// two exps in one out-of-line call: the two Horner chains interleave (each one's fma latency hidden behind the
// other's), where two calls would run them back to back; the same bits as two dexp calls
struct dexp_pair {
    double a, b;
};
__device__ __noinline__ dexp_pair dexp2(double x, double y) {
    dexp_pair r;
#if SHYFT_TABLE_CALLS
    if (__builtin_fabs(x) <= 708.0 && __builtin_fabs(y) <= 708.0) {
        const gsb_k k = gsb_load();
        r.a = gsb_exp(x, k);
        r.b = gsb_exp(y, k);
        return r;
    }
#endif
    if (__builtin_fabs(x) <= 708.0 && __builtin_fabs(y) <= 708.0) {
#pragma clang fp contract(off)
        // detmath::exp_poly on both arguments, step by step side by side
        const double tx = __builtin_fma(x, 1.4426950408889634, 6755399441055744.0),
                     ty = __builtin_fma(y, 1.4426950408889634, 6755399441055744.0);
        const double kx = tx - 6755399441055744.0, ky = ty - 6755399441055744.0;
        double rx = __builtin_fma(-kx, 6.93147180369123816490e-01, x), ry = __builtin_fma(-ky, 6.93147180369123816490e-01, y);
        rx = __builtin_fma(-kx, 1.90821492927058770002e-10, rx);
        ry = __builtin_fma(-ky, 1.90821492927058770002e-10, ry);
        double px = detmath::EXP_Q[0], py = detmath::EXP_Q[0];
#pragma unroll
        for (int i = 1; i < 11; ++i) {
            px = __builtin_fma(px, rx, detmath::EXP_Q[i]);
            py = __builtin_fma(py, ry, detmath::EXP_Q[i]);
        }
        px = __builtin_fma(rx, px, 1.0);
        py = __builtin_fma(ry, py, 1.0);
        r.a = __builtin_ldexp(px, (int)kx);
        r.b = __builtin_ldexp(py, (int)ky);
    } else {
        r.a = detmath::exp(x);
        r.b = detmath::exp(y);
    }
    return r;
}
__device__ __noinline__ double dpow(double x, double y) { return detmath::pow(x, y); }
__device__ __noinline__ double dlgamma(double x) { return detmath::lgamma(x); }
// structured powers (detmath::pow4 / pow8 / powr, the oracle's OPOW4 / OPOW8 / OPOWR)
__device__ __forceinline__ double dpow4(double x) { return detmath::pow4(x); }
__device__ __forceinline__ double dpow8(double x) { return detmath::pow8(x); }
__device__ inline double dpowr(double x, double y) { return dexp(y * dlog(x)); }

// boost::math::gamma_p stand-in: detmath::gamma_pq (P(a,x), P(a+1,x) and the
// prefix x^a e^-x / Gamma(a) from ONE series / continued-fraction evaluation),
// with the out-of-line elementary functions above.
struct dev_math {
    __device__ static double exp(double x) { return dexp(x); }
    __device__ static double log(double x) { return dlog(x); }
};
using gamma_p_result = detmath::gamma_pq_result;
// lga = lgamma(a) supplied by the caller (shape changes rarely, so callers cache it);
// eps = the relative termination tolerance (boost precision policy of the caller)
__device__ inline gamma_p_result gamma_p_prefix(double a, double x, double lga, double eps) {
#ifdef SHYFT_ABLATE_GAMMA
    gamma_p_result r; r.p = 0.5; r.p1 = 0.4; r.prefix = 0.01; return r;  // timing ablation only (wrong results)
#endif
    return detmath::gamma_pq<dev_math>(a, x, lga, eps);
}


// gamma_snow's calls: boost precision policy by shape (gamma_snow.h:195-197)
__device__ inline gamma_p_result gs_gamma_pq(double a, double x, double lga) {
    return gamma_p_prefix(a, x, lga, detmath::gamma_snow_policy_eps(a));
}

// full double precision (boost default policy)
__device__ inline double gamma_p(double a, double x) { return gamma_p_prefix(a, x, dlgamma(a), 2.220446049250313e-16).p; }

}  // namespace shyft_dev
