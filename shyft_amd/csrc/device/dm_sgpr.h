// detmath::exp / detmath::log fast paths with the polynomial coefficients as SGPR operands (gfx950).
//
// For p = fma(p, r, C) the compiler picks v_fmac_f64 (accumulator = destination), so every coefficient C is first
// copied into the destination VGPR pair by two v_mov_b32: 26 of dexp's ~45 VALU instructions are those copies.
// gfx9's VOP3 v_fma_f64 reads one SGPR pair as an operand, so with C in SGPRs (s_mov_b32 pairs: scalar-unit
// issue, not VALU) each Horner step is one VALU instruction. The operations and their order are detmath's, so the
// results are the same bits (tests/test_ptgsk_parity.py checks detmath's device functions against the host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../detmath/detmath.h"

namespace shyft_dev {

// a * b + c, c an SGPR pair
__device__ __forceinline__ double dms_fma(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}

__device__ __forceinline__ double dm_exp_s(double x) {
#pragma clang fp contract(off)
    if (__builtin_fabs(x) <= 708.0) {
        const double t = x * 1.4426950408889634 + 6755399441055744.0;
        const double kf = t - 6755399441055744.0;
        double r = __builtin_fma(-kf, 6.93147180369123816490e-01, x);
        r = __builtin_fma(-kf, 1.90821492927058770002e-10, r);
        double p = dms_fma(r, 1.6059043836821614e-10, 2.0876756987868099e-09);
        p = dms_fma(p, r, 2.5052108385441720e-08);
        p = dms_fma(p, r, 2.7557319223985893e-07);
        p = dms_fma(p, r, 2.7557319223985888e-06);
        p = dms_fma(p, r, 2.4801587301587302e-05);
        p = dms_fma(p, r, 1.9841269841269841e-04);
        p = dms_fma(p, r, 1.3888888888888889e-03);
        p = dms_fma(p, r, 8.3333333333333333e-03);
        p = dms_fma(p, r, 4.1666666666666664e-02);
        p = dms_fma(p, r, 1.6666666666666666e-01);
        p = __builtin_fma(p, r, 0.5);
        p = __builtin_fma(p, r, 1.0);
        p = __builtin_fma(p, r, 1.0);
        return __builtin_ldexp(p, (int)kf);
    }
    return detmath::exp_general(x);
}

__device__ __forceinline__ double dm_log_s(double x) {
#pragma clang fp contract(off)
    if (!(x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308)) return detmath::log_general(x);
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    double m = __longlong_as_double((long long)((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const double f = m - 1.0;
    const double d = 2.0 + f;
    const double d_lo = (2.0 - d) + f;
    const double s = f / d;
    const double s_lo = (__builtin_fma(-s, d, f) - s * d_lo) / d;
    const double z = s * s;
    double t = dms_fma(z, 2.0 / 25, 2.0 / 23);
    t = dms_fma(t, z, 2.0 / 21);
    t = dms_fma(t, z, 2.0 / 19);
    t = dms_fma(t, z, 2.0 / 17);
    t = dms_fma(t, z, 2.0 / 15);
    t = dms_fma(t, z, 2.0 / 13);
    t = dms_fma(t, z, 2.0 / 11);
    t = dms_fma(t, z, 2.0 / 9);
    t = dms_fma(t, z, 2.0 / 7);
    t = dms_fma(t, z, 2.0 / 5);
    t = dms_fma(t, z, 2.0 / 3);
    const double tail = (s * z) * t;
    const double ed = (double)e;
    const double a_hi = ed * 6.93147180369123816490e-01;
    const double a_lo = ed * 1.90821492927058770002e-10;
    const double b = 2.0 * s;
    const double sum = a_hi + b;
    const double bb = sum - a_hi;
    const double err = (a_hi - (sum - bb)) + (b - bb);
    const double small = ((err + 2.0 * s_lo) + tail) + a_lo;
    return sum + small;
}

}  // namespace shyft_dev
