// detmath exp / log fast paths with their polynomial constants in SGPRs (gfx950).
//
// detmath::exp and detmath::log (detmath/detmath.h) evaluate fixed polynomials; the compiler materialises every
// fp64 coefficient with two v_mov_b32 per use, more VALU issue than the polynomial's own v_fma_f64s. Here the
// coefficients come from a constant table by scalar loads (s_load, once per region that uses them: a loop hoists
// them) and enter v_fma_f64 as SGPR operands (fm_fma_s). The arithmetic is detmath's, operation for operation, so
// the results are the same bits (checked on the device against detmath: tests/test_ptgsk_parity.py, and
// tools/mb/mb_exp.cpp). Outside the fast domains the general detmath code runs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../detmath/detmath.h"

namespace shyft_dev {

// exp: INV_LN2 SHIFT LN2_HI LN2_LO, 1/13! .. 1/3! (detmath::exp_poly); log: 2/25 .. 2/3 (detmath::log_dd)
static __constant__ double fm_const[32] = {
    1.4426950408889634, 6755399441055744.0, 6.93147180369123816490e-01, 1.90821492927058770002e-10,
    1.6059043836821614e-10, 2.0876756987868099e-09, 2.5052108385441720e-08, 2.7557319223985893e-07,
    2.7557319223985888e-06, 2.4801587301587302e-05, 1.9841269841269841e-04, 1.3888888888888889e-03,
    8.3333333333333333e-03, 4.1666666666666664e-02, 1.6666666666666666e-01,
    2.0 / 25, 2.0 / 23, 2.0 / 21, 2.0 / 19, 2.0 / 17, 2.0 / 15, 2.0 / 13, 2.0 / 11, 2.0 / 9, 2.0 / 7, 2.0 / 5,
    2.0 / 3, 0.0, 0.0, 0.0, 0.0, 0.0};

typedef __attribute__((address_space(4))) const double fm_cdouble;

// a * b + c with c an SGPR pair (wave-uniform constant): one v_fma_f64, no v_mov of the constant
__device__ __forceinline__ double fm_fma_s(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}

__device__ __forceinline__ const fm_cdouble* fm_table() {
    const fm_cdouble* p = (const fm_cdouble*)fm_const;
    asm volatile("" : "+s"(p));  // opaque: scalar loads into SGPRs, not folded literals
    return p;
}

struct fm_exp_k {
    double c[15];
};
struct fm_log_k {
    double c[12];
};

__device__ __forceinline__ fm_exp_k fm_exp_load() {
    const fm_cdouble* __restrict__ p = fm_table();
    fm_exp_k k;
#pragma unroll
    for (int i = 0; i < 15; ++i) k.c[i] = p[i];
    return k;
}
__device__ __forceinline__ fm_log_k fm_log_load() {
    const fm_cdouble* __restrict__ p = fm_table();
    fm_log_k k;
#pragma unroll
    for (int i = 0; i < 12; ++i) k.c[i] = p[15 + i];
    return k;
}

// detmath::exp
__device__ __forceinline__ double fm_exp(double x, const fm_exp_k& k) {
#pragma clang fp contract(off)
    if (__builtin_fabs(x) <= 708.0) {
        const double t = x * k.c[0] + k.c[1];
        const double kf = t - k.c[1];
        double r = __builtin_fma(-kf, k.c[2], x);
        r = __builtin_fma(-kf, k.c[3], r);
        double p = fm_fma_s(r, k.c[4], k.c[5]);
#pragma unroll
        for (int i = 6; i <= 14; ++i) p = fm_fma_s(p, r, k.c[i]);
        p = __builtin_fma(p, r, 0.5);
        p = __builtin_fma(p, r, 1.0);
        p = __builtin_fma(p, r, 1.0);
        return __builtin_ldexp(p, (int)kf);
    }
    return detmath::exp_general(x);
}

// detmath::log (ek: LN2_HI / LN2_LO from the exp table)
__device__ __forceinline__ double fm_log(double x, const fm_log_k& k, const fm_exp_k& ek) {
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
    double t = fm_fma_s(k.c[0], z, k.c[1]);
#pragma unroll
    for (int i = 2; i <= 11; ++i) t = fm_fma_s(t, z, k.c[i]);
    const double tail = (s * z) * t;
    const double ed = (double)e;
    const double a_hi = ed * ek.c[2];
    const double a_lo = ed * ek.c[3];
    const double b = 2.0 * s;
    const double sum = a_hi + b;
    const double bb = sum - a_hi;
    const double err = (a_hi - (sum - bb)) + (b - bb);
    const double small = ((err + 2.0 * s_lo) + tail) + a_lo;
    return sum + small;
}

}  // namespace shyft_dev
