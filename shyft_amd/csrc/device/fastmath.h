// The |x| <= 708 exp and the positive-normal log of detmath (detmath/detmath.h: exp_poly + one ldexp; log_dd's hi
// part without its subnormal branch) with their polynomial constants read from a constant table into SGPRs and
// used as SGPR operands of v_fma_f64 (gs_fma_s): no v_mov_b32 pair per 64-bit constant per evaluation. The same
// bits as detmath::exp / detmath::log on those domains (tests: every kernel's parity suite; tools/mb/mb_brent).
// Included by device/special.h; the inline users are device/gamma_lean.h and the kernels' kmath<true>.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../detmath/detmath.h"

namespace shyft_dev {

// exp: INV_LN2 SHIFT LN2_HI LN2_LO and detmath::exp_poly's q coefficients; log: LN2_HI LN2_LO and
// detmath::log_core's Lg1 .. Lg7
static __constant__ double gsb_const[32] = {
    1.4426950408889634, 6755399441055744.0, 6.93147180369123816490e-01, 1.90821492927058770002e-10,
    detmath::EXP_Q[0], detmath::EXP_Q[1], detmath::EXP_Q[2], detmath::EXP_Q[3], detmath::EXP_Q[4], detmath::EXP_Q[5],
    detmath::EXP_Q[6], detmath::EXP_Q[7], detmath::EXP_Q[8], detmath::EXP_Q[9], detmath::EXP_Q[10],
    detmath::LOG_LG1, detmath::LOG_LG2, detmath::LOG_LG3, detmath::LOG_LG4, detmath::LOG_LG5, detmath::LOG_LG6,
    detmath::LOG_LG7, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};

typedef __attribute__((address_space(4))) const double gsb_cdouble;

// a * b + c with c an SGPR pair (wave-uniform constant): one v_fma_f64, no v_mov of the constant
__device__ __forceinline__ double gs_fma_s(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}

struct gsb_k {
    double c[22];
};

__device__ __forceinline__ gsb_k gsb_load() {
    gsb_k k;
    const gsb_cdouble* __restrict__ p = (const gsb_cdouble*)gsb_const;
    asm volatile("" : "+s"(p));  // keep the table opaque: scalar loads into SGPRs, not folded literals
#pragma unroll
    for (int i = 0; i < 22; ++i) k.c[i] = p[i];
    return k;
}

// detmath::exp for |x| <= 708 (exp_poly + one ldexp)
__device__ __forceinline__ double gsb_exp(double x, const gsb_k& k) {
    const double t = gs_fma_s(x, k.c[0], k.c[1]);
    const double kf = t - k.c[1];
    double r = __builtin_fma(-kf, k.c[2], x);
    r = __builtin_fma(-kf, k.c[3], r);
    double q = gs_fma_s(r, k.c[4], k.c[5]);
#pragma unroll
    for (int i = 6; i <= 14; ++i) q = gs_fma_s(q, r, k.c[i]);
    return __builtin_ldexp(__builtin_fma(r, q, 1.0), (int)kf);
}

// detmath::log for positive normal finite x (detmath::log_core with k_adj = 0, step by step)
__device__ __forceinline__ double gsb_log(double x, const gsb_k& k) {
    uint64_t u = (uint64_t)__double_as_longlong(x);
    int e = (int)((u >> 52) & 0x7ff) - 1023;
    const uint32_t hx = (uint32_t)(u >> 32) & 0x000fffffu;
    const uint32_t i = (hx + 0x95f64u) & 0x100000u;
    u = (u & 0x000fffffffffffffull) | ((uint64_t)(i ^ 0x3ff00000u) << 32);
    e += (int)(i >> 20);
    const double f = __longlong_as_double((long long)u) - 1.0;
    const double s = f / (2.0 + f);
    const double dk = (double)e;
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * gs_fma_s(w, gs_fma_s(w, k.c[20], k.c[18]), k.c[16]);
    const double t2 = z * gs_fma_s(w, gs_fma_s(w, gs_fma_s(w, k.c[21], k.c[19]), k.c[17]), k.c[15]);
    const double R = t2 + t1;
    if (((int32_t)(hx - 0x6147au) | (int32_t)(0x6b851u - hx)) > 0) {
        const double hfsq = 0.5 * f * f;
        return dk * k.c[2] - ((hfsq - __builtin_fma(s, hfsq + R, dk * k.c[3])) - f);
    }
    return dk * k.c[2] - (__builtin_fma(s, f - R, -(dk * k.c[3])) - f);
}

}  // namespace shyft_dev
