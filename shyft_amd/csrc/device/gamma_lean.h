// The incomplete gamma of gamma_snow (boost gamma_p with the digits10<5>/<10> policy, gamma_snow.h:189-201, as
// detmath::gamma_pq restates it) in fewer instructions, for the fast domain -- shape a > 0, x positive normal,
// |a log x - x - lgamma(a)| <= 708 -- where it is bit-identical to detmath::gamma_pq<dev_math>:
//  - exp and log are inline (detmath's |x| <= 708 / positive-normal fast paths), their polynomial constants read
//    once from a constant table into SGPRs and used as SGPR operands of v_fma_f64 (gs_fma_s), no call;
//  - the series and the continued fraction run without their 2^-200 rescale test: with a > 0 the series'
//    E = (a+1)...(a+n) only grows, so a final E <= 2^200/... proves no term rescaled; the fraction's largest |P| is
//    kept with a max (no per-term branch) and checked after the loop. An evaluation that would have rescaled, or
//    that leaves the fast domain, is redone by the general detmath evaluation.
// Used by the Brent job of device/gs_brent.h (its f), by calc_snow_state (device/ptgsk_dev.h) and by Skaugen's
// sca_rel_red (device/ptssk_dev.h); exp_fast / log_fast are the kernels' inline exp / log (device/pt_dev.h kmath).
#pragma once
#include <hip/hip_runtime.h>

#include "special.h"

namespace shyft_dev {

// dexp / dlog bit for bit: the fast paths of device/fastmath.h inline, the out-of-line general function beyond them
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

// P(a, x), P(a+1, x) and the prefix by detmath::gamma_pq's series / continued fraction for the fast domain;
// ok = false: the caller takes the general evaluation (the value returned is then meaningless)
__device__ __forceinline__ gamma_p_result gsb_gamma_pq(double a, double x, double lga, double eps, double ap1,
                                                       const gsb_k& k, bool& ok) {
    const double lx = gsb_log(x, k);
    const double arg = a * lx - x - lga;
    ok = a > 0.0 && x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308 && __builtin_fabs(arg) <= 708.0;
    const double prefix = gsb_exp(arg, k);
    gamma_p_result r;
    r.prefix = prefix;
    r.p = r.p1 = 0.0;
    if (!ok) return r;  // (x = inf or NaN would not converge: no loop for a lane outside the domain)
    if (x < ap1) {
        // series (detmath::gamma_series_sums without the rescale test)
        double ap = a, E = 1.0, B = 0.0, xn = 1.0;
        for (int n = 1; n <= 2000; ++n) {
            ap = ap + 1.0;
            xn = xn * x;
            E = E * ap;
            B = __builtin_fma(B, ap, xn);
            if (xn < eps * (B + E)) break;
        }
        ok = ok && E <= detmath::GPQ_SCALE_HI;
        const double aE = a * E;
        const double pp = prefix * ((B + E) / aE);
        const double pp1 = prefix * (B / aE);
        r.p = pp < 1.0 ? pp : 1.0;
        r.p1 = pp1 < 1.0 ? pp1 : 1.0;
    } else {
        // continued fraction (detmath::gamma_cf_terms; the rescale test folded into the largest |P|)
        double bcf = x + 1.0 - a;
        double Pm = 1.0, Qm = 0.0, P = bcf, Qd = 1.0, di = 0.0, bigP = 0.0;
        for (int i = 1; i <= 2000; ++i) {
            di = di + 1.0;
            const double an = -di * (di - a);
            bcf = bcf + 2.0;
            const double Pn = __builtin_fma(bcf, P, an * Pm);
            const double Qn = __builtin_fma(bcf, Qd, an * Qm);
            const double cross = Pn * Qd;
            const double diff = cross - P * Qn;
            Pm = P; Qm = Qd;
            P = Pn; Qd = Qn;
            if (__builtin_fabs(diff) <= eps * __builtin_fabs(cross)) break;
            bigP = __builtin_fmax(bigP, __builtin_fabs(P));  // NaN P: no rescale there either
        }
        ok = ok && !(bigP > detmath::GPQ_SCALE_HI);
        const double q = prefix * (Qd / P);
        const double q1 = q + prefix / a;
        const double pp = 1.0 - q;
        const double pp1 = 1.0 - q1;
        r.p = pp > 0.0 ? pp : 0.0;
        r.p1 = pp1 > 0.0 ? pp1 : 0.0;
    }
    return r;
}

// the general evaluation (detmath::gamma_pq with the out-of-line exp / log), out of line
__device__ __noinline__ gamma_p_result gs_gamma_pq_general(double a, double x, double lga) {
    return gamma_p_prefix(a, x, lga, detmath::gamma_snow_policy_eps(a));
}

}  // namespace shyft_dev
