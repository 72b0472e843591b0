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

namespace shyft_dev {

__device__ __forceinline__ double smin(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double smax(double a, double b) { return (a < b) ? b : a; }
__device__ __forceinline__ double dexp(double x) { return detmath::exp(x); }
__device__ __forceinline__ double dlog(double x) { return detmath::log(x); }
__device__ __forceinline__ double dpow(double x, double y) { return detmath::pow(x, y); }
__device__ __forceinline__ double dlgamma(double x) { return detmath::lgamma(x); }

struct gamma_p_result {
    double p;       // P(a, x)
    double prefix;  // exp(a*log(x) - x - lgamma(a)); 0 when x <= 0
};

// lga = lgamma(a) supplied by the caller (shape changes rarely, so callers cache it)
__device__ inline gamma_p_result gamma_p_prefix(double a, double x, double lga) {
    gamma_p_result r;
    if (x <= 0.0) { r.p = 0.0; r.prefix = 0.0; return r; }
    if (__builtin_isinf(x)) { r.p = 1.0; r.prefix = 0.0; return r; }
    const double eps = 2.220446049250313e-16;
    const double prefix = dexp(a * dlog(x) - x - lga);
    r.prefix = prefix;
    if (x < a + 1.0) {
        double ap = a, del = 1.0 / a, sum = del;
        for (int n = 0; n < 1000; ++n) {
            ap += 1.0;
            del *= x / ap;
            sum += del;
            if (fabs(del) < fabs(sum) * eps) break;
        }
        r.p = smin(1.0, sum * prefix);
        return r;
    }
    const double fpmin = 1e-300;
    double b = x + 1.0 - a, c = 1.0 / fpmin, d = 1.0 / b, h = d;
    for (int i = 1; i < 1000; ++i) {
        const double an = -i * (i - a);
        b += 2.0;
        d = an * d + b;
        if (fabs(d) < fpmin) d = fpmin;
        c = b + an / c;
        if (fabs(c) < fpmin) c = fpmin;
        d = 1.0 / d;
        const double del = d * c;
        h *= del;
        if (fabs(del - 1.0) < eps) break;
    }
    r.p = smax(0.0, 1.0 - prefix * h);
    return r;
}

__device__ inline double gamma_p(double a, double x) {
    if (__builtin_isnan(a) || __builtin_isnan(x)) return __builtin_nan("");
    return gamma_p_prefix(a, x, dlgamma(a)).p;
}

}  // namespace shyft_dev
