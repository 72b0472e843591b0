// gamma_snow's corr_lwc Brent job (gamma_snow.h:214-227), written for the one solver wavefront that runs it.
//
// In the pt_gs_k kernels a workgroup's Brent jobs are solved by one wavefront while the workgroup's other
// wavefronts wait at a barrier (kernels/ptgsk.hip), so the job is a latency problem: a lone wavefront issues about
// one instruction per 4-7 cycles whatever the instruction, so the solve costs its instruction count. This is the
// same arithmetic as gs_corr_lwc (device/ptgsk_dev.h) -- the same Brent iterations (boost brent_find_minima), the
// same f = (calc_q(a2, b2, z) - Q1)^2, the same incomplete-gamma terms and detmath exp / log fast paths -- with
// fewer instructions around it:
//  - no calls: exp, log, the series and the continued fraction are inline in the one loop;
//  - the polynomial constants of exp and log are read once per job from a constant table into SGPRs and used as
//    SGPR operands of v_fma_f64 (gs_fma_s), instead of two v_mov_b32 per constant per evaluation;
//  - the series and continued fraction run without their 2^-200 rescale test (device/gamma_lean.h): a lane whose
//    evaluation would have rescaled, or that leaves the fast domain (x <= 0, x not normal, a <= 0, |exp argument|
//    > 708), is re-evaluated by the general gs_calc_q.
// Bit-identical to gs_corr_lwc (tests: test_ptgsk_parity.py, tools/mb/mb_brent.cpp's device check).
#pragma once
#include <hip/hip_runtime.h>

#include "ptgsk_dev.h"
#include "gamma_lean.h"

namespace shyft_dev {

// calc_q(a, b, z) = a b P(a+1, z/b) + z (1 - P(a, z/b)) for the fast domain (device/gamma_lean.h); ok = false:
// take gs_calc_q
__device__ __forceinline__ double gsb_calc_q(double a, double b, double z, double lga, double eps, double ap1,
                                             const gsb_k& k, bool& ok) {
    const gamma_p_result g = gsb_gamma_pq(a, z / b, lga, eps, ap1, k, ok);
    return a * b * g.p1 + z * (1.0 - g.p);
}

// the general evaluation, out of line (rare: Q1 without the opening state's gamma pair, or a lane outside the
// fast domain)
__device__ __noinline__ double gs_calc_q_general(double a, double b, double z, double lga) {
    return gs_calc_q(a, b, z, lga);
}

// f = (calc_q(a2, b2, z) - Q1)^2 of the job, fast path with the general fallback
struct gsb_f {
    double a2, b2, lga2, Q1, eps, ap1;
    bool a_ok;
    gsb_k k;
    __device__ __forceinline__ gsb_f(double z1, double a1, double b1, double a2_, double b2_, double q1, double lga2_)
        : a2(a2_), b2(b2_), lga2(lga2_) {
        Q1 = q1 == q1 ? q1 : gs_calc_q_general(a1, b1, z1, dlgamma(a1));
        k = gsb_load();
        eps = detmath::gamma_snow_policy_eps(a2);
        ap1 = a2 + 1.0;
        a_ok = a2 > 0.0;
    }
    __device__ __forceinline__ double operator()(double z) const {
        bool ok;
        double cq = gsb_calc_q(a2, b2, z, lga2, eps, ap1, k, ok);
        if (!(ok && a_ok)) cq = gs_calc_q_general(a2, b2, z, lga2);  // the general path (rare)
        const double v = cq - Q1;
        return v * v;
    }
};

// Speculative opening of the Brent search (small regions, where the solve is a latency problem). The first three
// points boost's brent_find_minima evaluates do not depend on f's values: x = w = v = z1 opens; iteration 1 takes
// the golden step u1 (delta2 starts at 0); iteration 2's parabola through (z1, u1) is degenerate whichever of
// f(u1) <= f(z1) holds (r == q, so p = q = 0 and the golden step is taken again), so its point is u2a (x = u1,
// max = z1) or u2b (x = z1, min = u1). gs_brent_point gives point k of {z1, u1, u2a, u2b} by the solver's own
// formulas; four lanes evaluate f at the four points at once and the solver then looks each of its f arguments up
// among them (bitwise) before evaluating. f is a pure function of its argument, so a hit returns the same bits;
// where an assumption fails (non-finite f values, an early exit) the argument simply misses and is evaluated.
__device__ __forceinline__ double gs_brent_point(double z1, int k) {
    const double tolerance = 0x1p-11;
    const double golden = (double)0.3819660f;
    auto golden_step = [&](double x, double lo, double hi) {
        const double mid = (lo + hi) / 2;
        const double fract1 = tolerance * fabs(x) + tolerance / 4;
        const double d2 = (x >= mid) ? lo - x : hi - x;
        const double delta = golden * d2;
        return (fabs(delta) >= fract1) ? (x + delta) : (delta > 0 ? x + fabs(fract1) : x - fabs(fract1));
    };
    if (k == 0) return z1;
    const double u1 = golden_step(z1, 0.0, z1);
    if (k == 1) return u1;
    double lo = 0.0, hi = z1, x = z1;
    if (k == 2) {  // f(u1) <= f(z1): x = u1, the old x bounds the side u1 moved from
        if (u1 >= x) lo = x; else hi = x;
        x = u1;
    } else {  // f(u1) > f(z1): u1 bounds its side
        if (u1 < x) lo = u1; else hi = u1;
    }
    return golden_step(x, lo, hi);
}

struct gsb_zf {
    double z, f;
};
__device__ __noinline__ gsb_zf gs_corr_lwc_spec(double z1, double a1, double b1, double a2, double b2, double q1,
                                                double lga2, int k) {
    const gsb_f f(z1, a1, b1, a2, b2, q1, lga2);
    gsb_zf r;
    r.z = gs_brent_point(z1, k);
    r.f = f(r.z);
    return r;
}

struct gsb_memo {
    double z[4], f[4];
};

template <bool MEMO>
__device__ __forceinline__ double gs_corr_lwc_lean_t(double z1, double a1, double b1, double a2, double b2, double q1,
                                                     double lga2, const gsb_memo* memo) {
#ifdef SHYFT_ABLATE_BRENT
    return z1 * 0.5;  // instruction-budget ablation only (wrong results)
#endif
    const gsb_f fe(z1, a1, b1, a2, b2, q1, lga2);
    gsb_memo mm;
    if (MEMO) mm = *memo;
    auto f = [&](double z) {
        if (MEMO) {
            const long long zb = __double_as_longlong(z);
            bool hit = false;
            double r = 0.0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (!hit && zb == __double_as_longlong(mm.z[i])) { hit = true; r = mm.f[i]; }
            if (hit) return r;
        }
        return fe(z);
    };
    double min = 0.0, max = z1;
    const double tolerance = 0x1p-11;  // ldexp(1, 1-12)
    const double golden = (double)0.3819660f;
    double x, w, v, u, delta, delta2, fu, fv, fw, fx, mid, fract1, fract2;
    x = w = v = max;
    fw = fv = fx = f(x);
    delta2 = delta = 0;
    int count = 60;
    do {
        mid = (min + max) / 2;
        fract1 = tolerance * fabs(x) + tolerance / 4;
        fract2 = 2 * fract1;
        if (fabs(x - mid) <= (fract2 - (max - min) / 2)) break;
        if (fabs(delta2) > fract1) {
            double r = (x - w) * (fx - fv);
            double q = (x - v) * (fx - fw);
            double p = (x - v) * q - (x - w) * r;
            q = 2 * (q - r);
            if (q > 0) p = -p;
            q = fabs(q);
            double td = delta2;
            delta2 = delta;
            if ((fabs(p) >= fabs(q * td / 2)) || (p <= q * (min - x)) || (p >= q * (max - x))) {
                delta2 = (x >= mid) ? min - x : max - x;
                delta = golden * delta2;
            } else {
                delta = p / q;
                u = x + delta;
                if (((u - min) < fract2) || ((max - u) < fract2)) delta = (mid - x) < 0 ? -fabs(fract1) : fabs(fract1);
            }
        } else {
            delta2 = (x >= mid) ? min - x : max - x;
            delta = golden * delta2;
        }
        u = (fabs(delta) >= fract1) ? (x + delta) : (delta > 0 ? x + fabs(fract1) : x - fabs(fract1));
        fu = f(u);
        if (fu <= fx) {
            if (u >= x) min = x; else max = x;
            v = w; w = x; x = u;
            fv = fw; fw = fx; fx = fu;
        } else {
            if (u < x) min = u; else max = u;
            if ((fu <= fw) || (w == x)) {
                v = w; w = u; fv = fw; fw = fu;
            } else if ((fu <= fv) || (v == x) || (v == w)) {
                v = u; fv = fu;
            }
        }
    } while (--count);
    return x;
}

__device__ __noinline__ double gs_corr_lwc_lean(double z1, double a1, double b1, double a2, double b2, double q1,
                                                double lga2) {
    return gs_corr_lwc_lean_t<false>(z1, a1, b1, a2, b2, q1, lga2, nullptr);
}

__device__ __noinline__ double gs_corr_lwc_memo(double z1, double a1, double b1, double a2, double b2, double q1,
                                                double lga2, const gsb_memo& memo) {
    return gs_corr_lwc_lean_t<true>(z1, a1, b1, a2, b2, q1, lga2, &memo);
}

}  // namespace shyft_dev
