// Skaugen snow (core/skaugen.h:43-380) for the pt_ss_k kernel (gfx950, fp64).
//
// Lane = cell; the whole snow state lives in registers. Unit counts are
// unsigned 64-bit like the reference's unsigned long (including its wrap-around
// on a negative lrint), lrint rounds half to even (v_rndne_f64).
//
// The expensive part is statistics::sca_rel_red (skaugen.h:57-82), evaluated
// only on a partial melt of a snowpack: a 2-bit Brent minimisation of
// pdf_m - pdf_a, a walk of the lower bracket, a 10-bit bisection and two gamma
// cdfs. The gamma distribution functions are boost's full-precision ones
// restated on detmath (pdf = prefix/z/theta, cdf = P(k, z)), the same
// expressions the CPU oracle evaluates (oracle/src/ptssk.hpp), so the kernel is
// bit-identical to it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "special.h"

namespace shyft_dev {

// time marks inside a job (profiling builds of kernels/ptssk.hip define them)
#ifndef SS_JOB_MARK
#define SS_JOB_T0() ((void)0)
#define SS_JOB_MARK(k) ((void)0)
#endif

struct ss_par {
    double alpha_0, d_range, unit_size, max_water_fraction, tx, cx, ts, cfr;
};

struct ss_state {
    double nu, alpha, sca, swe, free_water, residual;
    uint64_t num_units;
};

__device__ inline long ss_lrint(double x) { return (long)rint(x); }

// gamma_distribution(k, theta) pdf with boost's pole/zero handling at x = 0; err set on the pole
__device__ inline double ss_gamma_pdf(double k, double theta, double lgk, double x, int32_t& err) {
    if (x == 0) {
        if (k == 1) return 1 / theta;
        if (k < 1) {
            err = ERR_SKAUGEN_PDF;
            return 0.0;
        }
        return 0.0;
    }
    const double z = x / theta;
    const double prefix = dexp(k * dlog(z) - z - lgk);
    return prefix / z / theta;
}

// both pdfs of zero_func at one x: they share z = x / theta and its log, and their two exps go through one dexp2
// call -- the same bits as two ss_gamma_pdf calls (r05, 1M cells, 730-step chunks, year mean: 102.7 -> 90.9 ms;
// detmath exp / log inline with an SGPR constant table, or the lean incomplete gamma for the two final cdfs,
// measured slower: their SGPRs, clobbered in the kernel across the call, cost the step loop more than they save)
struct ss_pdf_pair {
    double m, a;
};
__device__ __forceinline__ ss_pdf_pair ss_gamma_pdf2(double nu_m, double nu_a, double theta, double lg_m, double lg_a,
                                                     double x, int32_t& err) {
    ss_pdf_pair r;
    if (x == 0) {
        r.m = ss_gamma_pdf(nu_m, theta, lg_m, x, err);
        r.a = ss_gamma_pdf(nu_a, theta, lg_a, x, err);
        return r;
    }
    const double z = x / theta;
    const double lz = dlog(z);
    const dexp_pair e = dexp2(nu_m * lz - z - lg_m, nu_a * lz - z - lg_a);
    r.m = e.a / z / theta;
    r.a = e.b / z / theta;
    return r;
}

__device__ inline double ss_c(uint64_t n, double d_range) { return dexp(-(double)n / d_range); }

// zero_func's value at x (ss_gamma_pdf2: pdf_m - pdf_a), or -1.0 / +1.0 where its sign is certain without the four
// divisions: pdf = exp(.) / z / theta with the same z > 0 and theta > 0 for both, and correctly rounded division is
// monotonic, so exp_m < exp_a by more than 2^-48 relative gives pdf_m < pdf_a, a negative, non-zero difference: the
// larger quotient is normal (exp_a, z and theta far from the ends of the range), each of its two roundings moves it by
// at most 2^-53 relative, and the smaller one -- normal, subnormal or zero -- stays below it. Two exps that underflowed
// to 0 give 0, as the divisions do (the bisection then stops at that midpoint, as the reference's does).
// The bisection looks only at the sign of its midpoint values and whether they are zero (its one product test
// uses the exact opening values), so its sequence of brackets is unchanged.
// r06: the exps themselves are skipped where their arguments A (pdf_m) and B (pdf_a) already decide the test below:
// detmath's exp is within 2^-51 relative of e^t on normal results, so B - A > 2^-40 gives exp(B) >= exp(A) (1 + 2^-41)
// > fl(exp(A) (1 + 2^-48)), and max(A, B) in [-660, 660] puts the larger exp in [2^-952.2, 2^952.2], inside [LO, HI]:
// the test below would return -1 (or +1 with A and B swapped). And detmath's exp is exactly 0 below
// -745.1332191019412 (exp_general), so two arguments below it are the underflow case. Of the bisection midpoints of
// the year's 1M recorded jobs, 87 % are decided by the arguments and 11 % underflow; every decision agrees with the
// full evaluation (tools/mb/ptssk_group_emu.cpp). (A single-precision log in front of this, deciding 93 % of the
// midpoints without the division and the double log, measured 1 % slower: a wavefront runs the full path whenever
// one of its lanes needs it, and the remaining 2.5 % -- pdfs near the bottom of the double range -- are spread over
// the jobs; profiles/r06/ptssk_flog_variant.txt.)
#ifndef SHYFT_PTSSK_EXP_SKIP
#define SHYFT_PTSSK_EXP_SKIP 1
#endif
__device__ __forceinline__ double ss_zero_sign(double nu_m, double nu_a, double theta, double lg_m, double lg_a,
                                               double x, int32_t& err) {
    if (x == 0) {
        const ss_pdf_pair f = ss_gamma_pdf2(nu_m, nu_a, theta, lg_m, lg_a, x, err);
        return f.m - f.a;
    }
    const double z = x / theta;
    const double lz = dlog(z);
    const double A = nu_m * lz - z - lg_m, B = nu_a * lz - z - lg_a;  // ss_gamma_pdf2's exp arguments, same order
    const bool in_range = z >= 0x1p-30 && z <= 0x1p30 && theta >= 0x1p-30 && theta <= 0x1p30;
    if (SHYFT_PTSSK_EXP_SKIP) {
        if (A < -745.1332191019412 && B < -745.1332191019412) return 0.0;  // both exps 0
        const double hi = A > B ? A : B;
        if (in_range && hi >= -660.0 && hi <= 660.0) {
            if (B - A > 0x1p-40) return -1.0;
            if (A - B > 0x1p-40) return 1.0;
        }
    }
    const dexp_pair e = dexp2(A, B);
    if (e.a == 0 && e.b == 0) return 0.0;  // both pdfs underflowed: 0 / z / theta - 0 / z / theta
    const double LO = 0x1p-960, HI = 0x1p960;  // the larger exp normal, far from both ends: so is its pdf
    if (in_range) {
        if (e.b >= LO && e.b <= HI && e.b > e.a * (1.0 + 0x1p-48)) return -1.0;
        if (e.a >= LO && e.a <= HI && e.a > e.b * (1.0 + 0x1p-48)) return 1.0;
    }
    return e.a / z / theta - e.b / z / theta;  // ss_gamma_pdf2's divisions, in its order
}

// x == 0 is the only point where either pdf of zero_func raises (the pole of a shape < 1, ss_gamma_pdf)
__device__ __forceinline__ bool ss_pdf_pole(double x, double nu_m, double nu_a) { return x == 0 && (nu_m < 1 || nu_a < 1); }

// value v of lane k of this lane's group of L consecutive lanes (L a power of two <= 64; the group's lanes run the
// same control flow, so every source lane is active)
__device__ __forceinline__ double grp_get(double v, int L, int k) {
    return __shfl(v, (int)(__lane_id() & ~(unsigned)(L - 1)) + k, 64);
}
__device__ __forceinline__ int grp_get_i(int v, int L, int k) {
    return __shfl(v, (int)(__lane_id() & ~(unsigned)(L - 1)) + k, 64);
}

// statistics::sca_rel_red (skaugen.h:57-82), evaluated by one lane (G = false) or by a group of L lanes (G = true,
// L = 2 or 4, the same on every lane of a wavefront; k = this lane's index in its group; all L lanes pass the same
// job and return the same value). The result is the sequential algorithm's, bit for bit: every zero_func value it
// uses is the one the sequential algorithm computes at the same point, by the same code.
//  - the 2-bit brent_find_minima stops at its first test for any finite positive bracket (|x - mid| = max/2 <=
//    fract2 - max/2 = max/2 + 1/4): its one evaluation, f(max), is the bisection's f(upper) -- the Brent keeps
//    fx = f(x) and returns x -- so the bisection does not evaluate it again;
//  - the bracket walk's last test evaluates both pdfs at the final `lower`, which is the bisection's f(lower);
//  - groups: lgamma(nu_m) / lgamma(nu_a), the two opening evaluations (f(max), and the walk's first test at the
//    mean of g_m) and the two final cdfs run on lanes 0 / 1 side by side;
//  - L = 4: the bisection evaluates the midpoints of the next 2 levels at once, one per lane (each point computed
//    from the bracket by the same midpoint additions the sequential loop performs on the way there), and the group
//    then replays the sequential loop over those levels -- its tests, its branch and its error on a pole at the
//    points the sequential loop would have evaluated; the other point is discarded, with anything it raised.
//    (tools/mb/ptssk_group_emu.cpp replays this on the 1M recorded jobs of a year against the oracle's bisect.)
// Groups of 8 lanes (3 levels per round: the same replay, checked by the same emulation) faulted the GPU with a
// memory-aperture violation in r06 (gpurun_out of the r06a variant run); the kernel caps L at 4.
template <bool G>
__device__ __forceinline__ double ss_sca_rel_red_body(uint64_t u, uint64_t n, double nu_a, double alpha, int L, int k,
                                                      int32_t& err) {
    SS_JOB_T0();
    const double nu_m = ((double)u / n) * nu_a;
    const double theta = 1.0 / alpha;
    double lg_m, lg_a;
    if (!G) {
        lg_m = dlgamma(nu_m);
        lg_a = dlgamma(nu_a);
    } else {
        const double lg = dlgamma(k == 1 ? nu_a : nu_m);
        lg_m = grp_get(lg, L, 0);
        lg_a = grp_get(lg, L, 1);
    }
    SS_JOB_MARK(0);
    const double g_a_mean = nu_a * theta;
    auto zero_func = [&](double x) {
        const ss_pdf_pair f = ss_gamma_pdf2(nu_m, nu_a, theta, lg_m, lg_a, x, err);
        return f.m - f.a;
    };
    double lower = nu_m * theta;
    // the opening evaluations: Brent's f(max), and the walk's first test f(lower) (pdf_m < pdf_a: walk on)
    double fx, f_low;
    bool walk_on;
    if (!G) {
        fx = zero_func(g_a_mean);
        const ss_pdf_pair f = ss_gamma_pdf2(nu_m, nu_a, theta, lg_m, lg_a, lower, err);
        walk_on = f.m < f.a;
        f_low = f.m - f.a;
    } else {
        int32_t e_spec = 0;  // both points are used: their poles are raised below
        const ss_pdf_pair f = ss_gamma_pdf2(nu_m, nu_a, theta, lg_m, lg_a, k == 0 ? g_a_mean : lower, e_spec);
        const double d = f.m - f.a;
        fx = grp_get(d, L, 0);
        f_low = grp_get(d, L, 1);
        walk_on = grp_get_i(f.m < f.a ? 1 : 0, L, 1) != 0;
        if (ss_pdf_pole(g_a_mean, nu_m, nu_a) || ss_pdf_pole(lower, nu_m, nu_a)) err = ERR_SKAUGEN_PDF;
    }
    SS_JOB_MARK(1);
    double upper;
    {  // brent_find_minima(zero_func, 0, g_a_mean, 2 bits), boost tools/minima.hpp
        double min = 0.0, max = g_a_mean;
        const double tolerance = 0.5;  // ldexp(1, 1-2)
        const double golden = (double)0.3819660f;
        double x, w, v, uu, delta, delta2, fu, fv, fw, mid, fract1, fract2;
        x = w = v = max;
        fw = fv = fx;
        delta2 = delta = 0;
        uint64_t count = ~uint64_t(0);
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
                    uu = x + delta;
                    if (((uu - min) < fract2) || ((max - uu) < fract2)) delta = (mid - x) < 0 ? -fabs(fract1) : fabs(fract1);
                }
            } else {
                delta2 = (x >= mid) ? min - x : max - x;
                delta = golden * delta2;
            }
            uu = (fabs(delta) >= fract1) ? (x + delta) : (delta > 0 ? x + fabs(fract1) : x - fabs(fract1));
            fu = zero_func(uu);
            if (fu <= fx) {
                if (uu >= x) min = x; else max = x;
                v = w; w = x; x = uu;
                fv = fw; fw = fx; fx = fu;
            } else {
                if (uu < x) min = uu; else max = uu;
                if ((fu <= fw) || (w == x)) {
                    v = w; w = uu; fv = fw; fw = fu;
                } else if ((fu <= fv) || (v == x) || (v == w)) {
                    v = uu; fv = fu;
                }
            }
        } while (--count);
        upper = x;  // fx = f(upper)
    }
    // while (pdf(g_m, lower) < pdf(g_a, lower)) lower *= 0.9; -- 0.9^k underflows to 0 within 7100 steps
    double fmin = f_low;
    bool have_fmin = true;
    if (walk_on) {
        lower *= 0.9;
        have_fmin = false;
        for (int it = 1; it < 8000; ++it) {
            const ss_pdf_pair f = ss_gamma_pdf2(nu_m, nu_a, theta, lg_m, lg_a, lower, err);
            if (!(f.m < f.a)) {
                fmin = f.m - f.a;
                have_fmin = true;
                break;
            }
            lower *= 0.9;
        }
    }
    SS_JOB_MARK(2);
    // bisect(zero_func, lower, upper, eps_tolerance(10), max_iter = 100), boost tools/roots.hpp
    double bmin = lower, bmax = upper;
    {
        if (!have_fmin) fmin = zero_func(bmin);
        const double fmax = fx;
        if (fmin == 0) {
            bmax = bmin;
        } else if (fmax == 0) {
            bmin = bmax;
        } else if (bmin >= bmax || fmin * fmax >= 0) {
            err = ERR_SKAUGEN_BISECT;  // boost raises evaluation_error
        } else {
            const double eps = 0x1p-9;  // max(ldexp(1, 1-10), 4*DBL_EPSILON)
            int count = 97;             // max_iter 100 minus the three evaluations so far
            auto go_on = [&]() { return count && !(fabs(bmin - bmax) <= eps * smin(fabs(bmin), fabs(bmax))); };
            if (!G || L < 4) {
                while (go_on()) {
                    const double mid = (bmin + bmax) / 2;
                    const double fmid = ss_zero_sign(nu_m, nu_a, theta, lg_m, lg_a, mid, err);
                    if ((mid == bmax) || (mid == bmin)) break;
                    if (fmid == 0) {
                        bmin = bmax = mid;
                        break;
                    }
                    const int sm = fmid > 0 ? 1 : (fmid < 0 ? -1 : 0), sn = fmin > 0 ? 1 : (fmin < 0 ? -1 : 0);
                    if (sm * sn < 0) {
                        bmax = mid;
                    } else {
                        bmin = mid;
                        fmin = fmid;
                    }
                    --count;
                }
            } else {
                constexpr int D = 2;  // levels per round: 2^D - 1 <= L points
                // this lane's point: heap node h (1 = the next midpoint, 2h / 2h+1 = the midpoints of its left /
                // right half); lanes beyond the tree repeat the root
                const int h = k < (1 << D) - 1 ? k + 1 : 1;
                const int depth = 31 - __builtin_clz((unsigned)h);
                bool more = go_on();
                while (more) {
                    double lo = bmin, hi = bmax;
                    for (int b = depth - 1; b >= 0; --b) {
                        const double m2 = (lo + hi) / 2;
                        if ((h >> b) & 1) lo = m2; else hi = m2;
                    }
                    int32_t e_spec = 0;  // raised below for the points the sequential loop evaluates
                    const double fk = ss_zero_sign(nu_m, nu_a, theta, lg_m, lg_a, (lo + hi) / 2, e_spec);
                    int node = 1;
                    for (int lev = 0; lev < D; ++lev) {
                        if (lev > 0 && !go_on()) {
                            more = false;
                            break;
                        }
                        const double mid = (bmin + bmax) / 2;
                        const double fmid = grp_get(fk, L, node - 1);
                        if (ss_pdf_pole(mid, nu_m, nu_a)) err = ERR_SKAUGEN_PDF;
                        if ((mid == bmax) || (mid == bmin)) {
                            more = false;
                            break;
                        }
                        if (fmid == 0) {
                            bmin = bmax = mid;
                            more = false;
                            break;
                        }
                        const int sm = fmid > 0 ? 1 : (fmid < 0 ? -1 : 0), sn = fmin > 0 ? 1 : (fmin < 0 ? -1 : 0);
                        if (sm * sn < 0) {
                            bmax = mid;
                            node = 2 * node;
                        } else {
                            bmin = mid;
                            fmin = fmid;
                            node = 2 * node + 1;
                        }
                        --count;
                    }
                    if (more) more = go_on();
                }
            }
        }
    }
    SS_JOB_MARK(3);
    const double x = (bmin + bmax) * 0.5;
    double m, a;
    if (!G) {
        m = gamma_p_prefix(nu_m, x / theta, lg_m, 2.220446049250313e-16).p;
        a = gamma_p_prefix(nu_a, x / theta, lg_a, 2.220446049250313e-16).p;
    } else {
        const double pk = gamma_p_prefix(k == 1 ? nu_a : nu_m, x / theta, k == 1 ? lg_a : lg_m, 2.220446049250313e-16).p;
        m = grp_get(pk, L, 0);
        a = grp_get(pk, L, 1);
    }
    SS_JOB_MARK(4);
    return a + 1.0 - m;
}

// one lane per job
__device__ __noinline__ double ss_sca_rel_red(uint64_t u, uint64_t n, double nu_a, double alpha, int32_t& err) {
    return ss_sca_rel_red_body<false>(u, n, nu_a, alpha, 1, 0, err);
}
// a group of L = 2 or 4 lanes per job
__device__ __noinline__ double ss_sca_rel_red_group(uint64_t u, uint64_t n, double nu_a, double alpha, int L, int k,
                                                    int32_t& err) {
    return ss_sca_rel_red_body<true>(u, n, nu_a, alpha, L, k, err);
}

// calculator::compute_shape_vars (skaugen.h:338-380)
__device__ inline void ss_compute_shape_vars(const ss_par& p, uint64_t nnn, uint64_t n, uint64_t u, double sca,
                                             double rel_red_sca, double& alpha, double& nu) {
    const double alpha_0 = p.alpha_0;
    const double nu_0 = p.alpha_0 * p.unit_size;
    const double dyn_var = nu / (alpha * alpha);
    const double init_var = nu_0 / (alpha_0 * alpha_0);
    double tot_var = 0.0;
    double tot_mean = 0.0;
    if (n > 0) {
        if (nnn == 0) {
            tot_var = (double)n * init_var * (1 + (double)(n - 1) * ss_c(n, p.d_range));
            tot_mean = (double)n * nu_0 / alpha_0;
        } else {
            const double old_var_cov =
                (double)(nnn + n) * init_var * (1 + (double)((nnn + n) - 1) * ss_c(nnn + n, p.d_range));
            const double new_var_cov = (double)n * init_var * (1 + (double)(n - 1) * ss_c(n, p.d_range));
            tot_var = old_var_cov * sca * sca + new_var_cov * (1.0 - sca) * (1.0 - sca);
            tot_mean = (sca * (double)(nnn + n) + (1.0 - sca) * (double)n) * p.unit_size;
        }
    }
    if (u > 0) {
        const double factor =
            (dyn_var / ((double)nnn * init_var) + 1.0 + (double)(nnn - 1) * ss_c(nnn, p.d_range)) / (double)(2 * nnn);
        const double non_cond_mean = (double)(nnn - u) * p.unit_size;
        tot_mean = non_cond_mean / (1.0 - rel_red_sca);
        const uint64_t cond_u = (uint64_t)ss_lrint((1.0 - rel_red_sca) * (double)nnn - (double)(nnn - u));
        const double auto_var =
            cond_u > 0 ? init_var * (double)cond_u * (1.0 + ((double)cond_u - 1.0) * ss_c(cond_u, p.d_range)) : 0.0;
        const double cross_var = cond_u > 0 ? init_var * (double)cond_u * 2.0 * factor * (double)cond_u : 0.0;
        tot_var = dyn_var + auto_var - cross_var;
    }
    if (fabs(tot_mean) < 1.0e-7) {
        nu = nu_0;
        alpha = alpha_0;
        return;
    }
    nu = tot_mean * tot_mean / tot_var;
    alpha = nu / (p.unit_size * (double)ss_lrint(tot_mean / p.unit_size));
}

// calculator::step (skaugen.h:151-336), split at its one expensive, divergent call -- sca_rel_red on a partial
// melt (skaugen.h:247) -- so that the kernel can hand those calls of a workgroup to as few wavefronts as possible
// (as pt_gs_k does with corr_lwc). ss_front runs the step up to that call and says whether it is needed (job
// arguments u, nnn, nu, alpha); ss_back finishes the step given its result. ss_step = front + call + back.
struct ss_mid {
    bool done;  // the early "no snow" return (skaugen.h:166-181): the step is complete
    bool need;  // sca_rel_red(u, nnn, nu, alpha) is needed
    uint64_t nnn, u, n;
    double swe, sca, nu, alpha, lwc, total_storage, snow, rain;
};

__device__ inline void ss_front(const ss_par& p, double step_in_days, double dt_hours, double T, double prec_mm_h,
                                ss_state& s, ss_mid& m, double& r_outflow, double& r_sca, double& r_swe) {
    const double snow_tol = 1.0e-10;
    const double unit_size = p.unit_size;
    const double prec = prec_mm_h * dt_hours;
    const double corr_prec = smax(0.0, prec + s.residual);
    s.residual = smin(0.0, prec + s.residual);
    const double snow = T < p.tx ? corr_prec : 0.0;
    const double rain = T < p.tx ? 0.0 : corr_prec;
    m.done = false;
    m.need = false;

    if (s.sca * s.swe < unit_size && snow < snow_tol) {
        r_outflow = rain + s.sca * (s.swe + s.free_water) + s.residual;
        if (dt_hours != 1.0) r_outflow = r_outflow / dt_hours;  // x / 1.0 == x exactly (hourly steps)
        s.residual = 0.0;
        if (r_outflow < 0.0) {
            s.residual = r_outflow;
            r_outflow = 0.0;
        }
        s.nu = p.alpha_0 * unit_size;
        s.alpha = p.alpha_0;
        s.sca = 0.0;
        s.swe = 0.0;
        s.free_water = 0.0;
        s.num_units = 0;
        r_sca = 0.0;
        r_swe = 0.0;
        m.done = true;
        return;
    }

    const double alpha_0 = p.alpha_0;
    double swe = s.swe;
    uint64_t nnn = s.num_units;
    double sca = s.sca;
    double nu = s.nu;
    double alpha = s.alpha;
    if (nnn > 0) {
        nu *= (double)nnn;
    } else {
        nu = alpha_0 * p.unit_size;
        alpha = alpha_0;
    }

    double total_new_snow = snow;
    double lwc = s.free_water;
    const double total_storage = swe + lwc;
    double pot_melt = p.cx * step_in_days * (T - p.ts);
    const double refreeze = smin(smax(0.0, -pot_melt * p.cfr), lwc);
    total_new_snow += sca * refreeze;
    lwc -= refreeze;
    pot_melt = smax(0.0, pot_melt);
    const double new_snow_reduction = smin(pot_melt, total_new_snow);
    pot_melt -= new_snow_reduction;
    total_new_snow -= new_snow_reduction;

    uint64_t n = 0, u = 0;
    if (total_new_snow > unit_size) {  // 1. accumulation
        n = (uint64_t)ss_lrint(total_new_snow / unit_size);
        ss_compute_shape_vars(p, nnn, n, 0, sca, 0.0, alpha, nu);
        nnn = (uint64_t)ss_lrint((double)nnn * sca) + n;
        sca = 1.0;
        swe = (double)nnn * unit_size;
    }
    if (pot_melt > unit_size) {  // 2. melting
        u = (uint64_t)ss_lrint(pot_melt / unit_size);
        if (nnn < u + 2) {
            nnn = 0;
            alpha = alpha_0;
            nu = alpha_0 * unit_size;
            swe = 0.0;
            lwc = 0.0;
            sca = 0.0;
        } else {
            m.need = true;  // sca_rel_red(u, nnn, nu, alpha)
        }
    }
    m.nnn = nnn; m.u = u; m.n = n;
    m.swe = swe; m.sca = sca; m.nu = nu; m.alpha = alpha; m.lwc = lwc;
    m.total_storage = total_storage; m.snow = snow; m.rain = rain;
}

__device__ inline void ss_back(const ss_par& p, double dt_hours, ss_state& s, const ss_mid& m, double rel_red_sca,
                               double& r_outflow, double& r_sca, double& r_swe) {
    if (m.done) return;
    const double unit_size = p.unit_size;
    const double alpha_0 = p.alpha_0;
    uint64_t nnn = m.nnn, u = m.u;
    const uint64_t n = m.n;
    double swe = m.swe, sca = m.sca, nu = m.nu, alpha = m.alpha, lwc = m.lwc;
    const double total_storage = m.total_storage, snow = m.snow, rain = m.rain;
    if (m.need) {  // 2. melting, the partial-melt branch (skaugen.h:246-275)
        const double sca_scale_factor = 1.0 - rel_red_sca;
        sca = s.sca * sca_scale_factor;
        swe = (double)(nnn - u) / sca_scale_factor * unit_size;
        if (swe >= (double)nnn * unit_size) {
            u = (uint64_t)((long)((double)nnn * rel_red_sca) + 1);
            swe = (double)(nnn - u) / sca_scale_factor * unit_size;
            if (nnn == u) sca = 0.0;
        }
        if (sca < 0.005) {
            nnn = 0;
            alpha = alpha_0;
            nu = alpha_0 * unit_size;
            swe = 0.0;
            lwc = 0.0;
            sca = 0.0;
        } else {
            ss_compute_shape_vars(p, nnn, n, u, sca, rel_red_sca, alpha, nu);
            nnn = (uint64_t)ss_lrint(swe / unit_size);
            swe = (double)nnn * unit_size;
        }
    }
    // 3. lwc from the swe*sca change
    if (s.sca * s.swe > sca * swe) lwc += smax(0.0, s.swe - swe);
    lwc *= smin(1.0, s.sca / sca);
    lwc = smin(lwc, swe * p.max_water_fraction);
    double discharge = s.sca * total_storage + snow - sca * (swe + lwc);
    if (discharge < 0.0) {
        s.residual += discharge;
        discharge = 0.0;
    }
    // 4. rain into lwc and/or discharge
    if (rain > swe * p.max_water_fraction - lwc) {
        discharge += sca * (rain - (swe * p.max_water_fraction - lwc)) + rain * (1.0 - sca);
        lwc = swe * p.max_water_fraction;
    } else {
        lwc += rain;
        discharge += rain * (1.0 - sca);
    }
    if (discharge >= -s.residual) {
        discharge += s.residual;
        s.residual = 0.0;
    }
    // 5. state and response
    if (nnn > 0) nu /= (double)nnn;
    r_outflow = dt_hours == 1.0 ? discharge : discharge / dt_hours;  // as in ss_front
    r_swe = sca * (swe + lwc);
    r_sca = sca;
    s.nu = nu;
    s.alpha = alpha;
    s.sca = sca;
    s.swe = swe;
    s.free_water = lwc;
    s.num_units = nnn;
}

__device__ inline void ss_step(const ss_par& p, double step_in_days, double dt_hours, double T, double prec_mm_h,
                               ss_state& s, double& r_outflow, double& r_sca, double& r_swe, int32_t& err) {
    ss_mid m;
    ss_front(p, step_in_days, dt_hours, T, prec_mm_h, s, m, r_outflow, r_sca, r_swe);
    const double rel = m.need ? ss_sca_rel_red(m.u, m.nnn, m.nu, m.alpha, err) : 0.0;
    ss_back(p, dt_hours, s, m, rel, r_outflow, r_sca, r_swe);
}

}  // namespace shyft_dev
