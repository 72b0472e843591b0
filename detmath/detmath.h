// detmath.h — deterministic fp64 elementary functions (exp, log, pow, lgamma).
//
// The engine's HIP kernels and the CPU oracle both evaluate their physics with
// these functions, playing the role libm plays in the reference build. They use
// only IEEE-754 basic operations (+ - * /, fused multiply-add, compares) and
// integer bit manipulation, written out explicitly, so that compiled with FP
// contraction off they return bit-identical results on an x86-64 host and on
// gfx950. Accuracy against glibc is pinned by tests/test_detmath.py (<= 1 ulp
// for exp/log, <= 2 ulp for pow, <= 4e-15 absolute for lgamma on x in (0, 1e3]).
//
// Algorithms (restated from the standard literature):
//   exp  : Cody-Waite reduction x = k ln2 + r, |r| <= ln2/2, e^r = 1 + r q(r) with a degree-10 Chebyshev
//          fit q in Horner form, scaling by 2^k through the exponent bits.
//   log  : x = 2^k (1+f), 1+f in [sqrt(1/2), sqrt(2)), s = f/(2+f), fdlibm's e_log.c polynomial (one division);
//          pow and lgamma use log_dd: log m = 2 atanh(s) in double-double for the leading terms.
//   pow  : exp(y * log x) with log x carried as a double-double.
//   lgamma (x > 0): Stirling series with 8 Bernoulli terms for x >= 10; upward
//          recurrence lgamma(x) = lgamma(x+n) - log(x (x+1) ... (x+n-1)) below.
#ifndef SHYFT_DETMATH_H
#define SHYFT_DETMATH_H

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define DM_FN __host__ __device__ inline
#define DM_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define DM_FABS(a) __builtin_fabs(a)
#else
#include <cmath>
#define DM_FN inline
#define DM_FMA(a, b, c) std::fma((a), (b), (c))
#define DM_FABS(a) std::fabs(a)
#endif

// DM_NO_SPECULATE(): marks a rarely taken branch (the incomplete gamma's 2^-200 rescaling) as a real branch.
// Without it the gfx950 compiler if-converts the rescale into every unrolled series iteration (three ldexp
// and six selects per term, more than the term itself); as a branch it costs one scalar exec test.
#if defined(__HIP_DEVICE_COMPILE__)
#define DM_NO_SPECULATE() asm volatile("")
#else
#define DM_NO_SPECULATE() ((void)0)
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

// DM_GPQ_BLOCKED: the incomplete gamma's series / continued fraction start with blocks of terms (below); the
// results are the same either way, so this is a code-shape choice only (register pressure vs branches)
#ifndef DM_GPQ_BLOCKED
#define DM_GPQ_BLOCKED 0
#endif

namespace detmath {


DM_FN uint64_t as_u64(double x) {
    uint64_t u;
    memcpy(&u, &x, sizeof u);
    return u;
}
DM_FN double as_f64(uint64_t u) {
    double x;
    memcpy(&x, &u, sizeof x);
    return x;
}
DM_FN bool is_nan(double x) { return x != x; }
DM_FN double inf() { return as_f64(0x7ff0000000000000ull); }
DM_FN double qnan() { return as_f64(0x7ff8000000000000ull); }

// 2^k for k in [-1074, 1023]
DM_FN double pow2i(int k) {
    if (k >= -1022) return as_f64((uint64_t)(k + 1023) << 52);
    return as_f64(1ull << (k + 1074));  // subnormal
}

// ---------------------------------------------------------------- exp
// exp(x) = 2^k e^r, x = k ln2 + r (Cody-Waite), e^r by a degree-11 polynomial (below). For |x| <= 708 the
// scaling by 2^k (k in [-1021, 1021], e^r in [0.70, 1.42]) is exact, so it is one ldexp; exp_general holds the
// overflow / underflow / NaN cases (and gives the same value on the fast range, which the tests check).
#if defined(__HIP_DEVICE_COMPILE__)
#define DM_LDEXP(p, k) __builtin_ldexp((p), (k))
#define DM_COLD
#else
#define DM_LDEXP(p, k) std::ldexp((p), (k))
#define DM_COLD
#endif
// e^r = 1 + r q(r) on |r| <= ln2/2 (a little beyond): q of degree 10, a Chebyshev fit of (e^r - 1)/r (mpmath,
// 200-bit; relative error of 1 + r q(r) below 8.5e-18), coefficients highest degree first. r06: replaces the degree-13
// Taylor polynomial (two fused multiply-adds fewer per exp) and t = x/ln2 + 1.5 * 2^52 is one fused multiply-add;
// within 1 ulp of glibc (tests/test_detmath.py)
constexpr double EXP_Q[11] = {2.5105217004720745e-08, 2.7626371065696354e-07, 2.7557255400206422e-06, 2.480150431378554e-05,
                              0.00019841269874820627, 0.001388888893251478, 0.008333333333326136, 0.041666666666573066,
                              0.1666666666666667, 0.5000000000000006, 1.0};
DM_FN double exp_poly(double x, double& kf_out) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const double INV_LN2 = 1.4426950408889634;
    const double LN2_HI = 6.93147180369123816490e-01;  // upper 32 bits of ln2
    const double LN2_LO = 1.90821492927058770002e-10;
    const double SHIFT = 6755399441055744.0;           // 1.5 * 2^52
    const double t = DM_FMA(x, INV_LN2, SHIFT);
    const double kf = t - SHIFT;                        // round-to-nearest integer
    double r = DM_FMA(-kf, LN2_HI, x);
    r = DM_FMA(-kf, LN2_LO, r);
    double q = EXP_Q[0];
#if defined(__clang__)
#pragma unroll
#endif
    for (int i = 1; i < 11; ++i) q = DM_FMA(q, r, EXP_Q[i]);
    kf_out = kf;
    return DM_FMA(r, q, 1.0);
}

// every x (the reference formulation: NaN, overflow, gradual underflow)
DM_COLD DM_FN double exp_general(double x) {
    if (is_nan(x)) return x;
    if (x > 709.782712893384) return inf();
    if (x < -745.1332191019412) return 0.0;
    double kf;
    const double p = exp_poly(x, kf);
    const int k = (int)kf;
    if (k > 1023) return (p * pow2i(1023)) * pow2i(k - 1023);
    if (k < -1021) return (p * pow2i(k + 1000)) * pow2i(-1000);
    return p * pow2i(k);
}

// returns exp(x); for |x| inside the finite range the error is < 1 ulp
DM_FN double exp(double x) {
    if (DM_FABS(x) <= 708.0) {
        double kf;
        const double p = exp_poly(x, kf);
        return DM_LDEXP(p, (int)kf);
    }
    return exp_general(x);
}

// ---------------------------------------------------------------- log (double-double core)
// log(x) = hi + lo for finite x > 0 (normal or subnormal): pow's and lgamma's double-double log
DM_FN void log_dd(double x, double& hi, double& lo) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    int e = 0;
    if (x < 2.2250738585072014e-308) {  // subnormal: scale up by 2^54
        x = x * 18014398509481984.0;
        e = -54;
    }
    uint64_t u = as_u64(x);
    e += (int)((u >> 52) & 0x7ff) - 1023;
    u = (u & 0x000fffffffffffffull) | 0x3ff0000000000000ull;  // m in [1, 2)
    double m = as_f64(u);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e += 1;
    }
    const double f = m - 1.0;  // exact (Sterbenz)
    // s = f / (2 + f) as s_hi + s_lo
    const double d = 2.0 + f;
    const double d_lo = (2.0 - d) + f;  // fast two-sum (|2| >= |f|)
    const double s = f / d;
#ifdef DM_ABLATE_LOG_SLO  // timing ablation only (wrong results)
    const double s_lo = 0.0 * d_lo;
#else
    const double s_lo = (DM_FMA(-s, d, f) - s * d_lo) / d;
#endif
    const double z = s * s;
    // 2 atanh(s) = 2s + s^3 * (2/3 + 2/5 z + 2/7 z^2 + ...); |s| <= 0.1716, z <= 0.02944
    double t = 2.0 / 25;
    t = DM_FMA(t, z, 2.0 / 23);
    t = DM_FMA(t, z, 2.0 / 21);
    t = DM_FMA(t, z, 2.0 / 19);
    t = DM_FMA(t, z, 2.0 / 17);
    t = DM_FMA(t, z, 2.0 / 15);
    t = DM_FMA(t, z, 2.0 / 13);
    t = DM_FMA(t, z, 2.0 / 11);
    t = DM_FMA(t, z, 2.0 / 9);
    t = DM_FMA(t, z, 2.0 / 7);
    t = DM_FMA(t, z, 2.0 / 5);
    t = DM_FMA(t, z, 2.0 / 3);
    const double tail = (s * z) * t;  // s^3 * P(z), |tail| <= 0.0035
    // e*ln2 in double-double (LN2_HI has 32 trailing zero bits: e*LN2_HI exact)
    const double LN2_HI = 6.93147180369123816490e-01;
    const double LN2_LO = 1.90821492927058770002e-10;
    const double ed = (double)e;
    const double a_hi = ed * LN2_HI;
    const double a_lo = ed * LN2_LO;
    // sum = a_hi + 2s (two-sum), then add the small parts
    const double b = 2.0 * s;
    const double sum = a_hi + b;
    const double bb = sum - a_hi;
    const double err = (a_hi - (sum - bb)) + (b - bb);
    const double small = ((err + 2.0 * s_lo) + tail) + a_lo;
    hi = sum + small;
    lo = small - (hi - sum);
}

// log(x) = k ln2 + log(1 + f) for positive normal finite x: the method of fdlibm's e_log.c (one division) -- 1 + f
// in [sqrt(2)/2, sqrt(2)), s = f / (2 + f), log(1 + f) = f - hfsq + s (hfsq + R(s^2)) with fdlibm's 7-term minimax R,
// here evaluated with fused multiply-adds; k_adj: an exponent the caller removed (subnormal scaling). Within 1 ulp of
// glibc (tests/test_detmath.py). r06: replaces log_dd's hi part (a double-double atanh series with two divisions:
// one division fewer on every log of every stack; log_dd stays for pow and lgamma, which use its low part).
constexpr double LOG_LG1 = 6.666666666666735130e-01, LOG_LG2 = 3.999999999940941908e-01,
                 LOG_LG3 = 2.857142874366239149e-01, LOG_LG4 = 2.222219843214978396e-01,
                 LOG_LG5 = 1.818357216161805012e-01, LOG_LG6 = 1.531383769920937332e-01,
                 LOG_LG7 = 1.479819860511658591e-01;
DM_FN double log_core(double x, int k_adj) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    const double LN2_HI = 6.93147180369123816490e-01;  // upper 32 bits of ln2: dk * LN2_HI is exact
    const double LN2_LO = 1.90821492927058770002e-10;
    uint64_t u = as_u64(x);
    int k = (int)((u >> 52) & 0x7ff) - 1023 + k_adj;
    const uint32_t hx = (uint32_t)(u >> 32) & 0x000fffffu;
    const uint32_t i = (hx + 0x95f64u) & 0x100000u;  // 1 + f >= sqrt(2): halve it
    u = (u & 0x000fffffffffffffull) | ((uint64_t)(i ^ 0x3ff00000u) << 32);
    k += (int)(i >> 20);
    const double f = as_f64(u) - 1.0;
    const double s = f / (2.0 + f);
    const double dk = (double)k;
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * DM_FMA(w, DM_FMA(w, LOG_LG6, LOG_LG4), LOG_LG2);
    const double t2 = z * DM_FMA(w, DM_FMA(w, DM_FMA(w, LOG_LG7, LOG_LG5), LOG_LG3), LOG_LG1);
    const double R = t2 + t1;
    if (((int32_t)(hx - 0x6147au) | (int32_t)(0x6b851u - hx)) > 0) {
        const double hfsq = 0.5 * f * f;
        return dk * LN2_HI - ((hfsq - DM_FMA(s, hfsq + R, dk * LN2_LO)) - f);
    }
    return dk * LN2_HI - (DM_FMA(s, f - R, -(dk * LN2_LO)) - f);
}

// every x (NaN, negative, zero, infinity, subnormal)
DM_COLD DM_FN double log_general(double x) {
    if (is_nan(x)) return x;
    if (x < 0.0) return qnan();
    if (x == 0.0) return -inf();
    if (x == inf()) return x;
    if (x < 2.2250738585072014e-308) return log_core(x * 18014398509481984.0, -54);  // subnormal: scale by 2^54
    return log_core(x, 0);
}

DM_FN double log(double x) {
    if (x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308) return log_core(x, 0);  // positive normal
    return log_general(x);
}

// ---------------------------------------------------------------- pow
DM_FN bool is_integer(double y) {
    // |y| >= 2^52 is always an integer
    if (!(y == y)) return false;
    const double ay = y < 0 ? -y : y;
    if (ay >= 4503599627370496.0) return true;
    const double t = (ay + 4503599627370496.0) - 4503599627370496.0;
    return t == ay;
}
DM_FN bool is_odd_integer(double y) {
    if (!is_integer(y)) return false;
    const double ay = y < 0 ? -y : y;
    if (ay >= 9007199254740992.0) return false;
    const double h = ay * 0.5;
    return !is_integer(h);
}

DM_FN double pow(double x, double y) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    if (y == 0.0) return 1.0;
    if (x == 1.0) return 1.0;
    if (y == 1.0) return x;  // exact, as a correctly rounded pow (distance_measure with factor 2)
    if (y == 2.0) return x * x;  // the correctly rounded square (hbv_soil's default beta = 2, hbv_soil.h:19-24)
    if (is_nan(x) || is_nan(y)) return qnan();
    const double ax = x < 0 ? -x : x;
    const double ay = y < 0 ? -y : y;
    if (ay == inf()) {
        if (ax == 1.0) return 1.0;
        return ((ax > 1.0) == (y > 0)) ? inf() : 0.0;
    }
    if (x == 0.0 || ax == inf()) {
        const bool odd = is_odd_integer(y);
        const bool neg = x < 0 || (x == 0.0 && as_u64(x) >> 63);
        double r = ((x == 0.0) == (y < 0)) ? inf() : 0.0;
        return (neg && odd) ? -r : r;
    }
    double sign = 1.0;
    if (x < 0) {
        if (!is_integer(y)) return qnan();
        if (is_odd_integer(y)) sign = -1.0;
    }
    double lh, ll;
    log_dd(ax, lh, ll);
    const double ph = y * lh;
    const double pl = DM_FMA(y, lh, -ph) + y * ll;
    if (ph > 709.782712893384) return sign * inf();
    if (ph < -745.1332191019412) return sign * 0.0;
    const double e = detmath::exp(ph);
    return sign * DM_FMA(e, pl, e);
}

// pow4 / pow8: x^4 and x^8 by repeated squaring (<= 1.5 / 3.5 ulp from the exact power). The physics raise
// to these small integer powers with std::pow (priestley_taylor.h:97-102, gamma_snow.h:368-410); two or three
// multiplications replace a full pow (~390 instructions on gfx950).
DM_FN double pow4(double x) {
    const double x2 = x * x;
    return x2 * x2;
}
DM_FN double pow8(double x) {
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return x4 * x4;
}
// powr(x, y) = exp(y * log x) for x >= 0 with the single-double log: error <= (|y ln x| + 2) ulp. Used for
// the physics' fractional powers of moderate arguments and for odeint's step-size controller, where the
// double-double log of pow buys nothing over the reference's own libm.
DM_FN double powr(double x, double y) { return detmath::exp(y * detmath::log(x)); }

// ---------------------------------------------------------------- lgamma (x > 0)
DM_FN double lgamma(double x) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    if (is_nan(x)) return x;
    if (x <= 0.0) return inf();  // poles / negative arguments are not used by the method stacks
    if (x == inf()) return x;
    double shift = 0.0;
    if (x < 10.0) {
        // lgamma(x) = lgamma(x+n) - log(prod_{k<n}(x+k)), x+n >= 10
        double prod = 1.0;
        while (x < 10.0) {
            prod = prod * x;
            x = x + 1.0;
        }
        shift = detmath::log(prod);
    }
    // Stirling: (x-1/2) log x - x + log(2pi)/2 + sum B2k / (2k(2k-1) x^(2k-1))
    const double HALF_LOG_2PI = 0.91893853320467274178;
    const double r = 1.0 / x;
    const double r2 = r * r;
    double s = -3617.0 / 122400.0;
    s = DM_FMA(s, r2, 1.0 / 156.0);
    s = DM_FMA(s, r2, -691.0 / 360360.0);
    s = DM_FMA(s, r2, 1.0 / 1188.0);
    s = DM_FMA(s, r2, -1.0 / 1680.0);
    s = DM_FMA(s, r2, 1.0 / 1260.0);
    s = DM_FMA(s, r2, -1.0 / 360.0);
    s = DM_FMA(s, r2, 1.0 / 12.0);
    s = s * r;
    double lh, ll;
    log_dd(x, lh, ll);
    const double xm = x - 0.5;
    // (x-1/2)(lh+ll) - x, with the large cancellation handled by fma
    const double a = xm * lh;
    const double a_lo = DM_FMA(xm, lh, -a) + xm * ll;
    const double v = (a - x) + (a_lo + (HALF_LOG_2PI + s));
    return v - shift;
}

// ---------------------------------------------------------------- incomplete gamma
// The method stacks call boost::math::gamma_p (gamma_snow.h:195-197). detmath
// supplies it the way it supplies libm: one deterministic implementation used
// by both the kernels and the oracle. M is the elementary-function policy
// (detmath itself, or the host libm for the oracle's libm variant).
//
// gamma_pq(a, x, lga) returns P(a,x), P(a+1,x) and prefix = x^a e^-x / Gamma(a)
// (lga = lgamma(a) supplied by the caller).
//   x < a+1 : series P(a,x) = prefix * sum_{n>=0} x^n / (a(a+1)...(a+n)), summed as
//             a rational (B + E) / (a E) with E = (a+1)...(a+n) and
//             B = sum_{k>=1} x^k E/(a+1..a+k) — one division instead of one per term.
//             P(a+1,x) = prefix * B / (a E) (the n>=1 tail; no cancellation).
//   x >= a+1: continued fraction Q(a,x) = prefix / (b0 + a1/(b1 + a2/(b2 + ...))),
//             b_i = x + 2i + 1 - a, a_i = -i (i - a), by the forward (Wallis)
//             recurrence with rescaling; P = 1 - Q, P(a+1,x) = 1 - (Q + prefix/a).
// Terms are added until the next one is below 2^-52 of the sum (at most 2000).
struct gamma_pq_result {
    double p, p1, prefix;
};

struct dm_policy {
    DM_FN static double exp(double x) { return detmath::exp(x); }
    DM_FN static double log(double x) { return detmath::log(x); }
};

// The evaluation in pieces: gamma_pq_kind picks the special case or the method, gamma_pq_prefix is the
// prefix, gamma_series_sums / gamma_cf_terms run the series / continued fraction, gamma_pq_finish combines.
// gamma_pq below is exactly their composition (the prefix, series and continued-fraction chains of one
// evaluation are independent until the finish, so a caller may also run them apart).
enum { GPQ_NAN = 0, GPQ_ZERO = 1, GPQ_INF = 2, GPQ_SERIES = 3, GPQ_CF = 4 };

DM_FN int gamma_pq_kind(double a, double x) {
    if (is_nan(a) || is_nan(x)) return GPQ_NAN;
    if (x <= 0.0) return GPQ_ZERO;
    if (x == inf()) return GPQ_INF;
    return x < a + 1.0 ? GPQ_SERIES : GPQ_CF;
}

template <class M>
DM_FN double gamma_pq_prefix(double a, double x, double lga) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    return M::exp(a * M::log(x) - x - lga);
}

constexpr double GPQ_SCALE_HI = 1.0e200, GPQ_SCALE = 6.2230152778611417e-61;  // 2^-200

// series: E = (a+1)...(a+n), B = sum_{k>=1} x^k E/(a+1..a+k)
// Blocks of 4 terms first: the four terms and their exit tests are computed before any test is looked at
// (straight-line code, one branch per block instead of two per term); the block whose test fires returns the
// state of its FIRST firing term, which is where the term-by-term loop stops. A block in which E passes the
// rescale threshold is run again term by term (the loop below), so every result is the loop's, bit for bit.
DM_FN void gamma_series_sums(double a, double x, double eps, double& B_out, double& E_out) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    double ap = a, E = 1.0, B = 0.0, xn = 1.0;
    int n0 = 1;
#if DM_GPQ_BLOCKED
    for (; n0 + 3 <= 2000; n0 += 4) {
        const double a1 = ap + 1.0, x1 = xn * x, E1 = E * a1, B1 = DM_FMA(B, a1, x1);
        const double a2 = a1 + 1.0, x2 = x1 * x, E2 = E1 * a2, B2 = DM_FMA(B1, a2, x2);
        const double a3 = a2 + 1.0, x3 = x2 * x, E3 = E2 * a3, B3 = DM_FMA(B2, a3, x3);
        const double a4 = a3 + 1.0, x4 = x3 * x, E4 = E3 * a4, B4 = DM_FMA(B3, a4, x4);
        const bool t1 = x1 < eps * (B1 + E1), t2 = x2 < eps * (B2 + E2), t3 = x3 < eps * (B3 + E3),
                   t4 = x4 < eps * (B4 + E4);
        if ((E1 > GPQ_SCALE_HI) | (E2 > GPQ_SCALE_HI) | (E3 > GPQ_SCALE_HI) | (E4 > GPQ_SCALE_HI)) break;
        if (t1 | t2 | t3 | t4) {
            B_out = t1 ? B1 : t2 ? B2 : t3 ? B3 : B4;
            E_out = t1 ? E1 : t2 ? E2 : t3 ? E3 : E4;
            return;
        }
        ap = a4; xn = x4; E = E4; B = B4;
    }
#endif
    for (int n = n0; n <= 2000; ++n) {
        ap = ap + 1.0;
        xn = xn * x;
        E = E * ap;
        B = DM_FMA(B, ap, xn);
        if (xn < eps * (B + E)) break;
        if (E > GPQ_SCALE_HI) {
            DM_NO_SPECULATE();
            E = E * GPQ_SCALE;
            B = B * GPQ_SCALE;
            xn = xn * GPQ_SCALE;
        }
    }
    B_out = B;
    E_out = E;
}

// Wallis recurrence for K = b0 + a1/(b1 + a2/(b2 + ...)) = P / Qd
// (blocks of 2 terms first, as gamma_series_sums)
DM_FN void gamma_cf_terms(double a, double x, double eps, double& P_out, double& Qd_out) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    double b = x + 1.0 - a;
    double Pm = 1.0, Qm = 0.0;  // n-1
    double P = b, Qd = 1.0;     // n (= 0)
    double di = 0.0;  // i as a double (exact), counted instead of converted each term
    int i0 = 1;
#if DM_GPQ_BLOCKED
    for (; i0 + 1 <= 2000; i0 += 2) {
        const double d1 = di + 1.0, an1 = -d1 * (d1 - a), b1 = b + 2.0;
        const double P1 = DM_FMA(b1, P, an1 * Pm), Q1 = DM_FMA(b1, Qd, an1 * Qm);
        const double c1 = P1 * Qd, e1 = c1 - P * Q1;
        const double d2 = d1 + 1.0, an2 = -d2 * (d2 - a), b2 = b1 + 2.0;
        const double P2 = DM_FMA(b2, P1, an2 * P), Q2 = DM_FMA(b2, Q1, an2 * Qd);
        const double c2 = P2 * Q1, e2 = c2 - P1 * Q2;
        const bool t1 = DM_FABS(e1) <= eps * DM_FABS(c1), t2 = DM_FABS(e2) <= eps * DM_FABS(c2);
        if (t1) { P_out = P1; Qd_out = Q1; return; }
        if (DM_FABS(P1) > GPQ_SCALE_HI || DM_FABS(P2) > GPQ_SCALE_HI) break;
        if (t2) { P_out = P2; Qd_out = Q2; return; }
        di = d2; b = b2; Pm = P1; Qm = Q1; P = P2; Qd = Q2;
    }
#endif
    for (int i = i0; i <= 2000; ++i) {
        di = di + 1.0;
        const double an = -di * (di - a);
        b = b + 2.0;
        const double Pn = DM_FMA(b, P, an * Pm);
        const double Qn = DM_FMA(b, Qd, an * Qm);
        // |Pn/Qn - P/Qd| < eps |Pn/Qn|  <=>  |Pn Qd - P Qn| < eps |Pn Qd|
        const double cross = Pn * Qd;
        const double diff = cross - P * Qn;
        Pm = P; Qm = Qd;
        P = Pn; Qd = Qn;
        if (DM_FABS(diff) <= eps * DM_FABS(cross)) break;
        const double aP = DM_FABS(P);
        if (aP > GPQ_SCALE_HI) {
            DM_NO_SPECULATE();
            P = P * GPQ_SCALE; Qd = Qd * GPQ_SCALE; Pm = Pm * GPQ_SCALE; Qm = Qm * GPQ_SCALE;
        }
    }
    P_out = P;
    Qd_out = Qd;
}

// kind from gamma_pq_kind; prefix from gamma_pq_prefix (SERIES / CF); (u, v) = (B, E) or (P, Qd)
DM_FN gamma_pq_result gamma_pq_finish(int kind, double a, double prefix, double u, double v) {
#if defined(__clang__)
#pragma clang fp contract(off)
#endif
    gamma_pq_result r;
    if (kind == GPQ_NAN) {
        r.p = r.p1 = r.prefix = qnan();
    } else if (kind == GPQ_ZERO) {
        r.p = r.p1 = r.prefix = 0.0;
    } else if (kind == GPQ_INF) {
        r.p = r.p1 = 1.0;
        r.prefix = 0.0;
    } else if (kind == GPQ_SERIES) {
        r.prefix = prefix;
        const double aE = a * v;
        const double p = prefix * ((u + v) / aE);
        const double p1 = prefix * (u / aE);
        r.p = p < 1.0 ? p : 1.0;
        r.p1 = p1 < 1.0 ? p1 : 1.0;
    } else {
        r.prefix = prefix;
        const double q = prefix * (v / u);
        const double q1 = q + prefix / a;
        const double p = 1.0 - q;
        const double p1 = 1.0 - q1;
        r.p = p > 0.0 ? p : 0.0;
        r.p1 = p1 > 0.0 ? p1 : 0.0;
    }
    return r;
}

template <class M>
DM_FN gamma_pq_result gamma_pq(double a, double x, double lga, double eps = 2.220446049250313e-16) {
    const int kind = gamma_pq_kind(a, x);
    if (kind < GPQ_SERIES) return gamma_pq_finish(kind, a, 0.0, 0.0, 0.0);
    const double prefix = gamma_pq_prefix<M>(a, x, lga);
    double u, v;
    if (kind == GPQ_SERIES) gamma_series_sums(a, x, eps, u, v);
    else gamma_cf_terms(a, x, eps, u, v);
    return gamma_pq_finish(kind, a, prefix, u, v);
}

DM_FN double gamma_p(double a, double x) { return gamma_pq<dm_policy>(a, x, detmath::lgamma(a)).p; }

// boost::math precision policies used by gamma_snow (gamma_snow.h:189-197):
// gamma_p(a, .) with digits10<10> when a < 2, digits10<5> otherwise. boost maps
// digits10<d> to digits2 = (d+1)*1000/301 bits and stops its series / continued
// fractions at a relative term size of ldexp(1, 1 - digits2):
//   digits10<10> -> 36 bits -> 2^-35;  digits10<5> -> 19 bits -> 2^-18.
// DETMATH_GAMMA_POLICY_FULL (oracle tolerance variants only): full double precision instead of the policy
#ifdef DETMATH_GAMMA_POLICY_FULL
DM_FN double gamma_snow_policy_eps(double) { return 2.220446049250313e-16; }
#else
DM_FN double gamma_snow_policy_eps(double a) { return a < 2.0 ? 0x1p-35 : 0x1p-18; }
#endif

}  // namespace detmath

#endif  // SHYFT_DETMATH_H
