// Host statistics of the January Brent jobs (tools/mb/jobs_jan.bin: z1 a1 b1 a2 b2): f evaluations per job,
// incomplete-gamma method (series / continued fraction) and terms per evaluation. Build:
//   g++ -O2 -std=c++17 -ffp-contract=off -o /tmp/brent_stats tools/mb/brent_stats.cpp && /tmp/brent_stats
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../detmath/detmath.h"

static long n_series = 0, n_cf = 0, n_other = 0, it_series = 0, it_cf = 0;
static long hist_s[64] = {0}, hist_c[64] = {0};

static double calc_q(double a, double b, double z, double lga) {
    const double x = z / b;
    const int kind = detmath::gamma_pq_kind(a, x);
    const double eps = detmath::gamma_snow_policy_eps(a);
    if (kind == detmath::GPQ_SERIES) {
        ++n_series;
        // count terms: rerun the loop
        double ap = a, E = 1.0, B = 0.0, xn = 1.0;
        int n = 1;
        for (; n <= 2000; ++n) {
            ap += 1.0; xn *= x; E *= ap; B = std::fma(B, ap, xn);
            if (xn < eps * (B + E)) break;
            if (E > 1e200) { E *= 6.2230152778611417e-61; B *= 6.2230152778611417e-61; xn *= 6.2230152778611417e-61; }
        }
        it_series += n; hist_s[n < 63 ? n : 63]++;
    } else if (kind == detmath::GPQ_CF) {
        ++n_cf;
        double b_ = x + 1.0 - a, Pm = 1.0, Qm = 0.0, P = b_, Qd = 1.0, di = 0.0;
        int i = 1;
        for (; i <= 2000; ++i) {
            di += 1.0; const double an = -di * (di - a); b_ += 2.0;
            const double Pn = std::fma(b_, P, an * Pm), Qn = std::fma(b_, Qd, an * Qm);
            const double cross = Pn * Qd, diff = cross - P * Qn;
            Pm = P; Qm = Qd; P = Pn; Qd = Qn;
            if (std::fabs(diff) <= eps * std::fabs(cross)) break;
            if (std::fabs(P) > 1e200) { P *= 6.2230152778611417e-61; Qd *= 6.2230152778611417e-61; Pm *= 6.2230152778611417e-61; Qm *= 6.2230152778611417e-61; }
        }
        it_cf += i; hist_c[i < 63 ? i : 63]++;
    } else {
        ++n_other;
    }
    const auto g = detmath::gamma_pq<detmath::dm_policy>(a, x, lga, eps);
    return a * b * g.p1 + z * (1.0 - g.p);
}

int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "tools/mb/jobs_jan.bin", "rb");
    std::vector<double> h(5 * 200000);
    const int n = (int)(fread(h.data(), sizeof(double), h.size(), f) / 5);
    fclose(f);
    long nf = 0;
    double amin = 1e300, amax = 0;
    for (int i = 0; i < n; ++i) {
        const double* j = &h[5 * i];
        const double z1 = j[0], a1 = j[1], b1 = j[2], a2 = j[3], b2 = j[4];
        amin = std::fmin(amin, a2); amax = std::fmax(amax, a2);
        const double lga2 = detmath::lgamma(a2);
        const double Q1 = calc_q(a1, b1, z1, detmath::lgamma(a1));
        auto fz = [&](double z) { ++nf; const double v = calc_q(a2, b2, z, lga2) - Q1; return v * v; };
        double min = 0.0, max = z1, x, w, v, u, delta, delta2, fu, fv, fw, fx, mid, fract1, fract2;
        const double tol = 0x1p-11, golden = (double)0.3819660f;
        x = w = v = max; fw = fv = fx = fz(x); delta2 = delta = 0; int count = 60;
        do {
            mid = (min + max) / 2; fract1 = tol * std::fabs(x) + tol / 4; fract2 = 2 * fract1;
            if (std::fabs(x - mid) <= (fract2 - (max - min) / 2)) break;
            if (std::fabs(delta2) > fract1) {
                double r = (x - w) * (fx - fv), q = (x - v) * (fx - fw), p = (x - v) * q - (x - w) * r;
                q = 2 * (q - r); if (q > 0) p = -p; q = std::fabs(q); double td = delta2; delta2 = delta;
                if ((std::fabs(p) >= std::fabs(q * td / 2)) || (p <= q * (min - x)) || (p >= q * (max - x))) {
                    delta2 = (x >= mid) ? min - x : max - x; delta = golden * delta2;
                } else {
                    delta = p / q; u = x + delta;
                    if (((u - min) < fract2) || ((max - u) < fract2)) delta = (mid - x) < 0 ? -std::fabs(fract1) : std::fabs(fract1);
                }
            } else { delta2 = (x >= mid) ? min - x : max - x; delta = golden * delta2; }
            u = (std::fabs(delta) >= fract1) ? (x + delta) : (delta > 0 ? x + std::fabs(fract1) : x - std::fabs(fract1));
            fu = fz(u);
            if (fu <= fx) { if (u >= x) min = x; else max = x; v = w; w = x; x = u; fv = fw; fw = fx; fx = fu; }
            else { if (u < x) min = u; else max = u;
                if ((fu <= fw) || (w == x)) { v = w; w = u; fv = fw; fw = fu; }
                else if ((fu <= fv) || (v == x) || (v == w)) { v = u; fv = fu; } }
        } while (--count);
    }
    printf("jobs %d, f evals %ld (%.2f per job), a2 in [%g, %g]\n", n, nf, (double)nf / n, amin, amax);
    printf("calc_q calls: series %ld (%.1f terms avg), cf %ld (%.1f terms avg), other %ld\n", n_series,
           (double)it_series / (n_series ? n_series : 1), n_cf, (double)it_cf / (n_cf ? n_cf : 1), n_other);
    printf("series term histogram:"); for (int i = 0; i < 64; ++i) if (hist_s[i]) printf(" %d:%ld", i, hist_s[i]); printf("\n");
    printf("cf term histogram:"); for (int i = 0; i < 64; ++i) if (hist_c[i]) printf(" %d:%ld", i, hist_c[i]); printf("\n");
}
