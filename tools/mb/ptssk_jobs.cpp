// Analysis tool (CPU, no GPU): what a pt_ss_k sca_rel_red job costs, on the jobs of the bench region.
//
// Runs Skaugen's snow routine (the oracle's restatement, oracle/src/ptssk.hpp) with the default PTSSKParameter on
// sampled cells of the 1M-cell synthetic region over the year (the device generator's forcing, synth_hash.h), and for
// every partial-melt call of statistics::sca_rel_red (core/skaugen.h:57-82) counts the zero_func evaluations of each
// phase (2-bit Brent, bracket walk, bisection) and the series / continued-fraction terms of the two final cdfs.
// Prints per-month counts and, with -o FILE, writes the jobs (u, n, nu_a, alpha, month) for tools/mb microbenchmarks.
// build: g++ -O2 -std=c++17 -mfma -ffp-contract=off -o tools/mb/ptssk_jobs tools/mb/ptssk_jobs.cpp
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../oracle/src/ptssk.hpp"
#include "../../shyft_amd/csrc/include_internal/synth_hash.h"

using namespace oracle;
using skaugen::ulong;

struct job_stat {
    long brent = 0, walk = 0, bisect = 0, terms_m = 0, terms_a = 0;
    int kind_m = 0, kind_a = 0;
};

// detmath's series / continued fraction with a term counter (the same loops, unblocked: the count is the loop's)
static int series_terms(double a, double x, double eps) {
    double ap = a, E = 1.0, B = 0.0, xn = 1.0;
    for (int n = 1; n <= 2000; ++n) {
        ap = ap + 1.0; xn = xn * x; E = E * ap; B = std::fma(B, ap, xn);
        if (xn < eps * (B + E)) return n;
        if (E > 1e200) { E *= 0x1p-200; B *= 0x1p-200; xn *= 0x1p-200; }
    }
    return 2000;
}
static int cf_terms(double a, double x, double eps) {
    double b = x + 1.0 - a, Pm = 1.0, Qm = 0.0, P = b, Qd = 1.0, di = 0.0;
    for (int i = 1; i <= 2000; ++i) {
        di += 1.0;
        const double an = -di * (di - a);
        b += 2.0;
        const double Pn = std::fma(b, P, an * Pm), Qn = std::fma(b, Qd, an * Qm);
        const double cross = Pn * Qd, diff = cross - P * Qn;
        Pm = P; Qm = Qd; P = Pn; Qd = Qn;
        if (std::fabs(diff) <= eps * std::fabs(cross)) return i;
        if (std::fabs(P) > 1e200) { P *= 0x1p-200; Qd *= 0x1p-200; Pm *= 0x1p-200; Qm *= 0x1p-200; }
    }
    return 2000;
}
static int terms(double a, double x, int& kind) {
    kind = detmath::gamma_pq_kind(a, x);
    if (kind == detmath::GPQ_SERIES) return series_terms(a, x, 2.220446049250313e-16);
    if (kind == detmath::GPQ_CF) return cf_terms(a, x, 2.220446049250313e-16);
    return 0;
}

// statistics::sca_rel_red as oracle/src/ptssk.hpp states it, with the evaluations counted per phase
static double sca_rel_red_counted(ulong u, ulong n, double nu_a, double alpha, job_stat& js) {
    const double nu_m = ((double)u / n) * nu_a;
    const skaugen::gamma_dist g_m{nu_m, 1.0 / alpha};
    const skaugen::gamma_dist g_a{nu_a, 1.0 / alpha};
    long* ctr = &js.brent;
    auto zero_func = [&](const double& x) { ++*ctr; return g_m.pdf(x) - g_a.pdf(x); };
    double lower = g_m.mean();
    uintmax_t brent_iter = std::numeric_limits<uintmax_t>::max();
    double upper = special::brent_find_minima(zero_func, 0.0, g_a.mean(), 2, brent_iter).first;
    while (g_m.pdf(lower) < g_a.pdf(lower)) { lower *= 0.9; ++js.walk; }
    ++js.walk;  // the final (failing) test
    ctr = &js.bisect;
    uintmax_t max_iter = 100;
    auto res = skaugen::bisect(zero_func, lower, upper, 10, max_iter);
    const double x = (res.first + res.second) * 0.5;
    js.terms_m = terms(nu_m, x * alpha, js.kind_m);
    js.terms_a = terms(nu_a, x * alpha, js.kind_a);
    return g_a.cdf(x) + 1.0 - g_m.cdf(x);
}

int main(int argc, char** argv) {
    int n_cells = 4096, stride = 256;
    const char* out = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) n_cells = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s") && i + 1 < argc) stride = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-o") && i + 1 < argc) out = argv[++i];
    }
    const uint64_t seed = 20251015ull;
    skaugen::parameter p;  // PTSSKParameter defaults (skaugen.h:89-112)
    const int64_t dt = HOUR_US;
    const int month_end[12] = {744, 1416, 2160, 2880, 3624, 4344, 5088, 5832, 6552, 7296, 8016, 8760};
    long steps_m[12] = {0}, jobs_m[12] = {0};
    job_stat sum_m[12];
    long hist_walk[8] = {0};  // 0,1,2-3,4-7,8-15,16-31,32-63,64+
    std::vector<double> rec;
    for (int c = 0; c < n_cells; ++c) {
        const uint64_t cell = (uint64_t)c * stride;
        const double z = synth_elevation(seed, cell);
        const uint64_t ck = synth_cell_key(seed, cell);
        skaugen::state s;
        skaugen::response r;
        int mon = 0;
        for (int i = 0; i < 8760; ++i) {
            while (i >= month_end[mon]) ++mon;
            double v[5];
            synth_values_ck(ck, (uint64_t)i, z, v);
            ++steps_m[mon];
            // the step's partial-melt call, found as skaugen::step finds it (skaugen.h:151-247)
            {
                const double dt_hours = 1.0, step_in_days = 1.0 / 24.0;
                const double prec = v[1] * dt_hours;
                const double corr_prec = std::max(0.0, prec + s.residual);
                const double snow = v[0] < p.tx ? corr_prec : 0.0;
                if (!(s.sca * s.swe < p.unit_size && snow < 1.0e-10)) {
                    ulong nnn = s.num_units;
                    double sca = s.sca, nu = s.nu, alpha = s.alpha;
                    if (nnn > 0) nu *= nnn; else { nu = p.alpha_0 * p.unit_size; alpha = p.alpha_0; }
                    double total_new_snow = snow, lwc = s.free_water;
                    double pot_melt = p.cx * step_in_days * (v[0] - p.ts);
                    const double refreeze = std::min(std::max(0.0, -pot_melt * p.cfr), lwc);
                    total_new_snow += sca * refreeze;
                    pot_melt = std::max(0.0, pot_melt);
                    const double nsr = std::min(pot_melt, total_new_snow);
                    pot_melt -= nsr;
                    total_new_snow -= nsr;
                    skaugen::statistics stat(p.alpha_0, p.d_range, p.unit_size);
                    if (total_new_snow > p.unit_size) {
                        const ulong n = (ulong)skaugen::lrint_(total_new_snow / p.unit_size);
                        skaugen::compute_shape_vars(stat, nnn, n, 0, sca, 0.0, alpha, nu);
                        nnn = (ulong)skaugen::lrint_(nnn * sca) + n;
                    }
                    if (pot_melt > p.unit_size) {
                        const ulong u = (ulong)skaugen::lrint_(pot_melt / p.unit_size);
                        if (!(nnn < u + 2)) {
                            job_stat js;
                            const double got = sca_rel_red_counted(u, nnn, nu, alpha, js);
                            const double want = skaugen::statistics::sca_rel_red(u, nnn, p.unit_size, nu, alpha);
                            if (memcmp(&got, &want, 8)) { fprintf(stderr, "mismatch\n"); return 1; }
                            ++jobs_m[mon];
                            sum_m[mon].brent += js.brent; sum_m[mon].walk += js.walk; sum_m[mon].bisect += js.bisect;
                            sum_m[mon].terms_m += js.terms_m; sum_m[mon].terms_a += js.terms_a;
                            sum_m[mon].kind_m += js.kind_m == detmath::GPQ_SERIES;
                            sum_m[mon].kind_a += js.kind_a == detmath::GPQ_SERIES;
                            int b = 0;
                            for (long w = js.walk - 1; w > 0 && b < 7; w >>= 1) ++b;
                            ++hist_walk[b];
                            if (out) {
                                const double row[9] = {(double)u, (double)nnn, nu, alpha, (double)mon, (double)js.brent,
                                                       (double)js.walk, (double)js.bisect,
                                                       (double)(js.terms_m + js.terms_a)};
                                rec.insert(rec.end(), row, row + 9);
                            }
                        }
                    }
                }
            }
            skaugen::step(dt, p, v[0], v[1], s, r);
        }
    }
    printf("month  job%%  evals/job: brent walk bisect | cdf terms m a | series%% m a\n");
    long tj = 0, tb = 0, tw = 0, tbi = 0, ttm = 0, tta = 0;
    for (int m = 0; m < 12; ++m) {
        const double J = jobs_m[m] ? (double)jobs_m[m] : 1.0;
        printf("%5d %5.1f  %6.2f %6.2f %6.2f | %6.1f %6.1f | %5.1f %5.1f\n", m + 1, 100.0 * jobs_m[m] / steps_m[m],
               sum_m[m].brent / J, sum_m[m].walk / J, sum_m[m].bisect / J, sum_m[m].terms_m / J, sum_m[m].terms_a / J,
               100.0 * sum_m[m].kind_m / J, 100.0 * sum_m[m].kind_a / J);
        tj += jobs_m[m]; tb += sum_m[m].brent; tw += sum_m[m].walk; tbi += sum_m[m].bisect;
        ttm += sum_m[m].terms_m; tta += sum_m[m].terms_a;
    }
    const double J = tj ? (double)tj : 1.0;
    printf("year  jobs %ld: brent %.2f walk %.2f bisect %.2f | terms m %.1f a %.1f\n", tj, tb / J, tw / J, tbi / J,
           ttm / J, tta / J);
    printf("walk-test histogram (1, 2, 3-4, 5-8, 9-16, 17-32, 33-64, 65+):");
    for (long h : hist_walk) printf(" %ld", h);
    printf("\n");
    if (out) {
        FILE* f = fopen(out, "wb");
        fwrite(rec.data(), sizeof(double), rec.size(), f);
        fclose(f);
        printf("wrote %zu jobs to %s\n", rec.size() / 9, out);
    }
    return 0;
}
