// Analysis (CPU): the pt_ss_k job solver's two rewrites of the bisection (device/ptssk_dev.h ss_sca_rel_red_body),
// replayed against the oracle's boost::math::tools::bisect restatement (oracle/src/ptssk.hpp) on recorded jobs:
//  1. the grouped rounds: the midpoints of the next D levels evaluated at once (D = 2: groups of 4 lanes; D = 3: 8),
//     then the sequential loop replayed over them;
//  2. ss_zero_sign: the midpoint's sign without the pdfs' divisions where it is certain, and (r06) without the exps
//     where their arguments decide it -- each such decision also checked against the full evaluation.
// Both must end on the oracle's bracket, bit for bit, for every job.
// jobs: tools/mb/ptssk_jobs -o jobs.bin (u, n, nu_a, alpha, ... per row of 9 doubles)
// build: g++ -O2 -std=c++17 -mfma -ffp-contract=off -o tools/mb/ptssk_group_emu tools/mb/ptssk_group_emu.cpp
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../oracle/src/ptssk.hpp"

using namespace oracle;

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: ptssk_group_emu jobs.bin\n"); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<double> J;
    double row[9];
    while (fread(row, sizeof(double), 9, f) == 9) J.insert(J.end(), row, row + 9);
    fclose(f);
    const size_t nr = J.size() / 9;
    long bad_group[4] = {0}, bad_sign = 0, fast = 0, slow = 0, checked = 0, exp_skipped = 0, bad_skip = 0, flog_decided = 0, flog_fallback = 0, bad_flog = 0;
    for (size_t r = 0; r < nr; ++r) {
        const double* q = &J[9 * r];
        const unsigned long u = (unsigned long)q[0], n = (unsigned long)q[1];
        const double nu_a = q[2], alpha = q[3];
        const double nu_m = ((double)u / n) * nu_a, theta = 1.0 / alpha;
        const skaugen::gamma_dist g_m{nu_m, theta}, g_a{nu_a, theta};
        const double lg_m = OLGAMMA(nu_m), lg_a = OLGAMMA(nu_a);
        auto zf = [&](double x) { return g_m.pdf(x) - g_a.pdf(x); };
        auto zs = [&](double x) {  // ss_zero_sign (x > 0 here)
            const double z = x / theta, lz = OLOG(z);
            const double A = nu_m * lz - z - lg_m, B = nu_a * lz - z - lg_a;
            const bool in_range = z >= 0x1p-30 && z <= 0x1p30 && theta >= 0x1p-30 && theta <= 0x1p30;
            double skip = 2.0;  // the exp-argument decision (r06), checked against the full evaluation below
            if (A < -745.1332191019412 && B < -745.1332191019412) {
                skip = 0.0;
            } else if (in_range) {
                const double hi = A > B ? A : B;
                if (hi >= -660.0 && hi <= 660.0) {
                    if (B - A > 0x1p-40) skip = -1.0;
                    else if (A - B > 0x1p-40) skip = 1.0;
                }
            }
            const double ea = OEXP(A), eb = OEXP(B);
            double full;
            const double LO = 0x1p-960, HI = 0x1p960;
            if (ea == 0 && eb == 0) full = 0.0;
            else if (in_range && eb >= LO && eb <= HI && eb > ea * (1.0 + 0x1p-48)) full = -1.0;
            else if (in_range && ea >= LO && ea <= HI && ea > eb * (1.0 + 0x1p-48)) full = 1.0;
            else full = ea / z / theta - eb / z / theta;
            {  // (r06) the single-precision-log decision, with logf perturbed by up to 4 float ulps either way
                const double za = x * alpha;
                if (za >= 0x1p-29 && za <= 0x1p29 && theta >= 0x1p-30 && theta <= 0x1p30) {
                    for (int pert = -4; pert <= 4; pert += 4) {
                        float l2 = std::log2((float)za);
                        for (int q = 0; q < (pert < 0 ? -pert : pert); ++q) l2 = std::nextafter(l2, pert < 0 ? -1e30f : 1e30f);
                        const double lza = (double)l2 * 0.6931471805599453;
                        const double alz = std::fabs(lza);
                        const double Aa = nu_m * lza - za - lg_m, Ba = nu_a * lza - za - lg_a;
                        const double S = nu_a * (alz + 1.0) + za + std::fabs(lg_m) + std::fabs(lg_a) + 1.0;
                        const double e = 0x1p-17 * nu_a * (1.0 + alz) + 0x1p-46 * S;
                        double dec = 2.0;
                        if (e < 1.0) {
                            if (Aa + e < -745.2 && Ba + e < -745.2) dec = 0.0;
                            else {
                                const double hi = Aa > Ba ? Aa : Ba;
                                if (hi >= -650.0 && hi <= 650.0) {
                                    const double d = Ba - Aa;
                                    if (d > 0x1p-40 + e) dec = -1.0;
                                    else if (-d > 0x1p-40 + e) dec = 1.0;
                                }
                            }
                        }
                        if (pert == 0) { if (dec != 2.0) ++flog_decided; else ++flog_fallback; }
                        if (dec != 2.0 && dec != (skip != 2.0 ? skip : full)) ++bad_flog;
                    }
                }
            }
            if (skip != 2.0) {
                ++exp_skipped;
                if (skip != full) ++bad_skip;
                return skip;
            }
            if (full == 1.0 || full == -1.0 || full == 0.0) ++fast; else ++slow;
            return full;
        };
        double lower = g_m.mean();
        uintmax_t bi = ~0ull;
        const double upper = special::brent_find_minima(zf, 0.0, g_a.mean(), 2, bi).first;
        while (g_m.pdf(lower) < g_a.pdf(lower)) lower *= 0.9;
        uintmax_t mi = 100;
        const auto ref = skaugen::bisect(zf, lower, upper, 10, mi);
        const double fmin0 = zf(lower), fmax0 = zf(upper);
        if (fmin0 == 0 || fmax0 == 0 || lower >= upper || fmin0 * fmax0 >= 0) continue;
        ++checked;
        const double eps = 0x1p-9;
        auto sgn = [](double v) { return v > 0 ? 1 : (v < 0 ? -1 : 0); };
        for (int mode = 0; mode < 3; ++mode) {  // 0: sign surrogate, sequential; 1: D = 2; 2: D = 3
            double bmin = lower, bmax = upper, fmin = fmin0;
            int count = 97;
            auto go_on = [&]() { return count && !(std::fabs(bmin - bmax) <= eps * std::min(std::fabs(bmin), std::fabs(bmax))); };
            if (mode == 0) {
                while (go_on()) {
                    const double mid = (bmin + bmax) / 2, fmid = zs(mid);
                    if (mid == bmax || mid == bmin) break;
                    if (fmid == 0) { bmin = bmax = mid; break; }
                    if (sgn(fmid) * sgn(fmin) < 0) bmax = mid; else { bmin = mid; fmin = fmid; }
                    --count;
                }
                if (bmin != ref.first || bmax != ref.second) ++bad_sign;
                continue;
            }
            const int D = mode + 1, P = (1 << D) - 1;
            bool more = go_on();
            while (more) {
                double fk[8];
                for (int k = 0; k < P; ++k) {  // lane k's point: heap node k + 1
                    const int h = k + 1, depth = 31 - __builtin_clz((unsigned)h);
                    double lo = bmin, hi = bmax;
                    for (int b = depth - 1; b >= 0; --b) {
                        const double m2 = (lo + hi) / 2;
                        if ((h >> b) & 1) lo = m2; else hi = m2;
                    }
                    fk[k] = zs((lo + hi) / 2);
                }
                int node = 1;
                for (int lev = 0; lev < D; ++lev) {
                    if (lev > 0 && !go_on()) { more = false; break; }
                    const double mid = (bmin + bmax) / 2, fmid = fk[node - 1];
                    if (mid == bmax || mid == bmin) { more = false; break; }
                    if (fmid == 0) { bmin = bmax = mid; more = false; break; }
                    if (sgn(fmid) * sgn(fmin) < 0) { bmax = mid; node = 2 * node; }
                    else { bmin = mid; fmin = fmid; node = 2 * node + 1; }
                    --count;
                }
                if (more) more = go_on();
            }
            if (bmin != ref.first || bmax != ref.second) ++bad_group[D];
        }
    }
    printf("jobs %zu, bisections checked %ld: differing brackets: sign surrogate %ld, D=2 %ld, D=3 %ld; "
           "surrogate evaluations decided by the exp arguments %ld (differing from the exps' decision: %ld), by the exps "
           "without the divisions %ld, with the divisions %ld\n",
           nr, checked, bad_sign, bad_group[2], bad_group[3], exp_skipped, bad_skip, fast, slow);
    printf("single-precision-log decisions: %ld decided, %ld left to the full path, %ld differing (logf exact and "
           "perturbed by 4 float ulps either way)\n", flog_decided, flog_fallback, bad_flog);
    return (bad_sign || bad_group[2] || bad_group[3] || bad_skip || bad_flog) ? 1 : 0;
}
