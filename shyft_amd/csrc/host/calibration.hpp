// Calibration over the MI355X region engine: the reference's model_calibration::optimizer
// (core/model_calibration.h:217-899), its goal functions (core/time_series.h:2198-2450) and the
// search algorithms it drives (core/sceua_optimizer.cpp, core/dream_optimizer.cpp; dlib's
// find_min_bobyqa / find_min_global for optimize / optimize_global).
//
// What is MI355X-specific: every goal-function evaluation is a device run_cells over the calculated
// catchments, and wherever the search algorithm evaluates several parameter vectors that do not depend
// on each other's results (SCE-UA's initial population, DREAM's initial chains, the trust-region
// method's interpolation/geometry sets, the global search's sampling rounds), those vectors go to the
// device as ONE parameter-ensemble launch (shyft_hip_ensemble_run: lanes = calculated cells x members)
// and the catchment sums of all members come back from one segmented reduction. The goal value of a
// member is bit-identical to the value of a sequential run with the same vector (same kernel arithmetic
// per lane, same fixed-order catchment reduction), so batching changes wall time, never results.
//
// Random streams: sceua and dream draw from std::default_random_engine through
// uniform_real_distribution<double>(0,1), default seeded per call, exactly as the reference
// (sceua_optimizer.h:64-70, dream_optimizer.h:56-62); built with the same libstdc++ the sequences
// are the reference's. Batching never reorders draws: all draws of a batch happen before it is evaluated,
// in the reference's order, and evaluation consumes no draws.
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <functional>
#include <limits>
#include <numeric>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "region_model.hpp"

namespace shyft_hip::host {

// ---- target specification (model_calibration.h:217-330) -----------------------------------------------------------
enum target_spec_calc_type : int { NASH_SUTCLIFFE = 0, KLING_GUPTA = 1, ABS_DIFF = 2, RMSE = 3 };
enum target_property_type : int {
    DISCHARGE = 0,
    SNOW_COVERED_AREA = 1,
    SNOW_WATER_EQUIVALENT = 2,
    ROUTED_DISCHARGE = 3,
    CELL_CHARGE = 4
};

struct target_specification {
    point_ts ts;                              // the observed series (any point time axis)
    std::vector<int64_t> catchment_indexes;   // catchment ids whose sum should match ts
    int64_t river_id = 0;                     // ROUTED_DISCHARGE: the river
    double scale_factor = 1.0;
    target_spec_calc_type calc_mode = NASH_SUTCLIFFE;
    target_property_type catchment_property = DISCHARGE;
    double s_r = 1.0, s_a = 1.0, s_b = 1.0;  // Kling-Gupta weights
    std::string uid;

    target_specification() = default;
    target_specification(const point_ts& ts_, std::vector<int64_t> cids, double scale,
                         target_spec_calc_type mode = NASH_SUTCLIFFE, double sr = 1.0, double sa = 1.0, double sb = 1.0,
                         target_property_type prop = DISCHARGE, std::string uid_ = "")
        : ts(ts_), catchment_indexes(std::move(cids)), scale_factor(scale), calc_mode(mode), catchment_property(prop),
          s_r(sr), s_a(sa), s_b(sb), uid(std::move(uid_)) {}
    target_specification(const point_ts& ts_, int64_t rid, double scale, target_spec_calc_type mode = NASH_SUTCLIFFE,
                         double sr = 1.0, double sa = 1.0, double sb = 1.0, std::string uid_ = "")
        : ts(ts_), river_id(rid), scale_factor(scale), calc_mode(mode), catchment_property(ROUTED_DISCHARGE), s_r(sr),
          s_a(sa), s_b(sb), uid(std::move(uid_)) {}
    bool operator==(const target_specification& x) const {
        return catchment_indexes == x.catchment_indexes && catchment_property == x.catchment_property &&
               river_id == x.river_id;
    }
};

// ---- goal functions (time_series.h:2301-2450), on already-resampled value vectors ------------------------------------
namespace goal {

inline double nan() { return std::numeric_limits<double>::quiet_NaN(); }

// nash_sutcliffe_goal_function: 1 - NSE over the pairs where both values are finite
inline double nash_sutcliffe(const std::vector<double>& obs, const std::vector<double>& sim) {
    if (obs.size() != sim.size() || obs.empty())
        throw std::runtime_error("nash_sutcliffe needs equal sized ts accessors with elements >1");
    double err2 = 0.0, mean = 0.0;
    size_t count = 0;
    for (size_t i = 0; i < obs.size(); ++i)
        if (std::isfinite(obs[i]) && std::isfinite(sim[i])) {
            const double d = obs[i] - sim[i];
            err2 += d * d;
            mean += obs[i];
            ++count;
        }
    mean /= double(count);
    double var2 = 0.0;
    for (size_t i = 0; i < obs.size(); ++i)
        if (std::isfinite(obs[i]) && std::isfinite(sim[i])) {
            const double d = obs[i] - mean;
            var2 += d * d;
        }
    return err2 / var2;
}

// rmse_goal_function: sqrt(mean squared error) / mean(obs)
inline double rmse(const std::vector<double>& obs, const std::vector<double>& sim) {
    if (obs.size() != sim.size() || obs.empty())
        throw std::runtime_error("rmse needs equal sized ts accessors with elements >1");
    double err2 = 0.0, mean = 0.0;
    size_t count = 0;
    for (size_t i = 0; i < obs.size(); ++i)
        if (std::isfinite(obs[i]) && std::isfinite(sim[i])) {
            const double d = obs[i] - sim[i];
            err2 += d * d;
            mean += obs[i];
            ++count;
        }
    mean /= double(count);
    return count ? std::sqrt(err2 / double(count)) / mean : nan();
}

// dlib::running_scalar_covariance<double> (dlib/statistics/statistics.h; third-party, not vendored under the
// reference): running sums; unbiased (n-1) covariance and variances, negative round-off variance clamped to 0.
struct running_scalar_covariance {
    double sum_xy = 0, sum_x = 0, sum_y = 0, sum_xx = 0, sum_yy = 0, n = 0;
    void add(double x, double y) {
        sum_xy += x * y;
        sum_x += x;
        sum_y += y;
        sum_xx += x * x;
        sum_yy += y * y;
        n += 1;
    }
    double mean_x() const { return sum_x / n; }
    double mean_y() const { return sum_y / n; }
    double covariance() const { return 1 / (n - 1) * (sum_xy - sum_y * sum_x / n); }
    double variance_x() const {
        const double v = 1 / (n - 1) * (sum_xx - sum_x * sum_x / n);
        return v >= 0 ? v : 0;
    }
    double variance_y() const {
        const double v = 1 / (n - 1) * (sum_yy - sum_y * sum_y / n);
        return v >= 0 ? v : 0;
    }
    double stddev_x() const { return std::sqrt(variance_x()); }
    double stddev_y() const { return std::sqrt(variance_y()); }
    double correlation() const { return covariance() / std::sqrt(variance_x() * variance_y()); }
};

// kling_gupta_goal_function: EDs = sqrt((s_r(r-1))^2 + (s_a(a-1))^2 + (s_b(b-1))^2), a = mean ratio, b = std ratio
inline double kling_gupta(const std::vector<double>& obs, const std::vector<double>& sim, double s_r, double s_a,
                          double s_b) {
    running_scalar_covariance rs;
    for (size_t i = 0; i < obs.size(); ++i)
        if (std::isfinite(obs[i]) && std::isfinite(sim[i])) rs.add(obs[i], sim[i]);
    const double qo = rs.mean_x(), qs = rs.mean_y(), us = rs.stddev_y(), uo = rs.stddev_x(), r = rs.correlation();
    double a = qs / qo, b = us / uo;
    if (!std::isfinite(a)) a = 1.0;
    if (!std::isfinite(b)) b = 1.0;
    const double eds2 = (s_r != 0.0 ? std::pow(s_r * (r - 1), 2) : 0.0) + (s_a != 0.0 ? std::pow(s_a * (a - 1), 2) : 0.0) +
                        (s_b != 0.0 ? std::pow(s_b * (b - 1), 2) : 0.0);
    return std::sqrt(eds2);
}

inline double abs_diff_sum(const std::vector<double>& obs, const std::vector<double>& sim) {
    double s = 0.0;
    for (size_t i = 0; i < obs.size(); ++i)
        if (std::isfinite(obs[i]) && std::isfinite(sim[i])) s += std::fabs(obs[i] - sim[i]);
    return s;
}

inline double abs_diff_sum_scaled(const std::vector<double>& obs, const std::vector<double>& sim,
                                  const std::vector<double>& scale) {
    const double scale_eps = 1e-20;
    double s = 0.0;
    for (size_t i = 0; i < obs.size(); ++i)
        if (std::isfinite(obs[i]) && std::isfinite(sim[i]) && std::isfinite(scale[i]) && std::fabs(scale[i]) > scale_eps)
            s += std::fabs(obs[i] - sim[i]) / scale[i];
    return s;
}

}  // namespace goal

// average_accessor<S, TA>(src, target time axis).value(i) for every interval of `axis`
// (time_series.h:2033-2072): NaN for intervals starting at/after the source's end.
inline std::vector<double> average_onto(const point_ts& src, const point_ts& axis) {
    const size_t n = axis.size();
    std::vector<double> r(n);
    const bool linear = src.fx == POINT_INSTANT_VALUE;
    const utctime src_end = src.total_period().end;
    size_t last_idx = 0;
    for (size_t i = 0; i < n; ++i) {
        const utctime s = axis.t[i], e = i + 1 < n ? axis.t[i + 1] : axis.t_end;
        r[i] = s >= src_end ? goal::nan() : average_value(src, utcperiod(s, e), last_idx, linear);
    }
    return r;
}
// max_abs_average_accessor (time_series.h:2198-2265): max of the averages of max(0, v) and max(0, -v)
inline std::vector<double> max_abs_average_onto(const point_ts& src, const point_ts& axis) {
    point_ts pos(src), neg(src);
    for (size_t i = 0; i < src.v.size(); ++i)
        if (std::isfinite(src.v[i])) {
            pos.v[i] = std::max(0.0, src.v[i]);
            neg.v[i] = std::max(0.0, -src.v[i]);
        }
    auto a = average_onto(pos, axis), b = average_onto(neg, axis);
    for (size_t i = 0; i < a.size(); ++i) a[i] = std::max(a[i], b[i]);
    return a;
}

// ---- search algorithms (all minimise f over the unit box [0,1]^n of scaled parameters) ------------------------------
struct scaled_fx {
    std::function<double(const std::vector<double>&)> one;
    std::function<std::vector<double>(const std::vector<std::vector<double>>&)> many;
    double operator()(const std::vector<double>& x) const { return one(x); }
    std::vector<double> operator()(const std::vector<std::vector<double>>& xs) const { return many(xs); }
};

enum class sceua_state : int {
    not_started = -1,
    searching,
    finished_fx_convergence,
    finished_x_convergence,
    finished_max_iterations,
    finished_user_request,
    finished_max_time
};

// Shuffled Complex Evolution (Duan et al. 1993) as implemented by sceua::find_min / evolve / mutate
// (core/sceua_optimizer.cpp:10-286): p = 5 complexes of m = 2n+1 points, sub-complexes of q = n+1 points,
// alpha = 1, beta = 2n+1 evolution steps per complex and shuffle. Reproduced including its quirks:
// the reflection is judged against the last *selected* point bf[q-1] (not the sorted worst), mutate's
// bounding box skips parameter 0 (j starts at 1), and the returned x is sample[0] of the unsorted pool.
class sceua_search {
    mutable std::default_random_engine gen_;
    mutable std::uniform_real_distribution<double> u01_{0.0, 1.0};
    double random01() const { return u01_(gen_); }
    void random_x(size_t n, double* x, const double* lo, const double* hi) const {
        for (size_t i = 0; i < n; ++i) x[i] = lo[i] + random01() * (hi[i] - lo[i]);
    }
    static std::vector<size_t> sorted_index(const std::vector<double>& v, size_t n) {  // construct_sorted_pivot_table
        std::vector<size_t> ix(n);
        std::iota(ix.begin(), ix.end(), size_t(0));
        std::sort(ix.begin(), ix.end(), [&](size_t a, size_t b) { return v[a] < v[b]; });
        return ix;
    }
    // new point uniformly inside the bounding box of the complex (mutate, sceua_optimizer.cpp:262-277)
    void mutate(const std::vector<std::vector<double>>& ax, std::vector<double>& x) const {
        const size_t n = x.size();
        std::vector<double> lo(ax[0]), hi(ax[0]);
        for (size_t i = 1; i < ax.size(); ++i)
            for (size_t j = 1; j < n; ++j) {
                if (ax[i][j] < lo[j]) lo[j] = ax[i][j];
                if (ax[i][j] > hi[j]) hi[j] = ax[i][j];
            }
        random_x(n, x.data(), lo.data(), hi.data());
    }
    // competitive complex evolution of one complex (evolve, sceua_optimizer.cpp:124-260)
    void evolve(std::vector<std::vector<double>>& ax, std::vector<double>& af, const scaled_fx& f,
                const std::vector<double>& lo, const std::vector<double>& hi, std::vector<double>& x,
                size_t& evaluations) const {
        const size_t m = ax.size(), n = x.size(), q = n + 1, beta = 2 * n + 1;
        std::vector<double> cp(m);
        for (size_t i = 0; i < m; ++i) {  // triangular selection probabilities, best point most likely
            const double pp = (2.0 * (m + 1.0 - (i + 1.0))) / (m * (m + 1.0));
            cp[i] = i > 0 ? cp[i - 1] + pp : pp;
        }
        std::vector<std::vector<double>> bx(q), sbx(q);
        std::vector<double> bf(q), sbf(q), g(n);
        std::vector<size_t> ll(q), sll(q);
        std::vector<char> selected(m);
        for (size_t k = 0; k < beta; ++k) {
            std::fill(selected.begin(), selected.end(), 0);
            size_t nsel = 0;
            while (nsel < q) {  // draw q distinct points of the complex by cp
                const double ff = random01();
                for (size_t i = 0; i < m; ++i)
                    if (ff <= cp[i] && !selected[i]) {
                        bx[nsel] = ax[i];
                        bf[nsel] = af[i];
                        ll[nsel] = i;
                        selected[i] = 1;
                        ++nsel;
                        break;
                    }
            }
            // alpha = 1 evolution step of the sub-complex
            auto ib = sorted_index(bf, q);
            for (size_t i = 0; i < q; ++i) {
                sbx[i] = bx[ib[i]];
                sll[i] = ll[ib[i]];
                sbf[i] = bf[ib[i]];
            }
            bool out_of_box = false;
            for (size_t i = 0; i < n; ++i) {
                g[i] = 0.0;
                for (size_t j = 0; j + 1 < q; ++j) g[i] = g[i] + sbx[j][i] / (q - 1);  // centroid of the q-1 best
                x[i] = 2.0 * g[i] - sbx[q - 1][i];                                     // reflection of the worst
                if (x[i] < lo[i] || x[i] > hi[i]) out_of_box = true;
            }
            if (out_of_box) mutate(ax, x);
            double fx = f(x);
            ++evaluations;
            if (!(fx < bf[q - 1])) {
                for (size_t i = 0; i < n; ++i) x[i] = (g[i] + sbx[q - 1][i]) / 2.0;  // contraction
                fx = f(x);
                ++evaluations;
                if (!(fx < bf[q - 1])) {
                    mutate(ax, x);
                    fx = f(x);
                    ++evaluations;
                }
            }
            sbf[q - 1] = fx;
            sbx[q - 1] = x;
            ll = sll;
            bf = sbf;
            bx = sbx;
            for (size_t i = 0; i < q; ++i) {  // back into the complex, which is then re-sorted
                ax[ll[i]] = bx[i];
                af[ll[i]] = bf[i];
            }
            auto ia = sorted_index(af, m);
            std::vector<std::vector<double>> sax(m);
            std::vector<double> saf(m);
            for (size_t i = 0; i < m; ++i) {
                saf[i] = af[ia[i]];
                sax[i] = ax[ia[i]];
            }
            af.swap(saf);
            ax.swap(sax);
        }
    }

  public:
    sceua_state find_min(const std::vector<double>& lo, const std::vector<double>& hi, std::vector<double>& x,
                         double& fx_min, const scaled_fx& f, double fx_eps, double fx_sol_min, double fx_sol_max,
                         const std::vector<double>& x_eps, size_t max_iterations, bool batch) const {
        const double eps = 1e-10;
        const size_t n = x.size(), m = 2 * n + 1, p = 5, npt = p * m;
        size_t evaluations = 0;
        std::vector<std::vector<double>> sample(npt), ssample(npt);
        std::vector<double> fv(npt), sf(npt);
        // step 1: the start point plus npt-1 uniform points (all drawn before any evaluation)
        sample[0] = x;
        for (size_t i = 1; i < npt; ++i) {
            random_x(n, x.data(), lo.data(), hi.data());
            sample[i] = x;
        }
        if (batch) {
            fv = f(sample);
        } else {
            for (size_t i = 0; i < npt; ++i) fv[i] = f(sample[i]);
        }
        evaluations += npt;
        auto resort = [&] {
            auto ix = sorted_index(fv, npt);
            for (size_t i = 0; i < npt; ++i) {
                sf[i] = fv[ix[i]];
                ssample[i] = sample[ix[i]];
            }
        };
        resort();
        sceua_state state = sceua_state::searching;
        std::vector<std::vector<double>> ax(m);
        std::vector<double> af(m);
        while (state == sceua_state::searching) {
            for (size_t c = 0; c < p; ++c) {  // partition into complexes: complex c takes ranks c, c+p, c+2p, ...
                for (size_t j = 0; j < m; ++j) {
                    ax[j] = ssample[j * p + c];
                    af[j] = sf[j * p + c];
                }
                evolve(ax, af, f, lo, hi, x, evaluations);
                for (size_t j = 0; j < m; ++j) {
                    sample[j * p + c] = ax[j];
                    fv[j * p + c] = af[j];
                }
            }
            resort();
            x = sample[0];
            fx_min = sf[0];
            if (fx_sol_min <= fx_min && fx_min < fx_sol_max) {
                state = sceua_state::finished_fx_convergence;
            } else if (2.0 * std::fabs(sf[0] - sf[npt - 1]) / (std::fabs(sf[0]) + std::fabs(sf[npt - 1]) + eps) < fx_eps) {
                state = sceua_state::finished_fx_convergence;
            } else {
                size_t frozen = 0;
                for (size_t i = 0; i < n; ++i)
                    if (std::fabs(ssample[0][i] - ssample[npt - 1][i]) < x_eps[i]) ++frozen;
                if (frozen == n) state = sceua_state::finished_x_convergence;
                if (evaluations > max_iterations) state = sceua_state::finished_max_iterations;
            }
        }
        return state;
    }
};

// DiffeRential Evolution Adaptive Metropolis (Vrugt et al. 2009) as dream::find_max
// (core/dream_optimizer.cpp:10-570): n_chains = n parameters, 4 crossover values with burn-in adaptation,
// outlier-chain reset by the inter-quartile rule, Gelman-Rubin convergence (R <= 1.2) on the last half of
// the chains since the last reset. Maximises g (the caller passes -goal).
class dream_search {
    mutable bool stored_normal_ = false;
    mutable double stored_normal_value_ = 0.0;
    mutable std::default_random_engine gen_;
    mutable std::uniform_real_distribution<double> u01_{0.0, 1.0};
    double random01() const { return u01_(gen_); }
    double random11() const { return random01() * 2.0 - 1.0; }
    // Marsaglia polar method, second variate kept for the next call (dream::std_norm)
    double std_norm() const {
        double u1 = 0, u2 = 0, s = 0;
        if (stored_normal_) {
            stored_normal_ = false;
            return stored_normal_value_;
        }
        do {
            u1 = random11();
            u2 = random11();
            s = u1 * u1 + u2 * u2;
        } while (s >= 1.0 || s == 0.0);
        s = std::sqrt(-2.0 * std::log(s) / s);
        stored_normal_value_ = u1 * s;
        stored_normal_ = true;
        return u2 * s;
    }
    double normal(double mean, double sd) const { return std_norm() * sd + mean; }

    // crossover-probability distribution from the jump distances per cr (dream::update_cr_dist)
    static void update_cr(std::vector<double>& cr_m, const std::vector<int>& cr_l, const std::vector<double>& cr_d) {
        const size_t ncr = cr_l.size();
        bool all_pos = true;
        for (size_t i = 0; all_pos && i < ncr; ++i)
            if (cr_d[i] == 0) all_pos = false;
        if (all_pos) {
            double sum = 0;
            for (size_t i = 0; i < ncr; ++i) {
                cr_m[i] = cr_d[i] / cr_l[i];
                sum += cr_m[i];
            }
            for (size_t i = 0; i < ncr; ++i) cr_m[i] /= sum;
        } else {
            for (size_t i = 0; i < ncr; ++i) cr_m[i] = 1.0 / ncr;
        }
    }

    // proposal for chain I from delta pairs of other chains (dream::generate_candidate_parameters)
    void propose(std::vector<double>& cand, size_t I, size_t N, size_t d, double cr, size_t& d_eff,
                 const std::vector<std::vector<double>>& states) const {
        size_t delta = 1 + size_t(std::floor(3 * random01()));
        delta = std::min(delta, (N - 1) / 2);
        delta = std::min(delta, size_t(3));
        size_t R[6];
        for (size_t k = 0; k < 2 * delta; ++k) {
            R[k] = I;
            while (R[k] == I) {
                R[k] = std::min(N - 1, size_t(std::floor(random01() * N)));
                for (size_t j = 0; j < k; ++j)
                    if (R[k] == R[j]) R[k] = I;
            }
        }
        std::fill(cand.begin(), cand.end(), 0.0);
        for (size_t k = 0; k < delta; ++k)
            for (size_t i = 0; i < d; ++i) cand[i] += states[R[2 * k]][i] - states[R[2 * k + 1]][i];
        const double keep = -std::numeric_limits<double>::max();
        d_eff = d;
        for (size_t i = 0; i < d; ++i)
            if (random01() >= cr) {
                --d_eff;
                cand[i] = keep;
            }
        const double gamma = random01() < 0.2 ? 1.0 : 2.38 / std::sqrt(2.0 * delta * d_eff);
        const double b = 0.05, sd = 0.001;
        for (size_t i = 0; i < d; ++i) {
            if (cand[i] == keep) {
                cand[i] = states[I][i];
            } else {
                const double e = random11() * b;
                cand[i] = states[I][i] + (1 + e) * gamma * cand[i] + normal(0, sd);
            }
        }
    }

    // outlier chains by the inter-quartile rule on the last-half mean log density (dream::check_for_outlier_chain)
    static bool outliers(const std::vector<std::vector<double>>& prob, size_t reset, std::vector<double>& omega,
                         double& limit) {
        const size_t n_it = prob.size(), nc = omega.size();
        const size_t start = reset + (n_it - reset) / 2;
        if (start > n_it) return false;
        const size_t len = n_it - start;
        if (len < 5) return false;
        std::fill(omega.begin(), omega.end(), 0.0);
        for (size_t i = start; i < n_it; ++i)
            for (size_t j = 0; j < nc; ++j) omega[j] += prob[i][j];
        for (size_t i = 0; i < nc; ++i) omega[i] /= len;
        auto s = omega;
        std::sort(s.begin(), s.end());
        limit = s[nc / 4] - 2 * (s[3 * nc / 4] - s[nc / 4]);
        for (size_t i = 0; i < nc; ++i)
            if (omega[i] < limit) return true;
        return false;
    }

    // Gelman-Rubin sqrt(R) of parameter p over the last half since reset (dream::get_gr_convergence)
    static double gelman_rubin(const std::vector<std::vector<std::vector<double>>>& states, size_t n_it, size_t nc,
                               size_t np, size_t reset, size_t p) {
        if (n_it < 1 || nc < 1 || np < 1) return -1.0;
        const size_t start = reset + (n_it - reset) / 2;
        if (start > n_it) return -1.0;
        const size_t len = n_it - start;
        if (len < 5) return -1.0;
        std::vector<double> cm(nc), cv(nc);
        const double m = double(nc), n = double(len);
        double mcm = 0, mcv = 0, vcm = 0, vcv = 0, msqcm = 0;
        for (size_t i = 0; i < nc; ++i) {
            cm[i] = cv[i] = 0.0;
            for (size_t j = start; j < n_it; ++j) {
                const double v = states[j][i][p];
                cm[i] += v;
                cv[i] += std::pow(v, 2);
            }
            cm[i] /= n;
            cv[i] /= n;
            cv[i] -= std::pow(cm[i], 2);
            if (cv[i] < 0) return -2.0;
            cv[i] *= n / (n - 1);
            mcm += cm[i];
            mcv += cv[i];
            vcm += std::pow(cm[i], 2);
            vcv += std::pow(cv[i], 2);
            msqcm += std::pow(cm[i], 2);
        }
        mcm /= m;
        msqcm /= m;
        mcv /= m;
        vcm /= m;
        vcm -= std::pow(mcm, 2);
        if (vcm < 0) return -2.0;
        vcm *= m / (m - 1);
        vcv /= m;
        vcv -= std::pow(mcv, 2);
        if (vcv < 0) return -2.0;
        vcv *= m / (m - 1);
        const double target_var = mcv * (n - 1) / n + vcm;
        const double v_hat = target_var + vcm / m;
        double cov_vm = 0, cov_vsqm = 0;
        for (size_t i = 0; i < m; ++i) {
            cov_vm += (cv[i] - mcv) * (cm[i] - mcm);
            cov_vsqm += (cv[i] - mcv) * (std::pow(cm[i], 2) - msqcm);
        }
        cov_vm /= m;
        cov_vsqm /= m;
        const double var_v_hat = std::pow((n - 1.0) / n, 2.0) * vcv / m +
                                 std::pow((m + 1.0) / (m * n), 2.0) * 2 * std::pow(vcm * n, 2) / (m - 1.0) +
                                 2 * (m + 1.0) * (n - 1.0) / (m * std::pow(n, 2.0)) * n / m * (cov_vsqm - 2 * mcm * cov_vm);
        const double df = 2 * std::pow(v_hat, 2) / var_v_hat;
        if (df <= 2.0) return -2.0;
        const double sqrt_r = std::sqrt(v_hat / mcv * df / (df - 2.0));
        if (!std::isfinite(sqrt_r)) return -2.0;
        return sqrt_r;
    }

  public:
    // g maximised; x in/out in [0,1]^n; returns the best g found
    double find_max(const scaled_fx& g, std::vector<double>& x, size_t /*max_iterations: unused, as the reference*/,
                    bool batch) const {
        const size_t np = x.size();
        double best = -std::numeric_limits<double>::max();
        if (np < 1) throw std::runtime_error("dream::find_max(): n_parameters must be >0 ");
        const size_t nc = np, ncr = 4, min_burnins = 100, burnin_inc = 10;
        size_t last_reset = 0, n_burnins = min_burnins, n_accepted = 0;
        std::vector<std::vector<std::vector<double>>> all_states;
        std::vector<std::vector<double>> all_prob;
        std::vector<std::vector<double>> states(nc, std::vector<double>(np));
        std::vector<double> prob(nc), cand(np, 0.0), omega(nc, 0.0), cr_d(ncr, 0.0), cr_m(ncr, 0.0), xvar(np, 0.0);
        std::vector<int> cr_l(ncr, 0);
        double limit = 0;
        for (size_t i = 0; i < nc; ++i)
            for (size_t p = 0; p < np; ++p) states[i][p] = random01();
        if (batch) {
            prob = g(states);
        } else {
            for (size_t i = 0; i < nc; ++i) prob[i] = g(states[i]);
        }
        for (size_t i = 0; i < nc; ++i)
            if (prob[i] > best) {
                best = prob[i];
                x = states[i];
            }
        all_states.push_back(states);
        all_prob.push_back(prob);
        update_cr(cr_m, cr_l, cr_d);
        bool burnin = true, converged = false;
        size_t it = 0;
        while (!converged) {
            ++it;
            bool have_outliers = false;
            if (burnin && outliers(all_prob, last_reset, omega, limit)) {
                have_outliers = true;
                last_reset = it;
            } else {
                converged = true;
                double avg = 0;
                for (size_t i = 0; i < np; ++i) {
                    const double grc = gelman_rubin(all_states, all_states.size(), nc, np, last_reset, i);
                    if (grc > 1.2 || grc < 0) converged = false;
                    if (grc < 0) {
                        avg = grc;
                        break;
                    }
                    avg += grc / np;
                }
                if (burnin && (avg > 1.5 || avg < 0)) n_burnins = std::max(n_burnins, it + burnin_inc);
                if (burnin) converged = false;
                if (converged) break;
            }
            for (size_t p = 0; p < np; ++p) {  // inter-chain variance per parameter
                double mean = 0.0;
                xvar[p] = 0.0;
                for (size_t c = 0; c < nc; ++c) {
                    mean += states[c][p];
                    xvar[p] += std::pow(states[c][p], 2);
                }
                mean /= nc;
                xvar[p] /= nc;
                xvar[p] -= std::pow(mean, 2);
            }
            for (size_t c = 0; c < nc; ++c) {
                double jump = 0;
                if (burnin && have_outliers && omega[c] < limit) {  // restart the outlier at the best state
                    for (size_t i = 0; i < np; ++i) {
                        jump += std::pow(states[c][i] - x[i], 2) / xvar[i];
                        states[c][i] = x[i];
                    }
                    prob[c] = best;
                    n_burnins = it + min_burnins;
                } else {
                    const double u = random01();
                    double psum = 0;
                    size_t icr = 0;
                    while (icr < ncr) {
                        psum += cr_m[icr];
                        if (psum > u || icr == ncr - 1) break;
                        ++icr;
                    }
                    const double cr = double(icr + 1) / double(ncr);
                    size_t d_eff = 0;
                    propose(cand, c, nc, np, cr, d_eff, states);
                    bool reject = false;
                    for (size_t i = 0; i < np; ++i)
                        if (cand[i] < 0 || cand[i] > 1) {
                            reject = true;
                            break;
                        }
                    if (!reject) {
                        const double cp = g(cand);
                        if (std::exp(cp - prob[c]) < random01()) {
                            // a posteriori rejected: the chain repeats its state
                        } else {
                            ++n_accepted;
                            prob[c] = cp;
                            for (size_t i = 0; i < np; ++i) {
                                jump += std::pow(states[c][i] - cand[i], 2) / xvar[i];
                                states[c][i] = cand[i];
                            }
                            if (prob[c] > best) {
                                best = prob[c];
                                x = states[c];
                            }
                        }
                    }
                    if (burnin) {
                        cr_l[icr]++;
                        cr_d[icr] += jump;
                    }
                }
            }
            if (burnin) {
                if (it >= n_burnins) {
                    if (n_accepted > nc * 20) burnin = false;
                    else n_burnins = n_burnins + burnin_inc;
                }
                update_cr(cr_m, cr_l, cr_d);
            }
            all_states.push_back(states);
            all_prob.push_back(prob);
        }
        if (!converged) throw std::runtime_error("dream::find_max: did not converge");
        return best;
    }
};

// optimize(): dlib::find_min_bobyqa (Powell's BOBYQA; dlib is third-party and not vendored under the
// reference) is not restated. In its place: a bound-constrained quadratic-model trust-region method with
// the same contract -- start x0 in [0,1]^n, 2n+1 initial interpolation points x0 and x0 +- rho_begin e_i
// (one device ensemble launch), radius shrinking from rho_begin to rho_end, at most max_eval evaluations.
// The model is a full quadratic fitted by regularised least squares to the stored points near the
// incumbent; the step minimises it over the box (bounds intersected with the infinity-norm trust region)
// by projected gradient descent. Geometry is restored with a batched +-rho coordinate stencil when a
// step fails. Parity with the reference: results, not traces (test_region_model_stacks.py:408-418).
class box_trust_region {
  public:
    struct result {
        std::vector<double> x;
        double f = 0;
        size_t evaluations = 0;
    };
    static result minimize(const scaled_fx& f, std::vector<double> x0, double rho_begin, double rho_end, size_t max_eval) {
        const size_t n = x0.size();
        for (auto& v : x0) v = std::min(1.0, std::max(0.0, v));
        std::vector<std::vector<double>> X;
        std::vector<double> F;
        size_t evals = 0;
        auto add_batch = [&](std::vector<std::vector<double>> pts) {
            if (pts.empty()) return;
            if (evals + pts.size() > max_eval) pts.resize(max_eval > evals ? max_eval - evals : 0);
            if (pts.empty()) return;
            auto fv = f(pts);
            for (size_t i = 0; i < pts.size(); ++i) {
                X.push_back(pts[i]);
                F.push_back(fv[i]);
            }
            evals += pts.size();
        };
        auto best_ix = [&] {
            size_t b = 0;
            for (size_t i = 1; i < F.size(); ++i)
                if (F[i] < F[b] || (!std::isfinite(F[b]) && std::isfinite(F[i]))) b = i;
            return b;
        };
        auto stencil = [&](const std::vector<double>& c, double rho) {
            std::vector<std::vector<double>> pts;
            for (size_t i = 0; i < n; ++i)
                for (int s : {+1, -1}) {
                    auto y = c;
                    double v = c[i] + s * rho;
                    if (v > 1.0) v = c[i] - 2 * rho >= 0.0 ? c[i] - 2 * rho : 0.0;
                    if (v < 0.0) v = c[i] + 2 * rho <= 1.0 ? c[i] + 2 * rho : 1.0;
                    y[i] = v;
                    bool dup = false;
                    for (const auto& p : pts) dup = dup || p == y;
                    if (!dup && y != c) pts.push_back(y);
                }
            return pts;
        };
        {
            auto init = stencil(x0, rho_begin);
            init.insert(init.begin(), x0);
            add_batch(init);
        }
        double rho = rho_begin;
        const size_t nq = n + n * (n + 1) / 2;  // gradient + upper Hessian coefficients
        while (evals < max_eval && rho >= rho_end) {
            const size_t b = best_ix();
            const std::vector<double> xb = X[b];
            const double fb = F[b];
            // least-squares quadratic fit on the points nearest the incumbent
            std::vector<size_t> near;
            for (size_t i = 0; i < X.size(); ++i) {
                if (i == b || !std::isfinite(F[i])) continue;
                double d = 0;
                for (size_t j = 0; j < n; ++j) d = std::max(d, std::fabs(X[i][j] - xb[j]));
                if (d <= 4 * rho && d > 0) near.push_back(i);
            }
            std::vector<double> g(n, 0.0), H(n * n, 0.0);
            bool model_ok = near.size() >= n;
            if (model_ok) {
                std::vector<double> A(nq * nq, 0.0), r(nq, 0.0), phi(nq);
                for (size_t i : near) {
                    size_t k = 0;
                    for (size_t j = 0; j < n; ++j) phi[k++] = (X[i][j] - xb[j]) / rho;
                    for (size_t j = 0; j < n; ++j)
                        for (size_t l = j; l < n; ++l) {
                            const double sj = (X[i][j] - xb[j]) / rho, sl = (X[i][l] - xb[l]) / rho;
                            phi[k++] = (j == l ? 0.5 : 1.0) * sj * sl;
                        }
                    const double y = F[i] - fb;
                    for (size_t a = 0; a < nq; ++a) {
                        r[a] += phi[a] * y;
                        for (size_t c = 0; c < nq; ++c) A[a * nq + c] += phi[a] * phi[c];
                    }
                }
                double tr = 0;
                for (size_t a = 0; a < nq; ++a) tr += A[a * nq + a];
                for (size_t a = n; a < nq; ++a) A[a * nq + a] += 1e-8 * (tr / nq + 1e-300);  // minimal-curvature tie break
                for (size_t a = 0; a < n; ++a) A[a * nq + a] += 1e-12 * (tr / nq + 1e-300);
                std::vector<double> theta;
                model_ok = solve_spd(A, r, nq, theta);
                if (model_ok) {
                    size_t k = 0;
                    for (size_t j = 0; j < n; ++j) g[j] = theta[k++] / rho;
                    for (size_t j = 0; j < n; ++j)
                        for (size_t l = j; l < n; ++l) {
                            H[j * n + l] = H[l * n + j] = theta[k++] / (rho * rho);
                        }
                }
            }
            std::vector<double> s(n, 0.0);
            double pred = 0;
            if (model_ok) {
                std::vector<double> lo(n), hi(n);
                for (size_t j = 0; j < n; ++j) {
                    lo[j] = std::max(-rho, -xb[j]);
                    hi[j] = std::min(rho, 1.0 - xb[j]);
                }
                double L = 0;
                for (double h : H) L += h * h;
                L = std::sqrt(L) + 1e-12;
                double gn = 0;
                for (double v : g) gn += v * v;
                if (gn > 0) L = std::max(L, std::sqrt(gn) / rho);
                auto mval = [&](const std::vector<double>& z) {
                    double v = 0;
                    for (size_t j = 0; j < n; ++j) {
                        v += g[j] * z[j];
                        for (size_t l = 0; l < n; ++l) v += 0.5 * z[j] * H[j * n + l] * z[l];
                    }
                    return v;
                };
                for (int it = 0; it < 500; ++it) {
                    std::vector<double> grad(g);
                    for (size_t j = 0; j < n; ++j)
                        for (size_t l = 0; l < n; ++l) grad[j] += H[j * n + l] * s[l];
                    double moved = 0;
                    for (size_t j = 0; j < n; ++j) {
                        const double v = std::min(hi[j], std::max(lo[j], s[j] - grad[j] / L));
                        moved = std::max(moved, std::fabs(v - s[j]));
                        s[j] = v;
                    }
                    if (moved < 1e-6 * rho) break;
                }
                pred = -mval(s);
            }
            double step = 0;
            for (double v : s) step = std::max(step, std::fabs(v));
            if (!model_ok || !(pred > 0) || step < 0.1 * rho_end) {
                // the model cannot propose a descent step: refresh the stencil at this radius, then shrink
                auto pts = stencil(xb, rho);
                std::vector<std::vector<double>> fresh;
                for (const auto& p : pts) {
                    bool have = false;
                    for (const auto& q : X) {
                        double d = 0;
                        for (size_t j = 0; j < n; ++j) d = std::max(d, std::fabs(q[j] - p[j]));
                        if (d < 0.25 * rho) { have = true; break; }
                    }
                    if (!have) fresh.push_back(p);
                }
                const double before = F[best_ix()];
                add_batch(fresh);
                if (fresh.empty() || !(F[best_ix()] < before)) rho *= 0.5;
                continue;
            }
            std::vector<double> xn(n);
            for (size_t j = 0; j < n; ++j) xn[j] = std::min(1.0, std::max(0.0, xb[j] + s[j]));
            add_batch({xn});
            if (evals >= max_eval && X.back() != xn) break;
            const double fn = F.back();
            const double ratio = (fb - fn) / pred;
            if (ratio > 0.75 && step >= 0.9 * rho) rho = std::min(2 * rho, 0.5);
            else if (!(ratio >= 0.1)) rho *= 0.5;
        }
        const size_t b = best_ix();
        return result{X[b], F[b], evals};
    }

  private:
    // Cholesky solve of a symmetric positive definite system (false if not SPD)
    static bool solve_spd(std::vector<double> A, const std::vector<double>& r, size_t n, std::vector<double>& x) {
        for (size_t j = 0; j < n; ++j) {
            double d = A[j * n + j];
            for (size_t k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
            if (!(d > 0)) return false;
            d = std::sqrt(d);
            A[j * n + j] = d;
            for (size_t i = j + 1; i < n; ++i) {
                double v = A[i * n + j];
                for (size_t k = 0; k < j; ++k) v -= A[i * n + k] * A[j * n + k];
                A[i * n + j] = v / d;
            }
        }
        x.assign(n, 0.0);
        for (size_t i = 0; i < n; ++i) {
            double v = r[i];
            for (size_t k = 0; k < i; ++k) v -= A[i * n + k] * x[k];
            x[i] = v / A[i * n + i];
        }
        for (size_t i = n; i-- > 0;) {
            double v = x[i];
            for (size_t k = i + 1; k < n; ++k) v -= A[k * n + i] * x[k];
            x[i] = v / A[i * n + i];
        }
        return true;
    }
};

// ---- the optimizer (model_calibration.h:404-899) ---------------------------------------------------------------------
template <class M>
class optimizer {
  public:
    using parameter_t = std::vector<double>;
    parameter_t parameter_lower_bound, parameter_upper_bound;
    std::vector<parameter_t> parameters_trace;  // every evaluated parameter vector, in evaluation order
    std::vector<double> goal_fn_trace;          // and its goal-function value
    M& model;
    std::vector<target_specification> targets;
    // MI355X: evaluate independent parameter vectors as one device ensemble launch (bit-identical goals)
    bool batch_evaluation = true;
    size_t max_batch_members = 512;  // members per ensemble launch (bounds device memory: members x cells x T)

    optimizer(M& m, const std::vector<target_specification>& targets_, const parameter_t& p_min, const parameter_t& p_max)
        : model(m), targets(targets_) {
        set_parameter_ranges(p_min, p_max);
    }
    explicit optimizer(M& m) : model(m) {
        parameter_lower_bound = model.get_region_parameter();
        parameter_upper_bound = model.get_region_parameter();
        prepare_optimize();
    }

    bool active_parameter(size_t i) const {
        return std::fabs(parameter_upper_bound.at(i) - parameter_lower_bound.at(i)) > activate_limit;
    }
    void set_target_specification(const std::vector<target_specification>& t, const parameter_t& lo, const parameter_t& hi) {
        targets = t;
        parameter_lower_bound = lo;
        parameter_upper_bound = hi;
        prepare_optimize();
    }
    void set_parameter_ranges(const parameter_t& p_min, const parameter_t& p_max) {
        parameter_lower_bound = p_min;
        parameter_upper_bound = p_max;
    }
    void establish_initial_state_from_model() { model.get_states(model.initial_state); }
    void set_verbose_level(int level) { verbose_ = level; }
    void reset_states() { model.revert_to_initial_state(); }
    std::vector<double> get_initial_state(size_t i) {
        auto_initial_state_check();
        return model.initial_state.at(i);
    }
    int trace_size() const { return int(goal_fn_trace.size()); }
    double trace_goal_fn(int i) const { return goal_fn_trace.at(size_t(i)); }
    parameter_t trace_parameter(int i) const { return parameters_trace.at(size_t(i)); }

    // snow collection, calculation filter and initial state as the targets need them (prepare_optimize :511-556)
    void prepare_optimize() {
        n_catchments_ = model.number_of_catchments();
        std::vector<int64_t> cids;
        model.set_snow_sca_swe_collection(-1, false);
        for (const auto& t : targets) {
            cids.insert(cids.end(), t.catchment_indexes.begin(), t.catchment_indexes.end());
            if (t.catchment_property == SNOW_WATER_EQUIVALENT || t.catchment_property == SNOW_COVERED_AREA)
                for (auto c : t.catchment_indexes) model.set_snow_sca_swe_collection(c, true);
            if (t.catchment_property == ROUTED_DISCHARGE)
                for (auto c : model.get_catchment_feeding_to_river(t.river_id)) cids.push_back(c);
        }
        std::sort(cids.begin(), cids.end());
        cids.erase(std::unique(cids.begin(), cids.end()), cids.end());
        for (auto c : cids)
            if (model.has_catchment_parameter(c)) throw std::runtime_error("Cannot calibrate on local parameters.");
        model.set_catchment_calculation_filter(cids);
        auto_initial_state_check();
        parameters_trace.clear();
        goal_fn_trace.clear();
    }

    // ---- search entry points; p is the full parameter vector, the result too
    parameter_t optimize(const parameter_t& p, size_t max_n_evaluations = 1500, double tr_start = 0.1,
                         double tr_stop = 1.0e-5) {
        prepare_optimize();
        p_expanded_ = p;
        auto res = box_trust_region::minimize(scaled(), to_scaled(reduce(p)), tr_start, tr_stop, max_n_evaluations);
        return expand(from_scaled(res.x));
    }
    parameter_t optimize_global(const parameter_t& p, size_t max_n_evaluations, double max_seconds, double solver_eps) {
        prepare_optimize();
        p_expanded_ = p;
        auto x = global_search(to_scaled(reduce(p)), max_n_evaluations, max_seconds, solver_eps);
        return expand(from_scaled(x));
    }
    parameter_t optimize_sceua(const parameter_t& p, size_t max_n_evaluations = 1500, double x_eps = 0.0001,
                               double y_eps = 1.0e-5) {
        prepare_optimize();
        p_expanded_ = p;
        auto xs = to_scaled(reduce(p));  // min_sceua (model_calibration.h:169-190)
        const size_t n = xs.size();
        std::vector<double> lo(n, 0.0), hi(n, 1.0), xe(n, x_eps);
        double y = 0;
        sceua_search opt;
        auto st = opt.find_min(lo, hi, xs, y, scaled(), y_eps, -1.0, -2.0, xe, max_n_evaluations, batch_evaluation);
        auto r = expand(from_scaled(xs));
        if (!(st == sceua_state::finished_fx_convergence || st == sceua_state::finished_x_convergence ||
              st == sceua_state::finished_max_iterations))
            throw std::runtime_error("sceua: terminated before convergence or max iterations");
        return r;
    }
    parameter_t optimize_dream(const parameter_t& p, size_t max_n_evaluations = 1500) {
        prepare_optimize();
        p_expanded_ = p;
        auto xs = to_scaled(reduce(p));  // min_dream (model_calibration.h:137-147): dream maximises -goal
        auto f = scaled();
        scaled_fx neg{[f](const std::vector<double>& x) { return -f(x); },
                      [f](const std::vector<std::vector<double>>& xs_) {
                          auto v = f(xs_);
                          for (auto& a : v) a = -a;
                          return v;
                      }};
        dream_search dr;
        dr.find_max(neg, xs, max_n_evaluations, batch_evaluation);
        return expand(from_scaled(xs));
    }

    // ---- goal function
    double calculate_goal_function(const parameter_t& full) {
        p_expanded_ = full;
        return run(reduce(full));
    }
    // MI355X addition: goal functions of many full parameter vectors (ensemble launches, bit-identical to
    // calling calculate_goal_function on each in turn; traced in the same order)
    std::vector<double> calculate_goal_functions(const std::vector<parameter_t>& fulls) {
        if (fulls.empty()) return {};
        p_expanded_ = fulls.back();
        return run_full_batch(fulls);  // each member with its own full vector (inactive parameters included)
    }
    // scaled-space evaluation (operator() of the reference, called by the search algorithms)
    double operator()(const std::vector<double>& p_s) { return run(from_scaled(p_s)); }

    std::vector<double> to_scaled(const std::vector<double>& rp) const {
        const auto lo = reduce(p_min()), hi = reduce(p_max());
        std::vector<double> r;
        for (size_t i = 0; i < rp.size(); ++i) r.push_back((rp[i] - lo[i]) / (hi[i] - lo[i]));
        return r;
    }
    std::vector<double> from_scaled(const std::vector<double>& ps) const {
        const auto lo = reduce(p_min()), hi = reduce(p_max());
        std::vector<double> r;
        for (size_t i = 0; i < ps.size(); ++i) r.push_back((hi[i] - lo[i]) * ps[i] + lo[i]);
        return r;
    }

  private:
    static constexpr double activate_limit = 0.000001;
    int verbose_ = 0;
    size_t n_catchments_ = 0;
    parameter_t p_expanded_;

    const parameter_t& p_min() const {
        if (parameter_lower_bound.empty()) throw std::runtime_error("Parameter ranges are not set");
        return parameter_lower_bound;
    }
    const parameter_t& p_max() const {
        if (parameter_upper_bound.empty()) throw std::runtime_error("Parameter ranges are not set");
        return parameter_upper_bound;
    }
    bool is_active(size_t i) const { return std::fabs(p_max().at(i) - p_min().at(i)) > activate_limit; }
    std::vector<double> reduce(const parameter_t& fp) const {
        std::vector<double> r;
        for (size_t i = 0; i < fp.size(); ++i)
            if (is_active(i)) r.push_back(fp[i]);
        return r;
    }
    parameter_t expand(const std::vector<double>& rp) const {
        parameter_t r;
        size_t j = 0;
        for (size_t i = 0; i < p_expanded_.size(); ++i) r.push_back(is_active(i) ? rp.at(j++) : p_expanded_[i]);
        return r;
    }
    void auto_initial_state_check() {
        if (model.initial_state.size() != model.size()) establish_initial_state_from_model();
    }

    scaled_fx scaled() {
        return scaled_fx{[this](const std::vector<double>& x) { return run(from_scaled(x)); },
                         [this](const std::vector<std::vector<double>>& xs) {
                             std::vector<parameter_t> fulls;
                             for (const auto& x : xs) fulls.push_back(expand(from_scaled(x)));
                             return run_full_batch(fulls);
                         }};
    }

    // per-run catchment aggregates the targets read (one member of an ensemble, or the model's own run)
    struct run_sums {
        std::function<const double*(size_t cix)> discharge, charge, sca_area, swe_area;
    };
    bool need(target_property_type p) const {
        for (const auto& t : targets)
            if (t.catchment_property == p) return true;
        return false;
    }

    // model_calibration.h:830-897 from the sums of one run
    double goal_of(const run_sums& s) {
        const size_t T = model.time_axis.size();
        double goal_value = 0.0, scale_sum = 0.0;
        std::vector<double> area(n_catchments_, 0.0);
        if (need(SNOW_COVERED_AREA) || need(SNOW_WATER_EQUIVALENT))
            for (size_t i = 0; i < model.size(); ++i) {  // extract_area_ts_property's area sums, cell order
                const size_t c = model.catchment_ix_of_cell(i);
                if (model.is_calculated_by_catchment_ix(c)) area[c] += model.cells_geo()[i].area();
            }
        for (const auto& t : targets) {
            std::vector<double> sum(T, 0.0);
            switch (t.catchment_property) {
                case DISCHARGE:
                case CELL_CHARGE: {
                    for (auto cid : t.catchment_indexes) {
                        const double* v = (t.catchment_property == DISCHARGE ? s.discharge : s.charge)(model.cix_from_cid(cid));
                        for (size_t i = 0; i < T; ++i) sum[i] += v[i];
                    }
                    break;
                }
                case SNOW_COVERED_AREA:
                case SNOW_WATER_EQUIVALENT: {
                    double a_sum = 0.0;
                    for (auto cid : t.catchment_indexes) {
                        const size_t c = model.cix_from_cid(cid);
                        const double* v = (t.catchment_property == SNOW_COVERED_AREA ? s.sca_area : s.swe_area)(c);
                        const double inv = 1 / area[c];
                        for (size_t i = 0; i < T; ++i) sum[i] += (v[i] * inv) * area[c];
                        a_sum += area[c];
                    }
                    const double inv = 1 / a_sum;
                    for (auto& x : sum) x *= inv;
                    break;
                }
                case ROUTED_DISCHARGE:
                    sum = model.river_output_flow_m3s(t.river_id);
                    break;
            }
            const point_ts prop(model.time_axis, std::move(sum), POINT_AVERAGE_VALUE);
            const std::vector<double> sim = average_onto(prop, t.ts);
            double partial;
            if (t.calc_mode == NASH_SUTCLIFFE) partial = goal::nash_sutcliffe(t.ts.v, sim);
            else if (t.calc_mode == KLING_GUPTA) partial = goal::kling_gupta(t.ts.v, sim, t.s_r, t.s_a, t.s_b);
            else if (t.calc_mode == RMSE) partial = goal::rmse(t.ts.v, sim);
            else if (t.catchment_property == CELL_CHARGE)
                partial = goal::abs_diff_sum_scaled(t.ts.v, sim, max_abs_average_onto(prop, t.ts));
            else partial = goal::abs_diff_sum(t.ts.v, sim);
            if (std::isfinite(partial)) {
                scale_sum += t.scale_factor;
                goal_value += t.scale_factor * partial;
            } else if (verbose_ > 0) {
                std::printf("warning: goal-function %d: evaluated as nan\n", int(t.catchment_property));
            }
        }
        return goal_value / scale_sum;
    }

    void trace(const parameter_t& p, double g) {
        parameters_trace.push_back(p);
        goal_fn_trace.push_back(g);
        if (verbose_ > 0) {
            std::printf("%g : ParameterVector(", g);
            for (size_t i = 0; i < p.size(); ++i) std::printf(i + 1 < p.size() ? "%g, " : "%g", p[i]);
            std::printf(")\n");
        }
    }

    // one sequential evaluation (optimizer::run, model_calibration.h:830-899)
    double run(const std::vector<double>& rp) {
        const parameter_t p = expand(rp);
        return run_full(p);
    }
    double run_full(const parameter_t& p) {
        model.set_region_parameter(p);
        reset_states();
        model.run_cells();
        std::vector<std::vector<double>> q, ch, sca, swe;
        if (need(DISCHARGE)) q = model.catchment_sums(0);
        if (need(CELL_CHARGE)) ch = model.catchment_sums(1);
        if (need(SNOW_COVERED_AREA)) sca = model.catchment_area_sums(2);
        if (need(SNOW_WATER_EQUIVALENT)) swe = model.catchment_area_sums(3);
        run_sums s{[&](size_t c) { return q[c].data(); }, [&](size_t c) { return ch[c].data(); },
                   [&](size_t c) { return sca[c].data(); }, [&](size_t c) { return swe[c].data(); }};
        const double g = goal_of(s);
        trace(p, g);
        return g;
    }
    // a batch of full parameter vectors: device ensembles where the targets allow, else one by one
    std::vector<double> run_full_batch(const std::vector<parameter_t>& fulls) {
        std::vector<double> r;
        if (!batch_evaluation || fulls.size() < 2 || need(ROUTED_DISCHARGE)) {
            for (const auto& p : fulls) r.push_back(run_full(p));
            return r;
        }
        const bool snow = need(SNOW_COVERED_AREA) || need(SNOW_WATER_EQUIVALENT);
        const size_t C = n_catchments_, T = model.time_axis.size();
        for (size_t b = 0; b < fulls.size(); b += max_batch_members) {
            const size_t e = std::min(fulls.size(), b + max_batch_members);
            std::vector<parameter_t> members(fulls.begin() + b, fulls.begin() + e);
            reset_states();
            model.ensemble_run(members, snow);
            std::vector<double> q, ch, sca, swe;
            if (need(DISCHARGE)) q = model.ensemble_sums(0, false);
            if (need(CELL_CHARGE)) ch = model.ensemble_sums(1, false);
            if (need(SNOW_COVERED_AREA)) sca = model.ensemble_sums(2, true);
            if (need(SNOW_WATER_EQUIVALENT)) swe = model.ensemble_sums(3, true);
            for (size_t k = 0; k < members.size(); ++k) {
                const size_t o = k * C * T;
                run_sums s{[&](size_t c) { return q.data() + o + c * T; }, [&](size_t c) { return ch.data() + o + c * T; },
                           [&](size_t c) { return sca.data() + o + c * T; }, [&](size_t c) { return swe.data() + o + c * T; }};
                const double g = goal_of(s);
                trace(members[k], g);
                r.push_back(g);
            }
        }
        // the reference leaves the last evaluated vector as the region parameter (parameter_accessor.set)
        model.set_region_parameter(fulls.back());
        return r;
    }

    // optimize_global: dlib::find_min_global (MaxLIPO + trust region; third-party, not restated). In its
    // place, rounds of one device ensemble each -- stratified uniform samples and samples around the
    // incumbent -- alternating with the trust-region method from the incumbent, until max_n_evaluations
    // or max_seconds; solver_eps is the local method's final radius. Deterministic (fixed seed).
    std::vector<double> global_search(std::vector<double> x0, size_t max_eval, double max_seconds, double solver_eps) {
        const size_t n = x0.size();
        const auto t_start = std::chrono::steady_clock::now();
        auto elapsed = [&] {
            return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
        };
        std::mt19937_64 rng(20251015);
        std::uniform_real_distribution<double> u(0.0, 1.0);
        std::normal_distribution<double> z(0.0, 1.0);
        auto f = scaled();
        std::vector<double> best = x0;
        double fbest = std::numeric_limits<double>::infinity();
        size_t evals = 0;
        double sigma = 0.2;
        const size_t batch = std::max<size_t>(8 * (n + 1), 32);
        while (evals < max_eval && elapsed() < max_seconds) {
            const size_t nb = std::min(batch, max_eval - evals);
            std::vector<std::vector<double>> pts;
            if (evals == 0) pts.push_back(x0);
            for (size_t k = pts.size(); k < nb; ++k) {  // half stratified uniform, half around the incumbent
                std::vector<double> y(n);
                for (size_t j = 0; j < n; ++j) {
                    if (k % 2 == 0 || !std::isfinite(fbest)) y[j] = (double((k / 2 + j * 7) % nb) + u(rng)) / double(nb);
                    else y[j] = std::min(1.0, std::max(0.0, best[j] + sigma * z(rng)));
                }
                pts.push_back(y);
            }
            auto fv = f(pts);
            evals += pts.size();
            for (size_t k = 0; k < pts.size(); ++k)
                if (fv[k] < fbest) {
                    fbest = fv[k];
                    best = pts[k];
                }
            if (evals >= max_eval || elapsed() >= max_seconds) break;
            const size_t local_budget = std::min(max_eval - evals, 30 * (n + 1));
            auto loc = box_trust_region::minimize(f, best, std::max(sigma / 2, 4 * solver_eps), std::max(solver_eps, 1e-9),
                                                  local_budget);
            evals += loc.evaluations;
            if (loc.f < fbest) {
                fbest = loc.f;
                best = loc.x;
            }
            sigma = std::max(sigma * 0.5, 1e-3);
        }
        return best;
    }
};

}  // namespace shyft_hip::host
