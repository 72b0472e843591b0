// ORACLE — test infrastructure only (see common.hpp header).
//
// routing.hpp: routing::model (core/routing.h:239-387) restated literally: every
// routed cell's avg_discharge is convolved with the cell's own UHG
// (cell_output_m3s :332-345), the cell outputs are summed per river in cell order
// (local_inflow :347-360), the upstream rivers' outputs are added recursively
// (upstream_inflow :362-376) and the total is convolved with the river's UHG
// (output_m3s :378-386). make_uhg_from_gamma (:399-421) needs boost's
// gamma_distribution quantile and pdf (boost 1.68, not under /root/reference):
// restated here as bisection of P(alpha, x) = 0.99 to the last bit and
// pdf = x^(a-1) e^-x / Gamma(a), with this build's elementary functions.
#pragma once
#include <algorithm>
#include <cmath>
#include <map>
#include <stdexcept>
#include <vector>

#include "common.hpp"
#include "methods.hpp"

namespace oracle {
namespace routing {

inline double gamma_quantile(double alpha, double p) {
    double lo = 0.0, hi = std::max(1.0, alpha);
    while (special::gamma_p(alpha, hi) < p) hi *= 2;
    for (int it = 0; it < 2000; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        if (special::gamma_p(alpha, mid) < p) lo = mid; else hi = mid;
    }
    return hi;
}

inline double gamma_pdf(double alpha, double x) {
    if (x == 0) return alpha > 1 ? 0.0 : (alpha == 1 ? 1.0 : INFINITY);
    return OEXP((alpha - 1) * OLOG(x) - x - OLGAMMA(alpha));
}

inline std::vector<double> make_uhg_from_gamma(int n_steps, double alpha, double base) {
    std::vector<double> r;
    if (n_steps > 1) {
        double s = 0.0;
        const double x_max = gamma_quantile(alpha, 0.99);
        const double d = x_max / double(n_steps);
        for (int i = 0; i < n_steps; ++i) {
            const double y = std::max(0.0, gamma_pdf(alpha, d * i) + base);
            s += y;
            r.push_back(y);
        }
        if (s > 0.0) for (auto& y : r) y /= s;
        else for (auto& y : r) y = 1 / double(n_steps);
    }
    if (r.empty()) r.push_back(1.0);
    return r;
}

inline int uhg_steps(double distance, double velocity, int64_t dt_us) {
    return int((distance / velocity) / to_seconds(dt_us) + 0.5);
}

// convolve_w_ts<...>::value with convolve_policy::USE_ZERO (time_series.h:966-974)
inline std::vector<double> convolve(const std::vector<double>& ts, const std::vector<double>& w) {
    std::vector<double> r(ts.size());
    for (size_t i = 0; i < ts.size(); ++i) {
        double v = 0.0;
        for (size_t j = 0; j < w.size(); ++j) v += j <= i ? w[j] * ts[i - j] : 0.0;
        r[i] = v;
    }
    return r;
}

struct river {
    int64_t id, downstream_id;
    double distance, velocity, alpha, beta;
};

struct cell_route {
    int64_t rid;                 // geo.routing.id
    double distance;             // geo.routing.distance
    double velocity, alpha, beta;  // the cell parameter's routing part
    const double* q;             // avg_discharge [T], element t at q[t*stride]
    size_t stride;
};

struct model {
    std::map<int64_t, river> rivers;
    std::vector<cell_route> cells;
    size_t T;
    int64_t dt_us;

    std::vector<double> local_inflow(int64_t rid) const {
        std::vector<double> r(T, 0.0);
        for (const auto& c : cells) {
            if (c.rid != rid) continue;
            std::vector<double> q(T);
            for (size_t t = 0; t < T; ++t) q[t] = c.q[t * c.stride];
            auto o = convolve(q, make_uhg_from_gamma(uhg_steps(c.distance, c.velocity, dt_us), c.alpha, c.beta));
            for (size_t t = 0; t < T; ++t) r[t] += o[t];
        }
        return r;
    }
    std::vector<double> upstream_inflow(int64_t rid) const {
        std::vector<double> r(T, 0.0);
        for (const auto& kv : rivers)
            if (kv.second.downstream_id == rid) {
                auto o = output(kv.first);
                for (size_t t = 0; t < T; ++t) r[t] += o[t];
            }
        return r;
    }
    std::vector<double> output(int64_t rid) const {
        const river& rv = rivers.at(rid);
        auto w = make_uhg_from_gamma(uhg_steps(rv.distance, rv.velocity, dt_us), rv.alpha, rv.beta);
        auto a = local_inflow(rid);
        auto b = upstream_inflow(rid);
        for (size_t t = 0; t < T; ++t) a[t] += b[t];
        return convolve(a, w);
    }
};

}  // namespace routing
}  // namespace oracle
