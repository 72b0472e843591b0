// Routing: river network + unit-hydrograph (UHG) aggregation of cell discharge
// (core/routing.h, region_model.h:906-949).
//
// The reference builds a routing::model on every river query and convolves each
// cell's avg_discharge with the cell's UHG (routing.h:326-345), sums the cell
// outputs per river (local_inflow :347-360), recursively adds the upstream
// rivers' outputs (upstream_inflow :362-376) and convolves the total with the
// river's own UHG (output_m3s :378-386).
//
// MI355X design: convolution is linear, so the per-cell convolutions of all cells
// sharing (river, UHG) collapse to ONE convolution of their summed discharge.
// The engine reduces avg_discharge over each (river, UHG) group on the device
// (shyft_hip_routing_group_sums, HBM-bound, 8 B per cell-step) and evaluates the
// group and river convolutions level by level through the network on the device
// (shyft_hip_route, kernels/routing.hip). This header holds the host-side pieces:
// the river network bookkeeping and the UHG weights. Results equal the reference
// up to the order of floating-point additions.
#pragma once
#include <cmath>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../detmath/detmath.h"
#include "time_series.hpp"

namespace shyft_hip::host {

inline bool valid_routing_id(int64_t rid) { return rid > 0; }  // routing.h:80

struct uhg_parameter {  // routing.h:70-76
    double velocity = 1.0, alpha = 7.0, beta = 0.0;
    uhg_parameter() = default;
    uhg_parameter(double v, double a, double b) : velocity(v), alpha(a), beta(b) {}
};

// boost::math::gamma_distribution<double>(alpha, 1): pdf and quantile (the functions
// make_uhg_from_gamma calls, routing.h:399-421), full double precision.
inline double gamma_pdf(double alpha, double x) {
    if (x < 0 || !(alpha > 0)) throw std::domain_error("gamma pdf: invalid argument");
    if (x == 0) {
        if (alpha > 1) return 0.0;
        if (alpha == 1) return 1.0;
        throw std::overflow_error("gamma pdf: pole at x = 0");
    }
    return std::exp((alpha - 1) * std::log(x) - x - std::lgamma(alpha));
}
inline double gamma_quantile(double alpha, double p) {
    // P(alpha, x) = p by bracketing + bisection to the last representable bit (monotone in x)
    double lo = 0.0, hi = std::max(1.0, alpha);
    while (detmath::gamma_p(alpha, hi) < p) hi *= 2;
    for (int it = 0; it < 2000 && lo < hi; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (mid <= lo || mid >= hi) break;
        if (detmath::gamma_p(alpha, mid) < p) lo = mid;
        else hi = mid;
    }
    return hi;
}

// make_uhg_from_gamma (routing.h:399-421)
inline std::vector<double> make_uhg_from_gamma(int n_steps, double alpha, double base) {
    std::vector<double> r;
    if (n_steps > 1) {
        r.reserve(n_steps);
        double s = 0.0;
        const double x_max = gamma_quantile(alpha, 0.99);
        const double d = x_max / double(n_steps);
        for (int i = 0; i < n_steps; ++i) {
            const double x = d * i;
            const double y = std::max(0.0, gamma_pdf(alpha, x) + base);
            s += y;
            r.push_back(y);
        }
        if (s > 0.0)
            for (auto& y : r) y /= s;
        else
            for (auto& y : r) y = 1 / double(n_steps);
    }
    if (r.empty()) r.push_back(1.0);
    return r;
}

// number of UHG steps from a routing distance (routing.h:119-123, :326-330)
inline int uhg_steps(double distance, double velocity, utctimespan dt) {
    const double steps = (distance / velocity) / to_seconds(dt);
    return int(steps + 0.5);
}

struct river {  // routing.h:94-124
    int64_t id = 0;
    int64_t downstream_id = 0;
    double downstream_distance = 0.0;
    uhg_parameter parameter;
    river() = default;
    river(int64_t i, int64_t ds_id, double ds_dist, const uhg_parameter& p)
        : id(i), downstream_id(ds_id), downstream_distance(ds_dist), parameter(p) {}
    std::vector<double> uhg(utctimespan dt) const {
        return make_uhg_from_gamma(uhg_steps(downstream_distance, parameter.velocity, dt), parameter.alpha, parameter.beta);
    }
};

// river_network (routing.h:140-233)
struct river_network {
    std::map<int64_t, river> rid_map;

    void check_rid(int64_t rid, bool must_exist = true) const {
        if (!valid_routing_id(rid)) throw std::runtime_error("valid river|routing id must be >0");
        if (must_exist && rid_map.find(rid) == rid_map.end())
            throw std::runtime_error(std::string("the supplied river|routing id is not registered/does not exist, id=") +
                                     std::to_string(rid));
    }
    bool network_contains_directed_cycle() const {
        std::map<int64_t, bool> not_visited;
        for (const auto& kv : rid_map) not_visited[kv.first] = false;
        for (const auto& kv : rid_map) {
            auto visited = not_visited;
            visited[kv.first] = true;
            auto ds = kv.second.downstream_id;
            while (valid_routing_id(ds)) {
                if (visited[ds]) return true;
                visited[ds] = true;
                ds = rid_map.find(ds)->second.downstream_id;
            }
        }
        return false;
    }
    river_network& add(const river& r) {
        check_rid(r.id, false);
        if (rid_map.find(r.id) != rid_map.end()) throw std::runtime_error("the supplied river id is already registered");
        if (r.id == r.downstream_id)
            throw std::runtime_error("the supplied river.downstream.id should not point to self (cycle!)");
        if (valid_routing_id(r.downstream_id) && rid_map.find(r.downstream_id) == rid_map.end())
            throw std::runtime_error(
                "the river.downstream.id does not yet exist in the network, please downstream river-segments first");
        rid_map[r.id] = r;
        if (network_contains_directed_cycle()) {
            rid_map.erase(r.id);
            throw std::runtime_error("adding this river caused circular reference");
        }
        return *this;
    }
    void remove_by_id(int64_t rid) {
        check_rid(rid);
        for (auto i : upstreams_by_id(rid)) rid_map[i].downstream_id = 0;
        rid_map.erase(rid);
    }
    const river& river_by_id(int64_t rid) const {
        check_rid(rid);
        return rid_map.find(rid)->second;
    }
    river& river_by_id(int64_t rid) {
        check_rid(rid);
        return rid_map[rid];
    }
    std::vector<int64_t> upstreams_by_id(int64_t rid) const {
        check_rid(rid);
        std::vector<int64_t> r;
        for (const auto& kv : rid_map)
            if (kv.second.downstream_id == rid) r.push_back(kv.first);
        return r;
    }
    std::vector<int64_t> all_upstreams_by_id(int64_t rid) const {
        auto r = upstreams_by_id(rid);
        const size_t n = r.size();
        for (size_t i = 0; i < n; ++i)
            for (auto x : all_upstreams_by_id(r[i])) r.push_back(x);
        return r;
    }
    int64_t downstream_by_id(int64_t rid) const {
        check_rid(rid);
        return rid_map.find(rid)->second.downstream_id;
    }
    void set_downstream_by_id(int64_t rid, int64_t downstream_rid) {
        check_rid(rid);
        if (valid_routing_id(downstream_rid)) check_rid(downstream_rid);
        const int64_t old = rid_map[rid].downstream_id;
        rid_map[rid].downstream_id = downstream_rid;
        if (network_contains_directed_cycle()) {
            rid_map[rid].downstream_id = old;
            throw std::runtime_error("connection would create a cycle, not allowed");
        }
    }
};

// cells sharing a river and a UHG: q = sum of their avg_discharge [T] (device-reduced)
struct uhg_group {
    int64_t rid = 0;
    std::vector<double> w;
    std::vector<double> q;
};

}  // namespace shyft_hip::host
