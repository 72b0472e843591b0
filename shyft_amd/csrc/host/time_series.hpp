// Host-side time primitives of the region_model drop-in (C++17, no device code).
//
// utctime is int64 microseconds since 1970-01-01Z like the reference's
// std::chrono utctime (core/utctime_utilities.h:29-34). fixed_dt is the
// region_model's time axis (core/time_axis.h:74-115). point_ts is the
// geo-located source series of a region environment (core/time_series.h:323-414)
// on a point time axis (core/time_axis.h:255-382), and average_values() is the
// average_accessor step that resamples a source onto the model time axis before
// interpolation (region_model.h:135-145 -> time_series.h:2033-2072 ->
// accumulate_value/average_value time_series.h:202-310).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

namespace shyft_hip::host {

using utctime = int64_t;      // microseconds
using utctimespan = int64_t;  // microseconds
constexpr utctime US = 1000000;
constexpr size_t npos = size_t(-1);
inline double to_seconds(utctimespan dt) { return double(dt) / 1e6; }

struct utcperiod {
    utctime start = 0, end = 0;
    utcperiod() = default;
    utcperiod(utctime s, utctime e) : start(s), end(e) {}
    utctimespan timespan() const { return end - start; }
    bool contains(utctime t) const { return t >= start && t < end; }
    bool valid() const { return start <= end; }
};

// core/time_axis.h:74-115
struct fixed_dt {
    utctime t = 0;
    utctimespan dt = 0;
    size_t n = 0;
    fixed_dt() = default;
    fixed_dt(utctime t0, utctimespan dt_, size_t n_) : t(t0), dt(dt_), n(n_) {}
    size_t size() const { return n; }
    utctime time(size_t i) const {
        if (i < n) return t + utctimespan(i) * dt;
        throw std::out_of_range("fixed_dt.time(i)");
    }
    utcperiod period(size_t i) const {
        if (i < n) return utcperiod(t + utctimespan(i) * dt, t + utctimespan(i + 1) * dt);
        throw std::out_of_range("fixed_dt.period(i)");
    }
    utcperiod total_period() const { return n == 0 ? utcperiod() : utcperiod(t, t + utctimespan(n) * dt); }
    size_t index_of(utctime tx) const {
        if (tx < t || dt == 0) return npos;
        size_t r = size_t((tx - t) / dt);
        return r < n ? r : npos;
    }
    bool operator==(const fixed_dt& o) const { return t == o.t && dt == o.dt && n == o.n; }
};

enum ts_point_fx : int { POINT_INSTANT_VALUE = 0, POINT_AVERAGE_VALUE = 1 };  // time_series.h:53-57

// A point series on a point time axis: points t[0..n) with the last interval ending at t_end.
// A fixed_dt series is stored the same way (t[i] = t0 + i*dt, t_end = t0 + n*dt).
struct point_ts {
    std::vector<utctime> t;
    utctime t_end = 0;
    std::vector<double> v;
    ts_point_fx fx = POINT_AVERAGE_VALUE;

    point_ts() = default;
    point_ts(const fixed_dt& ta, double fill, ts_point_fx f = POINT_AVERAGE_VALUE) : v(ta.size(), fill), fx(f) {
        t.resize(ta.size());
        for (size_t i = 0; i < ta.size(); ++i) t[i] = ta.time(i);
        t_end = ta.total_period().end;
    }
    point_ts(const fixed_dt& ta, std::vector<double> values, ts_point_fx f) : v(std::move(values)), fx(f) {
        if (v.size() != ta.size()) throw std::runtime_error("point_ts: values and time-axis differ in size");
        t.resize(ta.size());
        for (size_t i = 0; i < ta.size(); ++i) t[i] = ta.time(i);
        t_end = ta.total_period().end;
    }
    // point_dt(t, t_end) (time_axis.h:289-303): strictly increasing points, t_end > t.back()
    point_ts(std::vector<utctime> tp, utctime tend, std::vector<double> values, ts_point_fx f)
        : t(std::move(tp)), t_end(tend), v(std::move(values)), fx(f) {
        if (t.size() != v.size()) throw std::runtime_error("point_ts: values and time-axis differ in size");
        for (size_t i = 1; i < t.size(); ++i)
            if (!(t[i - 1] < t[i])) throw std::runtime_error("time_axis::point_dt() needs time-points in increasing order");
        if (!t.empty() && !(t_end > t.back())) throw std::runtime_error("time_axis::point_dt() illegal end-of-axis");
    }
    size_t size() const { return t.size(); }
    utcperiod total_period() const { return t.empty() ? utcperiod() : utcperiod(t.front(), t_end); }
    utctime time(size_t i) const { return t.at(i); }
    double value(size_t i) const { return v.at(i); }
    void set(size_t i, double x) { v.at(i) = x; }
    // point_dt::open_range_index_of (time_axis.h:329-374): lower-bound index, n-1 at/after t_end, npos before t[0]
    size_t open_range_index_of(utctime tx) const {
        const size_t n = t.size();
        if (n == 0) return npos;
        if (tx >= t_end) return n - 1;
        if (tx < t[0]) return npos;
        if (tx >= t.back()) return n - 1;
        return size_t(std::upper_bound(t.begin(), t.end(), tx) - t.begin()) - 1;
    }
    // f(t) of the series: stair-case or linear-between-points (time_series.h:360-380)
    double operator()(utctime tx) const {
        size_t i = open_range_index_of(tx);
        if (i == npos || tx >= t_end) return std::numeric_limits<double>::quiet_NaN();
        if (fx == POINT_INSTANT_VALUE && i + 1 < t.size()) {
            const double a = (v[i + 1] - v[i]) / to_seconds(t[i + 1] - t[i]);
            return v[i] + a * to_seconds(tx - t[i]);
        }
        return v[i];
    }
};

// accumulate_value (time_series.h:202-288), restated for point_ts; the hint is the
// lower-bound index of p.start (hint_based_search specialisation, time_series.h:2273-2285).
inline double accumulate_value(const point_ts& source, const utcperiod& p, size_t& last_idx, utctimespan& tsum,
                               bool linear = true, bool strict_linear_between = true) {
    const double nan = std::numeric_limits<double>::quiet_NaN();
    const size_t n = source.size();
    const bool extrapolate_flat = !linear || (linear && !strict_linear_between);
    if (n == 0) return nan;
    size_t i = source.open_range_index_of(p.start);
    struct pt { utctime t; double v; };
    auto get = [&](size_t k) { return pt{source.t[k], source.v[k]}; };
    pt l{0, nan};
    bool l_finite = false;
    if (i == npos) {
        i = 0;
        last_idx = 0;
        if (strict_linear_between) {
            l = get(i++);
            l_finite = std::isfinite(l.v);
            if (!p.contains(l.t)) return nan;
        }
    }
    double area = 0.0;
    tsum = 0;
    while (true) {
        if (!l_finite) {
            l = get(i++);
            l_finite = std::isfinite(l.v);
            if (i == n) {
                if (l_finite && l.t < p.end) {
                    if (extrapolate_flat) {
                        utctimespan dt = p.end - std::max(p.start, l.t);
                        tsum += dt;
                        area += to_seconds(dt) * l.v;
                    }
                }
                break;
            }
            if (l.t >= p.end) break;
        } else {
            pt r = get(i++);
            bool r_finite = std::isfinite(r.v);
            utcperiod px(std::max(l.t, p.start), std::min(r.t, p.end));
            utctimespan dt = px.timespan();
            if (linear && r_finite) {
                double a = (r.v - l.v) / to_seconds(r.t - l.t);
                double b = r.v - a * to_seconds(r.t);
                area += to_seconds(dt) * (0.5 * a * to_seconds(px.start + px.end) + b);
                tsum += dt;
            } else {
                if (extrapolate_flat) {
                    area += l.v * to_seconds(dt);
                    tsum += dt;
                }
            }
            if (i == n) {
                if (r_finite && r.t < p.end) {
                    if (extrapolate_flat) {
                        dt = p.end - r.t;
                        tsum += dt;
                        area += to_seconds(dt) * r.v;
                    }
                }
                break;
            }
            if (r.t >= p.end) break;
            l_finite = r_finite;
            l = r;
        }
    }
    last_idx = i - 1;
    return tsum ? area : nan;
}

// average_value (time_series.h:302-306)
inline double average_value(const point_ts& source, const utcperiod& p, size_t& last_idx, bool linear = true) {
    utctimespan tsum = 0;
    double area = accumulate_value(source, p, last_idx, tsum, linear);
    return tsum > 0 ? area / to_seconds(tsum) : std::numeric_limits<double>::quiet_NaN();
}

// average_accessor<S, fixed_dt>(source, ta).value(i) for every i (time_series.h:2033-2072), USE_NAN
// extension: periods starting at or after the source's end are NaN.
inline std::vector<double> average_values(const point_ts& source, const fixed_dt& ta) {
    std::vector<double> r(ta.size());
    const bool linear = source.fx == POINT_INSTANT_VALUE;
    const utctime src_end = source.total_period().end;
    size_t last_idx = 0;
    for (size_t i = 0; i < ta.size(); ++i) {
        if (ta.time(i) >= src_end) r[i] = std::numeric_limits<double>::quiet_NaN();
        else r[i] = average_value(source, ta.period(i), last_idx, linear);
    }
    return r;
}

// UTC calendar (core/utctime_utilities.cpp:230-277): civil date <-> utctime
inline int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}
inline utctime utc_time(int64_t y, int mo, int d, int h = 0, int mi = 0, int s = 0, int us = 0) {
    return (days_from_civil(y, mo, d) * 86400 + int64_t(h) * 3600 + int64_t(mi) * 60 + s) * US + us;
}
// calendar::day_of_year (UTC): 1 + days since Jan 1 of t's year
inline int day_of_year(utctime t) {
    const int64_t day_us = int64_t(86400) * US;
    int64_t days = t / day_us;
    if (t % day_us != 0 && t < 0) --days;
    int64_t z = days + 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy_mar = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy_mar + 2) / 153;
    const int m = int(mp < 10 ? mp + 3 : mp - 9);
    const int64_t y = yoe + era * 400 + (m <= 2);
    return int(1 + days - days_from_civil(y, 1, 1));
}

}  // namespace shyft_hip::host
