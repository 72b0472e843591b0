// ORACLE — test infrastructure only. CPU restatement of the reference
// (magneano/shyft @ /root/reference, VERSION 4.6.1675). Only tests/, the
// __graft_entry__.smoke() checker and bench.py's cpu_baseline leg may load
// this code; the product path (shyft_amd/) never links or calls it.
//
// common.hpp: time axis, UTC calendar, geo primitives and unit conversion.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstddef>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

#include "mathlib.hpp"

namespace oracle {

constexpr double nan = std::numeric_limits<double>::quiet_NaN();

// utctime in the reference is std::chrono::microseconds (core/utctime_utilities.h:29-34).
using utctime = int64_t;          // microseconds since 1970-01-01Z
constexpr int64_t US_PER_S = 1000000;
constexpr int64_t HOUR_US = 3600 * US_PER_S;
constexpr int64_t DAY_US = 24 * HOUR_US;

// to_seconds: core/utctime_utilities.h:68 (double(dt.count())/1e6)
inline double to_seconds(int64_t dt_us) { return double(dt_us) / double(US_PER_S); }

// fixed_dt: core/time_axis.h:74-115 — period(i) = [t + i*dt, t + (i+1)*dt)
struct fixed_dt {
    utctime t = 0;
    int64_t dt = 0;
    size_t n = 0;
    fixed_dt() = default;
    fixed_dt(utctime t, int64_t dt, size_t n) : t(t), dt(dt), n(n) {}
    size_t size() const { return n; }
    utctime time(size_t i) const { return t + int64_t(i) * dt; }
    bool operator==(const fixed_dt& o) const { return t == o.t && dt == o.dt && n == o.n; }
    bool operator!=(const fixed_dt& o) const { return !(*this == o); }
};

// UTC calendar (core/utctime_utilities.cpp:230-277). The reference computes
// civil dates from julian day numbers; here the proleptic Gregorian civil-from-days
// algorithm is used, which is the same mapping for UTC.
struct ymd { int64_t y; int m; int d; };

inline int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
    return q;
}

inline ymd civil_from_days(int64_t z) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int d = int(doy - (153 * mp + 2) / 5 + 1);
    const int m = int(mp < 10 ? mp + 3 : mp - 9);
    return ymd{y + (m <= 2), m, d};
}

inline int64_t days_from_civil(int64_t y, int m, int d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

// calendar::day_of_year (utctime_utilities.cpp:230-235): 1 + day_number(t) - day_number(Jan 1)
inline int day_of_year(utctime t) {
    int64_t days = floor_div(t, DAY_US);
    ymd c = civil_from_days(days);
    return int(1 + days - days_from_civil(c.y, 1, 1));
}

// calendar::trim(t, YEAR) (utctime_utilities.cpp:249-253)
inline utctime trim_year(utctime t) {
    int64_t days = floor_div(t, DAY_US);
    ymd c = civil_from_days(days);
    return days_from_civil(c.y, 1, 1) * DAY_US;
}

inline utctime utc_time(int64_t y, int m, int d, int h = 0, int mi = 0, int s = 0) {
    return (days_from_civil(y, m, d) * 86400 + h * 3600 + mi * 60 + s) * US_PER_S;
}

// geo_point: core/geo_point.h:20-60
struct geo_point {
    double x = 0, y = 0, z = 0;
    geo_point() = default;
    geo_point(double x, double y = 0.0, double z = 0.0) : x(x), y(y), z(z) {}
    // distance_measure (geo_point.h:41-43): pow(dx^2+dy^2+dz^2*zscale^2, p/2)
    static double distance_measure(const geo_point& a, const geo_point& b, double p, double zscale) {
        return OPOW((a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z) * zscale * zscale,
                        p / 2.0);
    }
};

// land_type_fractions / geo_cell_data: core/geo_cell_data.h:25-140
struct land_type_fractions {
    double glacier_ = 0, lake_ = 0, reservoir_ = 0, forest_ = 0;
    double glacier() const { return glacier_; }
    double lake() const { return lake_; }
    double reservoir() const { return reservoir_; }
    double forest() const { return forest_; }
    double unspecified() const { return 1.0 - glacier_ - lake_ - reservoir_ - forest_; }
    double snow_storage() const { return 1.0 - lake_ - reservoir_; }
    // set_fractions (geo_cell_data.h:67-79)
    void set_fractions(double glacier, double lake, double reservoir, double forest) {
        const double tol = 1.0e-3;
        const double sum = glacier + lake + reservoir + forest;
        if (sum > 1.0 && sum < 1.0 + tol) {
            glacier /= sum; lake /= sum; reservoir /= sum; forest /= sum;
        } else if (sum > 1.0 || (glacier < 0.0 || lake < 0.0 || reservoir < 0.0 || forest < 0.0))
            throw std::invalid_argument("LandTypeFractions:: must be >=0.0 and sum <= 1.0");
        glacier_ = glacier; lake_ = lake; reservoir_ = reservoir; forest_ = forest;
    }
};

struct routing_info { int64_t id = 0; double distance = 0.0; };

struct geo_cell_data {
    geo_point mid_point;
    double area = 1000000.0;
    int64_t catchment_id = -1;
    double radiation_slope_factor = 0.9;
    land_type_fractions fractions;
    routing_info routing;
    size_t catchment_ix = 0;
    // geo_cell_data_io::from_raw_vector layout (api/api.h:1617-1621):
    // x y z area cid slope glacier lake reservoir forest unspecified
    static geo_cell_data from_raw(const double* v) {
        geo_cell_data g;
        g.mid_point = geo_point(v[0], v[1], v[2]);
        g.area = v[3];
        g.catchment_id = int64_t(int(v[4]));
        g.radiation_slope_factor = v[5];
        g.fractions.set_fractions(v[6], v[7], v[8], v[9]);
        return g;
    }
};

// unit_conversion.h:6-15
constexpr double mmh_to_m3s_scale_factor = 1 / (3600.0 * 1000.0);
inline double mmh_to_m3s(double mm_pr_hour, double area_m2) { return area_m2 * mm_pr_hour * mmh_to_m3s_scale_factor; }
inline double m3s_to_mmh(double m3s, double area_m2) { return m3s / (mmh_to_m3s_scale_factor * area_m2); }

}  // namespace oracle
