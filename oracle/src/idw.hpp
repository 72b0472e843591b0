// ORACLE — test infrastructure only (see common.hpp header).
//
// idw.hpp: inverse-distance interpolation (core/inverse_distance.h:142-472)
// as driven by region_model::interpolate (core/region_model.h:397-527).
#pragma once
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.hpp"

namespace oracle {
namespace idw {

enum model_kind { TEMPERATURE = 0, PRECIPITATION = 1, RADIATION = 2, WIND_SPEED = 3, REL_HUM = 4 };

// inverse_distance.h:38-74 (parameter, temperature_parameter, precipitation_parameter)
struct parameter {
    size_t max_members = 10;
    double max_distance = 200000.0;
    double distance_measure_factor = 2.0;
    double zscale = 1.0;
    double default_temp_gradient = -0.006;  // temperature_parameter
    bool gradient_by_equation = false;      // temperature_parameter
    double scale_factor = 1.02;             // precipitation_parameter
};

struct source {
    geo_point p;
    const double* values;  // [T] on the model time axis (average_accessor already applied)
};

struct destination {
    geo_point p;
    double slope_factor;
};

// 3x3 solve for temperature_gradient_scale_computer::compute with
// gradient_by_equation (inverse_distance.h:296-303). The reference calls
// arma::solve(..., no_approx) which, for a 3x3 system, inverts the matrix via
// its determinant and cofactors (armadillo's tiny-matrix path) and fails on a
// singular matrix; restated here the same way. Returns false if singular.
inline bool solve3(const double A[3][3], const double b[3], double x[3]) {
    const double det = A[0][0] * (A[1][1] * A[2][2] - A[1][2] * A[2][1]) -
                       A[0][1] * (A[1][0] * A[2][2] - A[1][2] * A[2][0]) +
                       A[0][2] * (A[1][0] * A[2][1] - A[1][1] * A[2][0]);
    if (!(std::fabs(det) > 0.0) || !std::isfinite(det)) return false;
    double inv[3][3];
    inv[0][0] = (A[1][1] * A[2][2] - A[1][2] * A[2][1]) / det;
    inv[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) / det;
    inv[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) / det;
    inv[1][0] = (A[1][2] * A[2][0] - A[1][0] * A[2][2]) / det;
    inv[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) / det;
    inv[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) / det;
    inv[2][0] = (A[1][0] * A[2][1] - A[1][1] * A[2][0]) / det;
    inv[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) / det;
    inv[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) / det;
    for (int i = 0; i < 3; ++i) x[i] = inv[i][0] * b[0] + inv[i][1] * b[1] + inv[i][2] * b[2];
    return std::isfinite(x[0]) && std::isfinite(x[1]) && std::isfinite(x[2]);
}

// temperature_gradient_scale_computer::compute (inverse_distance.h:305-330) over
// the valid points (z, value) in neighbour order
inline double temperature_gradient(const std::vector<geo_point>& pts, const std::vector<double>& t, double default_gradient,
                                   bool by_equation) {
    const double minimum_z_distance = 50.0;
    const size_t n = pts.size();
    if (by_equation && n > 3) {
        const double A[3][3] = {{pts[1].x - pts[0].x, pts[1].y - pts[0].y, pts[1].z - pts[0].z},
                                {pts[2].x - pts[0].x, pts[2].y - pts[0].y, pts[2].z - pts[0].z},
                                {pts[3].x - pts[0].x, pts[3].y - pts[0].y, pts[3].z - pts[0].z}};
        const double b[3] = {t[1] - t[0], t[2] - t[0], t[3] - t[0]};
        double g[3];
        if (solve3(A, b, g)) return g[2];
    }
    if (n > 1) {
        size_t mx_i = 0, mn_i = 0;
        for (size_t i = 0; i < n; ++i) {
            const double h = pts[i].z;
            if (h < pts[mn_i].z) mn_i = i;
            else if (h > pts[mx_i].z) mx_i = i;
        }
        const double mi_mx_dz = pts[mx_i].z - pts[mn_i].z;
        return mi_mx_dz > minimum_z_distance ? (t[mx_i] - t[mn_i]) / mi_mx_dz : default_gradient;
    }
    return default_gradient;
}

struct neighbour {
    size_t s;
    double w;
};

// step 1 of run_interpolation (inverse_distance.h:177-201): per destination the
// sources with weight >= min_weight, weight = min(1, 1/distance_measure); if more
// than max_members, the max_members largest weights in descending order (the
// reference's partial_sort leaves ties in unspecified order; ties are broken by
// ascending source index here and in the kernel), else in source order.
inline std::vector<neighbour> neighbours(const geo_point& d, const std::vector<source>& src, const parameter& p) {
    const double max_weight = 1.0;
    const double min_weight =
        1.0 / geo_point::distance_measure(geo_point(0.0), geo_point(p.max_distance), p.distance_measure_factor, p.zscale);
    std::vector<neighbour> swl;
    for (size_t s = 0; s < src.size(); ++s) {
        const double weight =
            std::min(max_weight, 1.0 / geo_point::distance_measure(d, src[s].p, p.distance_measure_factor, p.zscale));
        if (weight >= min_weight) swl.push_back({s, weight});
    }
    if (swl.size() > p.max_members) {
        std::stable_sort(swl.begin(), swl.end(), [](const neighbour& a, const neighbour& b) { return a.w > b.w; });
        swl.resize(p.max_members);
    }
    return swl;
}

// run_interpolation (inverse_distance.h:142-250) for one model over [0, T), destinations [j0, j1) (default all;
// the destinations are independent, so the caller may split them over threads)
inline void run(model_kind kind, const std::vector<source>& src, const std::vector<destination>& dst, size_t T,
                const parameter& p, double* out /*[T][n_dst]*/, size_t j0 = 0, size_t j1 = SIZE_MAX) {
    const size_t N = dst.size();
    if (j1 > N) j1 = N;
    for (size_t j = j0; j < j1; ++j) {
        const auto nb = neighbours(dst[j].p, src, p);
        std::vector<geo_point> pts;
        std::vector<double> tv;
        for (size_t i = 0; i < T; ++i) {
            double scale = 1.0;
            if (kind == TEMPERATURE) {
                pts.clear();
                tv.clear();
                for (const auto& sw : nb) {
                    const double v = src[sw.s].values[i];
                    if (std::isfinite(v)) {
                        pts.push_back(src[sw.s].p);
                        tv.push_back(v);
                    }
                }
                scale = temperature_gradient(pts, tv, p.default_temp_gradient, p.gradient_by_equation);
            } else if (kind == PRECIPITATION) {
                scale = p.scale_factor;
            }
            double sum_weights = 0, sum_weight_value = 0;
            for (const auto& sw : nb) {
                const double v = src[sw.s].values[i];
                if (!std::isfinite(v)) continue;
                double tr;
                switch (kind) {
                    case TEMPERATURE: tr = v + scale * (dst[j].p.z - src[sw.s].p.z); break;                         // :390-392
                    case PRECIPITATION: tr = v * OPOW(scale, (dst[j].p.z - src[sw.s].p.z) / 100.0); break;          // :435-439
                    case RADIATION: tr = v * dst[j].slope_factor; break;                                              // :412-414
                    default: tr = v; break;                                                                           // :455, :472
                }
                sum_weight_value += sw.w * tr;
                sum_weights += sw.w;
            }
            out[i * N + j] = sum_weight_value / sum_weights;
        }
    }
}

}  // namespace idw
}  // namespace oracle
