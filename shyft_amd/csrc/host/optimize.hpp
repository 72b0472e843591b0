// Single-variable minimisation used by the state-to-flow tuning
// (region_model::adjust_state_to_target_flow, core/region_model.h:626-637 ->
// core/model_state_tuning.h:96-120).
//
// The reference calls dlib::find_min_single_variable (dlib 19.x,
// dlib/optimization/optimization_line_search.h; dlib is an external dependency
// that is not vendored under /root/reference). This is a restatement of that
// published algorithm: bracket a minimum with three points p1 < p2 < p3,
// f1 > f2 < f3 (expanding the search radius away from the start point, clamped
// to [begin, end]), then shrink the bracket with safeguarded 3-point
// Lagrange-polynomial (parabolic) steps until p3 - p1 <= eps. Running out of
// evaluations raises, as dlib's optimize_single_variable_failure does.
#pragma once

#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>

namespace shyft_hip::host {

struct optimize_single_variable_failure : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// minimiser of the parabola through (p1,f1),(p2,f2),(p3,f3), clamped to [p1,p3]
// (Ruszczynski, Nonlinear Optimization, section 5.2)
inline double lagrange_poly_min_extrap(double p1, double p2, double p3, double f1, double f2, double f3) {
    const double num = f1 * (p3 * p3 - p2 * p2) + f2 * (p1 * p1 - p3 * p3) + f3 * (p2 * p2 - p1 * p1);
    const double den = 2 * (f1 * (p3 - p2) + f2 * (p1 - p3) + f3 * (p2 - p1));
    if (den == 0) return p2;
    const double x = num / den;
    if (p1 <= x && x <= p3) return x;
    return std::min(std::max(p1, x), p3);
}

// Minimise f over [begin, end] starting at x (updated to the minimiser); returns f(x).
template <class F>
double find_min_single_variable(F&& f, double& x, double begin, double end, double eps, long max_iter,
                                double radius = 1.0) {
    if (!(eps > 0 && max_iter > 1 && begin <= x && x <= end && radius > 0))
        throw std::invalid_argument("find_min_single_variable: invalid arguments (eps=" + std::to_string(eps) +
                                    ", begin=" + std::to_string(begin) + ", x=" + std::to_string(x) +
                                    ", end=" + std::to_string(end) + ")");
    if (begin == end) return f(x);

    long evals = 1;
    double p1 = std::max(x - radius, begin), p3 = std::min(x + radius, end), p2;
    double f1 = f(p1), f3 = f(p3), f2;
    if (x == p1 || x == p3) {
        p2 = 0.5 * (p1 + p3);
        f2 = f(p2);
    } else {
        p2 = x;
        f2 = f(x);
    }
    evals += 2;

    // phase 1: find a bracket f1 > f2 < f3
    while (!(f1 > f2 && f2 < f3)) {
        if (evals >= max_iter || p3 - p1 < eps) break;
        if (f1 == f2 && f1 < f3 && p1 != begin) {  // flat on the left: widen left
            p1 = std::max(p1 - radius, begin);
            f1 = f(p1);
            ++evals;
            radius *= 2;
            continue;
        }
        if (f2 == f3 && f3 < f1 && p3 != end) {  // flat on the right: widen right
            p3 = std::min(p3 + radius, end);
            f3 = f(p3);
            ++evals;
            radius *= 2;
            continue;
        }
        if (f1 <= f3) {  // lower on the left
            if (p1 == begin || (f1 == f2 && (end - begin) < radius)) {
                p3 = p2;
                f3 = f2;
                p2 = 0.5 * (p1 + p2);
                f2 = f(p2);
            } else {
                p3 = p2;
                f3 = f2;
                p2 = p1;
                f2 = f1;
                p1 = std::max(p1 - radius, begin);
                f1 = f(p1);
                radius *= 2;
            }
        } else {  // lower on the right
            if (p3 == end || (f2 == f3 && (end - begin) < radius)) {
                p1 = p2;
                f1 = f2;
                p2 = 0.5 * (p2 + p3);
                f2 = f(p2);
            } else {
                p1 = p2;
                f1 = f2;
                p2 = p3;
                f2 = f3;
                p3 = std::min(p3 + radius, end);
                f3 = f(p3);
                radius *= 2;
            }
        }
        ++evals;
    }

    // phase 2: safeguarded parabolic steps inside the bracket
    const double tau = 0.1;
    while (evals < max_iter && p3 - p1 > eps) {
        double pm = lagrange_poly_min_extrap(p1, p2, p3, f1, f2, f3);
        if (pm < p2) {  // keep pm at least tau * (side width) from the known points
            const double d = (p2 - p1) * tau;
            if (std::abs(p1 - pm) < d)
                pm = p1 + d;
            else if (std::abs(p2 - pm) < d)
                pm = p2 - d;
        } else {
            const double d = (p3 - p2) * tau;
            if (std::abs(p2 - pm) < d)
                pm = p2 + d;
            else if (std::abs(p3 - pm) < d)
                pm = p3 - d;
        }
        const double ratio = std::abs(p1 - p2) / std::abs(p2 - p3);  // lopsided bracket: bisect the long side
        if (!(ratio < 10 && ratio > 0.1)) {
            if (ratio > 1 && pm > p2)
                pm = 0.5 * (p1 + p2);
            else if (pm < p2)
                pm = 0.5 * (p2 + p3);
        }
        const double fm = f(pm);
        if (pm < p2) {
            if (f1 > fm && fm < f2) {
                p3 = p2;
                f3 = f2;
                p2 = pm;
                f2 = fm;
            } else {
                p1 = pm;
                f1 = fm;
            }
        } else {
            if (f2 > fm && fm < f3) {
                p1 = p2;
                f1 = f2;
                p2 = pm;
                f2 = fm;
            } else {
                p3 = pm;
                f3 = fm;
            }
        }
        ++evals;
    }
    if (evals >= max_iter)
        throw optimize_single_variable_failure(
            "The max number of iterations of single variable optimization have been reached\nwithout converging.");
    x = p2;
    return f2;
}

}  // namespace shyft_hip::host
