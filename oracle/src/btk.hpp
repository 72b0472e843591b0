// ORACLE — test infrastructure only (see common.hpp header).
//
// btk.hpp: Bayesian temperature kriging, a step-by-step restatement of
// bayesian_kriging::btk_interpolation (core/bayesian_kriging.h:280-402) with
// its helpers utils::build_covariance_matrices / build_elevation_matrices
// (:93-162) and the parameter's covariance model (:46-56). The reference uses
// armadillo 9.200.6 (third-party, not vendored): inv() is restated as an LU
// factorisation with partial pivoting (LAPACK getrf/getri semantics), rank() of
// the 2x2 H^-1 by its singular values with armadillo's default tolerance
// max(m,n) * max(sigma) * eps, and every product in the order the reference
// writes it (operator* is left-associative).
#pragma once
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <string>
#include <vector>

#include "mathlib.hpp"

namespace oracle {
namespace btk {

struct parameter {  // bayesian_kriging::parameter (:204-230), gradient_sd already /100
    double gradient_sd = 0.0025, sill = 25.0, nug = 0.5, range = 200000.0, zscale = 20.0;
};

// dense row-major matrix
struct mat {
    size_t r = 0, c = 0;
    std::vector<double> a;
    mat() = default;
    mat(size_t r_, size_t c_, double v = 0.0) : r(r_), c(c_), a(r_ * c_, v) {}
    double& operator()(size_t i, size_t j) { return a[i * c + j]; }
    double operator()(size_t i, size_t j) const { return a[i * c + j]; }
};
inline mat mul(const mat& x, const mat& y) {
    if (x.c != y.r) throw std::runtime_error("btk oracle: matrix size mismatch");
    mat z(x.r, y.c);
    for (size_t i = 0; i < x.r; ++i)
        for (size_t j = 0; j < y.c; ++j) {
            double s = 0.0;
            for (size_t k = 0; k < x.c; ++k) s += x(i, k) * y(k, j);
            z(i, j) = s;
        }
    return z;
}
inline mat t(const mat& x) {
    mat z(x.c, x.r);
    for (size_t i = 0; i < x.r; ++i)
        for (size_t j = 0; j < x.c; ++j) z(j, i) = x(i, j);
    return z;
}
inline mat sub(const mat& x, const mat& y) {
    mat z(x);
    for (size_t i = 0; i < z.a.size(); ++i) z.a[i] -= y.a[i];
    return z;
}
// inverse by LU with partial pivoting (getrf), then column-by-column solves (getri)
inline mat inv(const mat& x) {
    const size_t n = x.r;
    mat lu(x);
    std::vector<size_t> piv(n);
    for (size_t k = 0; k < n; ++k) {
        size_t p = k;
        for (size_t i = k + 1; i < n; ++i)
            if (std::fabs(lu(i, k)) > std::fabs(lu(p, k))) p = i;
        piv[k] = p;
        if (lu(p, k) == 0.0) throw std::runtime_error("inv(): matrix is singular");
        if (p != k)
            for (size_t j = 0; j < n; ++j) std::swap(lu(k, j), lu(p, j));
        for (size_t i = k + 1; i < n; ++i) {
            lu(i, k) /= lu(k, k);
            for (size_t j = k + 1; j < n; ++j) lu(i, j) -= lu(i, k) * lu(k, j);
        }
    }
    mat r(n, n);
    for (size_t col = 0; col < n; ++col) {
        std::vector<double> b(n, 0.0);
        b[col] = 1.0;
        for (size_t k = 0; k < n; ++k) std::swap(b[k], b[piv[k]]);  // apply P
        for (size_t i = 0; i < n; ++i)
            for (size_t k = 0; k < i; ++k) b[i] -= lu(i, k) * b[k];
        for (size_t i = n; i-- > 0;) {
            for (size_t k = i + 1; k < n; ++k) b[i] -= lu(i, k) * b[k];
            b[i] /= lu(i, i);
        }
        for (size_t i = 0; i < n; ++i) r(i, col) = b[i];
    }
    return r;
}
// arma::rank of a 2x2 matrix (singular values vs max(m,n)*max(sigma)*eps)
inline int rank2(const mat& x) {
    const double a = x(0, 0), b = x(0, 1), c = x(1, 0), d = x(1, 1);
    const double s1 = a * a + b * b + c * c + d * d, det = a * d - b * c;
    const double disc = std::sqrt(std::max(0.0, s1 * s1 - 4 * det * det));
    const double smax = std::sqrt((s1 + disc) / 2), smin = std::sqrt(std::max(0.0, (s1 - disc) / 2));
    const double tol = 2 * smax * 2.220446049250313e-16;
    return (smax > tol ? 1 : 0) + (smin > tol ? 1 : 0);
}

// geo_point::zscaled_distance (core/geo_point.h:49-51)
inline double zdist(const double* p, const double* q, double zscale) {
    return std::sqrt((p[0] - q[0]) * (p[0] - q[0]) + (p[1] - q[1]) * (p[1] - q[1]) +
                     (p[2] - q[2]) * (p[2] - q[2]) * zscale * zscale);
}
inline double cov(double d, const parameter& p) { return (p.sill - p.nug) * OEXP(-d / p.range); }

// build_covariance_matrices K (S x S) for the sources (:93-113)
inline mat source_covariance(size_t S, const double* xyz, const parameter& p) {
    mat K(S, S);
    for (size_t i = 0; i < S; ++i) {
        K(i, i) = p.sill - p.nug;
        for (size_t j = i + 1; j < S; ++j) K(i, j) = K(j, i) = cov(zdist(xyz + 3 * i, xyz + 3 * j, p.zscale), p);
    }
    return K;
}

// btk_interpolation: src_values [T][S] (NaN = missing), prior_gradient[T] (parameter.temperature_gradient of
// each period), out [T][D]
inline void run(size_t S, const double* src_xyz, const double* src_values, size_t T, const double* prior_gradient,
                const parameter& p, size_t D, const double* dst_xyz, double* out) {
    mat F(S, 2), f(2, D);
    for (size_t i = 0; i < S; ++i) {
        F(i, 0) = 1.0;
        F(i, 1) = src_xyz[3 * i + 2];
    }
    for (size_t j = 0; j < D; ++j) {
        f(0, j) = 1.0;
        f(1, j) = dst_xyz[3 * j + 2];
    }
    const mat K = source_covariance(S, src_xyz, p);
    mat k(S, D);
    for (size_t i = 0; i < S; ++i)
        for (size_t j = 0; j < D; ++j) k(i, j) = cov(zdist(src_xyz + 3 * i, dst_xyz + 3 * j, p.zscale), p);
    mat eye(2, 2);
    eye(0, 0) = eye(1, 1) = 1.0;
    const double inv_sd2 = 1 / (p.gradient_sd * p.gradient_sd);
    struct ops {
        mat F, E_beta_w, omega, GH_inv, BM;
    };
    auto build = [&](const std::vector<size_t>& idx, bool full) {
        ops o;
        const size_t n = idx.size();
        mat Kr(n, n), kr(n, D);
        o.F = mat(n, 2);
        for (size_t a = 0; a < n; ++a) {
            o.F(a, 0) = F(idx[a], 0);
            o.F(a, 1) = F(idx[a], 1);
            for (size_t b = 0; b < n; ++b) Kr(a, b) = K(idx[a], idx[b]);
            for (size_t j = 0; j < D; ++j) kr(a, j) = k(idx[a], j);
        }
        const mat K_inv = inv(Kr);
        const mat H_inv = mul(mul(t(o.F), K_inv), o.F);
        if (full && rank2(H_inv) == 1)
            throw std::runtime_error("The bayestian temperature kriging algorithm needs at least two sources at different heights.");
        const mat H = inv(H_inv);
        mat G_inv = H_inv;
        G_inv(1, 1) += inv_sd2;
        const mat G = inv(G_inv);
        o.GH_inv = mul(G, H_inv);
        o.BM = mul(t(sub(f, mul(mul(t(o.F), K_inv), kr))), sub(eye, o.GH_inv));
        o.E_beta_w = mul(mul(H, t(o.F)), K_inv);
        o.omega = mul(t(kr), K_inv);
        return o;
    };
    std::vector<size_t> all(S), valid, prev;
    for (size_t i = 0; i < S; ++i) all[i] = i;
    ops full_ops = build(all, true), red;
    const ops* cur = nullptr;
    for (size_t ts = 0; ts < T; ++ts) {
        prev = valid;
        valid.clear();
        std::vector<double> temps;
        for (size_t i = 0; i < S; ++i) {
            const double v = src_values[ts * S + i];
            if (std::isfinite(v)) {
                valid.push_back(i);
                temps.push_back(v);
            }
        }
        if (valid != prev || valid.empty()) {
            if (valid.empty())
                throw std::runtime_error("bayesian kriging temperature: No valid sources for time period, giving up.");
            if (valid.size() == S) cur = &full_ops;
            else {
                red = build(valid, false);
                cur = &red;
            }
        }
        mat E_beta_pri(2, 1);
        E_beta_pri(1, 0) = prior_gradient[ts];
        mat T_obs(valid.size(), 1);
        for (size_t a = 0; a < valid.size(); ++a) T_obs(a, 0) = temps[a];
        const mat beta_hat = mul(cur->E_beta_w, T_obs);
        const mat T_hat = [&] {
            mat x = mul(t(f), beta_hat);
            const mat y = mul(cur->omega, sub(T_obs, mul(cur->F, beta_hat)));
            for (size_t i = 0; i < x.a.size(); ++i) x.a[i] += y.a[i];
            return x;
        }();
        const mat post = sub(T_hat, mul(cur->BM, sub(beta_hat, E_beta_pri)));
        for (size_t j = 0; j < D; ++j) out[ts * D + j] = post(j, 0);
    }
}

}  // namespace btk
}  // namespace oracle
