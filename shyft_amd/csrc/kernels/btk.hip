// Bayesian temperature kriging for gfx950 (core/bayesian_kriging.h:280-402).
//
// The reference evaluates, per time step, beta = E_beta_w T_obs, T_hat = f' beta + omega (T_obs - F beta)
// and E_temp_post = T_hat - BM (beta - E_beta_pri) with omega = k' K^-1 (destinations x sources). For a
// fixed set of valid sources every term is linear in T_obs, so the whole time loop is one matrix product:
//
//   temp[t][d] = sum_s A[s][d] T_obs[t][s] + u_d . beta(t) + BM[d][1] grad(t)
//   A = K^-T k,  v_d = f_d - (F' A)_d,  u_d = GH_inv' v_d,  BM_d = (I - GH_inv)' v_d,  beta(t) = E_beta_w T_obs(t)
//
// Host: the small (sources x sources) algebra per valid-source pattern -- K^-1, H, G, GH_inv, E_beta_w --
// and beta(t) per step. Device: the source-destination covariance k (one exp per pair), A = K^-T k
// (rocBLAS dgemm, S x S x D), the per-destination rows u_d, BM_d1 (one pass over A), and the time loop as
// ONE dgemm per pattern and block of steps: [D x (S+3)] x [(S+3) x steps], written straight into the
// forcing window ([step][cell], ld = cells) when every cell is a destination. Time steps whose valid-source
// set differs from the full set use the reference's reduced operators (its valid_inds branch), grouped by
// pattern so each distinct pattern is factorised once.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../detmath/detmath.h"
#include "../include_internal/kernels.h"

namespace {

void check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("btk ") + what + ": " + hipGetErrorString(e));
}
void check(rocblas_status s, const char* what) {
    if (s != rocblas_status_success)
        throw std::runtime_error(std::string("btk ") + what + ": " + rocblas_status_to_string(s));
}

template <class T>
struct devbuf {
    T* p = nullptr;
    size_t n = 0;
    devbuf() = default;
    devbuf(const devbuf&) = delete;
    devbuf& operator=(const devbuf&) = delete;
    ~devbuf() {
        if (p) (void)hipFree(p);
    }
    void alloc(size_t count) {
        if (count <= n && p) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        check(hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)), "hipMalloc");
        n = count;
    }
    void upload(const T* src, size_t count, hipStream_t s) {
        alloc(count);
        check(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, s), "upload");
    }
};

rocblas_handle blas_handle(int device) {
    static std::mutex mu;
    static std::map<int, rocblas_handle> handles;
    std::lock_guard<std::mutex> lock(mu);
    auto f = handles.find(device);
    if (f != handles.end()) return f->second;
    rocblas_handle h = nullptr;
    check(rocblas_create_handle(&h), "rocblas_create_handle");
    handles[device] = h;
    return h;
}

// ---- device kernels ---------------------------------------------------------------------------------------------
// k[j][d] = (sill - nug) exp(-zscaled_distance(src_j, dst_d) / range)  (utils::cov, bayesian_kriging.h:53-56)
__global__ __launch_bounds__(256) void btk_cov_kernel(const double* __restrict__ src_xyz, int n_src,
                                                      const double* __restrict__ dst_xyz, int n_dst, double c0,
                                                      double range, double zscale, double* __restrict__ k) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y;
    if (d >= n_dst || j >= n_src) return;
    const double dx = src_xyz[3 * j] - dst_xyz[3 * d], dy = src_xyz[3 * j + 1] - dst_xyz[3 * d + 1],
                 dz = src_xyz[3 * j + 2] - dst_xyz[3 * d + 2];
    const double dist = sqrt(dx * dx + dy * dy + dz * dz * zscale * zscale);
    k[size_t(j) * n_dst + d] = c0 * detmath::exp(-dist / range);
}

// rows n_src, n_src+1, n_src+2 of A: u_d0, u_d1, BM_d1 (see the file comment)
__global__ __launch_bounds__(256) void btk_dest_kernel(double* __restrict__ A, int n_src, const double* __restrict__ z_src,
                                                       const double* __restrict__ dst_xyz, int n_dst, double g00,
                                                       double g01, double g10, double g11) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= n_dst) return;
    double s0 = 0.0, s1 = 0.0;
    for (int j = 0; j < n_src; ++j) {
        const double a = A[size_t(j) * n_dst + d];
        s0 += a;
        s1 += a * z_src[j];
    }
    const double v0 = 1.0 - s0, v1 = dst_xyz[3 * d + 2] - s1;
    // u = GH_inv' v ; BM_d = (I - GH_inv)' v, of which only the gradient column (1) multiplies a non-zero prior
    A[size_t(n_src) * n_dst + d] = g00 * v0 + g10 * v1;
    A[size_t(n_src + 1) * n_dst + d] = g01 * v0 + g11 * v1;
    A[size_t(n_src + 2) * n_dst + d] = (-g01) * v0 + (1.0 - g11) * v1;
}

// out[steps[j]][index[d]] = C[j][d]
__global__ __launch_bounds__(256) void btk_scatter_kernel(const double* __restrict__ C, int n_dst, int n_steps,
                                                          const int32_t* __restrict__ steps,
                                                          const int32_t* __restrict__ index, double* __restrict__ out,
                                                          size_t ld_out) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y;
    if (d >= n_dst || j >= n_steps) return;
    out[size_t(steps[j]) * ld_out + (index ? size_t(index[d]) : size_t(d))] = C[size_t(j) * n_dst + d];
}

// ---- host dense algebra (armadillo's inv / rank as the reference uses them) ---------------------------------------
using rmat = std::vector<double>;  // row-major square or 2x2

// inverse by LU with partial pivoting (LAPACK getrf/getri semantics)
rmat lu_inverse(const rmat& x, size_t n) {
    rmat lu(x);
    std::vector<size_t> piv(n);
    for (size_t k = 0; k < n; ++k) {
        size_t p = k;
        for (size_t i = k + 1; i < n; ++i)
            if (std::fabs(lu[i * n + k]) > std::fabs(lu[p * n + k])) p = i;
        piv[k] = p;
        if (lu[p * n + k] == 0.0) throw std::runtime_error("inv(): matrix is singular");
        if (p != k)
            for (size_t j = 0; j < n; ++j) std::swap(lu[k * n + j], lu[p * n + j]);
        for (size_t i = k + 1; i < n; ++i) {
            lu[i * n + k] /= lu[k * n + k];
            for (size_t j = k + 1; j < n; ++j) lu[i * n + j] -= lu[i * n + k] * lu[k * n + j];
        }
    }
    rmat r(n * n);
    std::vector<double> b(n);
    for (size_t col = 0; col < n; ++col) {
        std::fill(b.begin(), b.end(), 0.0);
        b[col] = 1.0;
        for (size_t k = 0; k < n; ++k) std::swap(b[k], b[piv[k]]);
        for (size_t i = 0; i < n; ++i)
            for (size_t k = 0; k < i; ++k) b[i] -= lu[i * n + k] * b[k];
        for (size_t i = n; i-- > 0;) {
            for (size_t k = i + 1; k < n; ++k) b[i] -= lu[i * n + k] * b[k];
            b[i] /= lu[i * n + i];
        }
        for (size_t i = 0; i < n; ++i) r[i * n + col] = b[i];
    }
    return r;
}
int rank2(const double* m) {
    const double a = m[0], b = m[1], c = m[2], d = m[3];
    const double s1 = a * a + b * b + c * c + d * d, det = a * d - b * c;
    const double disc = std::sqrt(std::max(0.0, s1 * s1 - 4 * det * det));
    const double smax = std::sqrt((s1 + disc) / 2), smin = std::sqrt(std::max(0.0, (s1 - disc) / 2));
    const double tol = 2 * smax * 2.220446049250313e-16;
    return (smax > tol ? 1 : 0) + (smin > tol ? 1 : 0);
}
void mul2(const double* x, const double* y, double* z) {
    z[0] = x[0] * y[0] + x[1] * y[2];
    z[1] = x[0] * y[1] + x[1] * y[3];
    z[2] = x[2] * y[0] + x[3] * y[2];
    z[3] = x[2] * y[1] + x[3] * y[3];
}

// the reference's operators for one set of valid sources (bayesian_kriging.h:304-316, 362-374)
struct operators {
    rmat K_inv;          // n x n
    double GH_inv[4];    // 2 x 2
    rmat E_beta_w;       // 2 x n
};
operators factorise(const std::vector<size_t>& idx, const double* xyz, double c0, double range, double zscale,
                    double inv_sd2, bool full) {
    const size_t n = idx.size();
    rmat K(n * n);
    for (size_t a = 0; a < n; ++a) {
        K[a * n + a] = c0;
        for (size_t b = a + 1; b < n; ++b) {
            const double* p = xyz + 3 * idx[a];
            const double* q = xyz + 3 * idx[b];
            const double dist = std::sqrt((p[0] - q[0]) * (p[0] - q[0]) + (p[1] - q[1]) * (p[1] - q[1]) +
                                          (p[2] - q[2]) * (p[2] - q[2]) * zscale * zscale);
            K[a * n + b] = K[b * n + a] = c0 * detmath::exp(-dist / range);
        }
    }
    operators o;
    o.K_inv = lu_inverse(K, n);
    // KF = K^-1 F (n x 2), H_inv = F' K^-1 F
    std::vector<double> KF(2 * n);
    double H_inv[4] = {0, 0, 0, 0};
    for (size_t a = 0; a < n; ++a) {
        double s0 = 0, s1 = 0;
        for (size_t b = 0; b < n; ++b) {
            s0 += o.K_inv[a * n + b];
            s1 += o.K_inv[a * n + b] * xyz[3 * idx[b] + 2];
        }
        KF[2 * a] = s0;
        KF[2 * a + 1] = s1;
    }
    for (size_t a = 0; a < n; ++a) {
        const double za = xyz[3 * idx[a] + 2];
        H_inv[0] += KF[2 * a];
        H_inv[1] += KF[2 * a + 1];
        H_inv[2] += za * KF[2 * a];
        H_inv[3] += za * KF[2 * a + 1];
    }
    if (full && rank2(H_inv) == 1)
        throw std::runtime_error("The bayestian temperature kriging algorithm needs at least two sources at different heights.");
    const rmat H = lu_inverse(rmat(H_inv, H_inv + 4), 2);
    rmat G_inv(H_inv, H_inv + 4);
    G_inv[3] += inv_sd2;
    const rmat G = lu_inverse(G_inv, 2);
    mul2(G.data(), H_inv, o.GH_inv);
    // E_beta_w = H F' K^-1 (2 x n)
    o.E_beta_w.assign(2 * n, 0.0);
    for (size_t b = 0; b < n; ++b) {
        double f0 = 0, f1 = 0;  // (F' K^-1)[:, b]
        for (size_t a = 0; a < n; ++a) {
            f0 += o.K_inv[a * n + b];
            f1 += xyz[3 * idx[a] + 2] * o.K_inv[a * n + b];
        }
        o.E_beta_w[b] = H[0] * f0 + H[1] * f1;
        o.E_beta_w[n + b] = H[2] * f0 + H[3] * f1;
    }
    return o;
}

}  // namespace

// Operators of the full source set and the device matrix A = [K^-T k ; u ; BM_1] (D x (S+3)) of the last call,
// reused while sources, parameters and destinations are unchanged (a chunked run interpolates the same
// station network into the same cells window after window).
struct btk_cache {
    std::vector<double> key;
    operators full;
    devbuf<double> A;
    bool valid = false;
};
btk_cache* btk_cache_create() { return new btk_cache(); }
void btk_cache_destroy(btk_cache* c) { delete c; }

void btk_run(const btk_args& a, hipStream_t stream) {
    const size_t S = a.n_sources, D = a.n_dst, T = a.n_steps;
    if (S == 0 || D == 0 || T == 0) return;
    if (D > size_t(INT32_MAX) || S > 4096) throw std::runtime_error("btk: too many sources or destinations");
    int device = 0;
    check(hipGetDevice(&device), "hipGetDevice");
    rocblas_handle blas = blas_handle(device);
    check(rocblas_set_stream(blas, stream), "rocblas_set_stream");
    const double c0 = a.sill - a.nug, inv_sd2 = 1 / (a.gradient_sd * a.gradient_sd);

    // valid-source patterns in order of first appearance; an all-invalid step is the reference's error
    std::map<std::vector<char>, size_t> pattern_ix;
    std::vector<std::vector<size_t>> pattern_steps;
    std::vector<std::vector<char>> patterns;
    for (size_t t = 0; t < T; ++t) {
        std::vector<char> valid(S);
        bool any = false;
        for (size_t s = 0; s < S; ++s) any |= (valid[s] = std::isfinite(a.src_values[t * S + s]) ? 1 : 0) != 0;
        if (!any)
            throw std::runtime_error("bayesian kriging temperature: No valid sources for time period, giving up. step " +
                                     std::to_string(t));
        auto f = pattern_ix.find(valid);
        if (f == pattern_ix.end()) {
            f = pattern_ix.emplace(valid, patterns.size()).first;
            patterns.push_back(valid);
            pattern_steps.emplace_back();
        }
        pattern_steps[f->second].push_back(t);
    }
    // the reference factorises the full source set first and checks its rank whatever the data
    std::vector<double> key = {double(S), double(D), c0, a.range, a.zscale, inv_sd2};
    key.insert(key.end(), a.src_xyz, a.src_xyz + 3 * S);
    btk_cache local;
    btk_cache& cache = a.cache ? *a.cache : local;
    const bool hit = cache.valid && a.dst_version != 0 && cache.key.size() == key.size() + 1 &&
                     std::equal(key.begin(), key.end(), cache.key.begin()) && cache.key.back() == double(a.dst_version);
    if (!hit) {
        std::vector<size_t> all(S);
        for (size_t s = 0; s < S; ++s) all[s] = s;
        cache.valid = false;
        cache.full = factorise(all, a.src_xyz, c0, a.range, a.zscale, inv_sd2, true);
        cache.key = key;
        cache.key.push_back(double(a.dst_version));
    }
    const operators& full = cache.full;

    const double one = 1.0, zero = 0.0;
    devbuf<double> d_src, d_zsrc, d_k, d_A, d_kinv, d_tobs, d_C;
    devbuf<int32_t> d_steps;
    const size_t block_steps = std::max<size_t>(1, std::min<size_t>(T, (size_t(1) << 29) / D));  // temp <= 4 GiB
    for (size_t p = 0; p < patterns.size(); ++p) {
        std::vector<size_t> idx;
        for (size_t s = 0; s < S; ++s)
            if (patterns[p][s]) idx.push_back(s);
        const size_t n = idx.size();
        const bool is_full = idx.size() == S;
        const operators o = is_full ? full : factorise(idx, a.src_xyz, c0, a.range, a.zscale, inv_sd2, false);
        devbuf<double>& dA = is_full ? cache.A : d_A;
        const bool have_A = is_full && hit;
        if (!have_A) {
            std::vector<double> xyz(3 * n), z(n), kinv_cm(n * n);
            for (size_t j = 0; j < n; ++j) {
                for (int c = 0; c < 3; ++c) xyz[3 * j + c] = a.src_xyz[3 * idx[j] + c];
                z[j] = a.src_xyz[3 * idx[j] + 2];
            }
            for (size_t r = 0; r < n; ++r)
                for (size_t c = 0; c < n; ++c) kinv_cm[r + c * n] = o.K_inv[r * n + c];
            d_src.upload(xyz.data(), xyz.size(), stream);
            d_zsrc.upload(z.data(), n, stream);
            d_kinv.upload(kinv_cm.data(), n * n, stream);
            d_k.alloc(n * D);
            dA.alloc((n + 3) * D);
            hipLaunchKernelGGL(btk_cov_kernel, dim3(unsigned((D + 255) / 256), unsigned(n)), dim3(256), 0, stream, d_src.p,
                               int(n), a.d_dst_xyz, int(D), c0, a.range, a.zscale, d_k.p);
            check(hipGetLastError(), "cov kernel");
            // A' (D x n, ld D) = k' (D x n) K^-1 (n x n): rows 0..n-1 of A[s][d]
            check(rocblas_dgemm(blas, rocblas_operation_none, rocblas_operation_none, rocblas_int(D), rocblas_int(n),
                                rocblas_int(n), &one, d_k.p, rocblas_int(D), d_kinv.p, rocblas_int(n), &zero, dA.p,
                                rocblas_int(D)),
                  "dgemm A");
            hipLaunchKernelGGL(btk_dest_kernel, dim3(unsigned((D + 255) / 256)), dim3(256), 0, stream, dA.p, int(n),
                               d_zsrc.p, a.d_dst_xyz, int(D), o.GH_inv[0], o.GH_inv[1], o.GH_inv[2], o.GH_inv[3]);
            check(hipGetLastError(), "dest kernel");
            if (is_full) cache.valid = true;
        }
        // the steps of this pattern, in blocks: T_obs rows augmented with beta(t) and the prior gradient
        const auto& steps = pattern_steps[p];
        const size_t w = n + 3;
        for (size_t b0 = 0; b0 < steps.size(); b0 += block_steps) {
            const size_t nb = std::min(block_steps, steps.size() - b0);
            std::vector<double> tobs(nb * w);
            for (size_t j = 0; j < nb; ++j) {
                const size_t t = steps[b0 + j];
                double* row = &tobs[j * w];
                double b0v = 0.0, b1v = 0.0;
                for (size_t s = 0; s < n; ++s) {
                    const double v = a.src_values[t * S + idx[s]];
                    row[s] = v;
                    b0v += o.E_beta_w[s] * v;
                    b1v += o.E_beta_w[n + s] * v;
                }
                row[n] = b0v;
                row[n + 1] = b1v;
                row[n + 2] = a.prior_gradient[t];
            }
            d_tobs.upload(tobs.data(), tobs.size(), stream);
            const bool contiguous = steps[b0 + nb - 1] - steps[b0] == nb - 1;
            if (contiguous && !a.d_dst_index) {  // straight into the output rows
                check(rocblas_dgemm(blas, rocblas_operation_none, rocblas_operation_none, rocblas_int(D),
                                    rocblas_int(nb), rocblas_int(w), &one, dA.p, rocblas_int(D), d_tobs.p,
                                    rocblas_int(w), &zero, a.d_out + steps[b0] * a.ld_out, rocblas_int(a.ld_out)),
                      "dgemm temperatures");
            } else {
                d_C.alloc(nb * D);
                check(rocblas_dgemm(blas, rocblas_operation_none, rocblas_operation_none, rocblas_int(D),
                                    rocblas_int(nb), rocblas_int(w), &one, dA.p, rocblas_int(D), d_tobs.p,
                                    rocblas_int(w), &zero, d_C.p, rocblas_int(D)),
                      "dgemm temperatures");
                std::vector<int32_t> st(nb);
                for (size_t j = 0; j < nb; ++j) st[j] = int32_t(steps[b0 + j]);
                d_steps.upload(st.data(), nb, stream);
                hipLaunchKernelGGL(btk_scatter_kernel, dim3(unsigned((D + 255) / 256), unsigned(nb)), dim3(256), 0,
                                   stream, d_C.p, int(D), int(nb), d_steps.p, a.d_dst_index, a.d_out, a.ld_out);
                check(hipGetLastError(), "scatter kernel");
            }
            check(hipStreamSynchronize(stream), "sync");  // host buffers of this block are reused
        }
    }
}
