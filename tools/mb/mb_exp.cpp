// Microbenchmark (GPU box, analysis only): exp variants, lone-wave latency and 4/8-wave throughput.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -o tools/mb/mb_exp tools/mb/mb_exp.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../detmath/detmath.h"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#pragma clang fp contract(off)

static __constant__ double kc[16] = {1.4426950408889634, 6755399441055744.0, 6.93147180369123816490e-01,
    1.90821492927058770002e-10, 1.6059043836821614e-10, 2.0876756987868099e-09, 2.5052108385441720e-08,
    2.7557319223985893e-07, 2.7557319223985888e-06, 2.4801587301587302e-05, 1.9841269841269841e-04,
    1.3888888888888889e-03, 8.3333333333333333e-03, 4.1666666666666664e-02, 1.6666666666666666e-01, 0.5};

__device__ __forceinline__ double exp_tab(double x) {
    if (__builtin_fabs(x) <= 708.0) {
        typedef __attribute__((address_space(4))) const double cdouble;
        const cdouble* __restrict__ c = (const cdouble*)kc;
        asm volatile("" : "+s"(c));  // opaque: loaded with s_load, used as SGPR operands
        const double t = x * c[0] + c[1];
        const double kf = t - c[1];
        double r = __builtin_fma(-kf, c[2], x);
        r = __builtin_fma(-kf, c[3], r);
        double p = c[4];
        p = __builtin_fma(p, r, c[5]); p = __builtin_fma(p, r, c[6]); p = __builtin_fma(p, r, c[7]);
        p = __builtin_fma(p, r, c[8]); p = __builtin_fma(p, r, c[9]); p = __builtin_fma(p, r, c[10]);
        p = __builtin_fma(p, r, c[11]); p = __builtin_fma(p, r, c[12]); p = __builtin_fma(p, r, c[13]);
        p = __builtin_fma(p, r, c[14]); p = __builtin_fma(p, r, 0.5); p = __builtin_fma(p, r, 1.0);
        p = __builtin_fma(p, r, 1.0);
        return __builtin_ldexp(p, (int)kf);
    }
    return detmath::exp_general(x);
}
__device__ __forceinline__ double fma_s(double a, double b, double c) {
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
    return d;
}
__device__ __forceinline__ double exp_asm(double x) {
    if (__builtin_fabs(x) <= 708.0) {
        typedef __attribute__((address_space(4))) const double cdouble;
        const cdouble* __restrict__ c = (const cdouble*)kc;
        asm volatile("" : "+s"(c));
        const double t = x * c[0] + c[1];
        const double kf = t - c[1];
        double r = __builtin_fma(-kf, c[2], x);
        r = __builtin_fma(-kf, c[3], r);
        double p = fma_s(r, c[4], c[5]);
        p = fma_s(p, r, c[6]); p = fma_s(p, r, c[7]);
        p = fma_s(p, r, c[8]); p = fma_s(p, r, c[9]); p = fma_s(p, r, c[10]);
        p = fma_s(p, r, c[11]); p = fma_s(p, r, c[12]); p = fma_s(p, r, c[13]);
        p = fma_s(p, r, c[14]); p = __builtin_fma(p, r, 0.5); p = __builtin_fma(p, r, 1.0);
        p = __builtin_fma(p, r, 1.0);
        return __builtin_ldexp(p, (int)kf);
    }
    return detmath::exp_general(x);
}
__device__ __noinline__ double exp_tab_call(double x) { return exp_asm(x); }
__device__ __noinline__ double exp_dm_call(double x) { return detmath::exp(x); }

template <int K>
__global__ __launch_bounds__(64) void chain(const double* x0, int reps, double* out, unsigned long long* cyc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    double x = x0[g & 1023], y = x0[(g + 7) & 1023];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (K == 0) { x = detmath::exp(x) * 1e-3 - 0.5; }
        if (K == 1) { x = exp_dm_call(x) * 1e-3 - 0.5; }
        if (K == 2) { x = exp_asm(x) * 1e-3 - 0.5; }
        if (K == 3) { x = exp_tab_call(x) * 1e-3 - 0.5; }
        if (K == 4) { x = detmath::exp(x) * 1e-3 - 0.5; y = detmath::exp(y) * 1e-3 - 0.4; }   // two chains
        if (K == 5) { x = exp_asm(x) * 1e-3 - 0.5; y = exp_asm(y) * 1e-3 - 0.4; }
        if (K == 6) { x = exp_dm_call(x) * 1e-3 - 0.5; y = exp_dm_call(y) * 1e-3 - 0.4; }
        if (K == 7) { x = exp_tab_call(x) * 1e-3 - 0.5; y = exp_tab_call(y) * 1e-3 - 0.4; }
        if (K == 8) { x = detmath::log(x + 2.0) * 0.5; }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = x + y;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

__global__ void check(const double* xs, int n, int* bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = xs[i];
    const double a = exp_asm(x), b = detmath::exp(x), c = exp_tab_call(x);
    if (__double_as_longlong(a) != __double_as_longlong(b) || __double_as_longlong(c) != __double_as_longlong(b)) atomicAdd(bad, 1);
}

int main() {
    double *x0, *out; unsigned long long* cyc;
    const int maxw = 8192;
    CK(hipMalloc(&out, maxw * 64 * 8)); CK(hipMalloc(&cyc, maxw * 8)); CK(hipMalloc(&x0, 1024 * 8));
    std::vector<double> hx(1024); for (int i = 0; i < 1024; ++i) hx[i] = 0.1 + i * 1e-4;
    CK(hipMemcpy(x0, hx.data(), 1024 * 8, hipMemcpyHostToDevice));
    {
        const int n = 1 << 20;
        std::vector<double> hs(n);
        for (int i = 0; i < n; ++i) hs[i] = -750.0 + 1460.0 * ((i * 2654435761u) % n) / n;
        double* xs; int* bad; int hb = 0;
        CK(hipMalloc(&xs, n * 8)); CK(hipMalloc(&bad, 4));
        CK(hipMemcpy(xs, hs.data(), n * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(bad, &hb, 4, hipMemcpyHostToDevice));
        check<<<n / 256, 256>>>(xs, n, bad);
        CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
        printf("exp_asm vs detmath::exp on device: %d of %d differ\n", hb, n);
    }
    const char* names[] = {"exp inline", "exp call", "exp_asm inline", "exp_asm call", "2x exp inline",
                           "2x exp_asm inline", "2x exp call", "2x exp_asm call", "log inline"};
    const int creps = 400;
    for (int k = 0; k < 9; ++k) for (int waves : {1, 4096, 8192}) {
        if (waves > maxw) return 1;
        auto launch = [&](void) {
            switch (k) {
#define C(n) case n: chain<n><<<waves, 64>>>(x0, creps, out, cyc); break;
                C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8)
            }
        };
        launch(); CK(hipDeviceSynchronize());
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        double s = 0; for (auto v : c) s += (double)v;
        const int per = (k >= 4 && k <= 7) ? 2 : 1;
        printf("%-18s waves %5d: %7.1f cyc/iter (per wave), %.3g lane-exps/s\n", names[k], waves, s / waves / creps,
               (double)waves * 64 * creps * per / (ms * 1e-3));
    }
    printf("MB_DONE\n");
    return 0;
}
