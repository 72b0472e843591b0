// Microbenchmark (GPU box, analysis only): latency and throughput of the pt_gs_k Brent job (gs_corr_lwc) and of
// the elementary functions, on January jobs recorded from the oracle (tools/mb/jobs_jan.bin: z1 a1 b1 a2 b2).
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -o tools/mb/mb_brent tools/mb/mb_brent.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../shyft_amd/csrc/device/ptgsk_dev.h"
#include "../../shyft_amd/csrc/device/gs_brent.h"
using namespace shyft_dev;
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void prep(const double* J, double* q1, double* lga2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* j = J + 5 * i;
    q1[i] = gs_calc_q(j[1], j[2], j[0], dlgamma(j[1]));
    lga2[i] = dlgamma(j[3]);
}

// the lean solver against gs_corr_lwc on every job, bit for bit (q1 given, and q1 = NaN)
__global__ void check_lean(const double* J, const double* q1, const double* lga2, int n, int* bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* j = J + 5 * i;
    for (int mode = 0; mode < 2; ++mode) {
        const double q = mode ? __builtin_nan("") : q1[i];
        const double r0 = gs_corr_lwc(j[0], j[1], j[2], j[3], j[4], q, lga2[i]);
        const double r1 = gs_corr_lwc_lean(j[0], j[1], j[2], j[3], j[4], q, lga2[i]);
        if (__double_as_longlong(r0) != __double_as_longlong(r1)) atomicAdd(bad, 1);
    }
}

template <int LEAN>
__global__ __launch_bounds__(64) void solve2(const double* J, const double* q1, const double* lga2, int n, int reps,
                                             int active, double* out, unsigned long long* cyc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = (int)(((unsigned long long)g * 7919ull) % (unsigned long long)n);
    const double* j = J + 5 * i;
    double z1 = j[0], a1 = j[1], b1 = j[2], a2 = j[3], b2 = j[4], q = q1[i], lg = lga2[i];
    double acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if ((int)(threadIdx.x & 63) < active)
        for (int r = 0; r < reps; ++r)
            acc += LEAN ? gs_corr_lwc_lean(z1 + 0.0 * acc, a1, b1, a2, b2, q, lg)
                        : gs_corr_lwc(z1 + 0.0 * acc, a1, b1, a2, b2, q, lg);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = acc;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

// every lane solves job (gid % n), reps times (each solve's z1 depends on the previous result by +0*r)
__global__ __launch_bounds__(64) void solve(const double* J, const double* q1, const double* lga2, int n, int reps,
                                            int active, double* out, unsigned long long* cyc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = (int)(((unsigned long long)g * 7919ull) % (unsigned long long)n);  // 64-bit: g * 7919 overflows int
    const double* j = J + 5 * i;
    double z1 = j[0], a1 = j[1], b1 = j[2], a2 = j[3], b2 = j[4], q = q1[i], lg = lga2[i];
    double acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if ((int)(threadIdx.x & 63) < active)
        for (int r = 0; r < reps; ++r) acc += gs_corr_lwc(z1 + 0.0 * acc, a1, b1, a2, b2, q, lg);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = acc;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

// dependent chain of f evaluations of the Brent solver (gs_calc_q at the job's a2, b2; z walks over [0, z1])
__global__ __launch_bounds__(64) void calcq(const double* J, const double* lga2, int n, int reps, double* out,
                                            unsigned long long* cyc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = (int)(((unsigned long long)g * 7919ull) % (unsigned long long)n);
    const double* j = J + 5 * i;
    const double z1 = j[0], a2 = j[3], b2 = j[4], lg = lga2[i];
    double acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        const double z = z1 * (0.05 + 0.09 * (r % 10)) + 0.0 * acc;
        acc += gs_calc_q(a2, b2, z, lg);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = acc;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

// kirchner_step (dopri5, one hour) per lane, reps dependent calls: per-call instruction counts under rocprofv3 --pmc
__global__ __launch_bounds__(64) void kirch(const double* x0, int reps, double* out, unsigned long long* cyc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    double q = 0.5 + x0[g & 1023];
    double acc = 0.0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        double qa;
        kirchner_step(q, qa, 0.4 + 0.01 * (r & 7), 0.05, 1.0, -2.439, 0.966, -0.10);
        acc += qa;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = acc + q;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

template <int K>
__global__ __launch_bounds__(64) void chain(const double* x0, int reps, double* out, unsigned long long* cyc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    double x = x0[g & 1023];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (K == 0) x = dexp(x) * 1e-3 - 0.5;                  // out-of-line detmath exp
        if (K == 1) x = detmath::exp(x) * 1e-3 - 0.5;          // inlined detmath exp
        if (K == 2) x = __builtin_fma(x, 0.999, 1e-3);        // one fp64 fma
        if (K == 3) x = 1.0 / (x + 2.0);                      // fp64 division
        if (K == 4) x = dlog(x + 2.0) * 0.5;                  // out-of-line log
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = x;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

static double mean_cyc(const std::vector<unsigned long long>& c) {
    double s = 0; for (auto v : c) s += (double)v; return s / c.size();
}

int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "tools/mb/jobs_jan.bin", "rb");
    if (!f) { printf("no jobs file\n"); return 1; }
    std::vector<double> h(16384 * 5);
    const int n = (int)(fread(h.data(), sizeof(double), h.size(), f) / 5);
    fclose(f);
    double *J, *q1, *lg, *out, *x0; unsigned long long* cyc;
    const int maxw = 16384;
    CK(hipMalloc(&J, h.size() * 8)); CK(hipMalloc(&q1, n * 8)); CK(hipMalloc(&lg, n * 8));
    CK(hipMalloc(&out, maxw * 64 * 8)); CK(hipMalloc(&cyc, maxw * 8)); CK(hipMalloc(&x0, 1024 * 8));
    CK(hipMemcpy(J, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> hx(1024); for (int i = 0; i < 1024; ++i) hx[i] = 0.1 + i * 1e-4;
    CK(hipMemcpy(x0, hx.data(), 1024 * 8, hipMemcpyHostToDevice));
    prep<<<(n + 63) / 64, 64>>>(J, q1, lg, n);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    {
        int* bad; int hb = 0;
        CK(hipMalloc(&bad, 4)); CK(hipMemcpy(bad, &hb, 4, hipMemcpyHostToDevice));
        check_lean<<<(n + 63) / 64, 64>>>(J, q1, lg, n, bad);
        CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
        printf("lean vs gs_corr_lwc: %d of %d results differ\n", hb, 2 * n);
    }
    for (int lean = 0; lean < 2; ++lean) for (int active : {64, 22}) for (int waves : {1, 1024, 4096}) {
        const int reps = 4;
        auto go = [&]() {
            if (lean) solve2<1><<<waves, 64>>>(J, q1, lg, n, reps, active, out, cyc);
            else solve2<0><<<waves, 64>>>(J, q1, lg, n, reps, active, out, cyc);
        };
        go();
        CK(hipEventRecord(e0)); go(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        printf("%s active %2d waves %5d: %8.0f cyc/job (per wave), %.3g jobs/s\n", lean ? "lean " : "brent", active,
               waves, mean_cyc(c) / reps, (double)waves * active * reps / (ms * 1e-3));
    }
    if (getenv("MB_LEAN")) { printf("MB_DONE\n"); return 0; }
    // Brent jobs: waves = 1, 256 (1/CU), 1024 (1/SIMD), 4096 (4/SIMD), 8192
    const int reps = 4;
    for (int active : {64, 22}) for (int waves : {1, 1024, 4096}) {
        if (waves > maxw) { printf("grid too large\n"); return 1; }
        solve<<<waves, 64>>>(J, q1, lg, n, reps, active, out, cyc);
        CK(hipEventRecord(e0));
        solve<<<waves, 64>>>(J, q1, lg, n, reps, active, out, cyc);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        const double jobs = (double)waves * active * reps;
        printf("brent active %2d waves %5d: %8.0f cyc/job (per wave), wall %.3f ms, %.3g jobs/s\n", active, waves,
               mean_cyc(c) / reps, ms, jobs / (ms * 1e-3));
    }
    for (int waves : {1, 1024, 4096}) {
        const int creps = 40;
        calcq<<<waves, 64>>>(J, lg, n, creps, out, cyc);
        CK(hipEventRecord(e0));
        calcq<<<waves, 64>>>(J, lg, n, creps, out, cyc);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        printf("calc_q        waves %5d: %7.0f cyc/eval (per wave), %.3g lane-evals/s\n", waves, mean_cyc(c) / creps,
               (double)waves * 64 * creps / (ms * 1e-3));
    }
    for (int waves : {1, 4096}) {
        const int kreps = 20;
        kirch<<<waves, 64>>>(x0, kreps, out, cyc);
        CK(hipEventRecord(e0));
        kirch<<<waves, 64>>>(x0, kreps, out, cyc);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        printf("kirchner_step waves %5d: %7.0f cyc/call (per wave)\n", waves, mean_cyc(c) / kreps);
    }
    if (getenv("MB_QUICK")) { printf("MB_DONE\n"); return 0; }
    const char* names[] = {"dexp (call)", "exp (inline)", "fma", "div", "dlog (call)"};
    const int creps = 1000;
    for (int k = 0; k < 5; ++k) for (int waves : {1, 1024, 4096, 8192}) {
        auto launch = [&](void) {
            switch (k) {
                case 0: chain<0><<<waves, 64>>>(x0, creps, out, cyc); break;
                case 1: chain<1><<<waves, 64>>>(x0, creps, out, cyc); break;
                case 2: chain<2><<<waves, 64>>>(x0, creps, out, cyc); break;
                case 3: chain<3><<<waves, 64>>>(x0, creps, out, cyc); break;
                default: chain<4><<<waves, 64>>>(x0, creps, out, cyc); break;
            }
        };
        launch();
        CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        printf("%-13s waves %5d: %7.1f cyc/op (per wave), %.3g lane-ops/s\n", names[k], waves, mean_cyc(c) / creps,
               (double)waves * 64 * creps / (ms * 1e-3));
    }
    printf("MB_DONE\n");
    return 0;
}
