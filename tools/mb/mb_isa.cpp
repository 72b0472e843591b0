// Microbenchmark (GPU box, analysis only): issue and dependency costs of the instruction forms the pt_gs_k step is
// made of, for ONE wave alone on the GPU (the Brent solver's situation) and with 4 / 8 waves per SIMD.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/mb/mb_isa tools/mb/mb_isa.cpp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

#define R4(s) s s s s
#define R16(s) R4(R4(s))
#define R64(s) R16(R4(s))

template <int K>
__global__ __launch_bounds__(64) void body(const double* in, double* out, unsigned long long* cyc, int reps) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    double a = in[g & 255], b = in[(g + 1) & 255], c = in[(g + 2) & 255], d = in[(g + 3) & 255];
    float fa = (float)a, fb = (float)b;
    const double e = in[(g + 4) & 255];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        if (K == 0) asm volatile(R64("v_add_f64 %0, %0, %1\n") : "+v"(a) : "v"(b));                      // dependent f64 add
        if (K == 1) asm volatile(R16("v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4\n")
                                 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(e));                       // 4 independent chains
        if (K == 2) asm volatile(R64("v_fma_f64 %0, %0, %1, %1\n") : "+v"(a) : "v"(b));                  // dependent f64 fma
        if (K == 3) asm volatile(R64("v_add_f32 %0, %0, %1\n") : "+v"(fa) : "v"(fb));                    // dependent f32 add
        if (K == 4) asm volatile(R64("v_mov_b32 %0, 0x3ff00000\n") : "=v"(fa));                          // v_mov literal
        if (K == 5) asm volatile(R64("s_mov_b32 s0, 0x3ff00000\n") ::: "s0");                           // s_mov literal
        if (K == 6) asm volatile(R16("v_mov_b32 v40, 0\n v_mov_b32 v41, 0x3ff00000\n v_fma_f64 %0, %0, %1, v[40:41]\n v_nop\n")
                                 : "+v"(a) : "v"(b) : "v40", "v41");                                    // const via v_mov
        if (K == 7) asm volatile(R16("s_mov_b32 s0, 0\n s_mov_b32 s1, 0x3ff00000\n v_fma_f64 %0, %0, %1, s[0:1]\n v_nop\n")
                                 : "+v"(a) : "v"(b) : "s0", "s1");                                      // const via s_mov
        if (K == 8) asm volatile(R16("v_cmp_lt_f64 vcc, %0, %1\n s_and_saveexec_b64 s[0:1], vcc\n s_or_b64 exec, exec, s[0:1]\n v_add_f64 %0, %0, %1\n")
                                 : "+v"(a) : "v"(b) : "s0", "s1", "vcc");                                // cmp -> exec round trip
        if (K == 9) asm volatile(R64("v_rcp_f64 %0, %0\n") : "+v"(a));                                   // dependent rcp
        if (K == 10) asm volatile(R64("v_nop\n"));                                                       // v_nop
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[g] = a + b + c + d + fa;
    if ((threadIdx.x & 63) == 0) cyc[g / 64] = t1 - t0;
}

int main() {
    double *in, *out; unsigned long long* cyc;
    const int maxw = 8192;
    CK(hipMalloc(&in, 256 * 8)); CK(hipMalloc(&out, maxw * 64 * 8)); CK(hipMalloc(&cyc, maxw * 8));
    std::vector<double> h(256); for (int i = 0; i < 256; ++i) h[i] = 1.0 + i * 1e-3;
    CK(hipMemcpy(in, h.data(), 256 * 8, hipMemcpyHostToDevice));
    const char* names[] = {"f64 add dep", "f64 add x4 indep", "f64 fma dep", "f32 add dep", "v_mov_b32 lit",
                           "s_mov_b32 lit", "fma + 2 v_mov const", "fma + 2 s_mov const", "cmp->saveexec->or",
                           "f64 rcp dep", "v_nop"};
    const int reps = 50;
    for (int k = 0; k < 11; ++k) for (int waves : {1, 1024, 4096, 8192}) {
        if (waves > maxw) return 1;
        auto launch = [&]() {
            switch (k) {
#define C(n) case n: body<n><<<waves, 64>>>(in, out, cyc, reps); break;
                C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10)
            }
        };
        launch();
        CK(hipDeviceSynchronize());
        launch();
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> c(waves);
        CK(hipMemcpy(c.data(), cyc, waves * 8, hipMemcpyDeviceToHost));
        double s = 0; for (auto v : c) s += (double)v;
        s /= waves;
        printf("%-22s waves %5d: %6.2f cyc per instruction-slot (64 per rep)\n", names[k], waves, s / (reps * 64.0));
    }
    printf("MB_DONE\n");
    return 0;
}
