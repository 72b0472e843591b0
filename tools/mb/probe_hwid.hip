// Probe (GPU box, analysis only): where the wavefronts of 256-lane workgroups land. Each wavefront records
// HW_ID (SIMD, CU, SH, SE, TG_ID), XCC_ID and s_memtime at start / end; the workgroups hold ~38 KB of LDS, like the
// pt_gs_k kernel, so 4 are resident per CU. tools/mb/probe_hwid.py reads the dump and reports, per CU, how the
// solver wavefront of device/wave_place.h (the one on SIMD TG_ID & 3) spreads over the SIMDs among overlapping
// workgroups.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/mb/probe_hwid tools/mb/probe_hwid.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned* out, int spin) {
    __shared__ double pad[4800];  // 38.4 KB: 4 workgroups per CU
    const int w = threadIdx.x >> 6;
    pad[threadIdx.x] = threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double acc = pad[(threadIdx.x * 7) & 255];
    for (int i = 0; i < spin; ++i) acc = acc * 1.0000001 + 1e-9;
    __syncthreads();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) {
        unsigned* o = out + ((size_t)blockIdx.x * 4 + w) * 6;
        o[0] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_ID, all 32 bits
        o[1] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (3 << 11));   // XCC_ID bits 3:0
        o[2] = (unsigned)t0;
        o[3] = (unsigned)(t0 >> 32);
        o[4] = (unsigned)t1;
        o[5] = (unsigned)(t1 >> 32) + (acc == 12345.0 ? 1u : 0u);
    }
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 4096;
    const int spin = argc > 2 ? atoi(argv[2]) : 20000;
    unsigned* d;
    const size_t n = (size_t)blocks * 4 * 6;
    if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, d, spin);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<unsigned> h(n);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    FILE* f = fopen(argc > 3 ? argv[3] : "gpurun_out/probe_hwid.bin", "wb");
    fwrite(h.data(), 4, n, f);
    fclose(f);
    printf("probe: %d blocks written\n", blocks);
    hipFree(d);
    return 0;
}
