// Which wavefront of a workgroup solves the workgroup's job queue (pt_gs_k Brent jobs, pt_ss_k sca_rel_red jobs).
//
// While one wavefront solves, the workgroup's other wavefronts wait at a barrier, so the solving wavefronts of the
// workgroups resident on a CU are the CU's busy ones, and two of them on one SIMD share its issue slots while
// another SIMD idles. Wave 0's SIMD follows the dispatcher's rotation, which puts some co-resident workgroups' wave 0
// on the same SIMD (tools/mb/probe_hwid: 280 of 6,677 overlapping pairs of 256-lane workgroups). Here each
// wavefront reads its SIMD from the HW_ID hardware register (s_getreg, a register read), the workgroup publishes
// the four in LDS, and the solver is the wavefront on SIMD (HW_ID.TG_ID & 3): TG_ID is the workgroup's slot on its
// CU (0-3 with 4 resident), so co-resident workgroups solve on different SIMDs (probe: 0 of 6,677 pairs share one).
// Which wavefront solves changes no result (the same jobs, the same function); if no wavefront of the workgroup is
// on that SIMD the first one solves.
// Measured r05 (1M cells, 730-step chunks, year mean): pt_gs_k 82.7 -> 80.6 ms (January 131 -> 125, October
// 143 -> 134); rotating by block index instead (blockIdx & 3, blockIdx >> 3 & 3) changed nothing.
#pragma once
#include <hip/hip_runtime.h>

namespace shyft_dev {

// HW_ID (hwreg 4): SIMD_ID bits 5:4, TG_ID bits 19:16
__device__ __forceinline__ int hw_simd_id() { return (int)__builtin_amdgcn_s_getreg(4 | (4 << 6) | (1 << 11)); }
__device__ __forceinline__ int hw_tg_id() { return (int)__builtin_amdgcn_s_getreg(4 | (16 << 6) | (3 << 11)); }

// every wavefront's first lane records its SIMD (wsimd[B / 64]); a barrier must follow before solver_lane0
__device__ __forceinline__ void publish_wave_simd(int* wsimd) {
    if ((threadIdx.x & 63) == 0) wsimd[threadIdx.x >> 6] = hw_simd_id();
}

// the first lane of the solving wavefront
template <int B>
__device__ __forceinline__ int solver_lane0(const int* wsimd) {
    if (B <= 64) return 0;
    const int want = hw_tg_id() & 3;
    for (int w = 0; w < B / 64; ++w)
        if (wsimd[w] == want) return w * 64;
    return 0;
}

}  // namespace shyft_dev
