// Streamed forcing loads and response stores of the cell kernels: each value is read or written once per launch.
// NT = true gives them the nontemporal hint, so the stream does not displace the step loop's scratch lines (register
// spills, the callees' saved registers) from L2 (r06: pt_gs_k and pt_ss_k).
#pragma once
#include <hip/hip_runtime.h>

namespace shyft_dev {

template <bool NT, class T>
__device__ __forceinline__ T stream_ld(const T* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT, class T>
__device__ __forceinline__ void stream_st(T* p, T v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

}  // namespace shyft_dev
