// Diagnostic entry point: device elementary functions on host-supplied inputs.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../../include/shyft_hip.h"
#include "../device/special.h"

namespace {

__global__ void math_selftest_kernel(int fn, const double* __restrict__ x, const double* __restrict__ y, size_t n,
                                     double* __restrict__ out) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double r;
    switch (fn) {
        case 0: r = shyft_dev::dexp(x[i]); break;
        case 1: r = shyft_dev::dlog(x[i]); break;
        case 2: r = shyft_dev::dpow(x[i], y[i]); break;
        case 3: r = shyft_dev::dlgamma(x[i]); break;
        default: r = shyft_dev::gamma_p(x[i], y[i]); break;
    }
    out[i] = r;
}

}  // namespace

extern "C" int shyft_hip_math_selftest(int fn, const double* x, const double* y, size_t n, double* out) {
    if (fn < 0 || fn > 4 || !x || !out || ((fn == 2 || fn == 4) && !y)) return 1;
    if (n == 0) return 0;
    double *dx = nullptr, *dy = nullptr, *dout = nullptr;
    int rc = 1;
    if (hipMalloc(&dx, n * sizeof(double)) != hipSuccess) goto done;
    if (hipMalloc(&dy, n * sizeof(double)) != hipSuccess) goto done;
    if (hipMalloc(&dout, n * sizeof(double)) != hipSuccess) goto done;
    if (hipMemcpy(dx, x, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) goto done;
    if (y && hipMemcpy(dy, y, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) goto done;
    hipLaunchKernelGGL(math_selftest_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, dx, dy, n, dout);
    if (hipGetLastError() != hipSuccess) goto done;
    if (hipMemcpy(out, dout, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) goto done;
    rc = 0;
done:
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    if (dout) (void)hipFree(dout);
    return rc;
}
