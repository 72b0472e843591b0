// Device unit probe: evaluates device functions on given inputs and prints them.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../shyft_amd/csrc/device/ptgsk_dev.h"
using namespace shyft_dev;
__global__ void k(double* out, const double* in) {
    out[0] = gs_corr_lwc(in[0], in[1], in[2], in[3], in[4]);
    out[1] = gamma_p(in[1], in[0] / in[2]);
    out[2] = gs_calc_q(in[3], in[4], 0.108, lgamma(in[3]), lgamma(in[3] + 1.0));
    out[3] = gs_corr_lwc(4.0, 6.0, 1.0, 5.0, 2.0);
    out[4] = lgamma(in[1]);
}
int main() {
    double h_in[5] = {31.305, 0.66109370675674173 / 1.0, 0.1075697454579585 / 0.66109370675674173, 5.5212677668009338,
                      0.82499057947987453 / 5.5212677668009338};
    double *d_in, *d_out, h_out[5];
    hipMalloc(&d_in, sizeof h_in); hipMalloc(&d_out, sizeof h_out);
    hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
    k<<<1, 1>>>(d_out, d_in);
    hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
    for (int i = 0; i < 5; ++i) printf("out[%d] = %.17g\n", i, h_out[i]);
}
