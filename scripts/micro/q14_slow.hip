// Microbenchmark (diagnostic, not product): shader clocks of one exact
// tostring/tonumber round trip (rlq::q14) on the fast path and on the
// big-integer slow path (|x| < 1e-9), one lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../distributed-rate-limiter_amd/csrc/rl_q14.h"

__global__ void k_q14(double x0, double step, int iters, double* out, unsigned long long* cyc) {
    double acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) acc += rlq::q14(x0 + step * i + acc * 1e-30);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[0] = acc;
    cyc[0] = t1 - t0;
}

int main() {
    double* out;
    unsigned long long* cyc;
    hipMalloc(&out, 8);
    hipMalloc(&cyc, 8);
    const double xs[] = {0.37, 3.7e-9, 3.7e-12, 3.7e-300};
    for (double x : xs) {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        k_q14<<<1, 1>>>(x, x * 1e-9, 4, out, cyc);
        hipDeviceSynchronize();
        hipEventRecord(a);
        k_q14<<<1, 1>>>(x, x * 1e-9, 16, out, cyc);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        unsigned long long c;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("x %g: %.0f clocks per q14, %.1f us per q14 (events)\n", x, c / 16.0, ms * 1e3 / 16);
    }
    return 0;
}
