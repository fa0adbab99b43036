// Microbenchmark (diagnostic, not product): shader clocks per dependent
// token-bucket exact step (tb_step_d) and per wave scan, one wave alone on its
// SIMD vs. sharing the SIMD with busy waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../distributed-rate-limiter_amd/csrc/rl_replay.h"
using namespace rl;

__global__ void k_lat(double* out, uint64_t* cyc, int iters, int busy) {
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const double P = 1e14, R = 1e-14;
    double D = 5.0e13 + lane, acc = 0;
    if (wave == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; i++) {
            double tk;
            double Dn = tb_step_d<QM_DEC>(D, P, R, 1.3e-5, 1.0, tk);
            int32_t f = (int32_t)(Dn - (D + 1.3e9));
            int32_t inc = (int32_t)wave_scan_u32((uint32_t)f, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            D = Dn - (double)(inc & 1) - 1.2e9;
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) cyc[0] = t1 - t0;
        acc = D;
    } else if (busy) {
        double x = lane;
        for (int i = 0; i < iters * 40; i++) x = x * 1.0000001 + 0.5;
        acc = x;
    }
    out[threadIdx.x] = acc;
}

int main() {
    double* out; uint64_t* cyc;
    hipMalloc(&out, 8 * 1024); hipMalloc(&cyc, 8);
    for (int busy = 0; busy < 2; busy++)
        for (int nw : {1, 5, 8}) {
            k_lat<<<1, 64 * nw>>>(out, cyc, 1000, busy);
            hipDeviceSynchronize();
            uint64_t c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("waves %d busy %d: %.0f clocks per step+scan\n", nw, busy, c / 1000.0);
        }
    return 0;
}
