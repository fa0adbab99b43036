// Microbenchmark (diagnostic, not product): shader clocks of one chain
// window resolution (ch_resolve) on synthetic tiles, wave 0 alone in its block
// (busy = 0) or next to waves running a dependent FP64 chain (busy = 1).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../distributed-rate-limiter_amd/csrc/rl_replay.h"
using namespace rl;

__global__ __launch_bounds__(512) void k_res(uint64_t* cyc, uint32_t* iters_out, int reps, int busy, int nper,
                                             TbRuns runs) {
    __shared__ ChainShared sh;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const double P = 1e14, R = 1e-14;
    // 6 tiles of 256 requests, add = 1.3e-5 (r = 1.3e9 units); nper near entries per tile
    if (wave == 0) {
        for (int t = 0; t < CH_NP; t++) {
            if (lane == 0) {
                ChTile& T = sh.tile[1][t];
                T.S = (int64_t)256 * 1300000000LL;
                T.ymin = 1e300; T.cmax = 256 * 1.3e9; T.cmin = 1.3e9; T.dmax = 1e14; T.ev = NO_STOP; T.nc = nper;
            }
            for (int k = lane; k < CH_NE; k += 64) {
                sh.ne_pred[1][t][k] = (double)(k * (256 / (nper ? nper : 1))) * 1.3e9;
                sh.ne_add[1][t][k] = 1.3e-5 + 5e-15 * (k & 3);     // frac(add*P) = 0.5 +- small: near ties
                sh.ne_th[1][t][k] = 1.0;
            }
            sh.ne_rank[1][t][lane] = 0;
        }
    }
    __syncthreads();
    ChState s;
    s.D = 20000000000000LL; s.E = -1; s.mode = QM_DEC; s.cfirst = 0; s.ccnt = CH_W; s.pfirst = CH_W;
    s.pbuf = 0; s.cbuf = 1; s.hot = 0;
    ReqArgs a{};
    double acc = 0;
    if (wave == 0) {
        uint32_t iters = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; r++) {
            s.D += 1;
            ChOutcome o = ch_resolve<QM_DEC>(sh, s, P, R, a, runs, nullptr, iters, nullptr);
            acc += (double)o.D;
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0) { cyc[0] = t1 - t0; iters_out[0] = iters; }
    } else if (busy) {
        double x = lane;
        for (int i = 0; i < reps * 2000; i++) x = x * 1.0000001 + 0.5;
        acc = x;
    }
    if (acc == 12345.0) cyc[1] = 1;
}

int main() {
    uint64_t* cyc; uint32_t* it;
    hipMalloc(&cyc, 16); hipMalloc(&it, 4);
    TbRuns runs;
    hipMalloc(&runs.len, 2 * 4096); hipMalloc(&runs.E, 2 * 4096); hipMalloc(&runs.D0, 8 * 4096); hipMalloc(&runs.D1, 8 * 4096);
    for (int busy = 0; busy < 2; busy++)
        for (int nper : {0, 4, 9, 16}) {
            k_res<<<1, 512>>>(cyc, it, 200, busy, nper, runs);
            if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 1; }
            uint64_t c; uint32_t i;
            hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost); hipMemcpy(&i, it, 4, hipMemcpyDeviceToHost);
            printf("busy %d near/tile %2d: %.0f clocks per window, %.2f iterations per window\n", busy, nper,
                   c / 200.0, i / 200.0);
        }
    return 0;
}
