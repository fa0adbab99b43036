// rl_replay.h -- per-key segment replay kernels.
//
// After the sort, the requests of one state-table slot (one user key) form a
// contiguous segment in arrival order.  Replaying a segment applies, request
// by request, exactly what the reference does per call: the Go pre-arithmetic,
// the Lua script against the key's Redis state, and the Go post-arithmetic
// (rl_semantics.h).  State is gathered from the table once per segment, kept in
// registers across the segment, and scattered back once.
#pragma once

#include <hip/hip_runtime.h>

#include "rl_semantics.h"
#include "rl_table.h"

namespace rl {

struct ReqArgs {
    const uint64_t* key;
    const int64_t* ts;
    const int64_t* n;
    const uint32_t* cfg;
    const int64_t* sms;   // nullable: server clock = floor(ts / 1e6)
    uint8_t* dec;
    int64_t* rem;
    int64_t* retry;
    int64_t* reset;
    double* tok;          // nullable
};

__device__ inline int64_t req_server_ms(const ReqArgs& a, uint32_t i, int64_t t) {
    return a.sms ? a.sms[i] : floor_div(t, 1000000LL);
}

__device__ inline void write_out(const ReqArgs& a, uint32_t i, const Out& o) {
    a.dec[i] = o.decision;
    a.rem[i] = o.remaining;
    a.retry[i] = o.retry;
    a.reset[i] = o.reset_at;
    if (a.tok) a.tok[i] = o.tokens;
}

// end of the run of `k0` starting at j0 in the sorted keys (galloping search)
__device__ inline uint32_t seg_end(const uint32_t* sk, uint32_t m, uint32_t j0, uint32_t k0) {
    uint32_t lo = j0, step = 1;
    while (lo + step < m && sk[lo + step] == k0) { lo += step; step <<= 1; }
    uint32_t hi = (lo + step < m) ? lo + step : m;   // sk[hi] != k0 or hi == m
    while (hi - lo > 1) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (sk[mid] == k0) lo = mid; else hi = mid;
    }
    return lo + 1;
}

__device__ inline void replay_tb_serial(TbEntry* e, const uint32_t* sv, uint32_t j0, uint32_t j1,
                                        const CfgDev* cfgs, int32_t profile, const ReqArgs& a) {
    TbState st{e->tok, e->last, e->when};
    for (uint32_t j = j0; j < j1; j++) {
        uint32_t i = sv[j];
        int64_t t = a.ts[i];
        const CfgDev& c = cfgs[a.cfg[i]];
        Out o = tb_step(st, t, a.n[i], req_server_ms(a, i, t), c, profile);
        write_out(a, i, o);
    }
    e->tok = st.tok;
    e->last = st.last;
    e->when = st.when;
}

__device__ inline void replay_win_serial(WinEntry* e, const uint32_t* sv, uint32_t j0, uint32_t j1,
                                         const CfgDev* cfgs, int32_t profile, const ReqArgs& a,
                                         uint32_t* eflags) {
    WinState w;
    w.s[0] = e->s[0];
    w.s[1] = e->s[1];
    uint32_t ef = 0;
    for (uint32_t j = j0; j < j1; j++) {
        uint32_t i = sv[j];
        int64_t t = a.ts[i];
        const CfgDev& c = cfgs[a.cfg[i]];
        int64_t s_ms = req_server_ms(a, i, t);
        Out o = (c.alg == ALG_SLIDING_WINDOW) ? sw_step(w, t, a.n[i], s_ms, c, profile, ef)
                                              : fw_step(w, t, a.n[i], s_ms, c, profile, ef);
        write_out(a, i, o);
    }
    e->s[0] = w.s[0];
    e->s[1] = w.s[1];
    if (ef) atomicOr(eflags, ef);
}

// one thread per segment (grid-stride over the unordered segment list)
__global__ __launch_bounds__(256) void k_replay_serial(
    const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv, uint32_t m,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ nseg_p, uint32_t win_base,
    TbEntry* tb, WinEntry* win, const CfgDev* __restrict__ cfgs, int32_t profile, ReqArgs a,
    uint32_t* eflags) {
    const uint32_t nseg = *nseg_p;
    for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < nseg; u += gridDim.x * blockDim.x) {
        uint32_t j0 = seg_start[u];
        uint32_t k0 = sk[j0];
        uint32_t j1 = seg_end(sk, m, j0, k0);
        if (k0 < win_base) replay_tb_serial(&tb[k0], sv, j0, j1, cfgs, profile, a);
        else replay_win_serial(&win[k0 - win_base], sv, j0, j1, cfgs, profile, a, eflags);
    }
}

}  // namespace rl
