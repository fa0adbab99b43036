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
#include "rl_sort.h"
#include "rl_table.h"
#include "rl_window.h"

namespace rl {

struct ReqArgs {
    const uint64_t* key;
    const int64_t* ts;
    const int64_t* n;
    const uint32_t* cfg;
    const int64_t* sms;   // nullable: server clock = floor(ts / 1e6) (also in sorted order)
    uint8_t* dec;
    int64_t* rem;
    int64_t* retry;
    int64_t* reset;
    double* tok;          // nullable
    const uint8_t* fresh = nullptr;   // sorted order, nullable: the request inserted its key (REC_FRESH)
};

// State-independent token-bucket quantities of each request (sorted order),
// computed in the permute pass: the previous request of the same key is the
// previous sorted position (or, for a segment head, the table entry).  The
// rest of the script's state-free inputs are computed where they are used:
// reset_at in the finish (tb_result_reset), last_refill and the TTL of a
// segment's last request at its end (tb_store_end).
struct TbPre {
    double* add;       // elapsed * refill_rate (tokenbucket.go:36-37); NaN when HMGET finds
                       // no live key (tokenbucket.go:31-34: tokens = capacity, add = 0).
                       // A segment head's add depends on the table state, so the
                       // replay computes it (tb_head_add); k_permute fills the rest
    double* th;        // min(capacity, float64(n)): the script step allows or clamps
                       // exactly when capacity-free sum >= th (tokenbucket.go:38-43)
};

__device__ inline int64_t req_server_ms(const ReqArgs& a, uint32_t i, int64_t t) {
    return a.sms ? a.sms[i] : floor_div(t, 1000000LL);
}

// the stored state after a token-bucket segment's last request j: HSET
// last_refill = tostring(now) and the EXPIRE (tokenbucket.go:48-49)
__device__ inline void tb_store_end(TbEntry* e, double tok, uint32_t j, const CfgDev* cfgs, int32_t profile,
                                    const ReqArgs& a) {
    const int64_t t = a.ts[j];
    e->tok = tok;
    e->last = lua_tostring_roundtrip((double)t / 1e9, profile);
    e->when = expire_when(cfgs[a.cfg[j]].ttl_tb, req_server_ms(a, j, t));
}

// window counters: the replay writes the decision and Remaining only (in the
// value slot, as int64 bits); reset_at and retry_after are functions of the
// request's time and config that the finish evaluates (finish_result)
__device__ inline void write_out(const ReqArgs& a, uint32_t i, const Out& o) {
    a.dec[i] = o.decision;
    a.tok[i] = __longlong_as_double(o.remaining);
}

// token bucket: replay writes the decision and the unquantized tokens only;
// remaining/retry_after/reset_at are functions of (decision, tokens, n, time,
// config) that the finish evaluates (tokenbucket.go:114-130,161-165;
// tb_result below)
__device__ inline void write_out_tb(const ReqArgs& a, uint32_t i, uint8_t dec, double tokens) {
    a.dec[i] = dec;
    a.tok[i] = tokens;
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

// Replay kernels read the batch in SORTED order: k_permute has copied each
// request's fields to position j of its segment (coalesced loads, one level)
// and results are written at j (coalesced stores); k_unpermute moves them to
// the caller's order.  ReqArgs here always points at the permuted buffers.
struct Req {
    uint32_t c;
    int64_t t, n, sms;
};

__device__ inline Req load_req(const ReqArgs& a, uint32_t j) {
    Req r;
    r.t = a.ts[j];
    r.n = a.n[j];
    r.c = a.cfg[j];
    r.sms = req_server_ms(a, j, r.t);
    return r;
}

// one token-bucket script execution on precomputed inputs (tb_step's
// state-dependent part: tokenbucket.go:32-51 + 114-130)
__device__ inline Out tb_chain_step(double& tok, bool alive, double add, int64_t n, int64_t reset_at,
                                    const CfgDev& c, int32_t profile) {
    Out o;
    const double capacity = c.limit_d;
    double tokens = alive ? tok : capacity;
    double sum = tokens + add;
    tokens = (sum < capacity) ? sum : capacity;           // math.min(capacity, sum)
    bool allowed = false;
    if (tokens >= (double)n) { tokens = tokens - (double)n; allowed = true; }
    tok = lua_tostring_roundtrip(tokens, profile);
    int64_t rem = go_f2i(floor(tokens));
    o.tokens = tokens;
    o.decision = allowed ? DEC_ALLOWED : DEC_DENIED;
    o.remaining = rem;
    o.reset_at = reset_at;
    o.retry = 0;
    if (!allowed) {
        int64_t need = wsub(n, rem);
        double w = need == 1 ? c.inv_rate : (double)need / c.rate;   // tokensNeeded / refillRate
        int64_t d = go_f2i(w * 1e9);
        o.retry = d < 0 ? 0 : d;
    }
    return o;
}

// add of a segment head: its predecessor is the table entry (the state after
// the previous batch), read at replay time
__device__ inline double tb_head_add(const TbEntry* e, uint32_t j0, const CfgDev* cfgs, int32_t profile,
                                     const ReqArgs& a) {
    const CfgDev& C = cfgs[a.cfg[j0]];
    const double now = (double)a.ts[j0] / 1e9;
    return key_alive(e->when, req_server_ms(a, j0, a.ts[j0]), profile) ? (now - e->last) * C.rate
                                                                          : __builtin_nan("");
}

// fresh: the batch inserted the key (its entry holds the absent state, not read)
__device__ inline void replay_tb_serial(TbEntry* e, uint32_t j0, uint32_t j1, const CfgDev* cfgs,
                                        int32_t profile, const ReqArgs& a, const TbPre& pre, bool fresh = false) {
    double tok = fresh ? 0.0 : e->tok;
    const double add0 = fresh ? __builtin_nan("") : tb_head_add(e, j0, cfgs, profile, a);
    for (uint32_t j = j0; j < j1; j++) {
        const double add = j == j0 ? add0 : pre.add[j];
        const bool alive = add == add;
        Out o = tb_chain_step(tok, alive, alive ? add : 0.0, a.n[j], 0, cfgs[a.cfg[j]], profile);
        write_out_tb(a, j, o.decision, o.tokens);
    }
    tb_store_end(e, tok, j1 - 1, cfgs, profile, a);
}

// requests [j0, j1) of one window segment, one by one, from state w
__device__ inline void replay_win_steps(WinState& w, const Spill& S, uint32_t j0, uint32_t j1, const CfgDev* cfgs,
                                        int32_t profile, const ReqArgs& a, uint32_t& ef) {
    if (j0 >= j1) return;
    Req cur = load_req(a, j0);
    for (uint32_t j = j0; j < j1; j++) {
        Req nxt = cur;
        if (j + 1 < j1) nxt = load_req(a, j + 1);
        const CfgDev& c = cfgs[cur.c];
        Out o = (c.alg == ALG_SLIDING_WINDOW) ? sw_step(w, S, cur.t, cur.n, cur.sms, c, profile, ef)
                                              : fw_step(w, S, cur.t, cur.n, cur.sms, c, profile, ef);
        write_out(a, j, o);
        cur = nxt;
    }
}

// fresh: one request on a key the batch inserted -- the absent state, not
// read (one request on two free slots never reaches the spill, which alone
// needs the key)
__device__ inline void replay_win_serial(WinEntry* e, const Spill& S, uint32_t j0, uint32_t j1,
                                         const CfgDev* cfgs, int32_t profile, const ReqArgs& a, uint32_t* eflags,
                                         bool fresh = false) {
    WinState w;
    if (fresh) {
        w.key = EMPTY_KEY;
        w.nspill = 0;
        for (int k = 0; k < 2; k++) w.s[k] = WinSlot{0, 0, ABSENT};
    } else {
        w = win_load(e);
    }
    uint32_t ef = 0;
    replay_win_steps(w, S, j0, j1, cfgs, profile, a, ef);
    win_store(e, w);
    if (ef) atomicOr(eflags, ef);
}

struct TbQ {
    int64_t D;
    int32_t E;
};

__device__ inline TbQ tb_quant(double x, int32_t profile) {
    if (x == 0.0 || !(x - x == 0.0)) return TbQ{0, 0};
    if (profile == PROFILE_REDIS7) {
        double ax = x < 0 ? -x : x;
        int64_t D;
        int E;
        if (!rlq::dec14_fast(ax, D, E)) rlq::dec14_slow(ax, D, E);
        return TbQ{x < 0 ? -D : D, E};
    }
    int e;
    double m = frexp(x, &e);
    return TbQ{(int64_t)ldexp(m, 53), e - 53};
}

__device__ inline double tb_value(int64_t D, int32_t E, int32_t profile) {
    if (D == 0) return 0.0;
    if (profile == PROFILE_REDIS7) {
        double v = rlq::dec14_value(D < 0 ? -D : D, E);
        return D < 0 ? -v : v;
    }
    return ldexp((double)D, E);
}

// Barrier for LDS hand-offs only.  __syncthreads() is a workgroup-scope
// fence on gfx950 and waits for every outstanding global store (vmcnt(0));
// the replay rounds scatter results to HBM between barriers and must not wait
// for them.  LDS writes are complete once lgkmcnt reaches 0.
__device__ inline void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// 64-bit wave64 inclusive scan with DPP row shifts and row broadcasts (GFX9
// family): 6 steps of two v_mov_dpp + a 64-bit add, no LDS round trips.
template <int CTRL, int ROW_MASK>
__device__ inline int64_t dpp_add_step(int64_t inc) {
    uint32_t lo = (uint32_t)inc, hi = (uint32_t)((uint64_t)inc >> 32);
    // old = 0: lanes with no source (or outside ROW_MASK) contribute 0
    uint32_t slo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, CTRL, ROW_MASK, 0xf, false);
    uint32_t shi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, CTRL, ROW_MASK, 0xf, false);
    return inc + (int64_t)(((uint64_t)shi << 32) | slo);
}

__device__ inline int64_t wave_incl_scan_i64(int64_t v) {
    v = dpp_add_step<0x111, 0xf>(v);   // row_shr:1
    v = dpp_add_step<0x112, 0xf>(v);   // row_shr:2
    v = dpp_add_step<0x114, 0xf>(v);   // row_shr:4
    v = dpp_add_step<0x118, 0xf>(v);   // row_shr:8
    v = dpp_add_step<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
    v = dpp_add_step<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
    return v;
}

// configs cached in LDS per block (when the engine has at most MAX_LCFG)
constexpr int MAX_LCFG = 32;
constexpr double TAU_DEC = 0.03;   // > 0.0222: far lanes are exact by the bound

enum : int { QM_NONE = 0, QM_DEC = 1, QM_BIN = 2, QM_XDEC = 3 };   // QM_XDEC: rl_tb_xdec.h

struct TbEval {
    double tokens;
    bool allowed;
    bool clamped;
    bool inrange;   // Dact is the canonical stored representation in this decade
    int64_t Dact;
};

// the script step from a stored state given as digits Dpred in (mode, E)
__device__ inline TbEval tb_eval(int mode, int64_t Dpred, int32_t E, double P, double R, bool alive, double add,
                                 double cap, double nd, int32_t profile) {
    TbEval v;
    double T;
    if (!alive) T = cap;
    // strtod("D e(E-13)"): |D| < 2^47 and 10^k (k <= 22) are exact doubles,
    // so one correctly rounded division is strtod's result (Clinger's fast
    // path); RN is sign-symmetric
    else if (mode == QM_DEC) T = (double)Dpred / P;
    else if (mode == QM_BIN) T = (double)Dpred * R;                      // exact: R = 2^E
    else T = tb_value(Dpred, E, profile);
    const double sum = T + add;
    v.clamped = !(sum < cap);
    double tokens = v.clamped ? cap : sum;                               // math.min(capacity, sum)
    v.allowed = tokens >= nd;
    if (v.allowed) tokens = tokens - nd;
    v.tokens = tokens;
    v.Dact = 0;
    v.inrange = false;
    const double at = tokens < 0.0 ? -tokens : tokens;                   // %.14g is sign-symmetric
    if (mode == QM_DEC) {
        if (at > 0.0 && at * P < 1.4e14) {
            v.Dact = rlq::round_scaled_P(at, P);
            // the exact at*P must not be below 1e13: [1e13 - 0.5, 1e13) rounds to
            // 1e13 here, while %.14g keeps 14 digits of the decade below
            const double p = at * P, err = __builtin_fma(at, P, -p);
            const bool ge_lo = p > 1e13 || (p == 1e13 && err >= 0.0);
            v.inrange = ge_lo && v.Dact < 100000000000000LL;
        }
    } else if (mode == QM_BIN) {
        const double w = at * P;                                         // exact scaling
        if (w >= 4503599627370496.0 && w < 9007199254740992.0) {
            v.Dact = (int64_t)w;
            v.inrange = (double)v.Dact == w;
        }
    }
    if (tokens < 0.0) v.Dact = -v.Dact;
    return v;
}

__device__ inline Out tb_outputs(const TbEval& v, int64_t nn, int64_t reset_at, double rate, double inv_rate) {
    Out o;
    const int64_t rem = go_f2i(floor(v.tokens));
    o.tokens = v.tokens;
    o.decision = v.allowed ? DEC_ALLOWED : DEC_DENIED;
    o.remaining = rem;
    o.reset_at = reset_at;
    o.retry = 0;
    if (!v.allowed) {
        const int64_t need = wsub(nn, rem);
        // tokensNeeded / refillRate (tokenbucket.go:124-126); 1/rate precomputed
        const double w = need == 1 ? inv_rate : (double)need / rate;
        const int64_t d = go_f2i(w * 1e9);
        o.retry = d < 0 ? 0 : d;
    }
    return o;
}

// generic 32-bit wave64 inclusive scan with DPP; `op(self, earlier)`
template <int CTRL, int RM>
__device__ inline uint32_t dpp32(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, 0xf, false);
}
template <typename Op>
__device__ inline uint32_t wave_scan_u32(uint32_t v, uint32_t ident, Op op) {
    v = op(v, dpp32<0x111, 0xf>(v, ident));
    v = op(v, dpp32<0x112, 0xf>(v, ident));
    v = op(v, dpp32<0x114, 0xf>(v, ident));
    v = op(v, dpp32<0x118, 0xf>(v, ident));
    v = op(v, dpp32<0x142, 0xa>(v, ident));
    v = op(v, dpp32<0x143, 0xc>(v, ident));
    return v;
}
__device__ inline uint32_t wave_min_u32(uint32_t v) {
    v = wave_scan_u32(v, 0xffffffffu, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ inline int64_t readlane_i64(int64_t v, uint32_t l) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)l);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), (int)l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// one segment: the requests of one state-table slot, [j0, j0 + len) sorted
struct SegRec {
    uint32_t j0;
    uint32_t len;
};

// the segment work lists k_segments builds (see there)
struct SegLists {
    SegRec* list[4];
    uint32_t* count;      // 4 counters
    uint32_t* claim;      // per huge segment: claimed by a replay block (zeroed per batch)
};

}  // namespace rl

#include "rl_tb_chain.h"

namespace rl {


// segment heads -> (start, length), split into work lists:
//   [0] heavy token-bucket segments (the chain, k_tb_chain),
//   [1] light segments of any algorithm (one thread each),
//   [2] heavy window segments (one thread each, dequeued before the light ones),
//   [3] huge token-bucket segments (the chain dequeues these first: longest-first
//       keeps one hot key from starting last).
// One tile of SEG_TILE sorted positions per block, staged in LDS; thread t
// takes the SEG_ITEMS consecutive positions of chunk t.  A segment ends at the
// next head: inside the chunk, else at the first head of a later chunk (a
// block suffix-min over the chunks' first heads), else past the tile -- at most
// one head per tile (the tile's last), whose end one wave finds with a 64-ary
// search (wave_seg_end: a few rounds of one load per lane instead of one
// thread's dependent galloping).  List slots are reserved with ONE global
// atomic per list per block (a single contended word sustains only ~88
// atomics/us on MI355X).
#ifndef RL_SEG_ITEMS
#define RL_SEG_ITEMS 16
#endif
constexpr int SEG_ITEMS = RL_SEG_ITEMS;
constexpr int SEG_TILE = 256 * SEG_ITEMS;
constexpr uint32_t SEG_NONE = 0xffffffffu;

// the first position e >= from with e == m or sk[e] != k0, every position in
// [from0, from) holding k0; all 64 lanes call it with the same arguments
__device__ inline uint32_t wave_seg_end(const uint32_t* __restrict__ sk, uint32_t m, uint32_t from, uint32_t k0) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lo = from;
    uint64_t step = 1;
    for (int guard = 0; guard < 64; guard++) {
        const uint64_t p = (uint64_t)lo + step * lane;
        const bool diff = p >= m || sk[p] != k0;
        const uint64_t b = __ballot(diff);
        if (b) {
            const uint32_t f = (uint32_t)__ffsll((unsigned long long)b) - 1;
            if (step == 1 || f == 0) {
                if (f == 0) return lo;
                return lo + f;                            // step == 1
            }
            lo = (uint32_t)(lo + step * (f - 1) + 1);     // end in (p_{f-1}, p_f]
            step = (step + 63) / 64;
        } else {
            lo = (uint32_t)(lo + step * 63 + 1);
            step *= 64;
        }
    }
    return m;   // unreachable (the step grows 64x per round)
}

__device__ inline uint32_t seg_skew(uint32_t i) { return i + (i >> 4); }   // LDS bank skew of a 16-element chunk

__global__ __launch_bounds__(256) void k_segments(const uint32_t* __restrict__ sk, uint32_t m,
                                                  uint32_t invalid_key, uint32_t win_base, uint32_t heavy_min,
                                                  uint32_t huge_min, SegLists L, const uint32_t* skip,
                                                  const uint32_t* mdev = nullptr) {
    if (skip && *skip) return;   // k_sort_local built the lists
    if (mdev) m = min(m, *mdev);   // a batch sized on the device (the routed path)
    __shared__ uint32_t s_k[SEG_TILE + SEG_TILE / 16];
    __shared__ uint32_t s_next[256];      // first head of chunk t, then of chunks > t
    __shared__ uint32_t s_cnt[4], s_base[4], s_open, s_open_end;
    __shared__ uint64_t s_wsum[4];
    const uint32_t tid = threadIdx.x;
    for (uint32_t tile = blockIdx.x; tile * SEG_TILE < m; tile += gridDim.x) {
        const uint32_t t0 = tile * SEG_TILE;
        const uint32_t n = min((uint32_t)SEG_TILE, m - t0);
        if (tid == 0) s_open = SEG_NONE;
#pragma unroll
        for (int j = 0; j < SEG_ITEMS; j++) {   // coalesced
            const uint32_t i = j * 256 + tid;
            s_k[seg_skew(i)] = i < n ? sk[t0 + i] : invalid_key;
        }
        const uint32_t kprev = t0 > 0 ? sk[t0 - 1] : invalid_key;
        __syncthreads();
        const uint32_t c0 = tid * SEG_ITEMS;
        uint32_t key[SEG_ITEMS];
        uint32_t hmask = 0;
        uint32_t before = c0 == 0 ? kprev : s_k[seg_skew(c0 - 1)];
#pragma unroll
        for (int q = 0; q < SEG_ITEMS; q++) {
            key[q] = s_k[seg_skew(c0 + q)];
            const bool head = c0 + q < n && key[q] != invalid_key && key[q] != before;
            hmask |= head ? 1u << q : 0u;
            before = key[q];
        }
        // a chunk's first boundary for the segments before it: any head, or
        // an invalid key (rejected requests end a segment too)
        uint32_t bmask = hmask;
#pragma unroll
        for (int q = 0; q < SEG_ITEMS; q++)
            if (c0 + q >= n || key[q] == invalid_key) bmask |= 1u << q;
        s_next[tid] = bmask ? c0 + (uint32_t)__builtin_ctz(bmask) : SEG_NONE;
        __syncthreads();
        // suffix min over later chunks: s_next[t] = first boundary in chunks > t
        for (uint32_t d = 1; d < 256; d <<= 1) {
            const uint32_t v = tid + d < 256 ? s_next[tid + d] : SEG_NONE;
            const uint32_t mine = s_next[tid];
            __syncthreads();
            s_next[tid] = min(mine, v);
            __syncthreads();
        }
        // (s_next[t] now = min over chunks >= t; the boundary after chunk t is s_next[t + 1])
        const uint32_t after = tid + 1 < 256 ? s_next[tid + 1] : SEG_NONE;
        SegRec rec[SEG_ITEMS];
        uint32_t slot[SEG_ITEMS];
#pragma unroll
        for (int q = 0; q < SEG_ITEMS; q++) {
            slot[q] = 0xffffffffu;
            if (!((hmask >> q) & 1u)) continue;
            const uint32_t later = bmask & ~((2u << q) - 1u);   // boundaries after q in the chunk
            const uint32_t e = later ? c0 + (uint32_t)__builtin_ctz(later) : after;
            rec[q] = SegRec{t0 + c0 + q, e == SEG_NONE ? 0u : e - (c0 + q)};
            if (e == SEG_NONE) s_open = c0 + q;                 // the tile's last head: its end is past the tile
        }
        __syncthreads();
        if (s_open != SEG_NONE && tid < 64) {
            const uint32_t o = s_open;
            const uint32_t e = wave_seg_end(sk, m, t0 + n, s_k[seg_skew(o)]);
            if (tid == 0) s_open_end = e;
        }
        __syncthreads();
        // list slots in position order (a block scan of the per-chunk counts,
        // four 16-bit fields): light segments then replay with neighbouring
        // threads on neighbouring positions (coalesced)
        uint64_t cnt4 = 0;
#pragma unroll
        for (int q = 0; q < SEG_ITEMS; q++) {
            if (!((hmask >> q) & 1u)) continue;
            if (c0 + q == s_open) rec[q].len = s_open_end - (t0 + c0 + q);
            const uint32_t len = rec[q].len;
            const bool tb = key[q] < win_base;
            const uint32_t which = len < heavy_min ? 1u : !tb ? 2u : len >= huge_min ? 3u : 0u;
            slot[q] = (which << 30) | (uint32_t)((cnt4 >> (16 * which)) & 0xffffu);
            cnt4 += 1ull << (16 * which);
        }
        const uint64_t inc = wave_incl_scan_i64((int64_t)cnt4);
        if ((tid & 63) == 63) s_wsum[tid >> 6] = inc;
        __syncthreads();
        uint64_t exc = inc - cnt4;
        for (uint32_t w = 0; w < (tid >> 6); w++) exc += s_wsum[w];
        if (tid == 255) {
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const uint32_t tot = (uint32_t)(((exc + cnt4) >> (16 * w)) & 0xffffu);   // block total per list
                s_cnt[w] = tot;
            }
        }
        __syncthreads();
        if (tid < 4) s_base[tid] = s_cnt[tid] ? atomicAdd(&L.count[tid], s_cnt[tid]) : 0u;
        __syncthreads();
#pragma unroll
        for (int q = 0; q < SEG_ITEMS; q++) {
            if (slot[q] == 0xffffffffu) continue;
            const uint32_t which = slot[q] >> 30;
            slot[q] += (uint32_t)((exc >> (16 * which)) & 0xffffu);
        }
#pragma unroll
        for (int q = 0; q < SEG_ITEMS; q++) {
            if (slot[q] == 0xffffffffu) continue;
            const uint32_t which = slot[q] >> 30, off = slot[q] & 0x3fffffffu;
            L.list[which][s_base[which] + off] = rec[q];
        }
        __syncthreads();
    }
}

// The grouping sort's second half when every bucket of the MSD pass fits
// LDS (rl_engine.hip sort_shifts): one block per bucket -- the elements whose
// slot id has the MSD digit blockIdx.x, contiguous and in arrival order after
// the MSD pass -- sorts it by the `low_bits` bits below the digit with stable
// passes entirely in LDS (8 bits a pass, the last one narrower; the ranking of
// k_sort_pass: ballots per wave, digit counts per wave, a scan over (digit,
// wave)) and writes it to the same range of kout / vout (which may alias kin
// / vin: the bucket is read before anything is written).  Equal slots share
// a bucket, so this groups every key with its requests in arrival order like
// the LSD passes it replaces, and a key's segment never leaves its bucket:
// the block also builds the segment work lists k_segments would (same lists,
// same classes; heads in position order inside the block).  skip: the MSD
// pass found a bucket too large (the LSD passes and k_segments run instead).
constexpr int LOC_BLOCK = 1024;
constexpr int LOC_ITEMS = 12;
constexpr uint32_t LOC_MAX = LOC_BLOCK * LOC_ITEMS;   // 12288 elements per bucket
constexpr int LOC_WAVES = LOC_BLOCK / 64;

// A bucket larger than LDS, met only when the engine launched the grouping
// sort for "every bucket fits" on a prediction (the previous batches' plans,
// rl_engine.hip) that this batch breaks: the block sorts its bucket alone,
// with stable LSD passes over the bucket's range in HBM -- LOC_MAX elements
// at a time ranked in LDS as in k_sort_local, scattered at running digit
// offsets -- ping-ponging between (kin, vin) and the free MSD input buffers
// (xk, xv) so the last pass lands in (kout, vout), which is one of the two;
// then it builds the bucket's segment lists chunk by chunk (a segment running
// past a chunk ends where wave_seg_end finds it).  Slow (one CU), correct,
// and rare: a misprediction costs one batch this path, after which the engine
// launches the LSD passes again.
__device__ __noinline__ void loc_sort_big(const uint32_t* kin, const uint32_t* vin, uint32_t* kout, uint32_t* vout,
                                          uint32_t* xk, uint32_t* xv, uint32_t start, uint32_t cnt, int low_bits,
                                          uint32_t invalid_key, uint32_t win_base, uint32_t heavy_min,
                                          uint32_t huge_min, SegLists L, uint32_t* s_k, uint32_t* s_v,
                                          uint32_t (*s_cnt)[RADIX], uint32_t* s_base, uint32_t (*s_w)[4],
                                          uint32_t* s_lbase, uint32_t* s_run) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1ull;
    const int npass = (low_bits + 7) / 8;
    // buffers: P0 = (kin, vin), P1 = (xk, xv); the passes alternate from P0
    // and end in P(npass mod 2), which must be kout's: else copy P0 to P1 first
    const uint32_t *sk = kin, *sv = vin;
    uint32_t *dk = xk, *dv = xv;
    const bool out_p0 = kout == kin;
    if (out_p0 != ((npass & 1) == 0)) {
        for (uint32_t e = tid; e < cnt; e += LOC_BLOCK) {
            xk[start + e] = kin[start + e];
            xv[start + e] = vin[start + e];
        }
        __threadfence();
        __syncthreads();
        sk = xk;
        sv = xv;
        dk = const_cast<uint32_t*>(kin);
        dv = const_cast<uint32_t*>(vin);
    }
    for (int pass = 0; pass < npass; pass++) {
        const int shift = 8 * pass;
        const int bits = low_bits - shift < 8 ? low_bits - shift : 8;
        const uint32_t dm = (1u << bits) - 1u;
        if (tid < RADIX) s_run[tid] = 0;
        __syncthreads();
        for (uint32_t e = tid; e < cnt; e += LOC_BLOCK) atomicAdd(&s_run[(sk[start + e] >> shift) & dm], 1u);
        __syncthreads();
        {   // exclusive scan of the digit counts (threads < RADIX: 4 waves)
            const uint32_t v = tid < RADIX ? s_run[tid] : 0u;
            uint32_t inc = v;
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t t = __shfl_up(inc, off, 64);
                if (lane >= off) inc += t;
            }
            if (tid < RADIX && lane == 63) s_w[wave][0] = inc;
            __syncthreads();
            if (tid < RADIX) {
                uint32_t wp = 0;
                for (int w = 0; w < wave; w++) wp += s_w[w][0];
                s_run[tid] = wp + inc - v;
            }
            __syncthreads();
        }
        for (uint32_t c0 = 0; c0 < cnt; c0 += LOC_MAX) {
            const uint32_t ccnt = min((uint32_t)LOC_MAX, cnt - c0);
            const uint32_t per = (ccnt + LOC_BLOCK - 1) / LOC_BLOCK;
            const uint32_t base = (uint32_t)wave * (64 * per);
            uint32_t key[LOC_ITEMS], val[LOC_ITEMS], rank[LOC_ITEMS];
            for (int d = tid; d < LOC_WAVES * RADIX; d += LOC_BLOCK) (&s_cnt[0][0])[d] = 0;
#pragma unroll
            for (int j = 0; j < LOC_ITEMS; j++) {
                const uint32_t e = base + j * 64 + lane;
                const bool ok = (uint32_t)j < per && e < ccnt;
                key[j] = ok ? sk[start + c0 + e] : 0u;
                val[j] = ok ? sv[start + c0 + e] : 0u;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < LOC_ITEMS; j++) {
                if ((uint32_t)j < per) {   // block-uniform
                    const uint32_t e = base + j * 64 + lane;
                    const bool ok = e < ccnt;
                    const uint32_t d = (key[j] >> shift) & dm;
                    uint64_t peers = __ballot(ok);
                    for (int bt = 0; bt < bits; bt++) {
                        const uint32_t bit = (d >> bt) & 1u;
                        const uint64_t bb = __ballot(bit);
                        peers &= bit ? bb : ~bb;
                    }
                    if (ok) {
                        const uint32_t below = __popcll(peers & lt);
                        const uint32_t cur = s_cnt[wave][d];
                        rank[j] = cur + below;
                        if (below == 0) s_cnt[wave][d] = cur + (uint32_t)__popcll(peers);
                    }
                }
            }
            __syncthreads();
            if (tid < RADIX) {   // per digit: exclusive prefix over the waves, chunk total
                uint32_t tot = 0;
                for (int w = 0; w < LOC_WAVES; w++) {
                    const uint32_t c = s_cnt[w][tid];
                    s_cnt[w][tid] = tot;
                    tot += c;
                }
                s_base[tid] = tot;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < LOC_ITEMS; j++) {
                const uint32_t e = base + j * 64 + lane;
                if ((uint32_t)j < per && e < ccnt) {
                    const uint32_t d = (key[j] >> shift) & dm;
                    const uint32_t pos = s_run[d] + s_cnt[wave][d] + rank[j];
                    dk[start + pos] = key[j];
                    dv[start + pos] = val[j];
                }
            }
            __syncthreads();
            if (tid < RADIX) s_run[tid] += s_base[tid];
            __syncthreads();
        }
        __threadfence();   // this pass's stores before the next pass's loads (other waves, L1)
        __syncthreads();
        const uint32_t* tk = sk;
        const uint32_t* tv = sv;
        sk = dk;
        sv = dv;
        dk = const_cast<uint32_t*>(tk);
        dv = const_cast<uint32_t*>(tv);
    }
    // segment lists of the sorted bucket (kout), chunk by chunk
    const uint32_t* kb = kout + start;
    for (uint32_t c0 = 0; c0 < cnt; c0 += LOC_MAX) {
        const uint32_t ccnt = min((uint32_t)LOC_MAX, cnt - c0);
        const uint32_t per = (ccnt + LOC_BLOCK - 1) / LOC_BLOCK;
        const uint32_t base = (uint32_t)wave * (64 * per);
        uint32_t key[LOC_ITEMS], bnd[LOC_ITEMS], head[LOC_ITEMS];
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            const uint32_t e = base + j * 64 + lane;
            key[j] = ((uint32_t)j < per && e < ccnt) ? kb[c0 + e] : 0u;
            if ((uint32_t)j < per && e < ccnt) s_k[e] = key[j];
        }
        const uint32_t kprev = kb[c0 ? c0 - 1 : 0];
        if (tid == 0) s_lbase[0] = SEG_NONE;   // the chunk's open head (its end lies past the chunk)
        __syncthreads();
        uint32_t run = 0;
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            const uint32_t e = base + j * 64 + lane;
            const bool ok = (uint32_t)j < per && e < ccnt;
            const bool valid = ok && key[j] != invalid_key;
            const uint32_t before = e ? s_k[e ? e - 1 : 0] : kprev;
            const bool hd = valid && ((c0 == 0 && e == 0) || before != key[j]);
            const bool bd = hd || (ok && !valid);
            const uint64_t bm = __ballot(bd);
            bnd[j] = bd ? run + (uint32_t)__popcll(bm & lt) : SEG_NONE;
            head[j] = hd ? 1u : 0u;
            run += (uint32_t)__popcll(bm);
        }
        if (lane == 0) s_w[wave][0] = run;
        __syncthreads();
        uint32_t wpre = 0, nb = 0;
        for (int w = 0; w < LOC_WAVES; w++) {
            const uint32_t c = s_w[w][0];
            wpre += w < wave ? c : 0u;
            nb += c;
        }
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            if (bnd[j] != SEG_NONE) {
                bnd[j] += wpre;
                s_v[bnd[j]] = base + j * 64 + lane;
            }
        }
        __syncthreads();
        // the last boundary of the chunk, if a head, ends past the chunk
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++)
            if (head[j] && bnd[j] + 1 == nb && c0 + ccnt < cnt) s_lbase[0] = base + j * 64 + lane;
        __syncthreads();
        if (s_lbase[0] != SEG_NONE && wave == 0) {
            const uint32_t o = s_lbase[0];
            const uint32_t e = wave_seg_end(kb, cnt, c0 + ccnt, s_k[o]);
            if (lane == 0) s_lbase[1] = e - c0;
        }
        __syncthreads();
        const uint32_t open_end = s_lbase[1];
        uint32_t which[LOC_ITEMS], len[LOC_ITEMS];
        uint32_t lrun[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            which[j] = 4u;
            len[j] = 0u;
            if (head[j]) {
                const uint32_t e = base + j * 64 + lane;
                const uint32_t end = bnd[j] + 1 < nb ? s_v[bnd[j] + 1] : c0 + ccnt < cnt ? open_end : ccnt;
                len[j] = end - e;
                const bool tb = key[j] < win_base;
                which[j] = len[j] < heavy_min ? 1u : !tb ? 2u : len[j] >= huge_min ? 3u : 0u;
            }
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const uint64_t wm = __ballot(which[j] == (uint32_t)w);
                if (which[j] == (uint32_t)w) bnd[j] = lrun[w] + (uint32_t)__popcll(wm & lt);
                lrun[w] += (uint32_t)__popcll(wm);
            }
        }
        __syncthreads();   // s_w reused
        if (lane == 0)
            for (int w = 0; w < 4; w++) s_w[wave][w] = lrun[w];
        __syncthreads();
        if (tid < 4) {
            uint32_t t = 0;
            for (int w = 0; w < LOC_WAVES; w++) t += s_w[w][tid];
            s_base[tid] = t ? atomicAdd(&L.count[tid], t) : 0u;
        }
        __syncthreads();
        uint32_t wb[4];
#pragma unroll
        for (int w = 0; w < 4; w++) {
            uint32_t x = s_base[w];
            for (int v = 0; v < wave; v++) x += s_w[v][w];
            wb[w] = x;
        }
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            if (which[j] < 4u) {
                const uint32_t w = which[j];
                const uint32_t at = (w == 0 ? wb[0] : w == 1 ? wb[1] : w == 2 ? wb[2] : wb[3]) + bnd[j];
                L.list[w][at] = SegRec{start + c0 + base + j * 64 + lane, len[j]};
            }
        }
        __syncthreads();   // s_k, s_v, s_w, s_base, s_lbase reused by the next chunk
    }
}

__global__ __launch_bounds__(LOC_BLOCK) void k_sort_local(const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
                                                          uint32_t* vout, const uint32_t* __restrict__ ghist_msd,
                                                          int low_bits, const uint32_t* skip, uint32_t invalid_key,
                                                          uint32_t win_base, uint32_t heavy_min, uint32_t huge_min,
                                                          SegLists L, uint32_t* xk, uint32_t* xv) {
    if (skip && *skip) return;
    __shared__ uint32_t s_k[LOC_MAX], s_v[LOC_MAX];
    __shared__ uint32_t s_cnt[LOC_WAVES][RADIX];
    __shared__ uint32_t s_base[RADIX];
    __shared__ uint32_t s_w[LOC_WAVES][4];
    __shared__ uint32_t s_lbase[4];
    __shared__ uint32_t s_run[RADIX];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t cnt = ghist_msd[b];
    if (cnt == 0) return;
    // the bucket's range: exclusive prefix of the MSD histogram up to b
    uint32_t pre = (uint32_t)tid < b ? ghist_msd[tid] : 0u;
    for (int off = 32; off > 0; off >>= 1) pre += __shfl_xor(pre, off);
    if (lane == 0 && wave < 4) s_w[wave][0] = pre;
    __syncthreads();
    const uint32_t start = s_w[0][0] + s_w[1][0] + s_w[2][0] + s_w[3][0];
    if (cnt > LOC_MAX) {   // only in a launch without `skip` (a predicted plan; see loc_sort_big)
        __syncthreads();   // s_w
        loc_sort_big(kin, vin, kout, vout, xk, xv, start, cnt, low_bits, invalid_key, win_base, heavy_min, huge_min,
                     L, s_k, s_v, s_cnt, s_base, s_w, s_lbase, s_run);
        return;
    }
    const uint64_t lt = (1ull << lane) - 1ull;
    // every wave takes `per` consecutive rows of 64 elements (the fewest that
    // cover the bucket), so all waves share the ranking work; wave order is
    // element order (the passes stay stable)
    const uint32_t per = (cnt + LOC_BLOCK - 1) / LOC_BLOCK;
    const uint32_t base = (uint32_t)wave * (64 * per);
    // element e = base + 64 j + lane of the bucket, straight from HBM
    uint32_t key[LOC_ITEMS], val[LOC_ITEMS], rank[LOC_ITEMS];
#pragma unroll
    for (int j = 0; j < LOC_ITEMS; j++) {
        const uint32_t e = base + j * 64 + lane;
        const bool ok = (uint32_t)j < per && e < cnt;
        key[j] = ok ? kin[start + e] : 0u;
        val[j] = ok ? vin[start + e] : 0u;
    }
    for (int shift = 0; shift < low_bits; shift += 8) {
        const int bits = low_bits - shift < 8 ? low_bits - shift : 8;
        for (int d = tid; d < LOC_WAVES * RADIX; d += LOC_BLOCK) (&s_cnt[0][0])[d] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            if ((uint32_t)j < per) {   // block-uniform
                const uint32_t e = base + j * 64 + lane;
                const bool ok = e < cnt;
                const uint32_t d = (key[j] >> shift) & ((1u << bits) - 1u);
                uint64_t peers = __ballot(ok);
                for (int bt = 0; bt < bits; bt++) {
                    const uint32_t bit = (d >> bt) & 1u;
                    const uint64_t bb = __ballot(bit);
                    peers &= bit ? bb : ~bb;
                }
                if (ok) {
                    const uint32_t below = __popcll(peers & lt);
                    const uint32_t cur = s_cnt[wave][d];
                    rank[j] = cur + below;
                    if (below == 0) s_cnt[wave][d] = cur + (uint32_t)__popcll(peers);
                }
            }
        }
        __syncthreads();
        // per digit: exclusive prefix over the waves; digit totals scanned
        uint32_t tot = 0;
        if (tid < RADIX) {
            for (int w = 0; w < LOC_WAVES; w++) {
                const uint32_t c = s_cnt[w][tid];
                s_cnt[w][tid] = tot;
                tot += c;
            }
        }
        uint32_t inc = tot;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t t = __shfl_up(inc, off, 64);
            if (lane >= off) inc += t;
        }
        if (tid < RADIX && lane == 63) s_w[wave][0] = inc;
        __syncthreads();
        if (tid < RADIX) {
            uint32_t wp = 0;
            for (int w = 0; w < wave; w++) wp += s_w[w][0];
            s_base[tid] = wp + inc - tot;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            const uint32_t e = base + j * 64 + lane;
            if ((uint32_t)j < per && e < cnt) {
                const uint32_t d = (key[j] >> shift) & ((1u << bits) - 1u);
                const uint32_t pos = s_base[d] + s_cnt[wave][d] + rank[j];
                s_k[pos] = key[j];
                s_v[pos] = val[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {   // the next pass's elements, in the new order
            const uint32_t e = base + j * 64 + lane;
            const bool ok = (uint32_t)j < per && e < cnt;
            key[j] = ok ? s_k[e] : 0u;
            val[j] = ok ? s_v[e] : 0u;
        }
    }
    if (low_bits <= 0) {   // (never: the MSD digit is the top 8 of >= 12 bits) keep s_k valid
#pragma unroll
        for (int j = 0; j < LOC_ITEMS; j++) {
            const uint32_t e = base + j * 64 + lane;
            if ((uint32_t)j < per && e < cnt) s_k[e] = key[j];
        }
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < LOC_ITEMS; j++) {
        const uint32_t e = base + j * 64 + lane;
        if ((uint32_t)j < per && e < cnt) {
            kout[start + e] = key[j];
            vout[start + e] = val[j];
        }
    }
    // ---- segments of the bucket (k_segments' lists) ----
    // boundaries in position order: a head (a valid key unlike its
    // predecessor) or an invalid key (rejected requests end a segment); the
    // compacted boundary positions go to s_v (no longer needed)
    uint32_t bnd[LOC_ITEMS];
    uint32_t run = 0;   // boundaries of this wave so far
#pragma unroll
    for (int j = 0; j < LOC_ITEMS; j++) {
        const uint32_t e = base + j * 64 + lane;
        const bool ok = (uint32_t)j < per && e < cnt;
        const bool valid = ok && key[j] != invalid_key;
        const bool head = valid && (e == 0 || s_k[e - 1] != key[j]);
        const bool bd = head || (ok && !valid);
        const uint64_t bm = __ballot(bd);
        bnd[j] = bd ? run + (uint32_t)__popcll(bm & lt) : 0xffffffffu;
        rank[j] = head ? 1u : 0u;
        run += (uint32_t)__popcll(bm);
    }
    if (lane == 0) s_w[wave][0] = run;
    __syncthreads();
    uint32_t wpre = 0, nb = 0;
    for (int w = 0; w < LOC_WAVES; w++) {
        const uint32_t c = s_w[w][0];
        wpre += w < wave ? c : 0u;
        nb += c;
    }
#pragma unroll
    for (int j = 0; j < LOC_ITEMS; j++) {
        if (bnd[j] != 0xffffffffu) {
            bnd[j] += wpre;
            s_v[bnd[j]] = base + j * 64 + lane;
        }
    }
    __syncthreads();
    // each head: its end (the next boundary, or the bucket end), its list,
    // and its slot in the list (position order: per list a wave ballot rank,
    // then the waves before, then the block's base from one atomic per list)
    uint32_t which[LOC_ITEMS], len[LOC_ITEMS];
    uint32_t lrun[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < LOC_ITEMS; j++) {
        which[j] = 4u;
        len[j] = 0u;
        if (rank[j]) {
            const uint32_t e = base + j * 64 + lane;
            const uint32_t end = bnd[j] + 1 < nb ? s_v[bnd[j] + 1] : cnt;
            len[j] = end - e;
            const bool tb = key[j] < win_base;
            which[j] = len[j] < heavy_min ? 1u : !tb ? 2u : len[j] >= huge_min ? 3u : 0u;
        }
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const uint64_t wm = __ballot(which[j] == (uint32_t)w);
            if (which[j] == (uint32_t)w) bnd[j] = lrun[w] + (uint32_t)__popcll(wm & lt);
            lrun[w] += (uint32_t)__popcll(wm);
        }
    }
    __syncthreads();   // s_w reused
    if (lane == 0)
        for (int w = 0; w < 4; w++) s_w[wave][w] = lrun[w];
    __syncthreads();
    if (tid < 4) {
        uint32_t t = 0;
        for (int w = 0; w < LOC_WAVES; w++) t += s_w[w][tid];
        s_lbase[tid] = t ? atomicAdd(&L.count[tid], t) : 0u;
    }
    __syncthreads();
    uint32_t wb[4];
#pragma unroll
    for (int w = 0; w < 4; w++) {
        uint32_t x = s_lbase[w];
        for (int v = 0; v < wave; v++) x += s_w[v][w];
        wb[w] = x;
    }
#pragma unroll
    for (int j = 0; j < LOC_ITEMS; j++) {
        if (which[j] < 4u) {
            const uint32_t w = which[j];
            const uint32_t at = (w == 0 ? wb[0] : w == 1 ? wb[1] : w == 2 ? wb[2] : wb[3]) + bnd[j];
            L.list[w][at] = SegRec{start + base + j * 64 + lane, len[j]};
        }
    }
}

// One request as k_probe packs it in arrival order: the sorted-order gather
// of k_permute reads one 16-byte record per request instead of four scattered
// array elements -- time, arrival index, config and n in 16 bits each.  The
// grouping sort's first (MSD) pass moves it into bucket order (k_sort_pass
// rin/rout), where k_permute gathers it from an L2-resident bucket instead of
// from the whole batch.  A field that does not fit (REC_WIDE) is read at the
// arrival index from the caller's arrays, or, with an explicit server clock
// (XS: the routed path's store clock), from side arrays the probe filled for
// exactly those requests; the clock itself is floor(ts / 1e6) unless
// REC_SMSX says it differs (XS: then side.sms at the arrival index).
template <bool XS> struct alignas(16) ReqRec {
    int64_t ts;
    uint32_t ix;       // arrival index | REC_FRESH | REC_SMSX
    uint32_t cn;       // config id << 16 | n
};
constexpr uint32_t REC_WIDE = 0xffffu;    // a 16-bit field that does not fit
constexpr uint32_t REC_FRESH = 1u << 31;  // ix: the request's probe inserted its key (k_probe)
constexpr uint32_t REC_SMSX = 1u << 30;   // ix (XS): the server clock is not floor(ts / 1e6)
constexpr uint32_t REC_IX = REC_SMSX - 1u;
static_assert(sizeof(ReqRec<false>) == 16 && sizeof(ReqRec<true>) == 16, "request records");

// where an XS record's fields that do not fit go (arrival index)
struct RecSide {
    int64_t* n;
    uint32_t* cfg;
    int64_t* sms;
};

template <bool XS>
__device__ inline ReqRec<XS> rec_pack(int64_t t, int64_t n, int64_t sms, uint32_t c, uint32_t i, const RecSide& side) {
    const uint32_t c16 = c < REC_WIDE ? c : REC_WIDE;
    const uint32_t n16 = (n > 0 && n < (int64_t)REC_WIDE) ? (uint32_t)n : REC_WIDE;
    uint32_t ix = i;
    if constexpr (XS) {
        const uint32_t a = i & REC_IX;
        if (c16 == REC_WIDE) side.cfg[a] = c;
        if (n16 == REC_WIDE) side.n[a] = n;
        if (sms != floor_div(t, 1000000LL)) {
            side.sms[a] = sms;
            ix |= REC_SMSX;
        }
    } else {
        (void)sms;
        (void)side;
    }
    return ReqRec<XS>{t, ix, (c16 << 16) | n16};
}
template <bool XS>
__device__ inline int64_t rec_n(const ReqRec<XS>& r, const int64_t* __restrict__ n_in, uint32_t i) {
    const uint32_t n16 = r.cn & 0xffffu;
    return n16 != REC_WIDE ? (int64_t)n16 : n_in[i];
}
template <bool XS>
__device__ inline uint32_t rec_cfg(const ReqRec<XS>& r, const uint32_t* __restrict__ cfg_in, uint32_t i) {
    const uint32_t c16 = r.cn >> 16;
    return c16 != REC_WIDE ? c16 : cfg_in[i];
}
template <bool XS>
__device__ inline int64_t rec_sms(const ReqRec<XS>& r, const int64_t* __restrict__ sms_in) {
    if (XS && (r.ix & REC_SMSX)) return sms_in[r.ix & REC_IX];
    return floor_div(r.ts, 1000000LL);
}

// requests to sorted order + the state-free token-bucket precomputation.
// Each wave covers 64 consecutive sorted positions; a request's predecessor
// in its segment (position j-1) is the neighbouring lane's record, so only
// lane 0 gathers a second one.  n_in / cfg_in: the caller's n and config
// (arrival order), for a record whose field did not fit.
// The records are in the MSD pass's bucket order and sv holds each element's
// position there (the sort carried it), so consecutive sorted positions
// gather from one bucket's few-KB range (L2) instead of the whole batch; the
// arrival index comes from the record and goes to ix_out[j] (the finish reads
// it there).
template <bool XS>
__global__ __launch_bounds__(256) void k_permute(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                 uint32_t m, uint32_t invalid_key, uint32_t win_base,
                                                 const CfgDev* __restrict__ cfgs, int32_t profile,
                                                 const ReqRec<XS>* __restrict__ rec, const int64_t* __restrict__ n_in,
                                                 ReqArgs out, TbPre pre, const uint32_t* mdev,
                                                 const uint32_t* __restrict__ cfg_in, uint32_t* __restrict__ ix_out,
                                                 const int64_t* __restrict__ sms_in) {
    if (mdev) m = min(m, *mdev);   // a batch sized on the device (the routed path)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < m; base += stride) {
        const uint32_t j = base + lane;
        const uint32_t k0 = j < m ? sk[j] : invalid_key;
        // the record's position in bucket order (read for every element: the
        // finish needs every arrival index)
        const uint32_t at = j < m ? sv[j] : 0u;
        // lane 0: the predecessor at j-1 (a previous chunk's last lane)
        uint32_t kpl = invalid_key, atp = 0u;
        if (lane == 0 && j > 0 && k0 != invalid_key && k0 < win_base) {
            kpl = sk[j - 1];
            if (kpl == k0) atp = sv[j - 1];
        }
        ReqRec<XS> r{}, q{};
        if (j < m) r = rec[at];
        if (lane == 0 && kpl == k0 && k0 != invalid_key) q = rec[atp];
        const uint32_t ix = r.ix & REC_IX;
        if (j < m) {
            ix_out[j] = ix;
            if (out.fresh) const_cast<uint8_t*>(out.fresh)[j] = (uint8_t)(r.ix >> 31);
        }
        const bool valid = k0 != invalid_key;
        const int64_t sms = rec_sms<XS>(r, sms_in);
        // predecessor (j-1) fields from the lane below
        const uint32_t rc = valid ? rec_cfg<XS>(r, cfg_in, ix) : 0u;
        uint32_t kp = __shfl_up(k0, 1);
        int64_t tp = __shfl_up(r.ts, 1);
        int64_t smsp = __shfl_up(sms, 1);
        uint32_t cp = __shfl_up(rc, 1);
        if (lane == 0) {
            kp = invalid_key;
            if (kpl == k0 && valid) {
                kp = k0;
                tp = q.ts;
                smsp = rec_sms<XS>(q, sms_in);
                cp = rec_cfg<XS>(q, cfg_in, q.ix & REC_IX);
            }
        }
        if (!valid) continue;
        const int64_t nn = rec_n<XS>(r, n_in, ix);
        // `out` is the engine's own permuted buffers (ReqArgs keeps inputs const)
        const_cast<int64_t*>(out.ts)[j] = r.ts;
        const_cast<int64_t*>(out.n)[j] = nn;
        const_cast<uint32_t*>(out.cfg)[j] = rc;
        if (XS) const_cast<int64_t*>(out.sms)[j] = sms;   // only an explicit server clock
        if (k0 >= win_base) continue;
        const CfgDev& C = cfgs[rc];
        const double now = (double)r.ts / 1e9;
        // state-free: a head's add needs the table (tb_head_add, at replay)
        // and the table is still being updated by the previous batch; a
        // placeholder keeps the stores full lines (the replay writes the
        // head's own add where it is read)
        double add = __builtin_nan("");
        if (kp == k0) {
            const double prev_last = lua_tostring_roundtrip((double)tp / 1e9, profile);
            const int64_t prev_when = expire_when(cfgs[cp].ttl_tb, smsp);
            if (key_alive(prev_when, sms, profile)) add = (now - prev_last) * C.rate;
        }
        pre.add[j] = add;
        pre.th[j] = fmin(C.limit_d, (double)nn);
    }
}

// Go's result arithmetic of a token-bucket step from the script's reply
// (tokenbucket.go:114-130): Remaining = floor(tokens); RetryAfter from the
// missing tokens when denied
__device__ inline void tb_result(uint8_t dec, double tokens, int64_t n, const CfgDev& c, int64_t& rem,
                                 int64_t& retry);
// ... and ResetAt = calculateResetTime(now) (tokenbucket.go:161-165)
__device__ inline void tb_result_reset(uint8_t dec, double tokens, int64_t n, int64_t ts, const CfgDev& c,
                                       int64_t& rem, int64_t& retry, int64_t& reset) {
    tb_result(dec, tokens, n, c, rem, retry);
    reset = tb_reset_at((double)ts / 1e9, c);
}
__device__ inline void tb_result(uint8_t dec, double tokens, int64_t n, const CfgDev& c, int64_t& rem,
                                 int64_t& retry) {
    rem = go_f2i(floor(tokens));
    retry = 0;
    if (dec == DEC_DENIED) {
        const int64_t need = wsub(n, rem);
        const double w = need == 1 ? c.inv_rate : (double)need / c.rate;   // tokensNeeded / refillRate
        const int64_t d = go_f2i(w * 1e9);
        retry = d < 0 ? 0 : d;
    }
}

// The Result fields of one executed request from the replay's compact output
// -- the decision and one value: the Lua `tokens` of a token bucket, Remaining
// of a window counter -- and the request itself: token bucket
// tokenbucket.go:114-130 (remaining, retry) and :161-165 (reset_at); window
// counters fixedwindow.go:101-114 / slidingwindow.go:108-121 (reset_at =
// window start + W, retry = time to it when denied; 0 on a script error)
__device__ inline void finish_result(uint8_t dec, double val, int64_t t, int64_t n, const CfgDev& c, int64_t& rem,
                                     int64_t& retry, int64_t& reset, double& tok) {
    if (c.alg == ALG_TOKEN_BUCKET) {
        tb_result_reset(dec, val, n, t, c, rem, retry, reset);
        tok = val;
        return;
    }
    rem = __double_as_longlong(val);
    reset = wadd(wmul(window_start(t, c), NS_PER_S), c.window);
    retry = dec == DEC_DENIED ? until_reset(reset, t) : 0;
    tok = 0.0;
}

// results from sorted order back to the caller's order (batches above UP_MAX)
__global__ __launch_bounds__(256) void k_unpermute(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                   uint32_t m, uint32_t invalid_key, const CfgDev* __restrict__ cfgs,
                                                   ReqArgs sorted, ReqArgs out) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        const uint32_t k0 = sk[j];
        const uint32_t i = sv[j];
        uint8_t dec = DEC_INVALID;   // rejected by k_probe (n <= 0, unknown config or key, table full)
        int64_t rem = 0, retry = 0, reset = 0;
        double tok = 0.0;
        if (k0 != invalid_key) {
            dec = sorted.dec[j];
            finish_result(dec, sorted.tok[j], sorted.ts[j], sorted.n[j], cfgs[sorted.cfg[j]], rem, retry, reset, tok);
        }
        out.dec[i] = dec;
        out.rem[i] = rem;
        out.retry[i] = retry;
        out.reset[i] = reset;
        if (out.tok) out.tok[i] = tok;
    }
}

// Results to the caller's order without scattered stores (m <= UP_MAX), in
// two coalesced passes: (1) k_unpermute_bucket reads the replay's compact
// results in sorted order (decision + value) and writes one 16-byte record per
// request into the bucket of its arrival index (UP_BUCKET consecutive
// indices; every bucket is full, so bucket b starts at b * UP_BUCKET and a
// block-aggregated atomic per bucket hands out positions inside it); (2)
// k_unpermute_bucket_out places one bucket's records in LDS by arrival index
// and, reading each request's time, n and config in arrival order (the
// caller's inputs, coalesced), finishes the Result fields (finish_result) and
// writes every output array with full-line stores.
constexpr int UP_BUCKET_BITS = 11;
constexpr uint32_t UP_BUCKET = 1u << UP_BUCKET_BITS;   // arrival indices per bucket
constexpr uint32_t UP_MAX = 1u << 21;                  // batches up to 2^21: <= 1024 buckets
constexpr uint32_t UP_NB = UP_MAX / UP_BUCKET;
constexpr int UP_ITEMS = 8;                            // sorted positions per thread (k_unpermute_bucket)

struct alignas(16) UpRec {
    uint32_t i;        // arrival index
    uint32_t dec;
    double val;        // tokens (token bucket) / Remaining bits (window)
};

__global__ __launch_bounds__(256) void k_unpermute_bucket(const uint32_t* __restrict__ sk,
                                                          const uint32_t* __restrict__ sv, uint32_t m,
                                                          uint32_t invalid_key, ReqArgs sorted,
                                                          UpRec* __restrict__ bucketed, uint32_t* bucket_ctr,
                                                          const uint32_t* mdev = nullptr) {
    __shared__ uint32_t s_cnt[UP_NB], s_base[UP_NB];
    if (mdev) m = min(m, *mdev);   // a batch sized on the device (routed)
    const uint32_t nb = (m + UP_BUCKET - 1) >> UP_BUCKET_BITS;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) s_cnt[b] = 0;
    __syncthreads();
    const uint32_t j0 = blockIdx.x * (256 * UP_ITEMS);
    UpRec rec[UP_ITEMS];
    uint32_t at[UP_ITEMS];
#pragma unroll
    for (int q = 0; q < UP_ITEMS; q++) {
        const uint32_t j = j0 + q * 256 + threadIdx.x;
        at[q] = 0xffffffffu;
        if (j >= m) continue;
        const bool ok = sk[j] != invalid_key;   // else rejected by k_probe
        rec[q] = UpRec{sv[j], ok ? (uint32_t)sorted.dec[j] : (uint32_t)DEC_INVALID, ok ? sorted.tok[j] : 0.0};
        at[q] = atomicAdd(&s_cnt[rec[q].i >> UP_BUCKET_BITS], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 256)
        s_base[b] = s_cnt[b] ? atomicAdd(&bucket_ctr[b], s_cnt[b]) : 0u;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < UP_ITEMS; q++) {
        if (at[q] == 0xffffffffu) continue;
        const uint32_t b = rec[q].i >> UP_BUCKET_BITS;
        bucketed[(size_t)b * UP_BUCKET + s_base[b] + at[q]] = rec[q];
    }
}

__global__ __launch_bounds__(256) void k_unpermute_bucket_out(uint32_t m, const UpRec* __restrict__ bucketed,
                                                              const CfgDev* __restrict__ cfgs, ReqArgs out) {
    __shared__ double s_val[UP_BUCKET];
    __shared__ uint8_t s_dec[UP_BUCKET];
    const uint32_t b = blockIdx.x;
    const uint32_t base = b * UP_BUCKET;
    const uint32_t cnt = min(UP_BUCKET, m - base);
    for (uint32_t k = threadIdx.x; k < cnt; k += 256) {
        const UpRec r = bucketed[(size_t)base + k];
        const uint32_t o = r.i - base;
        s_dec[o] = (uint8_t)r.dec;
        s_val[o] = r.val;
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 256) {
        const uint32_t i = base + k;
        const uint8_t dec = s_dec[k];
        int64_t rem = 0, retry = 0, reset = 0;
        double tok = 0.0;
        if (dec != DEC_INVALID)
            finish_result(dec, s_val[k], out.ts[i], out.n[i], cfgs[out.cfg[i]], rem, retry, reset, tok);
        out.dec[i] = dec;
        out.rem[i] = rem;
        out.retry[i] = retry;
        out.reset[i] = reset;
        if (out.tok) out.tok[i] = tok;
    }
}

}  // namespace rl
