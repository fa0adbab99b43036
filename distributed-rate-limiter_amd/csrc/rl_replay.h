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

// State-independent token-bucket quantities of each request (sorted order),
// computed in the permute pass: the previous request of the same key is the
// previous sorted position (or, for a segment head, the table entry).
struct TbPre {
    double* add;       // elapsed * refill_rate (tokenbucket.go:36-37)
    int64_t* reset;    // calculateResetTime (tokenbucket.go:161-165)
    double* lq;        // tostring(now) as stored in last_refill (tokenbucket.go:48)
    int64_t* when;     // key expiry after this request's EXPIRE (tokenbucket.go:49)
    uint8_t* alive;    // did HMGET see the key (tokenbucket.go:31-33)
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
    r.sms = a.sms[j];
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

__device__ inline void replay_tb_serial(TbEntry* e, uint32_t j0, uint32_t j1, const CfgDev* cfgs,
                                        int32_t profile, const ReqArgs& a, const TbPre& pre) {
    double tok = e->tok;
    for (uint32_t j = j0; j < j1; j++) {
        Out o = tb_chain_step(tok, pre.alive[j] != 0, pre.add[j], a.n[j], pre.reset[j], cfgs[a.cfg[j]], profile);
        write_out(a, j, o);
    }
    e->tok = tok;
    e->last = pre.lq[j1 - 1];
    e->when = pre.when[j1 - 1];
}

__device__ inline void replay_win_serial(WinEntry* e, uint32_t j0, uint32_t j1, const CfgDev* cfgs,
                                         int32_t profile, const ReqArgs& a, uint32_t* eflags) {
    WinState w;
    w.s[0] = e->s[0];
    w.s[1] = e->s[1];
    uint32_t ef = 0;
    Req cur = load_req(a, j0);
    for (uint32_t j = j0; j < j1; j++) {
        Req nxt = cur;
        if (j + 1 < j1) nxt = load_req(a, j + 1);
        const CfgDev& c = cfgs[cur.c];
        Out o = (c.alg == ALG_SLIDING_WINDOW) ? sw_step(w, cur.t, cur.n, cur.sms, c, profile, ef)
                                              : fw_step(w, cur.t, cur.n, cur.sms, c, profile, ef);
        write_out(a, j, o);
        cur = nxt;
    }
    e->s[0] = w.s[0];
    e->s[1] = w.s[1];
    if (ef) atomicOr(eflags, ef);
}

// ---------------------------------------------------------------------------
// Block-cooperative token-bucket replay for heavy (Zipf hot-key) segments.
//
// The carried state of a token-bucket key is the *stored* tokens value, which
// Lua's tostring quantizes: in Redis 7 to 14 significant decimal digits, i.e.
// an integer D in [1e13, 1e14) and a decade E (value = D * 10^(E-13)); with
// miniredis to the exact double, i.e. an integer mantissa D and binary
// exponent E.  Between events a step's effect on D is the state-independent
// increment r_j = round(add_j * 10^(13-E)) (resp. add_j * 2^-E), because D is
// an integer and only the rounding of the fractional part of add_j matters.
//
// Guess-and-verify, one round per pass over the not-yet-committed lanes:
//   1. each lane computes its nominal r_j (state-independent),
//   2. block exclusive scan: guessed predecessor state Dg_j = D + sum r_<j,
//   3. each lane runs the reference step EXACTLY (tb_step's arithmetic) from
//      the guess and checks its exact result equals (Dg_j + r_j, E),
//   4. the first lane s that does not (a near-tie rounding flip, a decade
//      change, an allow, a clamp at capacity, an expired key) had a correct
//      guess -- every lane before it was verified -- so lanes <= s are
//      committed and s's exact result is the new base.
// The result is identical to serial replay by construction; the common case
// (denied requests accumulating refill) commits 256 steps per round.
// ---------------------------------------------------------------------------

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

// 1 / (unit of D) for decade/exponent E (only used for the nominal guess)
__device__ inline double tb_scale(int32_t E, int32_t profile) {
    if (profile != PROFILE_REDIS7) return ldexp(1.0, -E);
    int k = 13 - E;
    int ak = k < 0 ? -k : k;
    double s = 1.0;
    while (ak > 22) { s *= 1e22; ak -= 22; }
    s *= rlq::pow10_exact(ak);
    return k >= 0 ? s : 1.0 / s;
}

// Diagnostic build only (-DRL_STAMPS): per-phase shader-clock sums of the
// cooperative replay, read back through the debug counters; never in the
// product build (stamps serialize the phases they measure).
#ifdef RL_STAMPS
#define RL_STAMP(v) do { __builtin_amdgcn_sched_barrier(0); (v) = __builtin_amdgcn_s_memtime(); \
                         __builtin_amdgcn_s_waitcnt(0xc07f); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define RL_STAMP(v) do { } while (0)
#endif

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

// ---------------------------------------------------------------------------
// In-round flip resolution.
//
// Within a decade (Redis profile) or binade (miniredis profile) the stored
// state is an integer D, and a step maps D to D + r_j, r_j = round(add_j / u),
// except when add_j / u lies within TAU of a half-integer: then the IEEE
// rounding of T = strtod(D) and of T + add (|error| <= 0.0222 u, SURVEY-level
// bound 10^14 * 2^-52) can flip the rounded result by one.  So a lane whose
// fraction is far from 1/2 maps a predecessor error c to the same c; only
// near-tie lanes depend on the exact predecessor.  One round:
//   1. nominal r_j, near-tie flag; block scan of r (DPP) -> nominal
//      predecessor D + P_j; compaction rank of the near-tie lanes,
//   2. first lane e where an event (allow, clamp, decade change, expired key,
//      > 64 near lanes) is possible even with |c| <= 2,
//   3. every near-tie lane before e is evaluated EXACTLY for the five
//      candidate predecessors D + P_j + c, c in [-2, 2] (one (lane, c) pair
//      per thread): a table c -> c' (or STOP),
//   4. one wave composes the tables (a function-composition scan) -> the true
//      correction after each near-tie lane; a STOP shortens the round,
//   5. every lane up to e runs the step EXACTLY from its now-known true
//      predecessor and checks the result it implies; the first mismatch (none
//      if the bound holds) also ends the round -- correctness never rests on
//      the bound, only the speed does,
//   6. lanes up to e are committed; e's exact result is the next base.
// Rounds per chunk = 1 + events, not 1 + flips.
// ---------------------------------------------------------------------------

// One chunk's requests as the loader wave hands them to the compute waves
// (state-independent terms precomputed by k_permute).
struct ChunkSlot {
    double add;
    int64_t n;
    int64_t reset;
    uint32_t c;
    uint32_t alive;
};

// configs cached in LDS per block (when the engine has at most MAX_LCFG)
constexpr int MAX_LCFG = 32;
constexpr int MAX_NEAR = 64;
constexpr uint32_t STOPC = 7;
constexpr double TAU_DEC = 0.03;   // > 0.0222: far lanes are exact by the bound

enum : int { QM_NONE = 0, QM_DEC = 1, QM_BIN = 2 };

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
    else if (mode == QM_DEC) T = rlq::div_pow10((double)Dpred, P, R);   // strtod("D e(E-13)")
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
    if (mode == QM_DEC) {
        if (tokens > 0.0 && tokens * P < 1.4e14) {
            v.Dact = rlq::round_scaled_P(tokens, P);
            v.inrange = v.Dact >= 10000000000000LL && v.Dact < 100000000000000LL;
        }
    } else if (mode == QM_BIN) {
        const double w = tokens * P;                                     // exact scaling
        if (w >= 4503599627370496.0 && w < 9007199254740992.0) {
            v.Dact = (int64_t)w;
            v.inrange = (double)v.Dact == w;
        }
    }
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

__device__ inline uint32_t pack_ident() {   // identity table: c -> c
    uint32_t f = 0;
    for (int k = 0; k < 5; k++) f |= (uint32_t)k << (3 * k);
    return f;
}
// (f after g): apply g first, then f
__device__ inline uint32_t compose(uint32_t f, uint32_t g) {
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) {
        uint32_t gk = (g >> (3 * k)) & 7u;
        uint32_t hk = gk == STOPC ? STOPC : ((f >> (3 * gk)) & 7u);
        h |= hk << (3 * k);
    }
    return h;
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

template <int NC>
struct CoopShared {
    ChunkSlot ring[2][NC];            // chunk k in slot k&1, filled by the loader wave
    int64_t wtot[NC / 64];
    uint64_t wnear[NC / 64];
    uint32_t wev[NC / 64];
    uint32_t wbad[NC / 64];
    double nadd[MAX_NEAR], ncap[MAX_NEAR], nnd[MAX_NEAR];
    int64_t npred[MAX_NEAR], nr[MAX_NEAR];
    uint32_t nlane[MAX_NEAR];
    uint8_t ntab[MAX_NEAR * 5];
    int8_t cafter[MAX_NEAR];
    uint32_t stop_lane;
    int64_t baseD;
    int32_t baseE;
};

template <int NC>
__device__ inline void replay_tb_coop(CoopShared<NC>& sh, TbEntry* e, uint32_t j0, uint32_t j1,
                                      const CfgDev* __restrict__ cfgs, int32_t profile, const ReqArgs& a,
                                      const TbPre& pre, uint32_t* dbg) {
    constexpr int NWC = NC / 64;                 // compute waves
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const bool loader = wave == (uint32_t)NWC;
    const uint64_t lt = (1ull << lane) - 1ull;
    uint32_t nrounds = 0, nchunks = 0;
    uint64_t cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t0 = 0, t1 = 0;
    (void)cyc; (void)t0; (void)t1;
#ifdef RL_STAMPS
#define RL_PHASE(k) do { RL_STAMP(t1); cyc[k] += t1 - t0; t0 = t1; } while (0)
#else
#define RL_PHASE(k) do { } while (0)
#endif
    if (tid == 0) {
        TbQ q = tb_quant(e->tok, profile);
        sh.baseD = q.D;
        sh.baseE = q.E;
    }
    // loader: the chunk after next, NC/64 entries per loader lane
    ChunkSlot fld[NWC];
    auto ld_fields = [&](uint32_t base) {
#pragma unroll
        for (int q = 0; q < NWC; q++) {
            const uint32_t j = base + lane + 64 * q;
            ChunkSlot f{0.0, 1, 0, 0, 0};
            if (base < j1 && j < j1) {
                f.add = pre.add[j];
                f.n = a.n[j];
                f.reset = pre.reset[j];
                f.c = a.cfg[j];
                f.alive = pre.alive[j];
            }
            fld[q] = f;
        }
    };
    auto st_fields = [&](int slot) {
#pragma unroll
        for (int q = 0; q < NWC; q++) sh.ring[slot][lane + 64 * q] = fld[q];
    };
    if (loader) {
        ld_fields(j0);
        st_fields(0);
        ld_fields(j0 + NC);
    }
    __syncthreads();
    uint32_t k = 0;
    for (uint32_t base = j0; base < j1; base += NC, k++) {
        const uint32_t cnt = (j1 - base) < (uint32_t)NC ? (j1 - base) : (uint32_t)NC;
        const bool act = !loader && tid < cnt;
        const ChunkSlot rq = loader ? ChunkSlot{0.0, 1, 0, 0, 0} : sh.ring[k & 1][tid];
        const uint32_t i = base + tid;     // sorted position
        const CfgDev& cf = cfgs[rq.c];     // LDS copy (see k_replay)
        const double add = rq.add, cap = cf.limit_d, nd = (double)rq.n;
        const bool alive = rq.alive != 0;
        nchunks++;
        uint32_t first = 0;
        RL_STAMP(t0);
        while (first < cnt) {              // block-uniform
            nrounds++;
            const int64_t D = sh.baseD;
            const int32_t E = sh.baseE;
            int mode = QM_NONE;
            double P = 1.0, R = 1.0, tau = 0.0;
            if (profile == PROFILE_REDIS7) {
                if (13 - E >= 1 && 13 - E <= 22 && D >= 10000000000000LL && D < 100000000000000LL) {
                    mode = QM_DEC;
                    P = rlq::pow10_exact(13 - E);
                    R = 1.0 / P;
                    tau = TAU_DEC;
                }
            } else if (D >= (1LL << 52) && D < (1LL << 53) && E > -1000 && E < 900) {
                mode = QM_BIN;
                P = ldexp(1.0, -E);
                R = ldexp(1.0, E);
            }
            const bool mine = act && tid >= first;
            if (mode == QM_NONE) {
                // off the fast decades (or an empty/zero state): one exact step
                if (tid == first) {
                    TbEval v = tb_eval(QM_NONE, D, E, P, R, alive, add, cap, nd, profile);
                    write_out(a, i, tb_outputs(v, rq.n, rq.reset, cf.rate, cf.inv_rate));
                    TbQ q = tb_quant(v.tokens, profile);
                    sh.baseD = q.D;
                    sh.baseE = q.E;
                }
                lds_barrier();
                first++;
                continue;
            }
            // 1. nominal increment, near-tie flag, event flags that need no prefix
            int64_t r = 0;
            bool near = false, ev = !alive;
            if (mine) {
                const double pr = add * P;
                const double err = (mode == QM_DEC) ? __builtin_fma(add, P, -pr) : 0.0;
                const double rr = rint(pr);
                if (!(pr < 1e15 && pr > -1e15)) {
                    ev = true;
                } else {
                    r = (int64_t)rr;
                    const double dist = fabs((pr - rr) + err);       // distance to nearest integer
                    near = (mode == QM_DEC) ? dist > 0.5 - tau : dist >= 0.5;
                }
            }
            const int64_t rin = mine ? r : 0;
            const int64_t inc = wave_incl_scan_i64(rin);
            const uint64_t nmask = __ballot(mine && near);
            if (!loader) {
                if (lane == 63) sh.wtot[wave] = inc;
                if (lane == 0) sh.wnear[wave] = nmask;
            }
            lds_barrier();                                                   // 1
            RL_PHASE(0);
            // cross-wave prefixes: one LDS read per lane, DPP scans, readlane
            const int64_t wt = lane < (uint32_t)NWC ? sh.wtot[lane] : 0;
            const uint64_t wn = lane < (uint32_t)NWC ? sh.wnear[lane] : 0ull;
            const uint32_t wnc = (uint32_t)__popcll(wn);
            const int64_t wt_inc = wave_incl_scan_i64(wt);
            const uint32_t wn_inc = wave_scan_u32(wnc, 0u, [](uint32_t x, uint32_t y) { return x + y; });
            const uint32_t wsel = wave < (uint32_t)NWC ? wave : 0u;
            const int64_t pre_sum = wave < (uint32_t)NWC ? readlane_i64(wt_inc - wt, wsel) : 0;
            const uint32_t nbefore = wave < (uint32_t)NWC ? (uint32_t)__builtin_amdgcn_readlane((int)(wn_inc - wnc), (int)wsel) : 0u;
            const int64_t Pj = pre_sum + inc - rin;                          // exclusive prefix
            const uint32_t nrank = nbefore + (loader ? 0u : (uint32_t)__popcll(nmask & lt));
            // 2. events possible even with |c| <= 2
            if (mine && !ev) {
                const int64_t Dn = D + Pj + r;
                const int64_t M = 4;
                if (mode == QM_DEC) ev = (Dn - M < 10000000000000LL) || (Dn + M >= 100000000000000LL);
                else ev = (Dn - M < (1LL << 52)) || (Dn + M >= (1LL << 53));
                const double vhi = (double)(Dn + M) * R * (1.0 + 1e-9);
                ev = ev || vhi >= nd || vhi >= cap || (near && nrank >= (uint32_t)MAX_NEAR);
            }
            const uint64_t emask = __ballot(mine && ev);
            if (!loader && lane == 0)
                sh.wev[wave] = emask ? (uint32_t)(wave * 64 + __ffsll((unsigned long long)emask) - 1) : (uint32_t)NC;
            lds_barrier();                                                   // 2
            uint32_t eidx = wave_min_u32(lane < (uint32_t)NWC ? sh.wev[lane] : (uint32_t)NC);
            if (eidx >= cnt) eidx = cnt - 1;
            // near-tie lanes strictly before e: publish their inputs
            uint32_t NN = 0;
            {
                const uint32_t ew = eidx >> 6, el = eidx & 63;
                const uint32_t before = (uint32_t)__builtin_amdgcn_readlane((int)(wn_inc - wnc), (int)ew);
                const uint64_t wmask = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wn, (int)ew) |
                                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(wn >> 32), (int)ew) << 32);
                NN = before + (uint32_t)__popcll(wmask & ((1ull << el) - 1ull));
            }
            if (mine && near && tid < eidx) {
                sh.nadd[nrank] = add;
                sh.ncap[nrank] = cap;
                sh.nnd[nrank] = nd;
                sh.npred[nrank] = D + Pj;
                sh.nr[nrank] = r;
                sh.nlane[nrank] = tid;
            }
            lds_barrier();                                                   // 3
            RL_PHASE(1);
            // 3. candidate tables: one (near lane, c) pair per compute thread
            if (!loader && tid < NN * 5) {
                const uint32_t rk = tid / 5;
                const int32_t cc = (int32_t)(tid % 5) - 2;
                const int64_t base_pred = sh.npred[rk];
                TbEval v = tb_eval(mode, base_pred + cc, E, P, R, true, sh.nadd[rk], sh.ncap[rk], sh.nnd[rk],
                                   profile);
                uint32_t entry = STOPC;
                if (v.inrange && !v.allowed && !v.clamped) {
                    const int64_t cp = v.Dact - (base_pred + sh.nr[rk]);
                    if (cp >= -2 && cp <= 2) entry = (uint32_t)(cp + 2);
                }
                sh.ntab[rk * 5 + (cc + 2)] = (uint8_t)entry;
            }
            lds_barrier();                                                   // 4
            RL_PHASE(2);
            // 4. one wave composes the tables: correction after each near lane
            if (wave == 0) {
                uint32_t f = pack_ident();
                if (lane < NN) {
                    f = 0;
                    for (int q = 0; q < 5; q++) f |= (uint32_t)sh.ntab[lane * 5 + q] << (3 * q);
                }
                f = wave_scan_u32(f, pack_ident(), [](uint32_t x, uint32_t y) { return compose(x, y); });
                const uint32_t c0v = (f >> 6) & 7u;                          // entry for c = 0
                const uint64_t smask = __ballot(lane < NN && c0v == STOPC);
                if (lane < NN) sh.cafter[lane] = (int8_t)((int32_t)c0v - 2);
                if (lane == 0) sh.stop_lane = smask ? sh.nlane[__ffsll((unsigned long long)smask) - 1] : (uint32_t)NC;
            }
            lds_barrier();                                                   // 5
            RL_PHASE(3);
            if (sh.stop_lane < eidx) eidx = sh.stop_lane;
            // 5. every lane up to e: the exact step from its true predecessor
            bool bad = false;
            TbEval v{};
            int64_t Dexp = 0;
            if (mine && tid <= eidx) {
                const int32_t cin = nrank > 0 ? (int32_t)sh.cafter[nrank - 1] : 0;
                v = tb_eval(mode, D + Pj + cin, E, P, R, alive, add, cap, nd, profile);
                const int32_t cout = near ? (nrank < MAX_NEAR ? (int32_t)sh.cafter[nrank] : 99) : cin;
                Dexp = D + Pj + r + cout;
                if (tid < eidx) bad = !(alive && v.inrange && !v.allowed && !v.clamped && v.Dact == Dexp);
            }
            const uint64_t bmask = __ballot(bad);
            if (!loader && lane == 0)
                sh.wbad[wave] = bmask ? (uint32_t)(wave * 64 + __ffsll((unsigned long long)bmask) - 1) : (uint32_t)NC;
            lds_barrier();                                                   // 6
            RL_PHASE(4);
            {
                const uint32_t mb = wave_min_u32(lane < (uint32_t)NWC ? sh.wbad[lane] : (uint32_t)NC);
                eidx = mb < eidx ? mb : eidx;
            }
            // 6. commit lanes [first, e]; e's exact result is the next base
            if (mine && tid <= eidx) write_out(a, i, tb_outputs(v, rq.n, rq.reset, cf.rate, cf.inv_rate));
            if (tid == eidx) {
                TbQ q = (v.inrange && mode == QM_DEC) || (v.inrange && mode == QM_BIN) ? TbQ{v.Dact, E}
                                                                                     : tb_quant(v.tokens, profile);
                sh.baseD = q.D;
                sh.baseE = q.E;
            }
            lds_barrier();                                                   // 7
            RL_PHASE(5);
            first = eidx + 1;
        }
        if (loader) {          // chunk k+1 -> ring, start loading chunk k+2
            st_fields((k + 1) & 1);
            ld_fields(base + 2 * NC);
        }
        lds_barrier();
    }
    if (tid == 0) {
        e->tok = tb_value(sh.baseD, sh.baseE, profile);
        e->last = pre.lq[j1 - 1];
        e->when = pre.when[j1 - 1];
        if (dbg) { atomicAdd(&dbg[0], nrounds); atomicAdd(&dbg[1], nchunks); }
#ifdef RL_STAMPS
        if (dbg) {
            atomicMax(&dbg[2], nrounds);
            for (int q = 0; q < 6; q++) atomicMax((unsigned long long*)&dbg[8 + 2 * q], (unsigned long long)cyc[q]);
        }
#endif
    }
}

struct SegRec {
    uint32_t j0;
    uint32_t len;
};

// segment heads -> (start, length), split into heavy (cooperative) and light
// (one thread each) work lists.  One tile of SEG_TILE sorted positions per
// block; list slots are reserved with ONE global atomic per list per block
// (a single contended word sustains only ~88 atomics/us on MI355X).
constexpr int SEG_ITEMS = 16;
constexpr int SEG_TILE = 256 * SEG_ITEMS;

__global__ __launch_bounds__(256) void k_segments(const uint32_t* __restrict__ sk, uint32_t m,
                                                  uint32_t invalid_key, uint32_t heavy_min, SegRec* heavy,
                                                  uint32_t* nheavy, SegRec* light, uint32_t* nlight) {
    __shared__ uint32_t s_cnt[2], s_base[2];
    const uint32_t tid = threadIdx.x;
    for (uint32_t tile = blockIdx.x; tile * SEG_TILE < m; tile += gridDim.x) {
        if (tid < 2) s_cnt[tid] = 0;
        __syncthreads();
        SegRec rec[SEG_ITEMS];
        uint32_t slot[SEG_ITEMS];
#pragma unroll
        for (int j = 0; j < SEG_ITEMS; j++) {
            uint32_t i = tile * SEG_TILE + j * 256 + tid;
            slot[j] = 0xffffffffu;
            if (i >= m) continue;
            uint32_t k = sk[i];
            bool head = k != invalid_key && (i == 0 || sk[i - 1] != k);
            if (!head) continue;
            uint32_t len = seg_end(sk, m, i, k) - i;
            rec[j] = SegRec{i, len};
            uint32_t which = len >= heavy_min ? 0u : 1u;
            slot[j] = (which << 31) | atomicAdd(&s_cnt[which], 1u);
        }
        __syncthreads();
        if (tid == 0) s_base[0] = s_cnt[0] ? atomicAdd(nheavy, s_cnt[0]) : 0u;
        if (tid == 1) s_base[1] = s_cnt[1] ? atomicAdd(nlight, s_cnt[1]) : 0u;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < SEG_ITEMS; j++) {
            if (slot[j] == 0xffffffffu) continue;
            uint32_t which = slot[j] >> 31, off = slot[j] & 0x7fffffffu;
            if (which == 0) heavy[s_base[0] + off] = rec[j];
            else light[s_base[1] + off] = rec[j];
        }
        __syncthreads();
    }
}

// requests in sorted order (one coalesced pass; random reads of the 28 B
// request records, which stay in the Infinity Cache at 1M-request batches),
// plus the token-bucket precomputation (TbPre)
__global__ __launch_bounds__(256) void k_permute(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                 uint32_t m, uint32_t invalid_key, uint32_t win_base,
                                                 const TbEntry* __restrict__ tb, const CfgDev* __restrict__ cfgs,
                                                 int32_t profile, ReqArgs in, ReqArgs out, TbPre pre) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        const uint32_t k0 = sk[j];
        if (k0 == invalid_key) continue;
        const uint32_t i = sv[j];
        const int64_t t = in.ts[i];
        const uint32_t c = in.cfg[i];
        const int64_t sms = in.sms ? in.sms[i] : floor_div(t, 1000000LL);
        // `out` is the engine's own permuted buffers (ReqArgs keeps inputs const)
        const_cast<int64_t*>(out.ts)[j] = t;
        const_cast<int64_t*>(out.n)[j] = in.n[i];
        const_cast<uint32_t*>(out.cfg)[j] = c;
        const_cast<int64_t*>(out.sms)[j] = sms;
        if (k0 >= win_base) continue;
        const CfgDev& C = cfgs[c];
        const double now = (double)t / 1e9;
        double prev_last;
        int64_t prev_when;
        if (j == 0 || sk[j - 1] != k0) {
            prev_last = tb[k0].last;
            prev_when = tb[k0].when;
        } else {
            const uint32_t ip = sv[j - 1];
            const int64_t tp = in.ts[ip];
            const int64_t smsp = in.sms ? in.sms[ip] : floor_div(tp, 1000000LL);
            prev_last = lua_tostring_roundtrip((double)tp / 1e9, profile);
            prev_when = expire_when(cfgs[in.cfg[ip]].ttl_tb, smsp);
        }
        const bool alive = key_alive(prev_when, sms, profile);
        const double last = alive ? prev_last : now;
        pre.add[j] = (now - last) * C.rate;
        pre.alive[j] = alive ? 1 : 0;
        pre.reset[j] = tb_reset_at(now, C);
        pre.lq[j] = lua_tostring_roundtrip(now, profile);
        pre.when[j] = expire_when(C.ttl_tb, sms);
    }
}

// results from sorted order back to the caller's order
__global__ __launch_bounds__(256) void k_unpermute(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                   uint32_t m, uint32_t invalid_key, ReqArgs sorted, ReqArgs out) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        if (sk[j] == invalid_key) continue;
        uint32_t i = sv[j];
        out.dec[i] = sorted.dec[j];
        out.rem[i] = sorted.rem[j];
        out.retry[i] = sorted.retry[j];
        out.reset[i] = sorted.reset[j];
        if (out.tok) out.tok[i] = sorted.tok[j];
    }
}

// Work-queue replay: blocks first drain the heavy list (one segment per block,
// cooperative), then the light list (256 segments per grab, one per thread).
constexpr int COOP_NC = 448;                 // compute lanes per cooperative block
constexpr int REPLAY_BLOCK = COOP_NC + 64;  // + one loader wave

template <bool LCFG>
__global__ __launch_bounds__(REPLAY_BLOCK) void k_replay(
    const uint32_t* __restrict__ sk, const SegRec* __restrict__ heavy,
    const uint32_t* __restrict__ nheavy_p, const SegRec* __restrict__ light,
    const uint32_t* __restrict__ nlight_p, uint32_t* qctr, uint32_t win_base, TbEntry* tb, WinEntry* win,
    const CfgDev* __restrict__ gcfgs, uint32_t ncfg, int32_t profile, ReqArgs a, TbPre pre, uint32_t* eflags,
    uint32_t* dbg) {
    __shared__ CoopShared<COOP_NC> sh;
    __shared__ uint32_t s_u;
    __shared__ CfgDev s_cfg[LCFG ? MAX_LCFG : 1];
    if (LCFG) {
        for (uint32_t c = threadIdx.x; c < ncfg; c += blockDim.x) s_cfg[c] = gcfgs[c];
        __syncthreads();
    }
    const CfgDev* cfgs = LCFG ? s_cfg : gcfgs;
    const uint32_t nheavy = *nheavy_p, nlight = *nlight_p;
    for (;;) {
        if (threadIdx.x == 0) s_u = atomicAdd(&qctr[0], 1u);
        __syncthreads();
        const uint32_t u = s_u;
        __syncthreads();
        if (u >= nheavy) break;
        const SegRec sg = heavy[u];
        const uint32_t k0 = sk[sg.j0];
        if (k0 < win_base) {
            replay_tb_coop<COOP_NC>(sh, &tb[k0], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre, dbg);
        } else if (threadIdx.x == 0) {
            replay_win_serial(&win[k0 - win_base], sg.j0, sg.j0 + sg.len, cfgs, profile, a, eflags);
        }
        __syncthreads();
    }
    for (;;) {
        if (threadIdx.x == 0) s_u = atomicAdd(&qctr[1], (uint32_t)REPLAY_BLOCK);
        __syncthreads();
        const uint32_t u0 = s_u;
        __syncthreads();
        if (u0 >= nlight) break;
        const uint32_t u = u0 + threadIdx.x;
        if (u < nlight) {
            const SegRec sg = light[u];
            const uint32_t k0 = sk[sg.j0];
            if (k0 < win_base) replay_tb_serial(&tb[k0], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre);
            else replay_win_serial(&win[k0 - win_base], sg.j0, sg.j0 + sg.len, cfgs, profile, a, eflags);
        }
    }
}

}  // namespace rl
