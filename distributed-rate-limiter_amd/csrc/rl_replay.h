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

__device__ inline void replay_tb_serial(TbEntry* e, uint32_t j0, uint32_t j1, const CfgDev* cfgs,
                                        int32_t profile, const ReqArgs& a) {
    TbState st{e->tok, e->last, e->when};
    Req cur = load_req(a, j0);
    for (uint32_t j = j0; j < j1; j++) {
        Req nxt = cur;
        if (j + 1 < j1) nxt = load_req(a, j + 1);
        Out o = tb_step(st, cur.t, cur.n, cur.sms, cfgs[cur.c], profile);
        write_out(a, j, o);
        cur = nxt;
    }
    e->tok = st.tok;
    e->last = st.last;
    e->when = st.when;
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
constexpr int COOP = 256;
constexpr int COOP_WAVES = COOP / 64;

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

// One chunk's requests as the loader wave hands them to the compute waves.
struct ChunkSlot {
    int64_t t, n, sms;
    uint32_t c, pad;
};

// configs cached in LDS per block (when the engine has at most MAX_LCFG)
constexpr int MAX_LCFG = 32;

struct CoopShared {
    ChunkSlot ring[2][COOP];  // requests of chunk k (slot k&1), filled by the loader wave
    double L[COOP];           // stored last_refill after each lane's step
    int64_t W[COOP];          // key expiry after each lane's step
    int64_t scan_tmp[COOP_WAVES];
    uint32_t min_tmp[COOP_WAVES];
    int64_t baseD;
    int32_t baseE;
    uint32_t need_full;       // committed lane must re-quantize its tokens
    double carryL;
    int64_t carryW;
    double full_tokens;
};

// The replay block: COOP compute lanes (4 waves) + one loader wave.  The
// loader is the only wave that loads the (sorted-order) request fields, two
// chunks ahead, into an LDS ring.  On gfx9 loads and stores
// share vmcnt, so a compute wave that both scattered results and waited on
// its own prefetch would wait for its stores; here compute waves never wait
// on global memory in the steady state.
constexpr int REPLAY_BLOCK = COOP + 64;
constexpr uint32_t NO_REQ = 0xffffffffu;

__device__ inline void replay_tb_coop(CoopShared& sh, TbEntry* e, uint32_t j0, uint32_t j1,
                                      const CfgDev* __restrict__ cfgs, int32_t profile, const ReqArgs& a,
                                      uint32_t* dbg) {
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    const bool loader = wave == COOP_WAVES;
    uint32_t nrounds = 0, nchunks = 0;
    uint64_t cyc[5] = {0, 0, 0, 0, 0}, t0 = 0, t1 = 0;
    (void)cyc; (void)t0; (void)t1;
    if (tid == 0) {
        TbQ q = tb_quant(e->tok, profile);
        sh.baseD = q.D;
        sh.baseE = q.E;
        sh.carryL = e->last;
        sh.carryW = e->when;
    }
    // loader state: requests of the chunk after next (4 per loader lane).
    // Compute waves read only LDS (ring + config cache): on gfx9 a wait on any
    // global load would also wait for the result stores they keep in flight
    // (loads and stores share vmcnt).
    ChunkSlot fld[4];
    auto ld_fields = [&](uint32_t base) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t j = base + lane + 64 * q;
            ChunkSlot f{0, 1, 0, 0, 0};
            if (base < j1 && j < j1) {
                f.t = a.ts[j];
                f.n = a.n[j];
                f.sms = a.sms[j];
                f.c = a.cfg[j];
            }
            fld[q] = f;
        }
    };
    auto st_fields = [&](int slot) {
#pragma unroll
        for (int q = 0; q < 4; q++) sh.ring[slot][lane + 64 * q] = fld[q];
    };
    if (loader) {            // prologue: chunk 0 into slot 0, chunk 1 in flight
        ld_fields(j0);
        st_fields(0);
        ld_fields(j0 + COOP);
    }
    __syncthreads();
    uint32_t k = 0;
    for (uint32_t base = j0; base < j1; base += COOP, k++) {
        const uint32_t cnt = (j1 - base) < (uint32_t)COOP ? (j1 - base) : (uint32_t)COOP;
        const bool act = !loader && tid < cnt;
        RL_STAMP(t0);
        ChunkSlot rq = loader ? ChunkSlot{0, 1, 0, 0, 0} : sh.ring[k & 1][tid];
        const uint32_t i = base + tid;      // sorted position
        const int64_t t = rq.t, nn = rq.n, sms = rq.sms;
        const CfgDev& cf = cfgs[rq.c];      // LDS copy (see k_replay)
        nchunks++;
        const double now = (double)t / 1e9;
        const double Lq = act ? lua_tostring_roundtrip(now, profile) : 0.0;
        const int64_t wafter = expire_when(cf.ttl_tb, sms);
        const int64_t reset_at = tb_reset_at(now, cf);
        if (!loader) {
            sh.L[tid] = Lq;
            sh.W[tid] = wafter;
        }
        lds_barrier();
        const uint32_t pv = (tid > 0 && tid < (uint32_t)COOP) ? tid - 1 : 0;
        const double prevL = tid ? sh.L[pv] : sh.carryL;
        const int64_t prevW = tid ? sh.W[pv] : sh.carryW;
        const bool alive = key_alive(prevW, sms, profile);
        const double last = alive ? prevL : now;
        const double add = (now - last) * cf.rate;     // elapsed * refill_rate
        const double cap = cf.limit_d, nd = (double)nn, rate = cf.rate, inv_rate = cf.inv_rate;
        RL_STAMP(t1);
#ifdef RL_STAMPS
        cyc[0] += t1 - t0;
#endif
        uint32_t first = 0;
        int32_t scaleE = INT32_MIN;
        double scale = 0.0, P = 1.0, R = 1.0;
        bool fastdec = false;
        while (first < cnt) {                           // block-uniform
            const int64_t D = sh.baseD;
            const int32_t E = sh.baseE;
            const bool mine = act && tid >= first;
            nrounds++;
            if (E != scaleE) {
                scaleE = E;
                scale = tb_scale(E, profile);
                // Redis profile, decade with an exact power of ten: short chain
                fastdec = profile == PROFILE_REDIS7 && (13 - E) >= 1 && (13 - E) <= 22;
                if (fastdec) { P = rlq::pow10_exact(13 - E); R = 1.0 / P; }
            }
            int64_t r = 0;
            bool force = !alive;
            if (mine) {
                double v = add * scale;
                if (!(v < 1e15 && v > -1e15)) force = true;
                else r = (int64_t)rint(v);
            }
            // exclusive block scan of r: DPP within the wave, wave totals via LDS
            RL_STAMP(t0);
            const int64_t rin = mine ? r : 0;
            const int64_t inc = wave_incl_scan_i64(rin);
            if (lane == 63 && !loader) sh.scan_tmp[wave] = inc;
            lds_barrier();                                               // A
            int64_t pre = 0;
            for (uint32_t w = 0; w < wave && w < (uint32_t)COOP_WAVES; w++) pre += sh.scan_tmp[w];
            const int64_t Dg = D + pre + inc - rin;
            RL_STAMP(t1);
#ifdef RL_STAMPS
            cyc[1] += t1 - t0; t0 = t1;
#endif
            bool ok = false, full = false;
            Out o;
            TbQ q{0, 0};
            double tokens = 0.0;
            if (mine) {
                // tokenBucketScript from the guessed stored state (tokenbucket.go:32-51)
                double T;
                if (!alive) T = cap;
                else if (fastdec && Dg > 0) T = rlq::div_pow10((double)Dg, P, R);   // == strtod(D e(E-13))
                else T = tb_value(Dg, E, profile);
                double sum = T + add;
                tokens = (sum < cap) ? sum : cap;
                bool allowed = false;
                if (tokens >= nd) { tokens = tokens - nd; allowed = true; }
                // tonumber(tostring(tokens)) as (digits, decade), and is it the guess?
                const int64_t Dexp = Dg + r;
                if (fastdec && tokens > 0.0 && tokens * P < 1.4e14) {
                    const int64_t Dact = rlq::round_scaled_P(tokens, P);
                    const bool inrange = Dact >= 10000000000000LL && Dact < 100000000000000LL;
                    ok = !force && inrange && Dact == Dexp;
                    full = !inrange;
                    q = TbQ{Dact, E};
                } else if (profile != PROFILE_REDIS7) {
                    int64_t ad = Dexp < 0 ? -Dexp : Dexp;
                    ok = !force && ad >= (1LL << 52) && ad < (1LL << 53) && tokens == ldexp((double)Dexp, E);
                    full = !ok;
                    q = TbQ{Dexp, E};
                } else {
                    full = true;    // off the fast decades: quantize in full if this lane commits
                }
                int64_t rem = go_f2i(floor(tokens));
                o.tokens = tokens;
                o.decision = allowed ? DEC_ALLOWED : DEC_DENIED;
                o.remaining = rem;
                o.reset_at = reset_at;
                o.retry = 0;
                if (!allowed) {
                    int64_t need = wsub(nn, rem);
                    // tokensNeeded / refillRate (tokenbucket.go:124-126); 1/rate precomputed
                    double w = need == 1 ? inv_rate : (double)need / rate;
                    int64_t d = go_f2i(w * 1e9);
                    o.retry = d < 0 ? 0 : d;
                }
            }
            RL_STAMP(t1);
#ifdef RL_STAMPS
            cyc[2] += t1 - t0; t0 = t1;
#endif
            // first lane whose exact result differs from its guess
            const uint64_t bad = __ballot(mine && !ok);
            if (lane == 0 && !loader)
                sh.min_tmp[wave] = bad ? (uint32_t)(wave * 64 + __ffsll((unsigned long long)bad) - 1) : COOP;
            lds_barrier();                                               // B
            uint32_t s = COOP;
            for (int w = 0; w < COOP_WAVES; w++) s = sh.min_tmp[w] < s ? sh.min_tmp[w] : s;
            if (s >= cnt) s = cnt - 1;
            RL_STAMP(t1);
#ifdef RL_STAMPS
            cyc[3] += t1 - t0; t0 = t1;
#endif
            if (mine && tid <= s) write_out(a, i, o);
            if (tid == s) {
                if (full) q = tb_quant(tokens, profile);   // decade change, allow, zero, slow path
                sh.baseD = q.D;
                sh.baseE = q.E;
            }
            lds_barrier();                                               // C
            RL_STAMP(t1);
#ifdef RL_STAMPS
            cyc[4] += t1 - t0;
#endif
            first = s + 1;
        }
        if (tid == cnt - 1) {
            sh.carryL = Lq;
            sh.carryW = wafter;
        }
        if (loader) {        // chunk k+1 (loaded during this chunk) -> ring; start chunk k+2
            st_fields((k + 1) & 1);
            ld_fields(base + 2 * COOP);
        }
        lds_barrier();
    }
    if (tid == 0) {
        e->tok = tb_value(sh.baseD, sh.baseE, profile);
        e->last = sh.carryL;
        e->when = sh.carryW;
        if (dbg) { atomicAdd(&dbg[0], nrounds); atomicAdd(&dbg[1], nchunks); }
#ifdef RL_STAMPS
        // phase cycles of the LONGEST cooperative segment of the batch (max)
        if (dbg) for (int k = 0; k < 5; k++) atomicMax((unsigned long long*)&dbg[8 + 2 * k], (unsigned long long)cyc[k]);
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
// request records, which stay in the Infinity Cache at 1M-request batches)
__global__ __launch_bounds__(256) void k_permute(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                 uint32_t m, uint32_t invalid_key, ReqArgs in, ReqArgs out) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        if (sk[j] == invalid_key) continue;
        uint32_t i = sv[j];
        int64_t t = in.ts[i];
        // `out` is the engine's own permuted buffers (ReqArgs keeps inputs const)
        const_cast<int64_t*>(out.ts)[j] = t;
        const_cast<int64_t*>(out.n)[j] = in.n[i];
        const_cast<uint32_t*>(out.cfg)[j] = in.cfg[i];
        const_cast<int64_t*>(out.sms)[j] = in.sms ? in.sms[i] : floor_div(t, 1000000LL);
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
template <bool LCFG>
__global__ __launch_bounds__(REPLAY_BLOCK) void k_replay(
    const uint32_t* __restrict__ sk, const SegRec* __restrict__ heavy,
    const uint32_t* __restrict__ nheavy_p, const SegRec* __restrict__ light,
    const uint32_t* __restrict__ nlight_p, uint32_t* qctr, uint32_t win_base, TbEntry* tb, WinEntry* win,
    const CfgDev* __restrict__ gcfgs, uint32_t ncfg, int32_t profile, ReqArgs a, uint32_t* eflags,
    uint32_t* dbg) {
    __shared__ CoopShared sh;
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
            replay_tb_coop(sh, &tb[k0], sg.j0, sg.j0 + sg.len, cfgs, profile, a, dbg);
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
            if (k0 < win_base) replay_tb_serial(&tb[k0], sg.j0, sg.j0 + sg.len, cfgs, profile, a);
            else replay_win_serial(&win[k0 - win_base], sg.j0, sg.j0 + sg.len, cfgs, profile, a, eflags);
        }
    }
}

}  // namespace rl
