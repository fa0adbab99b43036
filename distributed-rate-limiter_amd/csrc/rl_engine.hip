// rl_engine.hip -- MI355X batched rate-limit decision engine: kernels + C-ABI.
//
// One batch = one launch sequence on the engine stream:
//   probe    hash each request's key id into its HBM table (find-or-insert by
//            CAS), emit the 32-bit slot id as sort key, and accumulate the
//            radix histograms of every sort pass (fused)
//   sort     P one-sweep LSD radix passes (rl_sort.h): requests grouped by
//            slot, arrival order kept
//   segments one head per distinct slot -> unordered segment list
//   replay   per segment, the reference's per-request semantics in arrival
//            order, state gathered once and scattered once (rl_replay.h)
// Reference boundary replaced: go-redis Eval + Redis Lua + the Go arithmetic
// around it (tokenbucket.go:90-193, slidingwindow.go:68-185,
// fixedwindow.go:65-163); see include/rl_engine.h.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rl_engine.h"
#include "../../include/rl_keyhash.h"
#include "../../include/rl_route.h"
#include "rl_replay.h"
#include "rl_semantics.h"
#include "rl_sort.h"
#include "rl_table.h"

using namespace rl;

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------

__global__ void k_init_tb(TbEntry* t, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        t[i].key = EMPTY_KEY;
        t[i].tok = 0.0;
        t[i].last = 0.0;
        t[i].when = ABSENT;
    }
}

__global__ void k_init_win(WinEntry* t, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        t[i].key = EMPTY_KEY;
        t[i].nspill = 0;
        for (int k = 0; k < 2; k++) { t[i].s[k].ws = 0; t[i].s[k].cnt = 0; t[i].s[k].when = ABSENT; }
    }
}

// Table GC of the spill table, after the window table's k_rehash: every live
// spill entry moves to the fresh spill table (strict CAS: two entries of one
// user key may be moved at once) and is counted in its user key's new window
// entry.  counters as k_rehash.
__global__ void k_spill_rehash(const SpillEntry* __restrict__ old, uint64_t n_old, SpillEntry* nu, uint64_t mask_new,
                               WinEntry* win, uint64_t win_mask, int64_t now_ms, int32_t profile,
                               unsigned long long* counters) {
    unsigned long long live = 0, lost = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n_old;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const SpillEntry x = old[i];
        if (!entry_live(x, now_ms, profile)) continue;
        live++;
        const uint32_t w = probe_find(win, win_mask, x.key);
        uint64_t h = spill_home(x.key, mask_new);
        bool placed = false;
        for (uint64_t p = 0; w != NO_SLOT && p <= mask_new && p < MAX_PROBES; p++) {
            if (atomicCAS((unsigned long long*)&nu[h].key, (unsigned long long)EMPTY_KEY,
                          (unsigned long long)x.key) == EMPTY_KEY) {
                nu[h].ws = x.ws;
                nu[h].cnt = x.cnt;
                nu[h].when = x.when;
                atomicAdd((unsigned long long*)&win[w].nspill, 1ull);
                placed = true;
                break;
            }
            h = (h + 1) & mask_new;
        }
        if (!placed) lost++;
    }
    if (live) atomicAdd(&counters[0], live);
    if (lost) atomicAdd(&counters[1], lost);
}

__global__ void k_init_spill(SpillEntry* t, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        t[i] = SpillEntry{EMPTY_KEY, 0, 0, ABSENT};
}

constexpr int PROBE_BLOCK = 256;

// A batch the routing layer merged (include/rl_route.h): request p is
// rec[order[p]] (its store clock in the server-clock array), p < *count --
// a size in device memory, so the grid is sized for the caller's bound and
// every kernel reads the actual size -- and its result goes to res[order[p]]
struct RouteIn {
    const rl_route_rec* rec;
    const uint32_t* order;
    const uint32_t* count;
    rl_route_res* res;
};

// find-or-insert one request's key: its global slot (token-bucket table
// first, then the window table at win_base), or invalid_key when the request
// is not executed (n <= 0, unknown config, reserved key, table full)
__device__ inline uint32_t probe_request(uint64_t k, uint32_t c, int64_t nn, const CfgDev* __restrict__ cfgs,
                                         uint32_t ncfg, TbEntry* tb, uint64_t tb_mask, WinEntry* win,
                                         uint64_t win_mask, uint32_t win_base, uint32_t invalid_key, uint32_t& ef) {
    if (k == EMPTY_KEY) ef |= EF_BAD_KEY;
    if (!(c < ncfg && nn > 0 && k != EMPTY_KEY)) return invalid_key;
    if (cfgs[c].alg == ALG_TOKEN_BUCKET) {
        const uint32_t s = probe_insert(tb, tb_mask, k);
        if (s == NO_SLOT) { ef |= EF_TABLE_FULL; return invalid_key; }
        return s;
    }
    const uint32_t s = probe_insert(win, win_mask, k);
    if (s == NO_SLOT) { ef |= EF_TABLE_FULL; return invalid_key; }
    return win_base + s;
}

// find-or-insert every request's key; sort key = global slot id; fused
// per-pass digit histograms (LDS, then one global atomic per bin per block);
// pass p's digit is 8 bits at shift (shifts >> 8p) & 31 (see sort_shifts).
// Each thread takes PROBE_R requests and issues their loads phase by phase
// (inputs, then every first table probe) before resolving any: the kernel is
// latency-bound on random table reads, and this keeps PROBE_R of them in
// flight per thread instead of one.
// RT: the routed batch of RouteIn (the records read in merge order; XS, the
// store clock per request, is then always given).
template <int PROBE_R, bool XS, bool RT = false>
__global__ __launch_bounds__(PROBE_BLOCK) void k_probe(
    uint32_t m, const uint64_t* __restrict__ key, const int64_t* __restrict__ n,
    const uint32_t* __restrict__ cfg, const CfgDev* __restrict__ cfgs, uint32_t ncfg, TbEntry* tb,
    uint64_t tb_mask, WinEntry* win, uint64_t win_mask, uint32_t win_base, uint32_t invalid_key,
    uint32_t* __restrict__ sk, uint32_t* ghist, int passes, uint32_t shifts, ReqArgs a,
    ReqRec<XS>* __restrict__ rec, uint32_t* eflags, RouteIn ri, uint32_t* head, uint32_t nhead, RecSide side) {
    static_assert(!RT || XS, "a routed batch carries its store clock");
    // the batch set's head words (rl_engine.hip CTRL_HEAD), before any later
    // kernel of the batch touches them
    if (blockIdx.x == 0)
        for (uint32_t k = threadIdx.x; k < nhead; k += PROBE_BLOCK) head[k] = 0u;
    if (RT) {
        // a count above the caller's bound m_max: the requests past it get no
        // result record -- reported, never silent (rl_engine_sync: RL_EOVERFLOW)
        const uint32_t cnt = *ri.count;
        if (cnt > m && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(eflags, EF_ROUTED_OVER);
        m = min(m, cnt);
    }
    // a routed batch in received order (RL_ORDER_IDENTITY): request i is
    // rec[i], its store clock from its ts and the clock of the earlier steps
    const bool ident = RT && m && ri.order[0] == RL_ORDER_IDENTITY;
    const int64_t clock0 = ident ? a.sms[0] : 0;
    __shared__ uint32_t lh[4][RADIX];
    for (int p = 0; p < 4; p++) lh[p][threadIdx.x] = 0;
    __syncthreads();
    uint32_t ef = 0;
    for (uint32_t i0 = blockIdx.x * (PROBE_BLOCK * PROBE_R) + threadIdx.x; i0 < m;
         i0 += gridDim.x * (PROBE_BLOCK * PROBE_R)) {
        uint64_t k[PROBE_R], h[PROBE_R], cur[PROBE_R];
        uint32_t c[PROBE_R];
        int64_t nn[PROBE_R], t[PROBE_R], sms[PROBE_R];
        bool tbk[PROBE_R], go[PROBE_R];
#pragma unroll
        for (int r = 0; r < PROBE_R; r++) {   // inputs
            const uint32_t i = i0 + r * PROBE_BLOCK;
            const bool v = i < m;
            if (RT) {
                rl_route_rec q{};
                if (v) q = ri.rec[ident ? i : ri.order[i]];
                k[r] = v ? q.key : EMPTY_KEY;
                c[r] = q.cfg;
                nn[r] = q.n;
                t[r] = q.ts;
                if (ident) {
                    const int64_t ms = floor_div(q.ts, 1000000LL);
                    sms[r] = ms > clock0 ? ms : clock0;
                } else {
                    sms[r] = v ? a.sms[i] : 0;
                }
            } else {
                k[r] = v ? key[i] : EMPTY_KEY;
                c[r] = v ? cfg[i] : 0u;
                nn[r] = v ? n[i] : 0;
                t[r] = v ? a.ts[i] : 0;
                sms[r] = v && XS ? a.sms[i] : 0;
            }
        }
#pragma unroll
        for (int r = 0; r < PROBE_R; r++) {   // first probes, all in flight
            const uint32_t i = i0 + r * PROBE_BLOCK;
            if (i < m && k[r] == EMPTY_KEY) ef |= EF_BAD_KEY;
            go[r] = i < m && c[r] < ncfg && nn[r] > 0 && k[r] != EMPTY_KEY;
            tbk[r] = go[r] && cfgs[c[r]].alg == ALG_TOKEN_BUCKET;
            h[r] = mix64(k[r]) & (tbk[r] ? tb_mask : win_mask);
            cur[r] = go[r] ? (tbk[r] ? tb[h[r]].key : win[h[r]].key) : EMPTY_KEY;
        }
#pragma unroll
        for (int r = 0; r < PROBE_R; r++) {   // resolve, record, histogram
            const uint32_t i = i0 + r * PROBE_BLOCK;
            if (i >= m) continue;
            uint32_t slot = invalid_key;
            bool ins = false;
            if (go[r]) {
                const uint32_t s = tbk[r] ? probe_insert_at(tb, tb_mask, k[r], h[r], cur[r], &ins)
                                          : probe_insert_at(win, win_mask, k[r], h[r], cur[r], &ins);
                if (s == NO_SLOT) ef |= EF_TABLE_FULL;
                else slot = tbk[r] ? s : win_base + s;
            }
            sk[i] = slot;
            // one record per request: k_permute's sorted-order gather then
            // touches one line fragment instead of four arrays
            // REC_FRESH: this request inserted its key, so no earlier batch
            // has it, and a request alone with its key in the batch starts
            // from the absent state (replay phase 3 then skips the entry read)
            rec[i] = rec_pack<XS>(t[r], nn[r], sms[r], c[r], i | (ins ? REC_FRESH : 0u), side);
            for (int p = 0; p < passes; p++)
                atomicAdd(&lh[p][(slot >> ((shifts >> (8 * p)) & 31u)) & (RADIX - 1)], 1u);
        }
    }
    if (ef) atomicOr(eflags, ef);
    __syncthreads();
    for (int p = 0; p < passes; p++) {
        uint32_t v = lh[p][threadIdx.x];
        if (v) atomicAdd(&ghist[p * RADIX + threadIdx.x], v);
    }
}

// Small batches (m <= SMALL_MAX): the whole launch sequence in one workgroup
// and one launch -- find-or-insert, a bitonic sort of (slot, arrival index) in
// LDS, the sorted-order copy with the state-free token-bucket precomputation
// (as k_permute), one thread per key segment replaying it serially
// (replay_tb_serial / replay_win_serial, the big path's exact fallbacks), and
// the results in the caller's order (as k_unpermute).  A request-coalescing
// server at moderate load sends batches of a few to a few thousand requests;
// for them the big path's ten launches on three streams cost more than the
// work.  Same semantics, same table: batches of either size may interleave.
#ifndef RL_SMALL_BLOCK
#define RL_SMALL_BLOCK 1024
#endif
constexpr int SMALL_BLOCK = RL_SMALL_BLOCK;
constexpr uint32_t SMALL_MAX = 4096;

__global__ __launch_bounds__(SMALL_BLOCK) void k_small(
    uint32_t m, ReqArgs in, const CfgDev* __restrict__ cfgs, uint32_t ncfg, TbEntry* tb, uint64_t tb_mask,
    WinEntry* win, uint64_t win_mask, Spill spill, uint32_t win_base, uint32_t invalid_key, int32_t profile,
    ReqArgs ps, TbPre pre, uint32_t heavy_min, uint32_t* eflags) {
    __shared__ uint64_t sk[SMALL_MAX];   // (slot << 32) | arrival index
    __shared__ uint64_t heavy[SMALL_MAX / 32];   // (end << 32) | start of each long segment
    __shared__ uint32_t nheavy;
    if (threadIdx.x == 0) nheavy = 0;
    uint32_t P = 64;
    while (P < m) P <<= 1;
    uint32_t ef = 0;
    for (uint32_t i = threadIdx.x; i < P; i += SMALL_BLOCK) {
        uint64_t v = ~0ull;
        if (i < m) {
            const uint32_t slot = probe_request(in.key[i], in.cfg[i], in.n[i], cfgs, ncfg, tb, tb_mask, win,
                                                win_mask, win_base, invalid_key, ef);
            v = ((uint64_t)slot << 32) | i;
        }
        sk[i] = v;
    }
    __syncthreads();
    // bitonic sort, ascending: the keys are unique (the index is in the low bits)
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < P; i += SMALL_BLOCK) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = sk[i], b = sk[l];
                    if ((a > b) == ((i & k) == 0)) { sk[i] = b; sk[l] = a; }
                }
            }
            __syncthreads();
        }
    }
    // sorted-order copy + token-bucket precomputation (k_permute)
    for (uint32_t j = threadIdx.x; j < m; j += SMALL_BLOCK) {
        const uint32_t k0 = (uint32_t)(sk[j] >> 32);
        if (k0 == invalid_key) continue;
        const uint32_t i = (uint32_t)sk[j];
        const int64_t t = in.ts[i];
        const uint32_t c = in.cfg[i];
        const int64_t sms = in.sms ? in.sms[i] : floor_div(t, 1000000LL);
        const int64_t nv = in.n[i];
        const_cast<int64_t*>(ps.ts)[j] = t;
        const_cast<int64_t*>(ps.n)[j] = nv;
        const_cast<uint32_t*>(ps.cfg)[j] = c;
        if (ps.sms) const_cast<int64_t*>(ps.sms)[j] = sms;
        if (k0 >= win_base) continue;
        const CfgDev& C = cfgs[c];
        const double now = (double)t / 1e9;
        if (j > 0 && (uint32_t)(sk[j - 1] >> 32) == k0) {
            const uint32_t ip = (uint32_t)sk[j - 1];
            const int64_t tp = in.ts[ip];
            const int64_t smsp = in.sms ? in.sms[ip] : floor_div(tp, 1000000LL);
            const double prev_last = lua_tostring_roundtrip((double)tp / 1e9, profile);
            const int64_t prev_when = expire_when(cfgs[in.cfg[ip]].ttl_tb, smsp);
            pre.add[j] = key_alive(prev_when, sms, profile) ? (now - prev_last) * C.rate : __builtin_nan("");
        }
        pre.th[j] = fmin(C.limit_d, (double)nv);
    }
    __syncthreads();
    // segments: short ones replay serially, one thread each (exact fallbacks
    // of the big path); segments of heavy_min or more go to a list that the
    // waves replay cooperatively (wave_segment / wave_win_segment, the big
    // path's per-wave heavy replay)
    for (uint32_t j = threadIdx.x; j < m; j += SMALL_BLOCK) {
        const uint32_t k0 = (uint32_t)(sk[j] >> 32);
        if (k0 == invalid_key || (j > 0 && (uint32_t)(sk[j - 1] >> 32) == k0)) continue;
        // end of the segment: galloping search in LDS
        uint32_t lo = j, step = 1;
        while (lo + step < m && (uint32_t)(sk[lo + step] >> 32) == k0) { lo += step; step <<= 1; }
        uint32_t hi = lo + step < m ? lo + step : m;
        while (hi - lo > 1) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if ((uint32_t)(sk[mid] >> 32) == k0) lo = mid; else hi = mid;
        }
        const uint32_t j1 = lo + 1;
        if (j1 - j >= heavy_min) {
            const uint32_t h = atomicAdd(&nheavy, 1u);
            heavy[h] = ((uint64_t)j1 << 32) | j;
            continue;
        }
        if (k0 < win_base) replay_tb_serial(&tb[k0], j, j1, cfgs, profile, ps, pre);
        else replay_win_serial(&win[k0 - win_base], spill, j, j1, cfgs, profile, ps, eflags);
    }
    __syncthreads();
    {
        const uint32_t nh = nheavy;
        uint32_t iters = 0;
        for (uint32_t h = threadIdx.x >> 6; h < nh; h += SMALL_BLOCK / 64) {
            const uint32_t j0 = (uint32_t)heavy[h], j1 = (uint32_t)(heavy[h] >> 32);
            const uint32_t k0 = (uint32_t)(sk[j0] >> 32);
            if (k0 < win_base) wave_segment(&tb[k0], j0, j1, cfgs, profile, ps, pre, eflags, iters);
            else wave_win_segment(&win[k0 - win_base], spill, j0, j1, cfgs, profile, ps, eflags);
        }
    }
    __syncthreads();
    // results to the caller's order (k_unpermute)
    for (uint32_t j = threadIdx.x; j < m; j += SMALL_BLOCK) {
        const uint32_t k0 = (uint32_t)(sk[j] >> 32);
        const uint32_t i = (uint32_t)sk[j];
        if (k0 == invalid_key) {
            in.dec[i] = DEC_INVALID;
            in.rem[i] = 0;
            in.retry[i] = 0;
            in.reset[i] = 0;
            if (in.tok) in.tok[i] = 0.0;
            continue;
        }
        const uint8_t dec = ps.dec[j];
        int64_t rem, retry, reset;
        double tok;
        finish_result(dec, ps.tok[j], ps.ts[j], ps.n[j], cfgs[ps.cfg[j]], rem, retry, reset, tok);
        in.dec[i] = dec;
        in.rem[i] = rem;
        in.retry[i] = retry;
        in.reset[i] = reset;
        if (in.tok) in.tok[i] = tok;
    }
    if (ef) atomicOr(eflags, ef);
}

// Reset: DEL of the key(s) AllowN would touch at ts (tokenbucket.go:136-144,
// slidingwindow.go:125-139, fixedwindow.go:118-128)
__global__ void k_reset(uint64_t key, int64_t ts, const CfgDev* cfgs, uint32_t cfg, TbEntry* tb,
                        uint64_t tb_mask, WinEntry* win, uint64_t win_mask, Spill spill) {
    const CfgDev& c = cfgs[cfg];
    if (c.alg == ALG_TOKEN_BUCKET) {
        uint32_t s = probe_find(tb, tb_mask, key);
        if (s != NO_SLOT) tb[s].when = ABSENT;
        return;
    }
    uint32_t s = probe_find(win, win_mask, key);
    if (s == NO_SLOT) return;
    const int64_t ws = window_start(ts, c);
    wk_delete(&win[s], spill, ws);
    if (c.alg == ALG_SLIDING_WINDOW) wk_delete(&win[s], spill, ws - c.ttl_c);
}

// Redis KEYS (rl_table_keys): every live key of the three tables
__device__ inline void key_emit(rl_key_rec* out, uint64_t cap, unsigned long long* cnt, uint64_t k, int64_t ws,
                                uint32_t kind) {
    const unsigned long long i = atomicAdd(cnt, 1ull);
    if (i < cap) out[i] = rl_key_rec{k, ws, kind, 0};
}
__global__ void k_table_keys(const TbEntry* tb, uint64_t ntb, const WinEntry* win, uint64_t nwin,
                             const SpillEntry* sp, uint64_t nsp, int64_t now_ms, int32_t profile, rl_key_rec* out,
                             uint64_t cap, unsigned long long* cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < ntb + nwin + nsp; i += stride) {
        if (i < ntb) {
            if (entry_live(tb[i], now_ms, profile)) key_emit(out, cap, cnt, tb[i].key, 0, RL_KIND_HASH);
        } else if (i < ntb + nwin) {
            const WinEntry& x = win[i - ntb];
            if (x.key == EMPTY_KEY) continue;
            for (int k = 0; k < 2; k++)
                if (x.s[k].when != ABSENT && key_alive(x.s[k].when, now_ms, profile))
                    key_emit(out, cap, cnt, x.key, x.s[k].ws, RL_KIND_WINDOW);
        } else {
            const SpillEntry& x = sp[i - ntb - nwin];
            if (entry_live(x, now_ms, profile)) key_emit(out, cap, cnt, x.key, x.ws, RL_KIND_WINDOW);
        }
    }
}

// results of a routed batch: one 32-byte result record per request at its
// receive index (the send layout of the result all-to-all)
__global__ __launch_bounds__(256) void k_unpermute_routed(const uint32_t* __restrict__ sk,
                                                          const uint32_t* __restrict__ sv, uint32_t m,
                                                          uint32_t invalid_key, const CfgDev* __restrict__ cfgs,
                                                          ReqArgs sorted, RouteIn ri) {
    m = min(m, *ri.count);
    const bool ident = m && ri.order[0] == RL_ORDER_IDENTITY;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        const uint32_t k0 = sk[j];
        const uint32_t p = sv[j];
        uint8_t dec = DEC_INVALID;   // rejected by k_probe (n <= 0, unknown config or key, table full)
        int64_t rem = 0, retry = 0, reset = 0;
        double tok = 0.0;
        if (k0 != invalid_key) {
            dec = sorted.dec[j];
            finish_result(dec, sorted.tok[j], sorted.ts[j], sorted.n[j], cfgs[sorted.cfg[j]], rem, retry, reset, tok);
        }
        ri.res[ident ? p : ri.order[p]] = rl_route_res{(int64_t)dec, rem, retry, reset};
    }
}

// the same through merge-position buckets (m <= UP_MAX): k_unpermute_bucket
// has placed each request's decision and value in the bucket of its merge
// position p; one block per bucket finishes the Result fields in p order from
// the request's record and writes the result records at p (identity) or
// order[p]
__global__ __launch_bounds__(256) void k_unpermute_routed_out(uint32_t m, const UpRec* __restrict__ bucketed,
                                                              const CfgDev* __restrict__ cfgs, RouteIn ri) {
    __shared__ double s_val[UP_BUCKET];
    __shared__ uint8_t s_dec[UP_BUCKET];
    m = min(m, *ri.count);
    const uint32_t base = blockIdx.x * UP_BUCKET;
    if (base >= m) return;   // block-uniform
    const bool ident = ri.order[0] == RL_ORDER_IDENTITY;
    const uint32_t cnt = min(UP_BUCKET, m - base);
    for (uint32_t k = threadIdx.x; k < cnt; k += 256) {
        const UpRec r = bucketed[(size_t)base + k];
        const uint32_t o = r.i - base;
        s_dec[o] = (uint8_t)r.dec;
        s_val[o] = r.val;
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += 256) {
        const uint32_t p = base + k;
        const uint32_t at = ident ? p : ri.order[p];
        const uint8_t dec = s_dec[k];
        int64_t rem = 0, retry = 0, reset = 0;
        double tok = 0.0;
        if (dec != DEC_INVALID) {
            const rl_route_rec q = ri.rec[at];
            finish_result(dec, s_val[k], q.ts, q.n, cfgs[q.cfg], rem, retry, reset, tok);
        }
        ri.res[at] = rl_route_res{(int64_t)dec, rem, retry, reset};
    }
}

// diagnostic timestamp (10 ns ticks) into *w
__global__ void k_stamp(uint32_t* w) { *w = (uint32_t)__builtin_amdgcn_s_memrealtime(); }

__global__ void k_q14(const double* in, double* out, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rlq::q14(in[i]);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------

namespace {

constexpr int NSTAGES = 5;
constexpr uint32_t STAMP_RING = 256;
constexpr int NSETS = 3;          // batch buffer sets: grouping b+1 | replay b | finish b-1
constexpr uint32_t LIGHT_MIN_BATCH = 1u << 19;   // batches this large may take k_replay_light
constexpr int GROUP_LDS = 4096;   // LDS floor of the grouping / finish kernels (see rl_engine::chain_pad)
// A set's zeroed words.  The head (list counts, queues, diagnostics) is read
// by the host after the batch (rl_engine_stats), so k_probe zeroes it when the
// set is next used; everything after it is zeroed on the finish stream as the
// batch ends (the next use of the set waits for that), so the grouping stream
// carries no memset.
constexpr uint32_t CTRL_NSEG = 0;              // [0..3] list counts (heavy TB, light, heavy window, huge TB)
                                               // [4] chain queue [5] per-thread queue [6] per-wave queue
constexpr uint32_t CTRL_DBG = CTRL_NSEG + 8;   // [0] rounds [1] near/exact iterations [2] max rounds
                                               // [3..6] round ends (full, stop, partial, first window)
                                               // [8..19] timers [20] exact tiles [21] serial steps
constexpr uint32_t CTRL_DBGN = 88;
constexpr uint32_t CTRL_HEAD = CTRL_DBG + CTRL_DBGN;  // words zeroed by k_probe
constexpr uint32_t CTRL_HIST = CTRL_HEAD;             // [4][256]
constexpr uint32_t CTRL_TILE = CTRL_HIST + 4 * RADIX;  // [4] tile counters
constexpr uint32_t CTRL_UPB = CTRL_TILE + 4;          // [UP_NB] bucket fill counters (k_unpermute_bucket)
constexpr uint32_t CTRL_PLAN = CTRL_UPB + UP_NB;      // [0] every MSD bucket fits k_sort_local [1] it does not
constexpr uint32_t CTRL_XRUN = CTRL_PLAN + 2;         // runs of multi-decade chain windows listed (k_tb_expand_x)
constexpr uint32_t CTRL_WORDS = CTRL_XRUN + 1;

// The grouping sort's digits.  One pass: bits [0, 8).  More: the MSD pass
// first, the top 8 bits [B - 8, B) of the B-bit slot ids, then either one
// k_sort_local over the buckets (each sorted in LDS by the bits below B - 8)
// or, when a bucket is too large for it (a hot key), the LSD passes at
// 0, 8, ... over bits [0, B - 8).  Every pass is stable and the digits cover
// every bit, so either way equal slots end up contiguous in arrival order.
static uint32_t sort_shifts(int bits, int passes) {
    if (passes <= 1) return 0u;
    uint32_t sh = (uint32_t)(bits - 8);
    for (int p = 1; p < passes; p++) sh |= (uint32_t)(8 * (p - 1)) << (8 * p);
    return sh;
}

uint64_t pow2_at_least(uint64_t v) {
    uint64_t p = 1;
    while (p < v) p <<= 1;
    return p;
}
int bitlen(uint64_t v) {
    int b = 0;
    while (v) { b++; v >>= 1; }
    return b;
}

}  // namespace

// Per-batch device buffers.  A batch runs in three parts on three engine
// streams: grouping (probe, sort, segments, permute) on `front`, the replay
// (k_tb_chain) on `chain`, the finish (run expansion, unpermute) on `tail`.
// The replays are ordered on `chain` (each one reads the table state the
// previous one wrote); nothing else orders batches, so batch b+1's grouping
// and batch b-1's finish overlap batch b's replay.  NSETS buffer sets: set
// b mod NSETS is reused by batch b+NSETS only after batch b's finish.  The
// caller's stream waits for the finish of every batch it enqueued.
struct BatchSet {
    uint32_t *sk0 = nullptr, *sk1 = nullptr, *sv0 = nullptr, *sv1 = nullptr;
    SegRec* list[4] = {nullptr, nullptr, nullptr, nullptr};   // heavy TB, light, heavy window, huge TB
    // requests and results in sorted order (k_permute / k_unpermute)
    int64_t *p_ts = nullptr, *p_n = nullptr, *p_sms = nullptr;
    uint32_t* p_cfg = nullptr;
    void* rec = nullptr;          // requests packed in arrival order (k_probe -> k_permute): ReqRec<XS>
    void* recb = nullptr;         // ReqRec in the MSD pass's bucket order (k_sort_pass -> k_permute)
    // an explicit server clock's record fields that do not fit (rec_pack), by arrival index
    int64_t* side_n = nullptr;
    uint32_t* side_cfg = nullptr;
    int64_t* side_sms = nullptr;
    uint8_t* p_fresh = nullptr;   // sorted order: the request inserted its key (k_permute -> replay phase 3)
    uint8_t* o_dec = nullptr;
    double* o_tok = nullptr;      // tokens (token bucket) / Remaining bits (window): finish_result
    // token-bucket precomputation (k_permute)
    double *q_add = nullptr, *q_th = nullptr;
    TbRuns runs{};                // the chain's committed runs (by start position)
    uint32_t* zero = nullptr;     // ctrl words + look-back status + huge claims (zeroed per batch)
    bool dirty = false;           // a batch began on the set and did not reach its finish's zeroing
    uint32_t* ctrl = nullptr;
    uint32_t* status = nullptr;
    uint32_t* claim = nullptr;
    hipEvent_t front_done = nullptr, chain_done = nullptr, back_done = nullptr;
    uint64_t* kid = nullptr;      // key ids hashed from raw keys (rl_decide_batch_keys_device; lazy)
    UpRec* upb = nullptr;         // results bucketed by arrival index (k_unpermute_bucket)
    bool used = false;
};

struct rl_engine {
    int device = 0;
    int32_t profile = PROFILE_REDIS7;
    uint32_t flags = 0;
    // the engine's stream (host API, device API without a stream, setup) is
    // `tail`: with the caller's stream the engine then uses four streams, one
    // hardware queue each at HIP's default of four queues per process (streams
    // sharing a queue would serialize the replay and the finish)
    hipStream_t stream = nullptr;
    hipStream_t front = nullptr;      // grouping
    hipStream_t chain = nullptr;      // replays, in batch order
    hipStream_t tail = nullptr;       // finishes
    hipEvent_t ev_in = nullptr;       // inputs ready (non-pipelined device API, host API)
    std::string err;

    std::vector<CfgDev> h_cfg;
    CfgDev* d_cfg = nullptr;
    uint32_t cfg_cap = 0;

    TbEntry* d_tb = nullptr;
    uint64_t tb_cap = 0;
    WinEntry* d_win = nullptr;
    uint64_t win_cap = 0;
    SpillEntry* d_spill = nullptr;    // window keys outside their user key's entry (rl_window.h)
    uint64_t spill_cap = 0;
    bool spill_follows = true;        // spill capacity = 2 x window capacity (also after a resize)
    Spill spill() const { return Spill{d_spill, spill_cap - 1}; }
    uint32_t win_base = 0, invalid_key = 0;
    int sort_bits = 0, sort_passes = 0;
    uint32_t sort_shifts = 0;   // digit shift of each histogram / pass (8 bits each; sort_shifts())

    uint32_t max_batch = 0;
    uint32_t max_tiles = 0;
    BatchSet set[NSETS];
    // k_small: batches up to small_max run as one workgroup on `chain`; its
    // sorted-order scratch (reused by consecutive small batches, which the
    // chain stream orders)
    uint32_t small_max = 0;
    int64_t *s_ts = nullptr, *s_n = nullptr, *s_sms = nullptr;
    uint32_t* s_cfg = nullptr;
    uint8_t* s_dec = nullptr;
    double *s_tok = nullptr, *s_add = nullptr, *s_th = nullptr;
    hipEvent_t ev_small = nullptr;
    hipEvent_t ev_reset = nullptr;    // rl_reset_device: the DEL on `chain` -> the caller's stream
    int next_set = 0, last_set = 0;   // set of the next / the last enqueued batch
    size_t zero_bytes = 0;
    int coop_grid = 128;        // k_tb_chain blocks launched (one per CU fits its LDS) ...
    int coop_base = 112;        // ... of which those past 112 of 256 CUs exit at once unless the batch
                                // has at least m / coop_light_div light segments: the other CUs run
                                // the neighbouring batches' grouping and finish (profiles/r3al_ab_replay_grid.txt;
                                // 96 -> 112 with the iterative-ILP build: configs[1] +1.1-1.5 %,
                                // profiles/r6zm_ab_coop_base.txt)
    uint32_t coop_light_div = 4;
    int probe_grid = 1024;      // k_probe blocks at most
    int perm_grid = 1024;       // k_permute / k_unpermute blocks at most
    uint32_t heavy_min = 32;    // segments this long replay cooperatively
    uint32_t huge_min = 4096;   // token-bucket segments this long are dequeued first
    // dynamic LDS that makes a k_tb_chain block fill its CU's LDS: with two
    // batches in flight, the other batches' grouping and finish kernels (each launched with
    // GROUP_LDS bytes at least) then never share a CU with a chain
    size_t chain_pad[2] = {0, 0};
    size_t light_pad[2] = {0, 0};    // k_replay_light: the same one-block-per-CU LDS floor
    uint32_t* h_huge = nullptr;      // mapped host word: huge segments of the last replay seen (k_tb_chain /
    uint32_t* d_huge = nullptr;      //   k_replay_light write it); 0 -> the next batches launch k_replay_light
    bool light_ok = true;            // RL_NO_LIGHT_REPLAY=1: always the chain kernel
    bool force_light = false;        // warm-up: load k_replay_light
    uint32_t* d_eflags = nullptr;
    uint32_t* d_zero = nullptr;       // a device word holding 0 (warm-up of the routed kernels)
    unsigned long long* d_count = nullptr;   // table counts / GC counters (rl_table_info_get, rl_table_gc)
    unsigned long long* h_count = nullptr;   // pinned host copy
    // the grouping sort's last plan (1: every MSD bucket fit LDS), written by
    // the MSD pass into mapped host memory; read when a batch is enqueued
    uint32_t* h_plan = nullptr;
    uint32_t* d_plan = nullptr;   // its device address
    uint32_t* stamp_ring = nullptr;   // RL_STAMP_KERNELS diagnostics

    // host-API staging (device side)
    uint64_t* d_key = nullptr;
    uint64_t* small_kid = nullptr;   // key ids hashed for k_small (rl_decide_batch_keys_device; lazy)
    int64_t *d_ts = nullptr, *d_n = nullptr, *d_sms = nullptr;
    uint32_t* d_cfgid = nullptr;
    uint8_t* d_dec = nullptr;
    int64_t *d_rem = nullptr, *d_retry = nullptr, *d_reset = nullptr;
    double* d_tok = nullptr;

    // timing: front start, after probe, after sort, after segments+permute
    // (front); replay start, end (chain); finish start, end (tail)
    bool timing = false;
    bool timing_all = false;    // level 2: every stage; level 1: the replay only (2 events per batch)
    uint32_t timing_stride = 1; // the replay events on every timing_stride-th batch only (level -k)
    uint64_t timing_seq = 0;
    bool stamps = false;        // RL_STAMP_KERNELS: timestamps around each replay (debug words 18, 19)
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::array<hipEvent_t, 8>> ev_pending;
    double stage_ms[NSTAGES] = {0, 0, 0, 0, 0};
    uint64_t timed_batches = 0;

    rl_stats stats{};
};

static int fail(rl_engine* e, int code, const std::string& msg) {
    if (e) e->err = msg;
    return code;
}

#define HIPCHK(e, call)                                                                  \
    do {                                                                                 \
        hipError_t _st = (call);                                                         \
        if (_st != hipSuccess)                                                           \
            return fail((e), RL_EDEVICE, std::string(#call) + ": " + hipGetErrorString(_st)); \
    } while (0)

// versioned output structs (include/rl_engine.h): the caller's struct_size
// bounds what is written, and struct_size comes back as the bytes actually
// filled in (min(caller's, library's)), so a caller built against a newer
// header sees which trailing fields this library knows; a size smaller than
// the header field is rejected
template <class T>
static int copy_out(T* dst, T src) {
    if (dst->struct_size < 8) return RL_EINVAL;
    const uint32_t n = (uint32_t)std::min<size_t>(dst->struct_size, sizeof(T));
    src.struct_size = n;
    memcpy(dst, &src, n);
    return RL_OK;
}

static void free_set(BatchSet& B) {
    (void)hipFree(B.sk0); (void)hipFree(B.sk1); (void)hipFree(B.sv0); (void)hipFree(B.sv1);
    for (auto* l : B.list) (void)hipFree(l);
    (void)hipFree(B.p_ts); (void)hipFree(B.p_n); (void)hipFree(B.p_sms); (void)hipFree(B.p_cfg);
    (void)hipFree(B.rec);
    (void)hipFree(B.recb);
    (void)hipFree(B.side_n); (void)hipFree(B.side_cfg); (void)hipFree(B.side_sms);
    (void)hipFree(B.p_fresh);
    (void)hipFree(B.o_dec);
    (void)hipFree(B.o_tok);
    (void)hipFree(B.q_add); (void)hipFree(B.q_th);
    (void)hipFree(B.runs.len); (void)hipFree(B.runs.E); (void)hipFree(B.runs.D0); (void)hipFree(B.runs.D1);
    (void)hipFree(B.runs.xlist);
    (void)hipFree(B.zero);
    (void)hipFree(B.kid);
    (void)hipFree(B.upb);
    if (B.front_done) (void)hipEventDestroy(B.front_done);
    if (B.back_done) (void)hipEventDestroy(B.back_done);
    if (B.chain_done) (void)hipEventDestroy(B.chain_done);
}

static bool alloc_set(BatchSet& B, size_t M, size_t zero_bytes, size_t status_words) {
    bool ok = true;
    ok &= hipMalloc(&B.sk0, 4 * M) == hipSuccess;
    ok &= hipMalloc(&B.sk1, 4 * M) == hipSuccess;
    ok &= hipMalloc(&B.sv0, 4 * M) == hipSuccess;
    ok &= hipMalloc(&B.sv1, 4 * M) == hipSuccess;
    ok &= hipMalloc(&B.list[0], sizeof(SegRec) * M) == hipSuccess;
    ok &= hipMalloc(&B.list[1], sizeof(SegRec) * M) == hipSuccess;
    ok &= hipMalloc(&B.list[2], sizeof(SegRec) * M) == hipSuccess;
    ok &= hipMalloc(&B.list[3], sizeof(SegRec) * (M / 4096 + 1)) == hipSuccess;
    ok &= hipMalloc(&B.p_ts, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.p_n, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.p_sms, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.p_cfg, 4 * M) == hipSuccess;
    ok &= hipMalloc(&B.rec, sizeof(ReqRec<false>) * M) == hipSuccess;
    ok &= hipMalloc(&B.side_n, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.side_cfg, 4 * M) == hipSuccess;
    ok &= hipMalloc(&B.side_sms, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.recb, sizeof(ReqRec<false>) * M) == hipSuccess;
    ok &= hipMalloc(&B.p_fresh, M) == hipSuccess;
    ok &= hipMalloc(&B.o_dec, M) == hipSuccess;
    ok &= hipMalloc(&B.o_tok, 8 * M) == hipSuccess;
    // q_add and q_th carry 128 elements of slack: the chain's loader wave
    // reads them in aligned 128-element chunks that may end past the batch
    ok &= hipMalloc(&B.q_add, 8 * (M + 128)) == hipSuccess;
    ok &= hipMalloc(&B.q_th, 8 * (M + 128)) == hipSuccess;
    ok &= hipMalloc(&B.runs.len, 2 * M) == hipSuccess;
    ok &= hipMalloc(&B.runs.E, 2 * M) == hipSuccess;
    ok &= hipMalloc(&B.runs.D0, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.runs.D1, 8 * M) == hipSuccess;
    ok &= hipMalloc(&B.runs.xlist, 4 * M) == hipSuccess;   // a run per start position at most
    ok &= hipMalloc(&B.zero, zero_bytes) == hipSuccess;
    ok &= hipMalloc(&B.upb, sizeof(UpRec) * std::min<size_t>(M, UP_MAX)) == hipSuccess;
    // front_done / chain_done only order the engine's own streams on this
    // device: a device-scope release (no system-scope cache writeback per
    // batch); back_done hands results to the caller and keeps the default
    const unsigned inner = hipEventDisableTiming | hipEventReleaseToDevice;
    ok &= hipEventCreateWithFlags(&B.front_done, inner) == hipSuccess;
    ok &= hipEventCreateWithFlags(&B.back_done, hipEventDisableTiming) == hipSuccess;
    ok &= hipEventCreateWithFlags(&B.chain_done, inner) == hipSuccess;
    if (!ok) return false;
    B.ctrl = B.zero;
    B.status = B.zero + CTRL_WORDS;
    B.runs.xcnt = B.ctrl + CTRL_XRUN;
    B.claim = B.status + status_words;
    // run lengths start at 0; k_tb_expand clears every one it consumes
    return hipMemset(B.runs.len, 0, 2 * M) == hipSuccess && hipMemset(B.zero, 0, zero_bytes) == hipSuccess;
}

static void free_all(rl_engine* e) {
    (void)hipFree(e->d_cfg);
    (void)hipFree(e->d_tb);
    (void)hipFree(e->d_win);
    (void)hipFree(e->d_spill);
    for (auto& B : e->set) free_set(B);
    (void)hipFree(e->d_eflags);
    (void)hipFree(e->d_zero);
    (void)hipFree(e->d_count);
    if (e->h_count) (void)hipHostFree(e->h_count);
    if (e->h_plan) (void)hipHostFree(e->h_plan);
    if (e->h_huge) (void)hipHostFree(e->h_huge);
    (void)hipFree(e->stamp_ring);
    (void)hipFree(e->small_kid);
    (void)hipFree(e->d_key); (void)hipFree(e->d_ts); (void)hipFree(e->d_n); (void)hipFree(e->d_sms); (void)hipFree(e->d_cfgid);
    (void)hipFree(e->d_dec); (void)hipFree(e->d_rem); (void)hipFree(e->d_retry); (void)hipFree(e->d_reset); (void)hipFree(e->d_tok);
    for (auto ev : e->ev_pool) (void)hipEventDestroy(ev);
    if (e->ev_in) (void)hipEventDestroy(e->ev_in);
    if (e->ev_small) (void)hipEventDestroy(e->ev_small);
    if (e->ev_reset) (void)hipEventDestroy(e->ev_reset);
    for (void* p : {(void*)e->s_ts, (void*)e->s_n, (void*)e->s_sms, (void*)e->s_cfg, (void*)e->s_dec, (void*)e->s_tok,
                    (void*)e->s_add, (void*)e->s_th})
        (void)hipFree(p);
    if (e->front) (void)hipStreamDestroy(e->front);
    if (e->chain) (void)hipStreamDestroy(e->chain);
    if (e->tail) (void)hipStreamDestroy(e->tail);
}

// every queued kernel of the engine has finished (the engine's streams and,
// through the back_done events, any caller stream a batch was enqueued on)
static int drain(rl_engine* e) {
    HIPCHK(e, hipStreamSynchronize(e->front));
    HIPCHK(e, hipStreamSynchronize(e->chain));
    HIPCHK(e, hipStreamSynchronize(e->tail));
    for (auto& B : e->set)
        if (B.used) HIPCHK(e, hipEventSynchronize(B.back_done));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return RL_OK;
}

static int warm_up(rl_engine* e);

extern "C" int rl_engine_create(const rl_opts* o, rl_engine** out) {
    if (!o || !out) return RL_EINVAL;
    *out = nullptr;
    if (o->struct_size != sizeof(rl_opts)) return RL_EINVAL;
    if (o->profile != PROFILE_REDIS7 && o->profile != PROFILE_MINIREDIS) return RL_EINVAL;
    if (o->max_batch == 0 || o->max_batch > (1u << 28)) return RL_EINVAL;
    if (o->flags & ~(uint32_t)RL_OPT_PIPELINE) return RL_EINVAL;
    rl_engine* e = new rl_engine();
    e->device = o->device;
    e->profile = o->profile;
    e->flags = o->flags;
    e->tb_cap = pow2_at_least(std::max<uint64_t>(o->tb_capacity, 1024));
    e->win_cap = pow2_at_least(std::max<uint64_t>(o->win_capacity, 1024));
    if (e->tb_cap + e->win_cap >= (1ull << 31)) { delete e; return RL_EINVAL; }
    e->spill_follows = o->spill_capacity == 0;
    e->spill_cap = pow2_at_least(std::max<uint64_t>(o->spill_capacity ? o->spill_capacity : 2 * e->win_cap, 1024));
    if (e->spill_cap > (1ull << 34)) { delete e; return RL_EINVAL; }
    e->win_base = (uint32_t)e->tb_cap;
    e->invalid_key = (uint32_t)(e->tb_cap + e->win_cap);
    e->sort_bits = bitlen(e->invalid_key);
    e->sort_passes = (e->sort_bits + 7) / 8;
    e->sort_shifts = sort_shifts(e->sort_bits, e->sort_passes);
    e->max_batch = o->max_batch;
    e->max_tiles = (o->max_batch + SORT_TILE - 1) / SORT_TILE;

    auto bail = [&](int code) { int r = code; free_all(e); delete e; return r; };
    if (hipSetDevice(e->device) != hipSuccess) return bail(RL_EDEVICE);
    {
        // grouping and finish kernels never use the reserved CUs (one per 8):
        // when a replay is launched those are free, so its first blocks -- the
        // longest segments -- start at once instead of waiting for a CU that
        // the other two streams' blocks have left empty
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, e->device) != hipSuccess) return bail(RL_EDEVICE);
        const int ncu = prop.multiProcessorCount;
        int every = 8;    // one reserved CU per `every` (0: none); one per 32 (round 2) held the
                          // grouping of the uniform workloads back: profiles/r3aq_ab_reserved_cus.txt
        if (const char* v = getenv("RL_RESERVE_EVERY")) every = atoi(v);
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int c = 0; c < ncu; c++)
            if (every <= 0 || c % every != every - 1 || ncu < 64) mask[c / 32] |= 1u << (c % 32);
        if (hipExtStreamCreateWithCUMask(&e->front, (uint32_t)mask.size(), mask.data()) != hipSuccess ||
            hipExtStreamCreateWithCUMask(&e->tail, (uint32_t)mask.size(), mask.data()) != hipSuccess)
            return bail(RL_EDEVICE);
    }
    {
        // the replay is the critical path: its blocks are dispatched first
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
        if (hipStreamCreateWithPriority(&e->chain, hipStreamNonBlocking, hi) != hipSuccess) return bail(RL_EDEVICE);
    }
    e->stream = e->tail;
    if (hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming) != hipSuccess) return bail(RL_EDEVICE);
    if (hipEventCreateWithFlags(&e->ev_small, hipEventDisableTiming) != hipSuccess) return bail(RL_EDEVICE);
    if (hipEventCreateWithFlags(&e->ev_reset, hipEventDisableTiming) != hipSuccess) return bail(RL_EDEVICE);
    e->small_max = SMALL_MAX;
    if (const char* v = getenv("RL_SMALL_MAX")) e->small_max = std::min<uint32_t>((uint32_t)atoi(v), SMALL_MAX);
    size_t M = e->max_batch;
    e->cfg_cap = 64;
    const size_t status_words = (size_t)4 * e->max_tiles * RADIX;
    e->zero_bytes = 4 * (CTRL_WORDS + status_words + M / 4096 + 1);
    bool ok = true;
    ok &= hipMalloc(&e->d_cfg, sizeof(CfgDev) * e->cfg_cap) == hipSuccess;
    ok &= hipMalloc(&e->d_tb, sizeof(TbEntry) * e->tb_cap) == hipSuccess;
    ok &= hipMalloc(&e->d_win, sizeof(WinEntry) * e->win_cap) == hipSuccess;
    ok &= hipMalloc(&e->d_spill, sizeof(SpillEntry) * e->spill_cap) == hipSuccess;
    for (auto& B : e->set) ok = ok && alloc_set(B, M, e->zero_bytes, status_words);
    ok &= hipMalloc(&e->d_eflags, 4) == hipSuccess;
    ok &= hipMalloc(&e->d_zero, 4) == hipSuccess && hipMemset(e->d_zero, 0, 4) == hipSuccess;
    ok &= hipMalloc(&e->d_count, 8 * sizeof(unsigned long long)) == hipSuccess;
    ok &= hipHostMalloc(&e->h_count, 8 * sizeof(unsigned long long), hipHostMallocDefault) == hipSuccess;
    ok &= hipHostMalloc(&e->h_plan, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
    if (ok) {
        *(volatile uint32_t*)e->h_plan = 0u;   // first batches: no prediction (the LSD passes are launched)
        ok &= hipHostGetDevicePointer((void**)&e->d_plan, e->h_plan, 0) == hipSuccess;
    ok &= hipHostMalloc(&e->h_huge, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
    if (ok) {
        *(volatile uint32_t*)e->h_huge = 1u;   // first batches: the chain kernel
        ok &= hipHostGetDevicePointer((void**)&e->d_huge, e->h_huge, 0) == hipSuccess;
    }
    }
    ok &= hipMalloc(&e->d_key, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_ts, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_n, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_sms, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_cfgid, 4 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_dec, M) == hipSuccess;
    ok &= hipMalloc(&e->d_rem, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_retry, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_reset, 8 * M) == hipSuccess;
    ok &= hipMalloc(&e->d_tok, 8 * M) == hipSuccess;
    for (int64_t** p : {&e->s_ts, &e->s_n, &e->s_sms})
        ok &= hipMalloc(p, 8 * SMALL_MAX) == hipSuccess;
    // add / th: 128 elements of slack, as the batch sets' (exact_span reads ahead)
    for (double** p : {&e->s_tok, &e->s_add, &e->s_th}) ok &= hipMalloc(p, 8 * (SMALL_MAX + 128)) == hipSuccess;
    ok &= hipMalloc(&e->s_cfg, 4 * SMALL_MAX) == hipSuccess;
    ok &= hipMalloc(&e->s_dec, SMALL_MAX) == hipSuccess;
    if (!ok) return bail(RL_ENOMEM);
    k_init_tb<<<2048, 256, 0, e->stream>>>(e->d_tb, e->tb_cap);
    k_init_win<<<2048, 256, 0, e->stream>>>(e->d_win, e->win_cap);
    k_init_spill<<<2048, 256, 0, e->stream>>>(e->d_spill, e->spill_cap);
    if (hipMemsetAsync(e->d_eflags, 0, 4, e->stream) != hipSuccess) return bail(RL_EDEVICE);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return bail(RL_EDEVICE);
    if (hipDeviceSynchronize() != hipSuccess) return bail(RL_EDEVICE);
    if (const char* v = getenv("RL_HEAVY_MIN")) e->heavy_min = (uint32_t)atoi(v);
    if (const char* v = getenv("RL_HUGE_MIN")) e->huge_min = (uint32_t)atoi(v);
    if (const char* v = getenv("RL_COOP_GRID")) e->coop_grid = atoi(v);
    if (const char* v = getenv("RL_COOP_BASE")) e->coop_base = atoi(v);
    if (const char* v = getenv("RL_COOP_LIGHT_DIV")) e->coop_light_div = (uint32_t)std::max(1, atoi(v));
    if (const char* v = getenv("RL_PROBE_GRID")) e->probe_grid = atoi(v);
    if (const char* v = getenv("RL_PERM_GRID")) e->perm_grid = atoi(v);
    e->stamps = getenv("RL_STAMP_KERNELS") != nullptr;
    if (e->stamps) {
        if (hipMalloc(&e->stamp_ring, 4 * 6 * STAMP_RING) != hipSuccess) return bail(RL_ENOMEM);
        if (hipMemset(e->stamp_ring, 0, 4 * 6 * STAMP_RING) != hipSuccess) return bail(RL_EDEVICE);
    }
    {
        int dev_lds = 0;
        (void)hipDeviceGetAttribute(&dev_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, e->device);
        hipFuncAttributes fa[2];
        if (hipFuncGetAttributes(&fa[0], reinterpret_cast<const void*>(&k_tb_chain<true>)) != hipSuccess ||
            hipFuncGetAttributes(&fa[1], reinterpret_cast<const void*>(&k_tb_chain<false>)) != hipSuccess)
            return bail(RL_EDEVICE);
        for (int k = 0; k < 2; k++)
            if (dev_lds > (int)fa[k].sharedSizeBytes + GROUP_LDS)
                e->chain_pad[k] = (size_t)dev_lds - fa[k].sharedSizeBytes - GROUP_LDS + 256;
        hipFuncAttributes fl[2];
        if (hipFuncGetAttributes(&fl[0], reinterpret_cast<const void*>(&k_replay_light<true>)) != hipSuccess ||
            hipFuncGetAttributes(&fl[1], reinterpret_cast<const void*>(&k_replay_light<false>)) != hipSuccess)
            return bail(RL_EDEVICE);
        for (int k = 0; k < 2; k++)
            if (dev_lds > (int)fl[k].sharedSizeBytes + GROUP_LDS)
                e->light_pad[k] = (size_t)dev_lds - fl[k].sharedSizeBytes - GROUP_LDS + 256;
        // the dynamic LDS that keeps one replay block per CU exceeds the
        // default per-kernel limit: raise it for the light kernel
        for (int k = 0; k < 2; k++) {
            const void* f = k ? reinterpret_cast<const void*>(&k_replay_light<false>)
                              : reinterpret_cast<const void*>(&k_replay_light<true>);
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->light_pad[k]) != hipSuccess)
                e->light_pad[k] = 0;
        }
    }
    if (getenv("RL_NO_LIGHT_REPLAY")) e->light_ok = false;
    e->stats.sort_bits = e->sort_bits;
    e->stats.sort_passes = e->sort_passes;
    {
        const int r = warm_up(e);
        if (r != RL_OK) return bail(r);
    }
    *out = e;
    return RL_OK;
}

extern "C" int rl_engine_destroy(rl_engine* e) {
    if (!e) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    (void)drain(e);
    free_all(e);
    delete e;
    return RL_OK;
}

extern "C" int rl_config_register(rl_engine* e, uint8_t alg, int64_t limit, int64_t window_ns,
                                  uint32_t* cfg_id) {
    if (!e || !cfg_id) return RL_EINVAL;
    // Validate (config.go:16-50)
    if (alg < RL_ALG_TOKEN_BUCKET || alg > RL_ALG_FIXED_WINDOW) return fail(e, RL_EINVAL, "unknown algorithm");
    if (limit <= 0) return fail(e, RL_EINVAL, "limit must be greater than 0");
    if (window_ns <= 0) return fail(e, RL_EINVAL, "window must be greater than 0");
    if (window_ns < 1000000LL) return fail(e, RL_EINVAL, "window too small");
    if (window_ns > 365LL * 24 * 3600 * NS_PER_S) return fail(e, RL_EINVAL, "window too large");
    CfgDev c = make_cfg(alg, limit, window_ns);
    (void)hipSetDevice(e->device);
    int r = drain(e);                  // queued batches read d_cfg
    if (r != RL_OK) return r;
    if (e->h_cfg.size() == e->cfg_cap) {
        CfgDev* nd = nullptr;
        HIPCHK(e, hipMalloc(&nd, sizeof(CfgDev) * e->cfg_cap * 2));
        HIPCHK(e, hipMemcpyAsync(nd, e->d_cfg, sizeof(CfgDev) * e->cfg_cap, hipMemcpyDeviceToDevice, e->stream));
        HIPCHK(e, hipStreamSynchronize(e->stream));
        (void)hipFree(e->d_cfg);
        e->d_cfg = nd;
        e->cfg_cap *= 2;
    }
    e->h_cfg.push_back(c);
    uint32_t id = (uint32_t)(e->h_cfg.size() - 1);
    HIPCHK(e, hipMemcpyAsync(e->d_cfg + id, &e->h_cfg[id], sizeof(CfgDev), hipMemcpyHostToDevice, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    *cfg_id = id;
    return RL_OK;
}

extern "C" int rl_config_table(rl_engine* e, uint32_t cfg_id) {
    if (!e || cfg_id >= e->h_cfg.size()) return RL_EINVAL;
    return e->h_cfg[cfg_id].alg == ALG_TOKEN_BUCKET ? 0 : 1;
}

static hipEvent_t take_event(rl_engine* e) {
    if (!e->ev_pool.empty()) {
        hipEvent_t ev = e->ev_pool.back();
        e->ev_pool.pop_back();
        return ev;
    }
    // timestamps only: a device-scope release
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventReleaseToDevice);
    return ev;
}

// raw keys of one chunk (rl_decide_batch_keys_device): hashed into key ids on
// the stream that runs the chunk's grouping, ahead of k_probe / k_small
struct KeyBytes {
    const uint8_t* bytes;
    uint64_t nbytes;
    const uint64_t* offsets;      // this chunk's m + 1 offsets (absolute into bytes)
    uint64_t seed;
    const char* prefix;
    size_t prefix_len;
    double mean_len;              // the whole batch's mean key length (group size choice)
};

// rl_keyhash.hip
int rl_hash_keys_launch(size_t m, const uint8_t* bytes, uint64_t nbytes, const uint64_t* offsets, uint64_t seed,
                        const uint32_t* cfg, const char* prefix, size_t prefix_len, double mean_len,
                        uint64_t* key_id, void* stream);

// enqueue one batch of m <= max_batch requests (see BatchSet); s waits for
// its finish.  inputs_ready: the caller guarantees the input arrays are
// complete now (RL_OPT_PIPELINE); otherwise the grouping waits for s.
static int run_small(rl_engine* e, uint32_t m, ReqArgs a, hipStream_t s, bool inputs_ready, const KeyBytes* kb) {
    hipStream_t c = e->chain;   // after every earlier replay (table state)
    if (!inputs_ready) {
        HIPCHK(e, hipEventRecord(e->ev_in, s));
        HIPCHK(e, hipStreamWaitEvent(c, e->ev_in, 0));
    }
    if (kb) {   // own buffer, ordered on c: written by the hash, read by k_small
        if (!e->small_kid && hipMalloc(&e->small_kid, 8 * (size_t)e->small_max) != hipSuccess) return RL_ENOMEM;
        int r = rl_hash_keys_launch(m, kb->bytes, kb->nbytes, kb->offsets, kb->seed, a.cfg, kb->prefix,
                                    kb->prefix_len, kb->mean_len, e->small_kid, c);
        if (r != RL_OK) return r;
        a.key = e->small_kid;
    }
    // sorted-order scratch; the server clock only when the caller gave one
    ReqArgs ps{nullptr, e->s_ts, e->s_n, e->s_cfg, a.sms ? e->s_sms : nullptr, e->s_dec, nullptr, nullptr,
               nullptr, e->s_tok};
    TbPre pre{e->s_add, e->s_th};
    k_small<<<1, SMALL_BLOCK, 0, c>>>(m, a, e->d_cfg, (uint32_t)e->h_cfg.size(), e->d_tb, e->tb_cap - 1, e->d_win,
                                      e->win_cap - 1, e->spill(), e->win_base, e->invalid_key, e->profile, ps, pre,
                                      std::max<uint32_t>(e->heavy_min, 32), e->d_eflags);
    HIPCHK(e, hipEventRecord(e->ev_small, c));
    HIPCHK(e, hipStreamWaitEvent(s, e->ev_small, 0));
    HIPCHK(e, hipGetLastError());
    e->stats.batches++;
    e->stats.decisions += m;
    return RL_OK;
}

// ri (nullable): a routed batch (RouteIn), at most m requests, its size in
// device memory; its inputs come from `s` (the merge)
// s_out (nullable): the stream that waits for the results, when not s
static int run_batch(rl_engine* e, uint32_t m, ReqArgs a, hipStream_t s, bool inputs_ready,
                     const KeyBytes* kb = nullptr, const RouteIn* ri = nullptr, hipStream_t s_out = nullptr,
                     hipEvent_t done_ev = nullptr) {
    if (m == 0) return RL_OK;
    if (m <= e->small_max && !e->timing && !ri) return run_small(e, m, a, s, inputs_ready, kb);
    const uint32_t* mdev = ri ? ri->count : nullptr;
    BatchSet& B = e->set[e->next_set];
    e->last_set = e->next_set;
    e->next_set = (e->next_set + 1) % NSETS;
    hipStream_t f = e->front;
    if (!inputs_ready) {
        HIPCHK(e, hipEventRecord(e->ev_in, s));
        HIPCHK(e, hipStreamWaitEvent(f, e->ev_in, 0));
    }
    if (B.used) HIPCHK(e, hipStreamWaitEvent(f, B.back_done, 0));   // set reuse
    if (kb) {
        if (!B.kid && hipMalloc(&B.kid, 8 * (size_t)e->max_batch) != hipSuccess) return RL_ENOMEM;
        int r = rl_hash_keys_launch(m, kb->bytes, kb->nbytes, kb->offsets, kb->seed, a.cfg, kb->prefix,
                                    kb->prefix_len, kb->mean_len, B.kid, f);
        if (r != RL_OK) return r;
        a.key = B.kid;
    }
    std::array<hipEvent_t, 8> ev{};
    // this batch carries timing events (every timing_stride-th batch: each
    // event pair on the replay's dispatch costs the chain stream ~10 us)
    const bool timed = e->timing && (e->timing_stride <= 1 || e->timing_seq++ % e->timing_stride == 0);
    const bool tall = timed && e->timing_all;   // stage events on every stream
    if (timed) {
        for (int k = 0; k < 8; k++)
            if (tall || k == 4 || k == 5) ev[k] = take_event(e);
        if (tall) (void)hipEventRecord(ev[0], f);
    }
    // diagnostic stamp ring (RL_STAMP_KERNELS): per batch the realtime of
    // front start / end, replay start / end, finish start / end
    uint32_t* sr = e->stamp_ring ? e->stamp_ring + 6 * (e->stats.batches % STAMP_RING) : nullptr;
    if (sr) k_stamp<<<1, 64, 0, f>>>(sr + 0);
    if (B.dirty) HIPCHK(e, hipMemsetAsync(B.zero, 0, e->zero_bytes, f));   // an earlier batch stopped early
    B.dirty = true;
    uint32_t* ghist = B.ctrl + CTRL_HIST;
    // few enough blocks that the per-block histogram flush (3 x 256 global
    // atomics per block on 768 shared words) stays cheap
    const int probe_grid = (int)std::min<uint32_t>((m + PROBE_BLOCK - 1) / PROBE_BLOCK, (uint32_t)e->probe_grid);
    const bool xs = a.sms != nullptr;   // explicit server clock: 32-byte request records
    // the grouping sort's predicted plan (below): with k_sort_local alone only
    // the MSD histogram is used, so the probe counts that pass only
    const bool pred_local = e->sort_passes > 1 && (m <= LOC_MAX || *(volatile uint32_t*)e->h_plan == 1u);
    const int hist_passes = pred_local ? 1 : e->sort_passes;
    const RouteIn rin = ri ? *ri : RouteIn{};
    // an explicit server clock: fields that do not fit the 16-byte record
    // go to the set's side arrays (rec_pack)
    const RecSide side{B.side_n, B.side_cfg, B.side_sms};
    if (ri)
        k_probe<1, true, true><<<probe_grid, PROBE_BLOCK, 0, f>>>(
            m, a.key, a.n, a.cfg, e->d_cfg, (uint32_t)e->h_cfg.size(), e->d_tb, e->tb_cap - 1, e->d_win,
            e->win_cap - 1, e->win_base, e->invalid_key, B.sk0, ghist, hist_passes, e->sort_shifts, a,
            static_cast<ReqRec<true>*>(B.rec), e->d_eflags, rin, B.ctrl, CTRL_HEAD, side);
    else if (xs)
        k_probe<1, true><<<probe_grid, PROBE_BLOCK, 0, f>>>(
            m, a.key, a.n, a.cfg, e->d_cfg, (uint32_t)e->h_cfg.size(), e->d_tb, e->tb_cap - 1, e->d_win,
            e->win_cap - 1, e->win_base, e->invalid_key, B.sk0, ghist, hist_passes, e->sort_shifts, a,
            static_cast<ReqRec<true>*>(B.rec), e->d_eflags, rin, B.ctrl, CTRL_HEAD, side);
    else
        k_probe<1, false><<<probe_grid, PROBE_BLOCK, 0, f>>>(
            m, a.key, a.n, a.cfg, e->d_cfg, (uint32_t)e->h_cfg.size(), e->d_tb, e->tb_cap - 1, e->d_win,
            e->win_cap - 1, e->win_base, e->invalid_key, B.sk0, ghist, hist_passes, e->sort_shifts, a,
            static_cast<ReqRec<false>*>(B.rec), e->d_eflags, rin, B.ctrl, CTRL_HEAD, side);
    if (tall) (void)hipEventRecord(ev[1], f);
    uint32_t tiles = (m + SORT_TILE - 1) / SORT_TILE;
    uint32_t *kin = B.sk0, *vin = B.sv0, *kout = B.sk1, *vout = B.sv1;
    const int P = e->sort_passes;
    uint32_t* segctr = B.ctrl + CTRL_NSEG;
    const SegLists lists{{B.list[0], B.list[1], B.list[2], B.list[3]}, segctr, B.claim};
    const uint32_t huge_min = std::max(e->huge_min, e->heavy_min);
    // the request records move with the first pass into its bucket order,
    // where k_permute gathers them (ReqRec, 16 bytes)
    const uint4* rec_in = static_cast<const uint4*>(B.rec);
    uint4* rec_out = static_cast<uint4*>(B.recb);
    const int rw = 1;
    if (P <= 1) {
        k_sort_pass<true><<<tiles, SORT_BLOCK, 0, f>>>(kin, vin, kout, vout, m, 0, ghist, B.status,
                                                       B.ctrl + CTRL_TILE, e->d_eflags, nullptr, nullptr, 0, nullptr,
                                                       mdev, rec_in, rec_out, rw);
        kin = B.sk1;
        vin = B.sv1;
    } else {
        // MSD pass (and the plan: every bucket fits LDS or not), then either
        // k_sort_local or the LSD passes over the lower bits; both end in
        // the same buffers
        uint32_t* plan = B.ctrl + CTRL_PLAN;
        k_sort_pass<true><<<tiles, SORT_BLOCK, 0, f>>>(B.sk0, B.sv0, B.sk1, B.sv1, m, e->sort_bits - 8, ghist,
                                                       B.status, B.ctrl + CTRL_TILE, e->d_eflags, nullptr, plan,
                                                       LOC_MAX, m > LOC_MAX ? e->d_plan : nullptr, mdev, rec_in, rec_out, rw);
        const bool odd = ((P - 1) & 1) != 0;     // LSD passes after the MSD pass end in sk0 when odd
        uint32_t* fk = odd ? B.sk0 : B.sk1;
        uint32_t* fv = odd ? B.sv0 : B.sv1;
        // predicted plan: when the batch cannot hold a bucket too large for
        // LDS, or the last plan the host sees had none (only batches larger
        // than LOC_MAX write it: a smaller one fits whatever its keys), only k_sort_local is
        // launched (it sorts a bucket too large for LDS itself, slowly: a
        // misprediction costs time, never a result) -- no LSD passes and no
        // k_segments, which would only find the plan flag and return
        k_sort_local<<<RADIX, LOC_BLOCK, 0, f>>>(B.sk1, B.sv1, fk, fv, ghist, e->sort_bits - 8,
                                                 pred_local ? nullptr : plan + 1, e->invalid_key, e->win_base,
                                                 e->heavy_min, huge_min, lists, B.sk0, B.sv0);
        if (pred_local) e->stats.sort_predicted++;
        kin = B.sk1;
        vin = B.sv1;
        kout = B.sk0;
        vout = B.sv0;
        for (int p = 1; p < P && !pred_local; p++) {
            uint32_t* status = B.status + (size_t)p * e->max_tiles * RADIX;
            k_sort_pass<false><<<tiles, SORT_BLOCK, 0, f>>>(kin, vin, kout, vout, m, 8 * (p - 1), ghist + p * RADIX,
                                                            status, B.ctrl + CTRL_TILE + p, e->d_eflags, plan, nullptr,
                                                            0, nullptr, mdev);
            std::swap(kin, kout);
            std::swap(vin, vout);
        }
        if (pred_local) {
            kin = fk;
            vin = fv;
        }
        // kin / vin == fk / fv
    }
    if (tall) (void)hipEventRecord(ev[2], f);
    // sorted keys/values are now in kin/vin
    int sgrid = (int)std::min<uint32_t>((m + SEG_TILE - 1) / SEG_TILE, 2048);
    if (!pred_local)
        k_segments<<<sgrid, 256, GROUP_LDS, f>>>(kin, m, e->invalid_key, e->win_base, e->heavy_min, huge_min, lists,
                                                 P > 1 ? B.ctrl + CTRL_PLAN : nullptr, mdev);
    // sorted-order buffers; tokens always kept (token-bucket results derive from them)
    // (the server clock only when the caller gave one: else floor(ts / 1e6) where it is read)
    ReqArgs ps{nullptr, B.p_ts, B.p_n, B.p_cfg, a.sms ? B.p_sms : nullptr, B.o_dec, nullptr, nullptr, nullptr,
               B.o_tok, B.p_fresh};
    int pgrid = (int)std::min<uint32_t>((m + 255) / 256, (uint32_t)e->perm_grid);
    const int pgrid_r = (int)std::min<uint32_t>((m + 255) / 256, (uint32_t)e->perm_grid);
    TbPre pre{B.q_add, B.q_th};
    // front_done rides on k_permute's dispatch packet (no marker packet)
    // unless a stamp kernel follows it
    const bool bind_front = !sr;
    // the arrival index of every sorted position for the finish: from the
    // moved records into the free value buffer
    uint32_t* vfin = vin == B.sv0 ? B.sv1 : B.sv0;
    if (xs)
        hipExtLaunchKernelGGL(k_permute<true>, dim3(pgrid_r), dim3(256), (uint32_t)GROUP_LDS, f, nullptr,
                              bind_front ? B.front_done : nullptr, 0u, kin, vin, m, e->invalid_key, e->win_base,
                              e->d_cfg, e->profile, static_cast<const ReqRec<true>*>(B.recb), B.side_n, ps, pre,
                              mdev, B.side_cfg, vfin, (const int64_t*)B.side_sms);
    else
        hipExtLaunchKernelGGL(k_permute<false>, dim3(pgrid_r), dim3(256), (uint32_t)GROUP_LDS, f, nullptr,
                              bind_front ? B.front_done : nullptr, 0u, kin, vin, m, e->invalid_key, e->win_base,
                              e->d_cfg, e->profile, static_cast<const ReqRec<false>*>(B.recb), a.n, ps, pre, mdev,
                              a.cfg, vfin, (const int64_t*)nullptr);
    if (tall) (void)hipEventRecord(ev[3], f);
    if (sr) k_stamp<<<1, 64, 0, f>>>(sr + 1);
    if (!bind_front) HIPCHK(e, hipEventRecord(B.front_done, f));

    // replay: after this batch's grouping and the previous replay (stream
    // order on `chain`: the table state)
    hipStream_t c = e->chain, t = e->tail;
    HIPCHK(e, hipStreamWaitEvent(c, B.front_done, 0));
    // replay timing: the two events ride on the replay's own dispatch packet
    // (hipExtLaunchKernel) instead of two marker packets around it, unless
    // the stamp kernels must sit inside the timed interval
    const bool bound_ev = timed && !e->stamps && !sr;
    if (timed && !bound_ev) (void)hipEventRecord(ev[4], c);
    if (e->stamps) k_stamp<<<1, 64, 0, c>>>(B.ctrl + CTRL_DBG + 18);
    if (sr) k_stamp<<<1, 64, 0, c>>>(sr + 2);
    const uint32_t ncfg = (uint32_t)e->h_cfg.size();
    uint32_t* dbg = B.ctrl + CTRL_DBG;
    // timing off: chain_done rides on the dispatch instead
    const bool bind_done = !timed && !e->stamps && !sr;
    const hipEvent_t ev_a = bound_ev ? ev[4] : nullptr, ev_b = bound_ev ? ev[5] : bind_done ? B.chain_done : nullptr;
    // no huge segment in the last replay seen: the light replay kernel
    // (k_replay_light; a huge segment that comes anyway is replayed exactly,
    // as a heavy one, and flips the prediction back).  Large batches only:
    // a server's batches swing from small ones (no huge segment) to a large
    // one after a stall, whose hot key the light kernel would replay as one
    // wave -- an 8 ms batch at 1e7 QPS (profiles/r5z2_e2e.json window 13)
    const bool light = e->light_ok && (e->force_light || (m >= LIGHT_MIN_BATCH && *(volatile uint32_t*)e->h_huge == 0u));
    e->stats.light_batches += light ? 1 : 0;
    const int lc = ncfg <= (uint32_t)MAX_LCFG ? 0 : 1;
    if (light)
        hipExtLaunchKernelGGL(lc == 0 ? k_replay_light<true> : k_replay_light<false>, dim3(e->coop_grid),
                              dim3(LT_BLOCK), (uint32_t)e->light_pad[lc], c, ev_a, ev_b, 0u, kin, lists, segctr + 4,
                              e->win_base, e->d_tb, e->d_win, e->spill(), e->d_cfg, ncfg, e->profile, ps, pre,
                              e->d_eflags, dbg, B.runs, (uint32_t)e->coop_base, m / e->coop_light_div, e->d_huge);
    else
        hipExtLaunchKernelGGL(lc == 0 ? k_tb_chain<true> : k_tb_chain<false>, dim3(e->coop_grid), dim3(CH_BLOCK),
                              (uint32_t)e->chain_pad[lc], c, ev_a, ev_b, 0u, kin, lists, segctr + 4, e->win_base,
                              e->d_tb, e->d_win, e->spill(), e->d_cfg, ncfg, e->profile, ps, pre, e->d_eflags, dbg,
                              B.runs, (uint32_t)e->coop_base, m / e->coop_light_div, e->d_huge);
    HIPCHK(e, hipGetLastError());
    if (e->stamps) k_stamp<<<1, 64, 0, c>>>(B.ctrl + CTRL_DBG + 19);
    if (sr) k_stamp<<<1, 64, 0, c>>>(sr + 3);
    // the replay's end: with timing on, its timing event also orders the
    // finish stream (no extra marker packet on the chain stream)
    hipEvent_t chain_end = B.chain_done;
    if (bound_ev) {
        chain_end = ev[5];
    } else if (timed) {
        HIPCHK(e, hipEventRecord(ev[5], c));
        chain_end = ev[5];
    } else if (!bind_done) {
        HIPCHK(e, hipEventRecord(B.chain_done, c));
    }
    // finish: outputs of the committed runs, results to the caller's order
    HIPCHK(e, hipStreamWaitEvent(t, chain_end, 0));
    if (tall) (void)hipEventRecord(ev[6], t);
    if (sr) k_stamp<<<1, 64, 0, t>>>(sr + 4);
    // runs come from the chain only: a light replay leaves none to expand
    // (mixed: 24 + 7 us per batch off the finish stream)
    if (!light) {
        // (a wave per multi-decade run: ~300 per configs[1] batch, 32 blocks took 43 us)
        if (e->profile == PROFILE_REDIS7) k_tb_expand_x<<<128, 256, GROUP_LDS, t>>>(B.runs, ps, pre, e->d_eflags);
        k_tb_expand<<<(int)std::min<uint32_t>((m + 4 * CH_TILE - 1) / (4 * CH_TILE), 2048), 256, GROUP_LDS, t>>>(
            m, B.runs, e->profile, ps, pre, e->d_eflags);
    }
    if (ri) {
        // a routed batch: one result record per request at its receive
        // index, through merge-position buckets (no scattered 32-byte stores:
        // routed mixed +3.5 %, profiles/r4w_ab_routed_finish.txt)
        if (m <= UP_MAX) {
            k_unpermute_bucket<<<(m + 256 * UP_ITEMS - 1) / (256 * UP_ITEMS), 256, GROUP_LDS, t>>>(
                kin, vfin, m, e->invalid_key, ps, B.upb, B.ctrl + CTRL_UPB, ri->count);
            k_unpermute_routed_out<<<(m + UP_BUCKET - 1) / UP_BUCKET, 256, 0, t>>>(m, B.upb, e->d_cfg, *ri);
        } else
            k_unpermute_routed<<<pgrid, 256, GROUP_LDS, t>>>(kin, vfin, m, e->invalid_key, e->d_cfg, ps, *ri);
    } else if (m <= UP_MAX) {
        // results to the caller's order through arrival-index buckets: no
        // scattered partial-line stores
        k_unpermute_bucket<<<(m + 256 * UP_ITEMS - 1) / (256 * UP_ITEMS), 256, GROUP_LDS, t>>>(
            kin, vfin, m, e->invalid_key, ps, B.upb, B.ctrl + CTRL_UPB);
        k_unpermute_bucket_out<<<(m + UP_BUCKET - 1) / UP_BUCKET, 256, 0, t>>>(m, B.upb, e->d_cfg, a);
    } else {
        k_unpermute<<<pgrid, 256, GROUP_LDS, t>>>(kin, vfin, m, e->invalid_key, e->d_cfg, ps, a);
    }
    if (sr) k_stamp<<<1, 64, 0, t>>>(sr + 5);
    if (timed) {
        if (tall) (void)hipEventRecord(ev[7], t);
        e->ev_pending.push_back(ev);
    }
    // the set's words for its next batch (all but the head: k_probe)
    HIPCHK(e, hipMemsetAsync(B.zero + CTRL_HEAD, 0, e->zero_bytes - 4 * CTRL_HEAD, t));
    B.dirty = false;
    HIPCHK(e, hipEventRecord(B.back_done, t));
    if (done_ev) HIPCHK(e, hipEventRecord(done_ev, t));   // the caller waits on it when it wants to
    else HIPCHK(e, hipStreamWaitEvent(s_out ? s_out : s, B.back_done, 0));
    B.used = true;
    HIPCHK(e, hipGetLastError());
    e->stats.batches++;
    e->stats.decisions += m;
    return RL_OK;
}

// Launch every kernel once at creation, on batches of requests that are all
// rejected (no config is registered yet), so no table entry is touched: HIP
// loads kernels lazily, and a server's first batch on either path (k_small, or
// the big path when load grows) would otherwise stall its queue for the load.
static int warm_up(rl_engine* e) {
    const uint32_t mb = std::min<uint32_t>(e->max_batch, e->small_max + 1);
    hipStream_t s = e->stream;
    HIPCHK(e, hipMemsetAsync(e->d_key, 0, 8 * (size_t)mb, s));
    HIPCHK(e, hipMemsetAsync(e->d_n, 0, 8 * (size_t)mb, s));
    HIPCHK(e, hipMemsetAsync(e->d_ts, 0, 8 * (size_t)mb, s));
    HIPCHK(e, hipMemsetAsync(e->d_cfgid, 0, 4 * (size_t)mb, s));
    ReqArgs a{e->d_key, e->d_ts, e->d_n, e->d_cfgid, nullptr, e->d_dec, e->d_rem, e->d_retry, e->d_reset, e->d_tok};
    HIPCHK(e, hipMemsetAsync(e->d_sms, 0, 8 * (size_t)mb, s));
    for (uint32_t m : {1u, mb}) {
        const int r = run_batch(e, m, a, s, false);
        if (r != RL_OK) return r;
    }
    {   // the record layout with an explicit server clock (k_probe / k_permute <true>)
        ReqArgs ax = a;
        ax.sms = e->d_sms;
        const int r = run_batch(e, mb, ax, s, false);
        if (r != RL_OK) return r;
    }
    {   // the light replay kernel too
        e->force_light = true;
        const int r = run_batch(e, mb, a, s, false);
        e->force_light = false;
        if (r != RL_OK) return r;
    }
    {   // the routed path's kernels (k_probe<.., true>, k_unpermute_routed) on a
        // batch whose device size is 0: every kernel returns at once
        ReqArgs ar{nullptr, nullptr, nullptr, nullptr, e->d_sms, nullptr, nullptr, nullptr, nullptr, nullptr};
        const RouteIn ri{nullptr, nullptr, e->d_zero, nullptr};
        const int r = run_batch(e, mb, ar, s, false, nullptr, &ri);
        if (r != RL_OK) return r;
    }
    // the table count / GC / key listing kernels, on empty ranges: a server's
    // first periodic count must not wait for their lazy load
    k_table_count<<<1, 256, 0, s>>>(e->d_tb, 0, 0, e->profile, e->d_count);
    k_table_count<<<1, 256, 0, s>>>(e->d_win, 0, 0, e->profile, e->d_count);
    k_table_count<<<1, 256, 0, s>>>(e->d_spill, 0, 0, e->profile, e->d_count);
    k_rehash<<<1, 256, 0, s>>>(e->d_tb, 0, e->d_tb, e->tb_cap - 1, 0, e->profile, e->d_count);
    k_rehash<<<1, 256, 0, s>>>(e->d_win, 0, e->d_win, e->win_cap - 1, 0, e->profile, e->d_count);
    k_spill_rehash<<<1, 256, 0, s>>>(e->d_spill, 0, e->d_spill, e->spill_cap - 1, e->d_win, e->win_cap - 1, 0,
                                     e->profile, e->d_count);
    HIPCHK(e, hipGetLastError());
    const int r = drain(e);
    if (r != RL_OK) return r;
    HIPCHK(e, hipMemset(e->d_eflags, 0, 4));
    // the warm-up batches had no huge segment: without this, the first real
    // batches (all those enqueued before one replays) would take the light
    // kernel, which replays a hot key as one wave (~0.75 ms per 1M batch)
    *(volatile uint32_t*)e->h_huge = 1u;
    e->stats = rl_stats{};
    e->stats.sort_bits = e->sort_bits;
    e->stats.sort_passes = e->sort_passes;
    return RL_OK;
}

static int check_flags(rl_engine* e, uint32_t f) {
    if (f & EF_TABLE_FULL) return fail(e, RL_ENOMEM, "state table full");
    if (f & EF_LOOKBACK) return fail(e, RL_ETIMEOUT, "radix sort look-back timed out");
    if (f & EF_ORDER) return fail(e, RL_EORDER, "per-key window ids went backwards");
    if (f & EF_INTERNAL) return fail(e, RL_EDEVICE, "cooperative replay invariant violated");
    if (f & EF_ROUTED_OVER) return fail(e, RL_EOVERFLOW, "routed batch count above m_max: requests past it undecided");
    return RL_OK;
}

extern "C" int rl_engine_sync(rl_engine* e) {
    if (!e) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    int r = drain(e);
    if (r != RL_OK) return r;
    uint32_t f = 0;
    HIPCHK(e, hipMemcpy(&f, e->d_eflags, 4, hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemset(e->d_eflags, 0, 4));
    return check_flags(e, f);
}

extern "C" int rl_decide_batch_device(rl_engine* e, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                                      const int64_t* n, const uint32_t* cfg_id, const int64_t* server_ms,
                                      uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                                      int64_t* reset_at_ns, double* tokens, void* stream) {
    if (!e || (m && (!key_id || !ts_ns || !n || !cfg_id || !decision || !remaining || !retry_after_ns || !reset_at_ns)))
        return RL_EINVAL;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    for (size_t off = 0; off < m; off += e->max_batch) {
        uint32_t c = (uint32_t)std::min<size_t>(e->max_batch, m - off);
        ReqArgs a{key_id + off, ts_ns + off, n + off, cfg_id + off, server_ms ? server_ms + off : nullptr,
                  decision + off, remaining + off, retry_after_ns + off, reset_at_ns + off,
                  tokens ? tokens + off : nullptr};
        int r = run_batch(e, c, a, s, (e->flags & RL_OPT_PIPELINE) != 0);
        if (r != RL_OK) return r;
    }
    return RL_OK;
}

extern "C" int rl_decide_routed_device_io(rl_engine* e, size_t m_max, const uint32_t* count,
                                          const rl_route_rec* recv, const uint32_t* order, const int64_t* server_ms,
                                          rl_route_res* res, void* in_stream, void* out_stream) {
    if (!e || !count || (m_max && (!recv || !order || !server_ms || !res))) return RL_EINVAL;
    if (m_max > e->max_batch) return fail(e, RL_EINVAL, "routed batch bound above max_batch");
    if (!m_max) return RL_OK;
    (void)hipSetDevice(e->device);
    hipStream_t s = in_stream ? (hipStream_t)in_stream : e->stream;
    hipStream_t so = out_stream ? (hipStream_t)out_stream : s;
    // the server-clock array is the routed records' store clock (always given)
    ReqArgs a{nullptr, nullptr, nullptr, nullptr, server_ms, nullptr, nullptr, nullptr, nullptr, nullptr};
    const RouteIn ri{recv, order, count, res};
    return run_batch(e, (uint32_t)m_max, a, s, false, nullptr, &ri, so);
}

extern "C" int rl_decide_routed_device_ev(rl_engine* e, size_t m_max, const uint32_t* count,
                                          const rl_route_rec* recv, const uint32_t* order, const int64_t* server_ms,
                                          rl_route_res* res, void* in_stream, void* done_event) {
    if (!e || !count || !done_event || (m_max && (!recv || !order || !server_ms || !res))) return RL_EINVAL;
    if (m_max > e->max_batch) return fail(e, RL_EINVAL, "routed batch bound above max_batch");
    (void)hipSetDevice(e->device);
    hipStream_t s = in_stream ? (hipStream_t)in_stream : e->stream;
    if (!m_max) {   // nothing to decide: the event marks the caller's stream
        HIPCHK(e, hipEventRecord((hipEvent_t)done_event, s));
        return RL_OK;
    }
    ReqArgs a{nullptr, nullptr, nullptr, nullptr, server_ms, nullptr, nullptr, nullptr, nullptr, nullptr};
    const RouteIn ri{recv, order, count, res};
    return run_batch(e, (uint32_t)m_max, a, s, false, nullptr, &ri, nullptr, (hipEvent_t)done_event);
}

extern "C" int rl_decide_routed_device(rl_engine* e, size_t m_max, const uint32_t* count, const rl_route_rec* recv,
                                       const uint32_t* order, const int64_t* server_ms, rl_route_res* res,
                                       void* stream) {
    return rl_decide_routed_device_io(e, m_max, count, recv, order, server_ms, res, stream, stream);
}

extern "C" int rl_decide_batch_keys_device(rl_engine* e, size_t m, const uint8_t* key_bytes, uint64_t nbytes,
                                           const uint64_t* key_offsets, uint64_t seed, const char* prefix,
                                           size_t prefix_len, const int64_t* ts_ns, const int64_t* n,
                                           const uint32_t* cfg_id, const int64_t* server_ms, uint8_t* decision,
                                           int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns,
                                           double* tokens, void* stream) {
    if (!e || prefix_len > RL_KEYHASH_MAX_PREFIX || (prefix_len && !prefix) ||
        (m && (!key_offsets || (nbytes && !key_bytes) || !ts_ns || !n || !cfg_id || !decision || !remaining ||
               !retry_after_ns || !reset_at_ns)))
        return RL_EINVAL;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    for (size_t off = 0; off < m; off += e->max_batch) {
        uint32_t c = (uint32_t)std::min<size_t>(e->max_batch, m - off);
        ReqArgs a{nullptr, ts_ns + off, n + off, cfg_id + off, server_ms ? server_ms + off : nullptr,
                  decision + off, remaining + off, retry_after_ns + off, reset_at_ns + off,
                  tokens ? tokens + off : nullptr};
        KeyBytes kb{key_bytes, nbytes, key_offsets + off, seed, prefix, prefix_len, (double)nbytes / (double)m};
        int r = run_batch(e, c, a, s, (e->flags & RL_OPT_PIPELINE) != 0, &kb);
        if (r != RL_OK) return r;
    }
    return RL_OK;
}

extern "C" int rl_decide_batch(rl_engine* e, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                               const int64_t* n, const uint32_t* cfg_id, const int64_t* server_ms,
                               uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                               int64_t* reset_at_ns, double* tokens) {
    if (!e || (m && (!key_id || !ts_ns || !n || !cfg_id || !decision || !remaining || !retry_after_ns || !reset_at_ns)))
        return RL_EINVAL;
    (void)hipSetDevice(e->device);
    hipStream_t s = e->stream;
    HIPCHK(e, hipMemsetAsync(e->d_eflags, 0, 4, s));
    for (size_t off = 0; off < m; off += e->max_batch) {
        uint32_t c = (uint32_t)std::min<size_t>(e->max_batch, m - off);
        HIPCHK(e, hipMemcpyAsync(e->d_key, key_id + off, 8 * (size_t)c, hipMemcpyHostToDevice, s));
        HIPCHK(e, hipMemcpyAsync(e->d_ts, ts_ns + off, 8 * (size_t)c, hipMemcpyHostToDevice, s));
        HIPCHK(e, hipMemcpyAsync(e->d_n, n + off, 8 * (size_t)c, hipMemcpyHostToDevice, s));
        HIPCHK(e, hipMemcpyAsync(e->d_cfgid, cfg_id + off, 4 * (size_t)c, hipMemcpyHostToDevice, s));
        if (server_ms) HIPCHK(e, hipMemcpyAsync(e->d_sms, server_ms + off, 8 * (size_t)c, hipMemcpyHostToDevice, s));
        ReqArgs a{e->d_key, e->d_ts, e->d_n, e->d_cfgid, server_ms ? e->d_sms : nullptr,
                  e->d_dec, e->d_rem, e->d_retry, e->d_reset, tokens ? e->d_tok : nullptr};
        int r = run_batch(e, c, a, s, false);
        if (r != RL_OK) return r;
        HIPCHK(e, hipMemcpyAsync(decision + off, e->d_dec, c, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipMemcpyAsync(remaining + off, e->d_rem, 8 * (size_t)c, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipMemcpyAsync(retry_after_ns + off, e->d_retry, 8 * (size_t)c, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipMemcpyAsync(reset_at_ns + off, e->d_reset, 8 * (size_t)c, hipMemcpyDeviceToHost, s));
        if (tokens) HIPCHK(e, hipMemcpyAsync(tokens + off, e->d_tok, 8 * (size_t)c, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipStreamSynchronize(s));
    }
    uint32_t f = 0;
    HIPCHK(e, hipMemcpy(&f, e->d_eflags, 4, hipMemcpyDeviceToHost));
    return check_flags(e, f);
}

// The DEL only writes `when` fields of table entries, which only the replays
// (k_tb_chain, k_small: both on `chain`) read; the grouping reads entry keys
// only and the finish no table state.  So one kernel on `chain` between two
// replays is exactly "after every earlier batch, before every later one".
extern "C" int rl_reset_device(rl_engine* e, uint32_t cfg_id, uint64_t key_id, int64_t ts_ns, void* stream) {
    if (!e || cfg_id >= e->h_cfg.size() || key_id == EMPTY_KEY) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    hipStream_t s = stream ? (hipStream_t)stream : e->stream;
    k_reset<<<1, 1, 0, e->chain>>>(key_id, ts_ns, e->d_cfg, cfg_id, e->d_tb, e->tb_cap - 1, e->d_win,
                                    e->win_cap - 1, e->spill());
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipEventRecord(e->ev_reset, e->chain));
    HIPCHK(e, hipStreamWaitEvent(s, e->ev_reset, 0));
    return RL_OK;
}

extern "C" int rl_reset(rl_engine* e, uint32_t cfg_id, uint64_t key_id, int64_t ts_ns) {
    const int r = rl_reset_device(e, cfg_id, key_id, ts_ns, nullptr);
    if (r != RL_OK) return r;
    HIPCHK(e, hipStreamSynchronize(e->stream));
    return RL_OK;
}

extern "C" int rl_table_info_get(rl_engine* e, int64_t now_ms, rl_table_info* out) {
    if (!e || !out || out->struct_size < 8) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    int r = drain(e);
    if (r != RL_OK) return r;
    // preallocated counters (no hipMalloc / hipFree, which synchronize the
    // device, on a server's periodic count)
    unsigned long long* d = e->d_count;
    unsigned long long* h = e->h_count;
    hipStream_t s = e->stream;
    bool ok = hipMemsetAsync(d, 0, 6 * sizeof(unsigned long long), s) == hipSuccess;
    k_table_count<<<1024, 256, 0, s>>>(e->d_tb, e->tb_cap, now_ms, e->profile, d);
    k_table_count<<<1024, 256, 0, s>>>(e->d_win, e->win_cap, now_ms, e->profile, d + 2);
    k_table_count<<<1024, 256, 0, s>>>(e->d_spill, e->spill_cap, now_ms, e->profile, d + 4);
    ok = ok && hipMemcpyAsync(h, d, 6 * sizeof(unsigned long long), hipMemcpyDeviceToHost, s) == hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    if (!ok) return fail(e, RL_EDEVICE, "table count failed");
    return copy_out(out, rl_table_info{sizeof(rl_table_info), 0, e->tb_cap, h[0], h[1], e->win_cap, h[2], h[3],
                                       e->spill_cap, h[4], h[5]});
}

extern "C" int rl_table_keys(rl_engine* e, int64_t now_ms, rl_key_rec* out, size_t cap, uint64_t* count) {
    if (!e || !count || (cap && !out)) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    int r = drain(e);
    if (r != RL_OK) return r;
    unsigned long long* d = nullptr;
    rl_key_rec* dout = nullptr;
    HIPCHK(e, hipMalloc(&d, sizeof(unsigned long long)));
    if (cap && hipMalloc(&dout, sizeof(rl_key_rec) * cap) != hipSuccess) {
        (void)hipFree(d);
        return fail(e, RL_ENOMEM, "table keys: allocation failed");
    }
    hipStream_t s = e->stream;
    unsigned long long n = 0;
    bool ok = hipMemsetAsync(d, 0, sizeof n, s) == hipSuccess;
    k_table_keys<<<1024, 256, 0, s>>>(e->d_tb, e->tb_cap, e->d_win, e->win_cap, e->d_spill, e->spill_cap, now_ms,
                                       e->profile, dout, cap, d);
    ok = ok && hipMemcpyAsync(&n, d, sizeof n, hipMemcpyDeviceToHost, s) == hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    if (ok && cap && n)
        ok = hipMemcpy(out, dout, sizeof(rl_key_rec) * std::min<uint64_t>(n, cap), hipMemcpyDeviceToHost) == hipSuccess;
    (void)hipFree(d);
    (void)hipFree(dout);
    if (!ok) return fail(e, RL_EDEVICE, "table keys failed");
    *count = n;
    return RL_OK;
}

extern "C" int rl_table_gc(rl_engine* e, int64_t now_ms, uint64_t tb_capacity, uint64_t win_capacity,
                           rl_table_info* out) {
    if (!e || (out && out->struct_size < 8)) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    const uint64_t tb_cap = tb_capacity ? pow2_at_least(std::max<uint64_t>(tb_capacity, 1024)) : e->tb_cap;
    const uint64_t win_cap = win_capacity ? pow2_at_least(std::max<uint64_t>(win_capacity, 1024)) : e->win_cap;
    const uint64_t spill_cap = e->spill_follows ? pow2_at_least(std::max<uint64_t>(2 * win_cap, 1024)) : e->spill_cap;
    if (tb_cap + win_cap >= (1ull << 31)) return fail(e, RL_EINVAL, "table capacities too large");
    int r = drain(e);
    if (r != RL_OK) return r;
    TbEntry* ntb = nullptr;
    WinEntry* nwin = nullptr;
    SpillEntry* nsp = nullptr;
    unsigned long long* d = nullptr;
    bool ok = hipMalloc(&ntb, sizeof(TbEntry) * tb_cap) == hipSuccess;
    ok = ok && hipMalloc(&nwin, sizeof(WinEntry) * win_cap) == hipSuccess;
    ok = ok && hipMalloc(&nsp, sizeof(SpillEntry) * spill_cap) == hipSuccess;
    ok = ok && hipMalloc(&d, 6 * sizeof(unsigned long long)) == hipSuccess;
    if (!ok) {
        (void)hipFree(ntb); (void)hipFree(nwin); (void)hipFree(nsp); (void)hipFree(d);
        return fail(e, RL_ENOMEM, "table gc: allocation failed");
    }
    unsigned long long h[6] = {0, 0, 0, 0, 0, 0};
    hipStream_t s = e->stream;
    k_init_tb<<<2048, 256, 0, s>>>(ntb, tb_cap);
    k_init_win<<<2048, 256, 0, s>>>(nwin, win_cap);
    k_init_spill<<<2048, 256, 0, s>>>(nsp, spill_cap);
    ok = hipMemsetAsync(d, 0, sizeof h, s) == hipSuccess;
    k_rehash<<<2048, 256, 0, s>>>(e->d_tb, e->tb_cap, ntb, tb_cap - 1, now_ms, e->profile, d);
    k_rehash<<<2048, 256, 0, s>>>(e->d_win, e->win_cap, nwin, win_cap - 1, now_ms, e->profile, d + 2);
    // after the window entries: each live spill entry is counted in its new entry
    k_spill_rehash<<<2048, 256, 0, s>>>(e->d_spill, e->spill_cap, nsp, spill_cap - 1, nwin, win_cap - 1, now_ms,
                                        e->profile, d + 4);
    ok = ok && hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, s) == hipSuccess;
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    (void)hipFree(d);
    if (!ok || h[1] || h[3] || h[5]) {
        (void)hipFree(ntb);
        (void)hipFree(nwin);
        (void)hipFree(nsp);
        return ok ? fail(e, RL_ENOMEM, "table gc: live keys do not fit the requested capacity")
                  : fail(e, RL_EDEVICE, "table gc failed");
    }
    (void)hipFree(e->d_tb);
    (void)hipFree(e->d_win);
    (void)hipFree(e->d_spill);
    e->d_tb = ntb;
    e->d_win = nwin;
    e->d_spill = nsp;
    // slot ids (the sort keys) follow the capacities
    e->tb_cap = tb_cap;
    e->win_cap = win_cap;
    e->spill_cap = spill_cap;
    e->win_base = (uint32_t)tb_cap;
    e->invalid_key = (uint32_t)(tb_cap + win_cap);
    e->sort_bits = bitlen(e->invalid_key);
    e->sort_passes = (e->sort_bits + 7) / 8;
    e->sort_shifts = sort_shifts(e->sort_bits, e->sort_passes);
    e->stats.sort_bits = e->sort_bits;
    e->stats.sort_passes = e->sort_passes;
    return out ? rl_table_info_get(e, now_ms, out) : RL_OK;
}

extern "C" int rl_engine_stats(rl_engine* e, rl_stats* out) {
    if (!e || !out || out->struct_size < 8) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    uint32_t c[4] = {0, 0, 0, 0}, d[24] = {0};
    int r = drain(e);
    if (r != RL_OK) return r;
    const uint32_t* ctrl = e->set[e->last_set].ctrl;
    HIPCHK(e, hipMemcpy(c, ctrl + CTRL_NSEG, sizeof c, hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(d, ctrl + CTRL_DBG, sizeof d, hipMemcpyDeviceToHost));
    // replay timers (10 ns ticks, k_tb_chain): [0] longest huge segment,
    // [2] longest light phase of a block, [4] first block start -> last block end
    for (auto& x : e->stats.stamp_cycles) x = 0;
    e->stats.stamp_cycles[0] = d[8];
    e->stats.stamp_cycles[2] = d[12];
    if (d[13]) e->stats.stamp_cycles[4] = (uint32_t)(d[14] - ~d[13]);
    e->stats.stamp_cycles[6] = d[2];   // max rounds of one segment
    e->stats.last_heavy = c[0] + c[3];                        // chain (token-bucket) segments
    e->stats.last_segments = (uint64_t)c[0] + c[1] + c[2] + c[3];
    e->stats.last_coop_rounds = d[0];
    e->stats.last_coop_iters = d[1];
    for (int k = 0; k < 4; k++) e->stats.coop_ends[k] = d[3 + k];
    return copy_out(out, e->stats);
}

extern "C" int rl_engine_set_timing(rl_engine* e, int on) {
    if (!e) return RL_EINVAL;
    e->timing = on != 0;
    e->timing_all = on > 1;    // 1 or -k: replay events only
    e->timing_stride = on < 0 ? (uint32_t)(-(int64_t)on) : 1u;
    e->timing_seq = 0;
    return RL_OK;
}

extern "C" int rl_engine_stage_times(rl_engine* e, double* ms, int nstages, uint64_t* batches) {
    if (!e) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    for (auto& ev : e->ev_pending) {
        HIPCHK(e, hipEventSynchronize(ev[7] ? ev[7] : ev[5]));
        static const int from[NSTAGES] = {0, 1, 2, 4, 6}, to[NSTAGES] = {1, 2, 3, 5, 7};
        for (int k = 0; k < NSTAGES; k++) {
            if (!ev[from[k]] || !ev[to[k]]) continue;
            float t = 0;
            HIPCHK(e, hipEventElapsedTime(&t, ev[from[k]], ev[to[k]]));
            e->stage_ms[k] += t;
        }
        e->timed_batches++;
        for (auto x : ev)
            if (x) e->ev_pool.push_back(x);
    }
    e->ev_pending.clear();
    for (int k = 0; k < nstages && k < NSTAGES; k++) ms[k] = e->stage_ms[k];
    if (batches) *batches = e->timed_batches;
    for (int k = 0; k < NSTAGES; k++) e->stage_ms[k] = 0;
    e->timed_batches = 0;
    return RL_OK;
}

// diagnostic (RL_STAMP_KERNELS=1): the stamp ring, 6 words per batch
// (realtime, 10 ns) for batches b mod STAMP_RING
extern "C" int rl_engine_debug_stamps(rl_engine* e, uint32_t* out, size_t n) {
    if (!e || !out) return RL_EINVAL;
    if (!e->stamp_ring) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    if (n > 6 * STAMP_RING) n = 6 * STAMP_RING;
    int r = drain(e);
    if (r != RL_OK) return r;
    HIPCHK(e, hipMemcpy(out, e->stamp_ring, 4 * n, hipMemcpyDeviceToHost));
    return RL_OK;
}

// diagnostic: device calls of the q14 big-integer slow paths so far
extern "C" int rl_engine_debug_q14_slow(rl_engine* e, uint64_t* out) {
    if (!e || !out) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    int r = drain(e);
    if (r != RL_OK) return r;
    unsigned long long v = 0;
    HIPCHK(e, hipMemcpyFromSymbol(&v, HIP_SYMBOL(rlq::q14_slow_calls), sizeof v, 0, hipMemcpyDeviceToHost));
    *out = v;
    return RL_OK;
}

// diagnostic: the last batch's replay debug words (include/rl_engine.h)
extern "C" int rl_engine_debug_words(rl_engine* e, uint32_t* out, size_t n) {
    if (!e || !out) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    if (n > CTRL_DBGN) n = CTRL_DBGN;
    int r = drain(e);
    if (r != RL_OK) return r;
    HIPCHK(e, hipMemcpy(out, e->set[e->last_set].ctrl + CTRL_DBG, 4 * n, hipMemcpyDeviceToHost));
    return RL_OK;
}

extern "C" int rl_last_error(rl_engine* e, char* buf, size_t len) {
    if (!e || !buf || !len) return RL_EINVAL;
    snprintf(buf, len, "%s", e->err.c_str());
    return RL_OK;
}

extern "C" int rl_selftest_q14_host(const double* in, double* out, size_t n) {
    if (!in || !out) return RL_EINVAL;
    for (size_t i = 0; i < n; i++) out[i] = rlq::q14(in[i]);
    return RL_OK;
}

extern "C" int rl_selftest_q14_device(rl_engine* e, const double* in, double* out, size_t n) {
    if (!e || !in || !out) return RL_EINVAL;
    (void)hipSetDevice(e->device);
    double *di = nullptr, *dout = nullptr;
    HIPCHK(e, hipMalloc(&di, 8 * std::max<size_t>(n, 1)));
    HIPCHK(e, hipMalloc(&dout, 8 * std::max<size_t>(n, 1)));
    HIPCHK(e, hipMemcpy(di, in, 8 * n, hipMemcpyHostToDevice));
    if (n) k_q14<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(di, dout, (uint32_t)n);
    HIPCHK(e, hipStreamSynchronize(e->stream));
    HIPCHK(e, hipMemcpy(out, dout, 8 * n, hipMemcpyDeviceToHost));
    (void)hipFree(di);
    (void)hipFree(dout);
    return RL_OK;
}
