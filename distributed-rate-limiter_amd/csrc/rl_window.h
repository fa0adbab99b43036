// rl_window.h -- the Redis keyspace of the window counters and the two window
// scripts over it.
//
// Redis names a window counter "B:ws" (fixedwindow.go:72-75,
// slidingwindow.go:74-79) and keeps any number of them per user key B, each
// with its own TTL.  Here a user key owns one 64-byte table entry holding its
// two newest window keys (WinEntry, rl_table.h) -- with per-key time moving
// forward only those two are ever read again -- and a spill table holding
// every other live one: a live key evicted from the entry, or an older window
// key created by a request whose time went back (N app servers with skewed
// clocks sharing one limiter).  So the keyspace is exact for any per-key
// order of request times.  Expiry follows Redis's lazy rule at the request's
// server clock; a dead entry is reclaimed, which equals Redis provided the
// per-key server clock never goes back (a Redis server's clock).
#pragma once

#include "rl_semantics.h"
#include "rl_table.h"

namespace rl {

// a user key's window keys while its segment runs (registers)
struct WinState {
    WinSlot s[2];
    uint64_t key;     // user key id: owner of its spill entries
    int64_t nspill;   // number of spill entries owned (WinEntry::nspill)
};

__device__ inline WinState win_load(const WinEntry* e) {
    WinState w;
    w.key = e->key;
    w.nspill = e->nspill;
    w.s[0] = e->s[0];
    w.s[1] = e->s[1];
    return w;
}

__device__ inline void win_store(WinEntry* e, const WinState& w) {
    e->nspill = w.nspill;
    e->s[0] = w.s[0];
    e->s[1] = w.s[1];
}

// key ids of spill slots are read past L1: another wave may claim a slot
// (EMPTY -> id) at any time, and a claim of our own must never read back stale
__device__ inline uint64_t spill_key(const SpillEntry* e) {
    return __hip_atomic_load(&e->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// k's spill entry of window ws (deleted or not), or null
__device__ inline SpillEntry* spill_lookup(const Spill& S, uint64_t k, int64_t nspill, int64_t ws) {
    if (nspill <= 0) return nullptr;
    uint64_t h = spill_home(k, S.mask);
    int64_t seen = 0;
    for (uint64_t p = 0; p <= S.mask && p < MAX_PROBES; p++) {
        SpillEntry* e = &S.tab[h];
        const uint64_t key = spill_key(e);
        if (key == EMPTY_KEY) break;
        if (key == k) {
            if (e->ws == ws && e->when != ABSENT) return e;
            if (++seen >= nspill) break;
        }
        h = (h + 1) & S.mask;
    }
    return nullptr;
}

// store window key (ws, cnt, when) of w.key in the spill: one of its own dead
// entries (deleted, or expired at s_ms) or a newly claimed slot; null when the
// spill table is full
__device__ inline SpillEntry* spill_put(const Spill& S, WinState& w, int64_t ws, int64_t cnt, int64_t when,
                                        int64_t s_ms, int32_t profile) {
    uint64_t h = spill_home(w.key, S.mask);
    for (uint64_t p = 0; p <= S.mask && p < MAX_PROBES; p++) {
        SpillEntry* e = &S.tab[h];
        uint64_t key = spill_key(e);
        bool mine = key == w.key && !key_alive(e->when, s_ms, profile);
        if (key == EMPTY_KEY) {
            // every lane of a wave replaying one segment claims together: a
            // claim by our own key is ours
            const uint64_t prev = atomicCAS((unsigned long long*)&e->key, (unsigned long long)EMPTY_KEY,
                                            (unsigned long long)w.key);
            mine = prev == EMPTY_KEY || prev == w.key;
            if (mine) w.nspill++;
        }
        if (mine) {
            e->ws = ws;
            e->cnt = cnt;
            e->when = when;
            return e;
        }
        h = (h + 1) & S.mask;
    }
    return nullptr;
}

// where a window key lives: slot 0 / 1 of the entry, or a spill entry
constexpr int WK_NONE = -1, WK_SPILL = 2;
struct WinRef {
    int slot;
    SpillEntry* sp;
};

__device__ inline int64_t wk_cnt(const WinState& w, const WinRef& r) {
    return r.slot == WK_SPILL ? r.sp->cnt : w.s[r.slot].cnt;
}
__device__ inline void wk_set_cnt(WinState& w, const WinRef& r, int64_t v) {
    if (r.slot == WK_SPILL) r.sp->cnt = v;
    else w.s[r.slot].cnt = v;
}
__device__ inline void wk_set_when(WinState& w, const WinRef& r, int64_t v) {
    if (r.slot == WK_SPILL) r.sp->when = v;
    else w.s[r.slot].when = v;
}

// lookupKey with lazy expiry: an expired key is deleted where it is found
__device__ inline WinRef wk_find(WinState& w, const Spill& S, int64_t ws, int64_t s_ms, int32_t profile) {
    for (int k = 0; k < 2; k++) {
        if (w.s[k].when == ABSENT || w.s[k].ws != ws) continue;
        if (!key_alive(w.s[k].when, s_ms, profile)) { w.s[k].when = ABSENT; continue; }
        return WinRef{k, nullptr};
    }
    SpillEntry* e = spill_lookup(S, w.key, w.nspill, ws);
    if (!e) return WinRef{WK_NONE, nullptr};
    if (!key_alive(e->when, s_ms, profile)) {
        e->when = ABSENT;
        return WinRef{WK_NONE, nullptr};
    }
    return WinRef{WK_SPILL, e};
}

// the key INCRBY is about to create (count 0, no TTL); `keep` (a slot or -1)
// stays in the entry.  A free or expired slot takes it; else the older of the
// slot keys moves to the spill, unless the new key is older than it, which
// then goes to the spill itself -- the entry keeps the newest windows.
__device__ inline WinRef wk_create(WinState& w, const Spill& S, int keep, int64_t ws, int64_t s_ms,
                                   int32_t profile, uint32_t& eflags) {
    int best = -1;
    for (int k = 0; k < 2; k++) {
        if (k == keep) continue;
        if (!key_alive(w.s[k].when, s_ms, profile)) {
            w.s[k] = WinSlot{ws, 0, NO_EXPIRY};
            return WinRef{k, nullptr};
        }
        if (best < 0 || w.s[k].ws < w.s[best].ws) best = k;
    }
    if (w.s[best].ws > ws) {
        SpillEntry* e = spill_put(S, w, ws, 0, NO_EXPIRY, s_ms, profile);
        if (!e) {
            eflags |= EF_TABLE_FULL;
            return WinRef{WK_NONE, nullptr};
        }
        return WinRef{WK_SPILL, e};
    }
    if (!spill_put(S, w, w.s[best].ws, w.s[best].cnt, w.s[best].when, s_ms, profile)) eflags |= EF_TABLE_FULL;
    w.s[best] = WinSlot{ws, 0, NO_EXPIRY};
    return WinRef{best, nullptr};
}

// fixedWindowScript (fixedwindow.go:21-27) + AllowN (fixedwindow.go:65-115)
__device__ inline Out fw_step(WinState& w, const Spill& S, int64_t t, int64_t n, int64_t s_ms, const CfgDev& c,
                              int32_t profile, uint32_t& eflags) {
    Out o;
    o.tokens = 0.0;
    const int64_t ws = window_start(t, c);
    o.reset_at = wadd(wmul(ws, NS_PER_S), c.window);
    WinRef r = wk_find(w, S, ws, s_ms, profile);
    const int64_t old = r.slot != WK_NONE ? wk_cnt(w, r) : 0;
    if (incr_overflows(old, n)) {
        o.decision = DEC_ERROR; o.remaining = 0; o.retry = 0;
        return o;
    }
    if (r.slot == WK_NONE) r = wk_create(w, S, -1, ws, s_ms, profile, eflags);
    const int64_t cur = old + n;
    if (r.slot != WK_NONE) {
        wk_set_cnt(w, r, cur);
        if ((double)cur == (double)n) wk_set_when(w, r, expire_when(c.ttl_c, s_ms));
    }
    const int64_t count = go_f2i((double)cur);
    const bool allowed = count <= c.limit;
    const int64_t rem = wsub(c.limit, count);
    o.remaining = rem < 0 ? 0 : rem;
    o.decision = allowed ? DEC_ALLOWED : DEC_DENIED;
    o.retry = allowed ? 0 : until_reset(o.reset_at, t);
    return o;
}

// slidingWindowScript (slidingwindow.go:22-30) + AllowN (slidingwindow.go:68-122)
__device__ inline Out sw_step(WinState& w, const Spill& S, int64_t t, int64_t n, int64_t s_ms, const CfgDev& c,
                              int32_t profile, uint32_t& eflags) {
    Out o;
    o.tokens = 0.0;
    const int64_t ws = window_start(t, c);
    const int64_t pws = ws - c.ttl_c;
    o.reset_at = wadd(wmul(ws, NS_PER_S), c.window);
    // local prev = tonumber(redis.call('GET', KEYS[2]) or 0)
    WinRef pr = wk_find(w, S, pws, s_ms, profile);
    const double prev = pr.slot != WK_NONE ? (double)wk_cnt(w, pr) : 0.0;
    // local curr = redis.call('INCRBY', KEYS[1], ARGV[1])
    WinRef cr = wk_find(w, S, ws, s_ms, profile);
    const int64_t old = cr.slot != WK_NONE ? wk_cnt(w, cr) : 0;
    if (incr_overflows(old, n)) {
        o.decision = DEC_ERROR; o.remaining = 0; o.retry = 0;
        return o;
    }
    if (cr.slot == WK_NONE) cr = wk_create(w, S, pr.slot == WK_SPILL ? -1 : pr.slot, ws, s_ms, profile, eflags);
    const int64_t cur = old + n;
    if (cr.slot != WK_NONE) {
        wk_set_cnt(w, cr, cur);
        // if curr == tonumber(ARGV[1]) then EXPIRE KEYS[1] ARGV[2]
        if ((double)cur == (double)n) wk_set_when(w, cr, expire_when(c.ttl_c, s_ms));
    }
    // EXPIRE KEYS[2] ARGV[3]  (no-op when the key does not exist)
    pr = wk_find(w, S, pws, s_ms, profile);
    if (pr.slot != WK_NONE) wk_set_when(w, pr, expire_when(c.ttl_p, s_ms));
    const int64_t p = go_f2i(prev);
    const int64_t cc = go_f2i((double)cur);
    // calculateWeightedCount (slidingwindow.go:190-197)
    const int64_t elapsed = wsub(t, wmul(ws, NS_PER_S));
    const double progress = (double)elapsed / (double)c.window;
    double weighted = (double)p * (1.0 - progress);
    weighted = weighted + (double)cc;
    const bool allowed = weighted <= c.limit_d;
    const int64_t rem = wsub(c.limit, go_f2i(weighted));
    o.remaining = rem < 0 ? 0 : rem;
    o.decision = allowed ? DEC_ALLOWED : DEC_DENIED;
    o.retry = allowed ? 0 : until_reset(o.reset_at, t);
    return o;
}

// DEL of window key ws of the entry's user key (Reset)
__device__ inline void wk_delete(WinEntry* e, const Spill& S, int64_t ws) {
    for (int k = 0; k < 2; k++)
        if (e->s[k].when != ABSENT && e->s[k].ws == ws) e->s[k].when = ABSENT;
    SpillEntry* sp = spill_lookup(S, e->key, e->nspill, ws);
    if (sp) sp->when = ABSENT;
}

}  // namespace rl
