// rl_semantics.h -- the per-request decision rules of the reference limiter,
// restated as __host__ __device__ code for the CDNA4 kernels.
//
// Reference (paths relative to the reference repo):
//   Go side     internal/ratelimiter/tokenbucket.go:90-133,155-193
//               internal/ratelimiter/slidingwindow.go:68-122,150-197
//               internal/ratelimiter/fixedwindow.go:65-115,139-163
//   Redis side  the Lua scripts tokenbucket.go:23-52, slidingwindow.go:22-30,
//               fixedwindow.go:21-27, with Redis 7 keyspace rules.
// Build with -ffp-contract=off: Go/amd64 and Lua round every op separately.
#pragma once

#include <stdint.h>

#include "rl_q14.h"

namespace rl {

constexpr int64_t NS_PER_S = 1000000000LL;
constexpr int64_t ABSENT = INT64_MIN;       // `when` of a key that does not exist
constexpr int64_t NO_EXPIRY = INT64_MAX;    // `when` of a key without TTL
constexpr uint64_t EMPTY_KEY = ~0ULL;       // table slot never used

enum : int32_t { ALG_TOKEN_BUCKET = 1, ALG_SLIDING_WINDOW = 2, ALG_FIXED_WINDOW = 3 };
enum : uint8_t { DEC_DENIED = 0, DEC_ALLOWED = 1, DEC_ERROR = 2, DEC_INVALID = 3 };
enum : int32_t { PROFILE_REDIS7 = 0, PROFILE_MINIREDIS = 1 };

// error-flag bits raised by kernels (sticky per engine)
enum : uint32_t {
    EF_TABLE_FULL = 1u,       // open-addressing table has no free slot
    EF_ORDER = 2u,            // reserved (no longer raised: window keys spill, rl_window.h)
    EF_LOOKBACK = 4u,         // radix-sort look-back spin bound hit
    EF_BAD_KEY = 8u,          // key id equal to the reserved empty marker
    EF_INTERNAL = 16u,        // cooperative replay invariant violated (never expected)
    EF_ROUTED_OVER = 32u,     // a routed batch's device count exceeded m_max (requests past it undecided)
};

// Per-config constants, precomputed on the host exactly as Go computes them.
struct CfgDev {
    int32_t alg;
    int32_t pad;
    int64_t limit;       // Config.Limit
    int64_t window;      // Config.Window (ns)
    double limit_d;      // float64(Limit) == Lua `capacity`
    double rate;         // calculateRefillRate(): float64(L) / W.Seconds()
    int64_t ttl_tb;      // int64(W.Seconds()*2)  (tokenbucket.go:170)
    int64_t ttl_c;       // int64(W.Seconds())    (fixedwindow.go:151, slidingwindow.go:161; also the pws delta :75)
    int64_t ttl_p;       // int64(W.Seconds()*2)  (slidingwindow.go:162)
    int64_t off_mod;     // (62135596800 s) mod W, for Truncate relative to year 1
    int64_t tb_full_ns;  // time.Duration(float64(L)/rate * 1e9) (tokenbucket.go:163-164)
    double inv_rate;     // float64(1) / rate: tokensNeeded / refillRate for tokensNeeded == 1
};

// Go's int64(float64) on amd64 (CVTTSD2SQ): truncate; NaN / out of range -> MinInt64.
// Redis's (long long) cast of a Lua number compiles to the same instruction.
RL_HD inline int64_t go_f2i(double x) {
    if (!(x < 9223372036854775808.0) || !(x >= -9223372036854775808.0)) return INT64_MIN;
    return (int64_t)x;
}

// Go's time.Duration.Seconds() (time/time.go): float64(d/Second) + float64(d%Second)/1e9
inline double go_duration_seconds(int64_t d) {
    int64_t sec = d / NS_PER_S, nsec = d % NS_PER_S;
    return (double)sec + (double)nsec / 1e9;
}

// Host-side construction of the per-config constants, exactly as Go computes
// them at each call (the values depend on the config only).
inline CfgDev make_cfg(int32_t alg, int64_t limit, int64_t window) {
    CfgDev c{};
    c.alg = alg;
    c.limit = limit;
    c.window = window;
    c.limit_d = (double)limit;
    double wsec = go_duration_seconds(window);
    c.rate = (double)limit / wsec;                 // tokenbucket.go:156
    c.ttl_tb = go_f2i(wsec * 2);                   // tokenbucket.go:170
    c.ttl_c = go_f2i(wsec);                        // fixedwindow.go:151, slidingwindow.go:75,161
    c.ttl_p = go_f2i(wsec * 2);                    // slidingwindow.go:162
    __int128 off = (__int128)62135596800LL * NS_PER_S;  // Go unixToInternal, in ns
    c.off_mod = (int64_t)(off % window);
    c.tb_full_ns = go_f2i((double)limit / c.rate * 1e9);  // tokenbucket.go:163-164
    c.inv_rate = 1.0 / c.rate;
    return c;
}

RL_HD inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
RL_HD inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
RL_HD inline int64_t wmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }

RL_HD inline int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
    return q;
}

// now.Truncate(W).Unix() (fixedwindow.go:72, slidingwindow.go:74); Truncate is
// relative to Jan 1 year 1, hence the precomputed off_mod.
// the window's start in Unix ns: time.Truncate(t, W) (relative to year 1)
RL_HD inline int64_t window_start_ns(int64_t t, const CfgDev& c) {
    int64_t tm = t % c.window;
    if (tm < 0) tm += c.window;
    int64_t r = tm + c.off_mod;
    if (r >= c.window) r -= c.window;
    return t - r;
}
RL_HD inline int64_t window_start(int64_t t, const CfgDev& c) {
    return floor_div(window_start_ns(t, c), NS_PER_S);
}

// Redis 7 keyIsExpired(): now > when.  miniredis: a key is gone once its
// remaining ttl <= 0 after FastForward, i.e. clock >= when.
RL_HD inline bool key_alive(int64_t when, int64_t s_ms, int32_t profile) {
    if (when == ABSENT) return false;
    if (when == NO_EXPIRY) return true;
    return profile == PROFILE_REDIS7 ? !(s_ms > when) : !(s_ms >= when);
}

// EXPIRE key ttl on an existing key: ttl <= 0 deletes it.
RL_HD inline int64_t expire_when(int64_t ttl, int64_t s_ms) {
    return ttl > 0 ? s_ms + ttl * 1000 : ABSENT;
}

RL_HD inline double lua_tostring_roundtrip(double x, int32_t profile) {
    return profile == PROFILE_REDIS7 ? rlq::q14(x) : x;
}

// ---------------------------------------------------------------------------
// Per-request outputs
// ---------------------------------------------------------------------------
struct Out {
    uint8_t decision;
    int64_t remaining;
    int64_t retry;
    int64_t reset_at;
    double tokens;
};

// calculateResetTime (tokenbucket.go:161-165) as Unix ns.
RL_HD inline int64_t tb_reset_at(double now, const CfgDev& c) {
    int64_t sec = go_f2i(now);
    int64_t nsec = go_f2i((now - (double)sec) * 1e9);
    return wadd(wadd(wmul(sec, NS_PER_S), nsec), c.tb_full_ns);
}

// ---------------------------------------------------------------------------
// Token bucket: one script execution (tokenbucket.go:23-52) plus the Go
// post-processing (tokenbucket.go:114-130).  State = the Redis hash
// {tokens, last_refill} (stored values, already string-round-tripped) + when.
// ---------------------------------------------------------------------------
struct TbState {
    double tok;
    double last;
    int64_t when;
};

RL_HD inline Out tb_step(TbState& st, int64_t t, int64_t n, int64_t s_ms, const CfgDev& c,
                         int32_t profile) {
    Out o;
    double now = (double)t / 1e9;
    double capacity = c.limit_d;
    double requested = (double)n;
    bool alive = key_alive(st.when, s_ms, profile);
    double tokens = alive ? st.tok : capacity;
    double last = alive ? st.last : now;
    double elapsed = now - last;
    double add = elapsed * c.rate;
    double sum = tokens + add;
    tokens = (sum < capacity) ? sum : capacity;           // math.min(capacity, sum)
    bool allowed = false;
    if (tokens >= requested) { tokens = tokens - requested; allowed = true; }
    // HMSET tokens tostring(tokens) last_refill tostring(now); EXPIRE key ttl
    st.tok = lua_tostring_roundtrip(tokens, profile);
    st.last = lua_tostring_roundtrip(now, profile);
    st.when = expire_when(c.ttl_tb, s_ms);
    int64_t rem = go_f2i(floor(tokens));                  // {allowed, math.floor(tokens)}
    o.tokens = tokens;
    o.decision = allowed ? DEC_ALLOWED : DEC_DENIED;
    o.remaining = rem;
    o.reset_at = tb_reset_at(now, c);
    o.retry = 0;
    if (!allowed) {
        int64_t need = wsub(n, rem);
        double w = need == 1 ? c.inv_rate : (double)need / c.rate;   // tokensNeeded / refillRate
        int64_t d = go_f2i(w * 1e9);
        o.retry = d < 0 ? 0 : d;
    }
    return o;
}

// ---------------------------------------------------------------------------
// Window counters: one Redis string key "B:ws" per (user key, window start)
// (fixedwindow.go:75, slidingwindow.go:78-79).  The keyspace holding them is
// in rl_window.h (a 2-slot entry per user key + a spill table).
// ---------------------------------------------------------------------------
struct WinSlot {
    int64_t ws;
    int64_t cnt;
    int64_t when;
};

RL_HD inline int64_t until_reset(int64_t reset_at, int64_t t) {
    int64_t d = wsub(reset_at, t);
    return d < 0 ? 0 : d;
}

// INCRBY overflow rule (t_string.c incrDecrCommand)
RL_HD inline bool incr_overflows(int64_t old, int64_t n) {
    return (n < 0 && old < 0 && n < (INT64_MIN - old)) || (n > 0 && old > 0 && n > (INT64_MAX - old));
}

}  // namespace rl
