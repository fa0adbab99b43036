/*
 * rl_oracle.h -- CPU restatement of the reference Go + Redis decision path.
 *
 * TEST INFRASTRUCTURE ONLY.  This oracle is the parity checker for the HIP
 * engine in distributed-rate-limiter_amd/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * It restates, single-threaded and in plain C, what one reference decision does
 * end to end (all paths relative to the reference repo):
 *   - Go side:   internal/ratelimiter/tokenbucket.go:90-133,155-193
 *                internal/ratelimiter/slidingwindow.go:68-122,150-197
 *                internal/ratelimiter/fixedwindow.go:65-115,139-163
 *                internal/ratelimiter/config.go:16-87 (Duration math)
 *   - Redis side: the three embedded Lua scripts
 *                tokenbucket.go:23-52, slidingwindow.go:22-30, fixedwindow.go:21-27
 *     executed with Redis 7 keyspace semantics (lazy expiry `now_ms > when`,
 *     EXPIRE on a missing key is a no-op, EXPIRE with ttl <= 0 deletes, INCRBY
 *     keeps the TTL and errors on int64 overflow) and Lua 5.1 numbers
 *     (doubles; tostring = sprintf("%.14g"), tonumber = strtod).
 *
 * Profiles:
 *   RLO_PROFILE_REDIS7     canonical: real Redis 7.x (Lua tostring "%.14g",
 *                          strict expiry `s_ms > when`, INCRBY overflow error)
 *   RLO_PROFILE_MINIREDIS  what the reference's own tests run on (miniredis
 *                          v2.36.1 + gopher-lua v1.1.1): shortest-repr
 *                          tostring (identity on doubles), TTL clock = the
 *                          FastForward accumulator, key gone once ttl <= 0
 *                          (`s_ms >= when`).
 *
 * Keys are identified by a 64-bit id standing for the formatted base key
 * FormatKey(key) = prefix + ":" + key (config.go:81-87).  Window keys are the
 * pair (id, windowStart) standing for fmt.Sprintf("%s:%d", base, ws)
 * (fixedwindow.go:139-141, slidingwindow.go:150-152).  Formatting is
 * injective, so this keyspace is isomorphic to the reference's string keys.
 */
#ifndef RL_ORACLE_H
#define RL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* algorithm codes (shared numbering with include/rl_engine.h) */
#define RLO_ALG_TOKEN_BUCKET   1
#define RLO_ALG_SLIDING_WINDOW 2
#define RLO_ALG_FIXED_WINDOW   3

#define RLO_PROFILE_REDIS7    0
#define RLO_PROFILE_MINIREDIS 1

/* per-request decision codes (shared numbering with include/rl_engine.h) */
#define RLO_DENIED  0
#define RLO_ALLOWED 1
#define RLO_ERROR   2 /* the script raised (INCRBY overflow): Go sees err != nil */
#define RLO_INVALID 3 /* n <= 0 or unknown cfg: never reaches Redis (ErrInvalidN) */

typedef struct rlo_sim rlo_sim;

rlo_sim* rlo_create(int profile);
void     rlo_destroy(rlo_sim* s);
/* returns cfg id >= 0, or -1 if the config fails Validate (config.go:16-50) */
int      rlo_add_config(rlo_sim* s, int alg, int64_t limit, int64_t window_ns);

/* One trace of m requests in arrival order.  server_ms may be NULL: then the
 * Redis clock is floor(ts/1e6) (client and server share one clock).
 * tokens (nullable) receives, for token-bucket requests, the Lua `tokens`
 * variable at the end of the script (before tostring); NaN otherwise. */
void rlo_decide(rlo_sim* s, size_t m, const uint64_t* key, const int64_t* ts,
                const int64_t* n, const uint32_t* cfg, const int64_t* server_ms,
                uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                int64_t* reset_at_ns, double* tokens);

/* rlo_decide request by request, each call timed: call_ns[i] (the per-call
 * latency of the restated path, for bench.py's cpu_baseline leg) */
void rlo_decide_timed(rlo_sim* s, size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n,
                      const uint32_t* cfg, uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                      int64_t* reset_at_ns, int64_t* call_ns);

/* Reset(ctx, key) at time ts (tokenbucket.go:136-144, slidingwindow.go:125-139,
 * fixedwindow.go:118-128): DEL of the keys the limiter would touch at ts. */
void rlo_reset(rlo_sim* s, uint32_t cfg, uint64_t key, int64_t ts, int64_t server_ms);

/* exposed pieces, pinned individually by the reference's unit tests */
double  rlo_duration_seconds(int64_t d_ns);                 /* Go Duration.Seconds */
int64_t rlo_go_f2i(double x);                               /* Go int64(float64), amd64 */
int64_t rlo_window_start(int64_t t_ns, int64_t w_ns);       /* Truncate(W).Unix() */
double  rlo_lua_tostring_roundtrip(double x, int profile);   /* tonumber(tostring(x)) */
double  rlo_sw_weighted(int64_t t_ns, int64_t ws, int64_t w_ns, int64_t prev, int64_t curr);
double  rlo_tb_refill_rate(int64_t limit, int64_t w_ns);
int64_t rlo_tb_reset_at(int64_t limit, int64_t w_ns, double now);
/* number of live keys in the simulated keyspace at server time s_ms */
size_t  rlo_live_keys(rlo_sim* s, int64_t s_ms);
/* the live keys themselves: (id, kind 0 hash / 1 window, ws), up to cap;
 * returns how many are live */
size_t  rlo_keys(rlo_sim* s, int64_t s_ms, uint64_t* id, uint8_t* kind, int64_t* ws, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
