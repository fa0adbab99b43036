/*
 * rl_oracle.c -- CPU restatement of the reference Go + Redis decision path.
 * TEST INFRASTRUCTURE ONLY (see rl_oracle.h).  Built with -ffp-contract=off:
 * Go on amd64 (GOAMD64=v1) and the Lua 5.1 VM in Redis never fuse a*b+c.
 */
#include "rl_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NS_PER_S 1000000000LL
/* seconds from Jan 1 year 1 to the Unix epoch (Go's unixToInternal) */
#define GO_UNIX_TO_INTERNAL 62135596800LL

/* ------------------------------------------------------------------------- */
/* Go arithmetic                                                              */
/* ------------------------------------------------------------------------- */

/* time.Duration.Seconds() (Go 1.25 time/time.go):
 *   sec := d / Second; nsec := d % Second
 *   return float64(sec) + float64(nsec)/1e9 */
double rlo_duration_seconds(int64_t d) {
    int64_t sec = d / NS_PER_S;
    int64_t nsec = d % NS_PER_S;
    return (double)sec + (double)nsec / 1e9;
}

/* int64(x) for float64 x as compiled by Go on amd64 (CVTTSD2SQ): truncation,
 * and 0x8000000000000000 for NaN or out-of-range.  Redis's (long long) cast of
 * a Lua number compiles to the same instruction. */
int64_t rlo_go_f2i(double x) {
    if (!(x < 9223372036854775808.0) || !(x >= -9223372036854775808.0))
        return INT64_MIN;
    return (int64_t)x;
}

static int64_t floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
    return q;
}

/* now.Truncate(W).Unix() (fixedwindow.go:72, slidingwindow.go:74).
 * Go's Truncate rounds down relative to the zero Time (Jan 1 year 1 UTC), not
 * the Unix epoch; Unix() then drops the sub-second part (floor). */
int64_t rlo_window_start(int64_t t, int64_t w) {
    __int128 abs_ns = (__int128)t + (__int128)GO_UNIX_TO_INTERNAL * NS_PER_S;
    __int128 r = abs_ns % w;
    if (r < 0) r += w;
    int64_t trunc_ns = (int64_t)((__int128)t - r);
    return floor_div(trunc_ns, NS_PER_S);
}

/* calculateWeightedCount (slidingwindow.go:190-197) */
double rlo_sw_weighted(int64_t t, int64_t ws, int64_t w, int64_t prev, int64_t curr) {
    int64_t elapsed = (int64_t)((uint64_t)t - (uint64_t)ws * (uint64_t)NS_PER_S);
    double progress = (double)elapsed / (double)w;
    double a = (double)prev * (1.0 - progress);
    return a + (double)curr;
}

/* calculateRefillRate (tokenbucket.go:155-157) */
double rlo_tb_refill_rate(int64_t limit, int64_t w) {
    return (double)limit / rlo_duration_seconds(w);
}

/* calculateResetTime (tokenbucket.go:161-165), as Unix nanoseconds:
 * time.Unix(int64(now), int64((now-float64(int64(now)))*1e9)).Add(
 *     time.Duration(secondsToFull * float64(time.Second))) */
int64_t rlo_tb_reset_at(int64_t limit, int64_t w, double now) {
    double rate = rlo_tb_refill_rate(limit, w);
    double seconds_to_full = (double)limit / rate;
    int64_t sec = rlo_go_f2i(now);
    int64_t nsec = rlo_go_f2i((now - (double)sec) * 1e9);
    int64_t d = rlo_go_f2i(seconds_to_full * 1e9);
    uint64_t r = (uint64_t)sec * (uint64_t)NS_PER_S + (uint64_t)nsec + (uint64_t)d;
    return (int64_t)r;
}

/* ------------------------------------------------------------------------- */
/* Lua number <-> string                                                      */
/* ------------------------------------------------------------------------- */

/* Redis 7's Lua 5.1: tostring(x) = sprintf("%.14g") (LUAI_NUMFFORMAT),
 * tonumber(s) = strtod.  miniredis/gopher-lua: tostring is Go's shortest
 * round-trip repr, so the round trip is the identity. */
static void lua_tostring(double x, int profile, char* buf, size_t len) {
    if (profile == RLO_PROFILE_REDIS7) {
        snprintf(buf, len, "%.14g", x);
    } else {
        /* shortest repr that round-trips, as strconv.FormatFloat(x,'g',-1,64) */
        for (int p = 1; p <= 17; p++) {
            snprintf(buf, len, "%.*g", p, x);
            if (strtod(buf, NULL) == x) return;
        }
    }
}

static double lua_tonumber(const char* s) { return strtod(s, NULL); }

double rlo_lua_tostring_roundtrip(double x, int profile) {
    char buf[64];
    lua_tostring(x, profile, buf, sizeof buf);
    return lua_tonumber(buf);
}

/* ------------------------------------------------------------------------- */
/* Simulated Redis keyspace                                                   */
/* ------------------------------------------------------------------------- */

enum { KIND_HASH = 0, KIND_WINDOW = 1 };

typedef struct {
    uint8_t used;       /* slot in the map is in use (the key may be deleted) */
    uint8_t present;    /* the Redis key exists */
    uint8_t kind;
    uint8_t has_exp;
    uint64_t id;
    int64_t ws;
    int64_t when;       /* absolute expiry, server ms */
    int64_t count;      /* string counter value (window keys) */
    char tokens[48];    /* hash field strings (token-bucket keys) */
    char last_refill[48];
} ent_t;

typedef struct {
    int alg;
    int64_t limit;
    int64_t window;
} cfg_t;

struct rlo_sim {
    int profile;
    ent_t* tab;
    size_t cap, used;
    cfg_t* cfgs;
    int ncfg, capcfg;
};

static uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33; return x;
}
static uint64_t key_hash(int kind, uint64_t id, int64_t ws) {
    return mix64(id ^ mix64((uint64_t)ws + 0x9e3779b97f4a7c15ULL * (uint64_t)(kind + 1)));
}

static void tab_grow(rlo_sim* s);

static ent_t* tab_find(rlo_sim* s, int kind, uint64_t id, int64_t ws, int create) {
    if (create && (s->used + 1) * 2 > s->cap) tab_grow(s);
    size_t mask = s->cap - 1, i = key_hash(kind, id, ws) & mask;
    for (;;) {
        ent_t* e = &s->tab[i];
        if (!e->used) {
            if (!create) return NULL;
            memset(e, 0, sizeof *e);
            e->used = 1; e->kind = (uint8_t)kind; e->id = id; e->ws = ws;
            s->used++;
            return e;
        }
        if (e->kind == kind && e->id == id && e->ws == ws) return e;
        i = (i + 1) & mask;
    }
}

static void tab_grow(rlo_sim* s) {
    size_t ocap = s->cap;
    ent_t* old = s->tab;
    s->cap = ocap ? ocap * 2 : 1024;
    s->tab = (ent_t*)calloc(s->cap, sizeof(ent_t));
    s->used = 0;
    for (size_t i = 0; i < ocap; i++) {
        if (!old[i].used) continue;
        ent_t* e = tab_find(s, old[i].kind, old[i].id, old[i].ws, 1);
        *e = old[i];
    }
    free(old);
}

/* Redis 7 keyIsExpired: now > when.  miniredis: FastForward deletes a key once
 * its remaining ttl <= 0, i.e. clock >= when. */
static int is_expired(const rlo_sim* s, const ent_t* e, int64_t s_ms) {
    if (!e->has_exp) return 0;
    return s->profile == RLO_PROFILE_REDIS7 ? (s_ms > e->when) : (s_ms >= e->when);
}

/* lookupKey with lazy expiry: returns the live key or NULL */
static ent_t* lookup(rlo_sim* s, int kind, uint64_t id, int64_t ws, int64_t s_ms) {
    ent_t* e = tab_find(s, kind, id, ws, 0);
    if (!e || !e->present) return NULL;
    if (is_expired(s, e, s_ms)) { e->present = 0; return NULL; }
    return e;
}

/* EXPIRE key ttl (seconds): no-op on a missing key; ttl <= 0 deletes
 * (Redis: when = now + ttl*1000 <= now => delete; miniredis: ttl <= 0 => del). */
static void cmd_expire(rlo_sim* s, int kind, uint64_t id, int64_t ws, int64_t ttl, int64_t s_ms) {
    ent_t* e = lookup(s, kind, id, ws, s_ms);
    if (!e) return;
    if (ttl <= 0) { e->present = 0; return; }
    e->has_exp = 1;
    e->when = s_ms + ttl * 1000;
}

/* INCRBY key n; returns 0 on success, -1 on the overflow error
 * ("increment or decrement would overflow", t_string.c incrDecrCommand). */
static int cmd_incrby(rlo_sim* s, uint64_t id, int64_t ws, int64_t n, int64_t s_ms, int64_t* out) {
    ent_t* e = lookup(s, KIND_WINDOW, id, ws, s_ms);
    int64_t old = e ? e->count : 0;
    /* both Redis 7 and miniredis v2.36 refuse an overflowing INCRBY */
    if ((n < 0 && old < 0 && n < (INT64_MIN - old)) ||
        (n > 0 && old > 0 && n > (INT64_MAX - old)))
        return -1;
    int64_t v = old + n;
    if (!e) {
        e = tab_find(s, KIND_WINDOW, id, ws, 1);
        e->present = 1;
        e->has_exp = 0; /* a freshly created key has no TTL */
    }
    e->count = v;
    *out = v;
    return 0;
}

static void cmd_del(rlo_sim* s, int kind, uint64_t id, int64_t ws) {
    ent_t* e = tab_find(s, kind, id, ws, 0);
    if (e) e->present = 0;
}

/* ------------------------------------------------------------------------- */
/* public API                                                                 */
/* ------------------------------------------------------------------------- */

rlo_sim* rlo_create(int profile) {
    rlo_sim* s = (rlo_sim*)calloc(1, sizeof *s);
    s->profile = profile;
    tab_grow(s);
    return s;
}

void rlo_destroy(rlo_sim* s) {
    if (!s) return;
    free(s->tab);
    free(s->cfgs);
    free(s);
}

int rlo_add_config(rlo_sim* s, int alg, int64_t limit, int64_t window) {
    /* Validate (config.go:16-50) */
    if (alg < RLO_ALG_TOKEN_BUCKET || alg > RLO_ALG_FIXED_WINDOW) return -1;
    if (limit <= 0 || window <= 0) return -1;
    if (window < 1000000LL || window > 365LL * 24 * 3600 * NS_PER_S) return -1;
    if (s->ncfg == s->capcfg) {
        s->capcfg = s->capcfg ? s->capcfg * 2 : 8;
        s->cfgs = (cfg_t*)realloc(s->cfgs, sizeof(cfg_t) * (size_t)s->capcfg);
    }
    s->cfgs[s->ncfg].alg = alg;
    s->cfgs[s->ncfg].limit = limit;
    s->cfgs[s->ncfg].window = window;
    return s->ncfg++;
}

typedef struct {
    uint8_t decision;
    int64_t remaining, retry, reset_at;
    double tokens;
} res_t;

/* tokenBucketLimiter.AllowN (tokenbucket.go:90-133) + tokenBucketScript (:23-52) */
static res_t tb_allow(rlo_sim* s, const cfg_t* c, uint64_t id, int64_t t, int64_t n, int64_t s_ms) {
    res_t r;
    double rate = rlo_tb_refill_rate(c->limit, c->window);
    double now = (double)t / 1e9;
    int64_t ttl = rlo_go_f2i(rlo_duration_seconds(c->window) * 2);

    /* ---- Lua (Redis side); ARGV round-trips exactly through go-redis ---- */
    double capacity = (double)c->limit;
    double requested = (double)n;
    double tokens, last_refill;
    ent_t* e = lookup(s, KIND_HASH, id, 0, s_ms);
    if (e) {
        tokens = lua_tonumber(e->tokens);
        last_refill = lua_tonumber(e->last_refill);
    } else {
        tokens = capacity;
        last_refill = now;
    }
    double elapsed = now - last_refill;
    double tokens_to_add = elapsed * rate;
    double sum = tokens + tokens_to_add;
    tokens = (sum < capacity) ? sum : capacity; /* math.min(capacity, sum) */
    int allowed = 0;
    if (tokens >= requested) {
        tokens = tokens - requested;
        allowed = 1;
    }
    /* HMSET (creates the key if needed, keeps any TTL) */
    if (!e) {
        e = tab_find(s, KIND_HASH, id, 0, 1);
        e->present = 1;
        e->has_exp = 0;
    }
    lua_tostring(tokens, s->profile, e->tokens, sizeof e->tokens);
    lua_tostring(now, s->profile, e->last_refill, sizeof e->last_refill);
    cmd_expire(s, KIND_HASH, id, 0, ttl, s_ms);
    int64_t rem = rlo_go_f2i(floor(tokens)); /* Lua number -> integer reply */

    /* ---- Go side ---- */
    r.tokens = tokens;
    r.decision = allowed ? RLO_ALLOWED : RLO_DENIED;
    r.remaining = rem;
    r.reset_at = rlo_tb_reset_at(c->limit, c->window, now);
    r.retry = 0;
    if (!allowed) {
        double needed = (double)(int64_t)((uint64_t)n - (uint64_t)rem);
        double wait_s = needed / rate;
        int64_t d = rlo_go_f2i(wait_s * 1e9);
        r.retry = d < 0 ? 0 : d;
    }
    return r;
}

static int64_t window_reset_at(int64_t ws, int64_t w) {
    return (int64_t)((uint64_t)ws * (uint64_t)NS_PER_S + (uint64_t)w);
}

static int64_t until(int64_t reset_at, int64_t t) {
    int64_t d = (int64_t)((uint64_t)reset_at - (uint64_t)t);
    return d < 0 ? 0 : d;
}

/* fixedWindowLimiter.AllowN (fixedwindow.go:65-115) + fixedWindowScript (:21-27) */
static res_t fw_allow(rlo_sim* s, const cfg_t* c, uint64_t id, int64_t t, int64_t n, int64_t s_ms) {
    res_t r;
    r.tokens = NAN;
    int64_t ws = rlo_window_start(t, c->window);
    int64_t ttl = rlo_go_f2i(rlo_duration_seconds(c->window));
    r.reset_at = window_reset_at(ws, c->window);
    int64_t cur;
    if (cmd_incrby(s, id, ws, n, s_ms, &cur) != 0) {
        r.decision = RLO_ERROR; r.remaining = 0; r.retry = 0;
        return r;
    }
    if ((double)cur == (double)n) cmd_expire(s, KIND_WINDOW, id, ws, ttl, s_ms);
    int64_t count = rlo_go_f2i((double)cur); /* `return current` (a Lua number) */
    int allowed = count <= c->limit;
    int64_t rem = (int64_t)((uint64_t)c->limit - (uint64_t)count);
    r.remaining = rem < 0 ? 0 : rem;
    r.decision = allowed ? RLO_ALLOWED : RLO_DENIED;
    r.retry = allowed ? 0 : until(r.reset_at, t);
    return r;
}

/* slidingWindowLimiter.AllowN (slidingwindow.go:68-122) + slidingWindowScript (:22-30) */
static res_t sw_allow(rlo_sim* s, const cfg_t* c, uint64_t id, int64_t t, int64_t n, int64_t s_ms) {
    res_t r;
    r.tokens = NAN;
    double wsec = rlo_duration_seconds(c->window);
    int64_t ws = rlo_window_start(t, c->window);
    int64_t pws = ws - rlo_go_f2i(wsec);
    int64_t ttl_c = rlo_go_f2i(wsec);
    int64_t ttl_p = rlo_go_f2i(wsec * 2);
    r.reset_at = window_reset_at(ws, c->window);

    ent_t* pe = lookup(s, KIND_WINDOW, id, pws, s_ms);
    double prev = pe ? (double)pe->count : 0.0; /* tonumber(GET or 0) */
    int64_t cur;
    if (cmd_incrby(s, id, ws, n, s_ms, &cur) != 0) {
        r.decision = RLO_ERROR; r.remaining = 0; r.retry = 0;
        return r;
    }
    if ((double)cur == (double)n) cmd_expire(s, KIND_WINDOW, id, ws, ttl_c, s_ms);
    cmd_expire(s, KIND_WINDOW, id, pws, ttl_p, s_ms);
    int64_t prev_i = rlo_go_f2i(prev);
    int64_t curr_i = rlo_go_f2i((double)cur);

    double weighted = rlo_sw_weighted(t, ws, c->window, prev_i, curr_i);
    int allowed = weighted <= (double)c->limit;
    int64_t rem = (int64_t)((uint64_t)c->limit - (uint64_t)rlo_go_f2i(weighted));
    r.remaining = rem < 0 ? 0 : rem;
    r.decision = allowed ? RLO_ALLOWED : RLO_DENIED;
    r.retry = allowed ? 0 : until(r.reset_at, t);
    return r;
}

void rlo_decide(rlo_sim* s, size_t m, const uint64_t* key, const int64_t* ts,
                const int64_t* n, const uint32_t* cfg, const int64_t* server_ms,
                uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                int64_t* reset_at_ns, double* tokens) {
    for (size_t i = 0; i < m; i++) {
        res_t r;
        int64_t s_ms = server_ms ? server_ms[i] : floor_div(ts[i], 1000000LL);
        if (cfg[i] >= (uint32_t)s->ncfg || n[i] <= 0) {
            r.decision = RLO_INVALID; r.remaining = 0; r.retry = 0; r.reset_at = 0; r.tokens = NAN;
        } else {
            const cfg_t* c = &s->cfgs[cfg[i]];
            switch (c->alg) {
            case RLO_ALG_TOKEN_BUCKET: r = tb_allow(s, c, key[i], ts[i], n[i], s_ms); break;
            case RLO_ALG_SLIDING_WINDOW: r = sw_allow(s, c, key[i], ts[i], n[i], s_ms); break;
            default: r = fw_allow(s, c, key[i], ts[i], n[i], s_ms); break;
            }
        }
        decision[i] = r.decision;
        remaining[i] = r.remaining;
        retry_after_ns[i] = r.retry;
        reset_at_ns[i] = r.reset_at;
        if (tokens) tokens[i] = r.tokens;
    }
}

void rlo_reset(rlo_sim* s, uint32_t cfg, uint64_t id, int64_t t, int64_t server_ms) {
    (void)server_ms; /* DEL ignores TTLs */
    if (cfg >= (uint32_t)s->ncfg) return;
    const cfg_t* c = &s->cfgs[cfg];
    if (c->alg == RLO_ALG_TOKEN_BUCKET) {
        cmd_del(s, KIND_HASH, id, 0);
        return;
    }
    int64_t ws = rlo_window_start(t, c->window);
    cmd_del(s, KIND_WINDOW, id, ws);
    if (c->alg == RLO_ALG_SLIDING_WINDOW)
        cmd_del(s, KIND_WINDOW, id, ws - rlo_go_f2i(rlo_duration_seconds(c->window)));
}

size_t rlo_live_keys(rlo_sim* s, int64_t s_ms) {
    size_t k = 0;
    for (size_t i = 0; i < s->cap; i++) {
        ent_t* e = &s->tab[i];
        if (e->used && e->present && !is_expired(s, e, s_ms)) k++;
    }
    return k;
}

/* Redis KEYS at server time s_ms: up to cap (id, kind, ws) triples of live
 * keys (miniredis Keys() in the reference's CustomPrefix tests); returns the
 * number of live keys */
size_t rlo_keys(rlo_sim* s, int64_t s_ms, uint64_t* id, uint8_t* kind, int64_t* ws, size_t cap) {
    size_t k = 0;
    for (size_t i = 0; i < s->cap; i++) {
        ent_t* e = &s->tab[i];
        if (!(e->used && e->present && !is_expired(s, e, s_ms))) continue;
        if (k < cap) {
            id[k] = e->id;
            kind[k] = e->kind;
            ws[k] = e->ws;
        }
        k++;
    }
    return k;
}

/* rlo_decide one request at a time with each call timed (CLOCK_MONOTONIC):
 * per-call latency of the restated store for the cpu_baseline leg (the
 * reference's per-call path: one EVAL per Allow).  call_ns[i] = the i-th
 * call's duration. */
void rlo_decide_timed(rlo_sim* s, size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n,
                      const uint32_t* cfg, uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                      int64_t* reset_at_ns, int64_t* call_ns) {
    for (size_t i = 0; i < m; i++) {
        struct timespec a, b;
        clock_gettime(CLOCK_MONOTONIC, &a);
        rlo_decide(s, 1, key + i, ts + i, n + i, cfg + i, NULL, decision + i, remaining + i, retry_after_ns + i,
                   reset_at_ns + i, NULL);
        clock_gettime(CLOCK_MONOTONIC, &b);
        call_ns[i] = (int64_t)(b.tv_sec - a.tv_sec) * 1000000000LL + (b.tv_nsec - a.tv_nsec);
    }
}
