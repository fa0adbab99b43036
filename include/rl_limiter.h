/*
 * rl_limiter.h -- C-ABI of the host mirror of the reference's Go API
 * (internal/ratelimiter: Config, RateLimiter.Allow/AllowN/Reset/Close), built
 * over include/rl_engine.h.  This is what a non-C++ host (Go via cgo, Python
 * via ctypes) binds when it wants the reference's per-call semantics instead
 * of raw batches; see INTEGRATION.md.
 *
 * Reference anchors: interface.go:26-145, config.go:16-87, errors.go:5-20,
 * tokenbucket.go:63-152, slidingwindow.go:41-147, fixedwindow.go:38-136.
 */
#ifndef RL_LIMITER_H
#define RL_LIMITER_H

#include <stddef.h>
#include <stdint.h>

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* return codes: which Go error value the reference would return */
#define RLL_OK           0  /* err == nil, *out is the Result */
#define RLL_ERR_INVALID_N 1  /* ErrInvalidN, Result nil (tokenbucket.go:91-93) */
#define RLL_ERR_FAILED   2  /* fmt.Errorf("failed to check rate limit: %w"), Result nil */
#define RLL_ERR_CONFIG   3  /* constructor error ("config cannot be nil", "invalid config: ...") */
#define RLL_ERR_RESET    4  /* fmt.Errorf("failed to reset rate limit: %w") */
#define RLL_ERR_ARG      5  /* bad C argument */

#define RLL_NOW_WALL   INT64_MIN  /* now_ns: read the wall clock (time.Now()) */
#define RLL_SMS_DEFAULT INT64_MIN /* server_ms: Redis clock = floor(now_ns / 1e6) */

typedef struct rll_engine rll_engine;    /* rl_engine + key interner */
typedef struct rll_limiter rll_limiter;

typedef struct rll_result {
    uint8_t allowed;
    int64_t limit;
    int64_t remaining;
    int64_t retry_after_ns;
    int64_t reset_at_ns;
} rll_result;

#define RLL_TIME_ZERO INT64_MIN   /* reset_at_ns of time.Time{} */

/* Result constructors (result.go:5-50): NewAllowedResult, NewDeniedResult,
 * NewFailOpenResult, NewFailClosedResult */
int rll_new_allowed_result(int64_t limit, int64_t remaining, int64_t reset_at_ns, rll_result* out);
int rll_new_denied_result(int64_t limit, int64_t retry_after_ns, int64_t reset_at_ns, rll_result* out);
int rll_new_fail_open_result(rll_result* out);
int rll_new_fail_closed_result(rll_result* out);

int rll_engine_new(const rl_opts* opts, rll_engine** out, char* err, size_t errlen);
int rll_engine_free(rll_engine* e);
rl_engine* rll_engine_raw(rll_engine* e);
/* test hook (miniredis FastForward replay): fixed Redis clock for every call;
 * RLL_SMS_DEFAULT restores the default */
int rll_engine_set_server_ms(rll_engine* e, int64_t server_ms);

/* Redis KEYS (what the reference's tests read with miniredis Keys()): the
 * live keys' names at Redis clock server_ms, sorted, one per line
 * ("prefix:key" for a token bucket, "prefix:key:ws" for a window counter).
 * Writes what fits in buf (NUL-terminated); returns the full length, or a
 * negative RLL_ERR_* code. */
int rll_keys(rll_engine* e, int64_t server_ms, char* buf, size_t len);

/* Config.Validate() (config.go:16-50); algorithm NULL means a nil *Config */
int rll_config_validate(const char* algorithm, int64_t limit, int64_t window_ns, char* err, size_t errlen);
/* Config.FormatKey(key) (config.go:81-87) for a config with this Prefix
 * (prefix NULL means a nil *Config); returns the length written */
int rll_format_key(const char* prefix, const char* key, char* out, size_t len);
/* Go time.Duration.String() */
int rll_duration_string(int64_t d, char* out, size_t len);

/* New{TokenBucket,SlidingWindow,FixedWindow} by algorithm name.  prefix NULL
 * == "" (defaults to "ratelimit" via WithDefaults).  config_nil != 0 models a
 * nil *Config. */
int rll_new(rll_engine* e, const char* algorithm, int64_t limit, int64_t window_ns,
            const char* prefix, int fail_open, int config_nil, rll_limiter** out, char* err,
            size_t errlen);

/* AllowN(ctx, key, n); Allow == n = 1.  ctx_cancelled != 0 models a cancelled
 * context. */
int rll_allow_n(rll_limiter* l, const char* key, size_t keylen, int64_t n, int64_t now_ns,
                int ctx_cancelled, rll_result* out, char* err, size_t errlen);

/* BatchAllow: m requests in one engine launch; per-request code in codes[] */
int rll_allow_batch(rll_limiter* l, size_t m, const char* const* keys, const size_t* keylens,
                    const int64_t* n, const int64_t* now_ns, rll_result* out, int32_t* codes);

/* Observability decorators (docs/ADR/003-decorator-pattern-for-observability.md):
 * wrap the limiter in place; every later call goes through them.
 * rll_metrics_expose writes the Prometheus text exposition
 * (rate_limiter_requests_total{algorithm,allowed,error},
 * rate_limiter_decision_seconds histogram) and returns its full length. */
int rll_add_metrics(rll_limiter* l);
int rll_metrics_expose(rll_limiter* l, char* buf, size_t len);
/* LoggingDecorator: records go to a bounded in-library queue that the
 * caller drains (pull style -- the library never calls back into Go; a full
 * queue drops its oldest record).  rll_log_drain writes whole records as
 * text lines "<level>\t<msg>\t<fields>\n" (level: 0 debug, 1 info, 2 warn,
 * 3 error; fields "k=v k=v") while they fit in buf (NUL-terminated), removes
 * them from the queue and returns how many it wrote; *dropped (nullable) =
 * records lost to overflow so far. */
int rll_add_logging(rll_limiter* l, size_t capacity);
int rll_log_drain(rll_limiter* l, char* buf, size_t len, uint64_t* dropped);

int rll_reset(rll_limiter* l, const char* key, size_t keylen, int64_t now_ns, char* err, size_t errlen);
int rll_close(rll_limiter* l);   /* Close(): later calls take the storage-error path */
int rll_free(rll_limiter* l);

#ifdef __cplusplus
}
#endif
#endif
