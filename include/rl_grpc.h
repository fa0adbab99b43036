/*
 * rl_grpc.h -- the native gRPC front end of the rate limiter service
 * (api/proto/ratelimiter.proto, api/proto/health.proto) over the request
 * coalescer (include/rl_coalescer.h).
 *
 * The reference plans `service RateLimiter { Allow; AllowN; Reset }` with a
 * health check, graceful shutdown and per-tenant limiter instances
 * (docs/ARCHITECTURE.md:287-304, cmd/server/main.go:13-17); its single Redis
 * decides about 35k token-bucket requests/s (docs/ARCHITECTURE.md:440).  This
 * server speaks gRPC over HTTP/2 cleartext (h2c) from `io_threads` event-loop
 * threads (epoll, one SO_REUSEPORT listener each), decodes the protobuf
 * messages itself and hands every request to the coalescer as it arrives: the
 * coalescer turns whatever is pending into the next GPU batch, so one engine
 * launch serves the RPCs of every connection.  Completions come back through
 * the coalescer's notification hook to the thread owning the RPC (eventfd);
 * no thread blocks per RPC.
 *
 * Semantics per RPC are the Go limiter's (internal/ratelimiter), as the
 * Python handlers in python/rl_server.py state them:
 *   - time.Now() is read once per RPC on arrival (tokenbucket.go:97,
 *     slidingwindow.go:73, fixedwindow.go:71);
 *   - n <= 0: INVALID_ARGUMENT "invalid n: must be greater than 0"
 *     (errors.go:16); an unknown limiter: NOT_FOUND;
 *   - key ids: XXH64(FormatKey(prefix, key)) with seed 0 (rl_hash_keys_host),
 *     the formatted key being the only namespace as in Redis (config.go:81-87),
 *     or one namespace per limiter (rl_cfg_seed) with `isolate`;
 *   - the grpc-timeout header is the submission's deadline (interface.go:75):
 *     a request not launched when it passes is never applied; an expired or
 *     cancelled request (client RST_STREAM) takes the error branch;
 *   - an engine error or an expired context: the fail-open result
 *     {Allowed, Limit, 0, 0, ResetAt} (tokenbucket.go:100-112 and twins) or,
 *     fail-closed, UNAVAILABLE / DEADLINE_EXCEEDED / CANCELLED
 *     "failed to check rate limit: <err>";
 *   - AllowBatch: one submission for the valid requests, per-request errors in
 *     AllowResponse.error;
 *   - Reset: a DEL ordered in the coalescer's sequence (rl_coalescer_reset);
 *   - Health/Check: SERVING until shutdown begins, then NOT_SERVING.
 */
#ifndef RL_GRPC_H
#define RL_GRPC_H

#include <stddef.h>
#include <stdint.h>

#include "rl_coalescer.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rl_grpc_server rl_grpc_server;

/* one configured limiter (a reference Config, interface.go:46-70), already
 * registered with the engine as cfg_id */
typedef struct rl_grpc_limiter {
    uint32_t struct_size;    /* sizeof(rl_grpc_limiter) */
    uint32_t cfg_id;
    const char* name;        /* AllowRequest.limiter */
    int32_t algorithm;       /* RL_ALG_* */
    int32_t fail_open;       /* FailOpen (interface.go:65-69) */
    int64_t limit;
    int64_t window_ns;
    const char* prefix;      /* Config.Prefix; "" -> "ratelimit" (config.go:62-64) */
} rl_grpc_limiter;

typedef struct rl_grpc_opts {
    uint32_t struct_size;    /* sizeof(rl_grpc_opts) */
    uint32_t io_threads;     /* event loops (0 = 4) */
    const char* host;        /* listen address (NULL = "127.0.0.1") */
    int32_t port;            /* 0 = any free port (rl_grpc_server_port) */
    int32_t isolate;         /* one key namespace per limiter */
    /* test clock: when clock_step_ns != 0, the k-th time.Now() read (k = 1,
     * 2, ...) returns clock_start_ns + k * clock_step_ns instead of the real
     * time (deterministic decisions for the parity tests) */
    int64_t clock_start_ns;
    int64_t clock_step_ns;
} rl_grpc_opts;

typedef struct rl_grpc_stats {
    uint32_t struct_size;    /* sizeof(rl_grpc_stats) */
    uint32_t pad_;
    uint64_t connections;    /* accepted */
    uint64_t rpcs;           /* completed with a response */
    uint64_t decisions;      /* requests submitted to the coalescer */
    uint64_t errors;         /* responses with a non-OK grpc-status */
    uint64_t cancelled;      /* RPCs the client reset before their response */
} rl_grpc_stats;

/* Start serving on the coalescer (which must outlive the server).  The
 * limiters are copied.  *out gets the server; it listens when this returns. */
int rl_grpc_server_start(rl_coalescer* c, const rl_grpc_limiter* limiters, size_t n_limiters,
                         const rl_grpc_opts* opts, rl_grpc_server** out);
/* the bound TCP port */
int rl_grpc_server_port(rl_grpc_server* s);
/* graceful shutdown: health NOT_SERVING, stop accepting, answer the RPCs in
 * flight (at most grace_ns), close every connection, join the threads */
int rl_grpc_server_shutdown(rl_grpc_server* s, int64_t grace_ns);
int rl_grpc_server_destroy(rl_grpc_server* s);
int rl_grpc_server_get_stats(rl_grpc_server* s, rl_grpc_stats* out);

#ifdef __cplusplus
}
#endif
#endif /* RL_GRPC_H */
