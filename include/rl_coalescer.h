/*
 * rl_coalescer.h -- request coalescing in front of the decision engine.
 *
 * The reference decides one request per Redis round trip: every
 * Limiter.Allow/AllowN (tokenbucket.go:90-133, slidingwindow.go:68-122,
 * fixedwindow.go:65-115) is one client.Eval.  The north star's BatchAllow path
 * (internal/ratelimiter + cmd/server; the planned
 * gRPC service of docs/ARCHITECTURE.md:287-304) instead gathers concurrent
 * calls into GPU batches.  This is that coalescer, as a C-ABI a cgo layer can
 * call from many goroutines (no callbacks into the caller, no caller pointers
 * retained after a call returns).
 *
 * Policy: one submitter thread owns the engine.  Whenever fewer than
 * `max_in_flight` batches are on the GPU and requests are pending, it takes up
 * to `max_batch` of them (after lingering up to `linger_ns` for more when the
 * GPU is idle) and launches them as one batch.  Light load therefore sees
 * batches of one or a few requests and the latency of one launch sequence;
 * under heavy load the queue grows while the GPU works and batches grow to
 * `max_batch`.
 *
 * Order: every submitted request gets a global sequence number under the
 * queue lock; batches take requests in sequence order and the engine replays
 * batches in launch order, so the decisions are those of the reference
 * limiter receiving the requests one by one in sequence order.  A ticket is
 * the sequence number of the first request of its submission.
 */
#ifndef RL_COALESCER_H
#define RL_COALESCER_H

#include <stddef.h>
#include <stdint.h>

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RL_EAGAIN (-11)   /* queue full (rl_coalescer_opts.queue_cap) */
#define RL_ECLOSED (-32)  /* coalescer destroyed / shutting down */

typedef struct rl_coalescer rl_coalescer;

typedef struct rl_coalescer_opts {
    uint32_t max_batch;      /* requests per launch (<= the engine's max_batch); 0 = 65536 */
    uint32_t max_in_flight;  /* batches on the GPU at once, 1..3; 0 = 3 */
    int64_t  linger_ns;      /* with the GPU idle, wait this long for more requests (0 = launch at once) */
    uint64_t queue_cap;      /* pending requests beyond which submit returns RL_EAGAIN; 0 = 1 << 24 */
} rl_coalescer_opts;

typedef struct rl_coalescer_stats {
    uint64_t submitted;      /* requests accepted */
    uint64_t decided;        /* requests completed */
    uint64_t batches;        /* launches */
    uint64_t max_batch_seen; /* largest launch */
    uint64_t pending;        /* requests queued, not yet launched */
} rl_coalescer_stats;

/* Signature of rl_decide_batch (host arrays, synchronous).  A backend of this
 * type replaces the GPU in rl_coalescer_create_with_backend: the CPU tests
 * use it to check the batching and ordering logic on hosts without a GPU. */
typedef int (*rl_batch_fn)(void* user, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                           const int64_t* n, const uint32_t* cfg_id, uint8_t* decision, int64_t* remaining,
                           int64_t* retry_after_ns, int64_t* reset_at_ns);

/* Reset(ctx, key) for the test seam's host backend (rl_reset's signature) */
typedef int (*rl_reset_fn)(void* user, uint32_t cfg_id, uint64_t key_id, int64_t ts_ns);

/* Coalescer over a GPU engine, on the device current on the calling thread
 * (the engine's: rl_engine_create makes it current).  The engine should be created with
 * RL_OPT_PIPELINE (batch b+1's grouping then overlaps batch b's replay) and
 * must not be used by anyone else while the coalescer lives. */
int rl_coalescer_create(rl_engine* e, const rl_coalescer_opts* opts, rl_coalescer** out);
/* Test seam: the same coalescer over a synchronous host backend. */
int rl_coalescer_create_with_backend(rl_batch_fn fn, void* user, const rl_coalescer_opts* opts,
                                     rl_coalescer** out);
/* ... with Reset too (reset_fn nullable: rl_coalescer_reset then fails with RL_EINVAL) */
int rl_coalescer_create_with_backends(rl_batch_fn fn, rl_reset_fn reset_fn, void* user,
                                      const rl_coalescer_opts* opts, rl_coalescer** out);
/* Completes the queued requests, then stops the threads and frees every
 * submission not yet waited for.  No rl_coalescer_wait may be in progress. */
int rl_coalescer_destroy(rl_coalescer* c);

/* Enqueue m requests (copied; thread-safe, never blocks on the GPU).
 * *ticket = sequence number of the first request. */
int rl_coalescer_submit(rl_coalescer* c, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                        const int64_t* n, const uint32_t* cfg_id, uint64_t* ticket);
/* Block until the submission `ticket` is decided (timeout_ns < 0: no limit)
 * and copy its results out (in submission order).  Each ticket is waited for
 * exactly once.  Returns the engine status of its batch(es), RL_ETIMEOUT, or
 * RL_EINVAL for an unknown ticket. */
int rl_coalescer_wait(rl_coalescer* c, uint64_t ticket, int64_t timeout_ns, uint8_t* decision,
                      int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns);
/* submit(1) + wait: what one Limiter.AllowN call does */
int rl_coalescer_decide(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, int64_t n, uint32_t cfg_id,
                        uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns);
/* Reset(ctx, key) at ts_ns (rl_reset, include/rl_engine.h; tokenbucket.go:136-144,
 * slidingwindow.go:125-139, fixedwindow.go:118-128) in sequence order: after
 * every request submitted before it, before every request submitted after
 * it.  Blocks until applied. */
int rl_coalescer_reset(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, uint32_t cfg_id);
int rl_coalescer_get_stats(rl_coalescer* c, rl_coalescer_stats* out);

#ifdef __cplusplus
}
#endif
#endif
