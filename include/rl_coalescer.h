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
 * the sequence number of the first request of its submission.  Reset, table
 * GC and table counts are queued like requests and take effect exactly
 * between the requests submitted before and after them.
 *
 * Contexts ("All methods should respect context cancellation and deadlines",
 * interface.go:75).  A submission may carry a deadline, and may be cancelled
 * (ctx.Done()).  go-redis checks the context before it sends a command and
 * returns ctx.Err() while it waits for the reply; the limiter then takes its
 * error branch, fail-open or fail-closed (tokenbucket.go:100-112,
 * slidingwindow.go:84-96, fixedwindow.go:80-92).  The coalescer does the same:
 *   - a submission none of whose requests has been launched when its deadline
 *     passes or when it is cancelled is dropped: it never reaches the state
 *     table (an EVAL never sent);
 *   - one already (partly) launched is applied in full (an EVAL already sent),
 *     but its waiter returns at the deadline / on cancellation all the same;
 *   - the wait returns RL_EDEADLINE (context.DeadlineExceeded) or
 *     RL_ECANCELED (context.Canceled); the caller maps it to the fail-open or
 *     fail-closed result exactly as for any other storage error.
 * Deadlines are on the clock rl_coalescer_now_ns() reads (CLOCK_MONOTONIC);
 * a Go caller converts with deadline_ns = rl_coalescer_now_ns() +
 * time.Until(d).
 *
 * ABI: every struct below starts with `struct_size`, which the caller sets to
 * sizeof the struct it was compiled with.  Inputs of an unknown size are
 * rejected with RL_EINVAL; outputs are written up to the caller's size.
 */
#ifndef RL_COALESCER_H
#define RL_COALESCER_H

#include <stddef.h>
#include <stdint.h>

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RL_EAGAIN     (-11)   /* queue full (rl_coalescer_opts.queue_cap) */
#define RL_ECLOSED    (-32)   /* coalescer destroyed / shutting down */
#define RL_EDEADLINE  (-62)   /* the submission's deadline passed (context.DeadlineExceeded) */
#define RL_ECANCELED (-125)   /* the submission was cancelled (context.Canceled) */

typedef struct rl_coalescer rl_coalescer;

typedef struct rl_coalescer_opts {
    uint32_t struct_size;    /* sizeof(rl_coalescer_opts) */
    uint32_t max_batch;      /* requests per launch (<= the engine's max_batch); 0 = 65536 */
    uint32_t max_in_flight;  /* batches on the GPU at once, 1..3; 0 = 3 */
    uint32_t gc_high_pct;    /* automatic GC: collect when a table's used slots pass this % (0 = 50) */
    int64_t  linger_ns;      /* with the GPU idle, wait this long for more requests (0 = launch at once) */
    uint64_t queue_cap;      /* pending requests beyond which submit returns RL_EAGAIN; 0 = 1 << 24 */
    /* Automatic table GC (Redis's active expiry; the TTLs of tokenbucket.go:170,
     * fixedwindow.go:151, slidingwindow.go:161-162).  0 = off.  Otherwise the
     * submitter counts the tables' slots (rl_table_info_get) at least every
     * gc_interval_ns, and sooner when the requests launched since the last count
     * could have filled the headroom to gc_high_pct; a table past gc_high_pct is
     * collected (rl_table_gc) at server clock floor(t / 1e6) - gc_margin_ms, t =
     * the time of the last request launched, and doubled first (up to the
     * gc_max_* capacities) when its live keys fill more than half of
     * gc_high_pct.  Exact while no later request carries a time more than
     * gc_margin_ms older than an earlier one. */
    int64_t  gc_interval_ns;
    int64_t  gc_margin_ms;         /* 0 = 1000 */
    uint64_t gc_max_tb_capacity;   /* growth limits (0 = no limit but the engine's) */
    uint64_t gc_max_win_capacity;
} rl_coalescer_opts;

typedef struct rl_coalescer_stats {
    uint32_t struct_size;    /* sizeof(rl_coalescer_stats) */
    uint32_t pad_;
    uint64_t submitted;      /* requests accepted */
    uint64_t decided;        /* requests completed (applied, or failed by the engine) */
    uint64_t batches;        /* launches */
    uint64_t max_batch_seen; /* largest launch */
    uint64_t pending;        /* requests queued, not yet launched */
    uint64_t expired;        /* requests dropped unapplied: deadline passed before launch */
    uint64_t cancelled;      /* requests dropped unapplied: cancelled before launch */
    uint64_t gc_runs;        /* table GCs (automatic and rl_coalescer_gc) */
    uint64_t gc_checks;      /* automatic occupancy counts */
    uint64_t gc_failures;    /* GCs that returned an error (the old tables stay) */
} rl_coalescer_stats;

/* Signature of rl_decide_batch (host arrays, synchronous).  A backend of this
 * type replaces the GPU in rl_coalescer_create_with_backend: the CPU tests
 * use it to check the batching and ordering logic on hosts without a GPU. */
typedef int (*rl_batch_fn)(void* user, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                           const int64_t* n, const uint32_t* cfg_id, uint8_t* decision, int64_t* remaining,
                           int64_t* retry_after_ns, int64_t* reset_at_ns);
/* Reset(ctx, key) for the test seam's host backend (rl_reset's signature) */
typedef int (*rl_reset_fn)(void* user, uint32_t cfg_id, uint64_t key_id, int64_t ts_ns);
/* table counts / GC for the host backend (rl_table_info_get / rl_table_gc) */
typedef int (*rl_info_fn)(void* user, int64_t now_ms, rl_table_info* out);
typedef int (*rl_gc_fn)(void* user, int64_t now_ms, uint64_t tb_capacity, uint64_t win_capacity,
                        rl_table_info* out);

/* A host backend (test seam): batch is required, the rest nullable (the
 * matching operation then fails with RL_EINVAL). */
typedef struct rl_coalescer_backend {
    uint32_t struct_size;    /* sizeof(rl_coalescer_backend) */
    rl_batch_fn batch;
    rl_reset_fn reset;
    rl_info_fn table_info;
    rl_gc_fn gc;
    void* user;
} rl_coalescer_backend;

/* Coalescer over a GPU engine, on the device current on the calling thread
 * (the engine's: rl_engine_create makes it current).  The engine should be created with
 * RL_OPT_PIPELINE (batch b+1's grouping then overlaps batch b's replay) and
 * must not be used by anyone else while the coalescer lives. */
int rl_coalescer_create(rl_engine* e, const rl_coalescer_opts* opts, rl_coalescer** out);
/* Test seam: the same coalescer over a synchronous host backend. */
int rl_coalescer_create_with_host_backend(const rl_coalescer_backend* be, const rl_coalescer_opts* opts,
                                          rl_coalescer** out);
/* shorthands of the above: batch only / batch + reset */
int rl_coalescer_create_with_backend(rl_batch_fn fn, void* user, const rl_coalescer_opts* opts,
                                     rl_coalescer** out);
int rl_coalescer_create_with_backends(rl_batch_fn fn, rl_reset_fn reset_fn, void* user,
                                      const rl_coalescer_opts* opts, rl_coalescer** out);
/* Completes the queued requests, then stops the threads and frees every
 * submission not yet waited for.  No rl_coalescer_wait may be in progress. */
int rl_coalescer_destroy(rl_coalescer* c);

/* the clock deadlines are measured on (CLOCK_MONOTONIC, ns) */
int64_t rl_coalescer_now_ns(void);

/* Enqueue m requests (copied; thread-safe, never blocks on the GPU).
 * *ticket = sequence number of the first request. */
int rl_coalescer_submit(rl_coalescer* c, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                        const int64_t* n, const uint32_t* cfg_id, uint64_t* ticket);
/* ... with a deadline (rl_coalescer_now_ns clock; 0 = none): see Contexts above */
int rl_coalescer_submit_deadline(rl_coalescer* c, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                                 const int64_t* n, const uint32_t* cfg_id, int64_t deadline_ns,
                                 uint64_t* ticket);
/* ctx.Done(): a submission not launched yet is dropped unapplied; a launched
 * one is applied and its results discarded.  Its wait (in progress or later)
 * returns RL_ECANCELED at once; the ticket is still waited for exactly once.
 * No effect on a submission already complete.  RL_EINVAL: unknown ticket. */
int rl_coalescer_cancel(rl_coalescer* c, uint64_t ticket);
/* Block until the submission `ticket` is decided (timeout_ns < 0: no limit)
 * and copy its results out (in submission order).  Each ticket is waited for
 * exactly once.  Returns the engine status of its batch(es); RL_EDEADLINE /
 * RL_ECANCELED (ticket released, outputs untouched); RL_ETIMEOUT when
 * timeout_ns ran out first (the ticket stays valid: wait again); RL_EINVAL for
 * an unknown ticket. */
int rl_coalescer_wait(rl_coalescer* c, uint64_t ticket, int64_t timeout_ns, uint8_t* decision,
                      int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns);
/* submit(1) + wait: what one Limiter.AllowN call does */
int rl_coalescer_decide(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, int64_t n, uint32_t cfg_id,
                        uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns);
/* ... with a deadline (AllowN(ctx, ...) with ctx.Deadline()) */
int rl_coalescer_decide_deadline(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, int64_t n, uint32_t cfg_id,
                                 int64_t deadline_ns, uint8_t* decision, int64_t* remaining,
                                 int64_t* retry_after_ns, int64_t* reset_at_ns);
/* Reset(ctx, key) at ts_ns (rl_reset_device, include/rl_engine.h;
 * tokenbucket.go:136-144, slidingwindow.go:125-139, fixedwindow.go:118-128) in
 * sequence order: after every request submitted before it, before every
 * request submitted after it.  Blocks until applied.  The DEL is enqueued on
 * the engine's replay stream like a batch: the pipeline is not drained. */
int rl_coalescer_reset(rl_coalescer* c, uint64_t key_id, int64_t ts_ns, uint32_t cfg_id);
/* rl_table_info_get / rl_table_gc in sequence order (both drain the
 * engine's in-flight batches first).  Block until done. */
int rl_coalescer_table_info(rl_coalescer* c, int64_t now_ms, rl_table_info* out);
int rl_coalescer_gc(rl_coalescer* c, int64_t now_ms, uint64_t tb_capacity, uint64_t win_capacity,
                    rl_table_info* out);
int rl_coalescer_get_stats(rl_coalescer* c, rl_coalescer_stats* out);

#ifdef __cplusplus
}
#endif
#endif
