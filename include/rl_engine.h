/*
 * rl_engine.h -- C-ABI of the MI355X batched rate-limit decision engine.
 *
 * This is the drop-in boundary that replaces the reference's storage seam:
 * every decision the reference makes with one go-redis EVAL round trip
 *   tokenbucket.go:172   client.Eval(ctx, tokenBucketScript, ...)
 *   slidingwindow.go:164 client.Eval(ctx, slidingWindowScript, ...)
 *   fixedwindow.go:152   client.Eval(ctx, fixedWindowScript, ...)
 * plus the Go arithmetic around it (AllowN, tokenbucket.go:90-133,
 * slidingwindow.go:68-122, fixedwindow.go:65-115) is made here, for a whole
 * batch, by HIP kernels over an HBM-resident state table.  Reset's DEL
 * (tokenbucket.go:139, slidingwindow.go:134, fixedwindow.go:123) maps to
 * rl_reset.  A cgo binding is shown in INTEGRATION.md.
 *
 * Conventions: plain C types only; arrays are caller-owned and only accessed
 * during the call (the *_device entry point: until the stream reaches it); the
 * engine owns all device memory.  Calls on one engine are not re-entrant.
 * Every function returns RL_OK (0) or a negative RL_E* status.
 * Every struct starts with `struct_size`, which the caller sets to sizeof the
 * struct it was compiled with: inputs of a size the library does not know are
 * rejected with RL_EINVAL, outputs are written up to the caller's size.
 */
#ifndef RL_ENGINE_H
#define RL_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes */
#define RL_OK          0
#define RL_EINVAL    (-22)  /* bad argument / config fails Validate (config.go:16-50) */
#define RL_ENOMEM    (-12)  /* device allocation failed or state table full */
#define RL_EDEVICE    (-5)  /* HIP runtime error (text in rl_last_error) */
#define RL_ETIMEOUT (-110)  /* a device-side bounded wait expired */
#define RL_EORDER    (-34)  /* reserved: no longer returned (window keys of any age are kept) */

/* algorithms (interface.go:11-23) */
#define RL_ALG_TOKEN_BUCKET   1
#define RL_ALG_SLIDING_WINDOW 2
#define RL_ALG_FIXED_WINDOW   3

/* backend semantics profile */
#define RL_PROFILE_REDIS7    0  /* real Redis 7: Lua tostring "%.14g", expiry now > when */
#define RL_PROFILE_MINIREDIS 1  /* miniredis + gopher-lua (the reference tests) */

/* per-request decision codes */
#define RL_DENIED  0
#define RL_ALLOWED 1
#define RL_ERROR   2  /* the script failed (INCRBY overflow): Go sees err != nil */
#define RL_INVALID 3  /* n <= 0, unknown cfg id or reserved key id: not executed */

/* reserved key id (marks an empty table slot) */
#define RL_KEY_RESERVED UINT64_MAX

typedef struct rl_engine rl_engine;

typedef struct rl_opts {
    uint32_t struct_size;   /* sizeof(rl_opts) */
    int32_t  device;        /* HIP device ordinal */
    int32_t  profile;       /* RL_PROFILE_* */
    uint64_t tb_capacity;   /* token-bucket table slots; rounded up to a power of 2 */
    uint64_t win_capacity;  /* window-counter table slots; rounded up to a power of 2 */
    uint32_t max_batch;     /* largest batch one launch sequence handles (<= 2^28) */
    uint32_t flags;         /* RL_OPT_* */
    uint64_t spill_capacity; /* window keys kept outside their user key's table entry (a live key
                                evicted by a newer window, or created out of order); rounded up to a
                                power of 2; 0 = 2 x win_capacity (a sliding window key holds ~2) */
} rl_opts;

/* rl_opts.flags: the device-API input arrays of every rl_decide_batch_device
 * call are complete when the call is made (not produced by work still queued
 * on `stream`).  The engine then runs each batch in three parts on three
 * internal streams -- grouping (hash, sort, permute), replay, finish -- so
 * that batch b+1's grouping and batch b-1's finish overlap batch b's replay
 * (three batches in flight, three internal buffer sets).  Replays stay in
 * call order; results are identical.  `stream` still orders the results:
 * work queued on it after the call sees them.  The inputs must stay
 * unmodified until then. */
#define RL_OPT_PIPELINE 1u

typedef struct rl_stats {
    uint32_t struct_size;     /* sizeof(rl_stats) */
    uint32_t pad_;
    uint64_t batches;
    uint64_t decisions;
    uint64_t last_segments;   /* distinct keys in the last batch */
    uint64_t last_heavy;      /* segments replayed cooperatively in the last batch */
    uint64_t last_coop_rounds; /* cooperative rounds of the last batch (all heavy segments) */
    uint64_t last_coop_iters;  /* offset fixed-point iterations of the last batch (all heavy segments) */
    uint32_t sort_bits;
    uint32_t sort_passes;
    uint64_t stamp_cycles[7];  /* replay timers of the last batch (10 ns ticks): [0] longest huge segment,
                                  [2] max per-block light phase, [4] first block start to last block end,
                                  [6] max rounds of one segment; [1] [3] [5] unused (0) */
    uint64_t coop_ends[4];     /* how the last batch's cooperative rounds ended: [0] window done,
                                  [1] stop request (allow / clamp / decade / expiry), [2] boundary
                                  (exact-pass mismatch safety net), [3] offset iteration cap */
    uint64_t sort_predicted;   /* batches whose grouping sort was launched as k_sort_local only (every
                                  MSD bucket predicted to fit LDS: no LSD passes, no k_segments) */
    uint64_t light_batches;    /* batches replayed by the light replay kernel (no huge segment expected) */
} rl_stats;

/* replaces redis.NewClient + NewTokenBucket/NewSlidingWindow/NewFixedWindow's
 * storage (tokenbucket.go:63-81 etc.) */
int rl_engine_create(const rl_opts* opts, rl_engine** out);
int rl_engine_destroy(rl_engine* e);

/* Register one limiter config (Config, interface.go:46-70; Validate config.go:16-50).
 * State is keyed by key_id only: callers give each (config, formatted key)
 * its own id, as FormatKey(key) is unique per prefix (config.go:81-87). */
int rl_config_register(rl_engine* e, uint8_t alg, int64_t limit, int64_t window_ns,
                       uint32_t* cfg_id);
/* The state table a config's keys live in: 0 the token-bucket table, 1 the
 * window table (whose keys may also move window keys to the spill table);
 * RL_EINVAL for an unknown id.  The coalescer's automatic GC budgets each
 * table by the requests that can insert into it. */
int rl_config_table(rl_engine* e, uint32_t cfg_id);

/* One batch in arrival order (array index = seq).  Host arrays; synchronous.
 *   ts_ns      request time, Unix ns (stands for time.Now() in AllowN)
 *   n          AllowN count (Allow = 1); n <= 0 yields RL_INVALID
 *   server_ms  Redis clock per request (nullable: floor(ts_ns / 1e6))
 * Outputs per request: decision (RL_DENIED/ALLOWED/ERROR/INVALID), remaining,
 * retry_after_ns, reset_at_ns (Unix ns; also valid for RL_ERROR, for the
 * fail-open Result), tokens (nullable; token-bucket only: the Lua `tokens`
 * value at the end of the script, bit-exact). */
int rl_decide_batch(rl_engine* e, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                    const int64_t* n, const uint32_t* cfg_id, const int64_t* server_ms,
                    uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                    int64_t* reset_at_ns, double* tokens);

/* Same, with device pointers, enqueued on `stream` (a hipStream_t; NULL = the
 * engine's stream).  Asynchronous: check errors with rl_engine_sync. */
int rl_decide_batch_device(rl_engine* e, size_t m, const uint64_t* key_id, const int64_t* ts_ns,
                           const int64_t* n, const uint32_t* cfg_id, const int64_t* server_ms,
                           uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns,
                           int64_t* reset_at_ns, double* tokens, void* stream);

/* wait for queued work; returns the sticky device status (RL_ENOMEM if the
 * table filled, RL_EORDER, RL_ETIMEOUT) and clears it */
int rl_engine_sync(rl_engine* e);

/* Reset(ctx, key) at time ts_ns: DEL of the key(s) AllowN would touch at ts_ns
 * (tokenbucket.go:136-144, slidingwindow.go:125-139, fixedwindow.go:118-128).
 * Synchronous. */
int rl_reset(rl_engine* e, uint32_t cfg_id, uint64_t key_id, int64_t ts_ns);
/* The same DEL enqueued in batch order: after every batch enqueued before the
 * call, before every batch enqueued after it (it runs on the engine's replay
 * stream, nothing is drained); `stream` (a hipStream_t, NULL = the engine's
 * stream) waits for it. */
int rl_reset_device(rl_engine* e, uint32_t cfg_id, uint64_t key_id, int64_t ts_ns, void* stream);

int rl_engine_stats(rl_engine* e, rl_stats* out);

/* State-table occupancy.  A key is live at server clock now_ms when its Redis
 * TTL has not expired (a window entry: either of its two counter keys). */
typedef struct rl_table_info {
    uint32_t struct_size;     /* sizeof(rl_table_info) */
    uint32_t pad_;
    uint64_t tb_capacity, tb_used, tb_live;
    uint64_t win_capacity, win_used, win_live;
    uint64_t spill_capacity, spill_used, spill_live;   /* spill slots ever claimed / live window keys */
} rl_table_info;
int rl_table_info_get(rl_engine* e, int64_t now_ms, rl_table_info* out);

/* Redis KEYS: every key live at server clock now_ms, as (key id, kind,
 * window start).  A token-bucket key is the hash FormatKey(key)
 * (tokenbucket.go:95); a window key is FormatKey(key):ws (fixedwindow.go:139-141,
 * slidingwindow.go:150-152).  Writes up to `cap` records (any order);
 * *count = how many keys are live.  Synchronous, waits for queued batches; a
 * diagnostic (the reference's tests list keys with miniredis Keys()). */
#define RL_KIND_HASH   0
#define RL_KIND_WINDOW 1
typedef struct rl_key_rec {
    uint64_t key_id;
    int64_t window_start;   /* Unix seconds (RL_KIND_WINDOW); 0 for a hash */
    uint32_t kind;          /* RL_KIND_* */
    uint32_t pad_;
} rl_key_rec;
int rl_table_keys(rl_engine* e, int64_t now_ms, rl_key_rec* out, size_t cap, uint64_t* count);

/* Table GC (the TTLs of tokenbucket.go:170,
 * slidingwindow.go:161-162, fixedwindow.go:151): drop every key expired at
 * server clock now_ms -- Redis's active expiry -- and optionally resize the
 * tables (0 = keep the capacity; the spill table follows win_capacity when
 * rl_opts.spill_capacity was 0, else keeps its capacity).  Keys are only ever inserted by the decision
 * path, so this is what keeps a long-running table from filling.  Decisions
 * are unchanged provided no later request carries a server clock below
 * now_ms (lazy expiry would see those keys as absent anyway).  Synchronous;
 * waits for queued batches.  RL_ENOMEM (old tables kept) when the live keys do
 * not fit the requested capacity.  `out` (nullable): the tables afterwards. */
int rl_table_gc(rl_engine* e, int64_t now_ms, uint64_t tb_capacity, uint64_t win_capacity, rl_table_info* out);

/* per-stage device time (ms) accumulated since the last call, measured with
 * HIP events on the stream the kernels run on; stages: 0 probe, 1 sort,
 * 2 segments + permute, 3 replay (k_tb_chain), 4 finish (run expansion +
 * unpermute).  rl_engine_set_timing(e, on): 0 off, 1 the replay only (two
 * events per batch on its stream), 2 every stage, -k (k >= 2) the replay
 * only on every k-th batch (the event pair costs the replay stream ~10 us per
 * batch; a timed benchmark samples).  *batches counts the batches timed. */
int rl_engine_set_timing(rl_engine* e, int on);
int rl_engine_stage_times(rl_engine* e, double* ms, int nstages, uint64_t* batches);
/* diagnostic: the last batch's replay debug counters (up to 88 words; layout in rl_engine.hip CTRL_DBG) */
int rl_engine_debug_words(rl_engine* e, uint32_t* out, size_t n);

int rl_last_error(rl_engine* e, char* buf, size_t len);

/* self-test hooks: exact tonumber(tostring(x)) of Redis Lua ("%.14g"),
 * host instantiation and device instantiation of the same code */
int rl_selftest_q14_host(const double* in, double* out, size_t n);
int rl_selftest_q14_device(rl_engine* e, const double* in, double* out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
