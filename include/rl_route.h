/*
 * rl_route.h -- hash-sharded routing of request batches across GPUs
 * (BASELINE.json configs[3]).
 *
 * The reference's deployment is N stateless app servers sharing one Redis
 * (docs/ARCHITECTURE.md:142-164): every server may ask about any key, and the
 * store applies each key's requests in arrival order.  Here the key space is
 * split over the GPUs of a node -- GPU owner(k) = (mix64(k) >> 32) mod G keeps
 * key k's state in its HBM tables -- and every GPU accepts requests for any
 * key.  One step of G ranks, each with a batch of requests, runs with no host
 * involvement at all (nothing is read back to size anything):
 *
 *   sender   rl_route_pack      owner of every request; requests grouped by
 *                               owner (stable) into fixed-capacity buckets of
 *                               `cap` 32-byte records, send[o * cap + j]; per
 *                               owner an info row {count sent, earliest ts,
 *                               latest ts, flags: 2 * count dropped + 1 if
 *                               the batch's ts ever decrease}.  A request past
 *                               its owner's capacity is dropped: never
 *                               executed, decision RL_DROPPED, and the
 *                               router's sticky status reports RL_EOVERFLOW
 *            equal-split all-to-alls of the info rows and of the buckets
 *            (RCCL over xGMI; the caller drives the collectives, e.g.
 *            torch.distributed "nccl"): every split is `cap` records, so the
 *            collectives need no host-side sizes
 *   owner    rl_route_merge     the received buckets -- source s's `count`
 *                               records at recv[s * cap], in its order -- in
 *                               the order ONE shared store sees them: by
 *                               arrival time, ties by (source rank, source
 *                               position), where a request arrives at the
 *                               running max of its source's ts so far (each
 *                               source's own order is kept, also for a batch
 *                               out of time order).  Planned on the device:
 *                               per-source running maxima, then a tree of
 *                               merge-path merges; writes the decision order
 *                               order[p] (a receive index), each request's
 *                               store clock server_ms[p] and the number
 *                               received into *count (device memory)
 *            rl_decide_routed_device: the owner's engine reads the received
 *                               records in that order and writes 32-byte
 *                               result records at their receive index
 *            equal-split all-to-all of the result buckets back
 *   sender   rl_route_unpack    results to the caller's order
 *
 * The store's clock (Redis TTLs) is one clock that never goes back: request
 * p of step b expires keys at server_ms = max(floor(arrival_p / 1e6), the
 * latest floor(ts / 1e6) of any request of any rank in steps before b).
 * Every owner learns each rank's latest ts through the info rows, so all
 * owners keep the same clock (in device memory), and per key the clock never
 * decreases (merge order is arrival order), which is what makes expiry exact
 * (rl_window.h).
 *
 * Every array is device memory; every call is asynchronous on `stream` (a
 * hipStream_t).  Calls on one router use its scratch: packs must run in step
 * order, merges too (the store clock), e.g. each on one stream or ordered by
 * events.
 */
#ifndef RL_ROUTE_H
#define RL_ROUTE_H

#include <stddef.h>
#include <stdint.h>

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RL_EOVERFLOW (-75)     /* a request exceeded its owner's bucket capacity (rl_router_sync) */
#define RL_DROPPED 4           /* decision: not executed, its owner's bucket was full (resubmit it) */
#define RL_ROUTE_INFO 4        /* int64 per info row: count sent, earliest ts, latest ts, 2 * dropped + unsorted */
#define RL_ORDER_IDENTITY 0xffffffffu   /* order[0]: the received order is the decision order (rl_route_merge) */

/* one routed request (send and receive buckets) */
typedef struct rl_route_rec {
    uint64_t key;
    int64_t ts;
    int64_t n;
    uint32_t cfg;
    uint32_t pos;      /* position in the sender's batch */
} rl_route_rec;

/* one routed result (the four Result fields of include/rl_engine.h) */
typedef struct rl_route_res {
    int64_t decision;
    int64_t remaining;
    int64_t retry_after_ns;
    int64_t reset_at_ns;
} rl_route_res;

typedef struct rl_router rl_router;

/* scratch for batches of up to max_batch requests and buckets of `cap`
 * records per peer (rounded up to a multiple of 2048; rl_router_capacity).
 * cap = max_batch can never drop a request; a hash partition of a uniform
 * key stream needs about max_batch / world plus a margin. */
int rl_router_create(int32_t device, int32_t world, uint32_t max_batch, uint32_t cap, rl_router** out);
int rl_router_destroy(rl_router* r);
/* the bucket capacity in records (every split of the collectives) */
uint32_t rl_router_capacity(const rl_router* r);
/* wait for the router's queued work on `stream`; returns and clears the
 * sticky status: RL_EOVERFLOW when a request was dropped since the last sync */
int rl_router_sync(rl_router* r, void* stream);

/* A stream on a hardware queue of its own (CU-masked with every CU, which
 * the runtime never shares): with more streams than the process's hardware
 * queues, a stream that waits on an event blocks every stream sharing its
 * queue; the routed pipeline's streams wait on the engine's, so they need
 * their own.  Returns a hipStream_t in *out. */
int rl_stream_create_dedicated(int32_t device, void** out);
int rl_stream_destroy(void* stream);

/* owner of each key id (the partition: (mix64(k) >> 32) mod world) */
int rl_route_owner(rl_router* r, size_t m, const uint64_t* key, uint32_t* owner, void* stream);

/* sender: request i for owner o is the j-th of the batch's requests for o
 * (batch order); j < cap: send[o * cap + j], slot[i] = o * cap + j; else
 * dropped, slot[i] = UINT32_MAX.  send_info[RL_ROUTE_INFO * o + k]: k = 0
 * requests sent to o (<= cap), 1 the batch's earliest ts, 2 its latest ts
 * (INT64_MAX / INT64_MIN if the batch is empty), 3 twice the requests for o
 * dropped, plus 1 when the batch's ts decrease somewhere (a source in time
 * order needs no running max of its arrival times at the owner).  Rows 1-2
 * cover the whole batch, dropped requests included: every owner must derive
 * the same store clock, and a dropped request's time is still a time the
 * shared store's clock (real time in the reference's single Redis) has
 * reached -- so a dropped request advances the store clock like a sent one
 * (tests/test_route_gpu.py::test_route_dropped_request_advances_store_clock). */
int rl_route_pack(rl_router* r, size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n,
                  const uint32_t* cfg, rl_route_rec* send, int64_t* send_info, uint32_t* slot, void* stream);

/* owner: recv[world * cap] (source s's bucket at s * cap) and recv_info (the
 * received info rows, source s's at RL_ROUTE_INFO * s) -> the decision order:
 * order[p] = receive index of the p-th request, server_ms[p] its store clock,
 * *count = requests received (p < *count are valid).  One source whose batch
 * is in time order (world 1, info flag clear) is its own decision order: the
 * merge then writes only order[0] = RL_ORDER_IDENTITY and server_ms[0] = the
 * store clock of the earlier steps, meaning order[p] = p and server_ms[p] =
 * max(server_ms[0], floor(recv[p].ts / 1e6)); rl_decide_routed_device reads
 * that form directly.  Call once per step, in step order (it advances the
 * store clock). */
int rl_route_merge(rl_router* r, const rl_route_rec* recv, const int64_t* recv_info, uint32_t* order,
                   int64_t* server_ms, uint32_t* count, void* stream);

/* owner: the engine on the merged requests -- request p is recv[order[p]]
 * with store clock server_ms[p], p < *count (device memory, at most m_max <=
 * the engine's max_batch); its result goes to res[order[p]].  The grouping
 * waits for `stream` (the merge); `stream` waits for the results.  m_max must
 * be at least world * rl_router_capacity (the most a merge can count): a
 * device count above m_max decides only the first m_max requests, and the
 * next rl_engine_sync returns RL_EOVERFLOW. */
int rl_decide_routed_device(rl_engine* e, size_t m_max, const uint32_t* count, const rl_route_rec* recv,
                            const uint32_t* order, const int64_t* server_ms, rl_route_res* res, void* stream);
/* the same with the two sides on two streams: the grouping waits for
 * in_stream (the merge), out_stream waits for the results -- so in_stream
 * can go on with the next step's pack and merge while this one decides */
int rl_decide_routed_device_io(rl_engine* e, size_t m_max, const uint32_t* count, const rl_route_rec* recv,
                               const uint32_t* order, const int64_t* server_ms, rl_route_res* res, void* in_stream,
                               void* out_stream);

/* the same with the results' completion recorded into done_event (a
 * hipEvent_t the caller owns) instead of a stream wait made at call time: a
 * pipeline that issues its result side later (after the next step's request
 * exchange) waits on the event then, so its result stream does not queue
 * behind this batch before the collectives issued in between */
int rl_decide_routed_device_ev(rl_engine* e, size_t m_max, const uint32_t* count, const rl_route_rec* recv,
                               const uint32_t* order, const int64_t* server_ms, rl_route_res* res, void* in_stream,
                               void* done_event);

/* sender: back[world * cap] (the result buckets, send layout) -> the caller's
 * order; a dropped request gets decision RL_DROPPED and zeros */
int rl_route_unpack(rl_router* r, size_t m, const uint32_t* slot, const rl_route_res* back, uint8_t* decision,
                    int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RL_ROUTE_H */
