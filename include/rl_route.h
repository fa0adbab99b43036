/*
 * rl_route.h -- hash-sharded routing of request batches across GPUs
 * (BASELINE.json configs[3]).
 *
 * The reference's deployment is N stateless app servers sharing one Redis
 * (docs/ARCHITECTURE.md:142-164): every server may ask about any key, and the
 * store applies each key's requests in arrival order.  Here the key space is
 * split over the GPUs of a node -- GPU owner(k) = (mix64(k) >> 32) mod G keeps
 * key k's state in its HBM tables -- and every GPU accepts requests for any
 * key.  One step of G ranks, each with a batch of requests:
 *
 *   sender   rl_route_pack      owner of every request; requests grouped by
 *                               owner (stable) into 32-byte records; per owner
 *                               {count, the batch's earliest and latest ts,
 *                               whether the batch is in time order} (int64)
 *            all-to-all of the counts, then of the records (RCCL over xGMI;
 *            the caller drives the collectives, e.g. torch.distributed "nccl")
 *   owner    rl_route_merge     the received records -- grouped by source rank,
 *                               each group in its source's order -- in the
 *                               order ONE shared store sees them: by arrival
 *                               time, ties by (source rank, source position),
 *                               where a request arrives at the running max of
 *                               its source's ts so far (each source's own order
 *                               is kept, also for a batch out of time order);
 *                               written as the key/ts/n/cfg/server_ms arrays
 *                               rl_decide_batch_device takes
 *            rl_decide_batch_device (include/rl_engine.h) on them
 *            rl_route_results   results back to received order, 32-byte records
 *            all-to-all of the results (the counts reversed)
 *   sender   rl_route_unpack    results to the caller's order
 *
 * The store's clock (Redis TTLs) is one clock that never goes back: request
 * p of step b expires keys at server_ms = max(floor(arrival_p / 1e6), the
 * latest floor(ts / 1e6) of any request of any rank in steps before b).
 * Every owner learns each rank's latest ts through the count exchange, so all
 * owners keep the same clock, and per key the clock never decreases (merge
 * order is arrival order), which is what makes expiry exact (rl_window.h).
 *
 * Every array is device memory; every call is asynchronous on `stream` (a
 * hipStream_t).  Requirement: the timestamps one owner receives in a step
 * span less than 2^48 ns (78 hours); a violation is reported by
 * rl_router_sync (RL_EINVAL) and the merge order is then unspecified.
 */
#ifndef RL_ROUTE_H
#define RL_ROUTE_H

#include <stddef.h>
#include <stdint.h>

#include "rl_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

/* one routed request (send and receive buffers) */
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

/* scratch for batches of up to max_batch sent and max_recv received requests */
int rl_router_create(int32_t device, int32_t world, uint32_t max_batch, uint32_t max_recv, rl_router** out);
int rl_router_destroy(rl_router* r);
/* wait for the router's queued work on `stream`; returns and clears the
 * sticky status (RL_EINVAL: ts span >= 2^48 ns, RL_ETIMEOUT: sort look-back) */
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

/* sender: requests grouped by owner -> send[m] (owner 0's first, each group in
 * batch order); send_info[RL_ROUTE_INFO * o + k]: k = 0 requests for owner o,
 * 1 the batch's earliest ts, 2 its latest ts (INT64_MAX / INT64_MIN if empty),
 * 3 nonzero when the batch's ts never decrease -- RL_ROUTE_INFO int64 per
 * owner, exchanged with an equal-split all-to-all; slot[i] = request i's
 * position in send (for rl_route_unpack) */
#define RL_ROUTE_INFO 4
int rl_route_pack(rl_router* r, size_t m, const uint64_t* key, const int64_t* ts, const int64_t* n,
                  const uint32_t* cfg, rl_route_rec* send, int64_t* send_info, uint32_t* slot, void* stream);

/* owner: recv[m_recv] (grouped by source rank) -> the decision order; writes
 * key/ts/n/cfg/server_ms[m_recv] for rl_decide_batch_device and at[i] = the
 * position of received record i in that order.  recv_info: the received
 * send_info rows (source r's at [RL_ROUTE_INFO * r]) in device memory, and
 * recv_info_host: the same rows on the host (the caller read them to size the
 * record exchange).  The merge is planned on the host from them: when only
 * one source sent records, the received order already is the decision order
 * and the merge is one gather kernel (when every source's batch is in time
 * order, arrival = ts and no running max is taken); otherwise only the sort
 * passes the step's time span needs are launched.  The rows also advance the
 * store clock after this step.  Call once per step, in step order, also when
 * m_recv is 0.  recv_info_host NULL (world 1 only: one source): the merge is
 * planned on the device -- no host read of the rows, the store clock kept in
 * device memory from then on (a router then takes no host-planned merge:
 * RL_EINVAL) -- as a per-tile max, one scan block and one gather. */
int rl_route_merge(rl_router* r, size_t m_recv, const rl_route_rec* recv, const int64_t* recv_info,
                   const int64_t* recv_info_host, uint64_t* key, int64_t* ts, int64_t* n, uint32_t* cfg,
                   int64_t* server_ms, uint32_t* at, void* stream);

/* owner: decisions (in the merge order) -> res[i] for received record i */
int rl_route_results(size_t m_recv, const uint32_t* at, const uint8_t* decision, const int64_t* remaining,
                     const int64_t* retry_after_ns, const int64_t* reset_at_ns, rl_route_res* res, void* stream);

/* sender: back[m] (send layout) -> the caller's order */
int rl_route_unpack(size_t m, const uint32_t* slot, const rl_route_res* back, uint8_t* decision,
                    int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns, void* stream);

/* one GPU (nothing exchanged between the two): rl_route_results and
 * rl_route_unpack in one pass -- the caller's outputs for request i from the
 * engine's outputs at position at[slot[i]] */
int rl_route_results_local(size_t m, const uint32_t* slot, const uint32_t* at, const uint8_t* decision_in,
                           const int64_t* remaining_in, const int64_t* retry_in, const int64_t* reset_in,
                           uint8_t* decision, int64_t* remaining, int64_t* retry_after_ns, int64_t* reset_at_ns,
                           void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RL_ROUTE_H */
