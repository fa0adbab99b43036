"""CPU restatement of the routing kernels (include/rl_route.h) -- TEST
INFRASTRUCTURE ONLY: it lets the world-size-2 gloo tests run the product's
pipeline orchestration (shard.RoutedPipeline) on CPU tensors.  The product
path is csrc/rl_route.hip; the GPU tests check that one against the oracle."""
import ctypes

import numpy as np

import shard


def _arr(ptr, n, dt):
    if n == 0:
        return np.zeros(0, dt)
    ct = {np.int64: ctypes.c_int64, np.int32: ctypes.c_int32, np.uint8: ctypes.c_uint8}[dt]
    return np.ctypeslib.as_array((ct * n).from_address(ptr))


def running_max_by_source(ts, src):
    """per element: the max of ts over the earlier-or-equal elements of the
    same source (sources contiguous)"""
    out = np.empty_like(ts)
    for s in np.unique(src):
        idx = np.nonzero(src == s)[0]
        out[idx] = np.maximum.accumulate(ts[idx])
    return out


CAP_ALIGN = 2048      # rl_route.hip: bucket capacities are multiples of the merge tile
DROPPED_SLOT = -1     # slot of a dropped request (UINT32_MAX as int32)


class NumpyRouteOps:
    """the routing kernels of include/rl_route.h on host pointers"""

    def __init__(self, world, cap):
        self.world = world
        self.capacity = (cap + CAP_ALIGN - 1) // CAP_ALIGN * CAP_ALIGN
        self.clock = -(1 << 63)     # the store clock of the next step (ms)
        self.overflow = False

    def pack(self, m, key, ts, n, cfg, send, scnt, slot, stream):
        cap = self.capacity
        k = _arr(key, m, np.int64).view(np.uint64)
        own = shard.owner_of(k, self.world)
        snd = _arr(send, 4 * self.world * cap, np.int64).reshape(self.world * cap, 4)
        c = _arr(cfg, m, np.int32).view(np.uint32).astype(np.int64)
        rec = np.stack([k.view(np.int64), _arr(ts, m, np.int64), _arr(n, m, np.int64),
                        c | (np.arange(m, dtype=np.int64) << 32)], 1)
        info = _arr(scnt, 4 * self.world, np.int64).reshape(self.world, 4)
        t = _arr(ts, m, np.int64)
        sl = _arr(slot, m, np.int32)
        for o in range(self.world):
            idx = np.nonzero(own == o)[0]          # batch order
            keep = idx[:cap]
            snd[o * cap:o * cap + keep.size] = rec[keep]
            sl[keep] = o * cap + np.arange(keep.size, dtype=np.int32)
            sl[idx[cap:]] = DROPPED_SLOT
            self.overflow |= idx.size > cap
            unsorted = int(m > 1 and bool(np.any(t[1:] < t[:-1])))
            info[o] = [keep.size, t.min() if m else (1 << 63) - 1, t.max() if m else -(1 << 63),
                       2 * (idx.size - keep.size) + unsorted]

    def merge(self, recv, info, order, sms, count, stream):
        cap, G = self.capacity, self.world
        rows = _arr(info, 4 * G, np.int64).reshape(G, 4)
        c0 = self.clock
        latest = rows[:, 2][rows[:, 2] != -(1 << 63)]
        if latest.size:
            self.clock = max(c0, int(latest.max()) // 1_000_000)
        rec = _arr(recv, 4 * G * cap, np.int64).reshape(G * cap, 4)
        cnt = np.clip(rows[:, 0], 0, cap)
        arrive, src, pos = [], [], []
        for s in range(G):
            a = np.maximum.accumulate(rec[s * cap:s * cap + cnt[s], 1]) if cnt[s] else np.zeros(0, np.int64)
            arrive.append(a)
            src.append(np.full(cnt[s], s))
            pos.append(np.arange(cnt[s]))
        arrive, src, pos = (np.concatenate(x) if x else np.zeros(0, np.int64) for x in (arrive, src, pos))
        o = np.lexsort((pos, src, arrive))          # arrival, ties by (source rank, source position)
        tot = int(cnt.sum())
        _arr(order, max(tot, 1), np.int32)[:tot] = (src[o] * cap + pos[o]).astype(np.int32)
        _arr(sms, max(tot, 1), np.int64)[:tot] = np.maximum(arrive[o] // 1_000_000, c0)
        _arr(count, 1, np.int32)[0] = tot

    def unpack(self, m, slot, back, dec, rem, retry, reset, stream):
        s = _arr(slot, m, np.int32)
        b = _arr(back, 4 * self.world * self.capacity, np.int64).reshape(self.world * self.capacity, 4)
        dropped = s == DROPPED_SLOT
        r = b[np.where(dropped, 0, s).astype(np.int64)]
        r[dropped] = [4, 0, 0, 0]                   # RL_DROPPED
        _arr(dec, m, np.uint8)[:] = r[:, 0]
        _arr(rem, m, np.int64)[:] = r[:, 1]
        _arr(retry, m, np.int64)[:] = r[:, 2]
        _arr(reset, m, np.int64)[:] = r[:, 3]


def oracle_decide(sim, world, cap):
    """the owner's engine (rl_decide_routed_device) over host pointers,
    backed by the CPU oracle: request p is recv[order[p]], p < count"""
    def decide(m_max, count, recv, order, sms, res, stream, out_stream=None):
        cnt = int(_arr(count, 1, np.int32)[0])
        if cnt == 0:
            return
        o = _arr(order, cnt, np.int32).astype(np.int64)
        rec = _arr(recv, 4 * world * cap, np.int64).reshape(world * cap, 4)[o]
        d, r, rt, rs, _ = sim.decide(rec[:, 0].view(np.uint64), rec[:, 1], rec[:, 2],
                                     (rec[:, 3] & 0xffffffff).astype(np.uint32), _arr(sms, cnt, np.int64))
        out = _arr(res, 4 * world * cap, np.int64).reshape(world * cap, 4)
        out[o] = np.stack([d.astype(np.int64), r, rt, rs], 1)
    return decide


def shared_limiter_expectations(all_batches, rank, configs, profile=0, cap=None):
    """decisions of ONE shared limiter over every rank's batches, step by step,
    each step in (arrival, source rank, source position) order -- a request's
    arrival is the running max of ts over the requests its rank sent to the
    same owner so far -- with the store's clock max(floor(arrival / 1e6), the
    latest ts of earlier steps) (include/rl_route.h); per step, `rank`'s
    results in its batch order.  cap: a rank's requests for one owner past the
    first `cap` of the step are dropped (never reach the store, RL_DROPPED)."""
    import oracle
    ref = oracle.OracleSim(profile)
    for a, L, W in configs:
        ref.add_config(a, L, W)
    world = len(all_batches)
    outs = []
    clock = -(1 << 63)
    for b in range(len(all_batches[0])):
        parts = [all_batches[r][b] for r in range(world)]
        U = [np.concatenate([p[f] for p in parts]) for f in range(4)]
        src = np.concatenate([np.full(p[0].size, r) for r, p in enumerate(parts)])
        pos = np.concatenate([np.arange(p[0].size) for p in parts])
        own = shard.owner_of(U[0].astype(np.uint64), world)
        arrive = np.empty_like(U[1])
        sent = np.ones(U[0].size, bool)
        for r in range(world):
            for w in range(world):
                idx = np.nonzero((src == r) & (own == w))[0]
                if cap is not None and idx.size > cap:
                    sent[idx[cap:]] = False
                    idx = idx[:cap]
                if idx.size:
                    arrive[idx] = np.maximum.accumulate(U[1][idx])
        live = np.nonzero(sent)[0]
        o = live[np.lexsort((pos[live], src[live], arrive[live]))]
        sms = np.maximum(arrive[o] // 1_000_000, clock)
        if U[1].size:
            clock = max(clock, int(U[1].max()) // 1_000_000)
        d, rm, rt, rs, _ = ref.decide(U[0][o], U[1][o], U[2][o], U[3][o], sms)
        full = [np.zeros(U[0].size, np.int64) for _ in range(4)]
        full[0][:] = 4                             # RL_DROPPED unless decided
        for f, x in enumerate((d, rm, rt, rs)):
            full[f][o] = x
        mine = src == rank
        outs.append([x[mine] for x in full])
    return outs
