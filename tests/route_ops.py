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


class NumpyRouteOps:
    def __init__(self, world):
        self.world = world
        self.clock = -(1 << 63)     # the store clock of the next step (ms)

    def pack(self, m, key, ts, n, cfg, send, scnt, slot, stream):
        k = _arr(key, m, np.int64).view(np.uint64)
        own = shard.owner_of(k, self.world)
        order = np.argsort(own, kind="stable")
        snd = _arr(send, 4 * m, np.int64).reshape(m, 4)
        c = _arr(cfg, m, np.int32).view(np.uint32).astype(np.int64)
        rec = np.stack([k.view(np.int64), _arr(ts, m, np.int64), _arr(n, m, np.int64),
                        c | (np.arange(m, dtype=np.int64) << 32)], 1)
        snd[:] = rec[order]
        info = _arr(scnt, 4 * self.world, np.int64).reshape(self.world, 4)
        t = _arr(ts, m, np.int64)
        info[:, 0] = np.bincount(own, minlength=self.world)
        info[:, 1] = t.min() if m else (1 << 63) - 1
        info[:, 2] = t.max() if m else -(1 << 63)
        info[:, 3] = int(bool(np.all(t[1:] >= t[:-1])))
        sl = _arr(slot, m, np.int32)
        sl[order] = np.arange(m, dtype=np.int32)

    def merge(self, m, recv, info, info_host, key, ts, n, cfg, sms, at, stream):
        latest = _arr(info, 4 * self.world, np.int64).reshape(self.world, 4)[:, 2]
        c0 = self.clock
        live = latest[latest != -(1 << 63)]
        if live.size:
            self.clock = max(c0, int(live.max()) // 1_000_000)
        if m == 0:
            return
        rec = _arr(recv, 4 * m, np.int64).reshape(m, 4)
        rows = _arr(info, 4 * self.world, np.int64).reshape(self.world, 4)
        sent = rows[:, 0] > 0
        arrive = rec[:, 1].copy()
        if not np.all(rows[sent, 3] != 0):
            # a request arrives at the running max of its source's ts so far
            src = np.minimum(np.searchsorted(np.cumsum(rows[:, 0]), np.arange(m), side="right"), self.world - 1)
            arrive = running_max_by_source(rec[:, 1], src)
        if np.count_nonzero(sent) <= 1:
            o = np.arange(m)                            # one source: its own order
        else:
            o = np.argsort(arrive, kind="stable")       # arrival order, ties by received order
        _arr(key, m, np.int64)[:] = rec[o, 0]
        _arr(ts, m, np.int64)[:] = rec[o, 1]
        _arr(n, m, np.int64)[:] = rec[o, 2]
        _arr(cfg, m, np.int32)[:] = (rec[o, 3] & 0xffffffff).astype(np.uint32).view(np.int32)
        _arr(sms, m, np.int64)[:] = np.maximum(arrive[o] // 1_000_000, c0)
        a = _arr(at, m, np.int32)
        a[o] = np.arange(m, dtype=np.int32)

    @staticmethod
    def results(m, at, dec, rem, retry, reset, res, stream):
        a = _arr(at, m, np.int32)
        r = _arr(res, 4 * m, np.int64).reshape(m, 4)
        r[:, 0] = _arr(dec, m, np.uint8)[a]
        r[:, 1] = _arr(rem, m, np.int64)[a]
        r[:, 2] = _arr(retry, m, np.int64)[a]
        r[:, 3] = _arr(reset, m, np.int64)[a]

    @staticmethod
    def unpack(m, slot, back, dec, rem, retry, reset, stream):
        s = _arr(slot, m, np.int32)
        b = _arr(back, 4 * m, np.int64).reshape(m, 4)[s]
        _arr(dec, m, np.uint8)[:] = b[:, 0]
        _arr(rem, m, np.int64)[:] = b[:, 1]
        _arr(retry, m, np.int64)[:] = b[:, 2]
        _arr(reset, m, np.int64)[:] = b[:, 3]


def oracle_decide(sim):
    """engine decide() over host pointers, backed by the CPU oracle"""
    def decide(m, key, ts, n, cfg, sms, dec, rem, retry, reset, stream):
        if m == 0:
            return
        d, r, rt, rs, _ = sim.decide(_arr(key, m, np.int64).view(np.uint64), _arr(ts, m, np.int64),
                                     _arr(n, m, np.int64), _arr(cfg, m, np.int32).view(np.uint32),
                                     _arr(sms, m, np.int64))
        _arr(dec, m, np.uint8)[:] = d
        _arr(rem, m, np.int64)[:] = r
        _arr(retry, m, np.int64)[:] = rt
        _arr(reset, m, np.int64)[:] = rs
    return decide


def shared_limiter_expectations(all_batches, rank, configs, profile=0):
    """decisions of ONE shared limiter over every rank's batches, step by step,
    each step in (arrival, source rank, source position) order -- a request's
    arrival is the running max of ts over the requests its rank sent to the
    same owner so far -- with the store's clock max(floor(arrival / 1e6), the
    latest ts of earlier steps) (include/rl_route.h); per step, `rank`'s
    results in its batch order"""
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
        for r in range(world):
            for w in range(world):
                idx = np.nonzero((src == r) & (own == w))[0]
                if idx.size:
                    arrive[idx] = np.maximum.accumulate(U[1][idx])
        o = np.lexsort((pos, src, arrive))
        sms = np.maximum(arrive[o] // 1_000_000, clock)
        if U[1].size:
            clock = max(clock, int(U[1].max()) // 1_000_000)
        d, rm, rt, rs, _ = ref.decide(U[0][o], U[1][o], U[2][o], U[3][o], sms)
        mine = src[o] == rank
        exp_pos = pos[o][mine]
        inv = np.empty_like(exp_pos)
        inv[exp_pos] = np.arange(exp_pos.size)
        outs.append([x[mine][inv] for x in (d, rm, rt, rs)])
    return outs
