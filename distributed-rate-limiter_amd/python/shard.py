"""Key-space sharding across GPUs (one process per GPU, torch.distributed).

Each rank owns the keys with owner(key) == rank (a 64-bit mix of the key id,
mod world size, include/rl_route.h) and keeps their state in its own HBM
tables.  Two ways to feed it:

  * routed ingress (RoutedPipeline, bench.py --gpus N): every rank receives
    arbitrary requests; the routing kernels group them by owner into
    fixed-capacity buckets, an equal-split all-to-all moves the buckets to
    their owners, the owner merges and decides, and the inverse all-to-all
    returns the results -- with no host read anywhere in the step.  On MI355X
    the "nccl" backend is RCCL over xGMI, where all-to-all drives all 7
    point-to-point links at once;
  * sharded ingress (bench.py --ingress sharded): every rank receives only
    requests of the keys it owns; no data-path collective (N replicas).

Order: the reference's N app servers share one Redis, which applies a key's
requests in arrival order.  The owner replays the union of the ranks'
requests ordered by (ts, source rank, source position), a deterministic total
order consistent with each rank's own order, under one monotone store clock.
"""
from __future__ import annotations

import collections
import warnings

import numpy as np
import torch
import torch.distributed as dist

_M1 = np.uint64(0xbf58476d1ce4e5b9)
_M2 = np.uint64(0x94d049bb133111eb)


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer (same function as rl_table.h mix64)."""
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return x


def owner_of(key: np.ndarray, world: int) -> np.ndarray:
    # high bits: the table uses the low bits of the same hash for slots
    return ((mix64(key) >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


# --- the native routed pipeline (include/rl_route.h) ---------------------------

INFO = 4   # RL_ROUTE_INFO


def _ctx(stream):
    import contextlib
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


class RoutedPipeline:
    """One rank of the routed decision path: every rank accepts requests for
    any key; the routing kernels (include/rl_route.h: `ops`, an rl_amd.Router)
    pack them into one fixed-capacity bucket per owner GPU, two equal-split
    RCCL all-to-alls over xGMI (torch.distributed "nccl" process groups) move
    the buckets to their owners and the result buckets back, and the owner's
    engine decides its keys in the order one shared store sees them -- by
    arrival time, ties by (source rank, source position).

    Nothing in a step is read by the host: every split of every collective is
    `ops.capacity` records, the owner's merge takes the received counts from
    the received info rows in device memory, and the engine reads the merged
    batch's size from device memory too (rl_decide_routed_device).  A request
    past its owner's capacity is dropped (decision RL_DROPPED, ops.sync()
    reports RL_EOVERFLOW); size `cap` for the key skew (a uniform hash
    partition needs ~max_batch / world plus a margin, a Zipf hot key more).

    Streams (two, each on a hardware queue of its own): the request stream R
    runs every step's pack, request-side collectives and merge in step order
    (the router's scratch and store clock are sequential) and hands the
    merged batch to the engine; the result stream U takes the engine's
    results, runs the result all-to-all and the unpack.  So R goes on with
    the next step while the engine decides this one.  `depth` buffer sets
    rotate; a set is rewritten only after the step that used it `depth`
    steps earlier has unpacked.  (Round 3-4 ran each step's merge, engine
    call, result exchange and unpack on one of `depth` step streams: with the
    engine's three streams that made up to nine queues, and the engine's
    grouping of step b waited for step b - depth's unpack on the same step
    stream.)

    Collective order (the first N > 1 run must not deadlock).  The request
    collectives run on the request group (`pg_req`), the result collective on
    `pg_res`: two communicators, two internal streams.  RCCL, like NCCL,
    guarantees progress only when every rank runs the collectives of its
    communicators in one consistent order (or every pending collective kernel
    can be resident at once).  So the GPU order is made the host's issue
    order, the same on every rank: each collective first waits for the last
    one issued on the other group.  The result side of step b is issued
    `lookahead` steps late, after step b + lookahead's request side, so the
    one order is Req(0..L), Res(0), Req(L+1), Res(1), ...: a step's request
    exchange never waits for the engine of the step before it, and its merge
    and grouping wait only for the engine of step b - L - 1, which the
    engine's three buffer sets make it wait for anyway at L = 1.

    decide(m_max, count, recv, order, sms, res, in_stream, out_stream) runs
    the owner's engine on the merged batch (rl_decide_routed_device_io;
    device pointers): the grouping waits for in_stream, out_stream waits for
    the results.
    exchange: run the collectives (world > 1 always; at world 1 they are
    loopback copies over a one-rank group, e.g. to exercise RCCL; without them
    the buckets and results are read in place)."""

    def __init__(self, ops, decide, world, max_batch, device, pg_req=None, pg_res=None, depth=4, exchange=None,
                 staged=False, lookahead=None, ordered=True, decide_ev=None):
        self.ops, self.decide, self.world = ops, decide, world
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.pg_req, self.pg_res = pg_req, pg_res
        self.depth = depth
        self.exchange = world > 1 if exchange is None else bool(exchange)
        if world > 1 and not self.exchange:
            raise ValueError("world > 1 needs the exchange")
        self.staged = staged          # all-to-alls through host memory (gloo with device tensors)
        self.max_batch = max_batch
        self.cap = cap = ops.capacity
        tot = world * cap
        self.m_max = tot              # the merged batch's bound (the engine's max_batch must hold it)
        d = self.dev
        # streams on hardware queues of their own (ops.dedicated_stream): the
        # step streams wait on the engine's events, and a waiting stream would
        # block every stream that shares its hardware queue
        mk = getattr(ops, "dedicated_stream", None)

        def new_stream():
            if not self.cuda:
                return None
            return mk() if mk is not None else torch.cuda.Stream(d)

        self.R = new_stream()
        self.U = new_stream()
        # decide_ev(m_max, count, recv, order, sms, res, in_stream, event):
        # the engine records its results' completion into `event` instead of
        # making U wait at call time -- with the result side issued
        # `lookahead` steps late, a wait made at call time would queue U
        # behind this step's engine before the result exchanges issued in
        # between, and serialize the engine's steps
        self.decide_ev = decide_ev if self.cuda else None
        self.slots = []
        for _ in range(depth):
            s = dict(
                send=torch.empty((tot, 4), dtype=torch.int64, device=d),
                slot=torch.empty(max_batch, dtype=torch.int32, device=d),
                # info rows (include/rl_route.h RL_ROUTE_INFO): {sent, earliest ts, latest ts, dropped}
                scnt=torch.zeros((world, INFO), dtype=torch.int64, device=d),   # per owner
                rcnt=torch.zeros((world, INFO), dtype=torch.int64, device=d) if self.exchange else None,
                recv=torch.empty((tot, 4), dtype=torch.int64, device=d) if self.exchange else None,
                order=torch.empty(tot, dtype=torch.int32, device=d),
                sms=torch.empty(tot, dtype=torch.int64, device=d),
                count=torch.zeros(1, dtype=torch.int32, device=d),
                res=torch.empty((tot, 4), dtype=torch.int64, device=d),
                back=torch.empty((tot, 4), dtype=torch.int64, device=d) if self.exchange else None,
                ev_done=None,
                ev_res=None,
            )
            if self.decide_ev is not None:
                s["ev_res"] = torch.cuda.Event()
                s["ev_res"].record(self.R)    # materialize the event: the engine records it from now on
            self.slots.append(s)
        # result sides issued `lookahead` steps late (exchange only: without
        # collectives there is nothing to order).  Default 1, except on CUDA
        # without decide_ev: there the decide call makes U wait for this
        # step's engine at call time, so a late result side would queue step
        # b-1's result collective behind engine(b) and serialize the steps
        if lookahead is None:
            lookahead = 0 if (self.cuda and self.decide_ev is None) else 1
        elif lookahead > 0 and self.cuda and self.decide_ev is None and self.exchange:
            warnings.warn("RoutedPipeline: lookahead > 0 without decide_ev serializes the engine's steps on CUDA")
        self.lookahead = max(0, int(lookahead)) if self.exchange else 0
        if depth <= self.lookahead:
            raise ValueError("depth must exceed lookahead (a buffer set is reused after its step unpacked)")
        self.ordered = bool(ordered)  # False: no cross-group waits (A/B only: the order is then unconstrained)
        self._pend = []               # (b, slot, m, dec, rem, retry, reset): result side not issued yet
        self._ev_req = None           # after the last request-side collective issued (stream R)
        self._ev_res = None           # after the last result-side collective issued (stream U)
        # ("req" | "res", step): the collective issue order, the last 4096 (tests)
        self.order_log = collections.deque(maxlen=4096)
        self.collectives = 0          # all-to-alls issued (tests: the exchange really ran)
        self.wait_s = 0.0             # host time spent waiting on the device: none by construction
        self.host_prof = {}

    @staticmethod
    def _p(t):
        return t.data_ptr()

    @staticmethod
    def _sp(stream):
        return stream.cuda_stream if stream is not None else None

    def _a2a(self, out, inp, group):
        """equal-split all-to-all (every split the same size: nothing to size)"""
        self.collectives += 1
        if self.staged:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), group=group)
            out.copy_(o, non_blocking=False)
        else:
            dist.all_to_all_single(out, inp, group=group)

    def _record(self, stream):
        if stream is None:
            return None
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    def step(self, b, key, ts, n, cfg, dec, rem, retry, reset):
        """route and decide batch b (device tensors: key/ts/n int64, cfg int32,
        complete now); its results reach dec/rem/retry/reset (the caller's
        order) once its result side is issued -- at once without the
        exchange, else `lookahead` steps later or at flush().  Returns the
        [(b', stream)] whose result sides this call issued: b' is complete on
        `stream`."""
        s = self.slots[b % self.depth]
        m = key.numel()
        assert m <= self.max_batch
        p, sp = self._p, self._sp
        R = self.R
        recv = s["recv"] if self.exchange else s["send"]
        rcnt = s["rcnt"] if self.exchange else s["scnt"]
        with _ctx(R):
            if s["ev_done"] is not None:
                R.wait_event(s["ev_done"])   # the set's previous step has unpacked
            self.ops.pack(m, p(key), p(ts), p(n), p(cfg), p(s["send"]), p(s["scnt"]), p(s["slot"]), sp(R))
            if self.exchange:
                if self._ev_res is not None and self.ordered and self.pg_res is not self.pg_req:
                    R.wait_event(self._ev_res)   # after the last result collective issued
                self._a2a(s["rcnt"], s["scnt"], self.pg_req)
                self._a2a(s["recv"], s["send"], self.pg_req)
                self.order_log.append(("req", b))
                self._ev_req = self._record(R)
            self.ops.merge(p(recv), p(rcnt), p(s["order"]), p(s["sms"]), p(s["count"]), sp(R))
            # the engine's grouping waits for R; U waits for its results
            if self.decide_ev is not None:
                self.decide_ev(self.m_max, p(s["count"]), p(recv), p(s["order"]), p(s["sms"]), p(s["res"]), sp(R),
                               s["ev_res"].cuda_event)
            else:
                self.decide(self.m_max, p(s["count"]), p(recv), p(s["order"]), p(s["sms"]), p(s["res"]), sp(R),
                            sp(self.U))
        self._pend.append((b, s, m, dec, rem, retry, reset))
        done = []
        while len(self._pend) > self.lookahead:
            done.append(self._result_side(*self._pend.pop(0)))
        return done

    def _result_side(self, b, s, m, dec, rem, retry, reset):
        p, sp, U = self._p, self._sp, self.U
        with _ctx(U):
            if self.decide_ev is not None:
                U.wait_event(s["ev_res"])        # this step's results (recorded by the engine)
            if self.exchange:
                if self._ev_req is not None and self.ordered and self.pg_res is not self.pg_req:
                    U.wait_event(self._ev_req)   # after the last request collective issued
                self._a2a(s["back"], s["res"], self.pg_res)
                self.order_log.append(("res", b))
                self._ev_res = self._record(U)
            self.ops.unpack(m, p(s["slot"]), p(s["back"] if self.exchange else s["res"]), p(dec), p(rem), p(retry),
                            p(reset), sp(U))
            if U is not None:
                s["ev_done"] = torch.cuda.Event()
                s["ev_done"].record(U)
        return b, U

    def flush(self):
        """issue every deferred result side; returns [(b, stream)]"""
        done = []
        while self._pend:
            done.append(self._result_side(*self._pend.pop(0)))
        return done

    def run(self, batches, outs, done=None):
        """all batches through the pipeline: batches[b] = (key, ts, n, cfg),
        outs[b] = (dec, rem, retry, reset); `done(b, stream)` after each"""
        for b in range(len(batches)):
            for bd, S in self.step(b, *batches[b], *outs[b]):
                if done is not None:
                    done(bd, S)
        for bd, S in self.flush():
            if done is not None:
                done(bd, S)
