"""Key-space sharding across GPUs (one process per GPU, torch.distributed).

Each rank owns the keys with owner(key) == rank (a 64-bit mix of the key id,
mod world size, include/rl_route.h) and keeps their state in its own HBM
tables.  Two ways to feed it:

  * routed ingress (RoutedPipeline, bench.py --gpus N): every rank receives
    arbitrary requests; the routing kernels group them by owner, an all-to-all
    moves the request records to their owners, the owner decides, and the
    inverse all-to-all returns the results.  On MI355X the "nccl" backend is
    RCCL over xGMI, where all-to-all drives all 7 point-to-point links at once;
  * sharded ingress (bench.py --ingress sharded): every rank receives only
    requests of the keys it owns; no data-path collective (N replicas).

Order: the reference's N app servers share one Redis, which applies a key's
requests in arrival order.  The owner replays the union of the ranks'
requests ordered by (ts, source rank, source position), a deterministic total
order consistent with each rank's own order, under one monotone store clock.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
import torch.distributed as dist

_PROF = os.environ.get("RL_ROUTE_PROFILE") is not None

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
    group them by owner GPU, two RCCL all-to-alls over xGMI (torch.distributed
    "nccl" process groups) move request records to their owners and results
    back, and the owner's engine decides its keys in the order one shared
    store sees them -- by request time, ties by (source rank, source position).

    Pipelining: batch b's pack and count exchange (stage A) are issued
    `lookahead` steps before its records move (stage B), so the host reads the
    counts that size the record all-to-all from a finished copy instead of
    stalling the GPU.  `depth` buffer sets rotate; a set is rewritten only
    after the batch that used it `depth` steps earlier has finished.  Requests go through their own process group and stream;
    results through a second group and one of `depth` streams, so a batch's
    result exchange never holds up the next batches' request exchange.

    decide(m, key, ts, n, cfg, sms, dec, rem, retry, reset, stream) enqueues
    the engine on the owner's merged requests (device pointers; the engine's
    rl_decide_batch_device without RL_OPT_PIPELINE: its grouping waits for
    `stream`, which has waited for the merge).  sms: the store clock
    (include/rl_route.h), the same on every owner."""

    def __init__(self, ops, decide, world, max_batch, device, pg_req=None, pg_res=None, depth=6, lookahead=2,
                 max_recv=None, staged=False, pg_cnt=None):
        self.ops, self.decide, self.world = ops, decide, world
        self.dev = torch.device(device)
        self.cuda = self.dev.type == "cuda"
        self.pg_req, self.pg_res = pg_req, pg_res
        # pg_cnt (optional): a process group of its own for the packs' count
        # exchange, on a stream of its own (C): a batch's counts then never
        # queue behind earlier batches' record exchanges, and the host, which
        # needs them for the split sizes, finds them ready
        self.pg_cnt = pg_cnt
        self.depth, self.lookahead = depth, lookahead
        self.staged = staged          # all-to-alls through host memory (gloo with device tensors)
        mb = max_batch
        mr = max_recv or world * max_batch
        self.max_batch, self.max_recv = mb, mr
        d = self.dev
        # streams on hardware queues of their own (ops.dedicated_stream): R and
        # the S streams wait on the engine's events, and a waiting stream would
        # block every stream that shares its hardware queue
        mk = getattr(ops, "dedicated_stream", None)
        if os.environ.get("RL_ROUTE_SHARED_QUEUES"):
            mk = None

        def new_stream():
            if not self.cuda:
                return None
            return mk() if mk is not None else torch.cuda.Stream(d)

        self.R = new_stream()
        self.C = new_stream() if pg_cnt is not None else self.R
        # one rank owns every key: nothing to exchange.  The records, counts and
        # results stay where the pack / results kernels wrote them (the merge
        # and unpack read them in place) -- no collective, no copy
        self.local = world == 1 and not staged
        self.slots = []
        for _ in range(depth):
            s = dict(
                send=torch.empty((mb, 4), dtype=torch.int64, device=d),
                slot=torch.empty(mb, dtype=torch.int32, device=d),
                # info rows (include/rl_route.h RL_ROUTE_INFO): {count, earliest ts, latest ts, in order}
                scnt=torch.zeros((world, INFO), dtype=torch.int64, device=d),   # per owner
                rcnt=torch.zeros((world, INFO), dtype=torch.int64, device=d),   # per source
                cnt_h=torch.zeros((2, world, INFO), dtype=torch.int64, pin_memory=self.cuda),
                recv=None if self.local else torch.empty((mr, 4), dtype=torch.int64, device=d),
                key=torch.empty(mr, dtype=torch.int64, device=d),
                ts=torch.empty(mr, dtype=torch.int64, device=d),
                n=torch.empty(mr, dtype=torch.int64, device=d),
                cfg=torch.empty(mr, dtype=torch.int32, device=d),
                sms=torch.empty(mr, dtype=torch.int64, device=d),
                at=torch.empty(mr, dtype=torch.int32, device=d),
                dec=torch.empty(mr, dtype=torch.uint8, device=d),
                rem=torch.empty(mr, dtype=torch.int64, device=d),
                retry=torch.empty(mr, dtype=torch.int64, device=d),
                reset=torch.empty(mr, dtype=torch.int64, device=d),
                res=torch.empty((mr, 4), dtype=torch.int64, device=d),
                back=None if self.local else torch.empty((mb, 4), dtype=torch.int64, device=d),
                S=new_stream(),
                ev_cnt=None, ev_merged=None, ev_done=None, m=0, busy=False,
            )
            self.slots.append(s)
        self.last_recv = 0
        # the merge on the batch's own stream S instead of R: R then carries
        # only packs and exchanges, so the count copies later batches wait for
        # are not queued behind merges; merges stay in step order (the router's
        # scratch and store clock) through ev_last_merge
        self.merge_on_s = self.cuda and not os.environ.get("RL_ROUTE_MERGE_ON_R")
        self.ev_last_merge = None
        self.wait_s = 0.0          # host time spent waiting for count copies
        self.host_prof = {}

    def _tick(self, name):
        """RL_ROUTE_PROFILE: host seconds per call site (since the last tick)"""
        if not _PROF:
            return
        now = time.perf_counter()
        if name is not None and getattr(self, "_t_last", None) is not None:
            self.host_prof[name] = self.host_prof.get(name, 0.0) + now - self._t_last
        self._t_last = now

    @staticmethod
    def _p(t):
        return t.data_ptr()

    def _sp(self, stream):
        return stream.cuda_stream if stream is not None else None

    def _a2a(self, out, inp, out_splits, in_splits, group):
        if self.staged:
            o = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o, inp.cpu(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                                   group=group)
            out.copy_(o, non_blocking=False)
        else:
            dist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits, group=group)

    def stage_a(self, b, key, ts, n, cfg):
        """pack batch b (device tensors: key/ts/n int64, cfg int32; complete
        now) and exchange its owner counts"""
        s = self.slots[b % self.depth]
        assert not s["busy"], "pipeline slot reused before its stage B"
        m = key.numel()
        assert m <= self.max_batch
        s["m"], s["busy"] = m, True
        p = self._p
        self._tick(None)
        C = self.C
        with _ctx(C):
            if s["ev_done"] is not None:
                C.wait_event(s["ev_done"])   # the set's previous batch has finished
            self.ops.pack(m, p(key), p(ts), p(n), p(cfg), p(s["send"]), p(s["scnt"]), p(s["slot"]),
                          self._sp(C))
            self._tick("a_pack")
            if not self.local:
                # the host reads the counts to size the record exchange
                self._a2a(s["rcnt"], s["scnt"], None, None, self.pg_cnt if self.pg_cnt is not None else self.pg_req)
                self._tick("a_a2a_cnt")
                s["cnt_h"][0].copy_(s["scnt"], non_blocking=True)
                s["cnt_h"][1].copy_(s["rcnt"], non_blocking=True)
            if self.cuda:
                s["ev_cnt"] = torch.cuda.Event()
                s["ev_cnt"].record(C)

    def stage_b(self, b, dec, rem, retry, reset):
        """move batch b's requests, decide them at their owners, bring the
        results back into dec/rem/retry/reset (device tensors, batch order);
        returns the stream on which they are complete"""
        s = self.slots[b % self.depth]
        if self.local:
            # world 1: every record is this rank's and the merge is planned on
            # the device (rl_route_merge without host rows): nothing to wait for
            m = tot = s["m"]
            sc = rc = [m]
        else:
            if s["ev_cnt"] is not None:
                t0 = time.perf_counter()
                s["ev_cnt"].synchronize()
                self.wait_s += time.perf_counter() - t0
            self._tick("b_wait")
            sc = s["cnt_h"][0][:, 0].tolist()
            rc = s["cnt_h"][1][:, 0].tolist()
            self._tick("b_counts")
            tot, m = int(sum(rc)), s["m"]
        assert tot <= self.max_recv, "received more than max_recv"
        self.last_recv = tot
        p = self._p
        recv = s["send"] if self.local else s["recv"]
        rcnt = s["scnt"] if self.local else s["rcnt"]

        def merge(stream):
            # the received info rows on the host too (read above): the merge is planned there
            self.ops.merge(tot, p(recv), p(rcnt), None if self.local else p(s["cnt_h"][1]), p(s["key"]), p(s["ts"]),
                           p(s["n"]),
                           p(s["cfg"]), p(s["sms"]), p(s["at"]), self._sp(stream))

        if self.local:
            # nothing to exchange: the merge waits for this step's pack only
            # (an event on R would also order it after the later steps'
            # packs issued since)
            s["ev_merged"] = s["ev_cnt"]
            if not self.merge_on_s:
                with _ctx(self.R):
                    merge(self.R)
                    if self.cuda:
                        s["ev_merged"] = torch.cuda.Event()
                        s["ev_merged"].record(self.R)
        else:
            with _ctx(self.R):
                if self.C is not self.R:
                    self.R.wait_event(s["ev_cnt"])    # the pack (send, rcnt) is complete
                self._a2a(s["recv"][:tot], s["send"][:m], rc, sc, self.pg_req)
                self._tick("b_a2a_req")
                if not self.merge_on_s:
                    merge(self.R)
                if self.cuda:
                    s["ev_merged"] = torch.cuda.Event()
                    s["ev_merged"].record(self.R)
        self._tick("b_merge")
        S = s["S"]
        with _ctx(S):
            if S is not None and s["ev_merged"] is not None:
                S.wait_event(s["ev_merged"])
            if self.merge_on_s:
                if self.ev_last_merge is not None:
                    S.wait_event(self.ev_last_merge)
                merge(S)
                self.ev_last_merge = torch.cuda.Event()
                self.ev_last_merge.record(S)
            self.decide(tot, p(s["key"]), p(s["ts"]), p(s["n"]), p(s["cfg"]), p(s["sms"]), p(s["dec"]),
                        p(s["rem"]), p(s["retry"]), p(s["reset"]), self._sp(S))
            self._tick("b_decide")
            if self.local and hasattr(self.ops, "results_local"):
                # nothing travels between results and unpack: one pass
                self.ops.results_local(m, p(s["slot"]), p(s["at"]), p(s["dec"]), p(s["rem"]), p(s["retry"]),
                                       p(s["reset"]), p(dec), p(rem), p(retry), p(reset), self._sp(S))
            else:
                self.ops.results(tot, p(s["at"]), p(s["dec"]), p(s["rem"]), p(s["retry"]), p(s["reset"]),
                                 p(s["res"]), self._sp(S))
                self._tick("b_results")
                if not self.local:
                    self._a2a(s["back"][:m], s["res"][:tot], sc, rc, self.pg_res)
                self._tick("b_a2a_res")
                self.ops.unpack(m, p(s["slot"]), p(s["res"] if self.local else s["back"]), p(dec), p(rem), p(retry),
                                p(reset), self._sp(S))
            if S is not None:
                s["ev_done"] = torch.cuda.Event()
                s["ev_done"].record(S)
        s["busy"] = False
        self._tick("b_unpack")
        return S

    def run(self, batches, outs, done=None):
        """all batches through the pipeline: batches[b] = (key, ts, n, cfg),
        outs[b] = (dec, rem, retry, reset); `done(b, stream)` after each"""
        nb = len(batches)
        L = min(self.lookahead, self.depth - 1)
        self.prime(batches, L)
        for b in range(nb):
            if b + L < nb:
                self.stage_a(b + L, *batches[b + L])
            S = self.stage_b(b, *outs[b])
            if done is not None:
                done(b, S)

    def prime(self, batches, L=None):
        L = min(self.lookahead, self.depth - 1) if L is None else L
        nb = len(batches)
        for b in range(min(L, nb)):
            self.stage_a(b, *batches[b])
