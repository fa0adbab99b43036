"""Request coalescer (include/rl_coalescer.h): concurrent submissions become
engine batches in sequence order, and every submitter gets exactly the results
the reference limiter would give when receiving all requests one by one in
ticket order.

CPU tests drive the coalescer over a synchronous host backend (the
rl_coalescer_create_with_backend test seam) that decides each batch with the
oracle; the GPU tests drive it over the MI355X engine.  In both, the check
replays every request in ticket (= sequence) order through a fresh oracle."""
import ctypes as C
import threading

import numpy as np
import pytest

NS = 1_000_000_000
T0 = (1_760_000_000 // 60) * 60 * NS   # a minute boundary: every window id below is the same
CONFIGS = [(1, 20, 12 * NS), (3, 100, 60 * NS), (2, 100, 60 * NS), (1, 5, NS)]


def _arr(p, t, m):
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(t)), shape=(m,))


def oracle_backend(oracle_mod, configs, log):
    sim = oracle_mod.OracleSim(oracle_mod.REDIS7)
    for a, L, W in configs:
        sim.add_config(a, L, W)

    def fn(user, m, key, ts, n, cfg, dec, rem, retry, reset):
        d, r, ra, rs, _ = sim.decide(_arr(key, C.c_uint64, m).copy(), _arr(ts, C.c_int64, m).copy(),
                                     _arr(n, C.c_int64, m).copy(), _arr(cfg, C.c_uint32, m).copy())
        _arr(dec, C.c_uint8, m)[:] = d
        _arr(rem, C.c_int64, m)[:] = r
        _arr(retry, C.c_int64, m)[:] = ra
        _arr(reset, C.c_int64, m)[:] = rs
        log.append(m)
        return 0
    return fn


def hammer(co, nthreads, subs_per_thread, max_sub, nkeys, ncfg, seed, span_ns=50 * NS):
    """Threads submit random chunks and wait for them; returns every
    (ticket, inputs, results) record."""
    out, lock, errors = [], threading.Lock(), []

    def worker(tid):
        rng = np.random.default_rng(seed + tid)
        for _ in range(subs_per_thread):
            m = int(rng.integers(1, max_sub + 1))
            key = rng.integers(0, nkeys, m).astype(np.uint64)
            ts = (T0 + rng.integers(0, span_ns, m)).astype(np.int64)
            n = rng.choice([1, 1, 1, 2, 3], m).astype(np.int64)
            cfg = (key % ncfg).astype(np.uint32)
            t = co.submit(key, ts, n, cfg)
            rc, res = co.wait(t, m)
            if rc != 0:
                errors.append(rc)
            with lock:
                out.append((t, key, ts, n, cfg, res))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    return out


def check_against_oracle(oracle_mod, configs, recs):
    recs.sort(key=lambda r: r[0])
    # tickets are the sequence numbers of each submission's first request (a
    # Reset or table operation in between takes one number of its own)
    seq = 0
    for t, key, *_ in recs:
        assert t >= seq
        seq = t + key.size
    cat = [np.concatenate([r[i] for r in recs]) for i in (1, 2, 3, 4)]
    sim = oracle_mod.OracleSim(oracle_mod.REDIS7)
    for a, L, W in configs:
        sim.add_config(a, L, W)
    dec, rem, retry, reset, _ = sim.decide(*cat)
    got = [np.concatenate([r[5][i] for r in recs]) for i in range(4)]
    assert np.array_equal(got[0], dec)
    assert np.array_equal(got[1], rem)
    assert np.array_equal(got[2], retry)
    assert np.array_equal(got[3], reset)


def test_concurrent_submitters_match_sequential_oracle(rl, oracle_mod):
    log = []
    co = rl.Coalescer(oracle_backend(oracle_mod, CONFIGS, log), max_batch=64, max_in_flight=3)
    recs = hammer(co, nthreads=6, subs_per_thread=60, max_sub=40, nkeys=30, ncfg=len(CONFIGS), seed=11)
    st = co.stats()
    co.close()
    total = sum(r[1].size for r in recs)
    assert st.submitted == total and st.decided == total and st.pending == 0
    assert max(log) <= 64 and sum(log) == total
    assert st.batches == len(log)
    check_against_oracle(oracle_mod, CONFIGS, recs)


def test_submissions_split_across_batches(rl, oracle_mod):
    log = []
    co = rl.Coalescer(oracle_backend(oracle_mod, CONFIGS, log), max_batch=7, max_in_flight=2)
    recs = hammer(co, nthreads=3, subs_per_thread=20, max_sub=50, nkeys=5, ncfg=len(CONFIGS), seed=5)
    co.close()
    assert max(log) <= 7
    assert any(r[1].size > 7 for r in recs)
    check_against_oracle(oracle_mod, CONFIGS, recs)


def test_single_decide_and_edge_cases(rl, oracle_mod):
    log = []
    co = rl.Coalescer(oracle_backend(oracle_mod, CONFIGS, log), max_batch=16, queue_cap=10)
    # one Allow: the first request of a token bucket of capacity 20
    rc, (d, rem, retry, reset) = co.decide(42, T0, 1, 0)
    assert rc == 0 and d == rl.ALLOWED and rem == 19 and retry == 0
    # empty submission: a unique ticket that is done at once
    t0 = co.submit(np.zeros(0, np.uint64), np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint32))
    rc, res = co.wait(t0, 0)
    assert rc == 0 and all(x.size == 0 for x in res)
    # unknown ticket, and a ticket waited for twice
    assert co.wait(10 ** 12, 1)[0] == rl.RL_EINVAL
    assert co.wait(t0, 0)[0] == rl.RL_EINVAL
    # queue capacity
    with pytest.raises(rl.EngineError) as ei:
        co.submit(np.arange(11, dtype=np.uint64), np.full(11, T0, np.int64), np.ones(11, np.int64),
                  np.zeros(11, np.uint32))
    assert ei.value.code == rl.RL_EAGAIN
    co.close()


def test_backend_error_reaches_every_waiter(rl):
    def failing(user, m, *ptrs):
        return -5   # RL_EDEVICE
    co = rl.Coalescer(failing, max_batch=8)
    ts = [co.submit(np.arange(5, dtype=np.uint64), np.full(5, T0, np.int64), np.ones(5, np.int64),
                    np.zeros(5, np.uint32)) for _ in range(4)]
    assert [co.wait(t, 5)[0] for t in ts] == [-5] * 4
    co.close()


@pytest.mark.gpu
def test_gpu_coalescer_matches_sequential_oracle(rl, oracle_mod):
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 12, win_capacity=1 << 12, max_batch=1 << 12,
                    device=0, flags=rl.OPT_PIPELINE)
    for a, L, W in CONFIGS:
        eng.register(a, L, W)
    co = rl.Coalescer(eng, max_batch=1 << 12, max_in_flight=3)
    recs = hammer(co, nthreads=8, subs_per_thread=40, max_sub=64, nkeys=50, ncfg=len(CONFIGS), seed=21)
    rc, (d, rem, retry, reset) = co.decide(7, T0 + 51 * NS, 1, 0)
    st = co.stats()
    co.close()
    assert rc == 0
    assert eng.sync() == 0
    eng.close()
    total = sum(r[1].size for r in recs)
    assert st.decided == total + 1
    check_against_oracle(oracle_mod, CONFIGS, recs)


@pytest.mark.gpu
def test_gpu_coalescer_hot_key_batches(rl, oracle_mod):
    """One hot key under concurrency: batches large enough to take the
    engine's cooperative replay paths, still equal to the sequential oracle."""
    cfgs = CONFIGS[:1]
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 12, win_capacity=1 << 10, max_batch=1 << 14,
                    device=0, flags=rl.OPT_PIPELINE)
    for a, L, W in cfgs:
        eng.register(a, L, W)
    co = rl.Coalescer(eng, max_batch=1 << 14, max_in_flight=3, linger_ns=200_000)
    recs = hammer(co, nthreads=4, subs_per_thread=10, max_sub=3000, nkeys=1, ncfg=1, seed=3)
    co.close()
    assert eng.sync() == 0
    eng.close()
    check_against_oracle(oracle_mod, cfgs, recs)


# ---------------------------------------------------------------------------
# contexts: deadlines and cancellation (interface.go:75; the cancelled-ctx case
# of interface_test.go:267-275).  A submission whose context ends before it is
# launched never reaches the store; one already launched is applied.
# ---------------------------------------------------------------------------

class GatedOracle:
    """the oracle as the coalescer's host backend, with a gate: while closed,
    the submitter thread blocks inside the backend call (a batch on the GPU)"""

    def __init__(self, oracle_mod, configs):
        self.sim = oracle_mod.OracleSim(oracle_mod.REDIS7)
        for a, L, W in configs:
            self.sim.add_config(a, L, W)
        self.gate = threading.Event()
        self.gate.set()
        self.entered = threading.Event()
        self.applied = []   # (key, ts, n, cfg) of every request the store saw, in order

    def batch(self, user, m, key, ts, n, cfg, dec, rem, retry, reset):
        self.entered.set()
        self.gate.wait(30)
        k, t, nn, c = (_arr(key, C.c_uint64, m).copy(), _arr(ts, C.c_int64, m).copy(),
                       _arr(n, C.c_int64, m).copy(), _arr(cfg, C.c_uint32, m).copy())
        d, r, ra, rs, _ = self.sim.decide(k, t, nn, c)
        _arr(dec, C.c_uint8, m)[:] = d
        _arr(rem, C.c_int64, m)[:] = r
        _arr(retry, C.c_int64, m)[:] = ra
        _arr(reset, C.c_int64, m)[:] = rs
        self.applied += list(zip(k.tolist(), t.tolist(), nn.tolist(), c.tolist()))
        return 0


def _one(key, t, n=1, cfg=0):
    return (np.array([key], np.uint64), np.array([t], np.int64), np.array([n], np.int64), np.array([cfg], np.uint32))


def test_deadline_before_launch_is_never_applied(rl, oracle_mod):
    """expired while queued behind a busy engine: RL_EDEADLINE, and the
    store never sees it -- later decisions equal an oracle without it"""
    be = GatedOracle(oracle_mod, CONFIGS[:1])
    co = rl.Coalescer(be.batch, max_batch=8, max_in_flight=1)
    be.gate.clear()
    t_block = co.submit(*_one(1, T0))                    # occupies the engine
    assert be.entered.wait(10)
    dl = rl.now_ns() + 30_000_000
    t_exp = [co.submit(*_one(7, T0 + i + 1), deadline_ns=dl) for i in range(3)]
    t_live = co.submit(*_one(7, T0 + 10))                # no deadline: applied
    # a waiter wakes at the deadline and withdraws its submission
    rc, _ = co.wait(t_exp[0], 1)
    assert rc == rl.RL_EDEADLINE and rl.now_ns() >= dl
    import time
    time.sleep(0.05)                                     # the others expire unwaited
    be.gate.set()
    assert co.wait(t_block, 1)[0] == 0
    rc, (d, rem, _, _) = co.wait(t_live, 1)
    # token bucket 20/12s: the live request is key 7's first, so 19 remain
    assert rc == 0 and d[0] == rl.ALLOWED and rem[0] == 19
    assert [co.wait(t, 1)[0] for t in t_exp[1:]] == [rl.RL_EDEADLINE] * 2
    st = co.stats()
    co.close()
    assert st.expired == 3 and st.decided == 2
    assert [a[1] for a in be.applied] == [T0, T0 + 10]


def test_cancel_before_and_after_launch(rl, oracle_mod):
    """ctx.Done(): a queued submission is dropped (RL_ECANCELED, never
    applied); a launched one returns RL_ECANCELED at once and is applied"""
    be = GatedOracle(oracle_mod, CONFIGS[:1])
    co = rl.Coalescer(be.batch, max_batch=8, max_in_flight=1)
    be.gate.clear()
    t_launched = co.submit(*_one(3, T0, n=5))
    assert be.entered.wait(10)
    t_queued = co.submit(*_one(3, T0 + 1, n=7))
    # cancel from another thread while the caller blocks in wait
    res = {}
    w = threading.Thread(target=lambda: res.setdefault("q", co.wait(t_queued, 1)[0]))
    w.start()
    import time
    time.sleep(0.02)
    assert co.cancel(t_queued) == 0
    w.join(10)
    assert res["q"] == rl.RL_ECANCELED
    # the launched one: the waiter returns at once, the EVAL still lands
    assert co.cancel(t_launched) == 0
    assert co.wait(t_launched, 1)[0] == rl.RL_ECANCELED
    be.gate.set()
    rc, (d, rem, _, _) = co.decide(3, T0 + 2, 1, 0)
    assert rc == 0 and d == rl.ALLOWED and rem == 20 - 5 - 1   # the n=7 never happened
    # cancelling an unknown ticket / a completed one
    assert co.cancel(10 ** 12) == rl.RL_EINVAL
    t = co.submit(*_one(4, T0 + 3))
    assert co.wait(t, 1)[0] == 0
    st = co.stats()
    co.close()
    assert st.cancelled == 1
    assert [a[2] for a in be.applied] == [5, 1, 1]


@pytest.mark.parametrize("how", ["cancel", "deadline"])
def test_split_submission_context_end_drops_the_rest(rl, oracle_mod, how):
    """a submission larger than max_batch, split across launches, whose context
    ends after its first launch: the launched part is applied (an EVAL already
    sent), the part not launched yet never reaches the store"""
    be = GatedOracle(oracle_mod, CONFIGS[:1])
    co = rl.Coalescer(be.batch, max_batch=8, max_in_flight=1)
    be.gate.clear()
    m = 20
    keys = np.full(m, 5, np.uint64)
    ts = T0 + np.arange(m, dtype=np.int64)
    dl = rl.now_ns() + 40_000_000 if how == "deadline" else 0
    t = co.submit(keys, ts, np.ones(m, np.int64), np.zeros(m, np.uint32), deadline_ns=dl)
    assert be.entered.wait(10)                      # the first 8 are on the "GPU"
    if how == "cancel":
        assert co.cancel(t) == 0
        assert co.wait(t, 1)[0] == rl.RL_ECANCELED
    else:
        assert co.wait(t, 1)[0] == rl.RL_EDEADLINE
    be.gate.set()
    rc, (d, rem, _, _) = co.decide(5, T0 + 100, 1, 0)
    assert rc == 0 and d == rl.ALLOWED and rem == 20 - 8 - 1   # the other 12 never happened
    st = co.stats()
    co.close()
    assert [a[0] for a in be.applied] == [5] * 9
    assert (st.cancelled if how == "cancel" else st.expired) == 12


def test_split_submission_deadline_unwaited_returns_the_deadline(rl, oracle_mod):
    """the submitter truncates a split submission whose deadline passed while
    its rest was queued and nobody waited (the gRPC server collects only after
    completion): wait() then returns RL_EDEADLINE and copies no results -- the
    tail never ran, so its result slots hold nothing of this submission"""
    import time
    be = GatedOracle(oracle_mod, CONFIGS[:1])
    co = rl.Coalescer(be.batch, max_batch=8, max_in_flight=1)
    # a pooled submission buffer left holding another request's results
    t_prev = co.submit(np.arange(20, dtype=np.uint64) + 100, np.full(20, T0, np.int64), np.ones(20, np.int64),
                       np.zeros(20, np.uint32))
    assert co.wait(t_prev, 20)[0] == 0
    be.entered.clear()
    be.gate.clear()
    m = 20
    t = co.submit(np.full(m, 5, np.uint64), T0 + 1 + np.arange(m, dtype=np.int64), np.ones(m, np.int64),
                  np.zeros(m, np.uint32), deadline_ns=rl.now_ns() + 30_000_000)
    assert be.entered.wait(10)                      # the first 8 are on the "GPU"
    time.sleep(0.06)                                # the deadline passes; nobody waits
    be.gate.set()
    time.sleep(0.1)                                 # the submitter meets the rest after the deadline
    sentinel = (np.full(m, 0xAB, np.uint8),) + tuple(np.full(m, -7, np.int64) for _ in range(3))
    rc = None
    for _ in range(200):                            # completion without a waiter
        rc, _ = co.wait(t, m, timeout_ns=0, out=sentinel)
        if rc != rl.RL_ETIMEOUT:
            break
        time.sleep(0.01)
    assert rc == rl.RL_EDEADLINE
    assert (sentinel[0] == 0xAB).all() and all((x == -7).all() for x in sentinel[1:])   # nothing copied
    assert co.wait(t, m)[0] == rl.RL_EINVAL         # the ticket is released
    rc, (d, rem, _, _) = co.decide(5, T0 + 100, 1, 0)
    st = co.stats()
    co.close()
    assert rc == 0 and rem == 20 - 8 - 1            # the other 12 never happened
    assert st.expired == 12


def test_cancelled_context_before_the_call(rl, oracle_mod):
    """interface_test.go:267-275: Allow with an already-cancelled context
    returns an error; the store is untouched"""
    be = GatedOracle(oracle_mod, CONFIGS[:1])
    co = rl.Coalescer(be.batch, max_batch=8)
    t = co.submit(*_one(9, T0), deadline_ns=rl.now_ns() - 1)   # deadline already passed
    assert co.wait(t, 1)[0] == rl.RL_EDEADLINE
    co.close()
    assert be.applied == []


def test_deadline_after_launch_is_applied(rl, oracle_mod):
    be = GatedOracle(oracle_mod, CONFIGS[:1])
    co = rl.Coalescer(be.batch, max_batch=8, max_in_flight=1)
    be.gate.clear()
    t = co.submit(*_one(5, T0, n=4), deadline_ns=rl.now_ns() + 40_000_000)
    assert be.entered.wait(10)
    assert co.wait(t, 1)[0] == rl.RL_EDEADLINE   # go-redis: ctx error while the reply is pending
    be.gate.set()
    rc, (d, rem, _, _) = co.decide(5, T0 + 1, 1, 0)
    co.close()
    assert rc == 0 and rem == 20 - 4 - 1


def test_deadlines_under_concurrency_match_the_oracle(rl, oracle_mod):
    """many threads, random tight deadlines and cancels: every completed
    request equals a sequential oracle over exactly the applied requests"""
    log = []
    be = GatedOracle(oracle_mod, CONFIGS)
    co = rl.Coalescer(be.batch, max_batch=16, max_in_flight=2)
    recs, lock = [], threading.Lock()

    def worker(tid):
        rng = np.random.default_rng(100 + tid)
        for _ in range(80):
            m = int(rng.integers(1, 6))
            key = rng.integers(0, 12, m).astype(np.uint64)
            ts = (T0 + rng.integers(0, 20 * NS, m)).astype(np.int64)
            n = rng.choice([1, 1, 2], m).astype(np.int64)
            cfg = (key % len(CONFIGS)).astype(np.uint32)
            mode = rng.integers(0, 4)
            dl = 0 if mode == 0 else rl.now_ns() + int(rng.integers(0, 400_000))
            t = co.submit(key, ts, n, cfg, deadline_ns=dl)
            if mode == 3:
                co.cancel(t)
            rc, res = co.wait(t, m)
            with lock:
                recs.append((t, key, ts, n, cfg, rc, res))
    th = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    st = co.stats()
    co.close()
    assert st.pending == 0
    assert {r[5] for r in recs} <= {0, rl.RL_EDEADLINE, rl.RL_ECANCELED}
    # replay exactly what the store applied, in its order: completed
    # submissions' results must match it
    ap = be.applied
    sim = oracle_mod.OracleSim(oracle_mod.REDIS7)
    for a, L, W in CONFIGS:
        sim.add_config(a, L, W)
    k, t, n, c = (np.array(x) for x in zip(*ap))
    dec, rem, retry, reset, _ = sim.decide(k.astype(np.uint64), t, n, c.astype(np.uint32))
    by_req = {}
    for i, (kk, tt, nn, cc) in enumerate(ap):
        by_req.setdefault((kk, tt, nn, cc), []).append((dec[i], rem[i], retry[i], reset[i]))
    completed = [r for r in recs if r[5] == 0]
    assert completed, "no submission completed"
    for _, key, ts, n, cfg, _, res in completed:
        for j in range(key.size):
            opts = by_req[(int(key[j]), int(ts[j]), int(n[j]), int(cfg[j]))]
            assert (res[0][j], res[1][j], res[2][j], res[3][j]) in opts
    # every applied request belongs to a submission that was not dropped
    dropped = sum(r[1].size for r in recs if r[5] != 0)
    assert len(ap) + st.expired + st.cancelled == sum(r[1].size for r in recs)
    assert st.expired + st.cancelled <= dropped


# ---------------------------------------------------------------------------
# table GC from the serving path (Redis active expiry; tokenbucket.go:49,170,
# fixedwindow.go:24-26,151, slidingwindow.go:25-28,161-162)
# ---------------------------------------------------------------------------

class FakeTables:
    """a host stand-in for the engine's state tables: slots are claimed by
    new keys, live while their TTL runs, reclaimed only by gc (what the
    coalescer's automatic GC policy sees through rl_table_info_get)"""

    TTL_MS = 2000

    def __init__(self, rl, cap):
        self.rl = rl
        self.cap = cap
        self.keys = {}          # key -> expiry ms
        self.max_used = 0
        self.gcs = []           # (now_ms, new capacity)
        self.min_sms_after = []  # per gc: the smallest server clock of a later request
        self.sms = []           # server clocks of every request, in order

    def batch(self, user, m, key, ts, n, cfg, dec, rem, retry, reset):
        k = _arr(key, C.c_uint64, m)
        t = _arr(ts, C.c_int64, m)
        for i in range(m):
            sms = int(t[i]) // 1_000_000
            self.sms.append(sms)
            self.keys[int(k[i])] = sms + self.TTL_MS
        if len(self.keys) > self.cap:
            return self.rl.RL_ENOMEM
        self.max_used = max(self.max_used, len(self.keys))
        _arr(dec, C.c_uint8, m)[:] = 1
        return 0

    def _info(self, now_ms, out):
        live = sum(1 for x in self.keys.values() if x >= now_ms)
        for a in ("tb", "win", "spill"):
            setattr(out.contents, a + "_capacity", self.cap)
        out.contents.tb_used, out.contents.tb_live = len(self.keys), live

    def table_info(self, user, now_ms, out):
        self._info(now_ms, out)
        return 0

    def gc(self, user, now_ms, tb_cap, win_cap, out):
        self.gcs.append((now_ms, tb_cap, len(self.sms)))
        keep = {k: x for k, x in self.keys.items() if x >= now_ms}
        cap = tb_cap or self.cap
        if len(keep) > cap:
            return self.rl.RL_ENOMEM
        self.keys, self.cap = keep, cap
        self._info(now_ms, out)
        return 0


def test_automatic_gc_keeps_the_table_from_filling(rl):
    """uniform new keys far beyond the table's capacity: the coalescer counts
    and collects before any table passes its high-water mark, grows the table
    when live keys need it, and every GC's server clock is at or below every
    later request's (the condition for decisions to stay exact)"""
    tab = FakeTables(rl, 4096)
    co = rl.Coalescer(tab.batch, max_batch=256, max_in_flight=2, table_info=tab.table_info, gc=tab.gc,
                      gc_interval_ns=10 ** 12, gc_high_pct=50, gc_margin_ms=50)
    rng = np.random.default_rng(1)
    t = T0
    nkeys = 0
    for step in range(400):
        m = int(rng.integers(1, 200))
        key = (nkeys + np.arange(m)).astype(np.uint64)      # every request a new key
        nkeys += m
        # 4 requests per ms of server time: keys live ~8k requests (2 s TTL);
        # the clock advances monotonically with jitter below the margin
        ts = (t + np.arange(m) * 250_000 + rng.integers(0, 20_000_000, m)).astype(np.int64)
        t += m * 250_000
        tk = co.submit(key, ts, np.ones(m, np.int64), np.zeros(m, np.uint32))
        assert co.wait(tk, m)[0] == 0, step
    st = co.stats()
    co.close()
    assert nkeys > 4 * 4096
    assert st.gc_runs >= 3 and st.gc_failures == 0
    assert tab.max_used <= 0.5 * tab.cap + 256
    # live keys (~8k) need a larger table than 4096 at 50 %: it grew
    assert tab.cap >= 16384
    for now_ms, _, nreq in tab.gcs:
        assert now_ms <= min(tab.sms[nreq:], default=now_ms)


def test_manual_gc_and_table_info_are_ordered(rl):
    tab = FakeTables(rl, 1 << 12)
    co = rl.Coalescer(tab.batch, max_batch=64, table_info=tab.table_info, gc=tab.gc)
    tk = co.submit(np.arange(100, dtype=np.uint64), np.full(100, T0, np.int64), np.ones(100, np.int64),
                   np.zeros(100, np.uint32))
    rc, info = co.table_info(T0 // 1_000_000)
    assert rc == 0 and info.tb_used == 100 and info.tb_live == 100   # after the submission before it
    assert co.wait(tk, 100)[0] == 0
    rc, info = co.gc(T0 // 1_000_000 + 10_000, 1 << 13)
    assert rc == 0 and info.tb_used == 0 and info.tb_capacity == 1 << 13
    rc, _ = co.gc(0, 1 << 13)
    assert rc == 0
    st = co.stats()
    co.close()
    assert st.gc_runs == 2
    # a backend without table functions: RL_EINVAL
    co = rl.Coalescer(tab.batch, max_batch=64)
    assert co.table_info(0)[0] == rl.RL_EINVAL and co.gc(0)[0] == rl.RL_EINVAL
    co.close()


def test_abi_struct_sizes_are_checked(rl):
    import ctypes as Cc
    o = rl.rl_coalescer_opts()
    o.struct_size = 8
    h = Cc.c_void_p()
    be = rl.rl_coalescer_backend(batch=rl.BATCH_FN(lambda *a: 0))
    assert rl.lib.rl_coalescer_create_with_host_backend(Cc.byref(be), Cc.byref(o), Cc.byref(h)) == rl.RL_EINVAL
    co = rl.Coalescer(lambda *a: 0)
    st = rl.rl_coalescer_stats()
    st.struct_size = 24   # an older caller: only the first fields are written
    st.batches = 12345
    assert rl.lib.rl_coalescer_get_stats(co.h, Cc.byref(st)) == 0
    assert st.batches == 12345 and st.struct_size == 24
    st.struct_size = 0
    assert rl.lib.rl_coalescer_get_stats(co.h, Cc.byref(st)) == rl.RL_EINVAL
    # a newer caller (struct larger than the library's): struct_size comes back
    # as the bytes the library filled in, and the trailing bytes are untouched
    big = (Cc.c_uint8 * (Cc.sizeof(rl.rl_coalescer_stats) + 64))()
    Cc.memset(big, 0xAB, Cc.sizeof(big))
    Cc.cast(big, Cc.POINTER(Cc.c_uint32))[0] = Cc.sizeof(big)
    assert rl.lib.rl_coalescer_get_stats(co.h, Cc.cast(big, Cc.POINTER(rl.rl_coalescer_stats))) == 0
    assert Cc.cast(big, Cc.POINTER(Cc.c_uint32))[0] == Cc.sizeof(rl.rl_coalescer_stats)
    assert bytes(big[Cc.sizeof(rl.rl_coalescer_stats):]) == b"\xab" * 64
    co.close()
    bad = rl.rl_opts(max_batch=16)
    bad.struct_size = 16
    e = Cc.c_void_p()
    assert rl.lib.rl_engine_create(Cc.byref(bad), Cc.byref(e)) == rl.RL_EINVAL


@pytest.mark.gpu
def test_gpu_coalescer_gc_many_more_keys_than_slots(rl, oracle_mod):
    """§8f rank 2 on the serving path: tables of 4096 slots, ~8x as many
    distinct keys over the run (all three algorithms, 1-2 s windows, time
    moving forward with sub-margin jitter), automatic GC plus a manual one:
    every decision equals the sequential oracle, no RL_ENOMEM"""
    cfgs = [(1, 5, NS), (3, 4, NS), (2, 3, 2 * NS)]
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=4096, win_capacity=4096, max_batch=1 << 13,
                    device=0, flags=rl.OPT_PIPELINE)
    for a, L, W in cfgs:
        eng.register(a, L, W)
    co = rl.Coalescer(eng, max_batch=1 << 13, max_in_flight=3, gc_interval_ns=10 ** 12, gc_high_pct=50,
                      gc_margin_ms=100)
    rng = np.random.default_rng(8)
    recs = []
    t = T0
    base = 0
    for step in range(240):
        m = int(rng.integers(1, 800))
        # a sliding key range: keys stay hot for a while, then go cold and expire
        key = (base + rng.integers(0, 3000, m)).astype(np.uint64)
        base += 170
        ts = (t + np.sort(rng.integers(0, 40_000_000, m))).astype(np.int64)
        t += 40_000_000
        n = rng.choice([1, 1, 2], m).astype(np.int64)
        cfg = (key % 3).astype(np.uint32)
        tk = co.submit(key, ts, n, cfg)
        rc, res = co.wait(tk, m)
        assert rc == 0, (step, rc)
        recs.append((tk, key, ts, n, cfg, res))
        if step == 120:
            rc, info = co.gc(int(t // 1_000_000) - 1000)
            assert rc == 0
    st = co.stats()
    co.close()
    assert eng.sync() == 0
    info = eng.table_info(int(t // 1_000_000))
    eng.close()
    distinct = len(np.unique(np.concatenate([r[1] for r in recs])))
    assert distinct > 4 * 4096 * 2
    assert st.gc_runs >= 3 and st.gc_failures == 0, (st.gc_runs, st.gc_failures)
    check_against_oracle(oracle_mod, cfgs, recs)


@pytest.mark.gpu
def test_gpu_coalescer_gc_budgets_each_table(rl, oracle_mod):
    """the automatic GC budgets each table by the requests that can insert
    into it (rl_config_table): token-bucket traffic in batches far larger than
    a tiny window table's headroom triggers no GC and few counts (round 3: a
    1024-slot window table made every batch of a token-bucket server count,
    then collect, the tables)"""
    cfgs = [(1, 20, 12 * NS), (3, 100, 60 * NS)]
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 16, win_capacity=1024, max_batch=1 << 13,
                    device=0, flags=rl.OPT_PIPELINE)
    for a, L, W in cfgs:
        eng.register(a, L, W)
    co = rl.Coalescer(eng, max_batch=1 << 13, max_in_flight=3, gc_interval_ns=10 ** 12, gc_high_pct=50)
    rng = np.random.default_rng(21)
    recs = []
    t = T0
    for step in range(40):
        m = 4000
        key = rng.integers(0, 20_000, m).astype(np.uint64)
        ts = (t + np.sort(rng.integers(0, 1_000_000, m))).astype(np.int64)
        t += 1_000_000
        n = np.ones(m, np.int64)
        cfg = np.zeros(m, np.uint32)
        if step % 10 == 9:                 # a few window requests now and then
            cfg[:50] = 1
        tk = co.submit(key, ts, n, cfg)
        rc, res = co.wait(tk, m)
        assert rc == 0, (step, rc)
        recs.append((tk, key, ts, n, cfg, res))
    st = co.stats()
    co.close()
    assert eng.sync() == 0
    eng.close()
    assert st.gc_runs == 0, st.gc_runs
    assert st.gc_checks <= 20, st.gc_checks     # (every batch before: 40)
    check_against_oracle(oracle_mod, cfgs, recs)
