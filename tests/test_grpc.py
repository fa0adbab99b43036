"""The gRPC service (api/proto/ratelimiter.proto, python/rl_server.py):
Allow / AllowN / Reset / AllowBatch / Health over a real gRPC channel.  On
the CPU the coalescer runs over its test seam with the CPU oracle as the
store (test infrastructure); on the GPU over the HIP engine.  Decisions must
equal the oracle's for the same requests at the same (injected) clock."""
import threading

import grpc
import numpy as np
import pytest

import oracle
import rl_amd
import rl_grpc
import rl_server
from tracegen import NS, T0

LIMITERS = ["fw:fixed_window:5:60s", "sw:sliding_window:3:2s:api", "tb:token_bucket:5:60s",
            "tb2:token_bucket:10:10s::true", "fwc:fixed_window:4:1s"]


class Clock:
    """deterministic time.Now(): advances 1.25 ms per read; records reads"""

    def __init__(self):
        self.t = T0
        self.lock = threading.Lock()

    def __call__(self):
        with self.lock:
            self.t += 1_250_000
            return self.t


class OracleStore:
    """the coalescer's host backend: the CPU oracle, keyed by engine key ids"""

    def __init__(self, fail=False):
        self.sim = oracle.OracleSim(oracle.REDIS7)
        self.fail = fail
        self.lock = threading.Lock()
        self.gate = threading.Event()   # cleared: the store hangs (a busy engine)
        self.gate.set()
        self.entered = threading.Event()
        self.applied = 0

    def register(self, alg, limit, window):
        return self.sim.add_config(alg, limit, window)

    def batch(self, user, m, key, ts, n, cfg, dec, rem, retry, reset):
        import ctypes
        if self.fail:
            return rl_amd.RL_EDEVICE
        self.entered.set()
        self.gate.wait(30)
        self.applied += m

        def arr(p, ct, dt):
            return np.ctypeslib.as_array((ct * m).from_address(p)).view(dt)
        d, r, rt, rs, _ = self.sim.decide(arr(key, ctypes.c_uint64, np.uint64), arr(ts, ctypes.c_int64, np.int64),
                                          arr(n, ctypes.c_int64, np.int64), arr(cfg, ctypes.c_uint32, np.uint32))
        arr(dec, ctypes.c_uint8, np.uint8)[:] = d
        arr(rem, ctypes.c_int64, np.int64)[:] = r
        arr(retry, ctypes.c_int64, np.int64)[:] = rt
        arr(reset, ctypes.c_int64, np.int64)[:] = rs
        return rl_amd.RL_OK

    def reset(self, user, cfg, key, ts):
        self.sim.reset(cfg, key, ts)
        return rl_amd.RL_OK


def start(service):
    stop = threading.Event()
    ready = threading.Event()
    port = []

    def run():
        rl_server.serve(service, "127.0.0.1:0", workers=16, grace_s=1.0,
                        ready=lambda p: (port.append(p), ready.set()), stop_event=stop)
    th = threading.Thread(target=run, daemon=True)
    th.start()
    assert ready.wait(30)
    ch = grpc.insecure_channel(f"127.0.0.1:{port[0]}")
    return ch, stop, th


@pytest.fixture
def cpu_server():
    store = OracleStore()
    co_box = []
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse(s) for s in LIMITERS], None, store.register,
                                       clock=Clock())
    co = rl_amd.Coalescer(store.batch, max_batch=256, reset=store.reset)
    svc.co = co
    co_box.append(co)
    ch, stop, th = start(svc)
    yield svc, ch
    ch.close()
    stop.set()
    th.join(10)
    co.close()


def _ns(svc, limiter, key):
    """the Redis key identity: FormatKey(prefix, key) -- limiters with one
    prefix share it (config.go:81-87)"""
    return (svc.by_name[limiter].prefix, key)


def _shadow(svc):
    """an oracle fed with the service's own key ids and clock readings"""
    sim = oracle.OracleSim(oracle.REDIS7)
    ids = {}
    for lim in sorted(svc.by_name.values(), key=lambda x: x.cfg_id):
        ids[lim.name] = sim.add_config(lim.alg, lim.limit, lim.window_ns)
    return sim, ids


def test_proto_matches_service():
    a = rl_grpc.api()
    assert [m for m, _, _ in a.services["RateLimiter"]] == ["Allow", "AllowN", "Reset", "AllowBatch"]
    f = {x.name: x.number for x in a.AllowResponse.DESCRIPTOR.fields}
    assert f == {"allowed": 1, "limit": 2, "remaining": 3, "retry_after_ns": 4, "reset_at_unix_ns": 5, "error": 6}


def test_parse_duration_and_reset_at():
    assert rl_server.parse_duration("1m30s") == 90 * NS
    assert rl_server.parse_duration("500ms") == 500_000_000
    sim = oracle.OracleSim(0)
    for i, (a, L, W) in enumerate([(1, 5, 60 * NS), (2, 3, 2 * NS), (3, 4, 7 * NS), (1, 20, 12 * NS)]):
        sim.add_config(a, L, W)
        for t in (T0, T0 + 123_456_789, T0 + 7 * NS - 1):
            _, _, _, reset, _ = sim.decide([100 + i], [t], [1], [i])
            assert rl_server.reset_at_ns(a, L, W, t) == reset[0]


def test_fixed_window_allow_sequence(cpu_server):
    svc, ch = cpu_server
    st = rl_grpc.rate_limiter_stub(ch)
    rems = [st.Allow(svc.a.AllowRequest(limiter="fw", key="user:1")).remaining for _ in range(5)]
    assert rems == [4, 3, 2, 1, 0]            # fixedwindow_integration_test.go:27-65
    r = st.Allow(svc.a.AllowRequest(limiter="fw", key="user:1"))
    assert not r.allowed and r.remaining == 0 and r.retry_after_ns > 0 and r.limit == 5


def test_allow_n_reset_and_errors(cpu_server):
    svc, ch = cpu_server
    st = rl_grpc.rate_limiter_stub(ch)
    r = [st.AllowN(svc.a.AllowNRequest(limiter="tb", key="k", n=n)) for n in (3, 5, 3)]
    assert [(x.allowed, x.remaining) for x in r] == [(True, 2), (False, 2), (False, 2)]
    with pytest.raises(grpc.RpcError) as e:
        st.AllowN(svc.a.AllowNRequest(limiter="tb", key="k", n=0))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT and e.value.details() == rl_server.ERR_INVALID_N
    with pytest.raises(grpc.RpcError) as e:
        st.Allow(svc.a.AllowRequest(limiter="nope", key="k"))
    assert e.value.code() == grpc.StatusCode.NOT_FOUND
    # Reset: the bucket is full again (tokenbucket_integration_test.go:203-241)
    st.Reset(svc.a.ResetRequest(limiter="tb", key="k"))
    assert st.AllowN(svc.a.AllowNRequest(limiter="tb", key="k", n=5)).remaining == 0


def test_decisions_equal_the_oracle(cpu_server):
    """a random mix of RPCs (unary and batched, all limiters) == the oracle
    replaying the same requests at the service's clock readings"""
    svc, ch = cpu_server
    st = rl_grpc.rate_limiter_stub(ch)
    rng = np.random.default_rng(12)
    sim, cid = _shadow(svc)
    names = list(svc.by_name)
    ids = {}
    for step in range(120):
        clock_before = svc.clock.t
        if step % 3 == 0:
            reqs = [svc.a.AllowNRequest(limiter=names[rng.integers(len(names))], key=f"u{rng.integers(6)}",
                                        n=int(rng.choice([1, 1, 2, 0]))) for _ in range(rng.integers(1, 40))]
            got = st.AllowBatch(svc.a.AllowBatchRequest(requests=reqs)).results
            t = clock_before + 1_250_000
            ok = [i for i, r in enumerate(reqs) if r.n > 0]
            key = np.array([ids.setdefault(_ns(svc, reqs[i].limiter, reqs[i].key), len(ids)) for i in ok], np.uint64)
            d, rem, retry, reset, _ = sim.decide(key, np.full(len(ok), t, np.int64),
                                                 np.array([reqs[i].n for i in ok], np.int64),
                                                 np.array([cid[reqs[i].limiter] for i in ok], np.uint32))
            for j, i in enumerate(ok):
                g = got[i]
                assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                    (bool(d[j]), rem[j], retry[j], reset[j]), (step, i)
            for i, r in enumerate(reqs):
                if r.n <= 0:
                    assert got[i].error == rl_server.ERR_INVALID_N
        else:
            lim, key = names[rng.integers(len(names))], f"u{rng.integers(6)}"
            g = st.Allow(svc.a.AllowRequest(limiter=lim, key=key))
            t = clock_before + 1_250_000
            d, rem, retry, reset, _ = sim.decide([ids.setdefault(_ns(svc, lim, key), len(ids))], [t], [1], [cid[lim]])
            assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                (bool(d[0]), rem[0], retry[0], reset[0]), step


def test_health_and_graceful_shutdown():
    store = OracleStore()
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse(LIMITERS[0])], None, store.register, clock=Clock())
    svc.co = rl_amd.Coalescer(store.batch, max_batch=64, reset=store.reset)
    ch, stop, th = start(svc)
    h = rl_grpc.health_stub(ch)
    assert h.Check(svc.h.HealthCheckRequest()).status == 1
    assert h.Check(svc.h.HealthCheckRequest(service="other")).status == 3
    assert rl_grpc.rate_limiter_stub(ch).Allow(svc.a.AllowRequest(limiter="fw", key="a")).allowed
    stop.set()
    th.join(10)
    assert not th.is_alive() and not svc.serving
    ch.close()
    svc.co.close()


@pytest.mark.parametrize("fail_open", [True, False])
def test_storage_failure_fail_open_closed(fail_open):
    """an engine error: fail-open returns {Allowed, Limit, 0, 0, ResetAt},
    fail-closed returns "failed to check rate limit" (tokenbucket.go:100-112)"""
    store = OracleStore(fail=True)
    spec = "t:token_bucket:10:10s::" + ("true" if fail_open else "false")
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse(spec)], None, store.register, clock=Clock())
    svc.co = rl_amd.Coalescer(store.batch, max_batch=64, reset=store.reset)
    ch, stop, th = start(svc)
    st = rl_grpc.rate_limiter_stub(ch)
    if fail_open:
        r = st.Allow(svc.a.AllowRequest(limiter="t", key="a"))
        t = T0 + 1_250_000
        assert (r.allowed, r.limit, r.remaining, r.retry_after_ns) == (True, 10, 0, 0)
        assert r.reset_at_unix_ns == rl_server.reset_at_ns(1, 10, 10 * NS, t)
    else:
        with pytest.raises(grpc.RpcError) as e:
            st.Allow(svc.a.AllowRequest(limiter="t", key="a"))
        assert e.value.code() == grpc.StatusCode.UNAVAILABLE
        assert e.value.details().startswith("failed to check rate limit")
    stop.set()
    th.join(10)
    ch.close()
    svc.co.close()


@pytest.mark.gpu
def test_grpc_on_the_gpu_engine():
    """the production backend: engine + coalescer on cuda:0"""
    be = rl_server.GpuBackend(0, 1 << 12, 1 << 12, 1 << 12)
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse(s) for s in LIMITERS], None, be.register,
                                       clock=Clock())
    svc.co = be.start(1 << 12)
    ch, stop, th = start(svc)
    try:
        st = rl_grpc.rate_limiter_stub(ch)
        sim, cid = _shadow(svc)
        ids = {}
        rng = np.random.default_rng(5)
        for step in range(60):
            reqs = [svc.a.AllowNRequest(limiter=LIMITERS[rng.integers(len(LIMITERS))].split(":")[0],
                                        key=f"u{rng.integers(5)}", n=int(rng.choice([1, 2])))
                    for _ in range(rng.integers(1, 50))]
            t = svc.clock.t + 1_250_000
            got = st.AllowBatch(svc.a.AllowBatchRequest(requests=reqs)).results
            key = np.array([ids.setdefault(_ns(svc, r.limiter, r.key), len(ids)) for r in reqs], np.uint64)
            d, rem, retry, reset, _ = sim.decide(key, np.full(len(reqs), t, np.int64),
                                                 np.array([r.n for r in reqs], np.int64),
                                                 np.array([cid[r.limiter] for r in reqs], np.uint32))
            for j, g in enumerate(got):
                assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                    (bool(d[j]), rem[j], retry[j], reset[j]), (step, j)
            if step % 10 == 9:
                st.Reset(svc.a.ResetRequest(limiter="fw", key="u1"))
                sim.reset(cid["fw"], ids.setdefault(_ns(svc, "fw", "u1"), len(ids)), svc.clock.t)
    finally:
        ch.close()
        stop.set()
        th.join(10)
        be.close()


class FakeCtx:
    """a servicer context with a deadline time_remaining() seconds away"""

    def __init__(self, remaining):
        self.remaining = remaining

    def time_remaining(self):
        return self.remaining

    def abort(self, code, details):
        raise grpc.RpcError(code, details)


@pytest.mark.parametrize("fail_open", [True, False])
def test_expired_context_takes_the_error_branch(fail_open):
    """interface_test.go:267-275: a context already done -> error (fail-closed)
    or the fail-open result; the store never sees the request"""
    store = OracleStore()
    spec = "t:token_bucket:10:10s::" + ("true" if fail_open else "false")
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse(spec)], None, store.register, clock=Clock())
    svc.co = rl_amd.Coalescer(store.batch, max_batch=64, reset=store.reset)
    try:
        if fail_open:
            r = svc.Allow(svc.a.AllowRequest(limiter="t", key="a"), FakeCtx(0.0))
            assert (r.allowed, r.limit, r.remaining, r.retry_after_ns) == (True, 10, 0, 0)
        else:
            with pytest.raises(grpc.RpcError) as e:
                svc.Allow(svc.a.AllowRequest(limiter="t", key="a"), FakeCtx(0.0))
            assert e.value.args == (grpc.StatusCode.DEADLINE_EXCEEDED,
                                    "failed to check rate limit: context deadline exceeded")
        # AllowBatch: per-request errors
        rs = svc.AllowBatch(svc.a.AllowBatchRequest(requests=[svc.a.AllowNRequest(limiter="t", key="b", n=1)]),
                            FakeCtx(0.0)).results
        assert rs[0].allowed if fail_open else rs[0].error.endswith("context deadline exceeded")
        assert store.applied == 0
        # a live context is served
        r = svc.Allow(svc.a.AllowRequest(limiter="t", key="a"), FakeCtx(5.0))
        assert r.allowed and r.remaining == 9 and store.applied == 1
    finally:
        svc.co.close()


def test_short_deadlines_under_load_are_never_applied():
    """RPCs with a 50 ms deadline queue behind a hung store: the clients get
    DEADLINE_EXCEEDED, the requests are dropped before launch, and later
    decisions equal the oracle over the applied requests only"""
    store = OracleStore()
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse("tb:token_bucket:5:60s")], None, store.register,
                                       clock=Clock())
    svc.co = rl_amd.Coalescer(store.batch, max_batch=64, max_in_flight=1, reset=store.reset)
    ch, stop, th = start(svc)
    try:
        st = rl_grpc.rate_limiter_stub(ch)
        store.gate.clear()
        first = st.Allow.future(svc.a.AllowRequest(limiter="tb", key="k"))   # holds the store
        assert store.entered.wait(10)
        errs = []
        for _ in range(6):
            try:
                st.AllowN(svc.a.AllowNRequest(limiter="tb", key="k", n=2), timeout=0.05)
            except grpc.RpcError as e:
                errs.append(e.code())
        assert errs == [grpc.StatusCode.DEADLINE_EXCEEDED] * 6
        import time
        time.sleep(0.1)   # every server-side deadline has passed
        store.gate.set()
        assert first.result(10).remaining == 4
        r = st.Allow(svc.a.AllowRequest(limiter="tb", key="k"))
        assert r.allowed and r.remaining == 3      # none of the 6 x n=2 was applied
        s = svc.co.stats()
        assert s.expired == 6 and store.applied == 2
    finally:
        ch.close()
        stop.set()
        th.join(10)
        svc.co.close()


class FastClock(Clock):
    """time.Now() advancing 30 ms per read: keys expire during the run"""

    def __call__(self):
        with self.lock:
            self.t += 30_000_000
            return self.t


@pytest.mark.gpu
def test_grpc_gc_many_more_keys_than_slots():
    """the server collects its tables itself: 4096-slot tables, far more
    distinct keys over the run, every decision equal to the oracle"""
    lims = ["g1:token_bucket:5:1s", "g2:fixed_window:4:1s", "g3:sliding_window:3:1s:other"]
    be = rl_server.GpuBackend(0, 4096, 4096, 1 << 13)
    svc = rl_server.RateLimiterService([rl_server.Limiter.parse(s) for s in lims], None, be.register,
                                       clock=FastClock())
    svc.co = be.start(1 << 13, gc_interval_ns=10 ** 12, gc_margin_ms=100)
    ch, stop, th = start(svc)
    try:
        st = rl_grpc.rate_limiter_stub(ch)
        sim, cid = _shadow(svc)
        ids = {}
        rng = np.random.default_rng(9)
        base = 0
        for step in range(160):
            reqs = [svc.a.AllowNRequest(limiter=lims[rng.integers(3)].split(":")[0],
                                        key=f"u{base + rng.integers(2000)}", n=int(rng.choice([1, 2])))
                    for _ in range(rng.integers(200, 500))]
            base += 220
            t = svc.clock.t + 30_000_000
            got = st.AllowBatch(svc.a.AllowBatchRequest(requests=reqs)).results
            key = np.array([ids.setdefault(_ns(svc, r.limiter, r.key), len(ids)) for r in reqs], np.uint64)
            d, rem, retry, reset, _ = sim.decide(key, np.full(len(reqs), t, np.int64),
                                                 np.array([r.n for r in reqs], np.int64),
                                                 np.array([cid[r.limiter] for r in reqs], np.uint32))
            for j, g in enumerate(got):
                assert not g.error, (step, j, g.error)
                assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                    (bool(d[j]), rem[j], retry[j], reset[j]), (step, j)
        s = svc.co.stats()
        assert len(ids) > 4 * 2 * 4096
        assert s.gc_runs >= 2 and s.gc_failures == 0
    finally:
        ch.close()
        stop.set()
        th.join(10)
        be.close()
