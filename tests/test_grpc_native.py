"""The native gRPC front end (include/rl_grpc.h, host/grpc_server.cpp): the
same service as python/rl_server.py -- Allow / AllowN / Reset / AllowBatch /
Health over real gRPC channels (grpcio clients) -- served by C++ event loops
over the coalescer.  On the CPU the coalescer runs over its test seam with
the CPU oracle as the store (test infrastructure); on the GPU over the HIP
engine.  The server's time.Now() is its test clock (T0 + k * 1.25 ms on the
k-th read), so decisions must equal the oracle's for the same requests."""
import threading
import time

import grpc
import numpy as np
import pytest

import oracle
import rl_amd
import rl_grpc
import rl_server
from test_grpc import LIMITERS, OracleStore
from tracegen import NS, T0

STEP = 1_250_000


class Native:
    """a native server over a coalescer; `reads` counts its clock reads"""

    def __init__(self, specs, store=None, backend=None, max_batch=256, max_in_flight=3, io_threads=2,
                 isolate=False):
        self.lims = [rl_server.Limiter.parse(s) for s in specs]
        register = backend.register if backend is not None else store.register
        for lim in self.lims:
            lim.cfg_id = register(lim.alg, lim.limit, lim.window_ns)
        if backend is not None:
            self.co = backend.start(max_batch)
        else:
            self.co = rl_amd.Coalescer(store.batch, max_batch=max_batch, max_in_flight=max_in_flight,
                                       reset=store.reset)
        self.srv = rl_amd.GrpcServer(
            self.co, [(l.name, l.cfg_id, l.alg, l.limit, l.window_ns, l.prefix, l.fail_open) for l in self.lims],
            io_threads=io_threads, isolate=isolate, clock_start_ns=T0, clock_step_ns=STEP)
        self.ch = grpc.insecure_channel(f"127.0.0.1:{self.srv.port}")
        self.a = rl_grpc.api("ratelimiter.proto")
        self.h = rl_grpc.api("health.proto")
        self.st = rl_grpc.rate_limiter_stub(self.ch)
        self.reads = 0
        self.by_name = {l.name: l for l in self.lims}

    def t_next(self):
        """the time.Now() the next clock-reading RPC gets"""
        self.reads += 1
        return T0 + self.reads * STEP

    def close(self, backend=None):
        self.ch.close()
        self.srv.close()
        if backend is not None:
            backend.close()
        else:
            self.co.close()


def shadow(srv):
    sim = oracle.OracleSim(oracle.REDIS7)
    cid = {}
    for lim in sorted(srv.lims, key=lambda x: x.cfg_id):
        cid[lim.name] = sim.add_config(lim.alg, lim.limit, lim.window_ns)
    return sim, cid


@pytest.fixture
def native():
    store = OracleStore()
    srv = Native(LIMITERS, store)
    yield srv, store
    srv.close()


def test_native_fixed_window_allow_sequence(native):
    srv, _ = native
    rems = [srv.st.Allow(srv.a.AllowRequest(limiter="fw", key="user:1")).remaining for _ in range(5)]
    assert rems == [4, 3, 2, 1, 0]            # fixedwindow_integration_test.go:27-65
    r = srv.st.Allow(srv.a.AllowRequest(limiter="fw", key="user:1"))
    assert not r.allowed and r.remaining == 0 and r.retry_after_ns > 0 and r.limit == 5


def test_native_allow_n_reset_and_errors(native):
    srv, _ = native
    r = [srv.st.AllowN(srv.a.AllowNRequest(limiter="tb", key="k", n=n)) for n in (3, 5, 3)]
    assert [(x.allowed, x.remaining) for x in r] == [(True, 2), (False, 2), (False, 2)]
    with pytest.raises(grpc.RpcError) as e:
        srv.st.AllowN(srv.a.AllowNRequest(limiter="tb", key="k", n=0))
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT and e.value.details() == rl_server.ERR_INVALID_N
    with pytest.raises(grpc.RpcError) as e:
        srv.st.Allow(srv.a.AllowRequest(limiter="nope", key="k"))
    assert e.value.code() == grpc.StatusCode.NOT_FOUND and e.value.details() == "unknown limiter 'nope'"
    srv.st.Reset(srv.a.ResetRequest(limiter="tb", key="k"))   # tokenbucket_integration_test.go:203-241
    assert srv.st.AllowN(srv.a.AllowNRequest(limiter="tb", key="k", n=5)).remaining == 0


def _raw_h2_unary(port, path, body, extra_headers):
    """one gRPC unary call over a bare HTTP/2 connection (HPACK literals, no
    Huffman): lets a test send header values a gRPC client library never
    would; returns the response message, None when the call ended without
    one (an error status)"""
    import socket
    import struct

    def frame(ftype, flags, sid, payload):
        return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload

    def lit(name, value):        # literal header field without indexing, new name
        n, v = name.encode(), value.encode()
        assert len(n) < 127 and len(v) < 127
        return b"\x00" + bytes([len(n)]) + n + bytes([len(v)]) + v

    hdrs = [(":method", "POST"), (":scheme", "http"), (":path", path), (":authority", "127.0.0.1"),
            ("content-type", "application/grpc"), ("te", "trailers")] + extra_headers
    block = b"".join(lit(k, v) for k, v in hdrs)
    msg = b"\x00" + struct.pack(">I", len(body)) + body
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    s.sendall(b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n" + frame(4, 0, 0, b"") + frame(1, 4, 1, block) +
              frame(0, 1, 1, msg))
    buf = b""
    body_out, ended = None, False
    while not ended:
        chunk = s.recv(65536)
        assert chunk, "connection closed before the trailers"
        buf += chunk
        while len(buf) >= 9:
            ln = int.from_bytes(buf[:3], "big")
            if len(buf) < 9 + ln:
                break
            ftype, flags, sid, payload = buf[3], buf[4], int.from_bytes(buf[5:9], "big"), buf[9:9 + ln]
            buf = buf[9 + ln:]
            if ftype == 4 and not flags & 1:
                s.sendall(frame(4, 1, 0, b""))          # SETTINGS ack
            if sid == 1 and ftype == 0 and len(payload) >= 5:
                body_out = payload[5:]                 # the response message (a DATA frame)
            if sid == 1 and ftype in (0, 1) and flags & 1:
                ended = True                           # END_STREAM: the trailers (HPACK, not decoded here)
    s.close()
    return body_out


@pytest.mark.parametrize("timeout", ["2562047H", "99999999H", "99999999M"])
def test_native_huge_grpc_timeouts_are_no_deadline(native, timeout):
    """grpc-timeout values whose nanoseconds overflow int64 (grpc-go's
    2562047H maximum, 8-digit hour counts) saturate to no deadline instead of
    expiring the RPC at once (or overflowing)"""
    srv, _ = native
    body = srv.a.AllowRequest(limiter="fw", key="long-deadline-" + timeout).SerializeToString()
    out = _raw_h2_unary(srv.srv.port, "/ratelimiter.v1.RateLimiter/Allow", body, [("grpc-timeout", timeout)])
    assert out is not None, "the RPC ended without a response (deadline applied at once)"
    r = srv.a.AllowResponse.FromString(out)
    assert r.allowed and r.remaining == 4
    # and a tiny one still expires (the deadline is applied when it fits)
    assert srv.st.Allow(srv.a.AllowRequest(limiter="fw", key="after"), timeout=5).allowed


def test_native_decisions_equal_the_oracle(native):
    """a random mix of unary and batched RPCs over every limiter == the oracle
    replaying the same requests at the server's clock readings"""
    srv, _ = native
    rng = np.random.default_rng(12)
    sim, cid = shadow(srv)
    names = list(srv.by_name)
    ids = {}

    def kid(lim, key):      # FormatKey(prefix, key) is the identity (config.go:81-87)
        return ids.setdefault((srv.by_name[lim].prefix, key), len(ids))
    for step in range(150):
        if step % 3 == 0:
            reqs = [srv.a.AllowNRequest(limiter=names[rng.integers(len(names))], key=f"u{rng.integers(6)}",
                                        n=int(rng.choice([1, 1, 2, 0]))) for _ in range(rng.integers(1, 40))]
            if step % 9 == 0:
                reqs.append(srv.a.AllowNRequest(limiter="missing", key="x", n=1))
            t = srv.t_next()
            got = srv.st.AllowBatch(srv.a.AllowBatchRequest(requests=reqs)).results
            assert len(got) == len(reqs)
            ok = [i for i, r in enumerate(reqs) if r.n > 0 and r.limiter in srv.by_name]
            d, rem, retry, reset, _ = sim.decide(np.array([kid(reqs[i].limiter, reqs[i].key) for i in ok], np.uint64),
                                                 np.full(len(ok), t, np.int64),
                                                 np.array([reqs[i].n for i in ok], np.int64),
                                                 np.array([cid[reqs[i].limiter] for i in ok], np.uint32))
            for j, i in enumerate(ok):
                g = got[i]
                assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns, g.limit) == \
                    (bool(d[j]), rem[j], retry[j], reset[j], srv.by_name[reqs[i].limiter].limit), (step, i)
            for i, r in enumerate(reqs):
                if r.limiter not in srv.by_name:
                    assert got[i].error == "unknown limiter 'missing'"
                elif r.n <= 0:
                    assert got[i].error == rl_server.ERR_INVALID_N
        elif step % 17 == 5:
            lim, key = names[rng.integers(len(names))], f"u{rng.integers(6)}"
            t = srv.t_next()
            srv.st.Reset(srv.a.ResetRequest(limiter=lim, key=key))
            sim.reset(cid[lim], kid(lim, key), t)
        else:
            lim, key = names[rng.integers(len(names))], f"u{rng.integers(6)}"
            n = int(rng.choice([1, 2, 3]))
            t = srv.t_next()
            g = srv.st.AllowN(srv.a.AllowNRequest(limiter=lim, key=key, n=n))
            d, rem, retry, reset, _ = sim.decide([kid(lim, key)], [t], [n], [cid[lim]])
            assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                (bool(d[0]), rem[0], retry[0], reset[0]), step


def test_native_health_and_graceful_shutdown():
    store = OracleStore()
    srv = Native([LIMITERS[0]], store)
    h = rl_grpc.health_stub(srv.ch)
    assert h.Check(srv.h.HealthCheckRequest()).status == 1
    assert h.Check(srv.h.HealthCheckRequest(service="ratelimiter.v1.RateLimiter")).status == 1
    assert h.Check(srv.h.HealthCheckRequest(service="other")).status == 3
    # an RPC in flight when shutdown starts is answered
    store.gate.clear()
    fut = srv.st.Allow.future(srv.a.AllowRequest(limiter="fw", key="a"))
    assert store.entered.wait(10)
    stopper = threading.Thread(target=srv.srv.shutdown, args=(10.0,))
    stopper.start()
    time.sleep(0.2)
    store.gate.set()
    assert fut.result(10).allowed
    stopper.join(10)
    assert not stopper.is_alive()
    # no longer accepting
    ch2 = grpc.insecure_channel(f"127.0.0.1:{srv.srv.port}")
    with pytest.raises(grpc.RpcError):
        rl_grpc.rate_limiter_stub(ch2).Allow(srv.a.AllowRequest(limiter="fw", key="a"), timeout=2)
    ch2.close()
    srv.close()


@pytest.mark.parametrize("fail_open", [True, False])
def test_native_storage_failure_fail_open_closed(fail_open):
    """an engine error: fail-open returns {Allowed, Limit, 0, 0, ResetAt},
    fail-closed returns UNAVAILABLE "failed to check rate limit" (tokenbucket.go:100-112)"""
    store = OracleStore(fail=True)
    spec = "t:token_bucket:10:10s::" + ("true" if fail_open else "false")
    srv = Native([spec, "f:fixed_window:5:60s::" + ("true" if fail_open else "false")], store)
    try:
        for lim, alg, L, W in (("t", 1, 10, 10 * NS), ("f", 3, 5, 60 * NS)):
            t = srv.t_next()
            if fail_open:
                r = srv.st.Allow(srv.a.AllowRequest(limiter=lim, key="a"))
                assert (r.allowed, r.limit, r.remaining, r.retry_after_ns) == (True, L, 0, 0)
                assert r.reset_at_unix_ns == rl_server.reset_at_ns(alg, L, W, t)
            else:
                with pytest.raises(grpc.RpcError) as e:
                    srv.st.Allow(srv.a.AllowRequest(limiter=lim, key="a"))
                assert e.value.code() == grpc.StatusCode.UNAVAILABLE
                assert e.value.details().startswith("failed to check rate limit: engine status")
        rs = srv.st.AllowBatch(srv.a.AllowBatchRequest(requests=[srv.a.AllowNRequest(limiter="t", key="b", n=1)]))
        assert rs.results[0].allowed if fail_open else rs.results[0].error.startswith("failed to check rate limit")
    finally:
        srv.close()


def test_native_short_deadlines_under_load_are_never_applied():
    """RPCs with a 50 ms deadline (grpc-timeout) queue behind a hung store: the
    clients get DEADLINE_EXCEEDED, the server drops them before launch, and
    later decisions equal the oracle over the applied requests only"""
    store = OracleStore()
    srv = Native(["tb:token_bucket:5:60s"], store, max_batch=64, max_in_flight=1)
    try:
        store.gate.clear()
        first = srv.st.Allow.future(srv.a.AllowRequest(limiter="tb", key="k"))   # holds the store
        assert store.entered.wait(10)
        errs = []
        for _ in range(6):
            try:
                srv.st.AllowN(srv.a.AllowNRequest(limiter="tb", key="k", n=2), timeout=0.05)
            except grpc.RpcError as e:
                errs.append(e.code())
        assert errs == [grpc.StatusCode.DEADLINE_EXCEEDED] * 6
        time.sleep(0.1)
        store.gate.set()
        assert first.result(10).remaining == 4
        r = srv.st.Allow(srv.a.AllowRequest(limiter="tb", key="k"))
        assert r.allowed and r.remaining == 3      # none of the 6 x n=2 was applied
        s = srv.co.stats()
        assert s.expired + s.cancelled == 6 and store.applied == 2
    finally:
        srv.close()


def test_native_server_deadline_error_branch():
    """a request whose grpc-timeout passes while it is queued gets the error
    branch from the server itself: fail-open answers with the fail-open result"""
    store = OracleStore()
    srv = Native(["t:token_bucket:10:10s::true"], store, max_batch=64, max_in_flight=1)
    try:
        store.gate.clear()
        first = srv.st.Allow.future(srv.a.AllowRequest(limiter="t", key="k"))
        assert store.entered.wait(10)
        srv.t_next()
        t = srv.t_next()
        # the client allows 2 s, the server drops the request at 2 s: the
        # fail-open result arrives before the client gives up
        fut = srv.st.Allow.future(srv.a.AllowRequest(limiter="t", key="k"), timeout=2.0)
        time.sleep(2.3)
        store.gate.set()
        first.result(10)
        try:
            r = fut.result(10)
            assert (r.allowed, r.limit, r.remaining) == (True, 10, 0)
            assert r.reset_at_unix_ns == rl_server.reset_at_ns(1, 10, 10 * NS, t)
        except grpc.RpcError as e:   # the client's own deadline won the race
            assert e.code() == grpc.StatusCode.DEADLINE_EXCEEDED
        assert store.applied == 1
    finally:
        srv.close()


def test_native_concurrent_clients():
    """8 client threads x 200 RPCs on 4 channels, 2 event loops: every RPC is
    answered, the store applied each request exactly once, and the coalescer
    batched RPCs of different connections together"""
    store = OracleStore()
    srv = Native(["tb:token_bucket:1000000:1s", "fw:fixed_window:1000000:60s"], store, max_batch=512)
    try:
        chans = [grpc.insecure_channel(f"127.0.0.1:{srv.srv.port}") for _ in range(4)]
        errs, done = [], []

        def client(k):
            st = rl_grpc.rate_limiter_stub(chans[k % 4])
            futs = [st.AllowN.future(srv.a.AllowNRequest(limiter="tb" if i % 2 else "fw", key=f"k{i % 13}", n=1))
                    for i in range(200)]
            for f in futs:
                try:
                    r = f.result(30)
                    done.append(r.allowed)
                except grpc.RpcError as e:
                    errs.append(e)
        ths = [threading.Thread(target=client, args=(k,)) for k in range(8)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(60)
        assert not errs and len(done) == 1600 and all(done)
        assert store.applied == 1600
        s = srv.co.stats()
        assert s.batches < 1600
        gs = srv.srv.stats()
        assert gs.rpcs == 1600 and gs.errors == 0 and gs.decisions == 1600
        for c in chans:
            c.close()
    finally:
        srv.close()


@pytest.mark.gpu
def test_native_grpc_on_the_gpu_engine():
    """the production path: native front end + coalescer + engine on cuda:0"""
    be = rl_server.GpuBackend(0, 1 << 12, 1 << 12, 1 << 12)
    srv = Native(LIMITERS, backend=be, max_batch=1 << 12)
    try:
        sim, cid = shadow(srv)
        ids = {}
        rng = np.random.default_rng(5)
        for step in range(60):
            reqs = [srv.a.AllowNRequest(limiter=LIMITERS[rng.integers(len(LIMITERS))].split(":")[0],
                                        key=f"u{rng.integers(5)}", n=int(rng.choice([1, 2])))
                    for _ in range(rng.integers(1, 50))]
            t = srv.t_next()
            got = srv.st.AllowBatch(srv.a.AllowBatchRequest(requests=reqs)).results
            key = np.array([ids.setdefault((srv.by_name[r.limiter].prefix, r.key), len(ids)) for r in reqs],
                           np.uint64)
            d, rem, retry, reset, _ = sim.decide(key, np.full(len(reqs), t, np.int64),
                                                 np.array([r.n for r in reqs], np.int64),
                                                 np.array([cid[r.limiter] for r in reqs], np.uint32))
            for j, g in enumerate(got):
                assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                    (bool(d[j]), rem[j], retry[j], reset[j]), (step, j)
            if step % 10 == 9:
                t = srv.t_next()
                srv.st.Reset(srv.a.ResetRequest(limiter="fw", key="u1"))
                sim.reset(cid["fw"], ids.setdefault((srv.by_name["fw"].prefix, "u1"), len(ids)), t)
            lim, key = LIMITERS[rng.integers(len(LIMITERS))].split(":")[0], f"u{rng.integers(5)}"
            t = srv.t_next()
            g = srv.st.Allow(srv.a.AllowRequest(limiter=lim, key=key))
            d, rem, retry, reset, _ = sim.decide([ids.setdefault((srv.by_name[lim].prefix, key), len(ids))], [t], [1],
                                                 [cid[lim]])
            assert (g.allowed, g.remaining, g.retry_after_ns, g.reset_at_unix_ns) == \
                (bool(d[0]), rem[0], retry[0], reset[0]), step
    finally:
        srv.close(backend=be)
