"""The rate limiter's gRPC server (api/proto/ratelimiter.proto): the service
the reference plans in cmd/server/main.go:13-17 and docs/ARCHITECTURE.md
:287-304 -- per-tenant limiter instances, Allow / AllowN / Reset, a health
check, graceful shutdown -- backed by the MI355X engine through the request
coalescer (include/rl_coalescer.h): every RPC's requests join the next GPU
batch, and AllowBatch hands many requests to one batch at once.

Semantics per RPC follow the Go limiter (internal/ratelimiter):
  * time.Now() is read when the request arrives (tokenbucket.go:97,
    slidingwindow.go:73, fixedwindow.go:71);
  * n <= 0 -> INVALID_ARGUMENT "invalid n: must be greater than 0" (ErrInvalidN,
    errors.go:16; tokenbucket.go:91-93);
  * a storage (engine) error -> fail-open: {Allowed: true, Limit, Remaining 0,
    RetryAfter 0, ResetAt} (tokenbucket.go:100-112 and twins), fail-closed:
    UNAVAILABLE "failed to check rate limit: <err>";
  * keys are FormatKey(prefix, key) (config.go:81-87; prefix "" -> "ratelimit"),
    hashed to the engine's key ids on the host (rl_hash_keys_host).  As in
    Redis, the formatted key is the only namespace: two limiters with one
    prefix share state (a fixed and a sliding window of one length share
    their window counters, fixedwindow.go:139-141 / slidingwindow.go:150-152);
    --isolate-limiters gives every limiter a namespace of its own instead;
  * contexts (interface.go:75): the RPC deadline becomes the coalescer
    submission's deadline -- a request still queued when it passes is never
    applied -- and an expired or cancelled request takes the error branch
    (fail-open result, or DEADLINE_EXCEEDED / CANCELLED "failed to check rate
    limit: context ...");
  * the tables are collected from the serving path: the coalescer counts and
    GCs them between batches (rl_coalescer_opts.gc_*), so a long-running
    server never fills them.

Two front ends serve the same handlers' semantics: the native one (default,
include/rl_grpc.h: C++ event loops speaking HTTP/2 + protobuf themselves,
every RPC submitted to the coalescer as it arrives) and the Python one
(--frontend python: grpcio's server over RateLimiterService below, which
also documents the semantics the native server restates).

Run: python rl_server.py --address 127.0.0.1:8080 --limiter api:token_bucket:20:12s ...
"""
from __future__ import annotations

import argparse
import os
import re
import signal
import sys
import threading
import time
from concurrent import futures

import grpc
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import rl_amd  # noqa: E402
import rl_grpc  # noqa: E402

NS = 1_000_000_000
ERR_INVALID_N = "invalid n: must be greater than 0"            # errors.go:16
KEY_SEED = 0


def parse_duration(s: str) -> int:
    """Go time.ParseDuration subset: '1h2m3.5s', '500ms', '12s' -> ns"""
    units = {"ns": 1, "us": 1000, "µs": 1000, "ms": 1_000_000, "s": NS, "m": 60 * NS, "h": 3600 * NS}
    parts = re.findall(r"(\d+(?:\.\d*)?)(ns|us|µs|ms|s|m|h)", s)
    if not parts or "".join(a + b for a, b in parts) != s:
        raise ValueError(f"invalid duration {s!r}")
    return int(round(sum(float(a) * units[b] for a, b in parts)))


def _go_f2i(x: float) -> int:
    if not (x < 9223372036854775808.0) or not (x >= -9223372036854775808.0):
        return -(1 << 63)
    return int(x)


def _wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= 1 << 63 else v


def reset_at_ns(alg: int, limit: int, window_ns: int, t: int) -> int:
    """Result.ResetAt of a request at t, as the fail-open path computes it
    (tokenbucket.go:161-165; fixedwindow.go:144-146; slidingwindow.go:155-157)"""
    if alg == rl_amd.TOKEN_BUCKET:
        wsec = float(window_ns // NS) + float(window_ns % NS) / 1e9
        rate = float(limit) / wsec
        now = float(t) / 1e9
        sec = _go_f2i(now)
        nsec = _go_f2i((now - float(sec)) * 1e9)
        return _wrap64(sec * NS + nsec + _go_f2i(float(limit) / rate * 1e9))
    r = (t + 62135596800 * NS) % window_ns           # time.Truncate is relative to year 1
    ws = (t - r) // NS
    return _wrap64(ws * NS + window_ns)


class Limiter:
    """One configured limiter instance (a reference Config, interface.go:46-70)."""

    def __init__(self, name, algorithm, limit, window_ns, prefix="", fail_open=False):
        err = rl_amd.config_validate(algorithm, limit, window_ns)
        if err:
            raise ValueError(f"invalid config: {err}")
        self.name = name
        self.alg = rl_amd.ALG_BY_NAME[algorithm]
        self.limit, self.window_ns = limit, window_ns
        self.prefix = (prefix or "ratelimit").encode()      # WithDefaults, config.go:62-64
        self.fail_open = fail_open
        self.cfg_id = None

    @staticmethod
    def parse(spec: str) -> "Limiter":
        """name:algorithm:limit:window[:prefix[:fail_open]]"""
        f = spec.split(":")
        if len(f) < 4:
            raise ValueError(f"limiter spec {spec!r}: name:algorithm:limit:window[:prefix[:fail_open]]")
        return Limiter(f[0], f[1], int(f[2]), parse_duration(f[3]), f[4] if len(f) > 4 else "",
                       len(f) > 5 and f[5].lower() in ("1", "true", "open", "fail_open"))


class RateLimiterService:
    """The RPC handlers over a coalescer (GPU engine, or the test seam's host
    backend).  `register(alg, limit, window_ns) -> cfg_id` registers a config
    with the backend; `clock()` -> Unix ns (time.Now())."""

    def __init__(self, limiters, coalescer, register, clock=time.time_ns, isolate=False):
        self.a = rl_grpc.api("ratelimiter.proto")
        self.h = rl_grpc.api("health.proto")
        self.co = coalescer
        self.clock = clock
        self.isolate = isolate
        self.by_name = {}
        for lim in limiters:
            lim.cfg_id = register(lim.alg, lim.limit, lim.window_ns)
            self.by_name[lim.name] = lim
        self.serving = True

    # -- helpers -------------------------------------------------------------
    def _limiter(self, name, ctx):
        lim = self.by_name.get(name)
        if lim is None:
            ctx.abort(grpc.StatusCode.NOT_FOUND, f"unknown limiter {name!r}")
        return lim

    def _ids(self, lim, keys, m) -> np.ndarray:
        """FormatKey(prefix, key) hashed: the formatted key is the namespace
        (Redis), or one namespace per limiter with --isolate-limiters"""
        return rl_amd.hash_keys_host(keys, KEY_SEED, lim.prefix, cfg=[lim.cfg_id] * m if self.isolate else None)

    def _key_id(self, lim, key: str) -> int:
        return int(self._ids(lim, [key.encode()], 1)[0])

    @staticmethod
    def _deadline(ctx) -> int:
        """the RPC deadline on the coalescer's clock (0 = none)"""
        rem = ctx.time_remaining() if ctx is not None else None
        if rem is None or rem > 1e6:   # no deadline (gRPC reports an infinite one as huge)
            return 0
        return max(1, rl_amd.now_ns() + int(rem * 1e9))

    # rl_coalescer status -> (go error text, gRPC code) of the error branch
    _CTX_ERR = {rl_amd.RL_EDEADLINE: ("context deadline exceeded", grpc.StatusCode.DEADLINE_EXCEEDED),
                rl_amd.RL_ECANCELED: ("context canceled", grpc.StatusCode.CANCELLED)}

    def _result(self, lim, t, rc, dec, rem, retry, reset):
        """AllowResponse, or (None, fail-closed error text, gRPC code)"""
        if rc == rl_amd.RL_OK and dec in (rl_amd.ALLOWED, rl_amd.DENIED):
            return self.a.AllowResponse(allowed=dec == rl_amd.ALLOWED, limit=lim.limit, remaining=rem,
                                        retry_after_ns=retry, reset_at_unix_ns=reset), None, None
        if rc in self._CTX_ERR:
            err, code = self._CTX_ERR[rc]
        else:
            err = f"engine status {rc}" if rc != rl_amd.RL_OK else "script error (INCRBY overflow)"
            code = grpc.StatusCode.UNAVAILABLE
        if lim.fail_open:
            return self.a.AllowResponse(allowed=True, limit=lim.limit, remaining=0, retry_after_ns=0,
                                        reset_at_unix_ns=reset_at_ns(lim.alg, lim.limit, lim.window_ns, t)), \
                None, None
        return None, f"failed to check rate limit: {err}", code

    def _allow_n(self, name, key, n, ctx):
        lim = self._limiter(name, ctx)
        if n <= 0:
            ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, ERR_INVALID_N)
        t = self.clock()
        rc, (dec, rem, retry, reset) = self.co.decide(self._key_id(lim, key), t, n, lim.cfg_id,
                                                      deadline_ns=self._deadline(ctx))
        res, err, code = self._result(lim, t, rc, dec, rem, retry, reset)
        if err:
            ctx.abort(code, err)
        return res

    # -- RPCs ----------------------------------------------------------------
    def Allow(self, req, ctx):
        return self._allow_n(req.limiter, req.key, 1, ctx)

    def AllowN(self, req, ctx):
        return self._allow_n(req.limiter, req.key, req.n, ctx)

    def Reset(self, req, ctx):
        lim = self._limiter(req.limiter, ctx)
        rc = self.co.reset(self._key_id(lim, req.key), self.clock(), lim.cfg_id)
        if rc != rl_amd.RL_OK:
            ctx.abort(grpc.StatusCode.UNAVAILABLE, f"failed to reset rate limit: engine status {rc}")
        return self.a.ResetResponse()

    def AllowBatch(self, req, ctx):
        """many AllowN calls: one submission to the coalescer (one GPU batch
        when it fits); per-request errors in AllowResponse.error"""
        rs = req.requests
        m = len(rs)
        t = self.clock()
        out = [None] * m
        idx, keys, cfg, ns = [], [], [], []
        groups = {}
        for i, r in enumerate(rs):
            lim = self.by_name.get(r.limiter)
            if lim is None:
                out[i] = self.a.AllowResponse(error=f"unknown limiter {r.limiter!r}")
            elif r.n <= 0:
                out[i] = self.a.AllowResponse(error=ERR_INVALID_N)
            else:
                groups.setdefault(r.limiter, []).append(len(idx))
                idx.append(i)
                keys.append(r.key.encode())
                cfg.append(lim.cfg_id)
                ns.append(r.n)
        if idx:
            kid = np.empty(len(idx), np.uint64)
            for name, pos in groups.items():
                kid[pos] = self._ids(self.by_name[name], [keys[p] for p in pos], len(pos))
            tk = self.co.submit(kid, np.full(len(idx), t, np.int64), np.array(ns, np.int64), np.array(cfg, np.uint32),
                                deadline_ns=self._deadline(ctx))
            rc, (dec, rem, retry, reset) = self.co.wait(tk, len(idx))
            for j, i in enumerate(idx):
                lim = self.by_name[rs[i].limiter]
                res, err, _ = self._result(lim, t, rc, int(dec[j]), int(rem[j]), int(retry[j]), int(reset[j]))
                out[i] = res if res is not None else self.a.AllowResponse(error=err)
        return self.a.AllowBatchResponse(results=out)

    def Check(self, req, ctx):
        S = self.h.HealthCheckResponse
        if req.service not in ("", "ratelimiter.v1.RateLimiter"):
            return S(status=3)   # SERVICE_UNKNOWN
        return S(status=1 if self.serving else 2)


def build_server(service: RateLimiterService, address: str, workers: int = 64) -> tuple[grpc.Server, int]:
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                         options=[("grpc.so_reuseport", 0)])
    for a, sname, impl in ((service.a, "RateLimiter", service), (service.h, "Health", service)):
        handlers = {}
        for mname, inp, out in a.services[sname]:
            handlers[mname] = grpc.unary_unary_rpc_method_handler(
                getattr(impl, mname), request_deserializer=getattr(a, inp).FromString,
                response_serializer=getattr(a, out).SerializeToString)
        server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(a.full_service(sname), handlers),))
    port = server.add_insecure_port(address)
    return server, port


class GpuBackend:
    """engine + coalescer on one GPU (the production backend)"""

    def __init__(self, device=0, tb_capacity=1 << 22, win_capacity=1 << 22, max_batch=1 << 16):
        self.eng = rl_amd.Engine(profile=rl_amd.PROFILE_REDIS7, tb_capacity=tb_capacity, win_capacity=win_capacity,
                                 max_batch=max_batch, device=device, flags=rl_amd.OPT_PIPELINE)
        self.register = self.eng.register
        self.co = None

    def start(self, max_batch=1 << 16, gc_interval_ns=NS, gc_margin_ms=1000):
        """the coalescer, with the tables collected from the serving path"""
        self.co = rl_amd.Coalescer(self.eng, max_batch=max_batch, max_in_flight=3, gc_interval_ns=gc_interval_ns,
                                   gc_margin_ms=gc_margin_ms)
        return self.co

    def close(self):
        if self.co:
            self.co.close()
        self.eng.close()


def serve(service, address, workers=64, grace_s=5.0, ready=None, stop_event=None):
    """run until SIGTERM / SIGINT (or stop_event): then NOT_SERVING, stop
    accepting, finish in-flight RPCs within grace_s (graceful shutdown)"""
    server, port = build_server(service, address, workers)
    server.start()
    if ready:
        ready(port)
    stop = stop_event or threading.Event()
    if threading.current_thread() is threading.main_thread():
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: stop.set())
    stop.wait()
    service.serving = False
    server.stop(grace_s).wait()
    return port


def serve_native(co, limiters, address, io_threads=4, isolate=False, grace_s=5.0, ready=None, stop_event=None):
    """the native front end (include/rl_grpc.h) until SIGTERM / SIGINT (or
    stop_event): then health NOT_SERVING, stop accepting, answer the RPCs in
    flight within grace_s"""
    host, port = address.rsplit(":", 1)
    srv = rl_amd.GrpcServer(co, [(l.name, l.cfg_id, l.alg, l.limit, l.window_ns, l.prefix, l.fail_open)
                                 for l in limiters], host=host, port=int(port), io_threads=io_threads,
                            isolate=isolate)
    try:
        if ready:
            ready(srv.port)
        stop = stop_event or threading.Event()
        if threading.current_thread() is threading.main_thread():
            for sig in (signal.SIGTERM, signal.SIGINT):
                signal.signal(sig, lambda *_: stop.set())
        stop.wait()
        srv.shutdown(grace_s)
        if os.environ.get("RL_SERVER_STATS"):
            import json
            cs, gs = co.stats(), srv.stats()
            print(json.dumps({"coalescer": {k: getattr(cs, k) for k, _ in cs._fields_[2:]},
                              "grpc": {k: getattr(gs, k) for k, _ in gs._fields_[2:]}}), file=sys.stderr, flush=True)
    finally:
        srv.close()
    return srv.port


def main(argv=None):
    ap = argparse.ArgumentParser(description="rate limiter gRPC server (MI355X engine)")
    ap.add_argument("--address", default="127.0.0.1:8080", help="listen address (docs/ARCHITECTURE.md: port 8080)")
    ap.add_argument("--limiter", action="append", default=[],
                    help="name:algorithm:limit:window[:prefix[:fail_open]], repeatable")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--frontend", choices=["native", "python"], default="native",
                    help="native: C++ HTTP/2 event loops (include/rl_grpc.h); python: grpcio server")
    ap.add_argument("--io-threads", type=int, default=4, help="native front end: event-loop threads")
    ap.add_argument("--workers", type=int, default=64, help="python front end: handler threads")
    ap.add_argument("--max-batch", type=int, default=1 << 16)
    ap.add_argument("--tb-capacity", type=int, default=1 << 22)
    ap.add_argument("--win-capacity", type=int, default=1 << 22)
    ap.add_argument("--gc-interval-ms", type=float, default=1000.0,
                    help="count the tables at least this often and collect expired keys (0 = never)")
    ap.add_argument("--gc-margin-ms", type=int, default=1000,
                    help="GC at the last request's clock minus this (request clocks may lag by this much)")
    ap.add_argument("--isolate-limiters", action="store_true",
                    help="one key namespace per limiter (the reference shares state between limiters with "
                         "the same prefix, as Redis keys are the formatted strings)")
    args = ap.parse_args(argv)
    specs = args.limiter or ["default:token_bucket:20:12s"]
    limiters = [Limiter.parse(s) for s in specs]
    be = GpuBackend(args.device, args.tb_capacity, args.win_capacity, args.max_batch)
    print(f"rate limiter gRPC server on {args.address} ({args.frontend} front end): " + ", ".join(specs),
          file=sys.stderr, flush=True)
    try:
        if args.frontend == "native":
            for lim in limiters:
                lim.cfg_id = be.register(lim.alg, lim.limit, lim.window_ns)
            co = be.start(args.max_batch, int(args.gc_interval_ms * 1e6),
                          args.gc_margin_ms)
            serve_native(co, limiters, args.address, args.io_threads, args.isolate_limiters,
                         ready=lambda p: print(f"READY {p}", flush=True))
        else:
            svc = RateLimiterService(limiters, None, be.register, isolate=args.isolate_limiters)
            svc.co = be.start(args.max_batch, int(args.gc_interval_ms * 1e6), args.gc_margin_ms)
            serve(svc, args.address, args.workers, ready=lambda p: print(f"READY {p}", flush=True))
    finally:
        be.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
