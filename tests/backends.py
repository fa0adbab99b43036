"""Two interchangeable limiter backends for replaying the reference's tests.

Both expose the reference's per-call API (interface.go:76-145) with an explicit
clock, so a reference test written against time.Now()/time.Sleep and
miniredis.FastForward becomes a deterministic script:

  * OracleBackend -- the CPU restatement (oracle/, TEST INFRASTRUCTURE) plus the
    Go-layer glue (ErrInvalidN, FormatKey, fail-open/closed) restated here.
  * GpuBackend    -- the product: the C++ host mirror over the HIP engine
    (include/rl_limiter.h), driven through ctypes.

Virtual time: every call advances the client clock by CALL_NS (a call's
latency); sleep(d) advances it by d; fast_forward(d) moves only the Redis TTL
clock (miniredis FastForward), which starts at 0.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

T_START = 1_760_000_000_123_456_789
CALL_NS = 50_000
NS = 1_000_000_000

ALG = {"token_bucket": 1, "sliding_window": 2, "fixed_window": 3}


@dataclass
class Result:
    Allowed: bool
    Limit: int
    Remaining: int
    RetryAfter: int
    ResetAt: int


class ErrInvalidN(Exception):
    pass


class Clock:
    def __init__(self, start=T_START):
        self.t = start
        self.ff_ms = 0

    def tick(self):
        self.t += CALL_NS
        return self.t

    def sleep(self, ns):
        self.t += ns

    def fast_forward(self, ns):
        self.ff_ms += ns // 1_000_000


# ---------------------------------------------------------------------------
class _OracleLimiter:
    def __init__(self, be, algorithm, limit, window, prefix, fail_open):
        self.be, self.limit, self.window = be, limit, window
        self.prefix = prefix or "ratelimit"      # WithDefaults (config.go:54-67)
        self.fail_open = fail_open
        self.alg = ALG[algorithm]
        self.cfg = be.sim.add_config(self.alg, limit, window)
        assert self.cfg >= 0
        self.closed = False

    def _key(self, key):
        # FormatKey (config.go:81-87): the formatted name is the key's only
        # identity, so limiters with one prefix share it, as in Redis
        return self.be.intern("%s:%s" % (self.prefix, key))

    def allow(self, key):
        return self.allow_n(key, 1)

    def allow_n(self, key, n):
        if n <= 0:
            raise ErrInvalidN()
        t = self.be.clock.tick()
        if self.closed:
            if self.fail_open:
                return Result(True, self.limit, 0, 0, self._fail_open_reset(t))
            raise RuntimeError("failed to check rate limit: closed")
        dec, rem, retry, reset, _ = self.be.sim.decide(
            [self._key(key)], [t], [n], [self.cfg], [self.be.clock.ff_ms])
        d = int(dec[0])
        if d == 2:
            if self.fail_open:
                return Result(True, self.limit, 0, 0, int(reset[0]))
            raise RuntimeError("failed to check rate limit: overflow")
        return Result(d == 1, self.limit, int(rem[0]), int(retry[0]), int(reset[0]))

    def _fail_open_reset(self, t):
        lib = self.be.lib
        if self.alg == 1:
            return lib.rlo_tb_reset_at(self.limit, self.window, float(t) / 1e9)
        return lib.rlo_window_start(t, self.window) * NS + self.window

    def reset(self, key):
        self.be.sim.reset(self.cfg, self._key(key), self.be.clock.tick())

    def close(self):
        self.closed = True


class OracleBackend:
    name = "oracle"

    def __init__(self, profile=1):
        import oracle
        self.lib = oracle.c_oracle()
        self.sim = oracle.OracleSim(profile)
        self.clock = Clock()
        self._ids = {}

    def intern(self, k):
        return self._ids.setdefault(k, len(self._ids))

    def keys(self):
        """miniredis Keys(): the live keys' names, sorted"""
        names = {v: k for k, v in self._ids.items()}
        return sorted(names[i] + (":%d" % ws if kind == 1 else "") for i, kind, ws in self.sim.keys(self.clock.ff_ms))

    def new(self, algorithm, limit, window, prefix="", fail_open=False):
        return _OracleLimiter(self, algorithm, limit, window, prefix, fail_open)


# ---------------------------------------------------------------------------
class _GpuLimiter:
    def __init__(self, be, lim):
        self.be, self.lim = be, lim

    def allow(self, key):
        return self.allow_n(key, 1)

    def allow_n(self, key, n):
        import rl_amd
        t = self.be.clock.tick() if n > 0 else self.be.clock.t
        self.be.eng.set_server_ms(self.be.clock.ff_ms)
        res, err, code = self.lim.allow_n(key, n, now_ns=t)
        if code == rl_amd.RLL_ERR_INVALID_N:
            assert res is None
            raise ErrInvalidN()
        if code != rl_amd.RLL_OK:
            assert res is None
            raise RuntimeError(err)
        return Result(res.Allowed, res.Limit, res.Remaining, res.RetryAfter, res.ResetAt)

    def reset(self, key):
        err = self.lim.reset(key, now_ns=self.be.clock.tick())
        if err:
            raise RuntimeError(err)

    def close(self):
        self.lim.close()


class GpuBackend:
    name = "gpu"

    def __init__(self, profile=1):
        import rl_amd
        self.rl = rl_amd
        self.eng = rl_amd.LimiterEngine(profile=profile)
        self.clock = Clock()

    def new(self, algorithm, limit, window, prefix="", fail_open=False):
        return _GpuLimiter(self, self.rl.new_limiter(self.eng, algorithm, limit, window, prefix, fail_open))

    def keys(self):
        return self.eng.keys(self.clock.ff_ms)
