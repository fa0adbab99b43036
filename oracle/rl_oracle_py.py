"""Independent pure-Python restatement of the reference decision path.

TEST INFRASTRUCTURE ONLY: used by tests/ to cross-check the C oracle
(oracle/rl_oracle.c) bit for bit on small traces.  It is written separately
(dict keyspace keyed by the formatted Redis key string, Python's own correctly
rounded float formatting) so that the two restatements share no code.

Reference anchors (paths relative to the reference repo):
  tokenbucket.go:23-52   tokenBucketScript (Lua)
  tokenbucket.go:90-133  AllowN; :155-165 refill rate / reset time; :168-193 tryConsume
  slidingwindow.go:22-30 slidingWindowScript; :68-122 AllowN; :150-197 helpers
  fixedwindow.go:21-27   fixedWindowScript;  :65-115 AllowN; :139-163 helpers
  config.go:16-87        Validate / WithDefaults / FormatKey
"""
from __future__ import annotations

import math

NS = 1_000_000_000
UNIX_TO_INTERNAL = 62135596800  # Go: seconds from year 1 to 1970
INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1

TOKEN_BUCKET, SLIDING_WINDOW, FIXED_WINDOW = 1, 2, 3
DENIED, ALLOWED, ERROR, INVALID = 0, 1, 2, 3
REDIS7, MINIREDIS = 0, 1


def wrap64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def go_trunc_div(a: int, b: int) -> int:
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def duration_seconds(d: int) -> float:
    """time.Duration.Seconds(): float64(d/Second) + float64(d%Second)/1e9"""
    sec = go_trunc_div(d, NS)
    nsec = d - sec * NS
    return float(sec) + float(nsec) / 1e9


def go_f2i(x: float) -> int:
    """Go int64(float64) on amd64 (CVTTSD2SQ): NaN/out of range -> MinInt64."""
    if math.isnan(x) or x >= 9223372036854775808.0 or x < -9223372036854775808.0:
        return INT64_MIN
    return int(x)


def window_start(t: int, w: int) -> int:
    """time.Unix(0, t).Truncate(w).Unix(): Truncate is relative to Jan 1 year 1."""
    r = (t + UNIX_TO_INTERNAL * NS) % w
    return (t - r) // NS


def lua_roundtrip(x: float, profile: int) -> float:
    """tonumber(tostring(x)) in Redis 7's Lua 5.1 ("%.14g") or gopher-lua (exact)."""
    if profile == MINIREDIS:
        return x
    return float("%.14g" % x)


class Sim:
    def __init__(self, profile: int = REDIS7):
        self.profile = profile
        self.db: dict[str, list] = {}  # key -> [value, when_ms or None]
        self.cfgs: list[tuple[int, int, int]] = []

    # -- keyspace ---------------------------------------------------------
    def _expired(self, when, s_ms):
        if when is None:
            return False
        return s_ms > when if self.profile == REDIS7 else s_ms >= when

    def _get(self, k, s_ms):
        ent = self.db.get(k)
        if ent is None:
            return None
        if self._expired(ent[1], s_ms):
            del self.db[k]
            return None
        return ent

    def _expire(self, k, ttl, s_ms):
        ent = self._get(k, s_ms)
        if ent is None:
            return
        if ttl <= 0:
            del self.db[k]
        else:
            ent[1] = s_ms + ttl * 1000

    def _incrby(self, k, n, s_ms):
        ent = self._get(k, s_ms)
        old = ent[0] if ent is not None else 0
        v = old + n
        if v > INT64_MAX or v < INT64_MIN:
            return None
        if ent is None:
            self.db[k] = [v, None]
        else:
            ent[0] = v
        return v

    # -- config -----------------------------------------------------------
    def add_config(self, alg: int, limit: int, window: int) -> int:
        if alg not in (TOKEN_BUCKET, SLIDING_WINDOW, FIXED_WINDOW):
            return -1
        if limit <= 0 or window < 1_000_000 or window > 365 * 24 * 3600 * NS:
            return -1
        self.cfgs.append((alg, limit, window))
        return len(self.cfgs) - 1

    # -- algorithms -------------------------------------------------------
    def _tb(self, L, W, key, t, n, s_ms):
        rate = float(L) / duration_seconds(W)
        now = float(t) / 1e9
        ttl = go_f2i(duration_seconds(W) * 2)
        k = "tb:%d" % key
        ent = self._get(k, s_ms)
        cap = float(L)
        if ent is None:
            tokens, last = cap, now
        else:
            tokens, last = ent[0]
        s = tokens + (now - last) * rate
        tokens = s if s < cap else cap  # Lua math.min(capacity, s)
        allowed = 0
        if tokens >= float(n):
            tokens = tokens - float(n)
            allowed = 1
        stored = (lua_roundtrip(tokens, self.profile), lua_roundtrip(now, self.profile))
        if ent is None:
            self.db[k] = [stored, None]
        else:
            ent[0] = stored
        self._expire(k, ttl, s_ms)
        rem = go_f2i(math.floor(tokens))
        sec = go_f2i(now)
        reset_at = wrap64(sec * NS + go_f2i((now - float(sec)) * 1e9) + go_f2i((float(L) / rate) * 1e9))
        retry = 0
        if not allowed:
            retry = max(0, go_f2i((float(wrap64(n - rem)) / rate) * 1e9))
        return (ALLOWED if allowed else DENIED), rem, retry, reset_at, tokens

    def _fw(self, L, W, key, t, n, s_ms):
        ws = window_start(t, W)
        ttl = go_f2i(duration_seconds(W))
        reset_at = wrap64(ws * NS + W)
        k = "w:%d:%d" % (key, ws)
        cur = self._incrby(k, n, s_ms)
        if cur is None:
            return ERROR, 0, 0, reset_at, math.nan
        if float(cur) == float(n):
            self._expire(k, ttl, s_ms)
        count = go_f2i(float(cur))
        allowed = count <= L
        rem = max(0, wrap64(L - count))
        retry = 0 if allowed else max(0, wrap64(reset_at - t))
        return (ALLOWED if allowed else DENIED), rem, retry, reset_at, math.nan

    def _sw(self, L, W, key, t, n, s_ms):
        wsec = duration_seconds(W)
        ws = window_start(t, W)
        pws = ws - go_f2i(wsec)
        reset_at = wrap64(ws * NS + W)
        ck, pk = "w:%d:%d" % (key, ws), "w:%d:%d" % (key, pws)
        pent = self._get(pk, s_ms)
        prev = float(pent[0]) if pent is not None else 0.0
        cur = self._incrby(ck, n, s_ms)
        if cur is None:
            return ERROR, 0, 0, reset_at, math.nan
        if float(cur) == float(n):
            self._expire(ck, go_f2i(wsec), s_ms)
        self._expire(pk, go_f2i(wsec * 2), s_ms)
        p, c = go_f2i(prev), go_f2i(float(cur))
        progress = float(wrap64(t - ws * NS)) / float(W)
        weighted = float(p) * (1.0 - progress)
        weighted = weighted + float(c)
        allowed = weighted <= float(L)
        rem = max(0, wrap64(L - go_f2i(weighted)))
        retry = 0 if allowed else max(0, wrap64(reset_at - t))
        return (ALLOWED if allowed else DENIED), rem, retry, reset_at, math.nan

    def decide(self, key, t, n, cfg, server_ms=None):
        """One request; returns (decision, remaining, retry_ns, reset_at_ns, tokens)."""
        s_ms = server_ms if server_ms is not None else t // 1_000_000
        if cfg < 0 or cfg >= len(self.cfgs) or n <= 0:
            return INVALID, 0, 0, 0, math.nan
        alg, L, W = self.cfgs[cfg]
        fn = {TOKEN_BUCKET: self._tb, SLIDING_WINDOW: self._sw, FIXED_WINDOW: self._fw}[alg]
        return fn(L, W, key, t, n, s_ms)

    def reset(self, cfg, key, t):
        alg, L, W = self.cfgs[cfg]
        if alg == TOKEN_BUCKET:
            self.db.pop("tb:%d" % key, None)
            return
        ws = window_start(t, W)
        self.db.pop("w:%d:%d" % (key, ws), None)
        if alg == SLIDING_WINDOW:
            self.db.pop("w:%d:%d" % (key, ws - go_f2i(duration_seconds(W))), None)
