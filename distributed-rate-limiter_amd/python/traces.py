"""Seeded synthetic request traces for the BASELINE.json configs.

Each trace is four arrays in arrival order: key_id (u64), ts_ns (i64),
n (i64), cfg (u32 index into the trace's config list).  Time starts at
T0 = 1.76e18 ns and advances by exponential inter-arrival gaps, so per-key
time never goes backwards (the reference reads time.Now() per call).
"""
from __future__ import annotations

import numpy as np

T0 = 1_760_000_000_000_000_000
NS = 1_000_000_000

# configs as (algorithm, limit, window_ns)
TB_20_12S = (1, 20, 12 * NS)        # "Token Bucket 100/min burst 20" 
SW_100_60S = (2, 100, 60 * NS)
FW_100_60S = (3, 100, 60 * NS)


def zipf_cdf(nkeys: int, s: float) -> np.ndarray:
    w = np.arange(1, nkeys + 1, dtype=np.float64) ** (-s)
    c = np.cumsum(w)
    return c / c[-1]


class ZipfKeys:
    """Zipf(s) over nkeys ranks; rank -> key id by a seeded permutation."""

    def __init__(self, nkeys: int, s: float, perm_seed: int):
        self.cdf = zipf_cdf(nkeys, s)
        self.perm = np.random.default_rng(perm_seed).permutation(nkeys).astype(np.uint64)

    def sample(self, rng: np.random.Generator, m: int) -> np.ndarray:
        r = np.searchsorted(self.cdf, rng.random(m), side="right")
        np.minimum(r, self.cdf.size - 1, out=r)
        return self.perm[r]


def arrivals(rng: np.random.Generator, m: int, t_start: int, mean_ns: float) -> np.ndarray:
    gaps = rng.exponential(mean_ns, m)
    return t_start + np.cumsum(np.rint(gaps).astype(np.int64))


class TokenBucketZipf:
    """Config 1: TB {L=20, W=12s}; 1M keys Zipf s=1.1 (perm seed 2); arrivals
    exp(mean 1 us) from T0 (seed 3); n=1; batches of `batch` requests."""

    def __init__(self, nkeys=1_000_000, s=1.1, batch=1_000_000, mean_ns=1000.0, seed=3, perm_seed=2):
        self.keys = ZipfKeys(nkeys, s, perm_seed)
        self.batch = batch
        self.mean_ns = mean_ns
        self.rng = np.random.default_rng(seed)
        self.t = T0
        self.configs = [TB_20_12S]

    def next_batch(self):
        m = self.batch
        key = self.keys.sample(self.rng, m)
        ts = arrivals(self.rng, m, self.t, self.mean_ns)
        self.t = int(ts[-1])
        return key, ts, np.ones(m, np.int64), np.zeros(m, np.uint32)


class FixedWindowUniform:
    """Config 0: FW {L=100, W=60s}; 10k uniform keys (seed 1)."""

    def __init__(self, nkeys=10_000, batch=1_000_000, mean_ns=1000.0, seed=1):
        self.nkeys, self.batch, self.mean_ns = nkeys, batch, mean_ns
        self.rng = np.random.default_rng(seed)
        self.t = T0
        self.configs = [FW_100_60S]

    def next_batch(self):
        m = self.batch
        key = self.rng.integers(0, self.nkeys, m).astype(np.uint64)
        ts = arrivals(self.rng, m, self.t, self.mean_ns)
        self.t = int(ts[-1])
        return key, ts, np.ones(m, np.int64), np.zeros(m, np.uint32)


class SlidingWindowBursty:
    """Config 2: SW {L=100, W=60s}; nkeys uniform background + bursts (a
    uniformly chosen key emits `burst` requests within 1 s) (seed 4)."""

    def __init__(self, nkeys=100_000_000, batch=1_000_000, burst=200, span_s=180.0, seed=4, nbatches=64):
        self.nkeys, self.batch, self.burst = nkeys, batch, burst
        self.rng = np.random.default_rng(seed)
        self.mean_ns = span_s * NS / (batch * nbatches)
        self.t = T0
        self.configs = [SW_100_60S]

    def next_batch(self):
        m, rng = self.batch, self.rng
        ts = arrivals(rng, m, self.t, self.mean_ns)
        self.t = int(ts[-1])
        key = rng.integers(0, self.nkeys, m).astype(np.uint64)
        nb = (m // 2) // self.burst
        # burst keys: each owns `burst` slots placed within ~1 s of its start
        slots_per_s = max(1, int(NS / self.mean_ns))
        for b in range(nb):
            k = rng.integers(0, self.nkeys)
            start = rng.integers(0, max(1, m - min(m, slots_per_s)))
            pos = start + np.sort(rng.choice(min(m - start, slots_per_s), self.burst, replace=False))
            key[pos] = k
        return key, ts, np.ones(m, np.int64), np.zeros(m, np.uint32)


class MixedTenants:
    """Config 3: cfg = key_id mod 3 -> {TB 20/12s, SW 100/60s, FW 100/60s};
    keys uniform over nkeys (seed 5)."""

    def __init__(self, nkeys=1_000_000_000, batch=1_000_000, mean_ns=1000.0, seed=5):
        self.nkeys, self.batch, self.mean_ns = nkeys, batch, mean_ns
        self.rng = np.random.default_rng(seed)
        self.t = T0
        self.configs = [TB_20_12S, SW_100_60S, FW_100_60S]

    def next_batch(self):
        m = self.batch
        key = self.rng.integers(0, self.nkeys, m).astype(np.uint64)
        ts = arrivals(self.rng, m, self.t, self.mean_ns)
        self.t = int(ts[-1])
        return key, ts, np.ones(m, np.int64), (key % 3).astype(np.uint32)
