"""Seeded adversarial traces for parity tests (both the CPU oracle cross-check
and the GPU parity tests use these)."""
import numpy as np

NS = 1_000_000_000
T0 = 1_760_000_000_000_000_000

CONFIG_SETS = {
    "tb": [(1, 20, 12 * NS), (1, 5, 60 * NS), (1, 10, NS), (1, 3, 300_000_000), (1, 7, 1_500_000_000)],
    "sw": [(2, 100, 60 * NS), (2, 5, 2 * NS), (2, 3, 1_500_000_000), (2, 4, 700_000_000), (2, 2, 300_000_000)],
    "fw": [(3, 100, 60 * NS), (3, 5, 2 * NS), (3, 3, 1_500_000_000), (3, 4, 700_000_000), (3, 2, 7 * NS)],
}
CONFIG_SETS["mixed"] = CONFIG_SETS["tb"] + CONFIG_SETS["sw"] + CONFIG_SETS["fw"]


def random_trace(seed, m, nkeys, configs, fastforward=False, big_n=False, one_cfg_per_key=True):
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, m).astype(np.uint64)
    gaps = rng.choice([0, 1, 1000, 250_000, 50_000_000, 700_000_000, 3 * NS], m,
                      p=[0.05, 0.05, 0.4, 0.2, 0.2, 0.08, 0.02])
    ts = T0 + np.cumsum(gaps).astype(np.int64)
    n = rng.choice([1, 1, 1, 2, 3, 7, 50], m).astype(np.int64)
    if big_n:
        n[rng.random(m) < 0.02] = (1 << 62)
        n[rng.random(m) < 0.01] = 0
    if one_cfg_per_key:
        cfg = (keys % len(configs)).astype(np.uint32)
    else:
        cfg = rng.integers(0, len(configs), m).astype(np.uint32)
    sms = None
    if fastforward:
        sms = (ts // 1_000_000) + np.cumsum(rng.choice([0, 0, 0, 1500], m)).astype(np.int64)
    return keys, ts, n, cfg, sms


def skewed_trace(seed, m, nkeys, configs, skews_ns=(0, -2_500_000_000, -7 * NS, 4 * NS, -130 * NS),
                 big_n=False):
    """N app servers with skewed clocks sharing one limiter (docs/ARCHITECTURE.md
    :142-164): requests arrive in true-time order, each stamped with its
    server's clock (t = true time + skew), so per-key times go back by one or
    more windows; the Redis clock (server_ms) is the store's own, monotone."""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, nkeys, m).astype(np.uint64)
    gaps = rng.choice([0, 1000, 250_000, 50_000_000, 700_000_000], m, p=[0.1, 0.4, 0.2, 0.25, 0.05])
    true_t = T0 + np.cumsum(gaps).astype(np.int64)
    server = rng.integers(0, len(skews_ns), m)
    ts = true_t + np.asarray(skews_ns, np.int64)[server]
    n = rng.choice([1, 1, 1, 2, 3, 7], m).astype(np.int64)
    if big_n:
        n[rng.random(m) < 0.01] = (1 << 62)
    cfg = (keys % len(configs)).astype(np.uint32)
    sms = true_t // 1_000_000
    return keys, ts, n, cfg, sms


def random_config_trace(seed, alg, m, nk=None):
    """Seeded random configurations (limit 1 .. 1e12 log-uniform, window 1 ms
    .. ~1 day) and a few hot keys whose gaps are drawn around each config's
    refill period (limit / window): the chain's decades, multi-decade windows,
    allows, clamps and expiries at scales the fixed configs above never reach;
    for the window algorithms, runs that cross window starts at every scale."""
    rng = np.random.default_rng(seed)
    configs = []
    for _ in range(3):
        a = alg if alg else int(rng.integers(1, 4))
        L = max(1, int(round(10 ** rng.uniform(0, 12))))
        W = int(round(10 ** rng.uniform(6, 13.9)))
        configs.append((a, L, W))
    nk = nk or int(rng.integers(1, 5))
    key = rng.integers(0, nk, m).astype(np.uint64)
    cfg = (key % 3).astype(np.uint32)
    period = np.array([W / L for _, L, W in configs])[cfg]          # ns per token
    lim = np.array([L for _, L, _ in configs])[cfg]
    # per phase of 3000 requests: a request takes a fraction f of the bucket and
    # arrivals per refilled token drift around 1 -- long denial stretches (deep
    # near-empty balances, decade crossings), refills to the cap, and allows
    ph = m // 3000 + 1
    f = np.repeat(10 ** rng.uniform(-6, -1, ph), 3000)[:m]
    scale = np.repeat(10 ** rng.uniform(-1.5, 1, ph), 3000)[:m]
    n = np.maximum(1, np.rint(lim * f)).astype(np.int64) * rng.choice([1, 1, 1, 2], m)
    gaps = np.rint(rng.exponential(1.0, m) * period * n * scale / nk)
    gaps[rng.random(m) < 0.05] = 0
    gaps = np.minimum(gaps, 10 ** 12)                                # ts stays far from int64 overflow
    r = rng.random(m)
    big = r < 0.01
    n[big] = np.maximum(1, (lim[big] * rng.random(int(big.sum())) * 1.3).astype(np.int64))
    n[r > 0.999] = 1 << 62
    ts = T0 + np.cumsum(gaps).astype(np.int64)
    return configs, (key, ts, n, cfg, None)


DAY = 86400 * NS
# windows Validate accepts past a day (config.go:41-46: 1 ms <= W <= 365 d):
# one day; seven days (Truncate's year-1 offset is 259200 s, fixedwindow.go:72);
# 2^24 s and 31535999.999999999 s, where Duration.Seconds() rounds up
# (31536000.0: ttl, pws and rate all shift, tokenbucket.go:155-157,170,
# fixedwindow.go:151, slidingwindow.go:75,161-162); 365 days exactly; 30 days
LONG_WINDOWS = [DAY, 7 * DAY, 31_535_999_999_999_999, 365 * DAY, (1 << 24) * NS + 1, 30 * DAY]


def long_window_trace(seed, alg, m, wi=0, n_light=20_000, hot_share=0.6):
    """Reference-legal long windows (1 day .. 365 days) with limits 1 .. 1e12,
    so refill rates reach ~3e-8 tokens/s (L = 1, W = 365 d).  Three configs
    (key id mod 3): LONG_WINDOWS[wi] and LONG_WINDOWS[wi + 3], then a random
    window in [1 d, 365 d]; the first config's limit is 1 when wi is even,
    the third's is in [1e9, 1e12].  One hot key per config carries
    hot_share / 3 of the traffic (chain and wave segments) among n_light light
    keys.  Time runs in phases of 3000 requests at a gap scale around each hot
    key's refill period (capped at 1000 s), with jumps of hours to ~400 days
    between phases, so window starts of every config are crossed and buckets
    go from deep denial to the cap; the whole trace spans a few years."""
    rng = np.random.default_rng(seed)
    configs = []
    for i in range(3):
        a = alg if alg else int(rng.integers(1, 4))
        if i < 2:
            W = LONG_WINDOWS[(wi + 3 * i) % len(LONG_WINDOWS)]
        else:
            W = int(round(10 ** rng.uniform(np.log10(DAY), np.log10(365 * DAY))))
        if i == 0 and wi % 2 == 0:
            L = 1
        else:
            L = max(1, int(round(10 ** rng.uniform(9 if i == 2 else 0, 12))))
        configs.append((a, L, W))
    hot = rng.random(m) < hot_share
    key = np.where(hot, rng.integers(0, 3, m), rng.integers(3, 3 + n_light, m)).astype(np.uint64)
    cfg = (key % 3).astype(np.uint32)
    period = np.array([W / L for _, L, W in configs])[cfg]          # ns per token
    lim = np.array([L for _, L, _ in configs])[cfg]
    ph = m // 3000 + 1
    f = np.repeat(10 ** rng.uniform(-6, -0.5, ph), 3000)[:m]
    scale = np.repeat(10 ** rng.uniform(-2, 1, ph), 3000)[:m]
    n = np.maximum(1, np.rint(lim * f)).astype(np.int64) * rng.choice([1, 1, 1, 2], m)
    # a key with share s of the traffic sees one request per gap / s: its
    # consumption keeps pace with its refill at scale ~1 (no hot keys: every
    # key a light one, s = 1 / n_light)
    share = hot_share / 3 if hot_share > 0 else 1.0 / n_light
    gaps = np.rint(rng.exponential(1.0, m) * np.minimum(period * n * scale * share, 1e12))
    gaps[rng.random(m) < 0.05] = 0
    jumps = rng.choice([0, 3600 * NS, DAY, 5 * DAY, 40 * DAY, 400 * DAY], ph, p=[0.3, 0.2, 0.2, 0.15, 0.1, 0.05])
    jumps = (jumps * rng.random(ph)).astype(np.int64)
    gaps[::3000] += jumps[: gaps[::3000].size]
    r = rng.random(m)
    big = r < 0.01
    n[big] = np.maximum(1, (lim[big] * rng.random(int(big.sum())) * 1.3).astype(np.int64))
    n[r > 0.999] = 1 << 62
    ts = T0 + np.cumsum(gaps).astype(np.int64)
    assert int(ts[-1]) - T0 < 40 * 365 * DAY
    return configs, (key, ts, n, cfg, None)


def q14_edge_values(n=4000, seed=5):
    """values just below / at / above powers of ten (where rounding to 14
    digits carries into the next decade, or must not), 14-digit midpoints,
    and log-uniform tiny magnitudes down to 1e-340 (the wide and big-integer
    paths of rl_q14.h)"""
    rng = np.random.default_rng(seed)
    j = rng.integers(-330, 30, n)
    u = 10.0 ** rng.uniform(-17, -12, n)
    p10 = np.array([float(f"1e{k}") for k in j])
    below = p10 * (1.0 - u)
    above = p10 * (1.0 + u)
    D = rng.integers(10 ** 13, 10 ** 14, n)
    mids = np.array([float(f"{d}5e{k - 14}") for d, k in zip(D, j)])
    tiny = 10.0 ** rng.uniform(-340, -9, n) * rng.choice([-1.0, 1.0], n)
    fixed = [0.99999999999999, 0.999999999999994, 0.999999999999996, 9.9999999999999e-10, 999999999999.99,
             9.99999999999994e-300, 2.2250738585072014e-308, 1e-9, 1e-10, 1e-300]
    x = np.concatenate([below, above, mids, tiny, fixed])
    return x[np.isfinite(x) & (x != 0)]
