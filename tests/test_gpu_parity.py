"""HIP engine vs CPU oracle: bit-exact parity on seeded traces (GPU).

Integer/index outputs (decision, remaining, retry_after_ns, reset_at_ns) must be
identical; token-bucket `tokens` (the Lua variable at the end of the script)
must be the identical IEEE double (compared as bit patterns).
"""
import numpy as np
import pytest

import oracle
import traces
from tracegen import CONFIG_SETS, T0, NS, long_window_trace, random_config_trace, random_trace, skewed_trace

pytestmark = pytest.mark.gpu


def make_engine(rl, profile, tb=1 << 20, win=1 << 20, max_batch=1 << 20):
    return rl.Engine(profile=profile, tb_capacity=tb, win_capacity=win, max_batch=max_batch)


def assert_same(res, ref, configs, cfg, what=""):
    dec, rem, retry, reset, tok = ref
    bad = np.nonzero(res.decision != dec)[0]
    assert bad.size == 0, f"{what} decision mismatch at {bad[:10]}: gpu={res.decision[bad[:10]]} ref={dec[bad[:10]]}"
    ok = dec != 3
    for name, a, b in [("remaining", res.remaining, rem), ("retry", res.retry_after_ns, retry),
                       ("reset_at", res.reset_at_ns, reset)]:
        bad = np.nonzero((a != b) & ok)[0]
        assert bad.size == 0, f"{what} {name} mismatch at {bad[:10]}: gpu={a[bad[:10]]} ref={b[bad[:10]]}"
    if res.tokens is not None:
        is_tb = np.array([configs[c][0] == 1 if c < len(configs) else False for c in cfg]) & (dec <= 1)
        gb = res.tokens.view(np.uint64)[is_tb]
        rb = tok.view(np.uint64)[is_tb]
        bad = np.nonzero(gb != rb)[0]
        assert bad.size == 0, f"{what} tokens mismatch: gpu={res.tokens[is_tb][bad[:5]]} ref={tok[is_tb][bad[:5]]}"


def run_both(rl, profile, configs, batches, **kw):
    eng = make_engine(rl, profile, **kw)
    sim = oracle.OracleSim(profile)
    for a, L, W in configs:
        assert eng.register(a, L, W) == sim.add_config(a, L, W)
    for i, b in enumerate(batches):
        key, ts, n, cfg, sms = b if len(b) == 5 else (*b, None)
        res = eng.decide(key, ts, n, cfg, sms)
        ref = sim.decide(key, ts, n, cfg, sms)
        assert_same(res, ref, configs, cfg, what=f"batch {i}")
    return eng, sim


def split(trace, sizes):
    key, ts, n, cfg, sms = trace
    out, o = [], 0
    for s in sizes:
        out.append((key[o:o + s], ts[o:o + s], n[o:o + s], cfg[o:o + s], None if sms is None else sms[o:o + s]))
        o += s
    return out


# --- exact %.14g on the device -------------------------------------------------

def test_q14_device_matches_glibc(rl):
    eng = make_engine(rl, 0, tb=1024, win=1024, max_batch=1024)
    rng = np.random.default_rng(11)
    bits = rng.integers(0, 1 << 63, 400_000, dtype=np.int64).astype(np.uint64) | \
        (rng.integers(0, 2, 400_000).astype(np.uint64) << np.uint64(63))
    x = bits.view(np.float64)
    x = x[np.isfinite(x)]
    x = np.concatenate([x, rng.random(200_000) * 20, rng.random(200_000) * 1e-6,
                        (T0 + rng.integers(0, 10 ** 11, 200_000)) / 1e9,
                        [0.0, -0.0, 1.0000610351562500, 0.999999999999995, 5e-324, 1.7e308]])
    dev = eng.q14_device(x)
    host = rl.q14_host(x)
    assert np.array_equal(dev.view(np.uint64), host.view(np.uint64))
    ref = np.array([float("%.14g" % v) for v in x[::50]])
    assert np.array_equal(host[::50].view(np.uint64), ref.view(np.uint64))


def test_q14_device_decade_edges_and_tiny(rl):
    from tracegen import q14_edge_values
    eng = make_engine(rl, 0, tb=1024, win=1024, max_batch=1024)
    x = q14_edge_values(seed=9)
    dev = eng.q14_device(x)
    ref = np.array([float("%.14g" % v) for v in x])
    assert np.array_equal(dev.view(np.uint64), ref.view(np.uint64))


# --- randomized multi-config traces, multiple batches (state carried) ----------

@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("kind", ["tb", "sw", "fw", "mixed"])
@pytest.mark.parametrize("ff", [False, True])
def test_random_traces(rl, profile, kind, ff):
    configs = CONFIG_SETS[kind]
    seed = {"tb": 1, "sw": 2, "fw": 3, "mixed": 4}[kind] * 10 + profile * 2 + int(ff)
    tr = random_trace(seed, 60_000, 500, configs, fastforward=ff, big_n=True)
    run_both(rl, profile, configs, split(tr, [1, 7, 1000, 9000, 20000, 29992]))


@pytest.mark.parametrize("small", [True, False])
@pytest.mark.parametrize("kind", ["tb", "mixed"])
def test_small_batches(rl, kind, small, monkeypatch):
    """Batches at and around the single-workgroup path's limit (k_small, 4096),
    with that path on and off (RL_SMALL_MAX=0: the full launch sequence)."""
    monkeypatch.setenv("RL_SMALL_MAX", "4096" if small else "0")
    configs = CONFIG_SETS[kind]
    tr = random_trace(90 + len(kind), 30_000, 150, configs, big_n=True)
    sizes = [1, 2, 3, 63, 64, 65, 1000, 4095, 4096, 4097, 129, 2048, 7000]
    sizes.append(30_000 - sum(sizes))
    for profile in (0, 1):
        run_both(rl, profile, configs, split(tr, sizes))


@pytest.mark.parametrize("small", [True, False])
def test_small_batch_single_hot_key(rl, small, monkeypatch):
    monkeypatch.setenv("RL_SMALL_MAX", "4096" if small else "0")
    configs = [(1, 20, 12 * NS), (2, 100, 60 * NS), (3, 100, 60 * NS)]
    rng = np.random.default_rng(8)
    for c in range(3):
        m = 4096 * 3
        key = np.full(m, 5 + c, np.uint64)
        ts = T0 + np.cumsum(rng.integers(0, 3_000_000, m)).astype(np.int64)
        cfg = np.full(m, c, np.uint32)
        run_both(rl, 0, configs, split((key, ts, np.ones(m, np.int64), cfg, None), [4096, 4096, 4096]))


def test_hot_keys_long_segments(rl):
    # a few keys carrying most traffic: long per-key segments in one batch
    configs = CONFIG_SETS["mixed"]
    rng = np.random.default_rng(5)
    m = 200_000
    key = rng.choice(np.arange(15, dtype=np.uint64), m, p=np.full(15, 1 / 15))
    ts = T0 + np.cumsum(rng.integers(0, 20_000, m)).astype(np.int64)
    n = np.ones(m, np.int64)
    cfg = (key % len(configs)).astype(np.uint32)
    for profile in (0, 1):
        run_both(rl, profile, configs, split((key, ts, n, cfg, None), [100_000, 100_000]))


def _chain_trace(kind, seed, m=120_000):
    """Few keys, long token-bucket segments, chosen to drive the chain through
    its regimes: deep denial (near steps, decade crossings), frequent allows
    (regime exits every few steps), sub-nanosecond gaps and huge n."""
    rng = np.random.default_rng(seed)
    if kind == "deny":        # one hot key: 8 us gaps against 20 tokens / 12 s
        key = np.zeros(m, np.uint64)
        gaps = np.rint(rng.exponential(8_000, m))
        n = np.ones(m, np.int64)
    elif kind == "allow":     # 3 keys, 10/s with 40 ms gaps: allows mixed with denials
        key = rng.integers(0, 3, m).astype(np.uint64)
        gaps = np.rint(rng.exponential(15_000_000, m))
        n = rng.choice([1, 1, 1, 2], m).astype(np.int64)
    else:                     # "mixed": bursts of zero gaps, rare long gaps, huge n
        key = rng.integers(0, 2, m).astype(np.uint64)
        gaps = rng.choice([0, 1, 1000, 90_000, 400_000_000], m, p=[0.2, 0.2, 0.3, 0.29, 0.01])
        n = rng.choice([1, 1, 1, 2, 7], m).astype(np.int64)
        n[rng.random(m) < 0.001] = 1 << 62
    ts = T0 + np.cumsum(gaps).astype(np.int64)
    cfg = (key % 3).astype(np.uint32)
    return key, ts, n, cfg, None


@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("kind", ["deny", "allow", "mixed"])
def test_chain_regimes(rl, profile, kind):
    configs = [(1, 20, 12 * NS), (1, 10, NS), (1, 3, 300_000_000)]
    seed = {"deny": 1, "allow": 2, "mixed": 3}[kind] * 10 + profile
    run_both(rl, profile, configs, split(_chain_trace(kind, seed), [50_000, 70_000]))


@pytest.mark.parametrize("seed", range(16))
def test_chain_random_configs(rl, seed):
    configs, tr = random_config_trace(700 + seed, 1, 90_000)
    run_both(rl, seed % 2, configs, split(tr, [30_000, 60_000]), tb=1 << 12, win=1 << 12)


@pytest.mark.parametrize("seed", range(8))
def test_window_random_configs(rl, seed):
    configs, tr = random_config_trace(800 + seed, 2 + seed % 2 if seed < 4 else 0, 90_000)
    run_both(rl, seed % 2, configs, split(tr, [30_000, 60_000]), tb=1 << 12, win=1 << 12)


@pytest.mark.parametrize("wi", range(3))
@pytest.mark.parametrize("alg", [1, 2, 3, 0])
@pytest.mark.parametrize("profile", [0, 1])
def test_long_windows(rl, profile, alg, wi):
    """Windows of 1 to 365 days (config.go:41-46 accepts up to 365 d): 7-day
    windows (year-1 Truncate offset, fixedwindow.go:72), W = 2^24 s + 1 ns and
    31535999.999999999 s (Duration.Seconds() rounds up into ttl, pws and rate:
    tokenbucket.go:155-157,170, slidingwindow.go:74-75,161-162,
    fixedwindow.go:151), W = 365 d with L = 1 (refill 3.2e-8 tokens/s), limits
    up to 1e12.  A hot key per config through the chain (huge segments in the
    second batch) and the wave replay, 20k light keys, time spanning years."""
    configs, tr = long_window_trace(1100 + 10 * wi + alg + 5 * profile, alg, 120_000, wi=wi)
    run_both(rl, profile, configs, split(tr, [3000, 27_000, 90_000]), tb=1 << 16, win=1 << 16)


@pytest.mark.parametrize("alg,profile,wi", [(1, 0, 0), (2, 1, 1), (3, 0, 2), (0, 1, 0)])
def test_long_windows_many_keys(rl, alg, profile, wi, monkeypatch):
    """The long-window configurations over many light keys and no hot key:
    k_small (batches up to 4096), the full launch sequence, then batches of
    2^19 and more, which after the first take the light replay kernel
    (k_replay_light)."""
    monkeypatch.setenv("RL_SMALL_MAX", "4096")
    configs, tr = long_window_trace(1300 + 10 * wi + alg + 5 * profile, alg, 1_300_000, wi=wi,
                                    n_light=50_000, hot_share=0.0)
    eng, _ = run_both(rl, profile, configs, split(tr, [3000, 4096, 90_000, 600_000, 602_904]),
                      tb=1 << 17, win=1 << 17)
    assert eng.stats().light_batches >= 1


@pytest.mark.parametrize("seed", range(4))
def test_random_configs_many_keys(rl, seed, monkeypatch):
    """The same random configurations over many keys: batches below the
    single-workgroup limit (k_small), mid-size batches (the full launch
    sequence, light segments) and batches of 2^19 and more with no hot key,
    which after the first take the light replay kernel."""
    monkeypatch.setenv("RL_SMALL_MAX", "4096")
    configs, tr = random_config_trace(900 + seed, 0, 1_300_000, nk=40_000 + 20_000 * seed)
    eng, _ = run_both(rl, seed % 2, configs, split(tr, [3000, 4096, 90_000, 600_000, 602_904]),
                      tb=1 << 17, win=1 << 17)
    assert eng.stats().light_batches >= 1


@pytest.mark.parametrize("counts", [
    [4096, 4095, 4097, 1, 8191, 8192, 1, 2, 3, 4094, 1, 4096],     # boundaries at and around tile edges
    [4096] * 6,                                                   # m a multiple of the tile: no tail positions
    [1] * 5000 + [20_000, 3, 12_289],                             # many heads per chunk, then segments past tiles
])
def test_segment_tile_boundaries(rl, counts):
    # k_segments stages 4096-position tiles: segments starting / ending exactly
    # at, one before and one after a tile edge, a segment running over several
    # tiles to the batch end, and rejected requests (n = 0, sorted last)
    configs = CONFIG_SETS["mixed"]
    rng = np.random.default_rng(len(counts))
    key = np.concatenate([np.full(c, 1000 + i, np.uint64) for i, c in enumerate(counts)])
    key = key[rng.permutation(key.size)]
    m = key.size
    ts = T0 + np.cumsum(rng.integers(0, 400_000, m)).astype(np.int64)
    n = np.ones(m, np.int64)
    if m % 4096:
        n[rng.random(m) < 0.01] = 0
    cfg = (key % len(configs)).astype(np.uint32)
    run_both(rl, 0, configs, split((key, ts, n, cfg, None), [m]))


@pytest.mark.parametrize("counts", [
    [12_288, 5000, 3000, 1, 2],        # every MSD bucket fits LDS (12288): k_sort_local
    [12_289, 7, 9000, 4096],           # one key just past it: the LSD passes
    [20_000, 4000, 4000, 1, 64],       # a hot key: the LSD passes
])
def test_sort_local_and_lsd_paths(rl, counts):
    # the grouping sort's MSD pass picks k_sort_local when every bucket of its
    # digit fits LDS and the LSD passes otherwise; both must group every key's
    # requests in arrival order (tables of 2^16: 18-bit slot ids, 3 passes)
    configs = CONFIG_SETS["mixed"]
    rng = np.random.default_rng(sum(counts))
    key = np.concatenate([np.full(c, 77 + i, np.uint64) for i, c in enumerate(counts)])
    extra = rng.integers(1000, 60_000, 30_000).astype(np.uint64)    # many light keys around them
    key = np.concatenate([key, extra])[rng.permutation(key.size + extra.size)]
    m = key.size
    ts = T0 + np.cumsum(rng.integers(0, 300_000, m)).astype(np.int64)
    n = rng.choice([1, 1, 2], m).astype(np.int64)
    n[rng.random(m) < 0.003] = 0
    cfg = (key % len(configs)).astype(np.uint32)
    for profile in (0, 1):
        run_both(rl, profile, configs, split((key, ts, n, cfg, None), [m]), tb=1 << 16, win=1 << 16)


def test_sort_predicted_plan_and_misprediction(rl):
    # once a batch's MSD buckets all fit LDS the engine launches the next
    # batches' grouping sort as k_sort_local alone; a batch that then brings a
    # bucket too large for LDS (hot keys, one spanning three LDS chunks) is
    # sorted by k_sort_local's in-kernel LSD path (loc_sort_big) on that
    # misprediction, and the batches after it go back to the LSD passes until
    # a plan fits again -- every batch against the oracle
    configs = CONFIG_SETS["mixed"]
    rng = np.random.default_rng(5)
    batches, t = [], T0
    for kind in ["u", "u", "u", "hot", "hot", "u", "u"]:
        m = 60_000
        key = rng.integers(1000, 200_000, m).astype(np.uint64)
        if kind == "hot":
            r = rng.random(m)
            key[r < 0.5] = 77                      # 30k requests of one key
            key[(r >= 0.5) & (r < 0.75)] = 78      # and 15k of another algorithm's
        ts = t + np.cumsum(rng.integers(0, 300_000, m)).astype(np.int64)
        t = int(ts[-1])
        n = rng.choice([1, 1, 2], m).astype(np.int64)
        n[rng.random(m) < 0.003] = 0
        batches.append((key, ts, n, (key % len(configs)).astype(np.uint32), None))
    eng = make_engine(rl, 0, tb=1 << 18, win=1 << 18)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        assert eng.register(a, L, W) == sim.add_config(a, L, W)
    pred = []
    for i, (key, ts, n, cfg, sms) in enumerate(batches):
        before = eng.stats().sort_predicted
        res = eng.decide(key, ts, n, cfg, sms)
        assert_same(res, sim.decide(key, ts, n, cfg, sms), configs, cfg, what=f"batch {i}")
        pred.append(int(eng.stats().sort_predicted - before))
    assert pred == [0, 1, 1, 1, 0, 0, 1]        # batch 3 (hot) mispredicted: loc_sort_big


def test_light_replay_and_misprediction(rl):
    # after a large batch with no huge segment the engine launches the light
    # replay kernel (k_replay_light: no chain) for the next large batch; one
    # that brings a hot key anyway replays it exactly as a heavy segment (one
    # wave) and flips the prediction back to the chain kernel.  Small batches
    # always take the chain kernel.  Every batch against the oracle.
    configs = CONFIG_SETS["mixed"]
    rng = np.random.default_rng(11)
    batches, t = [], T0
    for kind, m in [("u", 600_000), ("hot", 600_000), ("hot", 600_000), ("u", 100_000), ("u", 600_000)]:
        key = rng.integers(1000, 3_000_000, m).astype(np.uint64)
        if kind == "hot":
            r = rng.random(m)
            key[r < 0.3] = 15                      # a token-bucket key (15 % 15 == 0): 180k requests
            key[(r >= 0.3) & (r < 0.4)] = 20       # and 60k of a sliding-window key
        ts = t + np.cumsum(rng.integers(0, 40_000, m)).astype(np.int64)
        t = int(ts[-1])
        n = rng.choice([1, 1, 2], m).astype(np.int64)
        batches.append((key, ts, n, (key % len(configs)).astype(np.uint32), None))
    eng = make_engine(rl, 0, tb=1 << 22, win=1 << 22)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        assert eng.register(a, L, W) == sim.add_config(a, L, W)
    light = []
    for i, (key, ts, n, cfg, sms) in enumerate(batches):
        before = eng.stats().light_batches
        res = eng.decide(key, ts, n, cfg, sms)
        assert_same(res, sim.decide(key, ts, n, cfg, sms), configs, cfg, what=f"batch {i}")
        light.append(int(eng.stats().light_batches - before))
    assert light == [0, 1, 0, 0, 1]


def test_single_hot_key_full_batch(rl):
    # the bench's diagnostic workload: one key carries the whole 1M batch
    g = traces.TokenBucketZipf(nkeys=1, batch=1_000_000)
    run_both(rl, 0, g.configs, [g.next_batch() for _ in range(2)], tb=1 << 10, win=1 << 10)


def test_zipf15_full_batch(rl):
    g = traces.TokenBucketZipf(s=1.5, batch=1_000_000)
    run_both(rl, 0, g.configs, [g.next_batch() for _ in range(2)], tb=1 << 21, win=1 << 10)


# --- BASELINE configs at full batch size ----------------------------------------

def test_config1_tb_zipf_full_batches(rl):
    g = traces.TokenBucketZipf(batch=1_000_000)
    run_both(rl, 0, g.configs, [g.next_batch() for _ in range(2)], tb=1 << 21, win=1 << 10)


def test_config0_fw_uniform(rl):
    g = traces.FixedWindowUniform(batch=1_000_000)
    run_both(rl, 0, g.configs, [g.next_batch() for _ in range(2)], tb=1 << 10, win=1 << 15)


def test_config2_sw_bursty(rl):
    g = traces.SlidingWindowBursty(nkeys=2_000_000, batch=500_000, span_s=180.0, nbatches=4)
    run_both(rl, 0, g.configs, [g.next_batch() for _ in range(4)], tb=1 << 10, win=1 << 22)


def test_config2_sw_bursty_full_size(rl):
    """BASELINE configs[2] at its stated size: 100M keys in an HBM window table
    of 2^27 entries (8 GiB) + spill, uniform + bursty, 24M requests over 180 s
    of virtual time (three 60-s windows: previous-window weighting, previous-key
    expiry and spills of live window keys all occur).  Keys never interact, so
    the oracle replays a seeded 1/32 sample of the keys (every request of those
    keys, in order) and must match bit for bit; the whole run is checked by
    size-independent properties: every request decided, the entries used equal
    the distinct keys seen, the spill holds window keys."""
    g = traces.SlidingWindowBursty(nkeys=100_000_000, batch=1_000_000, span_s=180.0, nbatches=24)
    eng = make_engine(rl, 0, tb=1 << 10, win=1 << 27, max_batch=1 << 20)
    sim = oracle.OracleSim(0)
    assert eng.register(*g.configs[0]) == sim.add_config(*g.configs[0])
    seen = []
    t_first = None
    for b in range(24):
        key, ts, n, cfg = g.next_batch()
        t_first = t_first if t_first is not None else int(ts[0])
        res = eng.decide(key, ts, n, cfg, want_tokens=False)
        assert np.all(res.decision <= 1)
        pick = (key * np.uint64(0x9E3779B97F4A7C15) >> np.uint64(59)) == np.uint64(0)   # 1/32 of keys
        ref = sim.decide(key[pick], ts[pick], n[pick], cfg[pick])
        sub = rl.Decisions(res.decision[pick], res.remaining[pick], res.retry_after_ns[pick],
                           res.reset_at_ns[pick], None)
        assert_same(sub, ref, g.configs, cfg[pick], what=f"batch {b}")
        seen.append(np.unique(key))
    t_last = int(ts[-1])
    assert t_last - t_first >= 179 * NS
    distinct = np.unique(np.concatenate(seen)).size
    info = eng.table_info(t_last // 1_000_000)
    assert info.win_used == distinct
    assert info.spill_used > 0 and info.spill_live > 0
    eng.close()


def test_config3_mixed(rl):
    g = traces.MixedTenants(nkeys=300_000, batch=500_000)
    run_both(rl, 0, g.configs, [g.next_batch() for _ in range(2)], tb=1 << 19, win=1 << 20)


@pytest.mark.parametrize("gpus", [8, 2])
def test_config3_per_gpu_scale(rl, gpus):
    """BASELINE configs[3] at its per-GPU share: 1B keys hash-sharded over G
    GPUs is 125M keys per GPU at G = 8 and 500M at G = 2.  Mixed tenants
    (cfg = key mod 3: TB 20/12s, SW 100/60s, FW 100/60s) in 2M batches at
    1 us mean gaps, tables sized for the share at load ~0.6 (G = 8: TB 2^26,
    window 2^27 + spill 2^28, 18 GB of HBM; G = 2: TB 2^28, window 2^29 +
    spill 2^30, 72 GB).  G = 8 runs 132M requests (~80M distinct keys), G = 2
    256M (~200M distinct keys).  As configs[2]: a seeded 1/32 of the keys
    replayed by the oracle bit for bit, and whole-run properties -- every
    request decided, the entries used equal the distinct keys of each table,
    live spilled window keys."""
    share = 1_000_000_000 // gpus
    sh = 26 if gpus == 8 else 28
    nb = 66 if gpus == 8 else 128
    g = traces.MixedTenants(nkeys=share, batch=2_000_000)
    eng = make_engine(rl, 0, tb=1 << sh, win=1 << (sh + 1), max_batch=1 << 21)
    sim = oracle.OracleSim(0)
    for c in g.configs:
        assert eng.register(*c) == sim.add_config(*c)
    seen = np.zeros(share, np.bool_)
    for b in range(nb):
        key, ts, n, cfg = g.next_batch()
        res = eng.decide(key, ts, n, cfg, want_tokens=(b % 8 == 0))
        assert np.all(res.decision <= 1), f"batch {b}"
        pick = (key * np.uint64(0x9E3779B97F4A7C15) >> np.uint64(59)) == np.uint64(0)   # 1/32 of keys
        ref = sim.decide(key[pick], ts[pick], n[pick], cfg[pick])
        sub = rl.Decisions(res.decision[pick], res.remaining[pick], res.retry_after_ns[pick],
                           res.reset_at_ns[pick], None if res.tokens is None else res.tokens[pick])
        assert_same(sub, ref, g.configs, cfg[pick], what=f"batch {b}")
        seen[key] = True
    distinct = int(np.count_nonzero(seen))
    tb_keys = int(np.count_nonzero(seen[0::3]))
    del seen
    info = eng.table_info(int(ts[-1]) // 1_000_000)
    assert distinct > (80_000_000 if gpus == 8 else 190_000_000)
    assert info.tb_used == tb_keys and info.win_used == distinct - tb_keys
    assert info.spill_used > 0 and info.spill_live > 0
    assert eng.sync() == 0
    eng.close()


# --- per-key time going back (window keys beyond the 2-slot entry) -------------

@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("kind", ["sw", "fw", "mixed"])
@pytest.mark.parametrize("nkeys", [40, 3000])
def test_skewed_clocks(rl, profile, kind, nkeys):
    """App servers whose clocks differ by up to 130 s share the limiter: a
    key's requests go back by one or more windows, so older live window keys
    are spilled from the 2-slot entry and read back (rl_window.h).  Few keys:
    heavy segments (wave replay); many keys: light ones; small batches: k_small.
    The Redis clock is the store's own and monotone."""
    configs = CONFIG_SETS[kind]
    tr = skewed_trace(600 + profile * 7 + nkeys, 80_000, nkeys, configs, big_n=True)
    run_both(rl, profile, configs, split(tr, [3000, 500, 20_000, 26_500, 30_000]), tb=1 << 14, win=1 << 14)


def test_skewed_clocks_gc_and_reset(rl):
    """Table GC (grow, then shrink) and Reset with spilled window keys."""
    configs = CONFIG_SETS["mixed"]
    tr = skewed_trace(640, 60_000, 500, configs)
    eng = make_engine(rl, 0, tb=1 << 13, win=1 << 13, max_batch=1 << 15)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    caps = [(0, 0), (1 << 15, 1 << 15), (1 << 12, 1 << 12)]
    for i, (key, ts, n, cfg, sms) in enumerate(split(tr, [15_000] * 4)):
        if i:
            now_ms = int(sms[0])
            before = eng.table_info(now_ms)
            _, after = eng.table_gc(now_ms, *caps[i - 1])
            assert after.spill_live == before.spill_live
            assert after.spill_used == after.spill_live <= before.spill_used
        res = eng.decide(key, ts, n, cfg, sms)
        assert_same(res, sim.decide(key, ts, n, cfg, sms), configs, cfg, what=f"batch {i}")
        t, s_ms = int(ts[-1]), int(sms[-1])
        for k in range(0, 500, 7):
            # DEL of the keys AllowN would touch at a skewed server's time
            for tt in (t, t - 7 * NS):
                eng.reset(k % len(configs), k, tt)
                sim.reset(k % len(configs), k, tt, s_ms)
    assert eng.table_info(int(tr[4][-1])).spill_used > 0   # the spill was exercised
    eng.close()


# --- edges ----------------------------------------------------------------------

def test_empty_and_invalid(rl):
    eng = make_engine(rl, 0, tb=1024, win=1024, max_batch=4096)
    c = eng.register(1, 10, 60 * NS)
    res = eng.decide(np.zeros(0, np.uint64), np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint32))
    assert res.decision.size == 0
    key = np.array([1, 2, rl.KEY_RESERVED, 3], np.uint64)
    res = eng.decide(key, np.full(4, T0), np.array([1, 0, 1, -3]), np.array([c, c, c, 7], np.uint32), check=False)
    assert list(res.decision) == [1, 3, 3, 3]


def test_batches_larger_than_max_batch(rl):
    configs = CONFIG_SETS["mixed"]
    tr = random_trace(77, 50_000, 300, configs)
    eng = make_engine(rl, 0, tb=1 << 12, win=1 << 12, max_batch=4096)   # forces 13 chunks
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    assert_same(eng.decide(*tr[:4]), sim.decide(*tr[:4]), configs, tr[3])


def test_reset_between_batches(rl):
    configs = CONFIG_SETS["mixed"]
    tr = random_trace(78, 20_000, 50, configs)
    eng = make_engine(rl, 0, tb=1 << 12, win=1 << 12)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    for part in split(tr, [5000, 5000, 5000, 5000]):
        assert_same(eng.decide(*part[:4]), sim.decide(*part[:4]), configs, part[3])
        t = int(part[1][-1])
        for k in range(0, 50, 3):
            eng.reset(k % len(configs), k, t)
            sim.reset(k % len(configs), k, t)


def test_table_full_is_reported(rl):
    eng = make_engine(rl, 0, tb=1024, win=1024, max_batch=4096)
    c = eng.register(1, 10, 60 * NS)
    key = np.arange(2000, dtype=np.uint64)
    res = eng.decide(key, np.full(2000, T0), np.ones(2000, np.int64), np.full(2000, c, np.uint32), check=False)
    assert res.status == rl.RL_ENOMEM


def test_deterministic_repeat(rl):
    g1, g2 = traces.TokenBucketZipf(batch=200_000), traces.TokenBucketZipf(batch=200_000)
    outs = []
    for g in (g1, g2):
        eng = make_engine(rl, 0, tb=1 << 21, win=1024)
        eng.register(*g.configs[0])
        outs.append([eng.decide(*g.next_batch()) for _ in range(2)])
    for a, b in zip(*outs):
        assert np.array_equal(a.decision, b.decision)
        assert np.array_equal(a.tokens.view(np.uint64), b.tokens.view(np.uint64))


# --- device API, pipelined batches -----------------------------------------------

@pytest.mark.parametrize("pipeline", [False, True])
def test_device_api_batches_in_flight(rl, pipeline):
    """Several device-API batches enqueued back to back (with RL_OPT_PIPELINE
    the engine overlaps batch b+1's grouping with batch b's replay); every
    batch's results must equal the oracle's."""
    import torch
    configs = CONFIG_SETS["mixed"]
    tr = random_trace(91, 80_000, 400, configs, big_n=True)
    sizes = [20_000, 15_000, 25_000, 20_000]
    eng = rl.Engine(profile=0, tb_capacity=1 << 14, win_capacity=1 << 14, max_batch=1 << 15,
                    flags=rl.OPT_PIPELINE if pipeline else 0)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    dev = torch.device("cuda", 0)
    parts = split(tr, sizes)
    ins, outs = [], []
    for key, ts, n, cfg, _ in parts:     # inputs complete before the first call
        ins.append([torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
                    for x in (key, ts, n, cfg.view(np.int32))])
        m = key.size
        outs.append([torch.empty(m, dtype=torch.uint8, device=dev)] +
                    [torch.empty(m, dtype=torch.int64, device=dev) for _ in range(3)] +
                    [torch.empty(m, dtype=torch.float64, device=dev)])
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream
    for (k, t, n, c), o in zip(ins, outs):
        eng.decide_device(k.numel(), k.data_ptr(), t.data_ptr(), n.data_ptr(), c.data_ptr(), None,
                          *[x.data_ptr() for x in o], stream)
    torch.cuda.synchronize()
    assert eng.sync() == 0, eng.last_error()
    for i, ((key, ts, n, cfg, _), o) in enumerate(zip(parts, outs)):
        ref = sim.decide(key, ts, n, cfg)
        res = rl.Decisions(*[x.cpu().numpy() for x in o])
        assert_same(res, ref, configs, cfg, what=f"batch {i}")


@pytest.mark.parametrize("level", [1, 2, -2])
def test_timed_pipelined_batches(rl, level):
    """Stage timing on (level 1: the replay's events are bound to its dispatch
    and also order the finish stream; level 2: marker events around every
    stage; level -2: the replay's events on every 2nd batch, the others bind
    the plain done event) over pipelined hot-key batches: results equal the
    oracle's and the replay time is reported for the batches timed."""
    import torch
    g = traces.TokenBucketZipf(batch=100_000)
    eng = rl.Engine(profile=0, tb_capacity=1 << 20, win_capacity=1024, max_batch=1 << 17, flags=rl.OPT_PIPELINE)
    sim = oracle.OracleSim(0)
    for a, L, W in g.configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    eng.set_timing(level)
    eng.stage_times()
    dev = torch.device("cuda", 0)
    parts = [g.next_batch() for _ in range(4)]
    ins, outs = [], []
    for key, ts, n, cfg in parts:
        ins.append([torch.from_numpy(x.view(np.int64) if x.dtype == np.uint64 else x).to(dev)
                    for x in (key, ts, n, cfg.view(np.int32))])
        m = key.size
        outs.append([torch.empty(m, dtype=torch.uint8, device=dev)] +
                    [torch.empty(m, dtype=torch.int64, device=dev) for _ in range(3)] +
                    [torch.empty(m, dtype=torch.float64, device=dev)])
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream
    for (k, t, n, c), o in zip(ins, outs):
        eng.decide_device(k.numel(), k.data_ptr(), t.data_ptr(), n.data_ptr(), c.data_ptr(), None,
                          *[x.data_ptr() for x in o], stream)
    torch.cuda.synchronize()
    assert eng.sync() == 0, eng.last_error()
    ms, nb = eng.stage_times()
    eng.set_timing(0)
    assert nb == (len(parts) + 1) // 2 if level == -2 else len(parts)
    assert ms[3] > 0
    for i, ((key, ts, n, cfg), o) in enumerate(zip(parts, outs)):
        ref = sim.decide(key, ts, n, cfg)
        res = rl.Decisions(*[x.cpu().numpy() for x in o])
        assert_same(res, ref, g.configs, cfg, what=f"batch {i}")


# --- table GC / resize (rl_table_gc) ----------------------------------------------

@pytest.mark.parametrize("profile", [0, 1])
def test_table_gc_keeps_decisions(rl, profile):
    """GC at the clock of the next batch (then grow, then shrink) between
    batches: decisions stay identical to the oracle, which never collects."""
    configs = CONFIG_SETS["mixed"]
    tr = random_trace(200 + profile, 60_000, 3000, configs, big_n=True)
    eng = make_engine(rl, profile, tb=1 << 14, win=1 << 14, max_batch=1 << 15)
    sim = oracle.OracleSim(profile)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    parts = split(tr, [15_000, 15_000, 15_000, 15_000])
    caps = [(0, 0), (1 << 16, 1 << 15), (1 << 13, 1 << 13)]
    for i, (key, ts, n, cfg, sms) in enumerate(parts):
        if i:
            now_ms = int(ts[0]) // 1_000_000
            before = eng.table_info(now_ms)
            _, after = eng.table_gc(now_ms, *caps[i - 1])
            assert after.tb_live == before.tb_live and after.win_live == before.win_live
            assert after.tb_used == after.tb_live <= before.tb_used
            if caps[i - 1][0]:
                assert after.tb_capacity == caps[i - 1][0] and after.win_capacity == caps[i - 1][1]
        res = eng.decide(key, ts, n, cfg, sms)
        assert_same(res, sim.decide(key, ts, n, cfg, sms), configs, cfg, what=f"batch {i}")


@pytest.mark.parametrize("profile", [0, 1])
def test_table_gc_long_windows(rl, profile):
    """GC between batches of the long-window trace (windows of 1-365 days,
    TTLs that long, phase jumps of up to 400 days: keys expire between and
    within batches), with a grow and a shrink on the way: decisions stay the
    oracle's, and GC keeps exactly the live keys."""
    configs, tr = long_window_trace(1600 + profile, 0, 120_000, wi=profile, n_light=8_000)
    eng = make_engine(rl, profile, tb=1 << 15, win=1 << 15, max_batch=1 << 15)
    sim = oracle.OracleSim(profile)
    for a, L, W in configs:
        assert eng.register(a, L, W) == sim.add_config(a, L, W)
    parts = split(tr, [20_000] * 6)
    caps = [(0, 0), (1 << 16, 1 << 16), (0, 0), (1 << 14, 1 << 14), (0, 0)]
    collected = 0
    for i, (key, ts, n, cfg, sms) in enumerate(parts):
        if i:
            now_ms = int(ts[0]) // 1_000_000
            before = eng.table_info(now_ms)
            _, after = eng.table_gc(now_ms, *caps[i - 1])
            assert after.tb_live == before.tb_live and after.win_live == before.win_live
            assert after.tb_used == after.tb_live <= before.tb_used
            collected += (before.tb_used - after.tb_used) + (before.win_used - after.win_used)
            if caps[i - 1][0]:
                assert after.tb_capacity == caps[i - 1][0] and after.win_capacity == caps[i - 1][1]
        res = eng.decide(key, ts, n, cfg, sms)
        assert_same(res, sim.decide(key, ts, n, cfg, sms), configs, cfg, what=f"batch {i}")
    assert collected > 0          # the phase jumps expired keys that GC then dropped
    eng.close()


def test_table_gc_frees_a_full_table(rl):
    """A table that is full of expired keys accepts new keys after GC; a GC
    whose live keys do not fit the requested size fails and keeps the tables."""
    configs = [(1, 5, NS), (3, 5, NS)]   # TB ttl 2 s, FW ttl 1 s
    eng = make_engine(rl, 0, tb=1024, win=1024, max_batch=4096)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    m = 2000
    for rnd in range(3):
        key = (np.arange(m, dtype=np.uint64) + rnd * m)
        ts = np.full(m, T0 + rnd * 10 * NS, np.int64)
        n = np.ones(m, np.int64)
        cfg = (key % 2).astype(np.uint32)
        if rnd:
            info = eng.table_info(int(ts[0]) // 1_000_000)
            assert info.tb_used == 1000 and info.tb_live == 0 and info.win_live == 0
            eng.table_gc(int(ts[0]) // 1_000_000)
            info = eng.table_info(int(ts[0]) // 1_000_000)
            assert info.tb_used == 0 and info.win_used == 0
        res = eng.decide(key, ts, n, cfg)
        assert_same(res, sim.decide(key, ts, n, cfg), configs, cfg, what=f"round {rnd}")
    eng.close()


def test_table_gc_refuses_a_too_small_table(rl):
    configs = [(1, 5, 60 * NS)]
    eng = make_engine(rl, 0, tb=4096, win=1024, max_batch=4096)
    sim = oracle.OracleSim(0)
    for a, L, W in configs:
        eng.register(a, L, W)
        sim.add_config(a, L, W)
    m = 3000
    key = np.arange(m, dtype=np.uint64)
    n = np.ones(m, np.int64)
    cfg = np.zeros(m, np.uint32)
    for rnd in range(2):
        ts = np.full(m, T0 + rnd * NS, np.int64)
        if rnd:
            rc, _ = eng.table_gc(int(ts[0]) // 1_000_000, 1024, 1024, check=False)
            assert rc == rl.RL_ENOMEM
            info = eng.table_info(int(ts[0]) // 1_000_000)
            assert info.tb_capacity == 4096 and info.tb_live == m
        res = eng.decide(key, ts, n, cfg)
        assert_same(res, sim.decide(key, ts, n, cfg), configs, cfg, what=f"round {rnd}")
    eng.close()
