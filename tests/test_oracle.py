"""CPU oracle: pinned against the reference's unit-test KATs and cross-checked
bit for bit against the independent Python restatement on random traces."""
import math

import numpy as np
import pytest

import oracle
from oracle import rl_oracle_py as P

NS = 1_000_000_000
T0 = 1_760_000_000_000_000_000


@pytest.fixture(scope="module")
def lib():
    oracle.build()
    return oracle.c_oracle()


# --- unit KATs transcribed from the reference's *_test.go ---------------------

def test_refill_rate_kats(lib):  # tokenbucket_test.go:85-131 (InDelta 1e-4)
    for limit, window, exp in [(10, 60 * NS, 10.0 / 60.0), (100, 3600 * NS, 100.0 / 3600.0), (60, NS, 60.0)]:
        assert abs(lib.rlo_tb_refill_rate(limit, window) - exp) < 1e-4
        assert lib.rlo_tb_refill_rate(limit, window) == float(limit) / P.duration_seconds(window)


def test_reset_time_kats(lib):  # fixedwindow_test.go:179-220, slidingwindow_test.go:133-174
    for ws, w, exp in [(1640000000, 60 * NS, 1640000060), (1640000000, 3600 * NS, 1640003600)]:
        assert ws * NS + w == exp * NS


def test_weighted_count_kats(lib):  # slidingwindow_test.go:176-238 (InDelta 0.1)
    ws = 1640000000
    for dt, prev, curr, exp in [(0, 50, 10, 60.0), (30, 50, 10, 35.0), (60, 50, 10, 10.0), (15, 40, 20, 50.0)]:
        got = lib.rlo_sw_weighted((ws + dt) * NS, ws, 60 * NS, prev, curr)
        assert abs(got - exp) < 0.1
        assert got == exp  # exact for these inputs


def test_window_start_alignment(lib):
    # windows dividing 86400 s align with the Unix epoch
    t = 1640000012 * NS + 345
    assert lib.rlo_window_start(t, 60 * NS) == 1640000012 - 1640000012 % 60 == 1639999980
    assert lib.rlo_window_start(t, 3600 * NS) == 1639998000
    # Go's Truncate is relative to Jan 1 year 1: 7 s windows are
    # offset by 62135596800 mod 7 = 4 s, one-week windows by 259200 s
    assert (62135596800 % 7) == 4
    for t in [T0, T0 + 123456789, 1640000000 * NS]:
        ws = lib.rlo_window_start(t, 7 * NS)
        assert (ws + 62135596800) % 7 == 0 and ws * NS <= t < ws * NS + 7 * NS
        wk = lib.rlo_window_start(t, 7 * 86400 * NS)
        assert (wk - 259200) % (7 * 86400) == 0 or (wk + 62135596800) % (7 * 86400) == 0
    # sub-second windows: Unix() drops the fraction
    assert lib.rlo_window_start(1640000000 * NS + 750_000_000, 500_000_000) == 1640000000


def test_tb_reset_at_seconds_to_full(lib):
    for L, wsec in [(5, 60), (20, 12), (100, 60), (10, 1), (7, 3600), (1000, 86400)]:
        rate = lib.rlo_tb_refill_rate(L, wsec * NS)
        assert L / rate == float(wsec)


def test_go_f2i(lib):
    for x in [0.0, -0.5, 1.9, -1.9, 9.2e18, -9.2e18, 2.0 ** 63, -(2.0 ** 63), float("nan"), float("inf"),
              -float("inf"), 1e300]:
        assert lib.rlo_go_f2i(x) == P.go_f2i(x), x
    assert lib.rlo_go_f2i(2.0 ** 63) == -(1 << 63)
    assert lib.rlo_go_f2i(-(2.0 ** 63)) == -(1 << 63)


def test_duration_seconds(lib):
    for d in [1, 999_999_999, NS, 1_500_000_000, 12 * NS, 365 * 86400 * NS, 31535999999999999]:
        assert lib.rlo_duration_seconds(d) == P.duration_seconds(d)
    # Seconds() rounds up near 2^24 s (SURVEY.md §7 hard part 4)
    assert P.duration_seconds(31535999999999999) == 31536000.0


def test_lua_tostring_roundtrip(lib):
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.random(2000) * 20, rng.random(2000) * 1e-6, T0 / 1e9 + rng.random(2000),
                         [1.0000610351562500, 0.999999999999995, 1e-300, 5e-324, 1.7e308]])
    for x in xs:
        x = float(x)
        assert lib.rlo_lua_tostring_roundtrip(x, 0) == float("%.14g" % x)
        assert lib.rlo_lua_tostring_roundtrip(x, 1) == x
    # the flip called out in SURVEY.md §0.4
    assert float("%.14g" % 0.999999999999995) == 1.0


# --- C oracle vs independent Python restatement --------------------------------

from tracegen import CONFIG_SETS, random_config_trace, random_trace, skewed_trace  # noqa: E402


@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("kind", ["tb", "sw", "fw", "mixed"])
@pytest.mark.parametrize("ff", [False, True])
def test_c_vs_python(lib, profile, kind, ff):
    configs = CONFIG_SETS[kind]
    seed = {"tb": 1, "sw": 2, "fw": 3, "mixed": 4}[kind] * 10 + profile * 2 + int(ff)
    # one config per key (contract: key ids are unique per config)
    keys, ts, n, cfg, sms = random_trace(seed, 3000, 40, configs, fastforward=ff, big_n=True)
    c = oracle.OracleSim(profile)
    p = P.Sim(profile)
    for a, L, W in configs:
        assert c.add_config(a, L, W) == p.add_config(a, L, W)
    dec, rem, retry, reset, tok = c.decide(keys, ts, n, cfg, sms)
    for i in range(len(keys)):
        d = p.decide(int(keys[i]), int(ts[i]), int(n[i]), int(cfg[i]), None if sms is None else int(sms[i]))
        got = (int(dec[i]), int(rem[i]), int(retry[i]), int(reset[i]))
        assert got == d[:4], (i, got, d)
        if configs[cfg[i]][0] == 1 and d[0] in (0, 1):
            assert tok[i] == d[4] or (math.isnan(tok[i]) and math.isnan(d[4]))


@pytest.mark.parametrize("seed", range(8))
def test_c_vs_python_random_configs(lib, seed):
    # the GPU parity suite's random configurations (limits 1 .. 1e12, windows
    # 1 ms .. a day): the two restatements agree at those scales too
    configs, (keys, ts, n, cfg, _) = random_config_trace(1000 + seed, 0 if seed >= 4 else 1 + seed % 3, 3000)
    profile = seed % 2
    c = oracle.OracleSim(profile)
    p = P.Sim(profile)
    for a, L, W in configs:
        assert c.add_config(a, L, W) == p.add_config(a, L, W)
    dec, rem, retry, reset, tok = c.decide(keys, ts, n, cfg)
    for i in range(len(keys)):
        d = p.decide(int(keys[i]), int(ts[i]), int(n[i]), int(cfg[i]), None)
        got = (int(dec[i]), int(rem[i]), int(retry[i]), int(reset[i]))
        assert got == d[:4], (i, got, d)
        if configs[cfg[i]][0] == 1 and d[0] in (0, 1):
            assert tok[i] == d[4] or (math.isnan(tok[i]) and math.isnan(d[4]))


@pytest.mark.parametrize("wi", range(3))
@pytest.mark.parametrize("alg", [1, 2, 3, 0])
def test_c_vs_python_long_windows(lib, alg, wi):
    # the GPU suite's long windows (1 d .. 365 d, Seconds() rounding at 2^24 s,
    # refill rates down to 3e-8 tokens/s): both restatements agree there too
    from tracegen import long_window_trace
    configs, (keys, ts, n, cfg, _) = long_window_trace(1200 + 10 * wi + alg, alg, 4000, wi=wi, n_light=300)
    profile = (alg + wi) % 2
    c = oracle.OracleSim(profile)
    p = P.Sim(profile)
    for a, L, W in configs:
        assert c.add_config(a, L, W) == p.add_config(a, L, W)
    dec, rem, retry, reset, tok = c.decide(keys, ts, n, cfg)
    for i in range(len(keys)):
        d = p.decide(int(keys[i]), int(ts[i]), int(n[i]), int(cfg[i]), None)
        got = (int(dec[i]), int(rem[i]), int(retry[i]), int(reset[i]))
        assert got == d[:4], (i, got, d)
        if configs[cfg[i]][0] == 1 and d[0] in (0, 1):
            assert tok[i] == d[4] or (math.isnan(tok[i]) and math.isnan(d[4]))


@pytest.mark.parametrize("profile", [0, 1])
@pytest.mark.parametrize("kind", ["sw", "fw", "mixed"])
def test_c_vs_python_skewed_clocks(lib, profile, kind):
    # per-key times going back by one or more windows (skewed app servers)
    configs = CONFIG_SETS[kind]
    keys, ts, n, cfg, sms = skewed_trace(500 + profile, 3000, 30, configs, big_n=True)
    c = oracle.OracleSim(profile)
    p = P.Sim(profile)
    for a, L, W in configs:
        assert c.add_config(a, L, W) == p.add_config(a, L, W)
    dec, rem, retry, reset, tok = c.decide(keys, ts, n, cfg, sms)
    for i in range(len(keys)):
        d = p.decide(int(keys[i]), int(ts[i]), int(n[i]), int(cfg[i]), int(sms[i]))
        assert (int(dec[i]), int(rem[i]), int(retry[i]), int(reset[i])) == d[:4], i


def test_overflow_is_an_error(lib):
    c = oracle.OracleSim(0)
    cid = c.add_config(3, 10, 60 * NS)
    big = (1 << 63) - 1
    dec, rem, retry, reset, _ = c.decide([1, 1, 1], [T0, T0 + 1, T0 + 2], [big, 1, 5], [cid] * 3)
    # count == MaxInt64 comes back through a Lua double as 2^63, which the
    # (long long) cast turns into MinInt64 <= Limit: the reference ALLOWS it.
    assert list(dec) == [1, 2, 2]   # then INCRBY overflows -> script error -> err != nil


def test_invalid_requests(lib):
    c = oracle.OracleSim(0)
    cid = c.add_config(1, 10, 60 * NS)
    dec, *_ = c.decide([1, 1, 1], [T0, T0, T0], [0, -5, 1], [cid, cid, 9])
    assert list(dec) == [3, 3, 3]
