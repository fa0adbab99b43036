"""bench.py's host-side arithmetic (CPU): the hot-owner bound the N > 1 line
reports, and the replay-timeline words it reads back (10-ns realtime ticks,
low 32 bits, so every difference must survive a wrap of the counter)."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_hot_owner_bound_is_batch_over_chain_time(bench):
    # chain rate / hot share = (hot / t) / (hot / m) = m / t, whatever the share
    for hot, us, m in ((123847, 290.0, 1_000_000), (247051, 538.36, 2_000_000), (1, 0.5, 10)):
        b = bench.hot_owner_bound(hot, us, m)
        assert b["bound_decisions_per_s"] == pytest.approx(m / (us * 1e-6), rel=1e-12)
        assert b["hot_share"] == pytest.approx(hot / m)
        assert b["chain_steps_per_s"] == pytest.approx(hot / (us * 1e-6))
        assert b["hot_key_requests_per_step"] == hot


@pytest.mark.parametrize("hot,us", [(0, 10.0), (100, 0.0), (-1, 5.0)])
def test_hot_owner_bound_absent_without_a_chain(bench, hot, us):
    assert bench.hot_owner_bound(hot, us, 1000) is None


@pytest.mark.parametrize("start", [0, 12345, 0xffffffff - 500, 0xffffffff])
def test_timeline_words_wrap(bench, start):
    dbgw = [0] * 96
    dbgw[13] = ~start & 0xffffffff               # the kernel keeps the first block's start complemented
    dbgw[16] = (start + 264) & 0xffffffff        # hot segment start, 2.64 us in
    dbgw[17] = (start + 29368) & 0xffffffff      # hot segment end, 293.68 us in
    dbgw[51] = (start + 239) & 0xffffffff        # a stamps-build word
    assert bench.hot_chain_us(dbgw) == pytest.approx(291.04)
    assert bench._rel_us(dbgw, 51) == pytest.approx(2.39)
    assert bench._rel_us(dbgw, 52) is None       # unset: a product build
