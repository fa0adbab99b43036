"""Observability decorators (docs/ADR/003-decorator-pattern-for-observability.md
:26-125) over the GPU limiter: decisions pass through unchanged; metrics count
(allowed, error type) and a latency histogram; logging records errors and
denials."""
import re

import pytest

pytestmark = pytest.mark.gpu

NS = 1_000_000_000
T0 = 1_760_000_000 * NS


def test_metrics_and_logging_decorators(rl):
    eng = rl.LimiterEngine(tb_capacity=1 << 12, win_capacity=1 << 12, max_batch=1 << 12)
    lim = rl.new_limiter(eng, "token_bucket", 3, 60 * NS)
    plain = rl.new_limiter(eng, "token_bucket", 3, 60 * NS, prefix="plain")
    lim.add_metrics()
    lim.add_logging(capacity=64)
    got, want = [], []
    for i in range(5):   # capacity 3: allow x3, deny x2 -- same as the undecorated limiter
        got.append(lim.allow("alice", T0 + i)[0])
        want.append(plain.allow("alice", T0 + i)[0])
    assert got == want
    assert [r.Allowed for r in got] == [True, True, True, False, False]
    r, err, code = lim.allow_n("alice", 0, T0 + 10)            # ErrInvalidN
    assert r is None and code == rl.RLL_ERR_INVALID_N
    text = lim.metrics_text()
    count = lambda allowed, error: int(re.search(
        r'rate_limiter_requests_total\{algorithm="token_bucket",allowed="%s",error="%s"\} (\d+)' % (allowed, error),
        text).group(1))
    assert count("true", "none") == 3
    assert count("false", "none") == 2
    assert count("false", "invalid_n") == 1
    assert 'rate_limiter_decision_seconds_bucket{algorithm="token_bucket",le="+Inf"} 6' in text
    assert 'rate_limiter_decision_seconds_count{algorithm="token_bucket"} 6' in text
    # logging wraps metrics: 2 denials at debug (0), the ErrInvalidN at error (3),
    # pulled from the library's queue (no callback into the caller)
    logs, dropped = lim.drain_logs()
    assert dropped == 0 and lim.drain_logs() == ([], 0)
    assert [lv for lv, _, _ in logs] == [0, 0, 3]
    assert logs[0][1] == "request denied" and "key=alice" in logs[0][2] and "limit=3" in logs[0][2]
    assert logs[2][1] == "rate limiter error" and "invalid n" in logs[2][2]
    # a full queue drops its oldest records
    small = rl.new_limiter(eng, "fixed_window", 1, 60 * NS, prefix="small")
    small.add_logging(capacity=2)
    for i in range(5):
        small.allow("bob", T0 + i)
    logs, dropped = small.drain_logs()
    assert len(logs) == 2 and dropped == 2
