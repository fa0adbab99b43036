"""The reference's integration tests, restated as backend-agnostic scenarios.

Each function mirrors one test in the reference repo (file:line cited) with
the same assertions; where the reference can only assert a range (real
time.Now()/time.Sleep), the deterministic clock lets us also pin the exact
value.  `be` is a tests/backends.py backend; limiters come from be.new().
The reference ran these against miniredis (profile MINIREDIS).
"""
from __future__ import annotations

import pytest

from backends import NS, ErrInvalidN

MINUTE = 60 * NS
SEC = NS


# ----------------------------------------------------------------- fixed window
def fw_allow(be):  # fixedwindow_integration_test.go:27-65
    lim = be.new("fixed_window", 5, MINUTE)
    r = lim.allow("user:123")
    assert r.Allowed and r.Limit == 5 and r.Remaining == 4 and r.RetryAfter == 0
    for _ in range(4):
        assert lim.allow("user:123").Allowed
    r = lim.allow("user:123")
    assert not r.Allowed and r.Remaining == 0 and r.RetryAfter > 0
    assert r.RetryAfter == r.ResetAt - be.clock.t           # single-clock RetryAfter


def fw_allow_n(be):  # fixedwindow_integration_test.go:67-102
    lim = be.new("fixed_window", 10, MINUTE)
    r = lim.allow_n("api:endpoint", 3)
    assert r.Allowed and r.Remaining == 7
    r = lim.allow_n("api:endpoint", 5)
    assert r.Allowed and r.Remaining == 2
    r = lim.allow_n("api:endpoint", 3)
    assert not r.Allowed and r.Remaining == 0 and r.RetryAfter > 0
    # the denied INCRBY still counted (fixedwindow.go:22): count is now 11
    r = lim.allow_n("api:endpoint", 1)
    assert not r.Allowed and r.Remaining == 0


def invalid_n(be, algorithm):  # *_integration_test.go AllowN_InvalidTokens
    lim = be.new(algorithm, 10, MINUTE)
    for n in (0, -1, -100):
        with pytest.raises(ErrInvalidN):
            lim.allow_n("test-key", n)


def fw_reset(be):  # fixedwindow_integration_test.go:104-142
    lim = be.new("fixed_window", 5, MINUTE)
    for _ in range(5):
        assert lim.allow("user:456").Allowed
    assert not lim.allow("user:456").Allowed
    lim.reset("user:456")
    r = lim.allow("user:456")
    assert r.Allowed and r.Remaining == 4


def fw_window_boundary(be):  # fixedwindow_integration_test.go:144-181
    lim = be.new("fixed_window", 3, 2 * SEC)
    # stay inside one Go window: start at a window boundary
    be.clock.t = (be.clock.t // (2 * SEC) + 1) * 2 * SEC
    for i in range(3):
        assert lim.allow("user:boundary").Allowed, f"request {i + 1} should be allowed"
    assert not lim.allow("user:boundary").Allowed
    be.clock.fast_forward(3 * SEC)
    r = lim.allow("user:boundary")
    assert r.Allowed and r.Remaining == 2


def fw_multiple_keys(be):  # fixedwindow_integration_test.go:183-219
    lim = be.new("fixed_window", 2, MINUTE)
    r = lim.allow_n("user:1", 2)
    assert r.Allowed and r.Remaining == 0
    r = lim.allow("user:2")
    assert r.Allowed and r.Remaining == 1
    assert not lim.allow("user:1").Allowed


def fail_open(be, algorithm):  # *_integration_test.go FailOpen
    lim = be.new(algorithm, 5, MINUTE, fail_open=True)
    lim.close()  # reference: mr.Close() -- storage unavailable
    r = lim.allow("user:failopen")
    assert r.Allowed and r.Remaining == 0 and r.Limit == 5 and r.RetryAfter == 0


def fail_closed(be, algorithm):  # *_integration_test.go FailClosed
    lim = be.new(algorithm, 5, MINUTE, fail_open=False)
    lim.close()
    with pytest.raises(RuntimeError, match="failed to check rate limit"):
        lim.allow("user:failclosed")


def reset_at(be, algorithm):  # fixedwindow_integration_test.go:276-305 / slidingwindow :310-338
    lim = be.new(algorithm, 10, MINUTE)
    now = be.clock.t + 50_000   # the call's own time
    r = lim.allow("user:reset-time")
    assert r.ResetAt > now
    expected = (now // MINUTE) * MINUTE + MINUTE   # 60 s windows align with the epoch
    assert r.ResetAt == expected


# --------------------------------------------------------------- sliding window
def sw_allow(be):  # slidingwindow_integration_test.go:27-65
    lim = be.new("sliding_window", 5, MINUTE)
    # start early in a window so the previous (absent) window has no weight
    be.clock.t = (be.clock.t // MINUTE + 1) * MINUTE
    r = lim.allow("user:123")
    assert r.Allowed and r.Limit == 5 and r.Remaining == 4 and r.RetryAfter == 0
    for _ in range(4):
        assert lim.allow("user:123").Allowed
    r = lim.allow("user:123")
    assert not r.Allowed and r.Remaining == 0 and r.RetryAfter > 0


def sw_allow_n(be):  # slidingwindow_integration_test.go:67-102
    lim = be.new("sliding_window", 10, MINUTE)
    r = lim.allow_n("api:endpoint", 3)
    assert r.Allowed and r.Remaining == 7
    r = lim.allow_n("api:endpoint", 5)
    assert r.Allowed and r.Remaining == 2
    r = lim.allow_n("api:endpoint", 3)
    assert not r.Allowed and r.Remaining == 0 and r.RetryAfter > 0


def sw_reset(be):  # slidingwindow_integration_test.go:138-176
    lim = be.new("sliding_window", 5, MINUTE)
    for _ in range(5):
        assert lim.allow("user:456").Allowed
    assert not lim.allow("user:456").Allowed
    lim.reset("user:456")
    r = lim.allow("user:456")
    assert r.Allowed and r.Remaining == 4


def sw_window_boundary(be):  # slidingwindow_integration_test.go:178-215
    lim = be.new("sliding_window", 3, 2 * SEC)
    be.clock.t = (be.clock.t // (2 * SEC) + 1) * 2 * SEC
    for i in range(3):
        assert lim.allow("user:boundary").Allowed, f"request {i + 1} should be allowed"
    assert not lim.allow("user:boundary").Allowed
    be.clock.fast_forward(3 * SEC)
    r = lim.allow("user:boundary")
    assert r.Allowed and r.Remaining == 2


def sw_multiple_keys(be):  # slidingwindow_integration_test.go:217-253
    lim = be.new("sliding_window", 2, MINUTE)
    be.clock.t = (be.clock.t // MINUTE + 1) * MINUTE
    r = lim.allow_n("user:1", 2)
    assert r.Allowed and r.Remaining == 0
    r = lim.allow("user:2")
    assert r.Allowed and r.Remaining == 1
    assert not lim.allow("user:1").Allowed


def sw_smooth(be):  # slidingwindow_integration_test.go:370-403
    lim = be.new("sliding_window", 10, 10 * SEC)
    be.clock.fast_forward(-5 * SEC)
    for _ in range(8):
        lim.allow("user:smooth")
    be.clock.fast_forward(10 * SEC)
    assert lim.allow("user:smooth").Allowed


def sw_weighted_prev_window(be):
    """Beyond the reference tests: the previous window's count is weighted by
    (1 - progress) (slidingwindow.go:190-197) -- 8 requests late in window k,
    then at 50% of window k+1 the weighted count is 8*0.5 + 1 = 5."""
    lim = be.new("sliding_window", 10, 10 * SEC)
    w0 = (be.clock.t // (10 * SEC) + 1) * 10 * SEC
    be.clock.t = w0 + 9 * SEC
    for _ in range(8):
        assert lim.allow("k").Allowed
    be.clock.t = w0 + 15 * SEC - 50_000
    r = lim.allow("k")           # at exactly 50% of the next window
    assert r.Allowed and r.Remaining == 10 - 5


# ---------------------------------------------------------------- token bucket
def tb_allow(be):  # tokenbucket_integration_test.go:27-64
    lim = be.new("token_bucket", 5, MINUTE)
    r = lim.allow("user:123")
    assert r.Allowed and r.Limit == 5 and r.Remaining == 4
    for _ in range(4):
        assert lim.allow("user:123").Allowed
    r = lim.allow("user:123")
    assert not r.Allowed and r.Remaining == 0 and r.RetryAfter > 0
    assert r.RetryAfter == 12 * SEC                     # 1 / (5/60.0) == 12.0 exactly


def tb_allow_n(be):  # tokenbucket_integration_test.go:66-100
    lim = be.new("token_bucket", 10, MINUTE)
    r = lim.allow_n("api:endpoint", 3)
    assert r.Allowed and r.Remaining == 7
    r = lim.allow_n("api:endpoint", 5)
    assert r.Allowed and r.Remaining == 2
    r = lim.allow_n("api:endpoint", 3)
    assert not r.Allowed and r.Remaining == 2           # denied: floor(tokens), not 0


def tb_refill(be):  # tokenbucket_integration_test.go:136-172
    lim = be.new("token_bucket", 10, SEC)
    r = lim.allow_n("user:refill", 10)
    assert r.Allowed and r.Remaining == 0
    assert not lim.allow("user:refill").Allowed
    be.clock.sleep(500_000_000)
    assert lim.allow_n("user:refill", 4).Allowed


def tb_burst(be):  # tokenbucket_integration_test.go:174-201
    lim = be.new("token_bucket", 100, MINUTE)
    r = lim.allow_n("user:burst", 100)
    assert r.Allowed and r.Remaining == 0
    assert not lim.allow("user:burst").Allowed


def tb_reset(be):  # tokenbucket_integration_test.go:203-241
    lim = be.new("token_bucket", 5, MINUTE)
    for _ in range(5):
        assert lim.allow("user:456").Allowed
    assert not lim.allow("user:456").Allowed
    lim.reset("user:456")
    r = lim.allow("user:456")
    assert r.Allowed and r.Remaining == 4


def tb_multiple_keys(be):  # tokenbucket_integration_test.go:243-279
    lim = be.new("token_bucket", 5, MINUTE)
    r = lim.allow_n("user:1", 5)
    assert r.Allowed and r.Remaining == 0
    r = lim.allow("user:2")
    assert r.Allowed and r.Remaining == 4
    assert not lim.allow("user:1").Allowed


def tb_retry_after(be):  # tokenbucket_integration_test.go:336-367
    lim = be.new("token_bucket", 10, 10 * SEC)
    assert lim.allow_n("user:retry", 10).Allowed
    r = lim.allow_n("user:retry", 5)
    assert not r.Allowed
    assert 4 * SEC < r.RetryAfter < 6 * SEC
    assert r.RetryAfter == 5 * SEC                      # rate 1/s, floor(tokens) == 0


def tb_continuous_refill(be):  # tokenbucket_integration_test.go:397-430
    lim = be.new("token_bucket", 20, SEC)
    r = lim.allow_n("user:continuous", 10)
    assert r.Allowed and r.Remaining == 10
    be.clock.sleep(100_000_000)
    r = lim.allow("user:continuous")
    assert r.Allowed and 10 <= r.Remaining <= 12


def tb_max_capacity(be):  # tokenbucket_integration_test.go:432-462
    lim = be.new("token_bucket", 10, SEC)
    assert lim.allow("user:maxcap").Remaining == 9
    be.clock.sleep(2 * SEC)
    r = lim.allow("user:maxcap")
    assert r.Allowed and r.Remaining == 9


# ------------------------------------------------------------- key names
def _minute_start(t):
    return t // NS // 60 * 60      # Truncate(time.Minute): year 1 is minute-aligned with the Unix epoch


def fw_custom_prefix(be):  # fixedwindow_integration_test.go:307-333
    lim = be.new("fixed_window", 5, MINUTE, prefix="custom")
    assert lim.allow("test-key").Allowed
    keys = be.keys()
    assert len(keys) == 1 and "custom:" in keys[0]
    assert keys == ["custom:test-key:%d" % _minute_start(be.clock.t)]   # fixedwindow.go:139-141


def sw_custom_prefix(be):  # slidingwindow_integration_test.go:340-368
    lim = be.new("sliding_window", 5, MINUTE, prefix="custom")
    assert lim.allow("test-key").Allowed
    keys = be.keys()
    assert len(keys) >= 1 and all("custom:" in k for k in keys)
    # EXPIRE on the missing previous-window key is a no-op: one key
    assert keys == ["custom:test-key:%d" % _minute_start(be.clock.t)]   # slidingwindow.go:150-152


def tb_custom_prefix(be):  # tokenbucket_integration_test.go:369-395
    lim = be.new("token_bucket", 5, MINUTE, prefix="custom")
    assert lim.allow("test-key").Allowed
    keys = be.keys()
    assert len(keys) == 1 and "custom:" in keys[0]
    assert keys == ["custom:test-key"]                                 # tokenbucket.go:95


def prefix_isolation(be):  # builder scenario: FormatKey namespaces (config.go:81-87)
    a = be.new("token_bucket", 5, MINUTE, prefix="custom")
    b = be.new("token_bucket", 5, MINUTE)                  # "ratelimit" (config.go:62-64)
    assert a.allow_n("k", 5).Remaining == 0
    r = b.allow("k")
    assert r.Allowed and r.Remaining == 4                   # ratelimit:k is another key
    a.reset("k")                                            # DEL custom:k only
    assert a.allow("k").Remaining == 4
    assert b.allow("k").Remaining == 3
    assert be.keys() == ["custom:k", "ratelimit:k"]


def shared_prefix(be):  # builder scenario: two limiters, one prefix, one Redis key
    a = be.new("token_bucket", 5, MINUTE)
    b = be.new("token_bucket", 5, MINUTE)
    assert a.allow_n("k", 3).Remaining == 2
    r = b.allow_n("k", 2)
    assert r.Allowed and r.Remaining == 0                   # the same bucket
    assert not a.allow("k").Allowed
    fw = be.new("fixed_window", 5, MINUTE, prefix="p")
    sw = be.new("sliding_window", 5, MINUTE, prefix="p")
    be.clock.t = (be.clock.t // MINUTE + 1) * MINUTE        # both in one window
    assert fw.allow_n("w", 3).Remaining == 2
    r = sw.allow("w")                                       # INCRBY on the same p:w:ws counter
    assert r.Allowed and r.Remaining == 1
    assert not fw.allow_n("w", 2).Allowed
    assert be.keys() == ["p:w:%d" % _minute_start(be.clock.t), "ratelimit:k"]


ALL = [
    ("fw_allow", fw_allow), ("fw_allow_n", fw_allow_n),
    ("fw_invalid_n", lambda be: invalid_n(be, "fixed_window")),
    ("fw_reset", fw_reset), ("fw_window_boundary", fw_window_boundary),
    ("fw_multiple_keys", fw_multiple_keys),
    ("fw_fail_open", lambda be: fail_open(be, "fixed_window")),
    ("fw_fail_closed", lambda be: fail_closed(be, "fixed_window")),
    ("fw_reset_at", lambda be: reset_at(be, "fixed_window")),
    ("sw_allow", sw_allow), ("sw_allow_n", sw_allow_n),
    ("sw_invalid_n", lambda be: invalid_n(be, "sliding_window")),
    ("sw_reset", sw_reset), ("sw_window_boundary", sw_window_boundary),
    ("sw_multiple_keys", sw_multiple_keys), ("sw_smooth", sw_smooth),
    ("sw_weighted_prev_window", sw_weighted_prev_window),
    ("sw_fail_open", lambda be: fail_open(be, "sliding_window")),
    ("sw_fail_closed", lambda be: fail_closed(be, "sliding_window")),
    ("sw_reset_at", lambda be: reset_at(be, "sliding_window")),
    ("tb_allow", tb_allow), ("tb_allow_n", tb_allow_n),
    ("tb_invalid_n", lambda be: invalid_n(be, "token_bucket")),
    ("tb_refill", tb_refill), ("tb_burst", tb_burst), ("tb_reset", tb_reset),
    ("tb_multiple_keys", tb_multiple_keys), ("tb_retry_after", tb_retry_after),
    ("tb_continuous_refill", tb_continuous_refill), ("tb_max_capacity", tb_max_capacity),
    ("tb_fail_open", lambda be: fail_open(be, "token_bucket")),
    ("tb_fail_closed", lambda be: fail_closed(be, "token_bucket")),
    ("fw_custom_prefix", fw_custom_prefix), ("sw_custom_prefix", sw_custom_prefix),
    ("tb_custom_prefix", tb_custom_prefix),
    ("prefix_isolation", prefix_isolation), ("shared_prefix", shared_prefix),
]
