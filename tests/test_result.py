"""Result constructors (reference result.go:5-50), checked as the reference's
result_test.go:8-95 checks them; host code only (no GPU)."""
import ctypes as C

TIME_ZERO = -(1 << 63)   # RLL_TIME_ZERO: time.Time{}
NS = 1_000_000_000


def _fields(r):
    return (bool(r.allowed), r.limit, r.remaining, r.retry_after_ns, r.reset_at_ns)


def test_new_allowed_result(rl):
    # result_test.go:8-30
    reset = 1_760_000_060 * NS
    r = rl.rll_result()
    assert rl.lib.rll_new_allowed_result(100, 50, reset, C.byref(r)) == rl.RLL_OK
    assert _fields(r) == (True, 100, 50, 0, reset)


def test_new_denied_result(rl):
    # result_test.go:32-54
    reset = 1_760_000_060 * NS
    r = rl.rll_result()
    assert rl.lib.rll_new_denied_result(100, 30 * NS, reset, C.byref(r)) == rl.RLL_OK
    assert _fields(r) == (False, 100, 0, 30 * NS, reset)


def test_new_fail_open_result(rl):
    # result_test.go:56-74: allowed, zero limit/remaining/retry, zero ResetAt
    r = rl.rll_result()
    assert rl.lib.rll_new_fail_open_result(C.byref(r)) == rl.RLL_OK
    assert _fields(r) == (True, 0, 0, 0, TIME_ZERO)


def test_new_fail_closed_result(rl):
    # result_test.go:76-95
    r = rl.rll_result()
    assert rl.lib.rll_new_fail_closed_result(C.byref(r)) == rl.RLL_OK
    assert _fields(r) == (False, 0, 0, 0, TIME_ZERO)


def test_null_out_is_an_argument_error(rl):
    assert rl.lib.rll_new_fail_open_result(None) == rl.RLL_ERR_ARG
