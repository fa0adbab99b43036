"""The C-ABI library: loads on a CPU-only host and exports every function that
include/*.h declares (no GPU compute is called here)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include"))) if h.endswith(".h")]


def declared_functions(header_filter=None):
    names = []
    for h in HEADERS:
        if header_filter and not header_filter(os.path.basename(h)):
            continue
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names += re.findall(r"^\s*(?:int|rl_engine\s*\*)\s+(rll?_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


# include/rl_grpc.h is lib/librl_grpc.so (the native gRPC front end); every
# other header is lib/librl_amd.so
GRPC_H = "rl_grpc.h"


def test_headers_declare_the_boundary():
    names = declared_functions()
    for must in ["rl_engine_create", "rl_engine_destroy", "rl_config_register", "rl_decide_batch",
                 "rl_decide_batch_device", "rl_reset", "rl_last_error", "rll_new", "rll_allow_n",
                 "rl_coalescer_create", "rl_coalescer_submit", "rl_coalescer_wait", "rl_route_pack",
                 "rl_route_merge", "rl_decide_routed_device", "rl_route_unpack"]:
        assert must in names


@pytest.mark.parametrize("name", declared_functions(lambda h: h != GRPC_H))
def test_symbol_exported(rl, name):
    assert hasattr(rl.lib, name), name


@pytest.mark.parametrize("name", declared_functions(lambda h: h == GRPC_H))
def test_grpc_symbol_exported(rl, name):
    assert hasattr(rl.grpc_lib(), name), name


def test_q14_host_instantiation(rl):
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.random(20000) * 20, rng.random(20000) * 1e-7, 1.76e9 + rng.random(20000),
                        (rng.integers(0, 1 << 62, 20000).astype(np.uint64)).view(np.float64)])
    x = x[np.isfinite(x)]
    got = rl.q14_host(x)
    ref = np.array([float("%.14g" % v) for v in x])
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


def test_q14_host_decade_edges_and_tiny(rl):
    # regression: a value just below 10^k must keep decade k-1's 14 digits
    # (0.99999999999999 stays, it does not become 1)
    from tracegen import q14_edge_values
    x = q14_edge_values()
    got = rl.q14_host(x)
    ref = np.array([float("%.14g" % v) for v in x])
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64))


def test_host_mirror_without_gpu(rl):
    # config_test.go:8-178: Validate messages
    S, M, H = 10 ** 9, 60 * 10 ** 9, 3600 * 10 ** 9
    cases = [
        (None, 0, 0, "config cannot be nil"),
        ("token_bucket", 100, M, ""),
        ("sliding_window", 1000, H, ""),
        ("fixed_window", 50, S, ""),
        ("", 100, M, "algorithm is required"),
        ("invalid_algo", 100, M, "unknown algorithm"),
        ("token_bucket", 0, M, "limit must be greater than 0"),
        ("token_bucket", -10, M, "limit must be greater than 0"),
        ("token_bucket", 100, 0, "window must be greater than 0"),
        ("token_bucket", 100, -S, "window must be greater than 0"),
        ("token_bucket", 100, 500, "window too small"),
        ("token_bucket", 100, 400 * 24 * H, "window too large"),
    ]
    for alg, limit, window, want in cases:
        got = rl.config_validate(alg, limit, window)
        if want:
            assert want in got, (alg, limit, window, got)
        else:
            assert got == ""
    assert rl.config_validate("invalid_algo", 100, M) == \
        "unknown algorithm: invalid_algo (must be one of: token_bucket, sliding_window, fixed_window)"
    assert rl.config_validate("token_bucket", 100, -S) == "window must be greater than 0, got: -1s"
    assert rl.config_validate("token_bucket", 100, 500) == "window too small: 500ns (minimum: 1ms)"
    assert rl.config_validate("token_bucket", 100, 400 * 24 * H) == \
        "window too large: 9600h0m0s (maximum: 365 days)"
    # config_test.go:276-345: FormatKey (prefix None == nil *Config)
    assert rl.format_key("ratelimit", "user:123") == "ratelimit:user:123"
    assert rl.format_key("api", "user:123") == "api:user:123"
    assert rl.format_key("", "user:123") == "user:123"
    assert rl.format_key(None, "user:123") == "ratelimit:user:123"
    assert rl.format_key("app", "tenant:abc:user:xyz:resource:file") == "app:tenant:abc:user:xyz:resource:file"
    # Go time.Duration.String()
    for d, s in [(0, "0s"), (1, "1ns"), (1500, "1.5µs"), (1_000_000, "1ms"), (S, "1s"), (M, "1m0s"),
                 (H + 1, "1h0m0.000000001s"), (-S, "-1s"), (90 * M, "1h30m0s")]:
        assert rl.duration_string(d) == s
    # constructor with a nil engine (tokenbucket_test.go "nil client")
    with pytest.raises(rl.GoError, match="engine cannot be nil"):
        rl.new_limiter(None, "token_bucket", 10, M)
