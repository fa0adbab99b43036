"""CPU oracle package -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
always as the checker / baseline, never as the product path.

  c_oracle()       ctypes handle on oracle/librl_oracle.so (C restatement,
                   rl_oracle.c; glibc "%.14g"/strtod = Redis's Lua conversions)
  rl_oracle_py     independent pure-Python restatement (small traces)
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(_HERE, "librl_oracle.so")

TOKEN_BUCKET, SLIDING_WINDOW, FIXED_WINDOW = 1, 2, 3
REDIS7, MINIREDIS = 0, 1


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


_lib = None


def c_oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        lib = C.CDLL(SO)
        vp = C.c_void_p
        lib.rlo_create.restype = vp
        lib.rlo_create.argtypes = [C.c_int]
        lib.rlo_destroy.argtypes = [vp]
        lib.rlo_add_config.restype = C.c_int
        lib.rlo_add_config.argtypes = [vp, C.c_int, C.c_int64, C.c_int64]
        lib.rlo_decide.argtypes = [vp, C.c_size_t] + [vp] * 10
        lib.rlo_reset.argtypes = [vp, C.c_uint32, C.c_uint64, C.c_int64, C.c_int64]
        lib.rlo_duration_seconds.restype = C.c_double
        lib.rlo_duration_seconds.argtypes = [C.c_int64]
        lib.rlo_go_f2i.restype = C.c_int64
        lib.rlo_go_f2i.argtypes = [C.c_double]
        lib.rlo_window_start.restype = C.c_int64
        lib.rlo_window_start.argtypes = [C.c_int64, C.c_int64]
        lib.rlo_lua_tostring_roundtrip.restype = C.c_double
        lib.rlo_lua_tostring_roundtrip.argtypes = [C.c_double, C.c_int]
        lib.rlo_sw_weighted.restype = C.c_double
        lib.rlo_sw_weighted.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64]
        lib.rlo_tb_refill_rate.restype = C.c_double
        lib.rlo_tb_refill_rate.argtypes = [C.c_int64, C.c_int64]
        lib.rlo_tb_reset_at.restype = C.c_int64
        lib.rlo_tb_reset_at.argtypes = [C.c_int64, C.c_int64, C.c_double]
        lib.rlo_live_keys.restype = C.c_size_t
        lib.rlo_live_keys.argtypes = [vp, C.c_int64]
        lib.rlo_decide_timed.argtypes = [vp, C.c_size_t] + [vp] * 9
        lib.rlo_keys.restype = C.c_size_t
        lib.rlo_keys.argtypes = [vp, C.c_int64, vp, vp, vp, C.c_size_t]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleSim:
    """The reference Go+Redis path on the CPU (oracle/rl_oracle.c)."""

    def __init__(self, profile=REDIS7):
        self.lib = c_oracle()
        self.h = self.lib.rlo_create(profile)

    def __del__(self):
        try:
            self.lib.rlo_destroy(self.h)
        except Exception:
            pass

    def add_config(self, alg, limit, window_ns):
        return self.lib.rlo_add_config(self.h, alg, limit, window_ns)

    def decide(self, key, ts, n, cfg, server_ms=None):
        key = np.ascontiguousarray(key, np.uint64)
        ts = np.ascontiguousarray(ts, np.int64)
        n = np.ascontiguousarray(n, np.int64)
        cfg = np.ascontiguousarray(cfg, np.uint32)
        sms = None if server_ms is None else np.ascontiguousarray(server_ms, np.int64)
        m = key.size
        dec = np.empty(m, np.uint8)
        rem = np.empty(m, np.int64)
        retry = np.empty(m, np.int64)
        reset = np.empty(m, np.int64)
        tok = np.empty(m, np.float64)
        self.lib.rlo_decide(self.h, m, _p(key), _p(ts), _p(n), _p(cfg), _p(sms), _p(dec), _p(rem),
                            _p(retry), _p(reset), _p(tok))
        return dec, rem, retry, reset, tok

    def decide_timed(self, key, ts, n, cfg):
        """one call per request, each timed: (decision, call_ns)"""
        key = np.ascontiguousarray(key, np.uint64)
        ts = np.ascontiguousarray(ts, np.int64)
        n = np.ascontiguousarray(n, np.int64)
        cfg = np.ascontiguousarray(cfg, np.uint32)
        m = key.size
        dec, rem, retry, reset, call = (np.empty(m, np.uint8), np.empty(m, np.int64), np.empty(m, np.int64),
                                        np.empty(m, np.int64), np.empty(m, np.int64))
        self.lib.rlo_decide_timed(self.h, m, _p(key), _p(ts), _p(n), _p(cfg), _p(dec), _p(rem), _p(retry),
                                  _p(reset), _p(call))
        return dec, call

    def reset(self, cfg, key, ts, server_ms=0):
        self.lib.rlo_reset(self.h, cfg, key, ts, server_ms)

    def keys(self, s_ms):
        """live keys at server time s_ms: [(id, kind, ws)] (kind 0 hash, 1 window)"""
        n = self.lib.rlo_keys(self.h, s_ms, None, None, None, 0)
        ids, kind, ws = np.empty(n, np.uint64), np.empty(n, np.uint8), np.empty(n, np.int64)
        self.lib.rlo_keys(self.h, s_ms, _p(ids), _p(kind), _p(ws), n)
        return list(zip(ids.tolist(), kind.tolist(), ws.tolist()))
