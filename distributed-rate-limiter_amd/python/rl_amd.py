"""ctypes binding of the MI355X rate-limit engine (include/rl_engine.h) and of
its host mirror of the reference Go API (include/rl_limiter.h).

This is plumbing for tests and bench.py: the product is the HIP library
lib/librl_amd.so.  There is no CPU fallback: if the library is missing,
importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RL_AMD_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "librl_amd.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"HIP engine library not built: {LIB_PATH} (run `make -C distributed-rate-limiter_amd` "
        "or __graft_entry__.build())"
    )
lib = C.CDLL(LIB_PATH)

# --- constants (include/rl_engine.h) -----------------------------------------
RL_OK, RL_EINVAL, RL_ENOMEM, RL_EDEVICE, RL_ETIMEOUT, RL_EORDER = 0, -22, -12, -5, -110, -34
TOKEN_BUCKET, SLIDING_WINDOW, FIXED_WINDOW = 1, 2, 3
ALG_BY_NAME = {"token_bucket": TOKEN_BUCKET, "sliding_window": SLIDING_WINDOW, "fixed_window": FIXED_WINDOW}
PROFILE_REDIS7, PROFILE_MINIREDIS = 0, 1
DENIED, ALLOWED, ERROR, INVALID = 0, 1, 2, 3
KEY_RESERVED = (1 << 64) - 1

RLL_OK, RLL_ERR_INVALID_N, RLL_ERR_FAILED, RLL_ERR_CONFIG, RLL_ERR_RESET, RLL_ERR_ARG = 0, 1, 2, 3, 4, 5
NOW_WALL = -(1 << 63)
SMS_DEFAULT = -(1 << 63)


class _Sized(C.Structure):
    """an ABI struct whose first field is struct_size (include/rl_engine.h)"""

    def __init__(self, *args, **kw):
        super().__init__(C.sizeof(self), *args, **kw)


class rl_opts(_Sized):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("device", C.c_int32),
        ("profile", C.c_int32),
        ("tb_capacity", C.c_uint64),
        ("win_capacity", C.c_uint64),
        ("max_batch", C.c_uint32),
        ("flags", C.c_uint32),
        ("spill_capacity", C.c_uint64),
    ]


class rl_stats(_Sized):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("pad_", C.c_uint32),
        ("batches", C.c_uint64),
        ("decisions", C.c_uint64),
        ("last_segments", C.c_uint64),
        ("last_heavy", C.c_uint64),
        ("last_coop_rounds", C.c_uint64),
        ("last_coop_iters", C.c_uint64),
        ("sort_bits", C.c_uint32),
        ("sort_passes", C.c_uint32),
        ("stamp_cycles", C.c_uint64 * 7),
        ("coop_ends", C.c_uint64 * 4),
        ("sort_predicted", C.c_uint64),
        ("light_batches", C.c_uint64),
    ]


class rll_result(C.Structure):
    _fields_ = [
        ("allowed", C.c_uint8),
        ("limit", C.c_int64),
        ("remaining", C.c_int64),
        ("retry_after_ns", C.c_int64),
        ("reset_at_ns", C.c_int64),
    ]


class rl_table_info(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("pad_", C.c_uint32)] + [(k, C.c_uint64) for k in ("tb_capacity", "tb_used", "tb_live", "win_capacity", "win_used",
                                          "win_live", "spill_capacity", "spill_used", "spill_live")]


class rl_coalescer_opts(_Sized):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("max_batch", C.c_uint32),
        ("max_in_flight", C.c_uint32),
        ("gc_high_pct", C.c_uint32),
        ("linger_ns", C.c_int64),
        ("queue_cap", C.c_uint64),
        ("gc_interval_ns", C.c_int64),
        ("gc_margin_ms", C.c_int64),
        ("gc_max_tb_capacity", C.c_uint64),
        ("gc_max_win_capacity", C.c_uint64),
    ]


class rl_coalescer_stats(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("pad_", C.c_uint32)] + [
        (k, C.c_uint64) for k in ("submitted", "decided", "batches", "max_batch_seen", "pending", "expired",
                                  "cancelled", "gc_runs", "gc_checks", "gc_failures")]


vp = C.c_void_p
# rl_batch_fn (include/rl_coalescer.h)
BATCH_FN = C.CFUNCTYPE(C.c_int, vp, C.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp)
RESET_FN = C.CFUNCTYPE(C.c_int, vp, C.c_uint32, C.c_uint64, C.c_int64)
INFO_FN = C.CFUNCTYPE(C.c_int, vp, C.c_int64, C.POINTER(rl_table_info))
GC_FN = C.CFUNCTYPE(C.c_int, vp, C.c_int64, C.c_uint64, C.c_uint64, C.POINTER(rl_table_info))


class rl_coalescer_backend(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("batch", BATCH_FN), ("reset", RESET_FN), ("table_info", INFO_FN),
                ("gc", GC_FN), ("user", vp)]

_sig = {
    "rl_engine_create": (C.c_int, [C.POINTER(rl_opts), C.POINTER(vp)]),
    "rl_engine_destroy": (C.c_int, [vp]),
    "rl_config_register": (C.c_int, [vp, C.c_uint8, C.c_int64, C.c_int64, C.POINTER(C.c_uint32)]),
    "rl_decide_batch": (C.c_int, [vp, C.c_size_t] + [vp] * 10),
    "rl_decide_batch_device": (C.c_int, [vp, C.c_size_t] + [vp] * 11),
    "rl_engine_sync": (C.c_int, [vp]),
    "rl_reset": (C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_int64]),
    "rl_reset_device": (C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_int64, vp]),
    "rl_engine_stats": (C.c_int, [vp, C.POINTER(rl_stats)]),
    "rl_engine_set_timing": (C.c_int, [vp, C.c_int]),
    "rl_table_info_get": (C.c_int, [vp, C.c_int64, C.POINTER(rl_table_info)]),
    "rl_table_gc": (C.c_int, [vp, C.c_int64, C.c_uint64, C.c_uint64, C.POINTER(rl_table_info)]),
    "rl_engine_stage_times": (C.c_int, [vp, vp, C.c_int, C.POINTER(C.c_uint64)]),
    "rl_last_error": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
    "rl_engine_debug_words": (C.c_int, [vp, vp, C.c_size_t]),
    "rl_engine_debug_stamps": (C.c_int, [vp, vp, C.c_size_t]),
    "rl_selftest_q14_host": (C.c_int, [vp, vp, C.c_size_t]),
    "rl_selftest_q14_device": (C.c_int, [vp, vp, vp, C.c_size_t]),
    "rll_engine_new": (C.c_int, [C.POINTER(rl_opts), C.POINTER(vp), C.c_char_p, C.c_size_t]),
    "rll_engine_free": (C.c_int, [vp]),
    "rll_engine_raw": (vp, [vp]),
    "rll_engine_set_server_ms": (C.c_int, [vp, C.c_int64]),
    "rll_keys": (C.c_int, [vp, C.c_int64, C.c_char_p, C.c_size_t]),
    "rl_table_keys": (C.c_int, [vp, C.c_int64, vp, C.c_size_t, C.POINTER(C.c_uint64)]),
    "rll_config_validate": (C.c_int, [C.c_char_p, C.c_int64, C.c_int64, C.c_char_p, C.c_size_t]),
    "rll_format_key": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]),
    "rll_duration_string": (C.c_int, [C.c_int64, C.c_char_p, C.c_size_t]),
    "rll_new": (C.c_int, [vp, C.c_char_p, C.c_int64, C.c_int64, C.c_char_p, C.c_int, C.c_int,
                          C.POINTER(vp), C.c_char_p, C.c_size_t]),
    "rll_allow_n": (C.c_int, [vp, C.c_char_p, C.c_size_t, C.c_int64, C.c_int64, C.c_int,
                              C.POINTER(rll_result), C.c_char_p, C.c_size_t]),
    "rll_allow_batch": (C.c_int, [vp, C.c_size_t, vp, vp, vp, vp, vp, vp]),
    "rll_reset": (C.c_int, [vp, C.c_char_p, C.c_size_t, C.c_int64, C.c_char_p, C.c_size_t]),
    "rll_close": (C.c_int, [vp]),
    "rll_free": (C.c_int, [vp]),
    "rll_new_allowed_result": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.POINTER(rll_result)]),
    "rll_new_denied_result": (C.c_int, [C.c_int64, C.c_int64, C.c_int64, C.POINTER(rll_result)]),
    "rll_new_fail_open_result": (C.c_int, [C.POINTER(rll_result)]),
    "rll_add_metrics": (C.c_int, [vp]),
    "rll_metrics_expose": (C.c_int, [vp, C.c_char_p, C.c_size_t]),
    "rll_add_logging": (C.c_int, [vp, C.c_size_t]),
    "rll_log_drain": (C.c_int, [vp, C.c_char_p, C.c_size_t, C.POINTER(C.c_uint64)]),
    "rll_new_fail_closed_result": (C.c_int, [C.POINTER(rll_result)]),
    "rl_coalescer_create": (C.c_int, [vp, C.POINTER(rl_coalescer_opts), C.POINTER(vp)]),
    "rl_coalescer_create_with_backend": (C.c_int, [BATCH_FN, vp, C.POINTER(rl_coalescer_opts), C.POINTER(vp)]),
    "rl_coalescer_create_with_backends": (C.c_int, [BATCH_FN, RESET_FN, vp, C.POINTER(rl_coalescer_opts),
                                                    C.POINTER(vp)]),
    "rl_coalescer_create_with_host_backend": (C.c_int, [C.POINTER(rl_coalescer_backend),
                                                        C.POINTER(rl_coalescer_opts), C.POINTER(vp)]),
    "rl_coalescer_reset": (C.c_int, [vp, C.c_uint64, C.c_int64, C.c_uint32]),
    "rl_coalescer_now_ns": (C.c_int64, []),
    "rl_coalescer_submit_deadline": (C.c_int, [vp, C.c_size_t, vp, vp, vp, vp, C.c_int64, C.POINTER(C.c_uint64)]),
    "rl_coalescer_cancel": (C.c_int, [vp, C.c_uint64]),
    "rl_coalescer_decide_deadline": (C.c_int, [vp, C.c_uint64, C.c_int64, C.c_int64, C.c_uint32, C.c_int64,
                                               vp, vp, vp, vp]),
    "rl_coalescer_table_info": (C.c_int, [vp, C.c_int64, C.POINTER(rl_table_info)]),
    "rl_coalescer_gc": (C.c_int, [vp, C.c_int64, C.c_uint64, C.c_uint64, C.POINTER(rl_table_info)]),
    "rl_hash_keys_host": (C.c_int, [C.c_size_t, vp, C.c_uint64, vp, C.c_uint64, vp, C.c_char_p, C.c_size_t, vp]),
    "rl_coalescer_destroy": (C.c_int, [vp]),
    "rl_coalescer_submit": (C.c_int, [vp, C.c_size_t, vp, vp, vp, vp, C.POINTER(C.c_uint64)]),
    "rl_coalescer_wait": (C.c_int, [vp, C.c_uint64, C.c_int64, vp, vp, vp, vp]),
    "rl_coalescer_decide": (C.c_int, [vp, C.c_uint64, C.c_int64, C.c_int64, C.c_uint32, vp, vp, vp, vp]),
    "rl_coalescer_get_stats": (C.c_int, [vp, C.POINTER(rl_coalescer_stats)]),
    "rl_hash_keys_device": (C.c_int, [C.c_size_t, vp, C.c_uint64, vp, C.c_uint64, C.c_char_p, C.c_size_t, vp, vp]),
    "rl_decide_batch_keys_device": (C.c_int, [vp, C.c_size_t, vp, C.c_uint64, vp, C.c_uint64, C.c_char_p,
                                              C.c_size_t] + [vp] * 10),
    "rl_hash_keys": (C.c_int, [C.c_int32, C.c_size_t, vp, C.c_uint64, vp, C.c_uint64, C.c_char_p, C.c_size_t, vp]),
    "rl_router_create": (C.c_int, [C.c_int32, C.c_int32, C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "rl_router_destroy": (C.c_int, [vp]),
    "rl_router_sync": (C.c_int, [vp, vp]),
    "rl_route_owner": (C.c_int, [vp, C.c_size_t, vp, vp, vp]),
    "rl_stream_create_dedicated": (C.c_int, [C.c_int32, C.POINTER(vp)]),
    "rl_stream_destroy": (C.c_int, [vp]),
    "rl_router_capacity": (C.c_uint32, [vp]),
    "rl_route_pack": (C.c_int, [vp, C.c_size_t] + [vp] * 8),
    "rl_route_merge": (C.c_int, [vp] + [vp] * 6),
    "rl_route_unpack": (C.c_int, [vp, C.c_size_t] + [vp] * 7),
    "rl_decide_routed_device": (C.c_int, [vp, C.c_size_t] + [vp] * 6),
    "rl_decide_routed_device_io": (C.c_int, [vp, C.c_size_t] + [vp] * 7),
    "rl_decide_routed_device_ev": (C.c_int, [vp, C.c_size_t] + [vp] * 7),
}
for _name, (_res, _args) in _sig.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def _ptr(a):
    return None if a is None else a.ctypes.data_as(vp)


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{msg} (status {code})")
        self.code = code


def q14_host(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    lib.rl_selftest_q14_host(_ptr(x), _ptr(out), x.size)
    return out


@dataclass
class Decisions:
    decision: np.ndarray
    remaining: np.ndarray
    retry_after_ns: np.ndarray
    reset_at_ns: np.ndarray
    tokens: np.ndarray | None


# rl_opts.flags (include/rl_engine.h)
OPT_PIPELINE = 1


class Engine:
    """rl_engine: the batched decision engine on one GPU."""

    def __init__(self, profile=PROFILE_REDIS7, tb_capacity=1 << 16, win_capacity=1 << 16,
                 max_batch=1 << 20, device=0, flags=0, spill_capacity=0):
        o = rl_opts(device=device, profile=profile, tb_capacity=tb_capacity, win_capacity=win_capacity,
                    max_batch=max_batch, flags=flags, spill_capacity=spill_capacity)
        h = vp()
        rc = lib.rl_engine_create(C.byref(o), C.byref(h))
        if rc != RL_OK:
            raise EngineError(rc, "rl_engine_create failed")
        self.h = h
        self.profile = profile

    def close(self):
        if self.h:
            lib.rl_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        buf = C.create_string_buffer(512)
        lib.rl_last_error(self.h, buf, 512)
        return buf.value.decode()

    def register(self, alg: int, limit: int, window_ns: int) -> int:
        cid = C.c_uint32()
        rc = lib.rl_config_register(self.h, alg, limit, window_ns, C.byref(cid))
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())
        return cid.value

    def decide(self, key, ts, n, cfg, server_ms=None, want_tokens=True, check=True) -> Decisions:
        key = np.ascontiguousarray(key, dtype=np.uint64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = np.ascontiguousarray(n, dtype=np.int64)
        cfg = np.ascontiguousarray(cfg, dtype=np.uint32)
        sms = None if server_ms is None else np.ascontiguousarray(server_ms, dtype=np.int64)
        m = key.size
        out = Decisions(np.empty(m, np.uint8), np.empty(m, np.int64), np.empty(m, np.int64),
                        np.empty(m, np.int64), np.empty(m, np.float64) if want_tokens else None)
        rc = lib.rl_decide_batch(self.h, m, _ptr(key), _ptr(ts), _ptr(n), _ptr(cfg), _ptr(sms),
                                 _ptr(out.decision), _ptr(out.remaining), _ptr(out.retry_after_ns),
                                 _ptr(out.reset_at_ns), _ptr(out.tokens))
        if check and rc != RL_OK:
            raise EngineError(rc, self.last_error())
        out.status = rc
        return out

    def decide_routed(self, m_max, count_p, recv_p, order_p, sms_p, res_p, stream=None, out_stream=None):
        """rl_decide_routed_device(_io) (include/rl_route.h): the merged
        routed batch (its size in device memory at count_p, at most m_max);
        the grouping waits for `stream`, `out_stream` (default: `stream`)
        waits for the results"""
        if out_stream is None:
            rc = lib.rl_decide_routed_device(self.h, m_max, count_p, recv_p, order_p, sms_p, res_p, stream)
        else:
            rc = lib.rl_decide_routed_device_io(self.h, m_max, count_p, recv_p, order_p, sms_p, res_p, stream,
                                                out_stream)
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())

    def decide_routed_ev(self, m_max, count_p, recv_p, order_p, sms_p, res_p, stream, event_p):
        """rl_decide_routed_device_ev: the grouping waits for `stream`; the
        results' completion is recorded into the hipEvent_t at event_p"""
        rc = lib.rl_decide_routed_device_ev(self.h, m_max, count_p, recv_p, order_p, sms_p, res_p, stream, event_p)
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())

    def decide_device(self, m, key_p, ts_p, n_p, cfg_p, sms_p, dec_p, rem_p, retry_p, reset_p, tok_p,
                      stream=None):
        rc = lib.rl_decide_batch_device(self.h, m, key_p, ts_p, n_p, cfg_p, sms_p, dec_p, rem_p,
                                        retry_p, reset_p, tok_p, stream)
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())

    def sync(self) -> int:
        return lib.rl_engine_sync(self.h)

    def reset(self, cfg: int, key: int, ts: int):
        rc = lib.rl_reset(self.h, cfg, key, ts)
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())

    def stats(self) -> rl_stats:
        s = rl_stats()
        lib.rl_engine_stats(self.h, C.byref(s))
        return s

    def debug_stamps(self) -> np.ndarray | None:
        """RL_STAMP_KERNELS=1 diagnostics: [256, 6] realtime (10 ns) stamps per
        batch slot (front start/end, replay start/end, finish start/end)"""
        out = np.zeros(6 * 256, np.uint32)
        if lib.rl_engine_debug_stamps(self.h, _ptr(out), out.size) != 0:
            return None
        return out.reshape(256, 6)

    def debug_words(self, n=88) -> np.ndarray:
        out = np.zeros(n, np.uint32)
        lib.rl_engine_debug_words(self.h, _ptr(out), n)
        return out

    def table_info(self, now_ms: int) -> rl_table_info:
        out = rl_table_info()
        rc = lib.rl_table_info_get(self.h, now_ms, C.byref(out))
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())
        return out

    def table_gc(self, now_ms: int, tb_capacity=0, win_capacity=0, check=True):
        out = rl_table_info()
        rc = lib.rl_table_gc(self.h, now_ms, tb_capacity, win_capacity, C.byref(out))
        if check and rc != RL_OK:
            raise EngineError(rc, self.last_error())
        return rc, out

    def set_timing(self, level):
        """0 off, 1 replay events only, 2 every stage (True == 2), -k replay
        events on every k-th batch only (timed runs: each event pair costs the
        replay stream ~10 us)"""
        lib.rl_engine_set_timing(self.h, 2 if level is True else int(level))

    def stage_times(self):
        ms = np.zeros(5, np.float64)
        nb = C.c_uint64()
        lib.rl_engine_stage_times(self.h, _ptr(ms), 5, C.byref(nb))
        return ms, nb.value

    def q14_device(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty_like(x)
        rc = lib.rl_selftest_q14_device(self.h, _ptr(x), _ptr(out), x.size)
        if rc != RL_OK:
            raise EngineError(rc, self.last_error())
        return out


_DEDICATED_STREAMS = []   # rl_stream_create_dedicated handles (release_dedicated_streams)


def release_dedicated_streams():
    """destroy every Router.dedicated_stream: call once nothing uses them any
    more (pipelines and their tensors dropped); synchronizes the device and
    empties torch's allocator cache first, whose blocks may carry events on
    those streams"""
    import gc

    import torch
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    while _DEDICATED_STREAMS:
        lib.rl_stream_destroy(_DEDICATED_STREAMS.pop())


# rl_route.h
RL_EOVERFLOW = -75
DROPPED = 4


class Router:
    """rl_router (include/rl_route.h): the routing kernels of one rank.  All
    arguments are device pointers (ints) and a hipStream_t; asynchronous.
    `cap`: records per peer bucket (rounded up: self.capacity)."""

    def __init__(self, device, world, max_batch, cap):
        h = vp()
        rc = lib.rl_router_create(device, world, max_batch, cap, C.byref(h))
        if rc != RL_OK:
            raise EngineError(rc, "rl_router_create failed")
        self.h = h
        self.world = world
        self.device = device
        self.capacity = lib.rl_router_capacity(h)

    def _chk(self, rc, what):
        if rc != RL_OK:
            raise EngineError(rc, what)

    def dedicated_stream(self):
        """a torch stream on a hardware queue of its own
        (rl_stream_create_dedicated)"""
        import torch
        h = vp()
        self._chk(lib.rl_stream_create_dedicated(self.device, C.byref(h)), "rl_stream_create_dedicated")
        # kept for the life of the process: torch's allocator and process
        # groups may still hold events on them after the router is closed
        _DEDICATED_STREAMS.append(h)
        return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", self.device))

    def owner(self, m, key, owner, stream):
        self._chk(lib.rl_route_owner(self.h, m, key, owner, stream), "rl_route_owner")

    def pack(self, m, key, ts, n, cfg, send, send_info, slot, stream):
        self._chk(lib.rl_route_pack(self.h, m, key, ts, n, cfg, send, send_info, slot, stream), "rl_route_pack")

    def merge(self, recv, recv_info, order, sms, count, stream):
        self._chk(lib.rl_route_merge(self.h, recv, recv_info, order, sms, count, stream), "rl_route_merge")

    def unpack(self, m, slot, back, dec, rem, retry, reset, stream):
        self._chk(lib.rl_route_unpack(self.h, m, slot, back, dec, rem, retry, reset, stream), "rl_route_unpack")

    def sync(self, stream=None) -> int:
        return lib.rl_router_sync(self.h, stream)

    def close(self):
        if self.h:
            lib.rl_router_destroy(self.h)
            self.h = None


    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --- host mirror of the Go API (include/rl_limiter.h) ------------------------

def pack_keys(keys) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate raw keys (bytes / str) into (bytes u8, offsets u64[m+1])."""
    bs = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    return np.frombuffer(b"".join(bs), dtype=np.uint8).copy(), off


def hash_keys(keys_or_packed, seed: int, prefix: bytes | str = b"", device=0, check=True) -> np.ndarray:
    """On-GPU FormatKey + XXH64 (include/rl_keyhash.h): key ids for rl_decide_batch."""
    data, off = keys_or_packed if isinstance(keys_or_packed, tuple) else pack_keys(keys_or_packed)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    pre = prefix.encode() if isinstance(prefix, str) else bytes(prefix)
    m = len(off) - 1
    out = np.zeros(max(m, 0), dtype=np.uint64)
    rc = lib.rl_hash_keys(device, m, _ptr(data), data.size, _ptr(off), seed, pre, len(pre), _ptr(out))
    if check and rc != RL_OK:
        raise EngineError(rc, "rl_hash_keys failed")
    return out if check else (rc, out)


def hash_keys_host(keys_or_packed, seed: int, prefix: bytes | str = b"", cfg=None) -> np.ndarray:
    """rl_hash_keys_host: the raw-key ids on the CPU (cfg: per-key config ids
    mixed into the seed, as rl_decide_batch_keys_device does)."""
    data, off = keys_or_packed if isinstance(keys_or_packed, tuple) else pack_keys(keys_or_packed)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    pre = prefix.encode() if isinstance(prefix, str) else bytes(prefix)
    m = len(off) - 1
    c = None if cfg is None else np.ascontiguousarray(cfg, dtype=np.uint32)
    out = np.zeros(max(m, 0), dtype=np.uint64)
    rc = lib.rl_hash_keys_host(m, _ptr(data), data.size, _ptr(off), seed, _ptr(c), pre, len(pre), _ptr(out))
    if rc != RL_OK:
        raise EngineError(rc, "rl_hash_keys_host failed")
    return out


def config_validate(algorithm, limit, window_ns):
    """Config.Validate(); algorithm None == nil *Config.  Returns '' or the message."""
    buf = C.create_string_buffer(512)
    a = None if algorithm is None else algorithm.encode()
    rc = lib.rll_config_validate(a, limit, window_ns, buf, 512)
    return "" if rc == RLL_OK else buf.value.decode()


def format_key(prefix, key):
    buf = C.create_string_buffer(4096)
    lib.rll_format_key(None if prefix is None else prefix.encode(), key.encode(), buf, 4096)
    return buf.value.decode()


def duration_string(d):
    buf = C.create_string_buffer(64)
    lib.rll_duration_string(d, buf, 64)
    return buf.raw.split(b"\0", 1)[0].decode("utf-8")


@dataclass
class Result:
    Allowed: bool
    Limit: int
    Remaining: int
    RetryAfter: int
    ResetAt: int


class GoError(Exception):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code
        self.msg = msg


class LimiterEngine:
    """rll_engine: one GPU engine + key interner shared by limiters."""

    def __init__(self, profile=PROFILE_REDIS7, tb_capacity=1 << 16, win_capacity=1 << 16,
                 max_batch=1 << 16, device=0):
        o = rl_opts(device=device, profile=profile, tb_capacity=tb_capacity, win_capacity=win_capacity,
                    max_batch=max_batch)
        h = vp()
        buf = C.create_string_buffer(512)
        rc = lib.rll_engine_new(C.byref(o), C.byref(h), buf, 512)
        if rc != RLL_OK:
            raise GoError(rc, buf.value.decode())
        self.h = h

    def set_server_ms(self, ms):
        lib.rll_engine_set_server_ms(self.h, SMS_DEFAULT if ms is None else ms)

    def keys(self, server_ms):
        """Redis KEYS: the live keys' formatted names, sorted (rll_keys)"""
        n = lib.rll_keys(self.h, server_ms, None, 0)
        if n < 0:
            raise GoError(-n, "rll_keys failed")
        buf = C.create_string_buffer(n + 1)
        lib.rll_keys(self.h, server_ms, buf, n + 1)
        return buf.value.decode().splitlines()

    def close(self):
        if self.h:
            lib.rll_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RateLimiter:
    """Mirror of the reference RateLimiter (interface.go:76-145)."""

    def __init__(self, h):
        self.h = h

    def allow(self, key, now_ns=NOW_WALL, cancelled=False):
        return self.allow_n(key, 1, now_ns, cancelled)

    def allow_n(self, key, n, now_ns=NOW_WALL, cancelled=False):
        """Returns (Result | None, error message | None, code)."""
        r = rll_result()
        buf = C.create_string_buffer(512)
        kb = key.encode()
        rc = lib.rll_allow_n(self.h, kb, len(kb), n, now_ns, 1 if cancelled else 0, C.byref(r), buf, 512)
        if rc == RLL_OK:
            return Result(bool(r.allowed), r.limit, r.remaining, r.retry_after_ns, r.reset_at_ns), None, rc
        return None, buf.value.decode(), rc

    def batch_allow(self, keys, n, now_ns=None):
        m = len(keys)
        kbs = [k.encode() for k in keys]
        arr = (C.c_char_p * m)(*kbs)
        lens = np.array([len(k) for k in kbs], np.uint64)
        nn = np.ascontiguousarray(n, np.int64)
        now = None if now_ns is None else np.ascontiguousarray(now_ns, np.int64)
        out = (rll_result * m)()
        codes = np.empty(m, np.int32)
        lib.rll_allow_batch(self.h, m, C.cast(arr, vp), _ptr(lens), _ptr(nn), _ptr(now), C.cast(out, vp),
                            _ptr(codes))
        res = [Result(bool(o.allowed), o.limit, o.remaining, o.retry_after_ns, o.reset_at_ns) for o in out]
        return res, codes

    def add_metrics(self):
        """MetricsDecorator (ADR-003) around this limiter, in place."""
        if lib.rll_add_metrics(self.h) != RLL_OK:
            raise GoError(RLL_ERR_ARG, "rll_add_metrics failed")

    def metrics_text(self) -> str:
        n = lib.rll_metrics_expose(self.h, None, 0)
        if n < 0:
            raise GoError(RLL_ERR_ARG, "no metrics decorator")
        buf = C.create_string_buffer(n + 1)
        lib.rll_metrics_expose(self.h, buf, n + 1)
        return buf.value.decode()

    def add_logging(self, capacity=4096):
        """LoggingDecorator (ADR-003): records queue in the library until drained."""
        if lib.rll_add_logging(self.h, capacity) != RLL_OK:
            raise GoError(RLL_ERR_ARG, "rll_add_logging failed")

    def drain_logs(self):
        """-> ([(level, msg, fields)], dropped)"""
        out = []
        dropped = C.c_uint64()
        while True:
            buf = C.create_string_buffer(1 << 16)
            n = lib.rll_log_drain(self.h, buf, 1 << 16, C.byref(dropped))
            if n < 0:
                raise GoError(RLL_ERR_ARG, "no logging decorator")
            for line in buf.value.decode().splitlines():
                lv, msg, fields = line.split("\t", 2)
                out.append((int(lv), msg, fields))
            if n == 0:
                return out, dropped.value

    def reset(self, key, now_ns=NOW_WALL):
        buf = C.create_string_buffer(512)
        kb = key.encode()
        rc = lib.rll_reset(self.h, kb, len(kb), now_ns, buf, 512)
        return None if rc == RLL_OK else buf.value.decode()

    def close(self):
        lib.rll_close(self.h)

    def __del__(self):
        try:
            lib.rll_free(self.h)
        except Exception:
            pass


def new_limiter(engine: LimiterEngine | None, algorithm, limit, window_ns, prefix="", fail_open=False,
                config_nil=False):
    """NewTokenBucket/NewSlidingWindow/NewFixedWindow by name; raises GoError like the constructor."""
    h = vp()
    buf = C.create_string_buffer(512)
    rc = lib.rll_new(None if engine is None else engine.h, algorithm.encode(), limit, window_ns,
                     prefix.encode(), 1 if fail_open else 0, 1 if config_nil else 0, C.byref(h), buf, 512)
    if rc != RLL_OK:
        raise GoError(rc, buf.value.decode())
    return RateLimiter(h)


RL_EAGAIN, RL_ECLOSED, RL_EDEADLINE, RL_ECANCELED = -11, -32, -62, -125


def now_ns() -> int:
    """the coalescer's deadline clock (rl_coalescer_now_ns: CLOCK_MONOTONIC)"""
    return lib.rl_coalescer_now_ns()


class Coalescer:
    """rl_coalescer (include/rl_coalescer.h): concurrent submissions gathered
    into engine batches.  `engine` is an Engine (GPU) or, for the CPU tests of
    the batching logic, a Python function with rl_decide_batch's host-array
    signature (the test seam rl_coalescer_create_with_host_backend; `reset`,
    `table_info`, `gc`: the other backend functions, optional).

    gc_interval_ns > 0 turns on the automatic table GC (rl_coalescer_opts)."""

    def __init__(self, engine, max_batch=65536, max_in_flight=3, linger_ns=0, queue_cap=0, reset=None,
                 table_info=None, gc=None, gc_interval_ns=0, gc_high_pct=0, gc_margin_ms=0,
                 gc_max_tb_capacity=0, gc_max_win_capacity=0):
        o = rl_coalescer_opts(max_batch=max_batch, max_in_flight=max_in_flight, gc_high_pct=gc_high_pct,
                              linger_ns=linger_ns, queue_cap=queue_cap, gc_interval_ns=gc_interval_ns,
                              gc_margin_ms=gc_margin_ms, gc_max_tb_capacity=gc_max_tb_capacity,
                              gc_max_win_capacity=gc_max_win_capacity)
        h = vp()
        if isinstance(engine, Engine):
            rc = lib.rl_coalescer_create(engine.h, C.byref(o), C.byref(h))
            self._be = None
        else:
            # the callbacks live as long as the coalescer
            self._be = rl_coalescer_backend(
                batch=BATCH_FN(engine), reset=RESET_FN(reset) if reset else C.cast(None, RESET_FN),
                table_info=INFO_FN(table_info) if table_info else C.cast(None, INFO_FN),
                gc=GC_FN(gc) if gc else C.cast(None, GC_FN), user=None)
            rc = lib.rl_coalescer_create_with_host_backend(C.byref(self._be), C.byref(o), C.byref(h))
        if rc != RL_OK:
            raise EngineError(rc, "rl_coalescer_create failed")
        self.h = h

    def submit(self, key, ts, n, cfg, deadline_ns=0) -> int:
        key = np.ascontiguousarray(key, dtype=np.uint64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        n = np.ascontiguousarray(n, dtype=np.int64)
        cfg = np.ascontiguousarray(cfg, dtype=np.uint32)
        t = C.c_uint64()
        rc = lib.rl_coalescer_submit_deadline(self.h, key.size, _ptr(key), _ptr(ts), _ptr(n), _ptr(cfg),
                                              deadline_ns, C.byref(t))
        if rc != RL_OK:
            raise EngineError(rc, "rl_coalescer_submit failed")
        return t.value

    def wait(self, ticket: int, m: int, timeout_ns=-1, out=None):
        if out is None:
            out = (np.empty(m, np.uint8), np.empty(m, np.int64), np.empty(m, np.int64), np.empty(m, np.int64))
        rc = lib.rl_coalescer_wait(self.h, ticket, timeout_ns, *[_ptr(x) for x in out])
        return rc, out

    def cancel(self, ticket: int) -> int:
        return lib.rl_coalescer_cancel(self.h, ticket)

    def decide(self, key, ts, n, cfg, deadline_ns=0):
        d, rem, retry, reset = C.c_uint8(), C.c_int64(), C.c_int64(), C.c_int64()
        rc = lib.rl_coalescer_decide_deadline(self.h, key, ts, n, cfg, deadline_ns, C.byref(d), C.byref(rem),
                                              C.byref(retry), C.byref(reset))
        return rc, (d.value, rem.value, retry.value, reset.value)

    def reset(self, key, ts, cfg) -> int:
        return lib.rl_coalescer_reset(self.h, key, ts, cfg)

    def table_info(self, now_ms):
        out = rl_table_info()
        rc = lib.rl_coalescer_table_info(self.h, now_ms, C.byref(out))
        return rc, out

    def gc(self, now_ms, tb_capacity=0, win_capacity=0):
        out = rl_table_info()
        rc = lib.rl_coalescer_gc(self.h, now_ms, tb_capacity, win_capacity, C.byref(out))
        return rc, out

    def stats(self) -> rl_coalescer_stats:
        st = rl_coalescer_stats()
        lib.rl_coalescer_get_stats(self.h, C.byref(st))
        return st

    def close(self):
        if self.h:
            lib.rl_coalescer_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --- the native gRPC front end (include/rl_grpc.h, lib/librl_grpc.so) ----------
GRPC_LIB_PATH = os.environ.get("RL_GRPC_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "librl_grpc.so")
_grpc_lib = None


def grpc_lib():
    global _grpc_lib
    if _grpc_lib is None:
        if not os.path.exists(GRPC_LIB_PATH):
            raise ImportError(f"native gRPC server not built: {GRPC_LIB_PATH} (make -C distributed-rate-limiter_amd)")
        _grpc_lib = C.CDLL(GRPC_LIB_PATH)
        _grpc_lib.rl_grpc_server_start.argtypes = [vp, C.c_void_p, C.c_size_t, C.c_void_p, C.POINTER(vp)]
        _grpc_lib.rl_grpc_server_shutdown.argtypes = [vp, C.c_int64]
        _grpc_lib.rl_grpc_server_destroy.argtypes = [vp]
        _grpc_lib.rl_grpc_server_port.argtypes = [vp]
        _grpc_lib.rl_grpc_server_get_stats.argtypes = [vp, C.c_void_p]
    return _grpc_lib


class rl_grpc_limiter(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("cfg_id", C.c_uint32), ("name", C.c_char_p), ("algorithm", C.c_int32),
                ("fail_open", C.c_int32), ("limit", C.c_int64), ("window_ns", C.c_int64), ("prefix", C.c_char_p)]


class rl_grpc_opts(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("io_threads", C.c_uint32), ("host", C.c_char_p), ("port", C.c_int32),
                ("isolate", C.c_int32), ("clock_start_ns", C.c_int64), ("clock_step_ns", C.c_int64)]


class rl_grpc_stats(_Sized):
    _fields_ = [("struct_size", C.c_uint32), ("pad_", C.c_uint32), ("connections", C.c_uint64), ("rpcs", C.c_uint64),
                ("decisions", C.c_uint64), ("errors", C.c_uint64), ("cancelled", C.c_uint64)]


class GrpcServer:
    """rl_grpc_server (include/rl_grpc.h): the rate limiter service served by
    native event loops over `coalescer`.  limiters: (name, cfg_id, algorithm,
    limit, window_ns, prefix, fail_open) tuples, already registered.  With
    clock_step_ns != 0 the server's time.Now() is the test clock
    clock_start_ns + k * clock_step_ns on its k-th read."""

    def __init__(self, coalescer, limiters, host="127.0.0.1", port=0, io_threads=4, isolate=False,
                 clock_start_ns=0, clock_step_ns=0):
        L = grpc_lib()
        self._lims = (rl_grpc_limiter * max(1, len(limiters)))()
        for i, (name, cfg, alg, limit, window, prefix, fail_open) in enumerate(limiters):
            self._lims[i] = rl_grpc_limiter(cfg_id=cfg, name=name.encode(), algorithm=alg, fail_open=int(fail_open),
                                            limit=limit, window_ns=window,
                                            prefix=prefix if isinstance(prefix, bytes) else prefix.encode())
        self._opts = rl_grpc_opts(io_threads=io_threads, host=host.encode(), port=port, isolate=int(isolate),
                                  clock_start_ns=clock_start_ns, clock_step_ns=clock_step_ns)
        self.co = coalescer
        h = vp()
        rc = L.rl_grpc_server_start(coalescer.h, C.cast(self._lims, C.c_void_p), len(limiters),
                                    C.cast(C.pointer(self._opts), C.c_void_p), C.byref(h))
        if rc != RL_OK:
            raise EngineError(rc, "rl_grpc_server_start failed")
        self.h = h
        self.port = L.rl_grpc_server_port(h)

    def stats(self) -> rl_grpc_stats:
        st = rl_grpc_stats()
        grpc_lib().rl_grpc_server_get_stats(self.h, C.byref(st))
        return st

    def shutdown(self, grace_s=5.0):
        if self.h:
            grpc_lib().rl_grpc_server_shutdown(self.h, int(grace_s * 1e9))

    def close(self):
        if self.h:
            grpc_lib().rl_grpc_server_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
