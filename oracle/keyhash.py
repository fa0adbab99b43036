"""CPU checker for the on-GPU key formatting + hashing -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/ (never by the product path, which is
k_key_hash in distributed-rate-limiter_amd/csrc/rl_keyhash.hip).

  format_key(prefix, key)   Config.FormatKey, config.go:81-87:
                            prefix == "" -> key, else prefix + ":" + key
  xxh64(data, seed)         pure-Python restatement of the published XXH64
                            algorithm (xxHash 0.8 specification)
  key_id(prefix, key, seed) what include/rl_keyhash.h promises per request

Pinned: xxh64 is checked against the published known answer XXH64("", 0) =
0xEF46DB3751D8E999 and, where the `xxhash` package (python-xxhash 3.8.1,
libxxhash 0.8.2, in this image) is importable, against it on every length
class (tests/test_keyhash.py).  The reference itself keys Redis by the
formatted string; parity of the decisions made through hashed ids against
string identity is checked in tests/test_keyhash.py (GPU).
"""
from __future__ import annotations

M64 = (1 << 64) - 1
P1 = 0x9E3779B185EBCA87
P2 = 0xC2B2AE3D27D4EB4F
P3 = 0x165667B19E3779F9
P4 = 0x85EBCA77C2B2AE63
P5 = 0x27D4EB2F165667C5
KEY_RESERVED = M64


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (64 - r))) & M64


def _round(acc: int, v: int) -> int:
    return (_rotl((acc + v * P2) & M64, 31) * P1) & M64


def _merge(acc: int, v: int) -> int:
    return ((acc ^ _round(0, v)) * P1 + P4) & M64


def xxh64(data: bytes, seed: int = 0) -> int:
    n, p = len(data), 0
    seed &= M64
    if n >= 32:
        v = [(seed + P1 + P2) & M64, (seed + P2) & M64, seed, (seed - P1) & M64]
        while p + 32 <= n:
            for i in range(4):
                v[i] = _round(v[i], int.from_bytes(data[p + 8 * i:p + 8 * i + 8], "little"))
            p += 32
        h = (_rotl(v[0], 1) + _rotl(v[1], 7) + _rotl(v[2], 12) + _rotl(v[3], 18)) & M64
        for x in v:
            h = _merge(h, x)
    else:
        h = (seed + P5) & M64
    h = (h + n) & M64
    while p + 8 <= n:
        h = (_rotl(h ^ _round(0, int.from_bytes(data[p:p + 8], "little")), 27) * P1 + P4) & M64
        p += 8
    if p + 4 <= n:
        h = (_rotl(h ^ ((int.from_bytes(data[p:p + 4], "little") * P1) & M64), 23) * P2 + P3) & M64
        p += 4
    while p < n:
        h = (_rotl(h ^ ((data[p] * P5) & M64), 11) * P1) & M64
        p += 1
    h ^= h >> 33
    h = (h * P2) & M64
    h ^= h >> 29
    h = (h * P3) & M64
    h ^= h >> 32
    return h


def format_key(prefix: bytes, key: bytes) -> bytes:
    return key if not prefix else prefix + b":" + key


def key_id(prefix: bytes, key: bytes, seed: int) -> int:
    h = xxh64(format_key(prefix, key), seed)
    return KEY_RESERVED - 1 if h == KEY_RESERVED else h


def cfg_seed(seed: int, cfg_id: int) -> int:
    """rl_cfg_seed (include/rl_keyhash.h): the seed the engine's raw-key entry
    point hashes a request of config `cfg_id` with."""
    return (seed ^ ((cfg_id * 0x9E3779B97F4A7C15) & M64)) & M64


def key_ids_fast(prefix: bytes, keys, seed: int):
    """Same as key_id over a list, through the xxhash package when importable
    (large GPU parity cases); falls back to the restatement."""
    try:
        import xxhash
        f = lambda b: xxhash.xxh64_intdigest(b, seed)  # noqa: E731
    except ImportError:  # pragma: no cover
        f = lambda b: xxh64(b, seed)  # noqa: E731
    out = []
    for k in keys:
        h = f(format_key(prefix, k))
        out.append(KEY_RESERVED - 1 if h == KEY_RESERVED else h)
    return out
