"""Latency of one small batch through the host API (copies included), with the
single-workgroup path (k_small) on and off; uniform keys and one hot key."""
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import rl_amd  # noqa: E402

NS = 10 ** 9
T0 = 1_760_000_000 * NS
for small in ("4096", "0"):
    os.environ["RL_SMALL_MAX"] = small
    eng = rl_amd.Engine(tb_capacity=1 << 21, win_capacity=1 << 10, max_batch=1 << 16)
    eng.register(1, 20, 12 * NS)
    rng = np.random.default_rng(1)
    t = T0
    for m in (1, 16, 256, 1024, 4096):
        for hot in (False, True):
            lat = []
            for r in range(30):
                key = np.zeros(m, np.uint64) if hot else rng.integers(0, 1 << 20, m).astype(np.uint64)
                ts = t + np.arange(m, dtype=np.int64) * 1000
                t += m * 1000 + 1000
                t0 = time.perf_counter()
                eng.decide(key, ts, np.ones(m, np.int64), np.zeros(m, np.uint32), want_tokens=False)
                lat.append(time.perf_counter() - t0)
            lat = np.array(lat[5:]) * 1e6
            print(f"small_max={small:>4} m={m:5d} hot={hot!s:5} median {np.median(lat):8.1f} us  max {lat.max():8.1f} us")
    eng.close()
