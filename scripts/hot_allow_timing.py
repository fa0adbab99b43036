"""One hot token-bucket key at 3.8M requests/s (the top key of configs[4] at
1e7 QPS), batches of a fixed size through the host API: per-batch time, to
find where the coalescer's periodic stalls (one per refilled token) come from."""
import os
import sys
import time

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import rl_amd  # noqa: E402

NS = 10 ** 9
T0 = 1_760_000_000 * NS
# HOT_GAP_NS: mean gap of the hot key (263 ns = 3.8M req/s; 2630 = the top key at 1e6 QPS)
# HOT_BATCHES: "size:total,..." batch sizes and request counts
GAP = float(os.environ.get("HOT_GAP_NS", "263"))
PLAN = [tuple(int(float(v)) for v in x.split(":")) for x in
        os.environ.get("HOT_BATCHES", "300:3e6,30000:3e6,300000:3e6").split(",")]
for bs, total in PLAN:
    eng = rl_amd.Engine(tb_capacity=1 << 12, win_capacity=1 << 10, max_batch=1 << 19)
    eng.register(1, 20, 12 * NS)
    rng = np.random.default_rng(1)
    t = T0
    times = []
    for b in range(total // bs):
        gaps = np.rint(rng.exponential(GAP, bs)).astype(np.int64)
        ts = t + np.cumsum(gaps)
        t = int(ts[-1])
        t0 = time.perf_counter()
        r = eng.decide(np.zeros(bs, np.uint64), ts, np.ones(bs, np.int64), np.zeros(bs, np.uint32), want_tokens=False)
        times.append((time.perf_counter() - t0, int((r.decision == 1).sum())))
    dt = np.array([x[0] for x in times]) * 1e3
    allows = np.array([x[1] for x in times])
    slow = np.argsort(dt)[-5:][::-1]
    print(f"batch {bs:6d}: median {np.median(dt):7.3f} ms  max {dt.max():7.3f} ms  "
          f"total {dt.sum():8.1f} ms for {total} requests; slowest {[(int(i), round(float(dt[i]), 2), int(allows[i])) for i in slow]}; "
          f"batches with allows: median {np.median(dt[allows > 0]) if (allows > 0).any() else 0:.3f} ms")
    eng.close()
