"""Debug helper (GPU box): run one randomized parity trace batch by batch with
progress output, so a hang or a mismatch names its batch."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "distributed-rate-limiter_amd", "python")]
import oracle  # noqa: E402
import rl_amd  # noqa: E402
from test_gpu_parity import split  # noqa: E402
from tracegen import CONFIG_SETS, random_trace  # noqa: E402

kind, profile, ff = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "1"
configs = CONFIG_SETS[kind]
seed = {"tb": 1, "sw": 2, "fw": 3, "mixed": 4}[kind] * 10 + profile * 2 + int(ff)
tr = random_trace(seed, 60_000, 500, configs, fastforward=ff, big_n=True)
eng = rl_amd.Engine(profile=profile, tb_capacity=1 << 20, win_capacity=1 << 20, max_batch=1 << 20)
sim = oracle.OracleSim(profile)
for a, L, W in configs:
    eng.register(a, L, W)
    sim.add_config(a, L, W)
for i, (key, ts, n, cfg, sms) in enumerate(split(tr, [1, 7, 1000, 9000, 20000, 29992])):
    print(f"batch {i} m={key.size} ...", flush=True)
    t = time.time()
    res = eng.decide(key, ts, n, cfg, sms, check=False)
    dec, rem, retry, reset, tok = sim.decide(key, ts, n, cfg, sms)
    bad = np.nonzero((res.decision != dec) | (res.tokens.view(np.uint64) != tok.view(np.uint64)) & (dec <= 1))[0]
    print(f"  status {res.status} {eng.last_error()!r} mismatches {bad.size} ({time.time() - t:.2f} s)", flush=True)
