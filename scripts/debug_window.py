"""Debug helper: a window-algorithm parity trace on the GPU; prints the first
mismatching key's request history (all batches) for both sides (GPU box only).
usage: debug_window.py [kind] [profile] [ff] [skewed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "distributed-rate-limiter_amd", "python")]
import oracle  # noqa: E402
import rl_amd  # noqa: E402
from tracegen import CONFIG_SETS, random_trace, skewed_trace  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "sw"
profile = int(sys.argv[2]) if len(sys.argv) > 2 else 0
ff = len(sys.argv) > 3 and sys.argv[3] == "1"
skewed = len(sys.argv) > 4 and sys.argv[4] == "1"
configs = CONFIG_SETS[kind]
if skewed:
    tr = skewed_trace(600 + profile * 7 + 40, 80_000, 40, configs, big_n=True)
    sizes = [3000, 500, 20_000, 26_500, 30_000]
else:
    seed = {"tb": 1, "sw": 2, "fw": 3, "mixed": 4}[kind] * 10 + profile * 2 + int(ff)
    tr = random_trace(seed, 60_000, 500, configs, fastforward=ff, big_n=True)
    sizes = [1, 7, 1000, 9000, 20000, 29992]
eng = rl_amd.Engine(profile=profile, tb_capacity=1 << 14, win_capacity=1 << 14, max_batch=1 << 20)
sim = oracle.OracleSim(profile)
for a, L, W in configs:
    eng.register(a, L, W)
    sim.add_config(a, L, W)
key, ts, n, cfg, sms = tr
gd, rd, grem, rrem = [], [], [], []
o = 0
first = None
for bi, s in enumerate(sizes):
    sl = slice(o, o + s)
    o += s
    args = (key[sl], ts[sl], n[sl], cfg[sl], None if sms is None else sms[sl])
    res = eng.decide(*args, check=False)
    ref = sim.decide(*args)
    gd.append(res.decision); rd.append(ref[0]); grem.append(res.remaining); rrem.append(ref[1])
    bad = np.nonzero((res.decision != ref[0]) | ((res.remaining != ref[1]) & (ref[0] < 2)))[0]
    print(f"batch {bi}: status {res.status} mismatches {bad.size}")
    if bad.size and first is None:
        first = sl.start + bad[0]
gd, rd, grem, rrem = map(np.concatenate, (gd, rd, grem, rrem))
if first is not None:
    k = key[first]
    c = configs[cfg[first]]
    print(f"first mismatch i={first} key={k} cfg={c}")
    idx = np.nonzero(key[:first + 1] == k)[0]
    W = c[2]
    for i in idx[-40:]:
        t = int(ts[i])
        r = (t + 62135596800 * 10**9) % W
        ws = (t - r) // 10**9
        sm = (t // 10**6) if sms is None else int(sms[i])
        print(f"  i={i} t={t} ws={ws} sms={sm} n={n[i]} gpu={gd[i]}/{grem[i]} ref={rd[i]}/{rrem[i]}"
              f"{'  <--' if gd[i] != rd[i] or grem[i] != rrem[i] else ''}")
