#!/usr/bin/env python3
"""k_key_hash roofline (include/rl_keyhash.h): raw keys -> FormatKey -> XXH64 ids.

Algorithmic bytes per launch = key bytes + 8 (m + 1) offsets + 8 m ids.  Time
per launch from HIP events on the launch stream (torch's current stream, which
the kernel is enqueued on).  Prints one JSON line.
  python scripts/bench_keyhash.py [--keys 16000000] [--min-len 8] [--max-len 40] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch  # before the engine library (see tests/conftest.py)
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))
import rl_amd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=int, default=16_000_000)
ap.add_argument("--min-len", type=int, default=8)
ap.add_argument("--max-len", type=int, default=40)
ap.add_argument("--prefix", default="ratelimit")
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()

rng = np.random.default_rng(1)
lens = rng.integers(a.min_len, a.max_len + 1, a.keys).astype(np.uint64)
off = np.zeros(a.keys + 1, np.uint64)
off[1:] = np.cumsum(lens)
nbytes = int(off[-1])
dev = torch.device("cuda", 0)
data = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev)
d_off = torch.from_numpy(off.view(np.int64)).to(dev)
ids = torch.empty(a.keys, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream().cuda_stream
pre = a.prefix.encode()


def launch():
    rc = rl_amd.lib.rl_hash_keys_device(a.keys, data.data_ptr(), nbytes, d_off.data_ptr(), 1, pre, len(pre),
                                        ids.data_ptr(), st)
    assert rc == 0, rc


for _ in range(3):
    launch()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    launch()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
alg_bytes = nbytes + 8 * (a.keys + 1) + 8 * a.keys
gbs = alg_bytes / (ms * 1e-3) / 1e9
# spot check against the oracle restatement (test infrastructure) on a sample
sys.path.insert(0, ROOT)
from oracle import keyhash as kh  # noqa: E402
host = data[: int(off[2000])].cpu().numpy()
got = ids[:2000].cpu().numpy().view(np.uint64)
ok = all(int(got[i]) == kh.key_id(pre, host[int(off[i]):int(off[i + 1])].tobytes(), 1) for i in range(2000))
print(json.dumps({"kernel": "k_key_hash", "keys": a.keys, "key_len": [a.min_len, a.max_len], "prefix": a.prefix,
                  "ms_per_launch": ms, "keys_per_s": a.keys / (ms * 1e-3),
                  "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                               "algorithmic_bytes_per_launch": alg_bytes},
                  "spot_check_2000_vs_oracle": ok}))
