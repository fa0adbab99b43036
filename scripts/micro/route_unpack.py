"""Isolated timing of rl_route_unpack (the routed step's gather of result
records into caller order) on 1M requests, three slot patterns: identity
(world 1), eight interleaved increasing streams (a hash split over 8 owners:
each owner's results come back in its requests' order) and a random
permutation; a device-to-device copy of the same bytes calibrates."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "distributed-rate-limiter_amd", "python"))
import rl_amd  # noqa: E402

M = 1 << 20
dev = torch.device("cuda", 0)
r = rl_amd.Router(0, 1, M, M)
back = torch.randint(0, 1 << 40, (M, 4), dtype=torch.int64, device=dev)
outs = [torch.empty(M, dtype=torch.uint8, device=dev)] + [torch.empty(M, dtype=torch.int64, device=dev) for _ in range(3)]
rng = np.random.default_rng(1)
own = rng.integers(0, 8, M)
pos = np.zeros(M, np.int64)
base = np.zeros(8, np.int64)
for o in range(8):
    idx = np.nonzero(own == o)[0]
    pos[idx] = o * (M // 8 + 65536) // 1 % M + np.arange(idx.size)
pats = {"identity": np.arange(M), "8 streams": np.minimum(pos, M - 1), "random": rng.permutation(M)}
s = torch.cuda.current_stream()
for name, sl in pats.items():
    slot = torch.from_numpy(sl.astype(np.uint32).view(np.int32)).to(dev)
    args = [slot.data_ptr(), back.data_ptr()] + [o.data_ptr() for o in outs]
    for _ in range(3):
        r.unpack(M, *args, s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        r.unpack(M, *args, s.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"unpack {name:10s} {us:7.1f} us  ({(4 + 32 + 25) * M / us / 1e3:.0f} GB/s of 61 B/request)")
a = torch.empty(61 * M, dtype=torch.uint8, device=dev)
b = torch.empty_like(a)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
b.copy_(a)
e0.record()
for _ in range(20):
    b.copy_(a)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
print(f"copy 61 MB      {us:7.1f} us  ({2 * 61 * M / us / 1e3:.0f} GB/s read+write)")
