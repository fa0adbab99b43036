#!/usr/bin/env python3
"""Diagnostic: does the probe's table access order matter?  Runs the mixed
workload (configs[3], 1B keys, tables of 2^26 entries each) through the
engine with per-stage timing, twice: batches as generated (arrival order:
random table lines) and with each batch's keys reordered by home slot (the
table line the probe reads first), timestamps kept in place.  The second is
not the reference's semantics (it moves requests in time); it only measures
the stage times of a home-ordered probe.  A third order ("xcd") puts each
key where a block of the XCD that owns its table eighth probes it (blocks
are dealt round-robin over the 8 XCDs), to measure per-XCD slicing of the
table instead of a full sort.  Prints one JSON line per order."""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))


def mix64(x):
    x = x.copy()
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xbf58476d1ce4e5b9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94d049bb133111eb)
        x ^= x >> np.uint64(31)
    return x


def main():
    import torch

    import rl_amd
    import traces
    nb, m = 24, 1_000_000
    cap = 1 << 26
    gen = traces.MixedTenants(batch=m)
    batches = [gen.next_batch() for _ in range(nb)]
    dev = torch.device("cuda:0")
    def xcd_order(key, cfg):
        # positions i with (i // 256) % 8 == s get keys whose home slot lies in
        # eighth s of its table: k_probe's block b (256 requests per grid step)
        # then touches one eighth of each table, and blocks b, b + 8, ... share
        # an XCD (round-robin placement), so each XCD touches one eighth
        home = mix64(key) & np.uint64(cap - 1)
        sl = (home >> np.uint64(23)).astype(np.int64)          # 2^26 / 8 = 2^23
        want = (np.arange(key.size) // 256) % 8
        o = np.empty(key.size, np.int64)
        pools = [list(np.nonzero(sl == x)[0]) for x in range(8)]
        ptr = [0] * 8
        rest = []
        pos_by = [np.nonzero(want == x)[0] for x in range(8)]
        for x in range(8):
            k = min(len(pools[x]), len(pos_by[x]))
            o[pos_by[x][:k]] = pools[x][:k]
            rest += list(pools[x][k:])
            ptr[x] = k
        free = np.concatenate([pos_by[x][ptr[x]:] for x in range(8)])
        o[np.sort(free)] = np.array(rest, np.int64)
        return o

    for order in ("arrival", "home", "xcd"):
        eng = rl_amd.Engine(profile=rl_amd.PROFILE_REDIS7, tb_capacity=cap, win_capacity=cap, max_batch=m,
                            device=0, flags=rl_amd.OPT_PIPELINE)
        for a, L, W in gen.configs:
            eng.register(a, L, W)
        algs = np.array([a for a, _, _ in gen.configs])
        dbs = []
        for key, ts, n, cfg in batches:
            if order == "xcd":
                o = xcd_order(key, cfg)
                key, cfg, n = key[o], cfg[o], n[o]
            if order == "home":
                table = (algs[cfg] != 1).astype(np.uint64)     # 1: token bucket table, else window table
                home = (table << np.uint64(40)) | (mix64(key) & np.uint64(cap - 1))
                o = np.argsort(home, kind="stable")
                key, cfg, n = key[o], cfg[o], n[o]
            dbs.append(tuple(torch.from_numpy(np.ascontiguousarray(x).view(v)).to(dev)
                             for x, v in ((key, np.int64), (ts, np.int64), (n, np.int64), (cfg, np.int32))))
        outs = [torch.empty(m, dtype=torch.uint8, device=dev)] + \
               [torch.empty(m, dtype=torch.int64, device=dev) for _ in range(3)] + \
               [torch.empty(m, dtype=torch.float64, device=dev)]
        s = torch.cuda.Stream(dev)
        eng.set_timing(2)
        for b, (k, t, n, c) in enumerate(dbs):
            eng.decide_device(m, k.data_ptr(), t.data_ptr(), n.data_ptr(), c.data_ptr(), None,
                              *[o.data_ptr() for o in outs], s.cuda_stream)
            if b == 3:
                eng.sync()
                eng.stage_times()   # drop the warm-up batches
        eng.sync()
        ms, nbat = eng.stage_times()
        print(json.dumps({"order": order, "batches": int(nbat),
                          "stages_us_per_batch": dict(zip(["probe", "sort", "segments", "replay", "finish"],
                                                          [round(x / max(nbat, 1) * 1e3, 1) for x in ms]))}),
              flush=True)
        eng.close()


if __name__ == "__main__":
    main()
