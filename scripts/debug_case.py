"""Debug helper: run test_chain_regimes' trace on the GPU and print the first
mismatches against the oracle with their neighbourhood (GPU box only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "distributed-rate-limiter_amd", "python")]
import oracle  # noqa: E402
import rl_amd  # noqa: E402
from test_gpu_parity import _chain_trace, split  # noqa: E402
from tracegen import NS  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "mixed"
profile = int(sys.argv[2]) if len(sys.argv) > 2 else 0
configs = [(1, 20, 12 * NS), (1, 10, NS), (1, 3, 300_000_000)]
seed = {"deny": 1, "allow": 2, "mixed": 3}[kind] * 10 + profile
eng = rl_amd.Engine(profile=profile, tb_capacity=1 << 20, win_capacity=1 << 20, max_batch=1 << 20)
sim = oracle.OracleSim(profile)
for a, L, W in configs:
    eng.register(a, L, W)
    sim.add_config(a, L, W)
for bi, (key, ts, n, cfg, sms) in enumerate(split(_chain_trace(kind, seed), [50_000, 70_000])):
    res = eng.decide(key, ts, n, cfg, sms, check=False)
    dec, rem, retry, reset, tok = sim.decide(key, ts, n, cfg, sms)
    bad = np.nonzero((res.decision != dec) | (res.tokens.view(np.uint64) != tok.view(np.uint64)))[0]
    print(f"batch {bi}: status {res.status} mismatches {bad.size} dbg {eng.debug_words(24)[:8]}")
    for i in bad[:3]:
        k = key[i]
        idx = np.nonzero(key == k)[0]
        j = np.searchsorted(idx, i)
        print(f"  i={i} key={k} seg_pos={j}/{idx.size} n={n[i]} dec gpu/ref {res.decision[i]}/{dec[i]} "
              f"tok gpu {res.tokens[i]!r} ref {tok[i]!r}")
        for jj in range(max(0, j - 3), min(idx.size, j + 3)):
            ii = idx[jj]
            print(f"     [{jj}] ts={ts[ii]} n={n[ii]} dec={dec[ii]}/{res.decision[ii]} ref={tok[ii]!r} gpu={res.tokens[ii]!r}")
