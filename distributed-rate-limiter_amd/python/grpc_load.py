"""Open-loop load generator for the gRPC server (BASELINE configs[4]):
Zipf s=1.5 keys over 1M users (the top key draws 38 % of requests), fixed
offered rates, latency per decision measured at the client from its
scheduled send time to the response (queueing included: no coordinated
omission).  `P` client processes, each with its own channel, share a level's
rate.  Two request shapes: unary Allow (one decision per RPC) and AllowBatch
(`batch` decisions per RPC, the BatchAllow path)."""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)


def _client(addr, limiter, rate, seconds, batch, seed, q):
    import threading

    import grpc

    import rl_grpc
    import traces
    a = rl_grpc.api()
    ch = grpc.insecure_channel(addr)
    st = rl_grpc.rate_limiter_stub(ch)
    keys = traces.ZipfKeys(1_000_000, 1.5, perm_seed=2)
    rng = np.random.default_rng(seed)
    n_rpc = max(1, int(rate * seconds))
    ids = keys.sample(rng, n_rpc * batch)
    lat = np.full(n_rpc, np.nan)
    errs = [0]
    lock = threading.Lock()
    pending = [0]
    # warm the channel
    st.Allow(a.AllowRequest(limiter=limiter, key="warm"))
    gap = 1.0 / rate
    t0 = time.perf_counter() + 0.05

    def cb(fut, i, ts):
        te = time.perf_counter()
        try:
            fut.result()
            lat[i] = te - ts
        except Exception:
            with lock:
                errs[0] += 1
        with lock:
            pending[0] -= 1

    for i in range(n_rpc):
        ts = t0 + i * gap
        d = ts - time.perf_counter()
        if d > 0:
            time.sleep(d)
        if batch == 1:
            req = a.AllowRequest(limiter=limiter, key=f"user:{ids[i]}")
            fut = st.Allow.future(req)
        else:
            req = a.AllowBatchRequest(requests=[a.AllowNRequest(limiter=limiter, key=f"user:{k}", n=1)
                                                for k in ids[i * batch:(i + 1) * batch]])
            fut = st.AllowBatch.future(req)
        with lock:
            pending[0] += 1
        fut.add_done_callback(lambda f, i=i, ts=ts: cb(f, i, ts))
    deadline = time.perf_counter() + 30
    while time.perf_counter() < deadline:
        with lock:
            if pending[0] == 0:
                break
        time.sleep(0.01)
    elapsed = time.perf_counter() - t0
    ch.close()
    q.put((lat.tolist(), errs[0], elapsed))


def run_level(addr, limiter, rate, seconds, batch, procs):
    q = mp.get_context("spawn").Queue()
    ps = [mp.get_context("spawn").Process(target=_client, args=(addr, limiter, rate / procs, seconds, batch,
                                                                  100 + k, q)) for k in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=seconds + 120) for _ in ps]
    for p in ps:
        p.join(30)
    lat = np.array([x for r in res for x in r[0]], np.float64)
    errs = sum(r[1] for r in res)
    elapsed = max(r[2] for r in res)
    ok = lat[~np.isnan(lat)] * 1e6
    if ok.size == 0:
        return {"offered_rpc_per_s": rate, "batch": batch, "errors": errs, "completed": 0}
    return {"offered_rpc_per_s": rate, "offered_decisions_per_s": rate * batch, "batch": batch,
            "achieved_decisions_per_s": ok.size * batch / elapsed, "completed_rpcs": int(ok.size),
            "errors": int(errs), "p50_us": float(np.percentile(ok, 50)), "p99_us": float(np.percentile(ok, 99)),
            "p999_us": float(np.percentile(ok, 99.9)), "max_us": float(ok.max())}


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--addr", required=True)
    ap.add_argument("--limiter", default="default")
    ap.add_argument("--unary", default="2000,5000,10000", help="unary Allow RPC rates")
    ap.add_argument("--batched", default="500,2000,4000", help="AllowBatch RPC rates")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--procs", type=int, default=6)
    args = ap.parse_args(argv)
    levels = []
    for r in [float(x) for x in args.unary.split(",") if x]:
        levels.append(run_level(args.addr, args.limiter, r, args.seconds, 1, args.procs))
    for r in [float(x) for x in args.batched.split(",") if x]:
        levels.append(run_level(args.addr, args.limiter, r, args.seconds, args.batch, args.procs))
    print(json.dumps({"levels": levels}))


if __name__ == "__main__":
    main()
