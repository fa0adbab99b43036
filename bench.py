#!/usr/bin/env python3
"""bench.py -- decisions/s of the MI355X rate-limit decision engine.

Workload (BASELINE.json configs[1], the metric's single-GPU config):
  Token Bucket "100/min burst 20" == {Limit 20, Window 12 s}; 1M keys Zipf
  s=1.1 (rank->id seeded permutation, seed 2); arrivals exp(mean 1 us) from
  t0 = 1.76e18 ns (seed 3); n = 1; batches of 1M requests.
A step = one batch through the full engine path (probe/insert into the HBM
table, radix sort by slot, segment discovery, per-key replay with exact Redis
Lua "%.14g" semantics), inputs already resident in HBM, results written to HBM.

Multi-GPU (torchrun, one rank per GPU): the key space shards by owner; each
rank decides its own shard's requests (no data-path collective: the shards
are independent), so per-GPU work is fixed -> "scaling": "weak".

Prints one JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "distributed-rate-limiter_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
STATE_BYTES = {1: 24, 2: 48, 3: 32}  # S_TB, S_SW, S_FW


def make_workload(name, batch, rank):
    import traces
    if name == "tb_zipf":
        return traces.TokenBucketZipf(batch=batch, seed=3 + 1000 * rank)
    if name == "fw_uniform":
        return traces.FixedWindowUniform(batch=batch, seed=1 + 1000 * rank)
    if name == "sw_bursty":
        return traces.SlidingWindowBursty(batch=batch, seed=4 + 1000 * rank)
    if name == "mixed":
        return traces.MixedTenants(batch=batch, seed=5 + 1000 * rank)
    if name == "tb_zipf15":
        return traces.TokenBucketZipf(batch=batch, s=1.5, seed=3 + 1000 * rank)
    if name == "tb_hot":
        return traces.TokenBucketZipf(nkeys=1, batch=batch, seed=3 + 1000 * rank)
    raise SystemExit(f"unknown workload {name}")


WORKLOAD_DESC = {
    "tb_zipf": "configs[1]: Token Bucket 100/min burst 20 (Limit 20, Window 12s), 1M keys Zipf s=1.1, batch 1M",
    "fw_uniform": "configs[0]: Fixed Window 100/min, 10k uniform keys",
    "sw_bursty": "configs[2]: Sliding Window 100/min, 100M keys, uniform + bursty",
    "mixed": "configs[3]: mixed TB/SW/FW by key mod 3, 1B keys uniform",
    "tb_zipf15": "configs[4] key mix: Token Bucket 20/12s, 1M keys Zipf s=1.5 (top key 38%), batch 1M",
    "tb_hot": "diagnostic: Token Bucket 20/12s, one key, batch 1M",
}


def host_cores():
    """Host cores this process may use: the GPU box grants a 16-core share
    (OMP_NUM_THREADS is set to it there; nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def cpu_baseline(workload, batch, per_core_sample):
    """The CPU restatement (oracle/rl_oracle.c, C) timed on a bounded sample of
    the same workload on this host's cores (the cpu_baseline leg: test
    infrastructure, never the measured product).  SURVEY.md §8(d): Go + Redis
    are absent, so the restatement runs multi-threaded, one key shard per core
    -- N app servers each with its own single-threaded store, the best case for
    the reference's deployment (one Redis runs scripts on one core).  Each
    batch is split by owner = hash(key) mod cores inside the timed region (the
    routing work), then every shard decides on its own thread (ctypes releases
    the GIL for the C call)."""
    from concurrent.futures import ThreadPoolExecutor

    import oracle
    cores = host_cores()
    sample = per_core_sample * cores
    gen = make_workload(workload, min(batch, sample), 0)
    sims = []
    for _ in range(cores):
        sim = oracle.OracleSim(oracle.REDIS7)
        for a, L, W in gen.configs:
            sim.add_config(a, L, W)
        sims.append(sim)
    pool = ThreadPoolExecutor(max_workers=cores)
    mult = np.uint64(0x9E3779B97F4A7C15)
    done, t, first = 0, 0.0, True
    while done < sample:
        key, ts, n, cfg = gen.next_batch()
        t0 = time.perf_counter()
        owner = ((key * mult) >> np.uint64(40)) % np.uint64(cores)
        order = np.argsort(owner, kind="stable")
        bounds = np.searchsorted(owner[order], np.arange(cores + 1, dtype=np.uint64))
        parts = [order[bounds[c]:bounds[c + 1]] for c in range(cores)]
        futs = [pool.submit(sims[c].decide, key[ix], ts[ix], n[ix], cfg[ix]) for c, ix in enumerate(parts)]
        for f in futs:
            f.result()
        if first:   # warm-up batch (the tables grow), as the GPU's warmup steps
            first = False
            continue
        t += time.perf_counter() - t0
        done += key.size
    pool.shutdown()
    return {"value": done / t, "unit": "decisions/s", "cores": cores, "kind": "port",
            "sample": f"{done} requests of the same workload through oracle/rl_oracle.c (C restatement of "
                      f"Go + Redis Lua, glibc %.14g/strtod; multi-threaded restatement, not the reference): "
                      f"{cores} threads, one key shard each (owner = hash(key) mod {cores}, split inside the "
                      f"timed region), after one untimed warm-up batch"}


def e2e(args, out_fd):
    """BASELINE configs[4] through the native load generator (a child process;
    this process never touches the GPU)."""
    import subprocess
    exe = os.path.join(ROOT, "distributed-rate-limiter_amd", "lib", "rl_bench_e2e")
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} not built (__graft_entry__.build())")
    p = subprocess.run([exe, "--qps", args.qps, "--seconds", str(args.seconds)], stdout=subprocess.PIPE, check=True)
    r = json.loads(p.stdout.decode().strip().splitlines()[-1])
    kept = [lv for lv in r["levels"] if lv["achieved_decisions_per_s"] >= 0.95 * lv["offered_qps"] and not lv["dropped"]]
    top = kept[-1] if kept else r["levels"][0]
    out = {"metric": "p99 decision latency at fixed offered QPS through the request coalescer (configs[4])",
           "value": top["p99_us"], "unit": "us", "n_gpus": 1, "higher_is_better": False,
           "vs_baseline": None, "dtype": "f64", "data": "synthetic (Zipf s=1.5 over 1M keys, Poisson arrivals)",
           "config": {"workload": "configs[4]: Token Bucket 20/12s, 1M keys Zipf 1.5, open loop, coalesced batches",
                      "value_at_qps": top["offered_qps"], "max_batch": r["max_batch"], "generators": r["gens"]},
           "levels": r["levels"], "engine_status": r["engine_status"]}
    os.write(out_fd, (json.dumps(out) + "\n").encode())


def main():
    # one JSON line on stdout: anything native libraries print (the RCCL banner,
    # ROCm notices) goes to stderr; the line is written to the saved stdout
    out_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--workload", default="tb_zipf", choices=sorted(WORKLOAD_DESC))
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="cpu_baseline requests per host core")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="one batch in flight at a time")
    ap.add_argument("--lat-batches", type=int, default=32,
                    help="batches of the latency phase (after the timed region): closed loop with the "
                         "pipeline's depth in flight, per-batch issue->results-complete time")
    ap.add_argument("--route", action="store_true",
                    help="routed ingress: every rank draws keys from the whole key space and an RCCL "
                         "all-to-all moves each request to its owner GPU and the result back")
    ap.add_argument("--string-keys", action="store_true",
                    help="requests carry raw string keys ('user:<rank>:<12 hex>'): every step runs the on-GPU "
                         "FormatKey + XXH64 (rl_hash_keys_device, prefix 'ratelimit') before the decisions")
    ap.add_argument("--e2e", action="store_true",
                    help="configs[4]: open-loop Zipf 1.5 traffic through the request coalescer at fixed QPS "
                         "levels (lib/rl_bench_e2e); reports per-request latency percentiles")
    ap.add_argument("--qps", default="1e5,1e6,1e7", help="--e2e offered QPS levels")
    ap.add_argument("--seconds", type=float, default=2.0, help="--e2e seconds per QPS level")
    args = ap.parse_args()
    if args.e2e:
        return e2e(args, out_fd)

    import torch
    import torch.distributed as dist

    import rl_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.route:
        # RCCL over xGMI: barrier + max-over-ranks (sharded), plus the request /
        # result all-to-alls (routed)
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    gen = make_workload(args.workload, args.batch, rank)
    nb = args.warmup + args.steps
    lat_n = 0 if args.route else max(0, args.lat_batches)
    host = [gen.next_batch() for _ in range(nb + lat_n)]
    # sharded ingress: this rank's shard of the key space (ids tagged with the
    # owner rank); routed ingress: the shared key space, routed per batch
    tag = np.uint64(0 if args.route else rank) << np.uint64(48)
    uniq = np.unique(host[-1][0]).size
    dev_batches = []
    for key, ts, n, cfg in host:
        dev_batches.append((
            torch.from_numpy((key | tag).view(np.int64)).to(dev),
            torch.from_numpy(ts).to(dev),
            torch.from_numpy(n).to(dev),
            torch.from_numpy(cfg.view(np.int32)).to(dev),
        ))
    key_strings = []
    if args.string_keys:
        # fixed-width raw keys 'user:RR:xxxxxxxxxxxx' (20 B), built vectorized
        hexd = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
        head = np.frombuffer(f"user:{rank % 100:02d}:".encode(), dtype=np.uint8)
        for key, _, _, _ in host:
            sh = np.arange(44, -4, -4, dtype=np.uint64)
            digits = hexd[((key[:, None] >> sh[None, :]) & np.uint64(15)).astype(np.int64)]
            raw = np.concatenate([np.broadcast_to(head, (key.size, head.size)), digits], axis=1)
            off = np.arange(key.size + 1, dtype=np.int64) * raw.shape[1]
            key_strings.append((torch.from_numpy(np.ascontiguousarray(raw).reshape(-1)).to(dev),
                                torch.from_numpy(off).to(dev), None))
    del host

    algs = {a for a, _, _ in gen.configs}
    need_tb = 1 in algs
    keyspace = {"tb_zipf": 1 << 21, "tb_zipf15": 1 << 21, "tb_hot": 1 << 10, "fw_uniform": 1 << 15,
                "sw_bursty": 1 << 27, "mixed": 1 << 26}[args.workload]
    eng = rl_amd.Engine(profile=rl_amd.PROFILE_REDIS7,
                        tb_capacity=keyspace if need_tb else 1024,
                        win_capacity=keyspace if algs - {1} else 1024,
                        max_batch=args.batch * (2 if args.route else 1), device=local_rank,
                        # inputs are resident before the timed region: batch b+1's
                        # hash/sort/permute overlaps batch b's replay
                        # (routed: the inputs come out of the all-to-all on torch's stream)
                        flags=0 if args.no_pipeline or args.route else rl_amd.OPT_PIPELINE)
    for a, L, W in gen.configs:
        eng.register(a, L, W)
    m = args.batch
    out_dec = torch.empty(m, dtype=torch.uint8, device=dev)
    out_rem = torch.empty(m, dtype=torch.int64, device=dev)
    out_retry = torch.empty(m, dtype=torch.int64, device=dev)
    out_reset = torch.empty(m, dtype=torch.int64, device=dev)
    out_tok = torch.empty(m, dtype=torch.float64, device=dev)
    # a stream of our own, not the legacy default stream (which would order the
    # engine's streams behind each call)
    stream_obj = torch.cuda.Stream(dev)
    stream = stream_obj.cuda_stream

    def step(b):
        k, t, n, c = dev_batches[b]
        if args.route:
            import shard
            shard.route_and_decide_torch(k, t, n, c, decide_owned)
            return
        if args.string_keys:
            # raw keys: hashed on the engine's grouping stream ahead of the probe
            raw, off, _ = key_strings[b]
            rc = rl_amd.lib.rl_decide_batch_keys_device(
                eng.h, m, raw.data_ptr(), raw.numel(), off.data_ptr(), 1, b"ratelimit", 9, t.data_ptr(),
                n.data_ptr(), c.data_ptr(), None, out_dec.data_ptr(), out_rem.data_ptr(), out_retry.data_ptr(),
                out_reset.data_ptr(), out_tok.data_ptr(), stream)
            if rc != 0:
                raise SystemExit(f"rl_decide_batch_keys_device: {rc}")
            return
        eng.decide_device(m, k.data_ptr(), t.data_ptr(), n.data_ptr(), c.data_ptr(), None,
                          out_dec.data_ptr(), out_rem.data_ptr(), out_retry.data_ptr(), out_reset.data_ptr(),
                          out_tok.data_ptr(), stream)

    def decide_owned(k, t, n, c):
        # the owner's merged requests, on this GPU, enqueued on torch's stream
        mm = k.numel()
        o = [torch.empty(mm, dtype=torch.uint8, device=dev)] + \
            [torch.empty(mm, dtype=torch.int64, device=dev) for _ in range(3)]
        eng.decide_device(mm, k.data_ptr(), t.data_ptr(), n.data_ptr(), c.data_ptr(), None,
                          *[x.data_ptr() for x in o], 0, torch.cuda.current_stream(dev).cuda_stream)
        return o

    for b in range(args.warmup):
        step(b)
    torch.cuda.synchronize()
    rc = eng.sync()
    if rc != 0:
        raise SystemExit(f"engine error during warmup: {rc} {eng.last_error()}")
    eng.set_timing(True)
    eng.stage_times()  # clear

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(args.warmup, nb):
        step(b)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    rc = eng.sync()
    if rc != 0:
        raise SystemExit(f"engine error during timed region: {rc} {eng.last_error()}")
    stage_ms, nbat = eng.stage_times()
    st = eng.stats()
    dbgw = eng.debug_words()
    eng.set_timing(False)

    # latency phase (p99 batch latency of the metric): the next lat_n batches of
    # the same trace, closed loop with `depth` batches in flight; a batch's
    # latency runs from the host call to the host seeing its results complete
    # on the caller's stream (an upper bound: batches are waited for in order)
    depth = 1 if args.no_pipeline else 3
    lat = []
    pend = []
    for b in range(nb, nb + lat_n):
        if len(pend) >= depth:
            tb, ev = pend.pop(0)
            ev.synchronize()
            lat.append(time.perf_counter() - tb)
        tb = time.perf_counter()
        step(b)
        ev = torch.cuda.Event()
        ev.record(stream_obj)
        pend.append((tb, ev))
    for tb, ev in pend:
        ev.synchronize()
        lat.append(time.perf_counter() - tb)
    rc = eng.sync()
    if rc != 0:
        raise SystemExit(f"engine error during latency phase: {rc} {eng.last_error()}")
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    decisions = args.steps * m * world
    value = decisions / elapsed
    # per-launch device time of each kernel (HIP events on the launch stream)
    per_launch_ms = {
        "probe": stage_ms[0] / nbat,
        "sort_pass": stage_ms[1] / nbat / st.sort_passes,
        "segments": stage_ms[2] / nbat,
        "replay": stage_ms[3] / nbat,
        "finish": stage_ms[4] / nbat,
    }
    dom = max(per_launch_ms, key=per_launch_ms.get)
    # HBM bytes per launch of that kernel from the committed rocprofv3 PMC
    # passes (scripts/profile.sh: FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction)
    traffic = None
    kname = {"replay": "k_tb_chain<true>", "probe": "k_probe", "sort_pass": "k_sort_pass<false>",
             "segments": "k_permute", "finish": "k_unpermute"}[dom]
    try:
        tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
        if args.workload == "tb_zipf" and kname in tj["kernels"]:
            traffic = tj["kernels"][kname]["bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        pass
    s_alg = max(STATE_BYTES[a] for a in algs)
    bytes_per_dec = 24 + 32 + 2 * s_alg * (uniq / m)
    achieved = bytes_per_dec * m / (per_launch_ms[dom] / 1e3) / 1e9
    latency = None
    if lat:
        la = np.array(lat) * 1e3
        latency = {"p50_batch_ms": float(np.percentile(la, 50)), "p99_batch_ms": float(np.percentile(la, 99)),
                   "max_batch_ms": float(la.max()), "batches": int(la.size), "in_flight": depth,
                   "batch": m, "how": "closed loop after the timed region; host call -> results complete"}
    out = {
        "metric": "decisions/sec @1/8 GPU, Zipf 1M keys; % HBM roofline; p99 batch latency",
        "value": value,
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded trace generators, distributed-rate-limiter_amd/python/traces.py)",
        "config": {"workload": WORKLOAD_DESC[args.workload], "batch": m, "unique_keys_per_batch": uniq,
                   "profile": "redis7 (Lua %.14g state round trip)", "parallelism": (f"routed all-to-all x{world}" if args.route else f"key-shard x{world}"),
                   "batches_in_flight": 1 if args.no_pipeline or args.route else 3,
                   "keys": ("raw strings, on-GPU FormatKey + XXH64 in every step" if args.string_keys
                            else "integer key ids")},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "algorithmic_bytes_per_launch": bytes_per_dec * m,
                     "bytes_per_decision": bytes_per_dec, "launch_ms": per_launch_ms[dom]},
        "replay_detail": {"heavy_segments": int(st.last_heavy), "segments": int(st.last_segments),
                          "stamp_cycles_longest_segment": [int(x) for x in st.stamp_cycles],
                          "coop_rounds": int(st.last_coop_rounds), "coop_iters": int(st.last_coop_iters),
                          "round_ends_full_stop_partial_first": [int(x) for x in st.coop_ends],
                          "exact_tiles": int(dbgw[20]), "serial_steps": int(dbgw[21]),
                          "replay_timeline_us": {"hot_start": ((int(dbgw[16]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100,
                                                 "hot_end": ((int(dbgw[17]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100,
                                                 "last_block_end": ((int(dbgw[14]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100,
                                                 "stamp_before": ((int(dbgw[18]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100 - (1 << 32) / 100 if dbgw[18] else None,
                                                 "stamp_after": ((int(dbgw[19]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100 if dbgw[19] else None},
                          "stamps_x16": [int(x) * 16 for x in dbgw[24:37]], "near_hot": [int(x) for x in dbgw[37:39]], "near_setup_x16": int(dbgw[39]) * 16,
                          "hw_id": [hex(int(x)) for x in dbgw[40:45]]},
        "latency": latency,
        "stages_ms_per_batch": {k: v for k, v in zip(["probe", "sort", "segments", "replay", "finish"],
                                                    (stage_ms / nbat).tolist())},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.workload, m, args.cpu_sample)
    if rank == 0:
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    eng.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
