#!/usr/bin/env python3
"""bench.py -- decisions/s of the MI355X rate-limit decision engine.

Workload (BASELINE.json configs[1], the metric's single-GPU config):
  Token Bucket "100/min burst 20" == {Limit 20, Window 12 s}; 1M keys Zipf
  s=1.1 (rank->id seeded permutation, seed 2); arrivals exp(mean 1 us) from
  t0 = 1.76e18 ns (seed 3); n = 1; batches of 1M requests.
A step = one batch through the full engine path (probe/insert into the HBM
table, radix sort by slot, segment discovery, per-key replay with exact Redis
Lua "%.14g" semantics), inputs already resident in HBM, results written to HBM.

Multi-GPU (one rank per GPU; `--gpus N` launches torch.distributed.run itself
when WORLD_SIZE is unset): the metric's own workload (configs[1], Zipf 1M
keys) drawn by every rank from the whole key space and routed to the key's
owner GPU and back by RCCL all-to-alls over xGMI (include/rl_route.h,
shard.RoutedPipeline).  Per-GPU work is fixed -> "scaling": "weak".  The
line carries `hot_owner_bound`: the hot key replays in order on its owner, so
chain steps/s / hot share caps this workload on any N.  BASELINE configs[3]
(mixed tenants over 1B keys) is reported beside it under its own metric name,
routed and as key-shard replicas (each rank its own keys, no data-path
collective), in `secondary`.

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


def cpu_config0(requests=1_000_000):
    """BASELINE.md's configs[0] CPU line: Fixed Window
    100/min, 10k uniform keys, a 1M-request trace, one request per call --
    the reference's per-call path (one EVAL per Allow on one single-threaded
    Redis) restated in C (oracle/rl_oracle.c, the cpu_baseline leg: test
    infrastructure).  Every call is timed on its own (clock_gettime around
    each): decisions/s and per-call p50 / p99 on one core."""
    import oracle
    gen = make_workload("fw_uniform", requests, 0)
    sim = oracle.OracleSim(oracle.REDIS7)
    for a, L, W in gen.configs:
        sim.add_config(a, L, W)
    key, ts, n, cfg = gen.next_batch()
    t0 = time.perf_counter()
    _, call_ns = sim.decide_timed(key, ts, n, cfg)
    wall = time.perf_counter() - t0
    return {"workload": WORKLOAD_DESC["fw_uniform"] + f", {requests} requests, one call per request",
            "value": requests / wall, "unit": "decisions/s", "cores": 1, "kind": "port",
            "p50_call_us": float(np.percentile(call_ns, 50)) / 1e3,
            "p99_call_us": float(np.percentile(call_ns, 99)) / 1e3,
            "mean_call_us": float(call_ns.mean()) / 1e3,
            "how": "oracle/rl_oracle.c rlo_decide_timed: each request its own call, timed with CLOCK_MONOTONIC; "
                   "the store is in-process (no Redis round trip or Lua VM: a lower bound on the reference's "
                   "per-call latency)"}


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


def grpc_bench(args, out_fd):
    """BASELINE configs[4] end to end: the gRPC server (rl_server.py, a child
    process that owns the GPU; native front end by default) and an open-loop
    gRPC load generator (lib/rl_grpc_load, C++ over HTTP/2; Zipf s=1.5 over 1M
    keys) at fixed offered rates; latency per RPC at the client from its
    scheduled send time.  This process never touches the GPU."""
    import subprocess
    py = os.path.join(ROOT, "distributed-rate-limiter_amd", "python")
    load = os.path.join(ROOT, "distributed-rate-limiter_amd", "lib", "rl_grpc_load")
    if not os.path.exists(load):
        raise SystemExit(f"{load} not built (__graft_entry__.build())")
    srv = subprocess.Popen([sys.executable, os.path.join(py, "rl_server.py"), "--address", "127.0.0.1:0",
                            "--frontend", args.grpc_frontend, "--io-threads", str(args.grpc_io_threads),
                            "--limiter", "default:token_bucket:20:12s", "--tb-capacity", str(1 << 21),
                            "--win-capacity", "1024"], stdout=subprocess.PIPE)
    levels = []
    try:
        line = srv.stdout.readline().decode()
        if not line.startswith("READY"):
            raise SystemExit(f"server did not start: {line!r}")
        addr = f"127.0.0.1:{int(line.split()[1])}"
        shapes = [(float(r), 1) for r in args.grpc_unary.split(",") if r] + \
                 [(float(r), 256) for r in args.grpc_batched.split(",") if r]
        for rate, batch in shapes:
            p = subprocess.run([load, "--addr", addr, "--rate", str(rate), "--seconds", str(args.seconds),
                                "--batch", str(batch), "--threads", str(args.grpc_threads), "--conns", "4",
                                "--limiter", "default", "--zipf", "1.5", "--keys", "1000000"],
                               stdout=subprocess.PIPE, timeout=args.seconds + 120, check=True)
            levels.append(json.loads(p.stdout.decode().strip().splitlines()[-1]))
            print(json.dumps(levels[-1]), file=sys.stderr, flush=True)
    finally:
        srv.terminate()
        srv.wait(60)
    ok = [lv for lv in levels if lv["batch"] == 1 and not lv["errors"] and not lv["unanswered"]
          and lv["achieved_rpc_per_s"] >= 0.95 * lv["offered_rpc_per_s"]]
    top = ok[-1] if ok else levels[0]
    out = {"metric": "p99 decision latency at fixed offered load through the gRPC server (configs[4])",
           "value": top.get("p99_us"), "unit": "us", "n_gpus": 1, "higher_is_better": False, "vs_baseline": None,
           "dtype": "f64", "data": "synthetic (Zipf s=1.5 over 1M keys 'user:<id>', fixed-rate open-loop clients)",
           "config": {"workload": "configs[4]: gRPC server (api/proto/ratelimiter.proto), Token Bucket 20/12s, "
                                  "coalesced GPU batches; unary Allow and AllowBatch (256 AllowN) RPCs",
                      "value_at": {"rpc_per_s": top.get("offered_rpc_per_s"), "batch": top.get("batch")},
                      "client": f"lib/rl_grpc_load: {args.grpc_threads} threads x 4 HTTP/2 connections",
                      "server": f"rl_server.py --frontend {args.grpc_frontend} ({args.grpc_io_threads} event loops)"
                      if args.grpc_frontend == "native" else "rl_server.py --frontend python (grpcio, 64 workers)",
                      "reference_single_redis_tb_estimate_rps": 35000},
           "levels": levels}
    os.write(out_fd, (json.dumps(out) + "\n").encode())


def spawn_ranks(args_list, n, out_fd):
    """`--gpus N` without a launcher: start torch.distributed.run as a child
    (before this process touches the GPU) and relay its one JSON line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + args_list
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
    if lines:
        os.write(out_fd, (lines[-1] + "\n").encode())
    return p.returncode


KEYSPACE = {"tb_zipf": (1 << 21, 1024), "tb_zipf15": (1 << 21, 1024), "tb_hot": (1 << 10, 1024),
            "fw_uniform": (1024, 1 << 15), "sw_bursty": (1024, 1 << 27), "mixed": (1 << 26, 1 << 26)}


REHEARSE = [False]     # --rehearse-gloo (main)
CDEV = [None]          # device of the small collective tensors: the GPU (RCCL), the CPU (gloo)


class AgreedError(RuntimeError):
    """an error every rank raises at the same point (agreed by an all_reduce)"""


REPLAY_EVENT_STRIDE = 4   # replay timing events on every 4th launch of the timed region


def roofline_of(replay_ms, algs, uniq, m, workload):
    """the dominant kernel is the replay (k_tb_chain: every decision's script
    replay, the path's critical kernel); its launch time comes from HIP events
    on its own stream over the timed region"""
    per_launch_ms = {"replay": replay_ms}
    dom = "replay"
    kname = {"replay": "k_tb_chain<true>", "probe": "k_probe", "sort_pass": "k_sort_pass<false>",
             "segments": "k_permute", "finish": "k_unpermute"}[dom]
    # HBM bytes per launch of that kernel from the committed rocprofv3 PMC
    # passes of this build (scripts/profile.sh: FETCH_SIZE x2 + WRITE_SIZE,
    # gfx950 correction); `traffic_profile` names the pass
    traffic, tag = None, None
    try:
        tj = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))
        if tj.get("workload", "tb_zipf") == workload and kname in tj["kernels"]:
            traffic = tj["kernels"][kname]["bytes_per_launch"]
            tag = tj.get("tag")
    except (OSError, ValueError, KeyError):
        pass
    s_alg = max(STATE_BYTES[a] for a in algs)
    bytes_per_dec = 24 + 32 + 2 * s_alg * (uniq / m)
    achieved = bytes_per_dec * m / (per_launch_ms[dom] / 1e3) / 1e9
    return {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_profile": tag,
            "algorithmic_bytes_per_launch": bytes_per_dec * m, "bytes_per_decision": bytes_per_dec,
            "launch_ms": per_launch_ms[dom]}, per_launch_ms


def _rel_us(dbgw, k):
    """debug word k (10-ns realtime ticks, low 32 bits) in us after the replay's first block start
    (dbg[13] holds its complement); None when unset (product builds)"""
    if not int(dbgw[k]):
        return None
    return ((int(dbgw[k]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100


def hot_chain_us(dbgw):
    """the last batch's longest huge segment (the hot key's chain), start to
    end in microseconds (replay kernel timeline words, 10 ns ticks)"""
    return ((int(dbgw[17]) - int(dbgw[16])) & 0xffffffff) / 100.0


def hot_owner_bound(hot_len, hot_us, m_total):
    """The ceiling the hot key puts on the whole job: its requests replay in
    order on one block of its owner GPU (tokenbucket.go:36-48 is a serial
    recurrence), so no number of GPUs decides faster than chain rate / hot
    share (12.4 % of every batch at Zipf 1.1)."""
    if hot_len <= 0 or hot_us <= 0:
        return None
    rate = hot_len / (hot_us * 1e-6)
    share = hot_len / m_total
    return {"hot_key_requests_per_step": int(hot_len), "hot_share": share, "chain_us": hot_us,
            "chain_steps_per_s": rate, "bound_decisions_per_s": rate / share,
            "how": "the last step's hottest segment on its owner: chain steps/s (replay kernel timeline) / the "
                   "key's share of all ranks' requests; no GPU count decides this workload faster"}


def bench_local(args, workload, world, rank, local_rank, dev, sharded):
    """each rank decides its own batches (N=1: the whole engine; N>1 with
    `sharded`: each rank owns a disjoint key space -- replicas)"""
    import torch
    import torch.distributed as dist

    import rl_amd
    gen = make_workload(workload, args.batch, rank)
    nb = args.warmup + args.steps
    lat_n = max(0, args.lat_batches) if world == 1 else 0
    extra = lat_n if lat_n else 4      # batches after the timed region (latency / stage breakdown)
    host = [gen.next_batch() for _ in range(nb + extra)]
    if os.environ.get("RL_BENCH_HOME_SORT"):
        # A/B experiment only: each batch stably reordered by the key's home
        # slot in the engine's tables ("full") or by its top 8 bits ("digit"),
        # to price a probe that walks the table in home order (per-key order
        # is kept, so decisions are those of a valid trace)
        import shard
        tb_cap, win_cap = KEYSPACE[workload]
        bits = int(tb_cap + win_cap).bit_length()
        tbc = np.array([a == 1 for a, _, _ in gen.configs])
        out = []
        for key, ts, n, cfg in host:
            h = shard.mix64(key)
            is_tb = tbc[cfg]
            g = np.where(is_tb, h & np.uint64(tb_cap - 1), np.uint64(tb_cap) + (h & np.uint64(win_cap - 1)))
            if os.environ["RL_BENCH_HOME_SORT"] == "digit":
                g = g >> np.uint64(bits - 8)
            o = np.argsort(g, kind="stable")
            out.append((key[o], ts[o], n[o], cfg[o]))
        host = out
    # sharded ingress: this rank's own key space (ids tagged with the rank)
    tag = np.uint64(rank if sharded else 0) << np.uint64(48)
    uniq, cnt = np.unique(host[-1][0], return_counts=True)
    uniq, hot_len = uniq.size, int(cnt.max())
    del cnt
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
    tb_cap, win_cap = KEYSPACE[workload]
    eng = rl_amd.Engine(profile=rl_amd.PROFILE_REDIS7, tb_capacity=tb_cap, win_capacity=win_cap,
                        max_batch=args.batch, device=dev.index,
                        # inputs are resident before the timed region: batch b+1's
                        # hash/sort/permute overlaps batch b's replay
                        flags=0 if args.no_pipeline else rl_amd.OPT_PIPELINE)
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

    for b in range(args.warmup):
        step(b)
    torch.cuda.synchronize()
    rc = eng.sync()
    if rc != 0:
        raise SystemExit(f"engine error during warmup: {rc} {eng.last_error()}")
    # timed region: events around the replay only, on every 4th launch (two
    # per sampled batch on its stream: each pair costs the replay stream
    # ~10 us, profiles/r4tm_timing_events.txt -- the measurement's own cost,
    # so it samples: 5 of the driver's 20 launches); the per-stage breakdown
    # comes from the latency phase below
    timing = 0 if os.environ.get("RL_BENCH_NO_TIMING") else -REPLAY_EVENT_STRIDE
    eng.set_timing(timing)
    eng.stage_times()  # clear

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(args.warmup, nb):
        step(b)
    t_host = time.perf_counter() - t0   # the host's enqueue time (device work runs behind it)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rc = eng.sync()
    if rc != 0:
        raise SystemExit(f"engine error during timed region: {rc} {eng.last_error()}")
    stage_ms, nbat = eng.stage_times()
    replay_ms = stage_ms[3] / nbat if timing else float("nan")
    replay_timed = int(nbat)
    st = eng.stats()
    dbgw = eng.debug_words()
    stamp_ring = None
    if os.environ.get("RL_STAMP_KERNELS"):
        sr = eng.debug_stamps()
        if sr is not None:
            first = (st.batches - args.steps) % 256   # slots of the timed batches
            rows = np.array([sr[(first + i) % 256] for i in range(min(args.steps, 256))], np.int64)
            rel = (rows - rows[0, 0]) & 0xffffffff
            us = rel / 100.0
            stamp_ring = {"per_batch_us [front0, front1, replay0, replay1, finish0, finish1]": us.round(1).tolist(),
                          "replay_us_mean": float(np.mean(us[:, 3] - us[:, 2])),
                          "replay_period_us_mean": float(np.mean(np.diff(us[:, 2]))) if len(us) > 1 else None,
                          "front_us_mean": float(np.mean(us[:, 1] - us[:, 0]))}
    eng.set_timing(2)   # every stage, for the breakdown

    # latency phase (p99 batch latency of the metric): the next lat_n batches of
    # the same trace, closed loop with `depth` batches in flight; a batch's
    # latency runs from the host call to the host seeing its results complete
    # on the caller's stream (an upper bound: batches are waited for in order)
    depth = 1 if args.no_pipeline else 3
    lat, pend = [], []
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
    if lat_n == 0:   # no latency phase: the next few batches of the trace for the breakdown
        for b in range(nb, nb + extra):
            step(b)
        torch.cuda.synchronize()
        eng.sync()
    stage_ms, nbat = eng.stage_times()
    eng.set_timing(0)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=CDEV[0])
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    roof, per_launch_ms = roofline_of(replay_ms, algs, uniq, m, workload)
    roof["launches_timed"] = replay_timed
    roof["launch_ms_how"] = (f"HIP events on the replay's dispatch packets, every {REPLAY_EVENT_STRIDE}th launch "
                             f"of the timed region")
    latency = None
    if lat:
        la = np.array(lat) * 1e3
        latency = {"p50_batch_ms": float(np.percentile(la, 50)), "p99_batch_ms": float(np.percentile(la, 99)),
                   "max_batch_ms": float(la.max()), "batches": int(la.size), "in_flight": depth,
                   "batch": m, "how": "closed loop after the timed region; host call -> results complete"}
    res = {
        "value": args.steps * m * world / elapsed,
        "ms_per_step": elapsed / args.steps * 1e3,
        "workload": WORKLOAD_DESC[workload],
        "ingress": "sharded (each rank its own key space, no data-path collective)" if sharded and world > 1
        else "local",
        "batch": m, "unique_keys_per_batch": uniq,
        "batches_in_flight": 1 if args.no_pipeline else 3,
        "host_ms_per_step": {"enqueue": t_host / args.steps * 1e3},
        "roofline": roof,
        "replay_detail": {"heavy_segments": int(st.last_heavy), "segments": int(st.last_segments),
                          "stamp_cycles_longest_segment": [int(x) for x in st.stamp_cycles],
                          "coop_rounds": int(st.last_coop_rounds), "coop_iters": int(st.last_coop_iters),
                          "round_ends_full_stop_partial_first": [int(x) for x in st.coop_ends],
                          "exact_tiles": int(dbgw[20]), "serial_steps": int(dbgw[21]),
                          # multi-decade windows: resolved, full, near passes, chain cycles / 16,
                          # windows summarized XDEC / DEC, exact tiles, their passes, near
                          # entries, near groups stopped unconverged
                          "xdec": [int(x) for x in dbgw[60:70]],
                          # speculative restart windows: adopted, rejected (the chain's exit
                          # ended 1 / 2-64 steps after the guess, other)
                          "spec_windows": [int(dbgw[22]), int(dbgw[23]), int(dbgw[9]), int(dbgw[10]),
                                           int(dbgw[15])],
                          "replay_timeline_us": {"hot_start": ((int(dbgw[16]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100,
                                                 "hot_end": ((int(dbgw[17]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100,
                                                 "last_block_end": ((int(dbgw[14]) - (~int(dbgw[13]) & 0xffffffff)) & 0xffffffff) / 100,
                                                 # RL_STAMP_KERNELS=1: one-lane kernels just before / after the replay on its stream
                                                 "stamp_before": (((int(dbgw[18]) - (~int(dbgw[13]) & 0xffffffff) + (1 << 31)) & 0xffffffff) - (1 << 31)) / 100 if dbgw[18] else None,
                                                 "stamp_after": (((int(dbgw[19]) - (~int(dbgw[13]) & 0xffffffff) + (1 << 31)) & 0xffffffff) - (1 << 31)) / 100 if dbgw[19] else None},
                          "stamps_x16": [int(x) * 16 for x in dbgw[24:37]], "near_hot": [int(x) for x in dbgw[37:39]],
                          "near_setup_x16": int(dbgw[39]) * 16,
                          # stamps build: producer 0's cycles on one-decade / multi-decade windows and their
                          # counts, then the chain's resolve cycles and counts the same way
                          "split_x16": [int(dbgw[70 + k]) * (16 if k in (0, 1, 4, 5) else 1) for k in range(8)]
                          + [int(dbgw[80]) * 16, int(dbgw[81]) * 16],
                          # stamps builds: the chain round's pipeline model (two / three
                          # summary buffers, sum of the rounds' max(producer, chain) work,
                          # the chain's and the slowest producer's work over the rounds)
                          "pipeline_model_x16": [int(dbgw[82 + k]) * 16 for k in range(5)],
                          "chain_round_tops_x16": int(dbgw[87]) * 16,
                          # stamps build: producer 0's plan cycles (after the exit guess)
                          "producer_plan_x16": int(dbgw[48]) * 16,
                          # of which in the window-plan calls: count, cycles
                          "plan_calls": [int(dbgw[49]), int(dbgw[50]) * 16],
                          # stamps build: the replay's tail (us from the first block's start): the
                          # latest block start, the latest end of a heavy phase, the latest light
                          # claim that got work; the longest heavy segment's replay (us, length)
                          "replay_tail_us": {"last_block_start": _rel_us(dbgw, 51), "last_heavy_end": _rel_us(dbgw, 53),
                                             "last_light_claim": _rel_us(dbgw, 54),
                                             "longest_heavy_segment": [int(dbgw[56]) / 100, int(dbgw[57])]},
                          # stamps build: the hot chain's exact tiles (cycles, passes)
                          "exact_hot_x16": [int(dbgw[7]) * 16, int(dbgw[11])],
                          # batches whose grouping sort ran as k_sort_local alone (predicted plan)
                          "sort_predicted_batches": int(st.sort_predicted), "batches": int(st.batches),
                          # replayed by the light kernel (no huge segment expected)
                          "light_batches": int(st.light_batches)},
        "latency": latency,
        "stamp_ring": stamp_ring,
        "hot_owner_bound": hot_owner_bound(hot_len, hot_chain_us(dbgw), m) if workload.startswith("tb_zipf")
        and not sharded else None,
        "stages_ms_per_batch": {k: v for k, v in zip(["probe", "sort", "segments", "replay", "finish"],
                                                    (stage_ms / max(nbat, 1)).tolist())},
        "stages_how": "HIP events on every stream, over the latency phase (after the timed region, which "
                      "records events around the replay only)",
    }
    eng.close()
    return res


def bench_routed(args, workload, world, rank, local_rank, dev, pg_res):
    """every rank draws requests from the whole key space; the native routed
    pipeline (include/rl_route.h) moves them to their owners and back in
    fixed-capacity buckets, with no host read in the step"""
    import torch
    import torch.distributed as dist

    import rl_amd
    import shard
    gen = make_workload(workload, args.batch, rank)
    nb = args.warmup + args.steps
    m = args.batch
    host = [gen.next_batch() for _ in range(nb)]
    # the hot key (Zipf rank 1: every rank's generator shares the rank->id
    # permutation) in this rank's last batch, for the hot-owner bound
    hot_mine = int(np.count_nonzero(host[-1][0] == gen.keys.perm[0])) if hasattr(gen, "keys") else 0
    # bucket capacity per peer (every rank the same: the all-to-alls' equal
    # splits).  A uniform hash partition needs ~m / world plus a margin; a Zipf
    # hot key lands on one owner (12.4 % of every rank's batch at s = 1.1).
    # Sized from the trace itself: the largest per-owner count of any rank's
    # batch, so no request of the run is ever dropped (RL_ROUTE_SLACK = f
    # sizes f * m / world instead)
    slack = float(os.environ.get("RL_ROUTE_SLACK", "0"))
    if world == 1:
        cap = m
    elif slack:
        cap = min(m, int(np.ceil(slack * m / world)))
    else:
        need = max(int(np.bincount(shard.owner_of(k, world), minlength=world).max()) for k, _, _, _ in host)
        need_t = torch.tensor([need], dtype=torch.int64, device=CDEV[0])
        dist.all_reduce(need_t, op=dist.ReduceOp.MAX)
        cap = min(m, max(int(need_t.item()), int(np.ceil(1.05 * m / world))))
    ins = [(torch.from_numpy(k.view(np.int64)).to(dev), torch.from_numpy(t).to(dev), torch.from_numpy(n).to(dev),
            torch.from_numpy(c.view(np.int32)).to(dev)) for k, t, n, c in host]
    del host
    algs = {a for a, _, _ in gen.configs}
    tb_cap, win_cap = KEYSPACE[workload]
    router = rl_amd.Router(dev.index, world, m, cap)
    eng = rl_amd.Engine(profile=rl_amd.PROFILE_REDIS7, tb_capacity=tb_cap, win_capacity=win_cap,
                        max_batch=world * router.capacity, device=dev.index, flags=0)
    for a, L, W in gen.configs:
        eng.register(a, L, W)
    exchange = world > 1 or args.route_exchange
    # A/B knobs: RL_ROUTE_LOOKAHEAD (result exchange that many steps late),
    # RL_ROUTE_ONE_PG=1 (both directions on the default group: one stream
    # orders them), RL_ROUTE_UNORDERED=1 (no cross-group waits)
    one_pg = bool(os.environ.get("RL_ROUTE_ONE_PG"))
    pipe = shard.RoutedPipeline(router, eng.decide_routed, world, m, dev, pg_req=None, staged=REHEARSE[0],
                                pg_res=None if one_pg else pg_res,
                                depth=int(os.environ.get("RL_ROUTE_DEPTH", "4")), exchange=exchange,
                                lookahead=int(os.environ.get("RL_ROUTE_LOOKAHEAD", "1")),
                                ordered=not os.environ.get("RL_ROUTE_UNORDERED"),
                                decide_ev=None if os.environ.get("RL_ROUTE_NO_EV") else eng.decide_routed_ev)
    outs = [(torch.empty(m, dtype=torch.uint8, device=dev),) +
            tuple(torch.empty(m, dtype=torch.int64, device=dev) for _ in range(3)) for _ in range(pipe.depth)]
    def check(when):   # raises AgreedError on every rank alike
        # every rank takes the same branch (a rank that stopped alone would
        # leave the others in a collective): the worst code over the ranks
        rcs = [eng.sync(), router.sync(None)]
        t = torch.tensor(rcs, dtype=torch.int64, device=CDEV[0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        for what, rc, mine in zip(("engine", "router"), t.tolist(), rcs):
            if rc != 0:
                raise AgreedError(f"{what} error during {when}: {rc}"
                                   + (f" {eng.last_error()}" if mine else " (on another rank)")
                                   + (" (bucket overflow: raise RL_ROUTE_SLACK)" if rc == rl_amd.RL_EOVERFLOW else ""))

    pipe.run(ins[:args.warmup], [outs[b % pipe.depth] for b in range(args.warmup)])
    torch.cuda.synchronize()
    check("warmup")
    eng.set_timing(0 if os.environ.get("RL_BENCH_NO_TIMING") else -REPLAY_EVENT_STRIDE)
    eng.stage_times()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.run(ins[args.warmup:], [outs[b % pipe.depth] for b in range(args.steps)])
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    check("timed region")
    stage_ms, nbat = eng.stage_times()
    st = eng.stats()
    dbgw = eng.debug_words()
    eng.set_timing(0)
    tt = torch.tensor([elapsed], dtype=torch.float64, device=CDEV[0])
    agg = [torch.zeros_like(tt) for _ in range(world)]
    dist.all_gather(agg, tt)
    elapsed = float(torch.stack(agg).max().cpu())
    # the hot key's owner has the longest chain; its requests come from every rank
    hot = torch.tensor([float(hot_mine), hot_chain_us(dbgw)], dtype=torch.float64, device=CDEV[0])
    hot_sum = hot[:1].clone()
    dist.all_reduce(hot_sum, op=dist.ReduceOp.SUM)
    dist.all_reduce(hot, op=dist.ReduceOp.MAX)
    hob = hot_owner_bound(int(hot_sum.item()), float(hot[1].item()), m * world) if hasattr(gen, "keys") else None
    # a hash partition: every owner receives ~m requests per step
    roof, _ = roofline_of(stage_ms[3] / nbat, algs, int(st.last_segments), m, workload)
    res = {
        "value": args.steps * m * world / elapsed,
        "ms_per_step": elapsed / args.steps * 1e3,
        "workload": WORKLOAD_DESC[workload],
        "ingress": (f"routed: owner = hash(key) mod {world}; per peer a fixed-capacity bucket of "
                    f"{router.capacity} 32-B request records and one of 32-B results, moved by equal-split "
                    + ("gloo all-to-alls through host memory (--rehearse-gloo: ranks share one GPU)" if REHEARSE[0]
                       else "RCCL all-to-alls over xGMI") + ("" if exchange else " (world 1: buckets read in place)")
                    + "; merge and engine sized on the device, no host read in the step (include/rl_route.h)"),
        "batch": m,
        "bucket_capacity": router.capacity,
        "collective_order": (("one group, one stream" if one_pg else "one order over both groups" if pipe.ordered
                              else "unordered (A/B)") + f", result exchange {pipe.lookahead} step(s) late")
        if exchange else "none (world 1, buckets read in place)",
        "host_ms_per_step": {"enqueue": t_host / args.steps * 1e3, "count_wait": pipe.wait_s / args.steps * 1e3},
        "roofline": roof,
        "hot_owner_bound": hob,
    }
    del pipe, outs, ins
    eng.close()
    router.close()
    rl_amd.release_dedicated_streams()
    return res


def main():
    # one JSON line on stdout: anything native libraries print (the RCCL banner,
    # ROCm notices) goes to stderr; the line is written to the saved stdout
    out_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=56,
                    help="timed steps (default: batches 5-60 of the 64-batch configs[1] trace)")
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--workload", default="tb_zipf", choices=sorted(WORKLOAD_DESC),
                    help="default: tb_zipf (configs[1], the metric's Zipf 1M keys) on every N; on N > 1 "
                         "configs[3] (mixed, 1B keys) is reported as a named secondary metric")
    ap.add_argument("--ingress", default=None, choices=["routed", "sharded"],
                    help="N > 1: routed (default; RCCL all-to-all to the key's owner) or sharded (replicas)")
    ap.add_argument("--no-secondary", action="store_true", help="N > 1: skip the secondary measurements")
    ap.add_argument("--route-exchange", action="store_true",
                    help="--ingress routed at N = 1: run the loopback all-to-alls too (the N > 1 step's work)")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="cpu_baseline requests per host core")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--rehearse-gloo", action="store_true",
                    help="N > 1 rehearsal on a one-GPU box: every rank on GPU 0, collectives over gloo (not a "
                         "measurement)")
    ap.add_argument("--no-pipeline", action="store_true", help="one batch in flight at a time")
    ap.add_argument("--lat-batches", type=int, default=32,
                    help="batches of the latency phase (after the timed region): closed loop with the "
                         "pipeline's depth in flight, per-batch issue->results-complete time")
    ap.add_argument("--string-keys", action="store_true",
                    help="requests carry raw string keys ('user:<rank>:<12 hex>'): every step runs the on-GPU "
                         "FormatKey + XXH64 (rl_hash_keys_device, prefix 'ratelimit') before the decisions")
    ap.add_argument("--e2e", action="store_true",
                    help="configs[4]: open-loop Zipf 1.5 traffic through the request coalescer at fixed QPS "
                         "levels (lib/rl_bench_e2e); reports per-request latency percentiles")
    ap.add_argument("--qps", default="1e5,1e6,1e7", help="--e2e offered QPS levels")
    ap.add_argument("--seconds", type=float, default=2.0, help="--e2e / --grpc seconds per level")
    ap.add_argument("--grpc", action="store_true",
                    help="configs[4] through the gRPC server: open-loop gRPC clients at fixed rates")
    ap.add_argument("--grpc-unary", default="10000,35000,70000,100000", help="--grpc unary Allow RPC rates")
    ap.add_argument("--grpc-batched", default="2000,8000", help="--grpc AllowBatch (256 per RPC) rates")
    ap.add_argument("--grpc-threads", type=int, default=4, help="--grpc load generator threads")
    ap.add_argument("--grpc-frontend", choices=["native", "python"], default="native", help="--grpc server front end")
    ap.add_argument("--grpc-io-threads", type=int, default=4, help="--grpc native server event loops")
    args = ap.parse_args()
    if args.e2e:
        return e2e(args, out_fd)
    if args.grpc:
        return grpc_bench(args, out_fd)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(sys.argv[1:], args.gpus, out_fd)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # --rehearse-gloo: every rank on GPU 0, collectives over gloo through host
    # memory -- the N > 1 code path of this script on a one-GPU box (the
    # numbers are not a measurement: ranks share one GPU)
    REHEARSE[0] = args.rehearse_gloo
    gpu = 0 if args.rehearse_gloo else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    CDEV[0] = torch.device("cpu") if args.rehearse_gloo else dev
    pg_res = None
    ingress = args.ingress or ("routed" if world > 1 else "local")
    workload = args.workload
    if world > 1 or ingress == "routed":
        # RCCL over xGMI: the request/count all-to-alls on the default group,
        # results on a second one (its own stream), barrier and timing
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29531"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        # the request group's internal stream at high priority: a hardware
        # queue apart from the result group's, whose stream waits on the
        # engine (a waiting stream blocks the streams that share its queue)
        opts = None
        if not os.environ.get("RL_ROUTE_PG_NORMAL"):
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
        if args.rehearse_gloo:
            dist.init_process_group("gloo")
            pg_res = dist.new_group(backend="gloo")
        else:
            dist.init_process_group("nccl", device_id=dev, pg_options=opts)
            pg_res = dist.new_group(backend="nccl")
    if ingress == "routed":
        res = bench_routed(args, workload, world, rank, local_rank, dev, pg_res)
    else:
        res = bench_local(args, workload, world, rank, local_rank, dev, sharded=world > 1)
    secondary = []
    if world > 1 and not args.no_secondary:
        # configs[3] (the multi-GPU config: mixed tenants over 1B keys) routed
        # and as key-shard replicas, each under its own metric name
        for wl, ing in (("mixed", "routed"), ("mixed", "sharded")):
            if (wl, ing) == (workload, ingress):
                continue
            try:
                r2 = (bench_routed(args, wl, world, rank, local_rank, dev, pg_res) if ing == "routed"
                      else bench_local(args, wl, world, rank, local_rank, dev, sharded=True))
                secondary.append({"metric": f"decisions/sec @{world} GPU, configs[3] mixed tenants 1B keys "
                                            f"({'routed to owners' if ing == 'routed' else 'key-shard replicas'})"}
                                 | {k: r2[k] for k in ("value", "ms_per_step", "workload", "ingress")}
                                 | {"unit": "decisions/s", "roofline_frac": r2["roofline"]["frac"]})
            except AgreedError as ex:
                # raised on every rank alike (the routed checks agree over the
                # ranks first): report it inside the line, the headline stands
                secondary.append({"workload": WORKLOAD_DESC.get(wl, wl), "ingress": ing, "error": str(ex)[:300]})
            except BaseException as ex:   # noqa: BLE001
                # raised on this rank alone: the other ranks may be waiting in a
                # collective for it, so end the job instead of hanging it
                print(f"rank {rank}: secondary {wl}/{ing} failed: {ex!r}", file=sys.stderr, flush=True)
                os._exit(3)
    out = {
        # BASELINE.json's metric names the Zipf 1M-key workload; a run of
        # another workload (--workload) is named by it instead
        "metric": ("decisions/sec @1/8 GPU, Zipf 1M keys; % HBM roofline; p99 batch latency"
                   if workload == "tb_zipf" else f"decisions/sec @{world} GPU, {WORKLOAD_DESC[workload]}"),
        "value": res["value"],
        "unit": "decisions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded trace generators, distributed-rate-limiter_amd/python/traces.py)",
        "config": {"workload": res["workload"], "batch": res["batch"],
                   "profile": "redis7 (Lua %.14g state round trip)",
                   "parallelism": res["ingress"] if world > 1 else "1 GPU",
                   "world_size_seen": world,
                   "keys": ("raw strings, on-GPU FormatKey + XXH64 in every step" if args.string_keys
                            else "integer key ids")},
        "roofline": res["roofline"],
    }
    for k in ("unique_keys_per_batch", "batches_in_flight", "bucket_capacity", "host_ms_per_step", "collective_order"):
        if k in res:
            out["config"][k] = res[k]
    for k in ("hot_owner_bound", "replay_detail", "latency", "stages_ms_per_batch", "stamp_ring"):
        if res.get(k) is not None:
            out[k] = res[k]
    if secondary:
        out["secondary"] = secondary
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(workload, args.batch, args.cpu_sample)
        out["cpu_baseline"]["configs0"] = cpu_config0()
    if rank == 0:
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
