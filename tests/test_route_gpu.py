"""The routing kernels (include/rl_route.h, csrc/rl_route.hip) and the routed
decision path on the GPU (BASELINE configs[3]: hash-sharded keys, all-to-all
routing).  Bit-exact against the CPU restatement of the kernels
(tests/route_ops.py) and, end to end, against ONE shared limiter (the oracle)
over the union of the ranks' requests."""
import os
import socket

import numpy as np
import pytest

from tracegen import CONFIG_SETS, T0

pytestmark = pytest.mark.gpu
CONFIGS = CONFIG_SETS["mixed"]


def _dev_tensors(torch, *arrays):
    out = []
    for x in arrays:
        if x.dtype == np.uint64:
            x = x.view(np.int64)
        elif x.dtype == np.uint32:
            x = x.view(np.int32)
        out.append(torch.from_numpy(np.ascontiguousarray(x)).cuda())
    return out


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_route_kernels_match_restatement(rl, world):
    import torch

    import route_ops
    rng = np.random.default_rng(40 + world)
    m = 70_001
    key = rng.integers(0, 1 << 63, m).astype(np.uint64)
    ts = T0 + rng.integers(0, 3_000_000_000, m).astype(np.int64)      # unsorted, 3 s span
    ts[rng.random(m) < 0.2] = T0 + 12345                              # many equal times
    n = rng.integers(1, 9, m).astype(np.int64)
    cfg = rng.integers(0, 15, m).astype(np.uint32)
    r = rl.Router(0, world, m, m)
    k, t, nn, c = _dev_tensors(torch, key, ts, n, cfg)
    send = torch.empty((m, 4), dtype=torch.int64, device="cuda")
    scnt = torch.empty((world, 4), dtype=torch.int64, device="cuda")
    slot = torch.empty(m, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    r.pack(m, k.data_ptr(), t.data_ptr(), nn.data_ptr(), c.data_ptr(), send.data_ptr(), scnt.data_ptr(),
           slot.data_ptr(), s)
    own = torch.empty(m, dtype=torch.int32, device="cuda")
    r.owner(m, k.data_ptr(), own.data_ptr(), s)
    # CPU restatement
    ops = route_ops.NumpyRouteOps(world)
    kc, tc, nc, cc = [torch.from_numpy(np.ascontiguousarray(x.view(np.int64) if x.dtype == np.uint64 else
                                                            (x.view(np.int32) if x.dtype == np.uint32 else x)))
                      for x in (key, ts, n, cfg)]
    send_h = torch.empty((m, 4), dtype=torch.int64)
    scnt_h = torch.empty((world, 4), dtype=torch.int64)
    slot_h = torch.empty(m, dtype=torch.int32)
    ops.pack(m, kc.data_ptr(), tc.data_ptr(), nc.data_ptr(), cc.data_ptr(), send_h.data_ptr(), scnt_h.data_ptr(),
             slot_h.data_ptr(), None)
    torch.cuda.synchronize()
    import shard
    assert np.array_equal(own.cpu().numpy(), shard.owner_of(key, world))
    assert torch.equal(scnt.cpu(), scnt_h) and torch.equal(send.cpu(), send_h) and torch.equal(slot.cpu(), slot_h)
    # merge of the packed records (as if received), twice: the second step
    # starts from the store clock the first one left
    info = torch.tensor([[m // world, int(ts.min()), int(ts.max()) + r * 100_000_000, 0] for r in range(world)],
                        dtype=torch.int64)
    for step in range(2):
        outs = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(3)] + \
               [torch.empty(m, dtype=torch.int32, device="cuda"), torch.empty(m, dtype=torch.int64, device="cuda"),
                torch.empty(m, dtype=torch.int32, device="cuda")]
        info_d = info.cuda()
        r.merge(m, send.data_ptr(), info_d.data_ptr(), info.data_ptr(), *[x.data_ptr() for x in outs], s)
        outs_h = [torch.empty(m, dtype=torch.int64) for _ in range(3)] + \
                 [torch.empty(m, dtype=torch.int32), torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=torch.int32)]
        ops.merge(m, send_h.data_ptr(), info.data_ptr(), info.data_ptr(), *[x.data_ptr() for x in outs_h], None)
        assert r.sync(s) == rl.RL_OK
        for a, b in zip(outs, outs_h):
            assert torch.equal(a.cpu(), b)
    # results + unpack
    dec = torch.from_numpy(rng.integers(0, 4, m).astype(np.uint8))
    rem, retry, reset = [torch.from_numpy(rng.integers(-5, 1 << 40, m).astype(np.int64)) for _ in range(3)]
    res = torch.empty((m, 4), dtype=torch.int64, device="cuda")
    dd = [x.cuda() for x in (dec, rem, retry, reset)]
    r.results(m, outs[5].data_ptr(), *[x.data_ptr() for x in dd], res.data_ptr(), s)
    res_h = torch.empty((m, 4), dtype=torch.int64)
    ops.results(m, outs_h[5].data_ptr(), *[x.data_ptr() for x in (dec, rem, retry, reset)], res_h.data_ptr(), None)
    back = [torch.empty(m, dtype=torch.uint8, device="cuda")] + [torch.empty(m, dtype=torch.int64, device="cuda")
                                                                 for _ in range(3)]
    r.unpack(m, slot.data_ptr(), res.data_ptr(), *[x.data_ptr() for x in back], s)
    back_h = [torch.empty(m, dtype=torch.uint8)] + [torch.empty(m, dtype=torch.int64) for _ in range(3)]
    ops.unpack(m, slot_h.data_ptr(), res_h.data_ptr(), *[x.data_ptr() for x in back_h], None)
    torch.cuda.synchronize()
    assert torch.equal(res.cpu(), res_h)
    for a, b in zip(back, back_h):
        assert torch.equal(a.cpu(), b)
    r.close()


def test_merge_single_sorted_source_keeps_order(rl):
    """one source whose batch is in time order: no sort, the received order
    is the decision order (and the store clock still advances)"""
    import torch

    import route_ops
    m = 9000
    rng = np.random.default_rng(4)
    ts = T0 + np.cumsum(rng.integers(0, 5000, m)).astype(np.int64)
    rec = np.stack([rng.integers(0, 1 << 62, m), ts, np.ones(m, np.int64), np.arange(m, dtype=np.int64) << 32], 1)
    info = np.array([[m, ts.min(), ts.max(), 1]], np.int64)
    r = rl.Router(0, 1, m, m)
    ops = route_ops.NumpyRouteOps(1)
    s = torch.cuda.current_stream().cuda_stream
    for step in range(2):
        d = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(3)] + \
            [torch.empty(m, dtype=torch.int32, device="cuda"), torch.empty(m, dtype=torch.int64, device="cuda"),
             torch.empty(m, dtype=torch.int32, device="cuda")]
        h = [torch.empty(m, dtype=torch.int64) for _ in range(3)] + \
            [torch.empty(m, dtype=torch.int32), torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=torch.int32)]
        rt, it = torch.from_numpy(rec).cuda(), torch.from_numpy(info).cuda()
        r.merge(m, rt.data_ptr(), it.data_ptr(), torch.from_numpy(info).data_ptr(), *[x.data_ptr() for x in d], s)
        rh, ih = torch.from_numpy(rec), torch.from_numpy(info)
        ops.merge(m, rh.data_ptr(), ih.data_ptr(), ih.data_ptr(), *[x.data_ptr() for x in h], None)
        assert r.sync(s) == rl.RL_OK
        for a, b in zip(d, h):
            assert torch.equal(a.cpu(), b)
        assert np.array_equal(d[5].cpu().numpy(), np.arange(m))
    r.close()


def test_merge_planned_on_the_device_one_source(rl):
    """world 1 without host rows (rl_route_merge(..., NULL, ...)): per-tile
    maxima, one scan block that advances the store clock in device memory, one
    gather -- the same outputs as the restatement over three steps, batches
    out of time order and one step whose times go back below the clock; a
    host-planned merge on that router is then refused"""
    import torch

    import route_ops
    m = 25_000
    rng = np.random.default_rng(17)
    r = rl.Router(0, 1, m, m)
    ops = route_ops.NumpyRouteOps(1)
    s = torch.cuda.current_stream().cuda_stream
    base = [T0, T0 + 4_000_000_000, T0 + 1_000_000_000]      # step 3 goes back in time
    for step in range(3):
        ts = base[step] + rng.integers(0, 3_000_000_000, m).astype(np.int64)   # unsorted, 3 s span
        rec = np.stack([rng.integers(0, 1 << 62, m), ts, rng.integers(1, 4, m), np.arange(m, dtype=np.int64) << 32],
                       1)
        info = np.array([[m, ts.min(), ts.max(), 0]], np.int64)
        d = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(3)] + \
            [torch.empty(m, dtype=torch.int32, device="cuda"), torch.empty(m, dtype=torch.int64, device="cuda"),
             torch.empty(m, dtype=torch.int32, device="cuda")]
        h = [torch.empty(m, dtype=torch.int64) for _ in range(3)] + \
            [torch.empty(m, dtype=torch.int32), torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=torch.int32)]
        rt, it = torch.from_numpy(rec).cuda(), torch.from_numpy(info).cuda()
        r.merge(m, rt.data_ptr(), it.data_ptr(), None, *[x.data_ptr() for x in d], s)
        rh, ih = torch.from_numpy(rec), torch.from_numpy(info)
        ops.merge(m, rh.data_ptr(), ih.data_ptr(), ih.data_ptr(), *[x.data_ptr() for x in h], None)
        assert r.sync(s) == rl.RL_OK
        for a, b in zip(d, h):
            assert torch.equal(a.cpu(), b)
    with pytest.raises(rl.EngineError):
        r.merge(m, rt.data_ptr(), it.data_ptr(), torch.from_numpy(info).data_ptr(), *[x.data_ptr() for x in d], s)
    r.close()


@pytest.mark.parametrize("span_bits", [33, 41])
def test_merge_wide_time_spans_and_unsorted_sources(rl, span_bits):
    """received times spanning more than 2^32 ns (five and six sort passes),
    three sources out of time order: arrival order against the restatement"""
    import torch

    import route_ops
    world = 3
    m = 30_000
    rng = np.random.default_rng(span_bits)
    ts = T0 + rng.integers(0, 1 << span_bits, m).astype(np.int64)
    rec = np.stack([rng.integers(0, 1 << 62, m), ts, np.ones(m, np.int64), np.arange(m, dtype=np.int64) << 32], 1)
    cnt = [10_000, 12_000, 8_000]
    info = np.array([[c, T0, T0 + (1 << span_bits), 0] for c in cnt], np.int64)
    info[:, 1] = [ts[:10_000].min(), ts[10_000:22_000].min(), ts[22_000:].min()]
    info[:, 2] = [ts[:10_000].max(), ts[10_000:22_000].max(), ts[22_000:].max()]
    r = rl.Router(0, world, m, m)
    ops = route_ops.NumpyRouteOps(world)
    s = torch.cuda.current_stream().cuda_stream
    d = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(3)] + \
        [torch.empty(m, dtype=torch.int32, device="cuda"), torch.empty(m, dtype=torch.int64, device="cuda"),
         torch.empty(m, dtype=torch.int32, device="cuda")]
    h = [torch.empty(m, dtype=torch.int64) for _ in range(3)] + \
        [torch.empty(m, dtype=torch.int32), torch.empty(m, dtype=torch.int64), torch.empty(m, dtype=torch.int32)]
    rt, it = torch.from_numpy(rec).cuda(), torch.from_numpy(info).cuda()
    r.merge(m, rt.data_ptr(), it.data_ptr(), torch.from_numpy(info).data_ptr(), *[x.data_ptr() for x in d], s)
    rh, ih = torch.from_numpy(rec), torch.from_numpy(info)
    ops.merge(m, rh.data_ptr(), ih.data_ptr(), ih.data_ptr(), *[x.data_ptr() for x in h], None)
    assert r.sync(s) == rl.RL_OK
    for a, b in zip(d, h):
        assert torch.equal(a.cpu(), b)
    r.close()


def test_merge_reports_a_too_wide_time_span(rl):
    import torch
    m = 5000
    r = rl.Router(0, 2, m, m)
    rec = torch.zeros((m, 4), dtype=torch.int64, device="cuda")
    rec[:, 1] = T0
    rec[7, 1] = T0 + (1 << 49)
    outs = [torch.empty(m, dtype=torch.int64, device="cuda") for _ in range(3)] + \
           [torch.empty(m, dtype=torch.int32, device="cuda"), torch.empty(m, dtype=torch.int64, device="cuda"),
            torch.empty(m, dtype=torch.int32, device="cuda")]
    s = torch.cuda.current_stream().cuda_stream
    info_h = torch.tensor([[m - 100, T0, T0 + (1 << 49), 0], [100, T0, T0, 1]], dtype=torch.int64)
    info = info_h.cuda()
    r.merge(m, rec.data_ptr(), info.data_ptr(), info_h.data_ptr(), *[x.data_ptr() for x in outs], s)
    assert r.sync(s) == rl.RL_EINVAL
    r.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _routed_rank(rank, world, port, backend, batches_of, q):
    """one rank of the native routed path on cuda:0: Router kernels, the HIP
    engine as owner, all-to-alls over `backend` (nccl: RCCL; gloo: through
    host memory, for two ranks sharing the box's one GPU)"""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "distributed-rate-limiter_amd", "python"), os.path.join(root, "tests")]
    import torch
    import torch.distributed as dist

    import route_ops
    import rl_amd
    import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    ok = False
    try:
        all_batches = [batches_of(r) for r in range(world)]
        mine = all_batches[rank]
        mb = max(b[0].size for b in mine)
        eng = rl_amd.Engine(profile=0, tb_capacity=1 << 20, win_capacity=1 << 20, max_batch=world * mb)
        for a, L, W in CONFIGS:
            eng.register(a, L, W)

        def decide(m, key, ts, n, cfg, sms, dec, rem, retry, reset, stream):
            eng.decide_device(m, key, ts, n, cfg, sms, dec, rem, retry, reset, None, stream)

        router = rl_amd.Router(0, world, mb, world * mb)
        pg_res = dist.new_group(backend=backend)
        pipe = shard.RoutedPipeline(router, decide, world, mb, "cuda:0", pg_req=None, pg_res=pg_res,
                                    staged=backend == "gloo")
        ins = [tuple(_dev_tensors(torch, *bt)) for bt in mine]
        outs = [(torch.empty(b[0].size, dtype=torch.uint8, device="cuda"),) +
                tuple(torch.empty(b[0].size, dtype=torch.int64, device="cuda") for _ in range(3)) for b in mine]
        torch.cuda.synchronize()
        pipe.run(ins, outs)
        torch.cuda.synchronize()
        assert eng.sync() == rl_amd.RL_OK, eng.last_error()
        assert router.sync(None) == rl_amd.RL_OK
        exp = route_ops.shared_limiter_expectations(all_batches, rank, CONFIGS)
        ok = True
        for b, (ob, eb) in enumerate(zip(outs, exp)):
            for f, (o, e) in enumerate(zip(ob, eb)):
                g, e = o.cpu().numpy().astype(np.int64), np.asarray(e, np.int64)
                bad = np.nonzero(g != e)[0]
                if bad.size:
                    ok = False
                    print(f"rank {rank} batch {b} field {f}: {bad.size} mismatches, first {bad[:5]} "
                          f"got {g[bad[:5]]} exp {e[bad[:5]]} keys {mine[b][0][bad[:5]]}", flush=True)
        eng.close()
        router.close()
    finally:
        q.put((rank, ok))
        dist.destroy_process_group()


def mixed_batches(rank, nbatch=4, m=150_000, nkeys=300_000):
    """configs[3]-shaped: cfg = key mod (configs), keys uniform, each rank one
    app server (own clock, skewed), several steps"""
    import test_distributed
    rng = np.random.default_rng(700 + rank)
    t = T0 + [0, -1_500_000_000][rank % 2]
    out = []
    for _ in range(nbatch):
        key = rng.integers(0, nkeys, m).astype(np.uint64)
        key[rng.random(m) < 0.2] = rng.integers(0, 40)      # hot keys shared by all ranks
        ts = t + np.cumsum(rng.choice([0, 1, 1000, 30_000], m)).astype(np.int64)
        t = int(ts[-1]) + 1
        n = rng.choice([1, 1, 2, 5], m).astype(np.int64)
        out.append((key, ts, n, (key % len(test_distributed.CONFIGS)).astype(np.uint32)))
    return out


def _spawn(world, backend, batches_of):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_routed_rank, args=(r, world, port, backend, batches_of, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


def test_routed_path_one_rank_rccl():
    """world size 1 over RCCL: the full native routed path (pack, count and
    record all-to-alls, time-order merge, engine, result all-to-all, unpack)"""
    assert _spawn(1, "nccl", mixed_batches) == {0: True}


def test_routed_path_two_ranks_one_gpu():
    """two ranks (two engines, two routers) on the box's one GPU; the
    all-to-alls go through host memory (gloo), the kernels are the GPU's"""
    assert _spawn(2, "gloo", mixed_batches) == {0: True, 1: True}


def skewed_batches(rank, nbatch=3, m=60_000, nkeys=20_000):
    """app servers with skewed clocks (tracegen.skewed_trace): every batch out
    of time order, spans of minutes (five sort passes), per-key time going
    back by windows"""
    import tracegen
    k, ts, n, cfg, _ = tracegen.skewed_trace(900 + rank, nbatch * m, nkeys, CONFIGS)
    return [(k[b * m:(b + 1) * m], ts[b * m:(b + 1) * m], n[b * m:(b + 1) * m], cfg[b * m:(b + 1) * m])
            for b in range(nbatch)]


def test_routed_path_one_rank_unsorted_batches():
    """world size 1 with batches out of time order: the routed path applies a
    rank's requests in its own order (as rl_decide_batch_device does), with
    the store clock at each request's arrival (the running max of ts)"""
    assert _spawn(1, "nccl", skewed_batches) == {0: True}


def test_routed_path_two_ranks_unsorted_batches():
    assert _spawn(2, "gloo", skewed_batches) == {0: True, 1: True}
