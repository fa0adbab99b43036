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


def _host(torch, *arrays):
    return [torch.from_numpy(np.ascontiguousarray(x.view(np.int64) if x.dtype == np.uint64 else
                                                  (x.view(np.int32) if x.dtype == np.uint32 else x)))
            for x in arrays]


@pytest.mark.parametrize("world,cap", [(1, 70_001), (2, 40_000), (3, 20_000), (8, 9_000), (8, 4096), (2, 30_000)])
def test_route_pack_matches_restatement(rl, world, cap):
    """owner buckets, info rows and slots; the last three cases overflow
    their buckets (dropped requests: slot UINT32_MAX, RL_EOVERFLOW)"""
    import torch

    import route_ops
    import shard
    rng = np.random.default_rng(40 + world)
    m = 70_001
    key = rng.integers(0, 1 << 63, m).astype(np.uint64)
    ts = T0 + rng.integers(0, 3_000_000_000, m).astype(np.int64)      # unsorted, 3 s span
    ts[rng.random(m) < 0.2] = T0 + 12345                              # many equal times
    n = rng.integers(1, 9, m).astype(np.int64)
    cfg = rng.integers(0, 15, m).astype(np.uint32)
    r = rl.Router(0, world, m, cap)
    ops = route_ops.NumpyRouteOps(world, cap)
    assert r.capacity == ops.capacity and r.capacity % 2048 == 0
    C = r.capacity
    k, t, nn, c = _dev_tensors(torch, key, ts, n, cfg)
    send = torch.empty((world * C, 4), dtype=torch.int64, device="cuda")
    scnt = torch.empty((world, 4), dtype=torch.int64, device="cuda")
    slot = torch.empty(m, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    r.pack(m, k.data_ptr(), t.data_ptr(), nn.data_ptr(), c.data_ptr(), send.data_ptr(), scnt.data_ptr(),
           slot.data_ptr(), s)
    own = torch.empty(m, dtype=torch.int32, device="cuda")
    r.owner(m, k.data_ptr(), own.data_ptr(), s)
    kc, tc, nc, cc = _host(torch, key, ts, n, cfg)
    send_h = torch.zeros((world * C, 4), dtype=torch.int64)
    scnt_h = torch.empty((world, 4), dtype=torch.int64)
    slot_h = torch.empty(m, dtype=torch.int32)
    ops.pack(m, kc.data_ptr(), tc.data_ptr(), nc.data_ptr(), cc.data_ptr(), send_h.data_ptr(), scnt_h.data_ptr(),
             slot_h.data_ptr(), None)
    torch.cuda.synchronize()
    assert np.array_equal(own.cpu().numpy(), shard.owner_of(key, world))
    assert torch.equal(scnt.cpu(), scnt_h) and torch.equal(slot.cpu(), slot_h)
    sd = send.cpu()
    for o in range(world):
        c_o = int(scnt_h[o, 0])
        assert torch.equal(sd[o * C:o * C + c_o], send_h[o * C:o * C + c_o])
    dropped = int((scnt_h[:, 3] >> 1).sum())   # row 3: 2 * dropped + unsorted
    assert (dropped > 0) == ops.overflow
    assert r.sync(s) == (rl.RL_EOVERFLOW if dropped else rl.RL_OK)
    assert r.sync(s) == rl.RL_OK        # sticky until read, then cleared
    r.close()


@pytest.mark.parametrize("world", [1, 3, 8])
def test_route_pack_repeated_calls(rl, world):
    """one router, many packs of varying sizes (empty, under one tile, ragged,
    many tiles, sorted and unsorted): the one-pass pack's look-back words and
    accumulators carry nothing from one call to the next"""
    import torch

    import route_ops
    rng = np.random.default_rng(77 + world)
    M = 50_000
    cap = 12_000
    r = rl.Router(0, world, M, cap)
    C = r.capacity
    s = torch.cuda.current_stream().cuda_stream
    for m in [5000, 0, 1, 1023, 1024, 1025, M, 3, 40_000, 777, M]:
        ops = route_ops.NumpyRouteOps(world, cap)
        key = rng.integers(0, 1 << 63, m).astype(np.uint64)
        ts = T0 + rng.integers(0, 2_000_000_000, m).astype(np.int64)
        if m % 2:
            ts.sort()
        n = rng.integers(1, 9, m).astype(np.int64)
        cfg = rng.integers(0, 15, m).astype(np.uint32)
        k, t, nn, c = _dev_tensors(torch, key, ts, n, cfg) if m else [torch.empty(1, dtype=torch.int64,
                                                                                  device="cuda")] * 4
        send = torch.empty((world * C, 4), dtype=torch.int64, device="cuda")
        scnt = torch.full((world, 4), -7, dtype=torch.int64, device="cuda")
        slot = torch.empty(max(m, 1), dtype=torch.int32, device="cuda")
        r.pack(m, k.data_ptr(), t.data_ptr(), nn.data_ptr(), c.data_ptr(), send.data_ptr(), scnt.data_ptr(),
               slot.data_ptr(), s)
        kc, tc, nc, cc = _host(torch, key, ts, n, cfg)
        send_h = torch.zeros((world * C, 4), dtype=torch.int64)
        scnt_h = torch.empty((world, 4), dtype=torch.int64)
        slot_h = torch.empty(max(m, 1), dtype=torch.int32)
        ops.pack(m, kc.data_ptr(), tc.data_ptr(), nc.data_ptr(), cc.data_ptr(), send_h.data_ptr(),
                 scnt_h.data_ptr(), slot_h.data_ptr(), None)
        torch.cuda.synchronize()
        assert torch.equal(scnt.cpu(), scnt_h), m
        assert torch.equal(slot.cpu()[:m], slot_h[:m]), m
        sd = send.cpu()
        for o in range(world):
            c_o = int(scnt_h[o, 0])
            assert torch.equal(sd[o * C:o * C + c_o], send_h[o * C:o * C + c_o]), (m, o)
        dropped = int((scnt_h[:, 3] >> 1).sum())
        assert r.sync(s) == (rl.RL_EOVERFLOW if dropped else rl.RL_OK), m
    r.close()


def _merge_case(rng, world, C, counts, span, step_base):
    """received buckets: source q's counts[q] records, times out of order in
    the even sources (flagged in the info row) and sorted in the odd ones,
    with ties across sources"""
    recv = np.zeros((world * C, 4), np.int64)
    info = np.zeros((world, 4), np.int64)
    for q in range(world):
        c = counts[q]
        ts = step_base + rng.integers(0, span, c).astype(np.int64)
        ts[rng.random(c) < 0.1] = step_base + 777_000                   # ties across sources
        recv[q * C:q * C + c] = np.stack([rng.integers(0, 1 << 62, c), ts, rng.integers(1, 4, c),
                                          np.arange(c, dtype=np.int64) << 32], 1)
        if q % 2 and c:                                                 # odd sources: in time order
            ts = np.sort(ts)
            recv[q * C:q * C + c, 1] = ts
        unsorted = int(c > 1 and bool(np.any(ts[1:] < ts[:-1])))
        info[q] = [c, ts.min() if c else (1 << 63) - 1, ts.max() if c else -(1 << 63), unsorted]
    return recv, info


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_route_merge_matches_restatement(rl, world):
    """the device-planned merge over three steps (the store clock carried in
    device memory; step 3's times go back below it): decision order, store
    clocks and received count against the restatement; empty and full
    buckets, sources out of time order, equal times across sources"""
    import torch

    import route_ops
    rng = np.random.default_rng(17 + world)
    cap = 9000
    r = rl.Router(0, world, 4096, cap)
    ops = route_ops.NumpyRouteOps(world, cap)
    C = r.capacity
    s = torch.cuda.current_stream().cuda_stream
    base = [T0, T0 + 4_000_000_000, T0 + 1_000_000_000]
    for step in range(3):
        counts = rng.integers(0, C + 1, world)
        counts[rng.integers(world)] = C if world > 1 else counts[0]
        if world > 2:
            counts[rng.integers(world)] = 0
        recv, info = _merge_case(rng, world, C, counts, 3_000_000_000, base[step])
        rt, it = torch.from_numpy(recv).cuda(), torch.from_numpy(info).cuda()
        order = torch.full((world * C,), -7, dtype=torch.int32, device="cuda")
        sms = torch.empty(world * C, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        r.merge(rt.data_ptr(), it.data_ptr(), order.data_ptr(), sms.data_ptr(), cnt.data_ptr(), s)
        rh, ih = torch.from_numpy(recv), torch.from_numpy(info)
        order_h = torch.empty(world * C, dtype=torch.int32)
        sms_h = torch.empty(world * C, dtype=torch.int64)
        cnt_h = torch.zeros(1, dtype=torch.int32)
        ops.merge(rh.data_ptr(), ih.data_ptr(), order_h.data_ptr(), sms_h.data_ptr(), cnt_h.data_ptr(), None)
        assert r.sync(s) == rl.RL_OK
        tot = int(counts.sum())
        assert int(cnt.cpu()[0]) == int(cnt_h[0]) == tot
        assert torch.equal(order.cpu()[:tot], order_h[:tot])
        assert torch.equal(sms.cpu()[:tot], sms_h[:tot])
    r.close()


def test_route_merge_one_source_in_order_is_identity(rl):
    """world 1, batches in time order: the merge writes only the identity
    marker (RL_ORDER_IDENTITY) and the earlier steps' clock, and that form
    expands to the restatement's order and store clocks; an out-of-order
    batch in between gets the full order"""
    import torch

    import route_ops
    rng = np.random.default_rng(23)
    r = rl.Router(0, 1, 4096, 4096)
    ops = route_ops.NumpyRouteOps(1, 4096)
    C = r.capacity
    s = torch.cuda.current_stream().cuda_stream
    for step, (c, in_order) in enumerate([(3000, True), (C, False), (C, True), (0, True), (17, True)]):
        ts = T0 + step * 2_000_000_000 + rng.integers(0, 3_000_000_000, c).astype(np.int64)
        if in_order:
            ts = np.sort(ts)
        if step == 2:
            ts = np.minimum(ts, T0)            # times back below the store clock
        recv = np.zeros((C, 4), np.int64)
        recv[:c] = np.stack([rng.integers(0, 1 << 62, c), ts, np.ones(c, np.int64),
                             np.arange(c, dtype=np.int64) << 32], 1)
        unsorted = int(c > 1 and bool(np.any(ts[1:] < ts[:-1])))
        info = np.array([[c, ts.min() if c else (1 << 63) - 1, ts.max() if c else -(1 << 63), unsorted]], np.int64)
        order = torch.full((C,), -7, dtype=torch.int32, device="cuda")
        sms = torch.empty(C, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        r.merge(torch.from_numpy(recv).cuda().data_ptr(), torch.from_numpy(info).cuda().data_ptr(),
                order.data_ptr(), sms.data_ptr(), cnt.data_ptr(), s)
        order_h = torch.empty(C, dtype=torch.int32)
        sms_h = torch.empty(C, dtype=torch.int64)
        cnt_h = torch.zeros(1, dtype=torch.int32)
        ops.merge(torch.from_numpy(recv).data_ptr(), torch.from_numpy(info).data_ptr(), order_h.data_ptr(),
                  sms_h.data_ptr(), cnt_h.data_ptr(), None)
        assert r.sync(s) == rl.RL_OK
        assert int(cnt.cpu()[0]) == int(cnt_h[0]) == c
        o, sm = order.cpu(), sms.cpu()
        if in_order:
            assert int(o[0]) == -1                       # RL_ORDER_IDENTITY as int32
            o = torch.arange(C, dtype=torch.int32)
            sm = torch.maximum(torch.from_numpy(recv[:, 1] // 1_000_000), sm[0])
        else:
            assert int(o[0]) != -1
        assert torch.equal(o[:c], order_h[:c])
        assert torch.equal(sm[:c], sms_h[:c])
    r.close()


@pytest.mark.parametrize("m,shift", [(20_000, 0), (20_003, 0), (20_001, 1)])
def test_route_unpack_dropped_and_kept(rl, m, shift):
    """dropped and kept requests, odd batch sizes and unaligned outputs
    (shift: every array one element in)"""
    import torch

    import route_ops
    rng = np.random.default_rng(5 + m)
    world, cap = 3, 4096
    r = rl.Router(0, world, m, cap)
    C = r.capacity
    slot = rng.integers(0, world * C, m).astype(np.int32)
    slot[rng.random(m) < 0.1] = -1
    back = rng.integers(-5, 1 << 40, (world * C, 4)).astype(np.int64)
    back[:, 0] = rng.integers(0, 4, world * C)
    st, bt = torch.from_numpy(slot).cuda(), torch.from_numpy(back).cuda()
    full = [torch.empty(m + shift, dtype=torch.uint8, device="cuda")] + \
        [torch.empty(m + shift, dtype=torch.int64, device="cuda") for _ in range(3)]
    outs = [x[shift:] for x in full]
    r.unpack(m, st.data_ptr(), bt.data_ptr(), *[x.data_ptr() for x in outs], torch.cuda.current_stream().cuda_stream)
    ops = route_ops.NumpyRouteOps(world, cap)
    outs_h = [torch.empty(m, dtype=torch.uint8)] + [torch.empty(m, dtype=torch.int64) for _ in range(3)]
    sh, bh = torch.from_numpy(slot), torch.from_numpy(back)
    ops.unpack(m, sh.data_ptr(), bh.data_ptr(), *[x.data_ptr() for x in outs_h], None)
    torch.cuda.synchronize()
    for a, b in zip(outs, outs_h):
        assert torch.equal(a.cpu(), b)
    assert int((outs_h[0] == rl.DROPPED).sum()) >= int((slot == -1).sum())
    r.close()


def test_route_dropped_request_advances_store_clock(rl):
    """a request dropped at the sender (bucket overflow) still advances the
    store clock to its time (include/rl_route.h): the shared store's clock is
    the real time any app server has reached, sent or not -- so the next
    step's requests expire keys at max(their time, the dropped request's)"""
    import torch
    rng = np.random.default_rng(31)
    m = 3000
    r = rl.Router(0, 1, m, 2048)
    C = r.capacity
    assert C < m
    s = torch.cuda.current_stream().cuda_stream
    late = T0 + 50_000_000_000                                   # the last request, 50 s later: dropped
    ts1 = np.sort(T0 + rng.integers(0, 1_000_000_000, m).astype(np.int64))
    ts1[-1] = late
    ts2 = np.sort(T0 + 2_000_000_000 + rng.integers(0, 1_000_000_000, 100).astype(np.int64))
    for step, ts in enumerate([ts1, ts2]):
        k = rng.integers(0, 1 << 62, ts.size).astype(np.uint64)
        kt, tt, nt, ct = _dev_tensors(torch, k, ts, np.ones(ts.size, np.int64), np.zeros(ts.size, np.uint32))
        send = torch.empty((C, 4), dtype=torch.int64, device="cuda")
        info = torch.empty((1, 4), dtype=torch.int64, device="cuda")
        slot = torch.empty(ts.size, dtype=torch.int32, device="cuda")
        r.pack(ts.size, kt.data_ptr(), tt.data_ptr(), nt.data_ptr(), ct.data_ptr(), send.data_ptr(),
               info.data_ptr(), slot.data_ptr(), s)
        order = torch.empty(C, dtype=torch.int32, device="cuda")
        sms = torch.empty(C, dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        r.merge(send.data_ptr(), info.data_ptr(), order.data_ptr(), sms.data_ptr(), cnt.data_ptr(), s)
        torch.cuda.synchronize()
        if step == 0:
            assert int(info.cpu()[0, 2]) == late and int(slot.cpu()[-1]) == -1
            assert r.sync(s) == rl.RL_EOVERFLOW
        else:
            assert int(order.cpu()[0]) == -1                      # identity form: sms[0] = earlier steps' clock
            assert int(sms.cpu()[0]) == late // 1_000_000
            assert r.sync(s) == rl.RL_OK
    r.close()


def test_routed_count_above_m_max_is_reported(rl):
    """rl_decide_routed_device with m_max below the merged count decides only
    the first m_max requests and says so: rl_engine_sync -> RL_EOVERFLOW"""
    import torch
    rng = np.random.default_rng(32)
    m = 4096
    r = rl.Router(0, 1, m, m)
    C = r.capacity
    eng = rl.Engine(profile=0, tb_capacity=1 << 14, win_capacity=1 << 12, max_batch=C)
    for a, L, W in CONFIGS:
        eng.register(a, L, W)
    s = torch.cuda.current_stream().cuda_stream
    ts = np.sort(T0 + rng.integers(0, 1_000_000_000, m).astype(np.int64))
    k = rng.integers(0, 1000, m).astype(np.uint64)
    kt, tt, nt, ct = _dev_tensors(torch, k, ts, np.ones(m, np.int64), (k % len(CONFIGS)).astype(np.uint32))
    send = torch.empty((C, 4), dtype=torch.int64, device="cuda")
    info = torch.empty((1, 4), dtype=torch.int64, device="cuda")
    slot = torch.empty(m, dtype=torch.int32, device="cuda")
    r.pack(m, kt.data_ptr(), tt.data_ptr(), nt.data_ptr(), ct.data_ptr(), send.data_ptr(), info.data_ptr(),
           slot.data_ptr(), s)
    order = torch.empty(C, dtype=torch.int32, device="cuda")
    sms = torch.empty(C, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    res = torch.zeros((C, 4), dtype=torch.int64, device="cuda")
    r.merge(send.data_ptr(), info.data_ptr(), order.data_ptr(), sms.data_ptr(), cnt.data_ptr(), s)
    eng.decide_routed(m // 2, cnt.data_ptr(), send.data_ptr(), order.data_ptr(), sms.data_ptr(), res.data_ptr(), s, s)
    torch.cuda.synchronize()
    assert int(cnt.cpu()[0]) == m
    assert eng.sync() == rl.RL_EOVERFLOW
    assert eng.sync() == rl.RL_OK                                  # reported once, then cleared
    eng.close()
    r.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _routed_rank(rank, world, port, backend, batches_of, q, exchange=None, cap=None, configs=None, profile=0):
    """one rank of the native routed path on cuda:0: Router kernels, the HIP
    engine as owner (rl_decide_routed_device), equal-split all-to-alls over
    `backend` (nccl: RCCL; gloo: through host memory, for two ranks sharing
    the box's one GPU)"""
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
    info = {}
    try:
        all_batches = [batches_of(r) for r in range(world)]
        mine = all_batches[rank]
        mb = max(b[0].size for b in mine)
        router = rl_amd.Router(0, world, mb, cap or mb)
        eng = rl_amd.Engine(profile=profile, tb_capacity=1 << 20, win_capacity=1 << 20,
                            max_batch=world * router.capacity)
        configs = configs or CONFIGS
        for a, L, W in configs:
            eng.register(a, L, W)
        pg_res = dist.new_group(backend=backend)
        pipe = shard.RoutedPipeline(router, eng.decide_routed, world, mb, "cuda:0", pg_req=None, pg_res=pg_res,
                                    exchange=exchange, staged=backend == "gloo", decide_ev=eng.decide_routed_ev)
        ins = [tuple(_dev_tensors(torch, *bt)) for bt in mine]
        outs = [(torch.empty(b[0].size, dtype=torch.uint8, device="cuda"),) +
                tuple(torch.empty(b[0].size, dtype=torch.int64, device="cuda") for _ in range(3)) for b in mine]
        torch.cuda.synchronize()
        pipe.run(ins, outs)
        torch.cuda.synchronize()
        assert eng.sync() == rl_amd.RL_OK, eng.last_error()
        info["router_status"] = router.sync(None)
        info["collectives"] = pipe.collectives
        info["exchange"] = pipe.exchange
        exp = route_ops.shared_limiter_expectations(all_batches, rank, configs, profile=profile,
                                                    cap=router.capacity)
        ok = True
        for b, (ob, eb) in enumerate(zip(outs, exp)):
            for f, (o, e) in enumerate(zip(ob, eb)):
                g, e = o.cpu().numpy().astype(np.int64), np.asarray(e, np.int64)
                bad = np.nonzero(g != e)[0]
                if bad.size:
                    ok = False
                    print(f"rank {rank} batch {b} field {f}: {bad.size} mismatches, first {bad[:5]} "
                          f"got {g[bad[:5]]} exp {e[bad[:5]]} keys {mine[b][0][bad[:5]]}", flush=True)
        info["dropped"] = int(sum((o[0].cpu().numpy() == rl_amd.DROPPED).sum() for o in outs))
        del pipe
        eng.close()
        router.close()
    finally:
        q.put((rank, ok, info))
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


def _spawn(world, backend, batches_of, **kw):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_routed_rank, args=(r, world, port, backend, batches_of, q), kwargs=kw)
             for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (ok, info) for r, ok, info in (q.get(timeout=240) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
    return res


def _check(res, world, nbatch, exchange, dropped=False):
    for r in range(world):
        ok, info = res[r]
        assert ok, (r, info)
        assert info["exchange"] == exchange
        # three equal-split collectives per step (info rows, request buckets,
        # result buckets), or none at all
        assert info["collectives"] == (3 * nbatch if exchange else 0), info
        assert (info["dropped"] > 0) == dropped
        assert info["router_status"] == (-75 if dropped else 0), info


def test_routed_path_one_rank_rccl():
    """world size 1 with the exchange forced on: the full native routed path
    over RCCL -- pack, loopback all-to-alls of the info rows and of the
    request buckets, device-planned merge, the engine on the received records,
    result all-to-all, unpack -- with device tensors"""
    _check(_spawn(1, "nccl", mixed_batches, exchange=True), 1, 4, True)


def test_routed_path_one_rank_local():
    """world size 1 without the exchange: buckets and results read in place"""
    _check(_spawn(1, "nccl", mixed_batches), 1, 4, False)


def test_routed_path_two_ranks_one_gpu():
    """two ranks (two engines, two routers) on the box's one GPU; the
    all-to-alls go through host memory (gloo), the kernels are the GPU's"""
    _check(_spawn(2, "gloo", mixed_batches), 2, 4, True)


def test_routed_path_two_ranks_bucket_overflow():
    """buckets smaller than a rank's requests for one owner: the requests past
    the capacity come back RL_DROPPED, were never applied, and every other
    decision equals the shared limiter without them; the router reports
    RL_EOVERFLOW"""
    _check(_spawn(2, "gloo", mixed_batches, cap=60_000), 2, 4, True, dropped=True)


def skewed_batches(rank, nbatch=3, m=60_000, nkeys=20_000):
    """app servers with skewed clocks (tracegen.skewed_trace): every batch out
    of time order, spans of minutes, per-key time going back by windows"""
    import tracegen
    k, ts, n, cfg, _ = tracegen.skewed_trace(900 + rank, nbatch * m, nkeys, CONFIGS)
    return [(k[b * m:(b + 1) * m], ts[b * m:(b + 1) * m], n[b * m:(b + 1) * m], cfg[b * m:(b + 1) * m])
            for b in range(nbatch)]


def test_routed_path_one_rank_unsorted_batches():
    """world size 1 over RCCL (exchange forced on) with batches out of time
    order: the routed path applies a rank's requests in its own order (as
    rl_decide_batch_device does), with the store clock at each request's
    arrival (the running max of ts)"""
    _check(_spawn(1, "nccl", skewed_batches, exchange=True), 1, 3, True)


def test_routed_path_two_ranks_unsorted_batches():
    _check(_spawn(2, "gloo", skewed_batches), 2, 3, True)


LONG_SEED = 1500


def long_window_batches(rank, nbatch=3, world=2):
    """one long-window trace (tracegen.long_window_trace: 1-365 d windows,
    L = 1, three hot keys, phase jumps of up to 400 days) dealt to the ranks
    request by request, so the ranks' clocks interleave; each rank's share in
    nbatch steps"""
    import tracegen
    _, (k, ts, n, cfg, _) = tracegen.long_window_trace(LONG_SEED, 0, 180_000, wi=0)
    k, ts, n, cfg = (x[rank::world] for x in (k, ts, n, cfg))
    m = k.size // nbatch
    return [(k[b * m:(b + 1) * m], ts[b * m:(b + 1) * m], n[b * m:(b + 1) * m], cfg[b * m:(b + 1) * m])
            for b in range(nbatch)]


def _long_configs():
    import tracegen
    return tracegen.long_window_trace(LONG_SEED, 0, 10, wi=0)[0]


@pytest.mark.parametrize("profile", [0, 1])
def test_routed_path_one_rank_long_windows(profile):
    """world size 1 over RCCL (exchange forced on) with reference-legal long
    windows (config.go:41-46): the store clock carries years of phase jumps
    through the merge and the engine's explicit-clock records"""
    import functools
    _check(_spawn(1, "nccl", functools.partial(long_window_batches, world=1), exchange=True,
                  configs=_long_configs(), profile=profile), 1, 3, True)


def test_routed_path_two_ranks_long_windows():
    _check(_spawn(2, "gloo", long_window_batches, configs=_long_configs(), profile=1), 2, 3, True)
