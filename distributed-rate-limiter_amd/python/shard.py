"""Key-space sharding across GPUs (one process per GPU, torch.distributed).

Each rank owns the keys with owner(key) == rank (a 64-bit mix of the key id,
mod world size) and keeps their state in its own HBM tables.  Two ways to
feed it:

  * sharded ingress (bench.py --gpus N): every rank receives only requests of
    the keys it owns; no data-path collective, weak scaling;
  * routed ingress (route_and_decide_torch, device-resident; route_and_decide,
    its host-side numpy twin): every rank receives arbitrary requests; one
    all-to-all moves each request record (key, ts, n, cfg, and its position)
    to its owner, the owner decides, and the inverse all-to-all returns the
    results.  On MI355X the "nccl" backend is RCCL over xGMI, where
    all-to-all drives all 7 point-to-point links at once.

Order: the reference's N app servers share one Redis, which sees requests in
arrival order.  The owner replays the union of the ranks' requests ordered by
(ts, source rank, source position), a deterministic total order consistent
with each rank's own order.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

_M1 = np.uint64(0xbf58476d1ce4e5b9)
_M2 = np.uint64(0x94d049bb133111eb)


def mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer (same function as rl_table.h mix64)."""
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return x


def owner_of(key: np.ndarray, world: int) -> np.ndarray:
    # high bits: the table uses the low bits of the same hash for slots
    return ((mix64(key) >> np.uint64(32)) % np.uint64(world)).astype(np.int64)


def _a2a(send: torch.Tensor, send_counts, recv_counts, group=None) -> torch.Tensor:
    out = torch.empty((int(sum(recv_counts)),) + tuple(send.shape[1:]), dtype=send.dtype, device=send.device)
    dist.all_to_all_single(out, send, output_split_sizes=list(recv_counts),
                           input_split_sizes=list(send_counts), group=group)
    return out


def route_and_decide(key, ts, n, cfg, decide, device="cpu", group=None):
    """Route this rank's requests to their owners, decide there, return the
    results in this rank's original order.

    decide(key, ts, n, cfg) -> (decision u8, remaining i64, retry i64, reset i64)
    runs on the owner over the merged, ordered requests it received.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    m = key.size
    own = owner_of(key, world)
    order = np.argsort(own, kind="stable")
    send_counts = np.bincount(own, minlength=world)
    # record: key, ts, n, cfg, src position (int64 each)
    rec = np.stack([key.view(np.int64), ts, n, cfg.astype(np.int64), np.arange(m, dtype=np.int64)], axis=1)[order]
    cnt_t = torch.tensor(send_counts, dtype=torch.int64, device=device)
    recv_t = torch.empty_like(cnt_t)
    dist.all_to_all_single(recv_t, cnt_t, group=group)
    recv_counts = recv_t.cpu().numpy()
    got = _a2a(torch.from_numpy(rec).to(device), send_counts, recv_counts, group).cpu().numpy()
    src = np.repeat(np.arange(world), recv_counts)
    # owner-side total order: (ts, source rank, source position)
    o = np.lexsort((got[:, 4], src, got[:, 1]))
    g = got[o]
    dec, rem, retry, reset = decide(g[:, 0].view(np.uint64).copy(), g[:, 1].copy(), g[:, 2].copy(),
                                    g[:, 3].astype(np.uint32))
    res = np.empty((g.shape[0], 4), np.int64)
    res[o] = np.stack([dec.astype(np.int64), rem, retry, reset], axis=1)  # back to arrival-from-src order
    back = _a2a(torch.from_numpy(res).to(device), recv_counts, send_counts, group).cpu().numpy()
    out = np.empty((m, 4), np.int64)
    out[order] = back
    return out[:, 0].astype(np.uint8), out[:, 1], out[:, 2], out[:, 3]


def _i64(c: int) -> int:
    """a 64-bit constant as the signed value torch's int64 arithmetic uses"""
    return c - (1 << 64) if c >= (1 << 63) else c


def mix64_torch(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 finalizer on int64 tensors (wrapping multiply, logical shifts)."""
    def shr(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)
    x = x ^ shr(x, 30)
    x = x * _i64(0xbf58476d1ce4e5b9)
    x = x ^ shr(x, 27)
    x = x * _i64(0x94d049bb133111eb)
    x = x ^ shr(x, 31)
    return x


def owner_of_torch(key: torch.Tensor, world: int) -> torch.Tensor:
    """owner_of for int64 tensors holding the u64 key ids (same partition)."""
    hi = (mix64_torch(key) >> 32) & 0xffffffff
    return hi % world


def route_and_decide_torch(key, ts, n, cfg, decide, group=None):
    """route_and_decide with every step on the tensors' device: owner hash,
    grouping by owner, the request all-to-all, the owner's (ts, source rank,
    source position) order, the decision, the inverse all-to-all.

    key, ts, n: int64 tensors (key holds the u64 ids); cfg: int32.
    decide(key, ts, n, cfg) -> (decision u8, remaining, retry, reset) tensors
    on the same device, over the merged, ordered requests this rank owns.
    Returns the four result tensors in this rank's original order.
    """
    world = dist.get_world_size(group)
    dev = key.device
    m = key.numel()
    own = owner_of_torch(key, world)
    order = torch.argsort(own, stable=True)
    send_counts = torch.bincount(own, minlength=world)
    rec = torch.stack([key, ts, n, cfg.to(torch.int64), torch.arange(m, dtype=torch.int64, device=dev)], 1)[order]
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    got = _a2a(rec, sc, rc, group)
    # received records are grouped by source rank, each in source order: a
    # stable sort by ts gives the (ts, source rank, source position) order
    o = torch.sort(got[:, 1], stable=True).indices
    g = got[o]
    dec, rem, retry, reset = decide(g[:, 0].contiguous(), g[:, 1].contiguous(), g[:, 2].contiguous(),
                                    g[:, 3].to(torch.int32).contiguous())
    res = torch.empty((g.shape[0], 4), dtype=torch.int64, device=dev)
    res[o] = torch.stack([dec.to(torch.int64), rem, retry, reset], 1)
    back = _a2a(res, rc, sc, group)
    out = torch.empty((m, 4), dtype=torch.int64, device=dev)
    out[order] = back
    return out[:, 0].to(torch.uint8), out[:, 1], out[:, 2], out[:, 3]
