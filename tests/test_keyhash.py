"""On-GPU FormatKey + XXH64 key ids (include/rl_keyhash.h, csrc/rl_keyhash.hip).

CPU: the oracle's XXH64 restatement against the published known answer and
the committed golden vectors (tests/golden/keyhash_golden.json, made by
tests/golden/make_keyhash_golden.py with the xxhash package); FormatKey against
the host mirror's rll_format_key (config.go:81-87); argument checks of the C-ABI
that return before any device call.

GPU: bit-exact ids against the oracle over every length class (LDS-staged and
oversized groups, unaligned and ragged buffers, bad offsets), and decisions
made through hashed ids equal to the oracle's decisions with string identity.
"""
import json
import os

import numpy as np
import pytest

from oracle import keyhash as kh

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "keyhash_golden.json")


def golden_cases():
    return json.load(open(GOLDEN))["cases"]


# --- CPU ---------------------------------------------------------------------

def test_xxh64_known_answer():
    assert kh.xxh64(b"", 0) == 0xEF46DB3751D8E999


def test_oracle_matches_golden():
    for c in golden_cases():
        f = kh.format_key(bytes.fromhex(c["prefix"]), bytes.fromhex(c["key"]))
        assert kh.xxh64(f, int(c["seed"])) == int(c["xxh64"]), c


def test_oracle_matches_xxhash_all_lengths():
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(5)
    for n in range(0, 140):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for seed in (0, 12345, (1 << 64) - 1):
            assert kh.xxh64(b, seed) == xxhash.xxh64_intdigest(b, seed)


@pytest.mark.parametrize("prefix,key", [("", "k"), ("ratelimit", "user:1"), ("api", ""), ("", ""),
                                        ("p", "a:b")])
def test_format_key_matches_host_mirror(rl, prefix, key):
    assert rl.format_key(prefix, key) == kh.format_key(prefix.encode(), key.encode()).decode()


def test_hash_keys_argument_errors(rl):
    data, off = rl.pack_keys([b"ab", b"c"])
    rc, _ = rl.hash_keys((data, off), 0, b"p" * 241, check=False)          # prefix too long
    assert rc == rl.RL_EINVAL
    bad = off.copy()
    bad[2] = 1                                                               # offsets decrease
    rc, _ = rl.hash_keys((data, bad), 0, check=False)
    assert rc == rl.RL_EINVAL
    past = off.copy()
    past[2] = 9                                                              # past nbytes
    rc, _ = rl.hash_keys((data, past), 0, check=False)
    assert rc == rl.RL_EINVAL
    rc, out = rl.hash_keys(([], np.zeros(1, np.uint64)), 0, check=False)    # empty batch
    assert rc == rl.RL_OK and out.size == 0


# --- GPU ---------------------------------------------------------------------

def random_keys(rng, m, lo, hi):
    lens = rng.integers(lo, hi + 1, m)
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    out, o = [], 0
    for n in lens:
        out.append(blob[o:o + n])
        o += n
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("prefix", [b"", b"ratelimit", b"p" * 240])
@pytest.mark.parametrize("lens", [(0, 40), (0, 300), (100, 400)])
def test_gpu_ids_match_oracle(rl, prefix, lens):
    rng = np.random.default_rng(len(prefix) * 1000 + lens[1])
    keys = random_keys(rng, 20_000 if lens[1] <= 40 else 5000, *lens)
    for seed in (0, 3, (1 << 64) - 1):
        got = rl.hash_keys(keys, seed, prefix)
        want = np.array(kh.key_ids_fast(prefix, keys, seed), dtype=np.uint64)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (bad[:5], [keys[i] for i in bad[:3]])


@pytest.mark.gpu
def test_gpu_golden_vectors(rl):
    by = {}
    for c in golden_cases():
        by.setdefault((c["prefix"], c["seed"]), []).append(c)
    for (p, seed), cs in by.items():
        keys = [bytes.fromhex(c["key"]) for c in cs]
        got = rl.hash_keys(keys, int(seed), bytes.fromhex(p))
        want = [int(c["xxh64"]) for c in cs]
        want = np.array([kh.KEY_RESERVED - 1 if w == kh.KEY_RESERVED else w for w in want], dtype=np.uint64)
        assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_device_entry_unaligned_ragged_and_bad_offsets(rl):
    import torch
    rng = np.random.default_rng(9)
    keys = random_keys(rng, 3000, 0, 50)
    data, off = rl.pack_keys(keys)
    for shift in (0, 1, 3, 8, 13):
        buf = torch.zeros(data.size + shift, dtype=torch.uint8, device="cuda")
        buf[shift:] = torch.from_numpy(data).cuda()
        o = torch.from_numpy(off.view(np.int64)).cuda()
        ids = torch.zeros(len(keys), dtype=torch.int64, device="cuda")
        rc = rl.lib.rl_hash_keys_device(len(keys), buf.data_ptr() + shift, data.size, o.data_ptr(), 11,
                                        b"rl", 2, ids.data_ptr(), None)
        assert rc == rl.RL_OK
        torch.cuda.synchronize()
        want = np.array(kh.key_ids_fast(b"rl", keys, 11), dtype=np.uint64)
        assert np.array_equal(ids.cpu().numpy().view(np.uint64), want), shift
    # offsets out of order / past nbytes: those requests get the reserved id
    bad = off.copy()
    bad[10] = bad[11] + 1
    bad[-1] = data.size + 5
    o = torch.from_numpy(bad.view(np.int64)).cuda()
    buf = torch.from_numpy(data).cuda()
    ids = torch.zeros(len(keys), dtype=torch.int64, device="cuda")
    assert rl.lib.rl_hash_keys_device(len(keys), buf.data_ptr(), data.size, o.data_ptr(), 0, None, 0,
                                      ids.data_ptr(), None) == rl.RL_OK
    got = ids.cpu().numpy().view(np.uint64)
    assert got[10] == rl.KEY_RESERVED and got[-1] == rl.KEY_RESERVED      # offsets[10] > offsets[11]; past nbytes
    assert got[9] == kh.key_id(b"", data[int(bad[9]):int(bad[10])].tobytes(), 0)   # the longer range it was given
    want = np.array(kh.key_ids_fast(b"", keys, 0), dtype=np.uint64)
    good = np.ones(len(keys), bool)
    good[[9, 10, len(keys) - 1]] = False
    assert np.array_equal(got[good], want[good])


@pytest.mark.gpu
def test_gpu_formatted_identity(rl):
    # FormatKey("", "a:b") == FormatKey("a", "b"): the same Redis key in the
    # reference, so the same id under one seed; other prefixes / seeds differ
    a = rl.hash_keys([b"a:b"], 5, b"")
    b = rl.hash_keys([b"b"], 5, b"a")
    c = rl.hash_keys([b"b"], 5, b"c")
    d = rl.hash_keys([b"b"], 6, b"a")
    assert a[0] == b[0] and a[0] != c[0] and a[0] != d[0]


@pytest.mark.gpu
@pytest.mark.parametrize("alg", [1, 2, 3])
def test_gpu_decisions_through_hashed_ids(rl, alg):
    """Decisions on string keys: GPU (hashed ids) vs oracle (string identity)."""
    import oracle
    from tracegen import NS, T0
    rng = np.random.default_rng(alg)
    names = [f"user:{i}".encode() for i in range(4000)]
    m = 60_000
    pick = np.minimum(rng.zipf(1.3, m) - 1, len(names) - 1)
    keys = [names[i] for i in pick]
    ts = T0 + np.cumsum(rng.integers(0, 300_000, m)).astype(np.int64)
    n = np.ones(m, np.int64)
    cfg = np.zeros(m, np.uint32)
    L, W = (20, 12 * NS) if alg == 1 else (50, 2 * NS)

    ids = rl.hash_keys(keys, 1, b"ratelimit")
    assert len(set(ids[np.unique(pick, return_index=True)[1]].tolist())) == len(np.unique(pick))
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 14, win_capacity=1 << 14, max_batch=1 << 16)
    sim = oracle.OracleSim(oracle.REDIS7)
    eng.register(alg, L, W)
    sim.add_config(alg, L, W)
    got = eng.decide(ids, ts, n, cfg)
    dec, rem, retry, reset, tok = sim.decide(pick.astype(np.uint64), ts, n, cfg)   # string identity = name index
    eng.close()
    assert np.array_equal(got.decision, dec)
    assert np.array_equal(got.remaining, rem)
    assert np.array_equal(got.retry_after_ns, retry)
    assert np.array_equal(got.reset_at_ns, reset)


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline", [False, True])
def test_gpu_decide_batch_keys_device(rl, pipeline):
    """rl_decide_batch_keys_device (hash on the grouping stream) == oracle with
    string identity, over big and small batches, batches in flight, chunking."""
    import torch

    import oracle
    from tracegen import NS, T0
    rng = np.random.default_rng(21 + pipeline)
    names = [f"tenant:{i}:{'x' * (i % 37)}".encode() for i in range(30_000)]
    sizes = [50_000, 3000, 70_000, 17, 40_000]
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 16, win_capacity=1 << 16, max_batch=1 << 15,
                    flags=rl.OPT_PIPELINE if pipeline else 0)
    sim = oracle.OracleSim(oracle.REDIS7)
    cfgs = [(1, 20, 12 * NS), (2, 30, 3 * NS), (3, 40, 2 * NS)]
    for a, L, W in cfgs:
        assert eng.register(a, L, W) == sim.add_config(a, L, W)
    dev = torch.device("cuda", 0)
    t_last = T0
    pending = []
    for m in sizes:
        pick = np.minimum(rng.zipf(1.2, m) - 1, len(names) - 1)
        data, off = rl.pack_keys([names[i] for i in pick])
        ts = t_last + np.cumsum(rng.integers(0, 200_000, m)).astype(np.int64)
        t_last = int(ts[-1])
        n = rng.choice([1, 1, 1, 3], m).astype(np.int64)
        # configs drawn independently of the key: one raw key is used under
        # several configs (two window configs with different W included), each
        # its own namespace (rl_cfg_seed)
        cfg = rng.integers(0, 3, m).astype(np.uint32)
        d = [torch.from_numpy(x).to(dev) for x in (data, off.view(np.int64), ts, n, cfg.view(np.int32))]
        o = [torch.empty(m, dtype=torch.uint8, device=dev)] + \
            [torch.empty(m, dtype=torch.int64, device=dev) for _ in range(3)] + \
            [torch.empty(m, dtype=torch.float64, device=dev)]
        torch.cuda.synchronize()   # inputs complete before the call (RL_OPT_PIPELINE contract)
        rc = rl.lib.rl_decide_batch_keys_device(eng.h, m, d[0].data_ptr(), data.size, d[1].data_ptr(), 4,
                                                b"ratelimit", 9, d[2].data_ptr(), d[3].data_ptr(),
                                                d[4].data_ptr(), None, *[x.data_ptr() for x in o], None)
        assert rc == rl.RL_OK
        # string identity for the oracle: the name index, one namespace per config
        pending.append((d, o, sim.decide(pick.astype(np.uint64) * 4 + cfg, ts, n, cfg)))
    assert eng.sync() == rl.RL_OK
    torch.cuda.synchronize()
    for d, o, (dec, rem, retry, reset, tok) in pending:
        assert np.array_equal(o[0].cpu().numpy(), dec)
        assert np.array_equal(o[1].cpu().numpy(), rem)
        assert np.array_equal(o[2].cpu().numpy(), retry)
        assert np.array_equal(o[3].cpu().numpy(), reset)
    eng.close()


def test_decide_batch_keys_device_argument_errors(rl):
    # rejected before any device call (no GPU needed)
    vp = None
    assert rl.lib.rl_decide_batch_keys_device(None, 0, vp, 0, vp, 0, None, 0, *([vp] * 10)) == rl.RL_EINVAL
    assert rl.lib.rl_hash_keys_device(1, vp, 0, vp, 0, None, 0, vp, vp) == rl.RL_EINVAL        # NULL offsets
    assert rl.lib.rl_hash_keys_device(0, vp, 0, vp, 0, b"p" * 241, 241, vp, vp) == rl.RL_EINVAL  # prefix too long
    assert rl.lib.rl_hash_keys_device(0, vp, 0, vp, 0, None, 0, vp, vp) == rl.RL_OK             # empty batch
