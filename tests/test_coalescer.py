"""Request coalescer (include/rl_coalescer.h): concurrent submissions become
engine batches in sequence order, and every submitter gets exactly the results
the reference limiter would give when receiving all requests one by one in
ticket order.

CPU tests drive the coalescer over a synchronous host backend (the
rl_coalescer_create_with_backend test seam) that decides each batch with the
oracle; the GPU tests drive it over the MI355X engine.  In both, the check
replays every request in ticket (= sequence) order through a fresh oracle."""
import ctypes as C
import threading

import numpy as np
import pytest

NS = 1_000_000_000
T0 = (1_760_000_000 // 60) * 60 * NS   # a minute boundary: every window id below is the same
CONFIGS = [(1, 20, 12 * NS), (3, 100, 60 * NS), (2, 100, 60 * NS), (1, 5, NS)]


def _arr(p, t, m):
    return np.ctypeslib.as_array(C.cast(p, C.POINTER(t)), shape=(m,))


def oracle_backend(oracle_mod, configs, log):
    sim = oracle_mod.OracleSim(oracle_mod.REDIS7)
    for a, L, W in configs:
        sim.add_config(a, L, W)

    def fn(user, m, key, ts, n, cfg, dec, rem, retry, reset):
        d, r, ra, rs, _ = sim.decide(_arr(key, C.c_uint64, m).copy(), _arr(ts, C.c_int64, m).copy(),
                                     _arr(n, C.c_int64, m).copy(), _arr(cfg, C.c_uint32, m).copy())
        _arr(dec, C.c_uint8, m)[:] = d
        _arr(rem, C.c_int64, m)[:] = r
        _arr(retry, C.c_int64, m)[:] = ra
        _arr(reset, C.c_int64, m)[:] = rs
        log.append(m)
        return 0
    return fn


def hammer(co, nthreads, subs_per_thread, max_sub, nkeys, ncfg, seed, span_ns=50 * NS):
    """Threads submit random chunks and wait for them; returns every
    (ticket, inputs, results) record."""
    out, lock, errors = [], threading.Lock(), []

    def worker(tid):
        rng = np.random.default_rng(seed + tid)
        for _ in range(subs_per_thread):
            m = int(rng.integers(1, max_sub + 1))
            key = rng.integers(0, nkeys, m).astype(np.uint64)
            ts = (T0 + rng.integers(0, span_ns, m)).astype(np.int64)
            n = rng.choice([1, 1, 1, 2, 3], m).astype(np.int64)
            cfg = (key % ncfg).astype(np.uint32)
            t = co.submit(key, ts, n, cfg)
            rc, res = co.wait(t, m)
            if rc != 0:
                errors.append(rc)
            with lock:
                out.append((t, key, ts, n, cfg, res))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    return out


def check_against_oracle(oracle_mod, configs, recs):
    recs.sort(key=lambda r: r[0])
    # tickets are the sequence numbers of each submission's first request
    seq = 0
    for t, key, *_ in recs:
        assert t == seq
        seq += key.size
    cat = [np.concatenate([r[i] for r in recs]) for i in (1, 2, 3, 4)]
    sim = oracle_mod.OracleSim(oracle_mod.REDIS7)
    for a, L, W in configs:
        sim.add_config(a, L, W)
    dec, rem, retry, reset, _ = sim.decide(*cat)
    got = [np.concatenate([r[5][i] for r in recs]) for i in range(4)]
    assert np.array_equal(got[0], dec)
    assert np.array_equal(got[1], rem)
    assert np.array_equal(got[2], retry)
    assert np.array_equal(got[3], reset)


def test_concurrent_submitters_match_sequential_oracle(rl, oracle_mod):
    log = []
    co = rl.Coalescer(oracle_backend(oracle_mod, CONFIGS, log), max_batch=64, max_in_flight=3)
    recs = hammer(co, nthreads=6, subs_per_thread=60, max_sub=40, nkeys=30, ncfg=len(CONFIGS), seed=11)
    st = co.stats()
    co.close()
    total = sum(r[1].size for r in recs)
    assert st.submitted == total and st.decided == total and st.pending == 0
    assert max(log) <= 64 and sum(log) == total
    assert st.batches == len(log)
    check_against_oracle(oracle_mod, CONFIGS, recs)


def test_submissions_split_across_batches(rl, oracle_mod):
    log = []
    co = rl.Coalescer(oracle_backend(oracle_mod, CONFIGS, log), max_batch=7, max_in_flight=2)
    recs = hammer(co, nthreads=3, subs_per_thread=20, max_sub=50, nkeys=5, ncfg=len(CONFIGS), seed=5)
    co.close()
    assert max(log) <= 7
    assert any(r[1].size > 7 for r in recs)
    check_against_oracle(oracle_mod, CONFIGS, recs)


def test_single_decide_and_edge_cases(rl, oracle_mod):
    log = []
    co = rl.Coalescer(oracle_backend(oracle_mod, CONFIGS, log), max_batch=16, queue_cap=10)
    # one Allow: the first request of a token bucket of capacity 20
    rc, (d, rem, retry, reset) = co.decide(42, T0, 1, 0)
    assert rc == 0 and d == rl.ALLOWED and rem == 19 and retry == 0
    # empty submission: a unique ticket that is done at once
    t0 = co.submit(np.zeros(0, np.uint64), np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint32))
    rc, res = co.wait(t0, 0)
    assert rc == 0 and all(x.size == 0 for x in res)
    # unknown ticket, and a ticket waited for twice
    assert co.wait(10 ** 12, 1)[0] == rl.RL_EINVAL
    assert co.wait(t0, 0)[0] == rl.RL_EINVAL
    # queue capacity
    with pytest.raises(rl.EngineError) as ei:
        co.submit(np.arange(11, dtype=np.uint64), np.full(11, T0, np.int64), np.ones(11, np.int64),
                  np.zeros(11, np.uint32))
    assert ei.value.code == rl.RL_EAGAIN
    co.close()


def test_backend_error_reaches_every_waiter(rl):
    def failing(user, m, *ptrs):
        return -5   # RL_EDEVICE
    co = rl.Coalescer(failing, max_batch=8)
    ts = [co.submit(np.arange(5, dtype=np.uint64), np.full(5, T0, np.int64), np.ones(5, np.int64),
                    np.zeros(5, np.uint32)) for _ in range(4)]
    assert [co.wait(t, 5)[0] for t in ts] == [-5] * 4
    co.close()


@pytest.mark.gpu
def test_gpu_coalescer_matches_sequential_oracle(rl, oracle_mod):
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 12, win_capacity=1 << 12, max_batch=1 << 12,
                    device=0, flags=rl.OPT_PIPELINE)
    for a, L, W in CONFIGS:
        eng.register(a, L, W)
    co = rl.Coalescer(eng, max_batch=1 << 12, max_in_flight=3)
    recs = hammer(co, nthreads=8, subs_per_thread=40, max_sub=64, nkeys=50, ncfg=len(CONFIGS), seed=21)
    rc, (d, rem, retry, reset) = co.decide(7, T0 + 51 * NS, 1, 0)
    st = co.stats()
    co.close()
    assert rc == 0
    assert eng.sync() == 0
    eng.close()
    total = sum(r[1].size for r in recs)
    assert st.decided == total + 1
    check_against_oracle(oracle_mod, CONFIGS, recs)


@pytest.mark.gpu
def test_gpu_coalescer_hot_key_batches(rl, oracle_mod):
    """One hot key under concurrency: batches large enough to take the
    engine's cooperative replay paths, still equal to the sequential oracle."""
    cfgs = CONFIGS[:1]
    eng = rl.Engine(profile=rl.PROFILE_REDIS7, tb_capacity=1 << 12, win_capacity=1 << 10, max_batch=1 << 14,
                    device=0, flags=rl.OPT_PIPELINE)
    for a, L, W in cfgs:
        eng.register(a, L, W)
    co = rl.Coalescer(eng, max_batch=1 << 14, max_in_flight=3, linger_ns=200_000)
    recs = hammer(co, nthreads=4, subs_per_thread=10, max_sub=3000, nkeys=1, ncfg=1, seed=3)
    co.close()
    assert eng.sync() == 0
    eng.close()
    check_against_oracle(oracle_mod, cfgs, recs)
