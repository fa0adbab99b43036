"""Offline analysis of the hot key's token-bucket chain (configs[1]).

Replays the hottest key of the first batches of the configs[1] trace with the
Python restatement of the step (Lua %.14g round trip = Python's correctly
rounded '%.14g' / float()), classifies every step as the chain sees it (far /
near / regime exit) and counts what the chain's near-step fixed point costs:
iterations of the current scheme (one evaluation per lane per iteration) and
of a scheme that evaluates every near step at three offsets at once (scan-only
iterations while the guesses stay inside the evaluated window).

Analysis tool (CPU only; reads nothing of the engine).
usage: python scripts/chain_sim.py [batches]
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-rate-limiter_amd", "python"))
import traces  # noqa: E402

DEC_LO, DEC_HI = 10**13, 10**14


def q14(x):
    return float("%.14g" % x)


def dec_of(v):
    """(D, E) of a stored %.14g value v > 0: v = D * 10^(E-13), D in [1e13, 1e14)"""
    s = "%.13e" % v
    mant, ex = s.split("e")
    D = int(mant.replace(".", "").replace("-", ""))
    return D, int(ex)


def step_at(D, E, add, cap, n=1.0):
    """one step from stored digits D (decade E); returns (allowed, tokens, D', E')"""
    t = float("%de%d" % (D, E - 13))
    s = t + add
    tok = s if s < cap else cap
    allowed = tok >= n
    if allowed:
        tok = tok - n
    return allowed, tok, q14(tok)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    gen = traces.TokenBucketZipf()
    L, W = 20, 12.0
    rate = L / W
    cap = float(L)
    keys, tss = [], []
    for _ in range(nb):
        k, t, _, _ = gen.next_batch()
        keys.append(k)
        tss.append(t)
    key = np.concatenate(keys)
    ts = np.concatenate(tss)
    vals, cnt = np.unique(key[:1_000_000], return_counts=True)
    hot = vals[np.argmax(cnt)]
    t_hot = ts[key == hot]
    print("hot key", hot, "requests", t_hot.size, "per batch", t_hot.size / nb)
    # exact sequence
    tok_q = cap          # stored tokens
    last_q = None
    far = near = flips = exits = neg = 0
    near_pos = []        # (index, D before, E, add, flip)
    seq = []
    for i, t in enumerate(t_hot):
        now = float(int(t)) / 1e9
        add = 0.0 if last_q is None else (now - last_q) * rate
        if tok_q > 0:
            D, E = dec_of(tok_q)
            P = 10.0 ** (13 - E)
            pr = add * P
            rr = round(pr)
            fr = abs(pr - rr)
        else:
            D = E = None
        s = tok_q + add
        tok = s if s < cap else cap
        allowed = tok >= 1.0
        if allowed:
            tok -= 1.0
        nq = q14(tok)
        kind = "exit"
        if D is not None and not allowed and s < cap and nq > 0:
            D2, E2 = dec_of(nq)
            if E2 == E:
                nominal = D + rr
                flip = D2 - nominal
                # band: binade bound of the near test (dmax ~ D)
                e = math.frexp(max(D, D2) / P)[1]
                band = math.ldexp(P, e - 53)
                lim = 0.5 - (band + 2**-40)
                if abs(pr - rr) > lim:
                    kind = "near"
                    near += 1
                    near_pos.append((i, D, E, add, flip))
                    flips += flip != 0
                else:
                    kind = "far"
                    far += 1
                    assert flip == 0, (i, D, E, add, flip)
        if kind == "exit":
            exits += 1
            if nq <= 0:
                neg += 1
        seq.append(kind)
        tok_q = nq
        last_q = q14(now)
    n = len(seq)
    print(f"steps {n}: far {far} near {near} ({near / n:.2%}) flips {flips} ({flips / max(near, 1):.1%} of near) "
          f"exits {exits} (state <= 0: {neg})")
    # fixed-point iterations per 64 consecutive near steps between exits
    # (the chain resolves a window's near steps 64 at a time)
    it_cur, it_scan, evals3, groups = [], [], [], 0
    idx = 0
    while idx < len(near_pos):
        grp = near_pos[idx:idx + 64]
        idx += 64
        groups += 1
        # true offsets: cumulative flips; guess: est (relative)
        true_flip = [g[4] for g in grp]

        def f(j, off):
            """flip of near step j when the offset before it is off (relative to truth 0)"""
            i, D, E, add, fl = grp[j]
            Dg = D + off
            if not (DEC_LO <= Dg < DEC_HI):
                return None
            P = 10.0 ** (13 - E)
            allowed, tok, nq = step_at(Dg, E, add, cap)
            if allowed or nq <= 0:
                return None
            D2, E2 = dec_of(nq)
            if E2 != E:
                return None
            return D2 - (Dg + round(add * P))

        tru = np.concatenate([[0], np.cumsum(true_flip)])[:-1]   # true offset before each (relative to group start)
        # current scheme: est = 0 everywhere, iterate
        est = np.zeros(len(grp), np.int64)
        for it in range(1, 65):
            fl = np.array([f(j, int(est[j] - tru[j])) or 0 for j in range(len(grp))])
            en = np.concatenate([[0], np.cumsum(fl)])[:-1]
            if np.array_equal(en, est):
                break
            est = en
        it_cur.append(it)
        # three-candidate scheme: evaluate at est-1, est, est+1; scan-iterate
        # over the table; re-evaluate when a guess leaves the window
        est = np.zeros(len(grp), np.int64)
        ev = 0
        scans = 0
        while True:
            ev += 1
            centre = est.copy()
            tab = {(j, d): f(j, int(centre[j] + d - tru[j])) or 0 for j in range(len(grp)) for d in (-1, 0, 1)}
            done = False
            while True:
                scans += 1
                fl = np.array([tab[(j, int(est[j] - centre[j]))] for j in range(len(grp))])
                en = np.concatenate([[0], np.cumsum(fl)])[:-1]
                if np.array_equal(en, est):
                    done = True
                    break
                est = en
                if np.any(np.abs(est - centre) > 1):
                    break
            if done:
                break
        evals3.append(ev)
        it_scan.append(scans)
    print(f"near groups of 64: {groups}; current scheme iterations (evaluations): mean {np.mean(it_cur):.2f} "
          f"max {max(it_cur)}; 3-candidate: evaluation passes mean {np.mean(evals3):.2f} max {max(evals3)}, "
          f"scan passes mean {np.mean(it_scan):.2f}")
    # stops: regime exits per batch and how far apart
    ex_idx = [i for i, k in enumerate(seq) if k == "exit"]
    gaps = np.diff(ex_idx) if len(ex_idx) > 1 else np.array([0])
    print(f"exits per batch {len(ex_idx) / nb:.1f}; gap between exits: median {np.median(gaps):.0f}, "
          f"<64: {(gaps < 64).sum()}, >=2240: {(gaps >= 2240).sum()}")


if __name__ == "__main__" and not (len(sys.argv) > 1 and sys.argv[1] == "exits"):
    main()


def exit_trace(s, nkeys, nb):
    """exact replay of the hottest key: per step (exit?, state positive after?)"""
    gen = traces.TokenBucketZipf(nkeys=nkeys, s=s)
    rate, cap = 20 / 12.0, 20.0
    tok_q, last_q = cap, None
    ex, pos = [], []
    hot = None
    for _ in range(nb):
        k, t, _, _ = gen.next_batch()
        if hot is None:
            vals, cnt = np.unique(k, return_counts=True)
            hot = vals[np.argmax(cnt)]
        for tt in t[k == hot]:
            now = float(int(tt)) / 1e9
            add = 0.0 if last_q is None else (now - last_q) * rate
            ssum = tok_q + add
            tok = ssum if ssum < cap else cap
            allowed = tok >= 1.0
            if allowed:
                tok -= 1.0
            nq = q14(tok)
            e_old = dec_of(tok_q)[1] if tok_q > 0 else None
            e_new = dec_of(nq)[1] if nq > 0 else None
            ex.append(allowed or ssum >= cap or tok_q <= 0 or nq <= 0 or e_old != e_new)
            pos.append(nq > 0)
            tok_q, last_q = nq, q14(now)
    return np.array(ex), np.array(pos)


def round_model(ex, pos, W=2240, serial_cap=64, linger=0):
    """rounds and serial steps of the chain's round structure (approximation of
    ch_segment): a full window costs one round; a window with a regime exit
    costs its round, exact serial steps from the exit, and a producers-only
    round for the next window.  Serial steps go on while the last step left
    the regime or the state is not positive (and, with `linger`, until
    `linger` steps past the last exit), at most serial_cap per round."""
    N = ex.size
    rounds = 1                       # first window
    serial = stops = 0
    p = 0
    while p < N:
        rounds += 1
        hit = np.flatnonzero(ex[p:p + W])
        if hit.size == 0:
            p += W
            continue
        stops += 1
        q = p + int(hit[0])
        k = 0
        last = q
        while q < N and k < serial_cap:
            need = k == 0 or ex[q - 1] or not pos[q - 1] or q - last < linger
            if not need:
                break
            if ex[q]:
                last = q
            q += 1
            k += 1
        serial += k
        p = q
        rounds += 1                  # producers-only round for the next window
    return rounds, serial, stops


def exits_main(argv):
    s = float(argv[0])
    nkeys = int(argv[1])
    nb = int(argv[2]) if len(argv) > 2 else 1
    ex, pos = exit_trace(s, nkeys, nb + 1)
    n0 = int(np.ceil(ex.size / (nb + 1)))     # skip the first batch (the bucket starts full)
    ex, pos = ex[n0:], pos[n0:]
    N = ex.size
    idx = np.flatnonzero(ex)
    gaps = np.diff(idx)
    print(f"s={s} nkeys={nkeys}: {N} hot steps over {nb} batches, exits {idx.size} ({idx.size / nb:.0f}/batch); "
          f"gaps <8: {(gaps < 8).sum()} <32: {(gaps < 32).sum()} <128: {(gaps < 128).sum()} <1024: {(gaps < 1024).sum()}")
    for linger in (0, 16, 32, 64, 128):
        for cap in (64, 256):
            r, se, st = round_model(ex, pos, serial_cap=cap, linger=linger)
            print(f"  linger {linger:4d} cap {cap:4d}: rounds {r / nb:7.1f}/batch serial {se / nb:8.1f}/batch "
                  f"stops {st / nb:6.1f}  model cycles/batch {(r * 8000 + se * 440) / nb / 1e3:8.0f}k")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "exits":
    exits_main(sys.argv[2:])
