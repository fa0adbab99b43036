"""Offline model of the hot key's token-bucket chain with multi-decade windows.

Replays the hottest key of a Zipf trace exactly (Python's '%.14g' / float()
round trip = the Lua tostring/tonumber of Redis 7) and counts, per batch, the
regime exits the chain's windows meet under two window kinds:

  DEC   one decade per window (the chain's fast mode): any decade change,
        sign change, allow, clamp or expiry ends the window;
  XDEC  a window spans the decades [E_top - 4, E_top] (states as integers of
        the floor decade's unit fit int64): only allows, clamps, expiries and
        states outside that range end it.  Near steps (state-dependent
        rounding) are then every upward decade crossing, every step that
        drops one decade inside the near band, or two or more decades, and
        the in-decade near band.

Policy modelled for XDEC: a window after a regime exit is XDEC; after a full
window the next one is DEC when its nominal path stays in one decade, else
XDEC.  Reports exits, windows (rounds) and near steps per window.

Analysis tool (CPU only).  usage: python scripts/xdec_sim.py s nkeys [batches]
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-rate-limiter_amd", "python"))
import traces  # noqa: E402

W = 2240


def q14(x):
    return float("%.14g" % x)


def dec(v):
    """decade E of a nonzero stored value: |v| in [10^E, 10^(E+1))"""
    s = "%.13e" % v
    return int(s.split("e")[1])


def trajectory(s, nkeys, nb):
    gen = traces.TokenBucketZipf(nkeys=nkeys, s=s)
    rate, cap = 20 / 12.0, 20.0
    tok_q, last_q = cap, None
    hot = None
    out = []   # per step: (state before, add, allowed/clamped, state after)
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
            out.append((tok_q, add, allowed or ssum >= cap, nq))
            tok_q, last_q = nq, q14(now)
    return out


def classify(x, a, nx):
    """(decade in, decade out, kind) of one non-exit step: 'far' (an integer
    add at the output decade for every state near x), 'near', 'up'"""
    if x == 0.0 or nx == 0.0:
        return None, None, "near"
    ei, eo = dec(x), dec(nx)
    if eo > ei:
        return ei, eo, "up"
    if ei - eo >= 2:
        return ei, eo, "near"
    # band (in output units) of the strtod and sum roundings
    u = 10.0 ** (eo - 13)
    band = (math.ulp(abs(x)) / 2 + math.ulp(abs(x + a)) / 2) / u
    f = a / u
    fr = abs(f - round(f))
    return ei, eo, "near" if fr > 0.5 - band - 1e-9 else "far"


def main(argv):
    s = float(argv[0])
    nkeys = int(argv[1])
    nb = int(argv[2]) if len(argv) > 2 else 2
    tr = trajectory(s, nkeys, nb + 1)
    n0 = len(tr) // (nb + 1)     # skip the first batch (the bucket starts full)
    tr = tr[n0:]
    N = len(tr)
    # DEC: exits
    exit_dec = np.zeros(N, bool)
    kinds, eis, eos = [], [], []
    for i, (x, a, al, nx) in enumerate(tr):
        ei, eo, kd = classify(x, a, nx)
        kinds.append(kd)
        eis.append(ei)
        eos.append(eo)
        exit_dec[i] = al or x <= 0 or nx <= 0 or ei != eo
    # windows under each policy
    def run(xdec):
        p = 0
        rounds = stops = 0
        near_w, up_w, nwin_x = [], [], 0
        prev_exit = True
        while p < N:
            rounds += 1
            lo = p
            hi = min(N, p + W)
            if xdec and prev_exit:
                mode = "X"
            elif xdec:
                # nominal one decade over the window?
                es = {eos[j] for j in range(lo, hi) if eos[j] is not None}
                es |= {eis[j] for j in range(lo, hi) if eis[j] is not None}
                mode = "D" if len(es) <= 1 and all(tr[j][0] > 0 and tr[j][3] > 0 for j in range(lo, hi)) else "X"
            else:
                mode = "D"
            q = hi
            if mode == "D":
                hit = np.flatnonzero(exit_dec[lo:hi])
                if hit.size:
                    q = lo + int(hit[0])
            else:
                nwin_x += 1
                top = max(dec(tr[j][3]) for j in range(lo, hi) if tr[j][3] != 0) if any(tr[j][3] for j in range(lo, hi)) else 0
                floor = top - 4
                for j in range(lo, hi):
                    x, a, al, nx = tr[j]
                    if al or (nx != 0 and dec(nx) < floor):
                        q = j
                        break
                near_w.append(sum(kinds[j] != "far" for j in range(lo, q)))
                up_w.append(sum(kinds[j] == "up" for j in range(lo, q)))
            if q < hi:
                stops += 1
                # serial steps: the exit, then on until a positive in-decade state (DEC) / the next step (XDEC)
                q += 1
                if not xdec:
                    while q < N and (exit_dec[q - 1] or tr[q - 1][3] <= 0) and q - lo < W:
                        q += 1
                prev_exit = True
            else:
                prev_exit = False
            p = q
        return rounds, stops, near_w, up_w, nwin_x
    for xd in (False, True):
        r, st, nw, uw, nx = run(xd)
        extra = ""
        if xd and nw:
            extra = (f"; XDEC windows {nx / nb:.1f}/batch, near steps per XDEC window mean {np.mean(nw):.0f} "
                     f"max {max(nw)}, upward crossings mean {np.mean(uw):.1f} max {max(uw)}")
        print(f"{'XDEC' if xd else 'DEC '}: rounds {r / nb:.1f}/batch, stops {st / nb:.1f}/batch{extra}")
    print(f"steps/batch {N / nb:.0f}; DEC exits/batch {exit_dec.sum() / nb:.0f}; "
          f"allows/batch {sum(t[2] for t in tr) / nb:.1f}; near (generalized) {sum(k != 'far' for k in kinds) / nb:.0f}/batch, "
          f"up {sum(k == 'up' for k in kinds) / nb:.0f}/batch")


if __name__ == "__main__":
    main(sys.argv[1:])
