"""Check of the multi-decade (XDEC) window arithmetic of rl_tb_chain.h on the
hot key's exact trajectory (Python's '%.14g' / float() = Redis 7's Lua
tostring / tonumber).

A window with floor decade F holds every state as an integer X of the unit
10^(F-13) (states of decades F..F+4: |X| < 1e18).  The producers' rule makes
a step "far" when its result is X + r for every state near the nominal one,
r = g * rint(A / g), A = add * 10^(13-F), g = 10^(decade out - F).  This
script replays the trajectory, classifies every step with that rule from the
nominal state (exact state + a random offset within the slack the chain
allows) and asserts that every far step's exact result equals X + r.  It also
reports how the steps split (far / near-add / near-reset / exit).

Analysis tool (CPU only).  usage: python scripts/xdec_model.py s nkeys [batches]
"""
import math
import random
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
import xdec_sim  # noqa: E402

T13 = 10 ** 13


def kidx(v):
    """decade index of |v| (X units) above the floor: 0..4, or None outside [1e13, 1e18)"""
    a = abs(v)
    if a < T13 or a >= 10 ** 18:
        return None
    k = 0
    while a >= 10 ** (14 + k):
        k += 1
    return k


def xstep(X, F, add, th):
    """exact Redis-7 step from state X (units 10^(F-13)); (X', tokens) or None (exit)"""
    if X == 0:
        T = 0.0
    else:
        k = kidx(X)
        D = X // 10 ** k if X > 0 else -((-X) // 10 ** k)
        T = D / 10 ** (13 - F - k)                 # correctly rounded (Python int / int)
    s = T + add
    if not (s < th):
        return None
    if s == 0.0:
        return 0, s
    txt = "%.13e" % abs(s)
    m, e = txt.split("e")
    Dn = int(m.replace(".", ""))
    En = int(e)
    if En < F or En > F + 4:
        return None
    Xn = Dn * 10 ** (En - F)
    return (-Xn if s < 0 else Xn), s


def classify(N_in, A, add, F, slack_rel=2.0 ** -24):
    """producers' rule from the nominal state N_in: (kind, r); kind in far / add / reset / exit"""
    V_out = N_in + A
    kin, kout = kidx(N_in), kidx(V_out)
    if kout is None:
        return "exit", 0
    g = 10 ** kout
    r = int(round(A / g)) * g if abs(A / g) < 2 ** 52 else 0
    N_out = N_in + r
    if N_in == 0 or kin is None:
        return "reset", r
    if kidx(N_out) != kout:
        return "reset", r
    if kout > kin:
        return "reset", r
    # distance of both states to decade boundaries / zero must exceed the slack
    u = 10.0 ** (F - 13)
    xm = abs(N_in) * (1 + 2 * slack_rel) * u
    sm = (abs(N_out) * (1 + 2 * slack_rel) + g) * u
    band = (math.ulp(xm) + math.ulp(sm)) / 2 / (u * g)
    f = A / g
    fr = abs(f - round(f))
    if fr > 0.5 - band - 2.0 ** -40:
        return "add", r
    return "far", r


def main(argv):
    s = float(argv[0])
    nkeys = int(argv[1])
    nb = int(argv[2]) if len(argv) > 2 else 1
    tr = xdec_sim.trajectory(s, nkeys, nb + 1)
    tr = tr[len(tr) // (nb + 1):]
    rng = random.Random(5)
    counts = {"far": 0, "add": 0, "reset": 0, "exit": 0, "skip": 0}
    bad = 0
    for (x, add, al, nx) in tr:
        if al or x == 0.0:
            counts["skip"] += 1
            continue
        E = xdec_sim.dec(x)
        for F in (E - 4, E - 2, E):       # the state in the window's top, middle and floor decade
            if F < -9:
                continue
            txt = "%.13e" % abs(x)
            D = int(txt.split("e")[0].replace(".", ""))
            X = D * 10 ** (E - F) * (1 if x > 0 else -1)
            # the nominal state: the exact one off by an offset within the chain's slack
            c = int(rng.uniform(-1, 1) * abs(X) * 2.0 ** -26)
            kind, r = classify(X - c, add * 10.0 ** (13 - F), add, F)
            counts[kind] += 1
            if kind == "far":
                res = xstep(X, F, add, 20.0)
                if res is None or res[0] != X + r:
                    bad += 1
                    if bad < 10:
                        print("far step wrong:", x, add, F, X, r, res)
            # the exact step agrees with the Lua round trip
            res = xstep(X, F, add, 1.0)
            if res is not None:
                want = float("%.14g" % (x + add))
                got = res[0] * 10.0 ** (F - 13)
                assert abs(got - want) <= abs(want) * 1e-15, (x, add, F, res, want)
    print(counts, "far steps wrong:", bad)


if __name__ == "__main__":
    main(sys.argv[1:])
