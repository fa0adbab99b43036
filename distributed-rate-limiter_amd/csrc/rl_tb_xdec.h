// rl_tb_xdec.h -- multi-decade ("XDEC") token-bucket windows of the chain.
// Included by rl_tb_chain.h (after the helpers it shares with the one-decade
// mode).
//
// Why.  A hot key's stored balance is quantized to 14 significant digits
// (tokenbucket.go:48, Lua tostring under Redis 7) and its last_refill to
// 100 us.  After an allow the balance sits near zero and climbs one token per
// refill period with a sawtooth of +-2.5e-4 .. 2e-3 tokens (the rounding of
// last_refill, tokenbucket.go:36-37): it changes sign and decade every few
// steps.  A one-decade window (QM_DEC) ends at each of those crossings, and
// every such regime exit costs the chain a round of its own.
//
// What.  A window with floor decade F holds every state as ONE integer X of
// the unit 10^(F-13): a stored value D * 10^(E-13) with E in [F, F + 4] is
// X = D * 10^(E-F) (|X| < 1e18, an int64), zero is X = 0.  A step whose
// result lands in the same or a lower decade than its input and whose
// increment add * 10^(13-F) is farther than the rounding band from a
// half-unit of the result's decade g = 10^(E'-F) is the integer add
// X' = X + g * rint(add * 10^(13-F) / g) for every state near the nominal one
// (X is a multiple of g): "far".  Every other step -- a result one or more
// decades UP (rounded coarser than its input's digits: its result depends on
// the exact digits, a "reset" step), a drop of two or more decades
// (cancellation), a step inside the band -- is "near" and is evaluated
// exactly by the chain's fixed point, as in one-decade windows.  Signs change
// freely.  Regime exits are what they are in the reference: an allow or a
// clamp (sum >= th), an expired key, and here also a state outside the
// window's five decades.  scripts/xdec_model.py checks the far rule on the
// exact hot-key trajectory (1.1M step instances, no far step wrong).
//
// Validity.  Producers classify from an approximate nominal value V (a double
// prefix of add * 10^(13-F) from the window's estimated start).  Per tile they
// record the slack of the classification -- the smallest distance of a far
// step's V to a decade boundary, the floor, the ceiling, and |V| 2^-17 (which
// bounds the binade of the rounding band) -- and how far the integer nominal
// may drift from V inside the tile.  The chain commits a tile only when the
// exact state's distance from V (known exactly at the tile start, plus the
// drift and the resolved near offsets) stays inside that slack, and when no
// allow or clamp is possible.  Any other tile is replayed exactly
// (exact_span_x); k_tb_expand replays every committed run exactly again and
// checks its end state.  So, as in one-decade windows, every result comes
// from an exact step on its exact predecessor.
#pragma once

namespace rl {

// the multi-decade work runs out of line in the chain kernel (see
// ch_resolve_x in rl_tb_chain.h); RL_XDEC_OOL=0 inlines it (A/B only)
#ifndef RL_XDEC_OOL
#define RL_XDEC_OOL 1
#endif
#if RL_XDEC_OOL
#define XDEC_FN __attribute__((noinline))
#else
#define XDEC_FN __attribute__((always_inline)) inline
#endif

constexpr int XDEC_FMIN = -9;          // 10^(13 - F) must be an exact double: 13 - F <= 22
constexpr int XDEC_FMAX = 8;           // decades F .. F + 4 <= 12
constexpr int16_t XRUN = 1000;         // TbRuns::E of a run committed in an XDEC window: F + XRUN
constexpr uint64_t X_T14 = 100000000000000ull, X_T15 = 1000000000000000ull, X_T16 = 10000000000000000ull,
                   X_T17 = 100000000000000000ull;

// decade of |X| above the floor: 0..4 for |X| in [1e13, 1e18)
__device__ inline int xk_of(uint64_t ax) {
    return (int)(ax >= X_T14) + (int)(ax >= X_T15) + (int)(ax >= X_T16) + (int)(ax >= X_T17);
}
__device__ inline int xk_of_d(double a) {
    return (int)(a >= 1e14) + (int)(a >= 1e15) + (int)(a >= 1e16) + (int)(a >= 1e17);
}
// 10^k and 10^-k, k in [0, 4], by selects (no lane-indexed memory)
__device__ inline int64_t xp10_i(int k) {
    int64_t p = 1;
    p = k >= 1 ? 10 : p;
    p = k >= 2 ? 100 : p;
    p = k >= 3 ? 1000 : p;
    p = k >= 4 ? 10000 : p;
    return p;
}
__device__ inline double xp10_d(int k) {
    double p = 1.0;
    p = k >= 1 ? 10.0 : p;
    p = k >= 2 ? 100.0 : p;
    p = k >= 3 ? 1000.0 : p;
    p = k >= 4 ? 10000.0 : p;
    return p;
}
__device__ inline double xp10_inv(int k) {   // inexact beyond k = 0: only ever rounded after
    double p = 1.0;
    p = k >= 1 ? 0.1 : p;
    p = k >= 2 ? 0.01 : p;
    p = k >= 3 ? 0.001 : p;
    p = k >= 4 ? 0.0001 : p;
    return p;
}

// A window's scale: PF = 10^(13 - F) and the scale of each of its decades,
// P[k] = 10^(13 - F - k) (all exact doubles; wave-uniform).  A lane's decade
// scale is computed, not indexed: P[k] = P4 10^(4 - k) exactly, and its
// reciprocal R0 10^k, within 2^-52 of 1 / P[k] (div_p10's bound).  An indexed
// pick from the array made the compiler keep it in scratch memory inside the
// out-of-line multi-decade resolve: four dependent scratch loads per near pass.
struct XScale {
    double P[5];
    double P4;     // P[4]
    double R0;     // RN(1 / P[0])
    int32_t F;
};
__device__ inline XScale xscale(int32_t F) {
    XScale s;
    s.F = F;
#pragma unroll
    for (int k = 0; k < 5; k++) s.P[k] = rlq::pow10_exact(13 - F - k);
    s.P4 = s.P[4];
    s.R0 = 1.0 / s.P[0];
    return s;
}
__device__ inline double xpick(const XScale& s, int k) { return s.P4 * xp10_d(4 - k); }
__device__ inline double xpick_r(const XScale& s, int k) { return s.R0 * xp10_d(k); }

// One Redis-7 script step (tokenbucket.go:32-48) on a state X of a window with
// floor F: strtod of the stored digits, the sum, %.14g of the result.  True
// with the next state in Xn and the unquantized tokens; false when the step
// leaves the window's regime: sum >= th (an allow or a clamp: n and the
// capacity decide, tb_eval), an expired key (add NaN) or a result outside the
// decades [F, F + 4] (or below 1e-9: no exact scale).  up: the result's
// decade is above the input's.
// Xin: the state the step actually started from -- X itself when X is a
// state (a multiple of its decade's unit), else the state X rounds to (the
// chain's guesses need not be states: changes are measured from Xin, so a
// guess that rounds onto the right state yields the right change).
__device__ __attribute__((always_inline)) inline bool xstep(int64_t X, const XScale& xs, double add, double th,
                                                           int64_t& Xn, double& tokens, bool& up, int64_t& Xin) {
    const uint64_t ax = X < 0 ? (uint64_t)(-X) : (uint64_t)X;
    const int kin = xk_of(ax);
    // the stored digits: D = X / 10^kin exactly (X is a multiple of it; the
    // product's error is below 0.05: (double)X is within ulp / 2 <= 64 of X
    // and the scaled value below 1e14 within 2^-52 relative)
    const double Dd = rint((double)X * xp10_inv(kin));
    Xin = (int64_t)Dd * xp10_i(kin);
    // strtod("D e(E-13)"): |D| < 2^47 and the decade's scale is an exact power
    // of ten, so one correctly rounded division is strtod (Clinger): div_p10
    const double T = div_p10(Dd, xpick(xs, kin), xpick_r(xs, kin));
    const double sum = T + add;
    tokens = sum;
    // %.14g's decade on the exact scaled value (as tb_dec_step), starting at
    // the decade the window's scale suggests; a second decade only when the
    // first misses (a wave-uniform branch: the near passes and exact tiles
    // step every lane, so the common path carries no divergent branches)
    const double a = sum < 0.0 ? -sum : sum;
    int k = xk_of_d(a * xs.P[0]);
    double P = xpick(xs, k);
    double p = a * P, err = __builtin_fma(a, P, -p);     // a*P == p + err exactly
    bool lo_ok = (p > 1e13) | ((p == 1e13) & (err >= 0.0));
    bool hi_ok = (p < 1e14) | ((p == 1e14) & (err < 0.0));
    bool kin_range = true;
    if (__ballot(!(lo_ok & hi_ok)) != 0ull) {
        const bool again = !(lo_ok & hi_ok);
        const int k2 = k + (lo_ok ? 1 : -1);
        kin_range = !again || (k2 >= 0 && k2 <= 4);      // outside the window's decades: not this regime
        k = again ? k2 : k;
        P = xpick(xs, k);
        const double p2 = a * P, e2 = __builtin_fma(a, P, -p2);
        p = again ? p2 : p;
        err = again ? e2 : err;
        lo_ok = (p > 1e13) | ((p == 1e13) & (err >= 0.0));
        hi_ok = (p < 1e14) | ((p == 1e14) & (err < 0.0));
    }
    // RNE of p; the exact product decides a tie of p
    double d = rint(p);
    const double h = p - d;
    d += ((h == 0.5) & (err > 0.0)) ? 1.0 : ((h == -0.5) & (err < 0.0)) ? -1.0 : 0.0;
    const bool carry = d == 1e14;                        // rounding carried into the next decade
    d = carry ? 1e13 : d;
    k += carry ? 1 : 0;
    const int64_t v = (int64_t)d * xp10_i(k);
    const bool zero = a == 0.0;                          // tostring(0) == "0"
    const bool ok = (sum < th) && (zero || (kin_range && lo_ok && hi_ok && k <= 4));
    Xn = !ok ? Xn : zero ? 0 : (sum < 0.0 ? -v : v);
    up = ok && !zero && X != 0 && k > kin;
    return ok;
}

// inclusive segmented scan over the wave: a lane with f set starts a segment
// with its own v; lanes before the first segment add to base
// (S, the scan of the other lanes' v, plus T, the offset of the lane's
// segment: v - S at its start lane, base before any; T travels forward by the
// DPP scan steps of wave_incl_scan_i64, a segment start keeping its own -- no
// LDS round trips, where lane-indexed shuffles cost four ds_bpermute)
template <int CTRL, int RM>
__device__ inline int64_t dpp_i64(int64_t v, int64_t old) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)v, CTRL, RM, 0xf,
                                                              false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)((uint64_t)old >> 32),
                                                              (int)(uint32_t)((uint64_t)v >> 32), CTRL, RM, 0xf, false);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
template <int CTRL, int RM>
__device__ inline void seg_step(int64_t& T, uint32_t& h) {
    const uint32_t nh = dpp32<CTRL, RM>(h, 0u);
    const int64_t nT = dpp_i64<CTRL, RM>(T, 0);
    T = (h == 0u && nh != 0u) ? nT : T;
    h |= nh;
}
__device__ inline int64_t seg_incl_scan_i64(bool f, int64_t v, int64_t base) {
    const int64_t S = wave_incl_scan_i64(f ? 0 : v);
    int64_t T = f ? v - S : base;
    uint32_t h = f ? 1u : 0u;
    seg_step<0x111, 0xf>(T, h);   // row_shr:1
    seg_step<0x112, 0xf>(T, h);   // row_shr:2
    seg_step<0x114, 0xf>(T, h);   // row_shr:4
    seg_step<0x118, 0xf>(T, h);   // row_shr:8
    seg_step<0x142, 0xa>(T, h);   // row_bcast:15 -> rows 1, 3
    seg_step<0x143, 0xc>(T, h);   // row_bcast:31 -> rows 2, 3
    return T + S;
}
// the value of the lane before (lane 0: first) -- DPP wave_shr:1
__device__ inline int64_t wave_prev_i64(int64_t v, int64_t first) { return dpp_i64<0x138, 0xf>(v, first); }
__device__ inline int32_t wave_prev_i32(int32_t v, int32_t first) {
    return (int32_t)dpp32<0x138, 0xf>((uint32_t)v, (uint32_t)first);
}


// Exact replay of [p, p + len) (len <= CH_TILE) from the exact state X0 of a
// window with floor xs.F by one wave (the multi-decade exact_span): lane l
// steps requests [p + K l, p + K l + K) from a guessed start state.  A lane
// whose steps went a decade up reports its end state (a coarser rounding
// forgets small errors of the start), the others their change; a segmented
// scan gives every lane its next guess, and when no guess changes before the
// first lane that leaves the regime, every guess up to there is exact
// (induction over lanes).  Returns the relative position of the first step
// that leaves the regime (len if none) and in Xend the exact state before it.
// OUT: writes tokens and DENIED for every in-regime step.
template <bool OUT, typename Src>
__device__ __attribute__((always_inline)) inline uint32_t exact_span_x(const Src& src, uint32_t p, uint32_t len,
                                                                       int64_t X0, const XScale& xs, int64_t& Xend,
                                                                       const ReqArgs& a, uint32_t& iters) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t off = lane * K;
    const uint32_t nv = off < len ? ((len - off) < (uint32_t)K ? (len - off) : (uint32_t)K) : 0u;
    double add[K], th[K];
    double SA = 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nv;
        add[q] = v ? src.add(p + off + q) : 0.0;
        th[q] = v ? src.th(p + off + q) : __builtin_inf();
        const double A = add[q] * xs.P[0];
        SA += fabs(A) < 0x1p62 ? A : 0.0;          // NaN / huge: a regime exit anyway
    }
    // first guesses: the double prefix of the adds (the integer states follow
    // within the roundings; the fixed point corrects them)
    const double ex = wave_incl_scan_f64(SA) - SA;
    int64_t st = X0 + (lane ? (int64_t)rint(fmin(fmax(ex, -0x1p62), 0x1p62)) : 0);
    const uint32_t last = len ? (len - 1) / K : 0u;
    for (uint32_t it = 0;; it++) {
        if (it > 70u) {            // cannot happen (one more exact lane per pass); never hang on it
            Xend = X0;
            return 0xffffffffu;
        }
        int64_t X = st, Xb = 0, X0e = st;
        uint32_t bq = NO_STOP;
        bool anyup = false;
#pragma unroll
        for (int q = 0; q < K; q++) {
            const bool act = (uint32_t)q < nv && bq == NO_STOP;
            int64_t Xn = X, Xin;
            double tk;
            bool up;
            const bool ok = xstep(X, xs, add[q], th[q], Xn, tk, up, Xin);
            if (q == 0) X0e = Xin;                     // the state the lane's steps start from
            const bool stop = act && !ok;
            const bool take = act && ok;
            bq = stop ? (uint32_t)q : bq;
            Xb = stop ? X : Xb;
            anyup |= take && up;
            if (OUT && take) {
                a.tok[p + off + q] = tk;
                a.dec[p + off + q] = DEC_DENIED;
            }
            X = take ? Xn : X;
        }
        const bool brk = bq != NO_STOP;
        const bool rs = anyup && !brk;
        // changes from the state the lane really started from (its guess
        // rounded onto a state): independent of the guess for far steps
        const int64_t incl = seg_incl_scan_i64(rs, rs ? X : (brk ? 0 : X - X0e), X0);
        const int64_t nst = wave_prev_i64(incl, X0);
        const uint32_t fb = first_lane(__ballot(brk));
        const uint32_t fd = first_lane(__ballot(nv > 0 && nst != st));
        iters++;
        if (fb == 64u ? fd == 64u : fd > fb) {
            if (fb < 64u) {
                Xend = readlane_i64(Xb, fb);
                return fb * K + (uint32_t)__builtin_amdgcn_readlane((int)bq, (int)fb);
            }
            Xend = readlane_i64(X, last);
            return len;
        }
        st = nst;
    }
}

// ---------------------------------------------------------------------------
// window plan and producers
// ---------------------------------------------------------------------------
// The plan of a window [first, first + cnt) from an estimate v0 (tokens) of
// its start state: every producer wave computes the same from the ring (the
// same instructions on the same data).  One decade (QM_DEC at E) when the
// envelope of the nominal path -- per tile its start plus the positive /
// negative parts of its adds -- stays positive inside one decade; else
// QM_XDEC with the floor four decades below the envelope's top; QM_NONE when
// neither fits (a state beyond 1e12 tokens or a non-finite estimate).
struct XPlan {
    int32_t mode;
    int32_t E;                 // DEC: the decade; XDEC: the floor F
    double vt[CH_NP];          // estimated value (tokens) at each tile's start
};

__device__ __attribute__((always_inline)) inline XPlan ch_plan(const ChainShared& sh, uint32_t first, uint32_t cnt,
                                                              double v0) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    XPlan pl;
    double v = v0, lo = v0, hi = v0;
#pragma unroll
    for (int t = 0; t < CH_NP; t++) {
        pl.vt[t] = v;
        double s = 0.0, sp = 0.0;
        double ra[K], rt[K];
        ring_read_k(sh, first + (uint32_t)t * CH_TILE + lane * K, ra, rt);
#pragma unroll
        for (int q = 0; q < K; q++) {
            const uint32_t o = (uint32_t)t * CH_TILE + lane * K + q;
            const double ad = ra[q];
            const double x = (o < cnt && fabs(ad) < 1e300) ? ad : 0.0;
            s += x;
            sp += x > 0.0 ? x : 0.0;
        }
        const double S = wave_reduce_f64(s, 0.0, [](double x, double y) { return x + y; });
        const double Sp = wave_reduce_f64(sp, 0.0, [](double x, double y) { return x + y; });
        hi = fmax(hi, v + Sp);
        lo = fmin(lo, v - (Sp - S));
        v += S;
    }
    pl.mode = QM_NONE;
    pl.E = 0;
    if (!(lo == lo) || !(hi == hi) || !(fabs(lo) < 1e12) || !(fabs(hi) < 1e12)) return pl;
    if (lo > 0.0) {
        const int E = (int)floor(log10(lo));
        if (E >= -9 && E <= 12 && lo > rlq::pow10_exact(E + 9) * 1e-9 * (1.0 + 1e-12) &&
            hi < rlq::pow10_exact(E + 10) * 1e-9 * (1.0 - 1e-12)) {
            pl.mode = QM_DEC;
            pl.E = E;
            return pl;
        }
    }
    const double m = fmax(fabs(lo), fabs(hi));
    const int Et = m > 0.0 ? (int)floor(log10(m)) : XDEC_FMIN + 4;
    const int F = max(Et - 4, XDEC_FMIN);
    if (F > XDEC_FMAX) return pl;
    pl.mode = QM_XDEC;
    pl.E = F;
    return pl;
}

// The same plan with the window's tiles split over the producer waves: wave
// pw sums tile pw alone (one ring read, two reductions instead of six and
// twelve), publishes its sums in LDS under the round's plan number `seq`, and
// every wave combines the six tiles in tile order -- the same operations on
// the same values as ch_plan, so the same plan.  All producer waves make the
// same sequence of plan calls (the plan's condition is block-uniform), so
// their seq counters agree.  A wave whose wait passes a bound (never
// expected) computes the whole plan itself.
__device__ __attribute__((always_inline)) inline XPlan ch_plan_par(ChainShared& sh, uint32_t first, uint32_t cnt,
                                                                  double v0, uint32_t pw, uint32_t seq) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    {
        double s = 0.0, sp = 0.0;
        double ra[K], rt[K];
        ring_read_k(sh, first + pw * CH_TILE + lane * K, ra, rt);
#pragma unroll
        for (int q = 0; q < K; q++) {
            const uint32_t o = pw * CH_TILE + lane * K + q;
            const double ad = ra[q];
            const double x = (o < cnt && fabs(ad) < 1e300) ? ad : 0.0;
            s += x;
            sp += x > 0.0 ? x : 0.0;
        }
        const double S = wave_reduce_f64(s, 0.0, [](double x, double y) { return x + y; });
        const double Sp = wave_reduce_f64(sp, 0.0, [](double x, double y) { return x + y; });
        if (lane == 0) {
            sh.plan_s[pw] = S;
            sh.plan_sp[pw] = Sp;
            __hip_atomic_store(&sh.plan_tag[pw], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    bool ok = true;
#pragma unroll
    for (int t = 0; t < CH_NP; t++) {
        uint32_t spins = 0;
        while (__hip_atomic_load(&sh.plan_tag[t], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != seq) {
            if (++spins > (1u << 20)) { ok = false; break; }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    if (!ok) return ch_plan(sh, first, cnt, v0);
    XPlan pl;
    double v = v0, lo = v0, hi = v0;
#pragma unroll
    for (int t = 0; t < CH_NP; t++) {
        pl.vt[t] = v;
        const double S = sh.plan_s[t], Sp = sh.plan_sp[t];
        hi = fmax(hi, v + Sp);
        lo = fmin(lo, v - (Sp - S));
        v += S;
    }
    pl.mode = QM_NONE;
    pl.E = 0;
    if (!(lo == lo) || !(hi == hi) || !(fabs(lo) < 1e12) || !(fabs(hi) < 1e12)) return pl;
    if (lo > 0.0) {
        const int E = (int)floor(log10(lo));
        if (E >= -9 && E <= 12 && lo > rlq::pow10_exact(E + 9) * 1e-9 * (1.0 + 1e-12) &&
            hi < rlq::pow10_exact(E + 10) * 1e-9 * (1.0 - 1e-12)) {
            pl.mode = QM_DEC;
            pl.E = E;
            return pl;
        }
    }
    const double m = fmax(fabs(lo), fabs(hi));
    const int Et = m > 0.0 ? (int)floor(log10(m)) : XDEC_FMIN + 4;
    const int F = max(Et - 4, XDEC_FMIN);
    if (F > XDEC_FMAX) return pl;
    pl.mode = QM_XDEC;
    pl.E = F;
    return pl;
}

// ulp of a positive normal double
__device__ inline double ulp_pos(double z) {
    const int64_t e = (__double_as_longlong(z) >> 52) & 0x7ff;
    return __longlong_as_double((e > 52 ? e - 52 : 1) << 52);
}

// Summary of tile t of an XDEC window [pfirst, pfirst + pcnt) with floor xs.F,
// the tile's start estimated at vt tokens: into tile[buf][t] -- S the nominal
// sum of r (exact int64), ymin = min (th PF Y - V') over the tile (V' the
// estimated result), cmax = V at the tile's start (X units), cmin = the drift
// bound sum |r - A|, dmax = the classification slack (see the header), ev,
// nc -- its near list (the integer nominal before each near step relative to
// the tile start in ne_pred, its add, its r in ne_th, kind bits in ne_kind)
// and the per-lane near ranks.
__device__ __attribute__((always_inline)) inline void ch_produce_x(ChainShared& sh, uint32_t buf, uint32_t t,
                                                                  uint32_t pfirst, uint32_t pcnt, const XScale& xs,
                                                                  double vt) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t toff = t * CH_TILE;
    if (toff >= pcnt) return;
    const uint32_t myoff = toff + lane * K;
    const uint32_t nv = myoff < pcnt ? ((pcnt - myoff) < (uint32_t)K ? (pcnt - myoff) : (uint32_t)K) : 0u;
    const uint32_t i0 = pfirst + myoff;
    const double PF = xs.P[0], uinv = 1.0 / PF;
    const double PY = PF * CH_YSCALE;
    double add[K], th[K], A[K];
    double SA = 0.0;
    uint32_t evq = NO_STOP;
    ring_read_k(sh, i0, add, th);
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nv;
        add[q] = v ? add[q] : 0.0;
        const double a2 = add[q] * PF;
        const bool ok = fabs(a2) < 0x1p62;                 // else NaN (expired key) or huge: a stop
        evq = (v && !ok && evq == NO_STOP) ? (uint32_t)q : evq;
        A[q] = ok ? a2 : 0.0;
        SA += A[q];
    }
    const double Vl = vt * PF + (wave_incl_scan_f64(SA) - SA);   // estimated state before my first step
    double V = Vl;
    int64_t r[K];
    int64_t Sr = 0;
    uint32_t nearm = 0, resm = 0;
    // The chain's commit test allows a fixed 4096 units for the rounding of
    // V (rl_tb_chain.h ch_resolve_x).  That margin holds while every state
    // estimate and vt PF stay below 2^60: the partial sums of A are then
    // differences of two of them (< 2^61), every one of the 2K + 8 roundings
    // on the way to a V is at most ulp(2^61) / 2 = 128 units (2560 in all),
    // and the test's own conversions and subtractions add under 512.  A tile
    // that reaches 2^60 anywhere gets slack -inf: it is never committed, the
    // chain replays it exactly.
    double ymin = __builtin_inf(), slack = fabs(Vl) < 0x1p60 && fabs(vt * PF) < 0x1p60 ? __builtin_inf()
                                                                                        : -__builtin_inf();
    double dev = 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nv;
        const double Vo = V + A[q];
        const double avi = fabs(V), avo = fabs(Vo);
        slack = (v && !(avo < 0x1p60)) ? -__builtin_inf() : slack;
        const int kin = xk_of_d(avi), kout = xk_of_d(avo);
        const double g = xp10_d(kout);
        // the exact add * 10^(13 - E') (E' = F + kout: in units of the
        // result's decade) against its nearest integer, as ch_produce does
        const double Po = xpick(xs, kout);
        const double f = add[q] * Po;
        const bool big = !(fabs(f) < 0x1p49);
        const double fs = big ? 0.0 : f;
        const double rr = rint(fs);
        const double fr = (fs - rr) + (big ? 0.0 : __builtin_fma(add[q], Po, -f));
        r[q] = (int64_t)rr * xp10_i(kout);
        // rounding band of strtod(x) and of the sum, in units of the result's
        // decade, from the binades of the largest plausible x and sum (the
        // exact states stay within |V| 2^-17 of V: the slack below)
        const double bx = ulp_pos((avi * (1.0 + 0x1p-16) + 1.0) * uinv) * PF;
        const double bs = ulp_pos((avo * (1.0 + 0x1p-16) + g) * uinv) * PF;
        const double band = (bx + bs) * 0.5 / g;
        const bool inr = avi >= 1e13 && avo >= 1e13 && avo < 1e18;
        const bool up = kout > kin;
        const bool nr = big || !inr || up || kin - kout >= 2 || fabs(fr) > 0.5 - band - 0x1p-40;
        nearm |= (v && nr) ? 1u << q : 0u;
        resm |= (v && nr && (up || avi < 1e13)) ? 1u << q : 0u;
        if (v && !nr) {
            // distance of both states to the decade boundaries, the floor and
            // the ceiling, and the binade margin of the band
            double d = fmin(avi * 0x1p-17, avo * 0x1p-17);
            d = fmin(d, fmin(avi - 1e13, 1e18 - avo));
            d = fmin(d, fmin(fabs(avi - 1e14), fabs(avo - 1e14)));
            d = fmin(d, fmin(fabs(avi - 1e15), fabs(avo - 1e15)));
            d = fmin(d, fmin(fabs(avi - 1e16), fabs(avo - 1e16)));
            d = fmin(d, fmin(fabs(avi - 1e17), fabs(avo - 1e17)));
            slack = fmin(slack, d);
        }
        if (v) {
            ymin = fmin(ymin, th[q] * PY - Vo);
            dev += fabs((double)r[q] - A[q]);
        }
        Sr += v ? r[q] : 0;
        V = Vo;
    }
    const int64_t incl = wave_incl_scan_i64(Sr);
    const int64_t ex = incl - Sr;
    const double ymin_t = wave_reduce_f64(ymin, __builtin_inf(), [](double x, double y) { return vmin_f64(x, y); });
    const double slack_t = wave_reduce_f64(slack, __builtin_inf(), [](double x, double y) { return vmin_f64(x, y); });
    const double dev_t = wave_reduce_f64(dev, 0.0, [](double x, double y) { return x + y; });
    const uint32_t ev_t = wave_min_u32(evq != NO_STOP ? lane * K + evq : NO_STOP);
    const uint32_t ncnt = (uint32_t)__popc(nearm);
    const uint32_t ninc = wave_scan_u32(ncnt, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    sh.ne_rank[buf][t][lane] = (uint16_t)(ninc - ncnt);
    // reset kinds of the tile's near entries: bit k of ne_kind[buf][t]
    uint64_t kb = 0;
    if (nearm) {
        uint32_t k = ninc - ncnt;
        int64_t cb = ex;
#pragma unroll
        for (int q = 0; q < K; q++) {
            if ((nearm >> q) & 1u) {
                if (k < (uint32_t)CH_NE) {
                    sh.ne_pred[buf][t][k] = __longlong_as_double(cb);
                    sh.ne_add[buf][t][k] = add[q];
                    sh.ne_th[buf][t][k] = __longlong_as_double(r[q]);
                    kb |= ((resm >> q) & 1u) ? 1ull << k : 0ull;
                }
                k++;
            }
            cb += (uint32_t)q < nv ? r[q] : 0;
        }
    }
    // OR of the lanes' kind bits (each entry's bit set by one lane)
    uint32_t klo = (uint32_t)kb, khi = (uint32_t)(kb >> 32);
    klo = wave_scan_u32(klo, 0u, [](uint32_t x, uint32_t y) { return x | y; });
    khi = wave_scan_u32(khi, 0u, [](uint32_t x, uint32_t y) { return x | y; });
    if (lane == 63) {
        sh.ne_kind[buf][t] = ((uint64_t)khi << 32) | klo;
        ChTile& T = sh.tile[buf][t];
        T.S = incl;
        T.Sd = (double)incl;
        T.ymin = ymin_t;
        T.cmax = vt * PF;
        T.cmin = dev_t;
        T.dmax = slack_t;
        T.ev = ev_t;
        T.nc = ninc;
    }
}

// an estimate of the state (tokens) for a window's plan
__device__ inline double st_value(int64_t D, int32_t E, int32_t mode) {
    if (mode == QM_XDEC) return (double)D / rlq::pow10_exact(13 - E);
    if (D == 0 || E < -9 || E > 13) return 0.0;
    return (double)D / rlq::pow10_exact(13 - E);
}

// The exact state as stored digits (D, E): a window's representation -> a
// stored value's (DEC: D in the decade E already; XDEC: X in floor F)
__device__ inline void x_to_dec(int64_t X, int32_t F, int64_t& D, int32_t& E) {
    if (X == 0) {
        D = 0;
        E = 0;
        return;
    }
    const uint64_t ax = X < 0 ? (uint64_t)(-X) : (uint64_t)X;
    const int k = xk_of(ax);
    const int64_t d = (int64_t)(ax / (uint64_t)xp10_i(k));
    D = X < 0 ? -d : d;
    E = F + k;
}
// stored digits (D, E) -> the representation of a window (mode, E or F);
// false when the state does not fit it
__device__ inline bool dec_to_win(int64_t D, int32_t E, int32_t wmode, int32_t wE, int64_t& out) {
    if (wmode == QM_DEC) {
        out = D;
        return D >= DEC_LO && D < DEC_HI && E == wE;
    }
    if (wmode == QM_XDEC) {
        if (D == 0) {
            out = 0;
            return true;
        }
        const int k = E - wE;
        if (k < 0 || k > 4) return false;
        out = D * xp10_i(k);
        return true;
    }
    return false;
}

}  // namespace rl
