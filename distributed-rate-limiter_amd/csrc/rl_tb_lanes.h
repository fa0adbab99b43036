// rl_tb_lanes.h -- block-cooperative token-bucket replay of one heavy
// (Zipf hot-key) segment.  Included by rl_replay.h after its helpers.
//
// What is replayed: the reference's token-bucket script step
// (tokenbucket.go:23-52 + the Go arithmetic at :114-130), request by request
// in arrival order, on one key.  The carried state is the STORED tokens value,
// which Lua's tostring quantizes (tokenbucket.go:48): under Redis 7 to 14
// significant decimal digits, i.e. an integer D in [1e13, 1e14) in a decade E
// (value = D * 10^(E-13)); under miniredis to the exact double, an integer
// mantissa D in [2^52, 2^53) in a binade E.
//
// Step algebra (u = the unit of D).  With T = strtod(D*u) and
// sum = RN(T + add), the next stored state is D' = round(sum / u) =
// round(D + add/u + delta) with |delta| <= (D + D') * 2^-53 < 0.0223 (two
// correct roundings of values below 1e14 u).  D is an integer, so whenever
// add/u is farther than (|D| + |D'|) 2^-53 (<= 0.0223, TAU_DEC = 0.03 as the
// state-free first cut) from a half-integer (a "far" step),
// D' = D + r with r = rint(add/u) for EVERY predecessor D in the decade: the
// step is an integer add, independent of the state.  Only "near" steps (about
// 6% of them) depend on the exact predecessor.
//
// Negative stored states (the reference does not clamp a negative elapsed
// time, tokenbucket.go:36-37, and last_refill is itself quantized to 14
// digits) are handled symmetrically: D is signed, |D| in the decade.
//
// One round covers a window of NC*K consecutive requests; lane L owns the K
// requests [L*K, L*K+K) of it.  The round resolves only the STATE CHAIN:
//   A. each lane computes r_q and the near flag of its K steps (state free);
//   B. block exclusive scan of the lane sums of r -> every lane's NOMINAL
//      start state; the true start differs by a small integer offset;
//   C. fixed-point iteration on the start offsets: a lane's end offset is its
//      start offset carried through its steps -- unchanged by far steps, and
//      through each near step by evaluating it exactly at the current
//      guess; a block scan of the (end - start) deltas gives the next guess.
//      When no delta changes, the guesses are a fixed point and, by
//      induction over lanes, the TRUE starts (typically 1-2 iterations);
//   D. with true starts, every request's next state D' is known exactly
//      (far: D + r, near: evaluated); the first request that may leave the
//      regime (allow, clamp at capacity, decade change, expired key) stops
//      the round -- exactly for the decade, conservatively (|error| < 2
//      units) for allow / clamp;
//   E. the stop request is run exactly (any regime) by its owner, which
//      publishes the next base; every lane records its committed run
//      {position, length, exact start state, exact end state}.
// k_tb_expand then replays every recorded run exactly and in parallel over
// the whole GPU -- the per-request outputs (decision, unquantized tokens) are
// produced there, off the chain's critical path -- and checks that each run
// ends in the state the chain recorded (EF_INTERNAL otherwise).  So every
// result still comes from an exact step on its exact predecessor, and the
// bound above is verified, never trusted silently.
//
// Data movement: one loader wave per block streams the segment's inputs
// (add, n|cfg) from HBM into an LDS ring ahead of the window, so compute
// waves never wait on a global load.
#pragma once

namespace rl {

constexpr int64_t DEC_LO = 10000000000000LL, DEC_HI = 100000000000000LL;
constexpr int64_t BIN_LO = 1LL << 52, BIN_HI = 1LL << 53;
constexpr uint32_t NO_STOP = 0xffffffffu;

// LDS ordering fence for a wave's own buffers (DS ops of one wave complete
// in order; this keeps the compiler from reordering around it)
__device__ inline void wave_lds_fence() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// cooperative replay geometry: NC compute lanes (7 waves) + 1 loader wave
constexpr int TB_NC = 448;
constexpr int TB_K = 8;                          // requests per lane per round
constexpr int TB_NW = TB_NC / 64;
constexpr uint32_t TB_WIN = (uint32_t)TB_NC * TB_K;
// LDS ring of request inputs, by absolute sorted position; padded so that
// lanes reading positions l*K+q (fixed q) hit distinct banks
constexpr uint32_t RING = 8192;
constexpr uint32_t RING_SLOTS = RING + RING / TB_K;
__host__ __device__ constexpr uint32_t ring_idx(uint32_t p) {
    return (p & (RING - 1)) + ((p & (RING - 1)) / TB_K);
}
static_assert(RING >= 2 * TB_WIN, "the ring must hold the next window while the current one is read");

struct LaneShared {
    double r_add[RING_SLOTS];
    uint64_t r_nc[RING_SLOTS];   // TbPre::nc
    int64_t wtot[TB_NW];         // lane-sum scan
    int64_t itot[TB_NW];         // offset-delta scan (per iteration)
    uint32_t ich[TB_NW];         // first lane whose delta changed
    uint32_t ibk[TB_NW];         // first lane that breaks
    uint32_t wmin[TB_NW];        // first stop
    int64_t baseD[2];            // round-parity double buffer
    int32_t baseE[2];
    uint32_t first[2];
};

// The loader wave: streams TbPre::{add, nc} of the segment into the ring,
// up to RING positions ahead of the current window.  Each pump() retires the
// chunk issued by the previous pump (its latency elapsed behind a compute
// phase) into LDS and issues the next one; pump() runs in every gap between
// two block barriers, so the loader keeps pace with no wait of its own.  It
// writes only positions >= the window's end, i.e. ring slots of positions
// already consumed.
constexpr int LD_CH = 4;                 // 128-position chunks per pump
struct TbLoader {
    uint32_t fill;                       // positions < fill are in the ring (even unless == j1)
    uint32_t pg, pend_end;               // issued, not yet written: [pg, pend_end)
    bool pend;
    double2 pa[LD_CH];
    ulonglong2 pn[LD_CH];
};

__device__ __attribute__((always_inline)) inline void ld_retire(TbLoader& L, LaneShared& sh, uint32_t lane) {
    if (!L.pend) return;
#pragma unroll
    for (int c = 0; c < LD_CH; c++) {
        const uint32_t g = L.pg + c * 128 + 2 * lane;
        if (g < L.pend_end) {
            sh.r_add[ring_idx(g)] = L.pa[c].x;
            sh.r_nc[ring_idx(g)] = L.pn[c].x;
        }
        if (g + 1 < L.pend_end) {
            sh.r_add[ring_idx(g + 1)] = L.pa[c].y;
            sh.r_nc[ring_idx(g + 1)] = L.pn[c].y;
        }
    }
    L.fill = L.pend_end;
    L.pend = false;
}

__device__ __attribute__((always_inline)) inline void ld_issue(TbLoader& L, uint32_t limit, const TbPre& pre, uint32_t lane) {
    if (L.pend || L.fill >= limit) return;
    L.pg = L.fill;
    L.pend_end = (limit - L.fill) < (uint32_t)(LD_CH * 128) ? limit : L.fill + LD_CH * 128;
#pragma unroll
    for (int c = 0; c < LD_CH; c++) {
        const uint32_t g = L.pg + c * 128 + 2 * lane;     // even: 16-byte aligned pair
        if (g < L.pend_end) {
            L.pa[c] = *reinterpret_cast<const double2*>(pre.add + g);
            L.pn[c] = *reinterpret_cast<const ulonglong2*>(pre.nc + g);
        }
    }
    L.pend = true;
}

// fill limit for a window starting at `first`: RING ahead, even-aligned
__device__ __attribute__((always_inline)) inline uint32_t ld_limit(uint32_t first, uint32_t j1) {
    const uint32_t lim = (first + RING) & ~1u;
    return lim < j1 ? lim : j1;
}

__device__ __attribute__((always_inline)) inline void ld_pump(TbLoader& L, LaneShared& sh, uint32_t first, uint32_t j1, const TbPre& pre,
                               uint32_t lane) {
    ld_retire(L, sh, lane);
    ld_issue(L, ld_limit(first, j1), pre, lane);
}

// synchronous: make sure [.., target) is in the ring (the next window)
__device__ __attribute__((always_inline)) inline void ld_until(TbLoader& L, LaneShared& sh, uint32_t first, uint32_t target, uint32_t j1,
                                const TbPre& pre, uint32_t lane) {
    const uint32_t lim = ld_limit(first, j1);
    if (target > lim) target = lim;
    while (L.fill < target) {
        ld_retire(L, sh, lane);
        ld_issue(L, lim, pre, lane);
    }
    ld_retire(L, sh, lane);
    ld_issue(L, lim, pre, lane);
}

// RNE(x * P) as an exact integer-valued double (x*P < 2^52), P = 10^k exact
__device__ inline double round_scaled_Pd(double x, double P) {
    const double p = x * P;
    const double err = __builtin_fma(x, P, -p);       // x*P == p + err exactly
    const double d0 = floor(p);
    const double f = p - d0;                          // exact
    const bool odd = d0 * 0.5 != floor(d0 * 0.5);
    const bool up = (f > 0.5) || (f == 0.5 && ((err > 0.0) || (err == 0.0 && odd)));
    return up ? d0 + 1.0 : d0;
}

// The live-key step in a fast mode with the (signed) state digits as an
// exact integer-valued double: tokens (the unquantized double) and the stored
// digits D' (NaN when tokens leaves the (decade, clamp, allow) regime).
template <int MODE>
__device__ inline double tb_step_d(double Dpred, double P, double R, double add, double cap, double nd,
                                   double& tokens) {
    double T;
    if (MODE == QM_DEC) {
        const double t = rlq::div_pow10(fabs(Dpred), P, R);         // strtod("D e(E-13)")
        T = Dpred < 0.0 ? -t : t;
    } else {
        T = Dpred * R;                                              // exact: R = 2^E
    }
    const double sum = T + add;
    tokens = sum;
    const double as = fabs(sum);
    double Dn;
    if (MODE == QM_DEC) {
        Dn = round_scaled_Pd(as, P);                                // %.14g: symmetric RNE
        if (!(Dn >= (double)DEC_LO && Dn < (double)DEC_HI)) Dn = __builtin_nan("");
    } else {
        Dn = as * P;                                                // exact scaling
        if (!(Dn >= (double)BIN_LO && Dn < (double)BIN_HI && Dn == floor(Dn))) Dn = __builtin_nan("");
    }
    if (sum < 0.0) Dn = -Dn;
    // math.min(capacity, sum) and the allow test: either one leaves the regime
    if (!(sum < cap) || !(sum < nd)) Dn = __builtin_nan("");
    return Dn;
}

// Committed runs of the chain, indexed by the run's first sorted position
// (k_tb_expand's input; len is reset to 0 once the run is expanded)
struct TbRuns {
    uint16_t* len;       // requests in the run starting here (0: none)
    int16_t* E;          // decade / binade exponent
    int64_t* D0;         // exact stored state before the run (signed digits)
    int64_t* D1;         // exact stored state after it, as the chain resolved it
};

// One round in a fast mode.  Reads the base state from parity slot `par`,
// publishes the next base into slot par^1; the caller's barrier ends the
// round.  Positions past the segment end are phantoms (add 0, live, never
// recorded).  State digits are carried as exact integer-valued doubles.
template <int MODE>
__device__ __attribute__((always_inline)) inline void tb_round(
    LaneShared& sh, uint32_t par, uint32_t first, uint32_t j1, int64_t D, int32_t E, double P, double R,
    const CfgDev* __restrict__ cfgs, int32_t profile, const ReqArgs& a, const TbPre& pre, uint32_t* eflags,
    uint64_t* cyc, uint32_t& iters, TbLoader& L, uint32_t* dbg, const TbRuns& runs) {
    constexpr int NW = TB_NW, K = TB_K;
    constexpr uint32_t WIN = TB_WIN;
    constexpr int ITMAX = 8;
    const double LO = MODE == QM_DEC ? (double)DEC_LO : (double)BIN_LO;
    const double HI = MODE == QM_DEC ? (double)DEC_HI : (double)BIN_HI;
    uint64_t t0 = 0, t1 = 0;
    (void)cyc; (void)t0; (void)t1;
#ifdef RL_STAMPS
#define RL_PHASE(k) do { RL_STAMP(t1); cyc[k] += t1 - t0; t0 = t1; } while (0)
#else
#define RL_PHASE(k) do { } while (0)
#endif
    RL_STAMP(t0);
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool loader = wave == (uint32_t)NW;
    const uint32_t np = par ^ 1u;
    const uint32_t cnt = (j1 - first) < WIN ? (j1 - first) : WIN;
    const uint32_t myoff = tid * K;       // loader lanes: >= WIN, no requests
    const uint32_t nvalid = myoff < cnt ? ((cnt - myoff) < (uint32_t)K ? (cnt - myoff) : (uint32_t)K) : 0u;
    const uint32_t i0 = first + myoff;

    // A. my K requests from the ring, nominal increments (inclusive lane
    // prefix cum[]), near flags
    double add[K], cum[K];
    int64_t nn[K];
    uint32_t cfq[K];
    uint32_t deadm = 0, nearm = 0, hardm = 0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nvalid;
        const uint32_t si = ring_idx(i0 + q);
        const double x = sh.r_add[si];
        const uint64_t w = sh.r_nc[si];
        if (v && !(x == x)) deadm |= 1u << q;           // NaN: key expired / absent
        if (v && (uint32_t)w == 0u) hardm |= 1u << q;   // n >= 2^31: exact path
        add[q] = v && x == x ? x : 0.0;
        nn[q] = v ? (int64_t)(uint32_t)w : 1;
        cfq[q] = v ? (uint32_t)(w >> 32) : 0u;
    }
    if (loader) ld_pump(L, sh, first, j1, pre, lane);
    double S = 0.0;
    float dq[K];         // distance of add/u from the nearest integer (near candidates)
#pragma unroll
    for (int q = 0; q < K; q++) {
        const double pr = add[q] * P;
        double rr = rint(pr);
        if (!(pr < 1e15 && pr > -1e15)) { hardm |= 1u << q; rr = 0.0; }
        dq[q] = 0.0f;
        if (MODE == QM_DEC) {
            const double err = __builtin_fma(add[q], P, -pr);           // add*P == pr + err exactly
            const double dist = fabs((pr - rr) + err);
            dq[q] = (float)dist;
            if (dist > 0.5 - TAU_DEC) nearm |= 1u << q;
        } else if (fabs(pr - rr) >= 0.5) {                              // exact tie: parity decides
            nearm |= 1u << q;
        }
        S += rr;                                                        // exact: |S| < 8e15
        cum[q] = S;
    }
    // a dead (expired) or hard (huge increment / n) request is always a stop
    const uint32_t evm = deadm | hardm;
    const uint32_t evq = evm ? (uint32_t)__builtin_ctz(evm) : (uint32_t)K;
    nearm &= evq >= 32 ? ~0u : ((1u << evq) - 1u);
    RL_PHASE(0);

    // B. block exclusive scan of the lane sums (int64: exact at any size)
    const int64_t Si = (int64_t)S;
    const int64_t inc = wave_incl_scan_i64(Si);
    if (lane == 63 && !loader) sh.wtot[wave] = inc;
    lds_barrier();                                                        // B1
    RL_PHASE(1);
    if (loader) ld_pump(L, sh, first, j1, pre, lane);
    int64_t pre_w = 0;
#pragma unroll
    for (int w = 0; w < NW; w++)
        if (w < (int)wave) pre_w += sh.wtot[w];
    // nominal predecessor of my first step; far outside the decade only if an
    // earlier request is a stop (then this lane never commits)
    const double Nb = (double)(D + pre_w + inc - Si);
    if (MODE == QM_DEC && nearm) {
        // lane-local near band: |delta| <= (|D| + |D'|) 2^-53 over my states
        // (nominal + an offset below 2^20: at most one flip per request)
        double dmax = fabs(Nb);
#pragma unroll
        for (int q = 0; q < K; q++) dmax = fmax(dmax, fabs(Nb + cum[q]));
        const double tau = (2.0 * (dmax + 1048576.0)) * 0x1.0000001p-53 + 1e-12;
        const float lim = (float)(0.5 - tau) - 1e-6f;     // dq is a float: stay conservative
        uint32_t nm = 0;
#pragma unroll
        for (int q = 0; q < K; q++)
            if (((nearm >> q) & 1u) && dq[q] > lim) nm |= 1u << q;
        nearm = nm;
    }

    // C. true start offsets by fixed-point iteration.  My end offset as a
    // function of my start offset s: far steps keep it, near steps are
    // evaluated exactly (dl[q]: the offset change at near step q); `brk` = a
    // near step leaves the regime or a stop request ends the lane.
    double dl[K];
    uint32_t bq = K;     // the near step that left the regime (K: none)
    auto near_walk = [&](double s, bool& brk) -> double {
        double c = s;
        bq = K;
#pragma unroll
        for (int k = 0; k < K; k++) dl[k] = 0.0;
        uint32_t todo = nearm;
        while (todo) {
            const uint32_t q = (uint32_t)__builtin_ctz(todo);
            todo &= todo - 1u;
            double xa = 0.0, xc = 0.0, xp = 0.0, nd = 1.0;
            uint32_t xcf = 0;
#pragma unroll
            for (int k = 0; k < K; k++)
                if ((uint32_t)k == q) {
                    xa = add[k];
                    nd = (double)nn[k];
                    xcf = cfq[k];
                    xc = cum[k];
                    xp = k ? cum[k - 1] : 0.0;
                }
            double tk;
            const double Dn = tb_step_d<MODE>(Nb + xp + c, P, R, xa, cfgs[xcf].limit_d, nd, tk);
            if (!(Dn == Dn)) { bq = q; break; }
            const double cn = Dn - (Nb + xc);
#pragma unroll
            for (int k = 0; k < K; k++)
                if ((uint32_t)k == q) dl[k] = cn - c;
            c = cn;
        }
        brk = evq < (uint32_t)K || bq < (uint32_t)K;
        return c;
    };
    // Iteration k: starts s^k = scan of the deltas taken at s^(k-1).  When no
    // delta (before the first break) changes at s^k, the starts are a fixed
    // point and, by induction over lanes, TRUE.  At the cap, lanes up to the
    // first changed one still have true starts; the round ends after it.
    bool brk;
    double soff = 0.0;
    double cend = near_walk(0.0, brk);
    RL_PHASE(2);
    uint32_t unstable = NO_STOP;
    for (int it = 0;; it++) {
        const double dd = cend - soff;
        const int64_t di = (brk || !(fabs(dd) < 4e18)) ? 0 : (int64_t)dd;
        const int64_t dinc = wave_incl_scan_i64(di);
        if (lane == 63 && !loader) sh.itot[wave] = dinc;
        lds_barrier();
        int64_t dw = 0;
#pragma unroll
        for (int w = 0; w < NW; w++)
            if (w < (int)wave) dw += sh.itot[w];
        const double snew = (double)(dw + dinc - di);
        bool changed = false;
        if (snew != soff) {
            const double dold = cend - soff;
            const bool bold = brk;
            cend = nearm ? near_walk(snew, brk) : cend + (snew - soff);
            changed = brk != bold || (!brk && cend - snew != dold);
            soff = snew;
        }
        const uint32_t fch = wave_min_u32(changed && nvalid ? tid : NO_STOP);
        const uint32_t fbk = wave_min_u32(brk && nvalid ? tid : NO_STOP);
        if (lane == 0 && !loader) { sh.ich[wave] = fch; sh.ibk[wave] = fbk; }
        lds_barrier();
        if (loader) ld_pump(L, sh, first, j1, pre, lane);
        uint32_t ch = NO_STOP, bk = NO_STOP;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            ch = sh.ich[w] < ch ? sh.ich[w] : ch;
            bk = sh.ibk[w] < bk ? sh.ibk[w] : bk;
        }
        iters++;
        if (ch == NO_STOP || ch >= bk) break;                 // block-uniform
        if (it + 1 == ITMAX) { unstable = ch; break; }
    }
    RL_PHASE(3);

    // D. every request's next state from my true start; the first one that
    // may leave the regime stops the lane (near steps were checked exactly)
    uint32_t stopq = evq < bq ? evq : bq;
    double spred = 0.0, Dlast = Nb + soff;
    {
        double c = soff;
#pragma unroll
        for (int q = 0; q < K; q++) {
            const double pred = Nb + (q ? cum[q - 1] : 0.0) + c;
            if ((uint32_t)q == stopq) spred = pred;
            if ((uint32_t)q < stopq) {
                c += dl[q];
                const double Dn = Nb + cum[q] + c;
                // decade: exact; allow / clamp: |tokens - D'u| <= 0.53 u
                const double vhi = (Dn + 2.0) * R * (1.0 + 1e-9);
                bool ev = !(fabs(Dn) >= LO && fabs(Dn) < HI);
                ev = ev || !(vhi < (double)nn[q]) || !(vhi < cfgs[cfq[q]].limit_d);
                if (ev && !((nearm >> q) & 1u) && (uint32_t)q < nvalid) {
                    stopq = q;
                    spred = pred;
                } else {
                    Dlast = Dn;
                }
            }
        }
    }
    // stop key: (position << 1) | kind; kind 0 = boundary after committed
    // requests (wins ties), 1 = a stop request stepped exactly by its owner
    uint32_t sg = NO_STOP;
    if (nvalid) {
        if (stopq < nvalid) sg = ((myoff + stopq) << 1) | 1u;
        else if (tid == unstable) sg = (myoff + nvalid) << 1;
    }
    const uint32_t wm = wave_min_u32(sg);
    if (lane == 0 && !loader) sh.wmin[wave] = wm;
    lds_barrier();                                                        // B3
    RL_PHASE(4);
    uint32_t em = NO_STOP;
#pragma unroll
    for (int w = 0; w < NW; w++) em = sh.wmin[w] < em ? sh.wmin[w] : em;
    const uint32_t epos = em == NO_STOP ? cnt : (em >> 1);
    const bool estep = em != NO_STOP && (em & 1u);
    if (tid == 0 && dbg)   // round-end reason
        atomicAdd(&dbg[3 + (em == NO_STOP ? 0 : (em & 1u) ? 1 : (unstable != NO_STOP ? 3 : 2))], 1u);

    if (loader) {
        // the next window must be in the ring before the round barrier
        const uint32_t nf = first + epos + (estep ? 1u : 0u);
        ld_until(L, sh, nf, nf + WIN, j1, pre, lane);
        RL_PHASE(5);
        return;
    }

    // E. record my committed run [i0, i0 + len); k_tb_expand produces its
    // outputs.  The stop request runs exactly here; next base.
    const uint32_t len = epos > myoff ? ((epos - myoff) < nvalid ? (epos - myoff) : nvalid) : 0u;
    if (len) {
        runs.len[i0] = (uint16_t)len;
        runs.E[i0] = (int16_t)E;
        runs.D0[i0] = (int64_t)(Nb + soff);
        runs.D1[i0] = (int64_t)Dlast;
    }
    if (estep) {
        if (epos >= myoff && epos < myoff + nvalid) {
            const uint32_t sq = epos - myoff;
            double sadd = 0.0;
            int64_t snn = 1;
            uint32_t scf = 0;
#pragma unroll
            for (int q = 0; q < K; q++)
                if ((uint32_t)q == sq) { sadd = add[q]; snn = nn[q]; scf = cfq[q]; }
            const CfgDev& C = cfgs[scf];
            if ((hardm >> sq) & 1u) snn = a.n[i0 + sq];
            const TbEval v = tb_eval(MODE, (int64_t)spred, E, P, R, ((deadm >> sq) & 1u) == 0, sadd, C.limit_d,
                                     (double)snn, profile);
            write_out_tb(a, i0 + sq, v.allowed ? DEC_ALLOWED : DEC_DENIED, v.tokens);
            const TbQ nq = v.inrange ? TbQ{v.Dact, E} : tb_quant(v.tokens, profile);
            sh.baseD[np] = nq.D;
            sh.baseE[np] = nq.E;
            sh.first[np] = first + epos + 1;
        }
    } else if (nvalid && myoff + nvalid == epos) {
        if (epos == 0) atomicOr(eflags, EF_INTERNAL);
        sh.baseD[np] = (int64_t)Dlast;
        sh.baseE[np] = E;
        sh.first[np] = first + epos;
    }
    RL_PHASE(5);
#undef RL_PHASE
}

// Replay one heavy token-bucket segment [j0, j1) with the whole block
// (TB_NC compute lanes + the loader wave).
__device__ __attribute__((always_inline)) inline void replay_tb_lanes(
    LaneShared& sh, TbEntry* e, uint32_t j0, uint32_t j1, const CfgDev* __restrict__ cfgs, int32_t profile,
    const ReqArgs& a, const TbPre& pre, uint32_t* eflags, uint32_t* dbg, const TbRuns& runs) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const bool loader = (tid >> 6) == (uint32_t)TB_NW;
    uint32_t nrounds = 0, niters = 0, par = 0;
    uint64_t cyc[6] = {0, 0, 0, 0, 0, 0};
    TbLoader L;
    L.fill = j0 & ~1u;
    L.pend = false;
    if (tid == 0) {
        const TbQ q = tb_quant(e->tok, profile);
        sh.baseD[0] = q.D;
        sh.baseE[0] = q.E;
        sh.first[0] = j0;
    }
    if (loader) ld_until(L, sh, j0, j0 + TB_WIN, j1, pre, lane);
    lds_barrier();
    for (;;) {
        const uint32_t first = sh.first[par];
        if (first >= j1) break;                      // block-uniform
        const int64_t D = sh.baseD[par];
        const int32_t E = sh.baseE[par];
        const uint32_t np = par ^ 1u;
        const int64_t aD = D < 0 ? -D : D;
        nrounds++;
        if (profile == PROFILE_REDIS7 && 13 - E >= 1 && 13 - E <= 22 && aD >= DEC_LO && aD < DEC_HI) {
            const double P = rlq::pow10_exact(13 - E);
            tb_round<QM_DEC>(sh, par, first, j1, D, E, P, 1.0 / P, cfgs, profile, a, pre, eflags, cyc, niters, L,
                             dbg, runs);
        } else if (profile != PROFILE_REDIS7 && aD >= BIN_LO && aD < BIN_HI && E > -1000 && E < 900) {
            tb_round<QM_BIN>(sh, par, first, j1, D, E, ldexp(1.0, -E), ldexp(1.0, E), cfgs, profile, a, pre,
                             eflags, cyc, niters, L, dbg, runs);
        } else {
            // off the fast decades (or an empty/zero state): one exact step
            if (tid == 0) {
                const uint32_t i = first;
                const uint64_t w = sh.r_nc[ring_idx(i)];
                const CfgDev& C = cfgs[(uint32_t)(w >> 32)];
                const int64_t nn = (uint32_t)w ? (int64_t)(uint32_t)w : a.n[i];
                const double add = sh.r_add[ring_idx(i)];
                const bool alive = add == add;
                const TbEval v = tb_eval(QM_NONE, D, E, 1.0, 1.0, alive, alive ? add : 0.0, C.limit_d,
                                         (double)nn, profile);
                write_out_tb(a, i, v.allowed ? DEC_ALLOWED : DEC_DENIED, v.tokens);
                const TbQ q = tb_quant(v.tokens, profile);
                sh.baseD[np] = q.D;
                sh.baseE[np] = q.E;
                sh.first[np] = first + 1;
            }
            if (loader) ld_until(L, sh, first + 1, first + 1 + TB_WIN, j1, pre, lane);
        }
        par = np;
        lds_barrier();                                                        // B4
    }
#ifdef RL_STAMPS
    // every wave reports: the max over waves of each phase shows who waits
    if ((tid & 63) == 0 && dbg)
        for (int k = 0; k < 6; k++) atomicMax(&dbg[8 + 2 * k], (uint32_t)(cyc[k] >> 4));   // 16-cycle units
#endif
    if (tid == 0) {
        e->tok = tb_value(sh.baseD[par], sh.baseE[par], profile);
        e->last = pre.lq[j1 - 1];
        e->when = pre.when[j1 - 1];
        if (dbg) {
            atomicAdd(&dbg[0], nrounds);
            atomicAdd(&dbg[1], niters);
            atomicMax(&dbg[2], nrounds);
        }
    }
}

// Outputs of the recorded runs: each run's requests replayed exactly from
// its exact start state (one thread per run, all runs in parallel), checked
// against the state the chain resolved at the run's end.
__global__ __launch_bounds__(256) void k_tb_expand(uint32_t m, TbRuns runs, const CfgDev* __restrict__ cfgs,
                                                   int32_t profile, ReqArgs a, TbPre pre, uint32_t* eflags) {
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < m; j += gridDim.x * blockDim.x) {
        const uint32_t len = runs.len[j];
        if (!len) continue;
        runs.len[j] = 0;
        const int32_t E = runs.E[j];
        double D = (double)runs.D0[j];
        bool ok = true;
        if (profile == PROFILE_REDIS7) {
            const double P = rlq::pow10_exact(13 - E), R = 1.0 / P;
            for (uint32_t q = 0; q < len; q++) {
                const uint64_t w = pre.nc[j + q];
                double tk;
                const double Dn = tb_step_d<QM_DEC>(D, P, R, pre.add[j + q], cfgs[(uint32_t)(w >> 32)].limit_d,
                                                    (double)(uint32_t)w, tk);
                a.tok[j + q] = tk;
                a.dec[j + q] = DEC_DENIED;
                ok = ok && Dn == Dn;
                D = Dn;
            }
        } else {
            const double P = ldexp(1.0, -E), R = ldexp(1.0, E);
            for (uint32_t q = 0; q < len; q++) {
                const uint64_t w = pre.nc[j + q];
                double tk;
                const double Dn = tb_step_d<QM_BIN>(D, P, R, pre.add[j + q], cfgs[(uint32_t)(w >> 32)].limit_d,
                                                    (double)(uint32_t)w, tk);
                a.tok[j + q] = tk;
                a.dec[j + q] = DEC_DENIED;
                ok = ok && Dn == Dn;
                D = Dn;
            }
        }
        if (!ok || D != (double)runs.D1[j]) atomicOr(eflags, EF_INTERNAL);
    }
}

}  // namespace rl
