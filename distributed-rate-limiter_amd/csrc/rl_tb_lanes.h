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

// cooperative replay geometry: NC compute lanes + 1 loader wave
#ifndef RL_TB_NC
#define RL_TB_NC 448
#endif
#ifndef RL_TB_K
#define RL_TB_K 8
#endif
constexpr int TB_NC = RL_TB_NC;
constexpr int TB_K = RL_TB_K;                    // requests per lane per round
constexpr int TB_NW = TB_NC / 64;
constexpr uint32_t TB_WIN = (uint32_t)TB_NC * TB_K;
// LDS ring of request inputs by absolute sorted position, in 16-byte
// granules (two positions).  Granule G lives in slot swz(G mod RING_G): an XOR
// of its column (G mod 16) with bits 4-5, so the 8 lanes of one ds_read_b128
// cycle (lane l reads granule G0 + 4l + j) always hit distinct banks, while a
// row of 16 slots still holds 16 consecutive granules (the loader's LDS-DMA
// writes slots lane-linearly and swizzles the SOURCE address instead).
constexpr uint32_t RING = 8192;                  // positions
constexpr uint32_t RING_G = RING / 2;            // granules
__host__ __device__ constexpr uint32_t swz(uint32_t g) { return (g & ~15u) | ((g & 15u) ^ ((g >> 4) & 3u)); }
__host__ __device__ constexpr uint32_t ring_slot(uint32_t granule) { return swz(granule & (RING_G - 1)); }
static_assert(RING >= 2 * TB_WIN + 256, "the ring must hold the next window while the current one is read");

constexpr uint32_t NL_MAX = 512;   // near steps resolved per round

struct LaneShared {
    double2 r_add[RING_G];       // TbPre::add
    ulonglong2 r_nc[RING_G];     // TbPre::nc
    int64_t wtot[TB_NW];         // lane-sum scan
    uint32_t ntot[TB_NW];        // near-step count scan
    uint32_t wmin[TB_NW];        // first stop
    // the round's near steps in sequence order (NL_MAX at most)
    double nl_pred[NL_MAX];      // nominal predecessor state
    double nl_add[NL_MAX];
    uint64_t nl_nc[NL_MAX];      // TbPre::nc
    int32_t nl_off[NL_MAX];      // resolved: offset after the step (true - nominal)
    uint32_t nstop;              // first near step that stops the round (list index)
    int64_t baseD[2];            // round-parity double buffer
    int32_t baseE[2];
    uint32_t first[2];
};

__device__ inline double ring_add(const LaneShared& sh, uint32_t p) {
    const double2 g = sh.r_add[ring_slot(p >> 1)];
    return (p & 1u) ? g.y : g.x;
}
__device__ inline uint64_t ring_nc(const LaneShared& sh, uint32_t p) {
    const ulonglong2 g = sh.r_nc[ring_slot(p >> 1)];
    return (p & 1u) ? g.y : g.x;
}

// The loader wave streams TbPre::{add, nc} into the ring in 128-position
// chunks by LDS-DMA (global_load_lds_dwordx4: no registers, lands
// asynchronously).  It issues every chunk the ring can take right after a
// round starts and waits for them only at the round's end, so the loads land
// behind a whole round of compute.  A chunk may only overwrite positions
// already consumed: chunk c is allowed once 128c + 128 <= first + RING.
// The source arrays carry 128 elements of slack past the batch.
struct TbLoader {
    uint32_t next;       // next chunk to issue
    uint32_t issued;     // chunks issued since the last wait
};

// one 16-byte LDS-DMA per lane into the slots starting at the wave-uniform
// LDS byte address `lds` (issued from asm: hipcc neither counts it nor drains
// it early; ld_until waits for it explicitly)
__device__ __attribute__((always_inline)) inline void glds16(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    __asm__ volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(gsrc), "s"(lds)
                     : "memory");
}

__device__ __attribute__((always_inline)) inline void ld_chunk(LaneShared& sh, uint32_t c, const TbPre& pre,
                                                              uint32_t lane) {
    const uint32_t s0 = (c * 64u) & (RING_G - 1);   // first slot of the chunk (row aligned)
    const uint32_t g = c * 64u + swz(lane);         // granule this lane's slot holds
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&sh.r_add[s0];
    const uint32_t ln = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&sh.r_nc[s0];
    glds16(pre.add + 2u * g, __builtin_amdgcn_readfirstlane(la));
    glds16(pre.nc + 2u * g, __builtin_amdgcn_readfirstlane(ln));
}

// issue every chunk the ring can take for a window starting at `first`
__device__ __attribute__((always_inline)) inline void ld_issue(TbLoader& L, LaneShared& sh, uint32_t first,
                                                              uint32_t j1, const TbPre& pre, uint32_t lane) {
    const uint32_t lim = (first + RING) / 128u;     // chunks c < lim fit
    const uint32_t endc = (j1 + 127u) / 128u;
    while (L.next < lim && L.next < endc && L.issued < 28u) {   // <= 56 outstanding (vmcnt <= 63)
        ld_chunk(sh, L.next, pre, lane);
        L.next++;
        L.issued++;
    }
}

// make [.., target) resident: issue what is missing and wait for everything
__device__ __attribute__((always_inline)) inline void ld_until(TbLoader& L, LaneShared& sh, uint32_t first,
                                                              uint32_t target, uint32_t j1, const TbPre& pre,
                                                              uint32_t lane) {
    const uint32_t need = ((target < j1 ? target : j1) + 127u) / 128u;
    for (;;) {
        ld_issue(L, sh, first, j1, pre, lane);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        L.issued = 0;
        if (L.next >= need) break;
    }
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

// Resolution of a round's near steps (list order = sequence order), by ONE
// wave, 64 steps at a time.  A step's exact result depends on its exact
// predecessor = nominal + (offset before it); far steps keep the offset, so
// the offset before step k is the batch's entry offset plus the flips
// (exact result - nominal result) of the batch's earlier steps.  Wave-local
// fixed point: evaluate every step at the current guess, scan the flips
// (DPP), re-guess; when no guess changes (before the first step that leaves
// the regime) the guesses are the true offsets, by induction over lanes.
// Writes nl_off[k] for every resolved step and nstop = the first step that
// stops the round (leaves the regime, or the iteration cap), else NO_STOP.
template <int MODE>
__device__ __attribute__((noinline)) void tb_near_resolve(LaneShared& sh, uint32_t nl, double P, double R,
                                                          const CfgDev* __restrict__ cfgs, uint32_t& iters) {
    constexpr int ITMAX = 16;
    const uint32_t lane = threadIdx.x & 63;
    int32_t cb = 0;                   // offset before the batch (exact)
    uint32_t nstop = NO_STOP;
    for (uint32_t b = 0; b < nl; b += 64) {
        const uint32_t k = b + lane;
        const bool v = k < nl;
        const double pn = v ? sh.nl_pred[k] : 0.0;
        const double ad = v ? sh.nl_add[k] : 0.0;
        const uint64_t w = v ? sh.nl_nc[k] : 1ull;
        const double cap = cfgs[(uint32_t)(w >> 32)].limit_d, nd = (double)(uint32_t)w;
        const double r = rint(ad * P);
        int32_t est = 0, flip = 0;
        uint32_t stop_lane = 64;
        for (int it = 0;; it++) {
            double tk;
            const double pred = pn + (double)(cb + est);
            const double Dn = tb_step_d<MODE>(pred, P, R, ad, cap, nd, tk);
            const bool brk = v && !(Dn == Dn);
            flip = (!v || brk) ? 0 : (int32_t)(Dn - (pred + r));
            const int32_t incl = (int32_t)wave_scan_u32((uint32_t)flip, 0u,
                                                        [](uint32_t x, uint32_t y) { return x + y; });
            const int32_t en = incl - flip;
            const uint64_t bm = __ballot(brk);
            const uint64_t cm = __ballot(v && en != est);
            const uint32_t fb = bm ? (uint32_t)__ffsll((unsigned long long)bm) - 1 : 64u;
            const uint32_t fc = cm ? (uint32_t)__ffsll((unsigned long long)cm) - 1 : 64u;
            iters++;
            if (fc >= fb) { stop_lane = fb; break; }             // converged up to the first break
            if (it + 1 == ITMAX) {                               // lanes < fc are exact
                stop_lane = fc;
                break;
            }
            est = en;
        }
        if (v && lane < stop_lane) sh.nl_off[k] = cb + est + flip;
        if (stop_lane < 64) {
            nstop = b + stop_lane;
            break;
        }
        cb += __builtin_amdgcn_readlane(est + flip, 63);
    }
    if (lane == 0) sh.nstop = nstop;
}

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
    {
        // my positions [i0, i0 + K): K/2 granules, one more when i0 is odd
        // (first is block-uniform, so is the parity)
        double ga[K + 2];
        uint64_t gn[K + 2];
        const uint32_t g0 = i0 >> 1;
#pragma unroll
        for (int j = 0; j < K / 2 + 1; j++) {
            if (j < K / 2 || (i0 & 1u)) {
                const double2 x = sh.r_add[ring_slot(g0 + j)];
                const ulonglong2 y = sh.r_nc[ring_slot(g0 + j)];
                ga[2 * j] = x.x; ga[2 * j + 1] = x.y;
                gn[2 * j] = y.x; gn[2 * j + 1] = y.y;
            } else {
                ga[2 * j] = ga[2 * j + 1] = 0.0;
                gn[2 * j] = gn[2 * j + 1] = 0;
            }
        }
        const uint32_t o = i0 & 1u;
#pragma unroll
        for (int q = 0; q < K; q++) {
            const bool v = (uint32_t)q < nvalid;
            const double x = o ? ga[q + 1] : ga[q];
            const uint64_t w = o ? gn[q + 1] : gn[q];
            if (v && !(x == x)) deadm |= 1u << q;           // NaN: key expired / absent
            if (v && (uint32_t)w == 0u) hardm |= 1u << q;   // n >= 2^31: exact path
            add[q] = v && x == x ? x : 0.0;
            nn[q] = v ? (int64_t)(uint32_t)w : 1;
            cfq[q] = v ? (uint32_t)(w >> 32) : 0u;
        }
    }
    RL_PHASE(0);
    if (loader) ld_issue(L, sh, first, j1, pre, lane);
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
    RL_PHASE(1);

    // B. block exclusive scan of the lane sums (int64: exact at any size)
    const int64_t Si = (int64_t)S;
    const int64_t inc = wave_incl_scan_i64(Si);
    if (lane == 63 && !loader) sh.wtot[wave] = inc;
    lds_barrier();                                                        // B1
    RL_PHASE(2);
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

    // C. near steps: compacted into an LDS list in sequence order, resolved
    // by wave 0 (tb_near_resolve), read back as offsets
    const uint32_t ncnt = (uint32_t)__popc(nearm);
    const uint32_t ninc = wave_scan_u32(ncnt, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    if (lane == 63 && !loader) sh.ntot[wave] = ninc;
    lds_barrier();                                                        // B2
    RL_PHASE(3);
    uint32_t rank0 = ninc - ncnt, nl = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        if (w < (int)wave) rank0 += sh.ntot[w];
        nl += sh.ntot[w];
    }
    {
        uint32_t k = rank0;
#pragma unroll
        for (int q = 0; q < K; q++) {
            if ((nearm >> q) & 1u) {
                if (k < NL_MAX) {
                    sh.nl_pred[k] = Nb + (q ? cum[q - 1] : 0.0);
                    sh.nl_add[k] = add[q];
                    sh.nl_nc[k] = ((uint64_t)cfq[q] << 32) | (uint32_t)nn[q];
                }
                k++;
            }
        }
    }
    lds_barrier();                                                        // B3
    RL_PHASE(4);
    if (wave == 0) tb_near_resolve<MODE>(sh, nl < NL_MAX ? nl : NL_MAX, P, R, cfgs, iters);
    lds_barrier();                                                        // B4
    RL_PHASE(5);
    // list capacity: the step of rank NL_MAX stops too (its predecessor is known)
    const uint32_t nstop = nl > NL_MAX && sh.nstop > NL_MAX ? NL_MAX : sh.nstop;

    // D. every request's next state from my true start; the first one that
    // may leave the regime stops the lane (near steps were checked exactly)
    uint32_t stopq = evq;
    double spred = 0.0;
    // my start offset: the offset after the last near step before my lane
    const double cstart = (rank0 > 0 && rank0 - 1 < nstop) ? (double)sh.nl_off[rank0 - 1] : 0.0;
    double Dlast = Nb + cstart;
    {
        double c = cstart;
        uint32_t k = rank0;
#pragma unroll
        for (int q = 0; q < K; q++) {
            const double pred = Nb + (q ? cum[q - 1] : 0.0) + c;
            if ((uint32_t)q == stopq) spred = pred;
            if ((uint32_t)q < stopq) {
                bool ev;
                if ((nearm >> q) & 1u) {
                    ev = k >= nstop;
                    if (!ev) c = (double)sh.nl_off[k];
                    k++;
                } else {
                    const double Dn = Nb + cum[q] + c;
                    // decade: exact; allow / clamp: |tokens - D'u| <= 0.53 u
                    const double vhi = (Dn + 2.0) * R * (1.0 + 1e-9);
                    ev = !(fabs(Dn) >= LO && fabs(Dn) < HI);
                    ev = ev || !(vhi < (double)nn[q]) || !(vhi < cfgs[cfq[q]].limit_d);
                }
                if (ev && (uint32_t)q < nvalid) {
                    stopq = q;
                    spred = pred;
                } else {
                    Dlast = Nb + cum[q] + c;
                }
            }
        }
    }
    const uint32_t unstable = NO_STOP;
    // stop key: (position << 1) | kind; kind 0 = boundary after committed
    // requests (wins ties), 1 = a stop request stepped exactly by its owner
    uint32_t sg = NO_STOP;
    if (nvalid) {
        if (stopq < nvalid) sg = ((myoff + stopq) << 1) | 1u;
        else if (tid == unstable) sg = (myoff + nvalid) << 1;
    }
    const uint32_t wm = wave_min_u32(sg);
    if (lane == 0 && !loader) sh.wmin[wave] = wm;
    lds_barrier();                                                        // B5
    RL_PHASE(6);
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
        RL_PHASE(7);
        return;
    }

    // E. record my committed run [i0, i0 + len); k_tb_expand produces its
    // outputs.  The stop request runs exactly here; next base.
    const uint32_t len = epos > myoff ? ((epos - myoff) < nvalid ? (epos - myoff) : nvalid) : 0u;
    if (len) {
        runs.len[i0] = (uint16_t)len;
        runs.E[i0] = (int16_t)E;
        runs.D0[i0] = (int64_t)(Nb + cstart);
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
    RL_PHASE(7);
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
    uint64_t cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    TbLoader L;
    L.next = j0 / 128u;
    L.issued = 0;
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
                const uint64_t w = ring_nc(sh, i);
                const CfgDev& C = cfgs[(uint32_t)(w >> 32)];
                const int64_t nn = (uint32_t)w ? (int64_t)(uint32_t)w : a.n[i];
                const double add = ring_add(sh, i);
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
    // every wave reports its own phase sums (16-cycle units), longest segment
    if ((tid & 63) == 0 && dbg)
        for (int k = 0; k < 8; k++) atomicMax(&dbg[24 + 8 * (tid >> 6) + k], (uint32_t)(cyc[k] >> 4));
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

// Cooperative replay of the heavy token-bucket segments: one segment per
// block from a work queue (window segments in the heavy list are k_replay's).
constexpr int TB_BLOCK = TB_NC + 64;    // 7 compute waves + 1 loader wave

template <bool LCFG>
__global__ __launch_bounds__(TB_BLOCK) void k_tb_coop(const uint32_t* __restrict__ sk,
                                                      const SegRec* __restrict__ heavy,
                                                      const uint32_t* __restrict__ nheavy_p, uint32_t* qctr,
                                                      uint32_t win_base, TbEntry* tb,
                                                      const CfgDev* __restrict__ gcfgs, uint32_t ncfg,
                                                      int32_t profile, ReqArgs a, TbPre pre, uint32_t* eflags,
                                                      uint32_t* dbg, TbRuns runs) {
    __shared__ LaneShared sh;
    __shared__ uint32_t s_u;
    __shared__ CfgDev s_cfg[LCFG ? MAX_LCFG : 1];
    if (LCFG) {
        for (uint32_t c = threadIdx.x; c < ncfg; c += blockDim.x) s_cfg[c] = gcfgs[c];
        __syncthreads();
    }
    const CfgDev* cfgs = LCFG ? s_cfg : gcfgs;
    const uint32_t nheavy = *nheavy_p;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t u;
            do {   // skip window segments (k_replay's)
                u = atomicAdd(qctr, 1u);
            } while (u < nheavy && sk[heavy[u].j0] >= win_base);
            s_u = u;
        }
        __syncthreads();
        const uint32_t u = s_u;
        __syncthreads();
        if (u >= nheavy) break;
        const SegRec sg = heavy[u];
        const uint64_t t_seg = __builtin_amdgcn_s_memrealtime();
        replay_tb_lanes(sh, &tb[sk[sg.j0]], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre, eflags, dbg, runs);
        __syncthreads();
        if (threadIdx.x == 0 && dbg) atomicMax(&dbg[8], (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seg));
    }
}

}  // namespace rl
