// rl_tb_chain.h -- pipelined token-bucket replay of heavy (Zipf hot-key)
// segments.  Included by rl_replay.h after its helpers.
//
// What is replayed: the reference's token-bucket script step
// (tokenbucket.go:23-52 + the Go arithmetic at :114-130), request by request
// in arrival order, on one key.  The carried state is the STORED tokens value,
// which Lua's tostring quantizes (tokenbucket.go:48): under Redis 7 to 14
// significant decimal digits, i.e. an integer D in [1e13, 1e14) in a decade E
// (value = D * 10^(E-13)); under miniredis to the exact double, an integer
// mantissa D in [2^52, 2^53) in a binade E.
//
// Step algebra (u = the unit of D, P = 1/u).  With T = strtod(D*u) and
// sum = RN(T + add), the next stored state is D' = round(sum * P) =
// round(D + add*P + delta) with |delta| <= (D + D') * 2^-53 < 0.0223 (two
// correct roundings of values below 1e14 u).  D is an integer, so whenever
// add*P is farther than TAU_DEC (0.03) from a half-integer (a "far" step),
// D' = D + r with r = rint(add*P) for EVERY predecessor D in the decade: the
// step is an integer add, independent of the state.  Only "near" steps
// (about 6% of them) depend on the exact predecessor.  A step leaves this
// regime when it allows (tokens >= n), clamps (sum >= capacity), leaves the
// decade, or finds the key expired; regime exits are rare for a hot key.
//
// One block replays one segment with three wave roles, in lock-step rounds
// separated by one LDS barrier:
//   producers (CH_NP waves)  summarize the NEXT window of CH_W requests at the
//       current decade: per 512-request tile the nominal sum of r, bounds of
//       the nominal prefix (decade exit), of the allow/clamp slack, the first
//       expired/huge step, and the tile's near steps compacted into an LDS
//       list -- all state-free, so they run one window ahead of the chain;
//   chain (wave 0)  resolves the window the producers summarized in the
//       previous round: near steps by a wave-wide fixed point on their exact
//       predecessors (64 at a time), then tile by tile either commits the tile
//       as a run {start, length, exact start state, exact end state} or, when
//       the bounds say the tile may leave the regime, replays it exactly
//       (exact_span) to find the first regime exit, which it executes exactly
//       (tb_eval) together with any further out-of-regime steps (serial loop);
//   loader (1 wave)  streams the segment's precomputed inputs (add, th) from
//       HBM into an LDS ring by LDS-DMA, two windows ahead.
// If the chain window ends early (regime exit), the producers' speculative
// window is discarded and the next round re-produces from the exit.
//
// k_tb_expand then replays every committed run exactly and in parallel over
// the whole GPU (one wave per run, exact_span with outputs) and checks that
// each run ends in the state the chain recorded (EF_INTERNAL otherwise).  So
// every result still comes from an exact step on its exact predecessor; the
// bounds above only decide WHERE the chain looks, never a result.
#pragma once

namespace rl {

constexpr int64_t DEC_LO = 10000000000000LL, DEC_HI = 100000000000000LL;
constexpr int64_t BIN_LO = 1LL << 52, BIN_HI = 1LL << 53;
constexpr uint32_t NO_STOP = 0xffffffffu;

#ifndef RL_CH_NP
#define RL_CH_NP 3
#endif
constexpr int CH_K = 8;                                // requests per producer lane
constexpr int CH_NP = RL_CH_NP;                        // producer waves
constexpr uint32_t CH_TILE = 64u * CH_K;               // requests per producer wave
constexpr uint32_t CH_W = (uint32_t)CH_NP * CH_TILE;   // requests per window
constexpr int CH_NE = 64;                              // near-list capacity per tile
constexpr int CH_LOADER = CH_NP + 1;                   // wave 0 chain, 1..NP producers
constexpr int CH_BLOCK = (CH_NP + 2) * 64;
constexpr int CH_SERIAL = 64;                          // serial exact steps per round at most
// conservative scale of the allow/clamp threshold th*P (covers the rounding of
// th*P and of the bound arithmetic with a wide margin)
constexpr double CH_YSCALE = 1.0 - 0x1p-28;

// LDS ring of the segment's inputs by absolute sorted position, in 16-byte
// granules (two positions).  Granule G lives in slot swz(G mod RING_G): an XOR
// of its column (G mod 16) with bits 4-5, so the 8 lanes of one ds_read_b128
// cycle (lane l reads granule G0 + 4l + j) hit distinct banks, while a row of
// 16 slots still holds 16 consecutive granules (the loader's LDS-DMA writes
// slots lane-linearly and swizzles the SOURCE address instead).
constexpr uint32_t RING = 8192;                  // positions
constexpr uint32_t RING_G = RING / 2;            // granules
__host__ __device__ constexpr uint32_t swz(uint32_t g) { return (g & ~15u) | ((g & 15u) ^ ((g >> 4) & 3u)); }
__host__ __device__ constexpr uint32_t ring_slot(uint32_t granule) { return swz(granule & (RING_G - 1)); }
// the chain window, the producers' window and the loader's next window
static_assert(RING >= 3 * CH_W + 256, "the ring must hold three windows");

struct ChTile {
    int64_t S;          // nominal sum of the tile's increments r
    double ymin;        // min over steps of (th * P * CH_YSCALE - inclusive nominal prefix)
    double cmax, cmin;  // max / min inclusive nominal prefix
    uint32_t ev;        // first expired / huge step (tile-relative) or NO_STOP
    uint32_t nc;        // near steps (> CH_NE: list overflow)
};

struct ChState {
    int64_t D;          // exact stored digits at cfirst (ccnt > 0) or at pfirst (ccnt == 0)
    int32_t E;
    int32_t mode;       // QM_DEC / QM_BIN when (D, E) is in a fast decade, else QM_NONE
    uint32_t cfirst;    // chain window [cfirst, cfirst + ccnt), summarized in tile[cbuf]
    uint32_t ccnt;
    uint32_t pfirst;    // producers' window start (== cfirst + ccnt when ccnt > 0)
    uint32_t pbuf, cbuf;
};

struct ChainShared {
    double2 r_add[RING_G];       // TbPre::add
    double2 r_th[RING_G];        // TbPre::th
    ChTile tile[2][CH_NP];
    double ne_pred[2][CH_NP][CH_NE];   // tile-relative nominal predecessor of each near step
    double ne_add[2][CH_NP][CH_NE];
    double ne_th[2][CH_NP][CH_NE];
    int32_t ne_off[CH_NP * CH_NE];     // chain: resolved offset after each near step
    ChState st[2];
};

__device__ inline double ring_add(const ChainShared& sh, uint32_t p) {
    const double2 g = sh.r_add[ring_slot(p >> 1)];
    return (p & 1u) ? g.y : g.x;
}
__device__ inline double ring_th(const ChainShared& sh, uint32_t p) {
    const double2 g = sh.r_th[ring_slot(p >> 1)];
    return (p & 1u) ? g.y : g.x;
}

// ---------------------------------------------------------------------------
// wave helpers (DPP row shifts / broadcasts, GFX9 family)
// ---------------------------------------------------------------------------
template <int CTRL, int RM>
__device__ inline double dpp_f64(double v, double old) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v), o = __builtin_bit_cast(uint64_t, old);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)b, CTRL, RM, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(b >> 32), CTRL,
                                                              RM, 0xf, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ inline double readlane_f64(double v, uint32_t l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, (int)l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), (int)l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <typename Op>
__device__ inline double wave_reduce_f64(double v, double ident, Op op) {
    v = op(v, dpp_f64<0x111, 0xf>(v, ident));
    v = op(v, dpp_f64<0x112, 0xf>(v, ident));
    v = op(v, dpp_f64<0x114, 0xf>(v, ident));
    v = op(v, dpp_f64<0x118, 0xf>(v, ident));
    v = op(v, dpp_f64<0x142, 0xa>(v, ident));
    v = op(v, dpp_f64<0x143, 0xc>(v, ident));
    return readlane_f64(v, 63);
}
__device__ inline uint32_t first_lane(uint64_t m) { return m ? (uint32_t)__ffsll((unsigned long long)m) - 1 : 64u; }
// arr[i] of a small register array without dynamic indexing (which would
// place the array in scratch memory)
template <typename T, int N>
__device__ inline T pick(const T (&arr)[N], uint32_t i) {
    T r = arr[0];
#pragma unroll
    for (int u = 1; u < N; u++) r = i == (uint32_t)u ? arr[u] : r;
    return r;
}

// ---------------------------------------------------------------------------
// loader: LDS-DMA of TbPre::{add, th} into the ring, 128 positions per chunk
// ---------------------------------------------------------------------------
// A chunk may only overwrite positions no longer needed: chunk c is allowed
// once 128c + 128 <= first + RING, `first` = the oldest position this round
// still reads.  The source arrays carry 128 elements of slack past the batch.
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

__device__ __attribute__((always_inline)) inline void ld_chunk(ChainShared& sh, uint32_t c, const TbPre& pre,
                                                              uint32_t lane) {
    const uint32_t s0 = (c * 64u) & (RING_G - 1);   // first slot of the chunk (row aligned)
    const uint32_t g = c * 64u + swz(lane);         // granule this lane's slot holds
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&sh.r_add[s0];
    const uint32_t lt = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)&sh.r_th[s0];
    glds16(pre.add + 2u * g, __builtin_amdgcn_readfirstlane(la));
    glds16(pre.th + 2u * g, __builtin_amdgcn_readfirstlane(lt));
}

// issue every chunk the ring can take while `first` is still needed
__device__ __attribute__((always_inline)) inline void ld_issue(TbLoader& L, ChainShared& sh, uint32_t first,
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
__device__ __attribute__((always_inline)) inline void ld_until(TbLoader& L, ChainShared& sh, uint32_t first,
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

// ---------------------------------------------------------------------------
// exact step in a fast mode
// ---------------------------------------------------------------------------
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

// The live-key step from stored digits Dpred (exact integer-valued double,
// positive, in the decade/binade of P) in a fast mode: tokens (the
// unquantized double) and the next stored digits D' -- NaN when the step
// leaves the regime: sum >= th (= min(capacity, n): clamp or allow), D' out of
// the decade, or an expired key (add NaN).
template <int MODE>
__device__ inline double tb_step_d(double Dpred, double P, double R, double add, double th, double& tokens) {
    const double T = MODE == QM_DEC ? rlq::div_pow10(Dpred, P, R)   // strtod("D e(E-13)")
                                    : Dpred * R;                    // exact: R = 2^E
    const double sum = T + add;
    tokens = sum;
    double Dn;
    if (MODE == QM_DEC) {
        Dn = round_scaled_Pd(sum, P);                               // %.14g of a positive sum
        if (!(Dn >= (double)DEC_LO && Dn < (double)DEC_HI)) Dn = __builtin_nan("");
    } else {
        Dn = sum * P;                                               // exact scaling
        if (!(Dn >= (double)BIN_LO && Dn < (double)BIN_HI && Dn == floor(Dn))) Dn = __builtin_nan("");
    }
    if (!(sum < th)) Dn = __builtin_nan("");
    return Dn;
}

__device__ inline int32_t fast_mode(int64_t D, int32_t E, int32_t profile) {
    if (profile == PROFILE_REDIS7)
        return (D >= DEC_LO && D < DEC_HI && 13 - E >= 1 && 13 - E <= 22) ? QM_DEC : QM_NONE;
    return (D >= BIN_LO && D < BIN_HI && E > -1000 && E < 900) ? QM_BIN : QM_NONE;
}
__device__ inline void mode_scale(int32_t mode, int32_t E, double& P, double& R) {
    if (mode == QM_DEC) {
        P = rlq::pow10_exact(13 - E);
        R = 1.0 / P;
    } else {
        P = ldexp(1.0, -E);
        R = ldexp(1.0, E);
    }
}

// Committed runs of the chain, indexed by the run's first sorted position
// (k_tb_expand's input; len is reset to 0 once the run is expanded)
struct TbRuns {
    uint16_t* len;       // requests in the run starting here (0: none), <= CH_TILE
    int16_t* E;          // decade / binade exponent
    int64_t* D0;         // exact stored state before the run
    int64_t* D1;         // exact stored state after it, as the chain resolved it
};

struct RingSrc {
    const ChainShared& sh;
    __device__ double add(uint32_t p) const { return ring_add(sh, p); }
    __device__ double th(uint32_t p) const { return ring_th(sh, p); }
};
struct GlobSrc {
    const double* a;
    const double* t;
    __device__ double add(uint32_t p) const { return a[p]; }
    __device__ double th(uint32_t p) const { return t[p]; }
};

// Exact replay of [p, p + len) (len <= CH_TILE) from the exact stored digits
// D0 by one wave: lane l steps requests [p + 8l, p + 8l + 8) from a guessed
// start; the guesses are refined by an exclusive scan of every lane's actual
// change until the first lane whose start changed lies past the first regime
// exit (by induction over lanes, every start up to there is then exact).
// Returns the relative position of the first step that leaves the regime
// (len if none) and in Dend the exact digits before it (after the span).
// OUT: writes tokens and DENIED for every in-regime step.
template <int MODE, bool OUT, typename Src>
__device__ __attribute__((always_inline)) inline uint32_t exact_span(const Src& src, uint32_t p, uint32_t len,
                                                                     int64_t D0, double P, double R, int64_t& Dend,
                                                                     const ReqArgs& a, uint32_t& iters) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t off = lane * K;
    const uint32_t nv = off < len ? ((len - off) < (uint32_t)K ? (len - off) : (uint32_t)K) : 0u;
    double add[K], th[K];
    int64_t S = 0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nv;
        add[q] = v ? src.add(p + off + q) : 0.0;
        th[q] = v ? src.th(p + off + q) : __builtin_inf();
        const double pr = add[q] * P;
        if (fabs(pr) < 0x1p49) S += (int64_t)rint(pr);     // NaN / huge: a regime exit anyway
    }
    const int64_t incl = wave_incl_scan_i64(S);
    int64_t st = D0 + incl - S;
    const uint32_t last = len ? (len - 1) / K : 0u;
    for (;;) {
        double D = (double)st, Db = 0.0;
        uint32_t bq = NO_STOP;
#pragma unroll
        for (int q = 0; q < K; q++) {
            if ((uint32_t)q < nv && bq == NO_STOP) {
                double tk;
                const double Dn = tb_step_d<MODE>(D, P, R, add[q], th[q], tk);
                if (!(Dn == Dn)) {
                    bq = q;
                    Db = D;
                } else {
                    if (OUT) {
                        a.tok[p + off + q] = tk;
                        a.dec[p + off + q] = DEC_DENIED;
                    }
                    D = Dn;
                }
            }
        }
        const bool brk = bq != NO_STOP;
        const int64_t A = brk ? 0 : (int64_t)D - st;
        const int64_t ai = wave_incl_scan_i64(A);
        const int64_t nst = D0 + ai - A;
        const uint32_t fb = first_lane(__ballot(brk));
        const uint32_t fd = first_lane(__ballot(nv > 0 && nst != st));
        iters++;
        if (fb == 64u ? fd == 64u : fd > fb) {
            if (fb < 64u) {
                Dend = (int64_t)readlane_f64(Db, fb);
                return fb * K + (uint32_t)__builtin_amdgcn_readlane((int)bq, (int)fb);
            }
            Dend = (int64_t)readlane_f64(D, last);
            return len;
        }
        st = nst;
    }
}

// ---------------------------------------------------------------------------
// producers
// ---------------------------------------------------------------------------
// Summary of tile t of the window [pfirst, pfirst + pcnt) at scale P, into
// tile[buf][t] and its near list.  State-free.
template <int MODE>
__device__ __attribute__((always_inline)) inline void ch_produce(ChainShared& sh, uint32_t buf, uint32_t t,
                                                                uint32_t pfirst, uint32_t pcnt, double P) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t toff = t * CH_TILE;
    if (toff >= pcnt) return;
    const uint32_t myoff = toff + lane * K;
    const uint32_t nv = myoff < pcnt ? ((pcnt - myoff) < (uint32_t)K ? (pcnt - myoff) : (uint32_t)K) : 0u;
    const uint32_t i0 = pfirst + myoff;

    // my positions [i0, i0 + K): K/2 granules, one more when i0 is odd
    // (pfirst is block-uniform, so is the parity)
    double add[K], th[K];
    {
        double ga[K + 2], gt[K + 2];
        const uint32_t g0 = i0 >> 1;
#pragma unroll
        for (int j = 0; j < K / 2 + 1; j++) {
            if (j < K / 2 || (i0 & 1u)) {
                const double2 x = sh.r_add[ring_slot(g0 + j)];
                const double2 y = sh.r_th[ring_slot(g0 + j)];
                ga[2 * j] = x.x; ga[2 * j + 1] = x.y;
                gt[2 * j] = y.x; gt[2 * j + 1] = y.y;
            } else {
                ga[2 * j] = ga[2 * j + 1] = 0.0;
                gt[2 * j] = gt[2 * j + 1] = 0.0;
            }
        }
        const uint32_t o = i0 & 1u;
#pragma unroll
        for (int q = 0; q < K; q++) {
            const bool v = (uint32_t)q < nv;
            add[q] = v ? (o ? ga[q + 1] : ga[q]) : 0.0;
            th[q] = v ? (o ? gt[q + 1] : gt[q]) : __builtin_inf();
        }
    }
    double cum = 0.0, cb[K];
    double ymin = __builtin_inf(), cmax = -__builtin_inf(), cmin = __builtin_inf();
    uint32_t nearm = 0, evq = NO_STOP;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const double a = add[q];
        cb[q] = cum;
        double pr = a * P;
        double rr = rint(pr);
        const bool ev = !(fabs(pr) < 0x1p49);                  // NaN (expired key) or huge
        if (ev && evq == NO_STOP) evq = q;
        if (ev) { pr = 0.0; rr = 0.0; }
        if (MODE == QM_DEC) {
            const double err = ev ? 0.0 : __builtin_fma(a, P, -pr);    // a*P == pr + err exactly
            if (fabs((pr - rr) + err) > 0.5 - TAU_DEC) nearm |= 1u << q;
        } else if (fabs(pr - rr) == 0.5) {                              // exact tie: parity decides
            nearm |= 1u << q;
        }
        cum += rr;                                                      // exact: |cum| < 2^52
        if ((uint32_t)q < nv) {
            cmax = fmax(cmax, cum);
            cmin = fmin(cmin, cum);
            ymin = fmin(ymin, th[q] * P * CH_YSCALE - cum);
        }
    }
    const int64_t Si = (int64_t)cum;
    const int64_t incl = wave_incl_scan_i64(Si);
    const double ex = (double)(incl - Si);
    const double ymin_t = wave_reduce_f64(ymin - ex, __builtin_inf(), [](double x, double y) { return fmin(x, y); });
    const double cmax_t = wave_reduce_f64(ex + cmax, -__builtin_inf(), [](double x, double y) { return fmax(x, y); });
    const double cmin_t = wave_reduce_f64(ex + cmin, __builtin_inf(), [](double x, double y) { return fmin(x, y); });
    const uint32_t ev_t = wave_min_u32(evq != NO_STOP ? lane * K + evq : NO_STOP);
    const uint32_t ncnt = (uint32_t)__popc(nearm);
    const uint32_t ninc = wave_scan_u32(ncnt, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    {
        uint32_t k = ninc - ncnt;
#pragma unroll
        for (int q = 0; q < K; q++) {
            if ((nearm >> q) & 1u) {
                if (k < (uint32_t)CH_NE) {
                    sh.ne_pred[buf][t][k] = ex + cb[q];
                    sh.ne_add[buf][t][k] = add[q];
                    sh.ne_th[buf][t][k] = th[q];
                }
                k++;
            }
        }
    }
    if (lane == 63) {
        ChTile& T = sh.tile[buf][t];
        T.S = incl;
        T.ymin = ymin_t;
        T.cmax = cmax_t;
        T.cmin = cmin_t;
        T.ev = ev_t;
        T.nc = ninc;
    }
}

// ---------------------------------------------------------------------------
// chain
// ---------------------------------------------------------------------------
enum : uint32_t { CH_FULL = 0, CH_STOP = 1, CH_PARTIAL = 2 };

struct ChOutcome {
    uint32_t kind;
    uint32_t q;        // FULL: window end; STOP: the exiting step; PARTIAL: end of the committed part
    int64_t D;         // exact stored digits before position q
};

__device__ inline void record_run(const TbRuns& runs, uint32_t pos, uint32_t len, int32_t E, int64_t D0, int64_t D1) {
    if ((threadIdx.x & 63) == 0 && len) {
        runs.len[pos] = (uint16_t)len;
        runs.E[pos] = (int16_t)E;
        runs.D0[pos] = D0;
        runs.D1[pos] = D1;
    }
}

// Resolve the chain window of state s (its tiles are in tile[s.cbuf]).
template <int MODE>
__device__ __attribute__((always_inline)) inline ChOutcome ch_resolve(ChainShared& sh, const ChState& s, double P,
                                                                     double R, const ReqArgs& a, const TbRuns& runs,
                                                                     uint32_t& iters, uint32_t* dbg) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t cb = s.cbuf;
    const uint32_t nt = (s.ccnt + CH_TILE - 1) / CH_TILE;
    const double LO = MODE == QM_DEC ? (double)DEC_LO : (double)BIN_LO;
    const double HI = MODE == QM_DEC ? (double)DEC_HI : (double)BIN_HI;
    // tile prefix sums and near-list prefix (tiles before the first overflow)
    int64_t TS[CH_NP];
    uint32_t NPF[CH_NP + 1];
    uint32_t ovt = nt;
    {
        int64_t acc = 0;
        uint32_t nacc = 0;
#pragma unroll
        for (int t = 0; t < CH_NP; t++) {
            TS[t] = acc;
            NPF[t] = nacc;
            if ((uint32_t)t < nt) {
                acc += sh.tile[cb][t].S;
                const uint32_t nc = sh.tile[cb][t].nc;
                if (ovt == nt && nc > (uint32_t)CH_NE) ovt = t;
                if ((uint32_t)t < ovt) nacc += nc;
            }
        }
        NPF[CH_NP] = nacc;
    }
    const uint32_t ne = NPF[CH_NP];

    // Near steps in sequence order, 64 at a time.  A step's exact result
    // depends on its exact predecessor = nominal + (offset before it); far
    // steps keep the offset, so the offset before step g is the flips (exact
    // result - nominal result) of the earlier near steps.  Wave fixed point:
    // evaluate every step at the current guess, scan the flips, re-guess; when
    // no guess changes before the first step that leaves the regime, the
    // guesses are the true offsets (induction over lanes).
    uint32_t nstop = NO_STOP;
    {
        constexpr int ITMAX = 16;
        int32_t cbo = 0;
        for (uint32_t b = 0; b < ne; b += 64) {
            const uint32_t g = b + lane;
            const bool v = g < ne;
            uint32_t t = 0;
#pragma unroll
            for (int u = 1; u < CH_NP; u++) t += g >= NPF[u] ? 1u : 0u;
            const uint32_t k = v ? g - pick(NPF, t) : 0u;
            const double pn = v ? (double)(s.D + pick(TS, t)) + sh.ne_pred[cb][t][k] : 0.0;
            const double ad = v ? sh.ne_add[cb][t][k] : 0.0;
            const double th = v ? sh.ne_th[cb][t][k] : __builtin_inf();
            const double r = rint(ad * P);
            int32_t est = 0, flip = 0;
            uint32_t stop_lane = 64;
            for (int it = 0;; it++) {
                double tk;
                const double pred = pn + (double)(cbo + est);
                const double Dn = tb_step_d<MODE>(pred, P, R, ad, th, tk);
                const bool brk = v && !(Dn == Dn);
                flip = (!v || brk) ? 0 : (int32_t)(Dn - (pred + r));
                const int32_t incl = (int32_t)wave_scan_u32((uint32_t)flip, 0u,
                                                            [](uint32_t x, uint32_t y) { return x + y; });
                const int32_t en = incl - flip;
                const uint32_t fb = first_lane(__ballot(brk));
                const uint32_t fc = first_lane(__ballot(v && en != est));
                iters++;
                if (fc >= fb) { stop_lane = fb; break; }             // converged up to the first exit
                if (it + 1 == ITMAX) { stop_lane = fc; break; }      // lanes < fc are exact
                est = en;
            }
            if (v && lane < stop_lane) sh.ne_off[g] = cbo + est + flip;
            if (stop_lane < 64) {
                nstop = b + stop_lane;
                break;
            }
            cbo += __builtin_amdgcn_readlane(est + flip, 63);
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // ne_off visible to this wave
    }

    // Tile walk: commit tiles whose bounds exclude a regime exit; replay the
    // others exactly.
    ChOutcome o;
    o.kind = CH_FULL;
    int64_t Dcur = s.D;        // exact digits at the current tile start
    int32_t off = 0;           // offset (exact - nominal) at the current tile start
    for (uint32_t t = 0; t < nt; t++) {
        const ChTile T = sh.tile[cb][t];
        const uint32_t pos = s.cfirst + t * CH_TILE;
        const uint32_t len = (s.ccnt - t * CH_TILE) < CH_TILE ? (s.ccnt - t * CH_TILE) : CH_TILE;
        const uint32_t npf1 = pick(NPF, t + 1);
        const bool nst_in = nstop != NO_STOP && nstop < npf1;
        const bool forced = t >= ovt || nst_in || T.ev != NO_STOP;
        const int32_t off_out = (!forced && T.nc) ? sh.ne_off[npf1 - 1] : off;
        const double Dt = (double)Dcur, nc = (double)T.nc;
        const bool cand = forced || !(Dt + nc + T.cmax < HI) || !(Dt - nc + T.cmin >= LO) ||
                          !(Dt + nc + 3.0 < T.ymin);
        if (!cand) {
            const int64_t D1 = Dcur + T.S + (off_out - off);
            record_run(runs, pos, len, s.E, Dcur, D1);
            Dcur = D1;
            off = off_out;
            continue;
        }
        int64_t Dq = 0;
        const uint32_t brk = exact_span<MODE, false>(RingSrc{sh}, pos, len, Dcur, P, R, Dq, a, iters);
        if (dbg && lane == 0) atomicAdd(&dbg[20], 1u);
        record_run(runs, pos, brk, s.E, Dcur, Dq);
        if (brk < len) {
            o.kind = CH_STOP;
            o.q = pos + brk;
            o.D = Dq;
            return o;
        }
        const bool agree = Dq == Dcur + T.S + (off_out - off);
        Dcur = Dq;
        off = off_out;
        if (forced || !agree) {
            if (t + 1 < nt) {
                o.kind = CH_PARTIAL;
                o.q = pos + len;
                o.D = Dcur;
                return o;
            }
        }
    }
    o.q = s.cfirst + s.ccnt;
    o.D = Dcur;
    return o;
}

// Replay one heavy token-bucket segment [j0, j1) with the whole block.
template <bool LCFG>
__device__ __attribute__((always_inline)) inline void ch_segment(ChainShared& sh, TbEntry* e, uint32_t j0, uint32_t j1,
                                                                const CfgDev* __restrict__ cfgs, int32_t profile,
                                                                const ReqArgs& a, const TbPre& pre, uint32_t* eflags,
                                                                uint32_t* dbg, const TbRuns& runs) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t nrounds = 0, iters = 0, par = 0, nserial = 0;
    TbLoader L;
    L.next = j0 / 128u;
    L.issued = 0;
    if (tid == 0) {
        const TbQ q = tb_quant(e->tok, profile);
        ChState s0;
        s0.D = q.D;
        s0.E = q.E;
        s0.mode = fast_mode(q.D, q.E, profile);
        s0.cfirst = j0;
        s0.ccnt = 0;
        s0.pfirst = j0;
        s0.pbuf = 0;
        s0.cbuf = 1;
        sh.st[0] = s0;
    }
    if (wave == (uint32_t)CH_LOADER) ld_until(L, sh, j0, j0 + 2 * CH_W, j1, pre, lane);
    lds_barrier();
    for (;;) {
        const ChState s = sh.st[par];
        if (s.ccnt == 0 && s.pfirst >= j1) break;                 // block-uniform
        const uint32_t pcnt = (s.mode != QM_NONE && s.pfirst < j1) ? ((j1 - s.pfirst) < CH_W ? (j1 - s.pfirst) : CH_W)
                                                                   : 0u;
        double P = 1.0, R = 1.0;
        if (s.mode != QM_NONE) mode_scale(s.mode, s.E, P, R);
        nrounds++;
        if (wave >= 1 && wave <= (uint32_t)CH_NP) {
            if (pcnt) {
                if (s.mode == QM_DEC) ch_produce<QM_DEC>(sh, s.pbuf, wave - 1, s.pfirst, pcnt, P);
                else ch_produce<QM_BIN>(sh, s.pbuf, wave - 1, s.pfirst, pcnt, P);
            }
        } else if (wave == (uint32_t)CH_LOADER) {
            const uint32_t first = s.ccnt ? s.cfirst : s.pfirst;
            ld_until(L, sh, first, s.pfirst + 2 * CH_W, j1, pre, lane);
        } else {
            // ---- chain wave ----
            ChState nx;
            nx.pbuf = s.pbuf ^ 1u;
            nx.cbuf = s.pbuf;
            ChOutcome o{CH_PARTIAL, s.pfirst, s.D};
            bool restart = true, force = false;
            if (s.ccnt > 0) {
                o = s.mode == QM_DEC ? ch_resolve<QM_DEC>(sh, s, P, R, a, runs, iters, dbg)
                                     : ch_resolve<QM_BIN>(sh, s, P, R, a, runs, iters, dbg);
                if (dbg && lane == 0) atomicAdd(&dbg[3 + o.kind], 1u);
                if (o.kind == CH_FULL) {
                    restart = false;
                    nx.D = o.D;                 // exact at s.pfirst
                } else {
                    force = o.kind == CH_STOP;
                }
            } else if (pcnt) {
                restart = false;                // first window of a run of rounds
                nx.D = s.D;
                if (dbg && lane == 0) atomicAdd(&dbg[6], 1u);
            }                                   // else off the fast decades: serial steps from s.pfirst
            if (!restart) {
                nx.E = s.E;
                nx.mode = s.mode;
                nx.cfirst = s.pfirst;
                nx.ccnt = pcnt;
                nx.pfirst = s.pfirst + pcnt;
            } else {
                // exact serial steps: the exiting step, then on while the state
                // is off the fast decades or the last step left the regime
                uint32_t q = o.q;
                int64_t D = o.D;
                int32_t E = s.E;
                int32_t mode = fast_mode(D, E, profile);
                const uint32_t lim = (j1 - s.pfirst) < CH_W ? j1 : s.pfirst + CH_W;   // resident in the ring
                const uint32_t pq = q + lane;
                const int64_t nvec = pq < j1 ? a.n[pq] : 1;
                const uint32_t cvec = pq < j1 ? a.cfg[pq] : 0u;
                for (uint32_t k = 0; q < lim && k < (uint32_t)CH_SERIAL && (force || mode == QM_NONE); k++) {
                    const double add = ring_add(sh, q);
                    const bool alive = add == add;
                    const int64_t nn = readlane_i64(nvec, k);
                    const CfgDev& C = cfgs[(uint32_t)__builtin_amdgcn_readlane((int)cvec, (int)k)];
                    const TbEval v = tb_eval(QM_NONE, D, E, 1.0, 1.0, alive, alive ? add : 0.0, C.limit_d,
                                             (double)nn, profile);
                    if (lane == 0) write_out_tb(a, q, v.allowed ? DEC_ALLOWED : DEC_DENIED, v.tokens);
                    force = v.allowed || v.clamped || !alive;
                    const TbQ nq = tb_quant(v.tokens, profile);
                    D = nq.D;
                    E = nq.E;
                    mode = fast_mode(D, E, profile);
                    q++;
                    nserial++;
                }
                nx.D = D;
                nx.E = E;
                nx.mode = mode;
                nx.cfirst = q;
                nx.ccnt = 0;
                nx.pfirst = q;
            }
            if (lane == 0) sh.st[par ^ 1u] = nx;
        }
        par ^= 1u;
        lds_barrier();
    }
    if (tid == 0) {
        const ChState s = sh.st[par];
        e->tok = tb_value(s.D, s.E, profile);
        e->last = pre.lq[j1 - 1];
        e->when = pre.when[j1 - 1];
        if (dbg) {
            atomicAdd(&dbg[0], nrounds);
            atomicAdd(&dbg[1], iters);
            atomicMax(&dbg[2], nrounds);
            atomicAdd(&dbg[21], nserial);
        }
    }
    (void)eflags;
}

// Outputs of the committed runs: one wave per run, exact_span with outputs
// from the run's exact start state, checked against the state the chain
// resolved at the run's end.  Waves scan the batch in 512-position blocks and
// expand the runs that start in their block.
__global__ __launch_bounds__(256) void k_tb_expand(uint32_t m, TbRuns runs, int32_t profile, ReqArgs a, TbPre pre,
                                                   uint32_t* eflags) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    uint32_t iters = 0;
    for (uint32_t b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; b * CH_TILE < m; b += nw) {
        uint32_t mask = 0;
#pragma unroll
        for (int q = 0; q < K; q++) {
            const uint32_t p = b * CH_TILE + lane * K + q;
            if (p < m && runs.len[p]) mask |= 1u << q;
        }
        for (;;) {
            const uint64_t any = __ballot(mask != 0);
            if (!any) break;
            const uint32_t L = first_lane(any);
            const uint32_t qm = (uint32_t)__builtin_amdgcn_readlane((int)mask, (int)L);
            const uint32_t p = b * CH_TILE + L * K + (uint32_t)__builtin_ctz(qm);
            if (lane == L) mask &= mask - 1u;
            const uint32_t len = runs.len[p];
            const int32_t E = runs.E[p];
            const int64_t D0 = runs.D0[p], D1 = runs.D1[p];
            int64_t Dend = 0;
            uint32_t brk;
            double P, R;
            if (profile == PROFILE_REDIS7) {
                mode_scale(QM_DEC, E, P, R);
                brk = exact_span<QM_DEC, true>(GlobSrc{pre.add, pre.th}, p, len, D0, P, R, Dend, a, iters);
            } else {
                mode_scale(QM_BIN, E, P, R);
                brk = exact_span<QM_BIN, true>(GlobSrc{pre.add, pre.th}, p, len, D0, P, R, Dend, a, iters);
            }
            if (lane == 0) {
                if (brk != len || Dend != D1) atomicOr(eflags, EF_INTERNAL);
                runs.len[p] = 0;
            }
        }
    }
}

// Heavy token-bucket segments: one per block from a work queue, the huge list
// (longest segments) first; window segments in the heavy list are k_replay's.
template <bool LCFG>
__global__ __launch_bounds__(CH_BLOCK) void k_tb_chain(const uint32_t* __restrict__ sk,
                                                       const SegRec* __restrict__ huge,
                                                       const uint32_t* __restrict__ nhuge_p,
                                                       const SegRec* __restrict__ heavy,
                                                       const uint32_t* __restrict__ nheavy_p, uint32_t* qctr,
                                                       uint32_t win_base, TbEntry* tb,
                                                       const CfgDev* __restrict__ gcfgs, uint32_t ncfg,
                                                       int32_t profile, ReqArgs a, TbPre pre, uint32_t* eflags,
                                                       uint32_t* dbg, TbRuns runs) {
    __shared__ ChainShared sh;
    __shared__ uint32_t s_u;
    __shared__ CfgDev s_cfg[LCFG ? MAX_LCFG : 1];
    if (LCFG) {
        for (uint32_t c = threadIdx.x; c < ncfg; c += blockDim.x) s_cfg[c] = gcfgs[c];
        __syncthreads();
    }
    const CfgDev* cfgs = LCFG ? s_cfg : gcfgs;
    const uint32_t nhuge = *nhuge_p, nheavy = *nheavy_p;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t u;
            do {   // huge first, then heavy; skip window segments (k_replay's)
                u = atomicAdd(qctr, 1u);
            } while (u >= nhuge && u - nhuge < nheavy && sk[heavy[u - nhuge].j0] >= win_base);
            s_u = u;
        }
        __syncthreads();
        const uint32_t u = s_u;
        __syncthreads();
        if (u >= nhuge + nheavy) break;
        const SegRec sg = u < nhuge ? huge[u] : heavy[u - nhuge];
        const uint64_t t_seg = __builtin_amdgcn_s_memrealtime();
        ch_segment<LCFG>(sh, &tb[sk[sg.j0]], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre, eflags, dbg, runs);
        __syncthreads();
        if (threadIdx.x == 0 && dbg) atomicMax(&dbg[8], (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_seg));
    }
}

}  // namespace rl
