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
//       current decade: per tile (64 lanes x CH_K requests) the nominal sum of r, bounds of
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

// 6 producers x 6 requests per lane: 8 waves per block, 2 per SIMD, so a
// wave may hold 256 VGPRs.  With the multi-decade windows' code the 9-wave
// shape (7 x 5, at most 168 VGPRs) spilled inside the chain's loops even with
// that code out of line: configs[1] 2.42 vs 2.80e9, Zipf 1.5 8.6 vs 9.4e8 on
// one box (profiles/r5_xdec_ab.txt)
#ifndef RL_CH_NP
#define RL_CH_NP 6
#endif
#ifndef RL_CH_K
#define RL_CH_K 6
#endif
constexpr int CH_K = RL_CH_K;                          // requests per producer lane
constexpr int CH_NP = RL_CH_NP;                        // producer waves
constexpr uint32_t CH_TILE = 64u * CH_K;               // requests per producer wave
constexpr uint32_t CH_W = (uint32_t)CH_NP * CH_TILE;   // requests per window
constexpr int CH_NE = 64;                              // near-list capacity per tile
// Wave roles.  Waves of a block are dealt to the CU's four SIMDs round-robin
// (wave w on SIMD (w + base) mod 4), so the chain (wave 0) shares its SIMD
// with the mostly idle loader (wave 4) and the producers pair up on the
// other three SIMDs.
constexpr int CH_LOADER = 4;
static_assert(CH_NP + 2 <= 16 && CH_NP >= 3, "wave roles");
__device__ inline int ch_producer_index(uint32_t wave) {
    if (wave == 0 || wave == (uint32_t)CH_LOADER) return -1;
    return (int)wave - (wave < (uint32_t)CH_LOADER ? 1 : 2);
}
constexpr int CH_BLOCK = (CH_NP + 2) * 64;
constexpr int CH_SERIAL = 64;                          // serial exact steps per round at most
#ifndef RL_CH_UNCHECKED
#define RL_CH_UNCHECKED 2
#endif
constexpr int CH_UNCHECKED = RL_CH_UNCHECKED;          // near fixed-point passes before the first convergence test
#ifndef RL_XDEC
#define RL_XDEC 1
#endif
constexpr bool CH_XDEC = RL_XDEC != 0;                 // multi-decade windows (rl_tb_xdec.h), Redis-7 profile
#ifndef RL_HEAVY_G
#define RL_HEAVY_G 2
#endif
constexpr int HEAVY_G = RL_HEAVY_G;                    // heavy segments per wave claim (k_tb_chain phase 2)
// conservative scale of the allow/clamp threshold th*P (covers the rounding of
// th*P and of the bound arithmetic with a wide margin)
constexpr double CH_YSCALE = 1.0 - 0x1p-28;

// LDS ring of the segment's inputs by absolute sorted position, in 16-byte
// granules (two positions).  Granule G lives in slot swz(G mod RING_G): an XOR
// of its column (G mod 16) with bits 4-5, so the 8 lanes of one ds_read_b128
// cycle (lane l reads granule G0 + 4l + j) hit distinct banks, while a row of
// 16 slots still holds 16 consecutive granules (the loader's LDS-DMA writes
// slots lane-linearly and swizzles the SOURCE address instead).
#ifndef RL_RING
#define RL_RING 8192
#endif
constexpr uint32_t RING = RL_RING;               // positions
constexpr uint32_t RING_G = RING / 2;            // granules
__host__ __device__ constexpr uint32_t swz(uint32_t g) { return (g & ~15u) | ((g & 15u) ^ ((g >> 4) & 3u)); }
__host__ __device__ constexpr uint32_t ring_slot(uint32_t granule) { return swz(granule & (RING_G - 1)); }
// the chain window, the producers' window and the loader's next window
static_assert(RING >= 3 * CH_W + 256, "the ring must hold three windows");

struct ChTile {
    int64_t S;          // nominal sum of the tile's increments r
    double Sd;          // S as a double (the producers' state bound sums it every round)
    double ymin;        // min over steps of (th * P * CH_YSCALE - inclusive nominal prefix)
    double cmax, cmin;  // max / min inclusive nominal prefix
    double dmax;        // the near band assumed every state of the tile is <= dmax
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
    uint32_t hot;       // diagnostics: segment of >= 65536 requests
};

// Speculative restart: in a round whose chain window will likely leave the
// regime, the producers predict the exit from nominal states (the exit step q
// and the decade E of its result) and summarize the window from q + 1 at scale
// 10^(13 - E) instead of the window after the chain's.  When the chain's
// exact exit and serial steps end at q + 1 in decade E, the next round
// resolves that window at once -- no producers-only round.
struct ChSpec {
    uint32_t valid;
    uint32_t first, cnt;   // window [first, first + cnt), summarized in tile[buf]
    uint32_t buf;
    int32_t E;             // decimal mode at 10^(13 - E) (without XDEC windows)
    double v0;             // XDEC: the guessed state after the exit (tokens): the window's plan starts there
};

// The window the producers summarized into tile[buf] (its representation:
// the chain converts its exact state into it before resolving the window)
struct ChWin {
    int32_t mode;          // QM_DEC / QM_BIN / QM_XDEC
    int32_t E;             // decade / binade, or the XDEC floor F
};

struct ChainShared {
    double2 r_add[RING_G];       // TbPre::add
    double2 r_th[RING_G];        // TbPre::th
    ChTile tile[2][CH_NP];
    // near steps: tile-relative nominal predecessor (XDEC: int64 bits), add,
    // th (XDEC: the step's nominal increment r, int64 bits)
    double ne_pred[2][CH_NP][CH_NE];
    double ne_add[2][CH_NP][CH_NE];
    double ne_th[2][CH_NP][CH_NE];
    uint64_t ne_kind[2][CH_NP];        // XDEC: bit k = near entry k is a reset step (a decade up)
    uint16_t ne_rank[2][CH_NP][64];    // near steps of the tile before each producer lane
    int32_t ne_off[CH_NP * CH_NE];     // chain: resolved offset after each near step
    ChState st[2];
    ChSpec spec[2];                    // producers' speculative window of the round
    ChWin win[2];                      // the representation of tile[buf]'s window
    double plan_s[CH_NP], plan_sp[CH_NP];   // ch_plan_par: each producer wave's tile sums
    uint32_t plan_tag[CH_NP];               // and the plan number they belong to (0 at kernel start)
#ifdef RL_STAMPS
    uint32_t wk[2];                    // the round's longest producer work (cycles / 16)
#endif
};

__device__ inline double ring_add(const ChainShared& sh, uint32_t p) {
    return reinterpret_cast<const double*>(&sh.r_add[ring_slot(p >> 1)])[p & 1u];
}
__device__ inline double ring_th(const ChainShared& sh, uint32_t p) {
    return reinterpret_cast<const double*>(&sh.r_th[ring_slot(p >> 1)])[p & 1u];
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
// max / min of two doubles that are never NaN: one v_max_f64 / v_min_f64 (the
// compiler's fmax/fmin canonicalize both inputs first, three instructions)
__device__ inline double vmax_f64(double a, double b) {
    double r;
    __asm__ volatile("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));   // volatile: never sunk into a branch
    return r;
}
__device__ inline double vmin_f64(double a, double b) {
    double r;
    __asm__ volatile("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
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
// inclusive wave scan of doubles (DPP, as wave_incl_scan_i64)
template <int CTRL, int RM>
__device__ inline double dpp_addf_step(double v) {
    return v + dpp_f64<CTRL, RM>(v, 0.0);
}
__device__ inline double wave_incl_scan_f64(double v) {
    v = dpp_addf_step<0x111, 0xf>(v);
    v = dpp_addf_step<0x112, 0xf>(v);
    v = dpp_addf_step<0x114, 0xf>(v);
    v = dpp_addf_step<0x118, 0xf>(v);
    v = dpp_addf_step<0x142, 0xa>(v);
    v = dpp_addf_step<0x143, 0xc>(v);
    return v;
}
// the same reduction, left in lane 63 only (its caller reads it there)
template <typename Op>
__device__ inline double wave_fold_f64(double v, double ident, Op op) {
    v = op(v, dpp_f64<0x111, 0xf>(v, ident));
    v = op(v, dpp_f64<0x112, 0xf>(v, ident));
    v = op(v, dpp_f64<0x114, 0xf>(v, ident));
    v = op(v, dpp_f64<0x118, 0xf>(v, ident));
    v = op(v, dpp_f64<0x142, 0xa>(v, ident));
    v = op(v, dpp_f64<0x143, 0xc>(v, ident));
    return v;
}
__device__ inline int64_t readfirstlane_i64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
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

// at most ~k LDS-DMA ops of this wave still in flight (k rounded down to a
// waitcnt immediate)
__device__ __attribute__((always_inline)) inline void ld_wait_at_most(uint32_t k) {
    if (k >= 48u) __asm__ volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (k >= 32u) __asm__ volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if (k >= 16u) __asm__ volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (k >= 8u) __asm__ volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (k >= 4u) __asm__ volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// make [.., target) resident: issue what is missing (and what the ring can
// take beyond it), then wait for the chunks below target only -- the ones
// issued after them (two LDS-DMA ops per chunk, completed in issue order as
// vmcnt counts them) stay in flight into the next round
__device__ __attribute__((always_inline)) inline void ld_until(TbLoader& L, ChainShared& sh, uint32_t first,
                                                              uint32_t target, uint32_t j1, const TbPre& pre,
                                                              uint32_t lane) {
    const uint32_t need = ((target < j1 ? target : j1) + 127u) / 128u;
    for (;;) {
        ld_issue(L, sh, first, j1, pre, lane);
        if (L.next >= need) {
            const uint32_t extra = L.next - need;      // chunks issued after the last needed one
            ld_wait_at_most(2u * (extra < L.issued ? extra : L.issued));
            L.issued = extra < L.issued ? extra : L.issued;
            break;
        }
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        L.issued = 0;
    }
}

// ---------------------------------------------------------------------------
// exact step in a fast mode
// ---------------------------------------------------------------------------
// RNE(x * P) as an exact integer-valued double (x*P < 2^52), P = 10^k exact;
// ge_lo: the exact x*P >= 1e13, i.e. x is not below the decade (a value in
// [1e13 - 0.5, 1e13) units rounds to 1e13 here but %.14g formats it with 14
// digits of the decade below)
__device__ inline double round_scaled_Pd(double x, double P, bool& ge_lo) {
    const double p = x * P;
    const double err = __builtin_fma(x, P, -p);       // x*P == p + err exactly
    ge_lo = (p > (double)DEC_LO) | ((p == (double)DEC_LO) & (err >= 0.0));
    // RNE of p, then the exact product decides a tie of p: p - rint(p) is
    // +-1/2 exactly only when p's fraction is 1/2 (p < 2^52 has ulp <= 1/2),
    // and |err| <= ulp(p)/2 cannot move a non-tie across the half
    double d = rint(p);
    const double h = p - d;                           // exact
    d += ((h == 0.5) & (err > 0.0)) ? 1.0 : 0.0;
    d -= ((h == -0.5) & (err < 0.0)) ? 1.0 : 0.0;
    return d;
}

// x / P correctly rounded (as IEEE division) for an integer-valued |x| < 2^47,
// P = 10^k (1 <= k <= 22, exact) and R within 2^-52 relative of 1/P (RN(1/P),
// or RN(1/10^j) times an exact 10^(j-k), rounded), in five dependent
// operations instead of the division's eleven.  q0 = RN(x R) is within 3 ulp
// of x/P and q1 = q0 + r R (r = x - q0 P, one rounding) within 1/2 ulp +
// 1e-15 ulp; the residual r1 = x - q1 P is then exact (|r1| <= 0.51 ulp(q1) P
// < 2^53 units of ulp(q1) ulp(P), as every 10^k has a mantissa below 2), and
// q1 + r1 R is within 0.51 ulp 2^-52 = 1.1e-16 ulp of x/P.  x/P = x /
// (2^k 5^k) with x an integer below 2^47 is never a rounding midpoint and lies
// at least ulp / (2 5^k) >= 2.1e-16 ulp from one (k <= 22), so the final
// rounding is RN(x/P).
// Checked against IEEE division on 1.3e9 random (x, k), with both reciprocals:
// scripts/div_p10_check.c.
__device__ __attribute__((always_inline)) inline double div_p10(double x, double P, double R) {
    const double q0 = x * R;
    const double q1 = __builtin_fma(__builtin_fma(-q0, P, x), R, q0);
    return __builtin_fma(__builtin_fma(-q1, P, x), R, q1);
}

// The live-key step from stored digits Dpred (exact integer-valued double,
// positive, in the decade/binade of P) in a fast mode: tokens (the
// unquantized double) and the next stored digits D' -- NaN when the step
// leaves the regime: sum >= th (= min(capacity, n): clamp or allow), D' out of
// the decade, or an expired key (add NaN).
template <int MODE>
__device__ inline double tb_step_d(double Dpred, double P, double R, double add, double th, double& tokens) {
    // strtod("D e(E-13)"): D < 2^47 and P = 10^k (k <= 22) are exact doubles,
    // so one correctly rounded division is strtod's result (Clinger's fast
    // path): div_p10 with R = RN(1/P) (mode_scale)
    const double T = MODE == QM_DEC ? div_p10(Dpred, P, R) : Dpred * R;   // binary: exact, R = 2^E
    const double sum = T + add;
    tokens = sum;
    double Dn;
    if (MODE == QM_DEC) {
        bool ge_lo;
        Dn = round_scaled_Pd(sum, P, ge_lo);                        // %.14g of a positive sum
        if (!(ge_lo & (Dn < (double)DEC_HI))) Dn = __builtin_nan("");
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
    if (mode == QM_DEC || mode == QM_XDEC) {   // XDEC: the window's floor scale 10^(13 - F)
        P = rlq::pow10_exact(13 - E);
        R = 1.0 / P;                       // RN(1/P): the decimal step's div_p10
    } else {
        P = ldexp(1.0, -E);
        R = ldexp(1.0, E);
    }
}

// Committed runs of the chain, indexed by the run's first sorted position
// (k_tb_expand's input; len is reset to 0 once the run is expanded)
struct TbRuns {
    uint16_t* len;       // requests in the run starting here (0: none), <= CH_TILE
    int16_t* E;          // decade / binade exponent (XDEC: the floor + XRUN)
    int64_t* D0;         // exact stored state before the run
    int64_t* D1;         // exact stored state after it, as the chain resolved it
    uint32_t* xlist;     // start positions of the runs of multi-decade windows (k_tb_expand_x)
    uint32_t* xcnt;      // their count (a zeroed control word of the batch set)
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
// D0 by one wave: lane l steps requests [p + K l, p + K l + K) from a guessed
// start (nominal prefix + goff, the caller's guess of the lane's offset); the
// guesses are refined by an exclusive scan of every lane's actual change until
// the first lane whose start changed lies past the first regime exit (by
// induction over lanes, every start up to there is then exact).  Returns the
// relative position of the first step that leaves the regime (len if none)
// and in Dend the exact digits before it (after the span).
// OUT: writes tokens and DENIED for every in-regime step.
template <int MODE, bool OUT, typename Src>
__device__ __attribute__((always_inline)) inline uint32_t exact_span(const Src& src, uint32_t p, uint32_t len,
                                                                     int64_t D0, int32_t goff, double P, double R,
                                                                     int64_t& Dend, const ReqArgs& a,
                                                                     uint32_t& iters) {
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
    int64_t st = D0 + incl - S + (lane ? goff : 0);
    const uint32_t last = len ? (len - 1) / K : 0u;
    for (uint32_t it = 0;; it++) {
        if (it > 64u) {            // cannot happen (one more exact lane per pass); never hang on it
            Dend = D0;
            return 0xffffffffu;
        }
        double D = (double)st, Db = 0.0;
        uint32_t bq = NO_STOP;
        // every lane evaluates every step (selects, no branches): a lane past
        // its steps or its first regime exit keeps its state
#pragma unroll
        for (int q = 0; q < K; q++) {
            const bool act = (uint32_t)q < nv && bq == NO_STOP;
            double tk;
            const double Dn = tb_step_d<MODE>(D, P, R, add[q], th[q], tk);
            const bool stop = act && !(Dn == Dn);
            const bool take = act && !stop;
            bq = stop ? (uint32_t)q : bq;
            Db = stop ? D : Db;
            if (OUT && take) {
                a.tok[p + off + q] = tk;
                a.dec[p + off + q] = DEC_DENIED;
            }
            D = take ? Dn : D;
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
// a lane's K consecutive adds and thresholds from the ring, positions i0 ..
// i0 + K - 1, in whole 16-byte granules: K / 2 or K / 2 + 1 ds_read_b128 per
// array instead of K ds_read_b64 (i0's parity must be wave-uniform: the
// callers' i0 is a window start plus an even offset)
__device__ __attribute__((always_inline)) inline void ring_read_k(const ChainShared& sh, uint32_t i0,
                                                                 double (&ra)[CH_K], double (&rt)[CH_K]) {
    constexpr int K = CH_K;
    if constexpr (K % 2 == 0) {
        const uint32_t g0 = i0 >> 1;
        if ((i0 & 1u) == 0u) {
#pragma unroll
            for (int j = 0; j < K / 2; j++) {
                const double2 a2 = sh.r_add[ring_slot(g0 + j)], t2 = sh.r_th[ring_slot(g0 + j)];
                ra[2 * j] = a2.x;
                ra[2 * j + 1] = a2.y;
                rt[2 * j] = t2.x;
                rt[2 * j + 1] = t2.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j <= K / 2; j++) {
                const double2 a2 = sh.r_add[ring_slot(g0 + j)], t2 = sh.r_th[ring_slot(g0 + j)];
                if (j > 0) {
                    ra[2 * j - 1] = a2.x;
                    rt[2 * j - 1] = t2.x;
                }
                if (j < K / 2) {
                    ra[2 * j] = a2.y;
                    rt[2 * j] = t2.y;
                }
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < K; q++) {
            ra[q] = ring_add(sh, i0 + q);
            rt[q] = ring_th(sh, i0 + q);
        }
    }
}


// Summary of tile t of the window [pfirst, pfirst + pcnt) at scale P, into
// tile[buf][t], its near list and per-lane near ranks.  State-free except for
// dmax, an estimated bound on the window's states that narrows the near band
// (|delta| <= (|D| + |D'|) 2^-53); the chain checks the bound per tile.
template <int MODE>
__device__ __attribute__((always_inline)) inline void ch_produce(ChainShared& sh, uint32_t buf, uint32_t t,
                                                                uint32_t pfirst, uint32_t pcnt, double P,
                                                                double dmax) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t toff = t * CH_TILE;
    if (toff >= pcnt) return;
    const uint32_t myoff = toff + lane * K;
    const uint32_t nv = myoff < pcnt ? ((pcnt - myoff) < (uint32_t)K ? (pcnt - myoff) : (uint32_t)K) : 0u;
    const uint32_t i0 = pfirst + myoff;
    // near band: a step is far when |frac(add P)| + |delta| < 1/2, with
    // delta = (eta + eps) P the rounding errors of x = strtod(D) and of
    // sum = x + add, |eta|, |eps| <= ulp / 2.  Every state is <= dmax, so x and
    // sum are <= dmax / P = f 2^e (f in [1/2, 1)) and their ulp <= 2^(e - 53):
    // |delta| <= 2^(e - 53) P -- the binade bound, up to 2x tighter than
    // (|D| + |D'|) 2^-53 (which the binary mode keeps)
    double band = 2.0 * dmax * 0x1.0000001p-53;
    if (MODE == QM_DEC) {
        // e: the binade of dmax / P, from the operands' binades and mantissas
        // (no division); the margin only ever picks the binade above
        int ed, ep;
        const double md = frexp(dmax, &ed), mp = frexp(P, &ep);
        const int e = ed - ep + (md * 0x1.00001p+0 >= mp ? 1 : 0);
        band = ldexp(P, e - 53) * 0x1.0000001p+0;
    }
    const double lim = 0.5 - (band + 0x1p-40);
    const double PY = P * CH_YSCALE;
    double add[K], th[K], cb[K];
    double cum = 0.0, ymin = __builtin_inf(), cmax = -__builtin_inf(), cmin = __builtin_inf();
    uint32_t nearm = 0, evq = NO_STOP;
    double ra[K], rt[K];
    ring_read_k(sh, i0, ra, rt);
    // branch-free: every ring slot is readable (positions past the window
    // read stale slots, masked by v), and the bounds use v_max / v_min on
    // values that are never NaN (no canonicalization)
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nv;
        const double araw = ra[q];
        const double h = rt[q];
        const double a = v ? araw : 0.0;
        add[q] = a;
        th[q] = h;
        cb[q] = cum;
        const double pr = a * P;
        const bool ok = fabs(pr) < 0x1p49;                 // else NaN (expired key) or huge: a stop
        evq = (!ok && evq == NO_STOP) ? (uint32_t)q : evq;
        const double prs = ok ? pr : 0.0;                  // rint on every lane (no branch)
        const double rr = rint(prs);
        if (MODE == QM_DEC) {
            const double fr = (prs - rr) + __builtin_fma(a, P, -pr);  // a*P - rr, one rounding (ok lanes)
            nearm |= (ok && fabs(fr) > lim) ? 1u << q : 0u;
        } else {
            nearm |= (ok && fabs(prs - rr) == 0.5) ? 1u << q : 0u;   // exact tie: parity decides
        }
        cum += rr;                                                    // exact: |cum| < 2^52
        const double mx = vmax_f64(cmax, cum), mn = vmin_f64(cmin, cum), ym = vmin_f64(ymin, h * PY - cum);
        cmax = v ? mx : cmax;
        cmin = v ? mn : cmin;
        ymin = v ? ym : ymin;
    }
    // the tile prefix: in doubles when every lane's sum is below 2^46 (the
    // tile's then below 2^52: exact), else in int64
    double ex, inclD;
    int64_t inclS;    // the exact tile sum (T.S: the nominal tile starts and runs' end states)
    if (__ballot(!(fabs(cum) < 0x1p46)) == 0ull) {
        inclD = wave_incl_scan_f64(cum);
        ex = inclD - cum;
        inclS = (int64_t)inclD;
    } else {
        const int64_t Si = (int64_t)cum;
        const int64_t incl = wave_incl_scan_i64(Si);
        ex = (double)(incl - Si);
        inclD = (double)incl;
        inclS = incl;
    }
    // the tile's bounds: lane 63 holds the reductions (no broadcast)
    const double ymin_t = wave_fold_f64(ymin - ex, __builtin_inf(), [](double x, double y) { return vmin_f64(x, y); });
    const double cmax_t = wave_fold_f64(ex + cmax, -__builtin_inf(), [](double x, double y) { return vmax_f64(x, y); });
    const double cmin_t = wave_fold_f64(ex + cmin, __builtin_inf(), [](double x, double y) { return vmin_f64(x, y); });
    const uint32_t ev_t = wave_scan_u32(evq != NO_STOP ? lane * K + evq : NO_STOP, 0xffffffffu,
                                        [](uint32_t a, uint32_t b) { return a < b ? a : b; });
    const uint32_t ncnt = (uint32_t)__popc(nearm);
    const uint32_t ninc = wave_scan_u32(ncnt, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    sh.ne_rank[buf][t][lane] = (uint16_t)(ninc - ncnt);
    if (nearm) {
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
        T.S = inclS;
        T.Sd = inclD;
        T.ymin = ymin_t;
        T.cmax = cmax_t;
        T.cmin = cmin_t;
        T.dmax = dmax;
        T.ev = ev_t;
        T.nc = ninc;
    }
}

// The chain window's likely regime exit (decimal mode; every producer wave
// computes the same): the first tile whose bounds admit an exit at the
// nominal state, the first nominal exit in it (nominal digit sums, no %.14g
// steps); the exit step's
// result (sum - th when it allows, else sum), carried on through the serial
// steps that follow an allow or a balance <= 0, decides the decade E.  A
// guess: the chain adopts the window only if its exact replay agrees
// (ch_segment).
__device__ __attribute__((always_inline)) inline ChSpec ch_predict(const ChainShared& sh, const ChState& s, double P,
                                                                  double R, uint32_t j1, bool xd) {
    constexpr int K = CH_K;
    ChSpec sp{0u, 0u, 0u, 0u, 0, 0.0};
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nt = (s.ccnt + CH_TILE - 1) / CH_TILE;
    const bool tv = lane < nt;
    // (a guess: nominal sums in doubles, exact below 2^53, and only a guess
    // beyond -- the chain adopts the window only if its exact replay agrees)
    const ChTile T = sh.tile[s.cbuf][tv ? lane : 0u];
    const double Sl = tv ? T.Sd : 0.0;
    const double dD = (double)s.D + (wave_incl_scan_f64(Sl) - Sl);   // nominal start of tile t
    const bool cand = tv && (T.ev != NO_STOP || !(dD + T.cmax < (double)DEC_HI) ||
                             !(dD + T.cmin >= (double)DEC_LO + 1.0) || !(dD + 3.0 < T.ymin));
    const uint64_t cm = __ballot(cand);
    if (!cm) return sp;
    const uint32_t c = first_lane(cm);
    const double Dc = readlane_f64(dD, c);
    const uint32_t p0 = s.cfirst + c * CH_TILE;
    const uint32_t clen = (s.ccnt - c * CH_TILE) < CH_TILE ? (s.ccnt - c * CH_TILE) : CH_TILE;
    const uint32_t off = lane * K;
    const uint32_t nv = off < clen ? ((clen - off) < (uint32_t)K ? (clen - off) : (uint32_t)K) : 0u;
    double add[K], th[K];
    ring_read_k(sh, p0 + off, add, th);
    double S = 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const bool v = (uint32_t)q < nv;
        add[q] = v ? add[q] : 0.0;
        th[q] = v ? th[q] : __builtin_inf();
        const double pr = add[q] * P;
        if (fabs(pr) < 0x1p49) S += rint(pr);
    }
    // nominal states (integer digits, no %.14g step): an exit where the sum
    // reaches th (D + add P >= th P) or the next digits leave the decade
    double D = Dc + (wave_incl_scan_f64(S) - S);
    uint32_t bq = NO_STOP;
    double D_b = 0.0, a_b = 0.0, th_b = 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const double pr = add[q] * P;
        const double Dn = D + rint(pr);
        const bool stop = (uint32_t)q < nv && bq == NO_STOP &&
                          (!(fabs(pr) < 0x1p49) || !(D + pr < th[q] * P) || !(Dn < (double)DEC_HI) ||
                           !(Dn >= (double)DEC_LO));
        bq = stop ? (uint32_t)q : bq;
        D_b = stop ? D : D_b;
        a_b = stop ? add[q] : a_b;
        th_b = stop ? th[q] : th_b;
        D = Dn;
    }
    const uint32_t fb = first_lane(__ballot(bq != NO_STOP));
    if (fb >= 64u) return sp;
    uint32_t first = p0 + fb * K + (uint32_t)__builtin_amdgcn_readlane((int)bq, (int)fb) + 1u;
    const double sum = readlane_f64(D_b, fb) / P + readlane_f64(a_b, fb), thv = readlane_f64(th_b, fb);
    const bool allow = sum >= thv;
    double post = allow ? sum - thv : sum;
    if (first >= j1 || !(post == post)) return sp;
    if (xd) {
        // multi-decade windows take any state after the exiting step: the
        // window starts right after it, its plan from the guessed state
        sp.valid = 1u;
        sp.first = first;
        sp.cnt = (j1 - first) < CH_W ? (j1 - first) : CH_W;
        sp.v0 = post;
        return sp;
    }
    if (allow || !(post > 0.0)) {
        // the serial steps go on after an allow (the next step too) and while
        // the balance is at or below zero (off the fast decades): they end
        // after the first step that leaves it positive -- the first positive
        // partial sum of the next adds, if no step on the way allows or
        // expires and the serial steps of one round reach it
        const uint32_t p = first + lane;
        const bool ok = p < j1 && lane < (uint32_t)CH_SERIAL - 1u;
        const double ad = ok ? ring_add(sh, p) : 0.0;
        const double tv2 = ok ? ring_th(sh, p) : __builtin_inf();
        double c = ad;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const double u = __shfl_up(c, o, 64);
            c = lane >= (uint32_t)o ? c + u : c;
        }
        const double vsum = post + c;
        const uint32_t fp = first_lane(__ballot(ok && vsum > 0.0));
        const uint32_t fx = first_lane(__ballot(ok && (vsum >= tv2 || !(ad == ad))));
        if (fp >= 64u || fx <= fp) return sp;
        post = readlane_f64(vsum, fp);
        first += fp + 1u;
        if (first >= j1) return sp;
    }
    if (!(post < 1e12)) return sp;
    const int e0 = (int)floor(log10(post));
#pragma unroll
    for (int d = -1; d <= 1; d++) {
        const int e = e0 + d, k = 13 - e;
        if (sp.valid || k < 1 || k > 22) continue;
        bool ge_lo;
        const double Dn = round_scaled_Pd(post, rlq::pow10_exact(k), ge_lo);
        if (ge_lo && Dn < (double)DEC_HI) {
            sp.valid = 1u;
            sp.E = e;
        }
    }
    sp.first = first;
    sp.cnt = (j1 - first) < CH_W ? (j1 - first) : CH_W;
    return sp;
}

}  // namespace rl
#include "rl_tb_xdec.h"
namespace rl {

// ---------------------------------------------------------------------------
// chain
// ---------------------------------------------------------------------------
enum : uint32_t { CH_FULL = 0, CH_STOP = 1, CH_PARTIAL = 2 };

// Diagnostic build only (-DRL_STAMPS): shader-clock sums per wave role and
// phase for segments of >= 65536 requests, added into dbg[24..39].
#ifdef RL_STAMPS
#define CH_T(v) do { __builtin_amdgcn_sched_barrier(0); (v) = __builtin_amdgcn_s_memtime(); \
                     __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define CH_T(v) do { } while (0)
#endif

struct ChOutcome {
    uint32_t kind;
    uint32_t q;        // FULL: window end; STOP: the exiting step; PARTIAL: end of the committed part
    int64_t D;         // exact stored digits before position q
    uint32_t iters;    // ch_resolve_x: the caller's pass count after the call
};

// Resolve the chain window of state s (its tiles are in tile[s.cbuf]).
template <int MODE>
__device__ __attribute__((always_inline)) inline ChOutcome ch_resolve(ChainShared& sh, const ChState& s, double P,
                                                                     double R, const XScale& xs, const ReqArgs& a,
                                                                     const TbRuns& runs, uint32_t* eflags,
                                                                     uint32_t& iters, uint32_t* dbg) {
    const uint32_t lane = threadIdx.x & 63;
#ifdef RL_STAMPS
    const uint64_t t_in = __builtin_amdgcn_s_memtime();
    const uint32_t it_in = iters;
#endif
    const uint32_t cb = s.cbuf;
    const uint32_t nt = (s.ccnt + CH_TILE - 1) / CH_TILE;
    const double LO = MODE == QM_DEC ? (double)DEC_LO : (double)BIN_LO;
    const double HI = MODE == QM_DEC ? (double)DEC_HI : (double)BIN_HI;
    // one lane per tile: lane t < nt holds tile t; tile prefix sums and the
    // near-list prefix (tiles before the first overflowing list) by wave scans
    const bool tv = lane < nt;
    const uint32_t tl = tv ? lane : 0u;
    const ChTile T = sh.tile[cb][tl];
    const uint32_t ovt = min(first_lane(__ballot(tv && T.nc > (uint32_t)CH_NE)), nt);
    const int64_t Sl = tv ? T.S : 0;
    const int64_t TS_t = wave_incl_scan_i64(Sl) - Sl;                 // nominal sum before tile t
    const uint32_t ncl = (tv && lane < ovt) ? T.nc : 0u;
    const uint32_t np1 = wave_scan_u32(ncl, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const uint32_t np0 = np1 - ncl;                                   // near entries before tile t
    const uint32_t ne = (uint32_t)__builtin_amdgcn_readlane((int)np1, 63);
    uint32_t NPF[CH_NP];                                              // wave-uniform copies
#pragma unroll
    for (int u = 0; u < CH_NP; u++) NPF[u] = (uint32_t)__builtin_amdgcn_readlane((int)np0, u);
    const int64_t tbase_i = s.D + TS_t;                               // nominal start of tile t
    const double tbase = (double)tbase_i;                              // (exact in the one-decade modes)
    uint32_t moff = 0;                                                 // XDEC: max |resolved offset|
#ifdef RL_STAMPS
    if (dbg && lane == 0 && s.hot) atomicAdd(&dbg[39], (uint32_t)((__builtin_amdgcn_s_memtime() - t_in) >> 4));
#endif

    // Near steps in sequence order, 64 at a time.  A step's exact result
    // depends on its exact predecessor = nominal + (offset before it); far
    // steps keep the offset, so the offset before step g is the flips (exact
    // result - nominal result) of the earlier near steps.  Wave fixed point:
    // evaluate every step at the current guess, scan the flips, re-guess; when
    // no guess changes before the first step that leaves the regime, the
    // guesses are the true offsets (induction over lanes).
    uint32_t nstop = NO_STOP;
    if constexpr (MODE == QM_XDEC) {
        // The same fixed point on the window's integer states: a guess is the
        // offset (exact - nominal) before the step; an add step reports its
        // flip (exact result - (guessed predecessor + r)), a reset step (a
        // decade up: its result forgets small errors of its predecessor) the
        // offset after it, and a segmented scan turns both into the offset
        // after every step.  No allow / clamp test here (th is not kept):
        // a tile where one is possible never commits (ymin below), and its
        // exact replay finds it.
        constexpr int ITMAX = 16;
        int32_t cbo = 0;
        const uint32_t it_x0 = iters;
        for (uint32_t b = 0; b < ne; b += 64) {
            const uint32_t g = b + lane;
            const bool v = g < ne;
            uint32_t t = 0, base = NPF[0];
#pragma unroll
            for (int u = 1; u < CH_NP; u++) {
                const bool ge = g >= NPF[u];
                t += ge ? 1u : 0u;
                base = ge ? NPF[u] : base;
            }
            const uint32_t k = v ? g - base : 0u;
            const int64_t pn = __shfl(tbase_i, (int)t, 64) + __double_as_longlong(sh.ne_pred[cb][t][k]);
            const double ad = sh.ne_add[cb][t][k];
            const int64_t r = __double_as_longlong(sh.ne_th[cb][t][k]);
            const bool rs = v && ((sh.ne_kind[cb][t] >> k) & 1ull);
            int32_t est = cbo, outv = cbo;
            uint32_t stop_lane = 64;
            for (int it = 0;; it++) {
                const int64_t pred = pn + est;
                int64_t Xn = pred, Xin;
                double tk;
                bool up;
                const bool ok = xstep(pred, xs, ad, __builtin_inf(), Xn, tk, up, Xin);
                // flips from the state the step started from (the guess
                // rounded onto a state), as in the one-decade modes
                const int64_t d64 = rs ? Xn - (pn + r) : Xn - (Xin + r);
                const bool brk = v && (!ok || d64 > 0x3fffffffLL || d64 < -0x3fffffffLL);
                const bool fl = rs && !brk;
                const int64_t incl = seg_incl_scan_i64(fl, (v && !brk) ? d64 : 0, (int64_t)cbo);
                outv = (int32_t)incl;
                const int32_t en = wave_prev_i32(outv, cbo);    // the guess: the offset after the lane before
                iters++;
                if (it + 1 < CH_UNCHECKED) {
                    est = en;
                    continue;
                }
                const uint32_t fb = first_lane(__ballot(brk));
                const uint32_t fc = first_lane(__ballot(v && en != est));
                if (fc >= fb) { stop_lane = fb; break; }
                if (it + 1 == ITMAX) {
                    stop_lane = fc;
                    if (dbg && lane == 0) atomicAdd(&dbg[69], 1u);   // XDEC groups stopped unconverged
                    break;
                }
                est = en;
            }
            const bool keep = v && lane < stop_lane;
            if (keep) sh.ne_off[g] = outv;
            const uint32_t ao = keep ? (uint32_t)(outv < 0 ? -outv : outv) : 0u;
            moff = max(moff, (uint32_t)__builtin_amdgcn_readlane(
                                 (int)wave_scan_u32(ao, 0u, [](uint32_t x, uint32_t y) { return x > y ? x : y; }), 63));
            if (stop_lane < 64) {
                nstop = b + stop_lane;
                break;
            }
            cbo = __builtin_amdgcn_readlane(outv, 63);
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // ne_off visible to this wave
        if (dbg && lane == 0) {   // dbg[62]: XDEC near passes, [68] near entries
            atomicAdd(&dbg[62], iters - it_x0);
            atomicAdd(&dbg[68], ne);
        }
    } else {
        constexpr int ITMAX = 16;
        int32_t cbo = 0;
        for (uint32_t b = 0; b < ne; b += 64) {
            const uint32_t g = b + lane;
            const bool v = g < ne;
            // the tile t holding near entry g and its first near index NPF[t]
            // (NPF is non-decreasing; selects on wave-uniform values: indexing
            // NPF by a lane-varying t made the compiler spill it to scratch)
            uint32_t t = 0, base = NPF[0];
#pragma unroll
            for (int u = 1; u < CH_NP; u++) {
                const bool ge = g >= NPF[u];
                t += ge ? 1u : 0u;
                base = ge ? NPF[u] : base;
            }
            const uint32_t k = v ? g - base : 0u;
            const double pn = __shfl(tbase, (int)t) + sh.ne_pred[cb][t][k];
            const double ad = sh.ne_add[cb][t][k];
            const double th = sh.ne_th[cb][t][k];
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
                iters++;
                // the first CH_UNCHECKED passes skip the convergence test (two
                // ballots, their scalar first-lane searches and a branch: about
                // half of a pass's latency): a pass past the fixed point
                // changes nothing, and most groups need several passes
                if (it + 1 < CH_UNCHECKED) {
                    est = en;
                    continue;
                }
                const uint32_t fb = first_lane(__ballot(brk));
                const uint32_t fc = first_lane(__ballot(v && en != est));
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
    const uint32_t nres = nstop < ne ? nstop : ne;      // ne_off[0, nres) are exact
#ifdef RL_STAMPS
    if (dbg && lane == 0 && s.hot) {
        atomicAdd(&dbg[36], (uint32_t)((__builtin_amdgcn_s_memtime() - t_in) >> 4));
        atomicAdd(&dbg[37], ne);
        atomicAdd(&dbg[38], iters - it_in);
        // [80]: the multi-decade windows' share of [36]
        if (MODE == QM_XDEC) atomicAdd(&dbg[80], (uint32_t)((__builtin_amdgcn_s_memtime() - t_in) >> 4));
    }
#endif

    // Tile checks, one lane per tile: a tile whose bounds exclude a regime
    // exit is committed as a run; the first other one is replayed exactly.
    const uint32_t i0 = np0 < nres ? np0 : nres, i1 = np1 < nres ? np1 : nres;
    const int32_t off_in = i0 ? sh.ne_off[i0 - 1] : 0;
    const int32_t off_out = i1 ? sh.ne_off[i1 - 1] : 0;
    const bool forced = tl >= ovt || (nstop != NO_STOP && nstop < np1) || T.ev != NO_STOP;
    const int64_t Dt = s.D + TS_t + off_in;
    const int64_t D1 = Dt + T.S + (off_out - off_in);
    {
        const double dD = (double)Dt, nc = (double)T.nc;
        bool cand;
        if constexpr (MODE == QM_XDEC) {
            // the exact state stays within the producers' classification slack
            // of their estimate V, and below every allow / clamp threshold:
            // |X - V| <= |X_t - V_t| + drift + the tile's offset changes,
            // plus 4096 units for V's own rounding (valid below 2^60, which
            // ch_produce_x enforces: rl_tb_xdec.h)
            const double bound = fabs(dD - T.cmax) + T.cmin + 2.0 * (double)moff + 4096.0;
            cand = forced || !(bound < T.dmax) || !(bound + 2.0 < T.ymin);
        } else {
            cand = forced || !(dD + nc + T.cmax < HI) || !(dD - nc + T.cmin >= LO + 1.0) ||
                   !(dD + nc + 3.0 < T.ymin) || !(dD + nc + fmax(T.cmax, 0.0) <= T.dmax);
        }
        const uint64_t candm = __ballot(tv && cand);
        uint32_t lo = 0;                                   // tiles [lo, c) commit now
        uint32_t c = first_lane(candm);
        const uint32_t pos = s.cfirst + tl * CH_TILE;
        const uint32_t len = (s.ccnt - tl * CH_TILE) < CH_TILE ? (s.ccnt - tl * CH_TILE) : CH_TILE;
        for (;;) {
            if (tv && lane >= lo && lane < c) {
                runs.len[pos] = (uint16_t)len;
                runs.E[pos] = (int16_t)(MODE == QM_XDEC ? s.E + XRUN : s.E);
                runs.D0[pos] = Dt;
                runs.D1[pos] = D1;
            }
            if constexpr (MODE == QM_XDEC) {   // listed for k_tb_expand_x
                const uint64_t cm = __ballot(tv && lane >= lo && lane < c);
                if (cm) {
                    uint32_t b0 = 0;
                    if (lane == 0) b0 = atomicAdd(runs.xcnt, (uint32_t)__popcll(cm));
                    b0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)b0);
                    if ((cm >> lane) & 1ull) runs.xlist[b0 + (uint32_t)__popcll(cm & ((1ull << lane) - 1ull))] = pos;
                }
            }
            ChOutcome o;
            if (c >= nt) {
                o.kind = CH_FULL;
                o.q = s.cfirst + s.ccnt;
                o.D = readlane_i64(D1, nt - 1);
                return o;
            }
            // exact replay of tile c from its exact start; lane guesses from
            // the resolved near offsets
            const uint32_t cpos = s.cfirst + c * CH_TILE;
            const uint32_t clen = (s.ccnt - c * CH_TILE) < CH_TILE ? (s.ccnt - c * CH_TILE) : CH_TILE;
            const int64_t Dc = readlane_i64(Dt, c);
            const uint32_t cn0 = (uint32_t)__builtin_amdgcn_readlane((int)np0, (int)c);
            const int32_t cin = (int32_t)__builtin_amdgcn_readlane(off_in, (int)c);
            int32_t goff = 0;
            if (MODE != QM_XDEC && c < ovt) {
                const uint32_t gi = cn0 + sh.ne_rank[cb][c][lane];
                const uint32_t gc = gi < nres ? gi : nres;
                goff = (gi > cn0 && gc) ? sh.ne_off[gc - 1] - cin : 0;
            }
            (void)cin;
            int64_t Dq = 0;
#ifdef RL_STAMPS
            const uint64_t t_ex = __builtin_amdgcn_s_memtime();
            const uint32_t it_ex = iters;
#endif
            uint32_t brk;
            if constexpr (MODE == QM_XDEC) {
                const uint32_t it_e = iters;
                brk = exact_span_x<false>(RingSrc{sh}, cpos, clen, Dc, xs, Dq, a, iters);
                if (dbg && lane == 0) atomicAdd(&dbg[67], iters - it_e);   // XDEC exact-tile passes
            }
            else brk = exact_span<MODE, false>(RingSrc{sh}, cpos, clen, Dc, goff, P, R, Dq, a, iters);
#ifdef RL_STAMPS
            if (dbg && lane == 0 && s.hot) {   // [7] cycles / 16, [11] passes of the hot chain's exact tiles
                atomicAdd(&dbg[7], (uint32_t)((__builtin_amdgcn_s_memtime() - t_ex) >> 4));
                atomicAdd(&dbg[11], iters - it_ex);
                if (MODE == QM_XDEC) atomicAdd(&dbg[81], (uint32_t)((__builtin_amdgcn_s_memtime() - t_ex) >> 4));
            }
#endif
            if (brk > clen) {       // (never) give up on the window: one exact serial step
                if (lane == 0) atomicOr(eflags, EF_INTERNAL);
                brk = 0;
                Dq = Dc;
            }
            if (dbg && lane == 0) atomicAdd(&dbg[MODE == QM_XDEC ? 66 : 20], 1u);
            if (lane == 0 && brk) {
                runs.len[cpos] = (uint16_t)brk;
                runs.E[cpos] = (int16_t)(MODE == QM_XDEC ? s.E + XRUN : s.E);
                runs.D0[cpos] = Dc;
                runs.D1[cpos] = Dq;
                if (MODE == QM_XDEC) runs.xlist[atomicAdd(runs.xcnt, 1u)] = cpos;
            }
            if (brk < clen) {
                o.kind = CH_STOP;
                o.q = cpos + brk;
                o.D = Dq;
                return o;
            }
            const bool agree = Dq == readlane_i64(D1, c);
            const bool fc = __builtin_amdgcn_readlane((int)forced, (int)c) != 0;
            if (fc || !agree) {
                o.kind = c + 1 < nt ? CH_PARTIAL : CH_FULL;
                o.q = cpos + clen;
                o.D = Dq;
                return o;
            }
            lo = c + 1;
            c = first_lane(candm & ~((2ull << c) - 1ull));
        }
    }
}

// One Redis-7 script step in decimal mode on the stored state as doubles:
// digits Dd (an integer-valued double, |Dd| in [1e13, 1e14), or 0) at scale
// P = 10^(13 - E), k = 13 - E in [1, 22].  The common serial step -- the key
// alive, the sum below th (no allow, no clamp) -- with %.14g's decade chosen
// on the exact scaled value (as dec14_fast: a >= 10^E and a < 10^(E+1) tested
// on a*P = p + err exactly; digits RNE, a carry to 1e14 moves up a decade) at
// the same, the next or the one after next decade.  False when the step needs
// the general path (tb_eval): sum >= th, or a decade outside k in [1, 22] or
// more than two away.  Sign-symmetric like %.14g and strtod.  The same
// arithmetic as tb_eval(QM_DEC) + its decade search, in about 25 dependent
// double operations instead of the general path's integer conversions,
// table lookups and branches.
__device__ __attribute__((always_inline)) inline bool tb_dec_step(double& Dd, int32_t& E, double& P, double add,
                                                                 double th, double& tokens) {
    const double T = Dd / P;                     // strtod: one correctly rounded division (Clinger)
    const double sum = T + add;
    if (!(sum < th)) return false;               // allow or clamp: n and the capacity decide
    tokens = sum;
    const double a = sum < 0.0 ? -sum : sum;
    if (a == 0.0) {                              // tostring(0) == "0": T = 0 at any scale
        Dd = 0.0;
        return true;
    }
    double Pn = P;
    int32_t En = E;
#pragma unroll
    for (int g = 0; g < 3; g++) {
        const double p = a * Pn, err = __builtin_fma(a, Pn, -p);    // a*Pn == p + err exactly
        const bool lo_ok = (p > 1e13) | ((p == 1e13) & (err >= 0.0));
        const bool hi_ok = (p < 1e14) | ((p == 1e14) & (err < 0.0));
        if (lo_ok & hi_ok) {
            double d = rint(p);                  // RNE of p; the exact product decides a tie of p
            const double h = p - d;
            d += ((h == 0.5) & (err > 0.0)) ? 1.0 : 0.0;
            d -= ((h == -0.5) & (err < 0.0)) ? 1.0 : 0.0;
            if (d == 1e14) {                     // rounding carried into the next decade
                d = 1e13;
                En += 1;
                Pn = Pn / 10.0;                  // exact: a smaller power of ten
            }
            if (En > 12 || En < -9) return false;
            Dd = sum < 0.0 ? -d : d;
            E = En;
            P = Pn;
            return true;
        }
        if (!lo_ok) {
            En -= 1;
            Pn = Pn * 10.0;
        } else {
            En += 1;
            Pn = Pn / 10.0;
        }
        if (En > 12 || En < -9) return false;    // 13 - E outside [1, 22]
    }
    return false;
}

// Exact serial steps by one wave (every lane computes the same values): from
// the exact stored state (D, E) before position q, the step at q when `force`
// (a step that leaves the regime), then on while the state is off the fast
// decades or the last step left the regime -- at most CH_SERIAL steps and
// never at or past lim.  add_at(p): TbPre::add of p.  Step k's outputs are
// collected in lane k % 64 and stored 64 positions at a time (coalesced),
// not one lane-0 store per step.  Redis 7 steps in decimal mode take
// tb_dec_step; the rest (allows, clamps, expired keys, far decade jumps, the
// binary profile) the general tb_eval.
struct SerialOut {
    uint32_t q;        // next position
    int64_t D;         // exact stored state before it
    int32_t E;
    int32_t mode;
    uint32_t steps;
};

// xd: multi-decade windows are available -- stop after the forced steps
// whenever the state fits one (any state of 1e-9 .. 1e12 tokens, or zero)
__device__ inline bool xdec_fit(int64_t D, int32_t E) { return D == 0 || (E >= XDEC_FMIN && E <= XDEC_FMAX + 4); }

template <typename AddAt, typename ThAt>
__device__ __attribute__((always_inline)) inline SerialOut serial_steps(AddAt add_at, ThAt th_at, uint32_t q, int64_t D, int32_t E,
                                                                       bool force, uint32_t lim, uint32_t j1,
                                                                       const CfgDev* __restrict__ cfgs,
                                                                       int32_t profile, const ReqArgs& a,
                                                                       bool xd = false) {
    const uint32_t lane = threadIdx.x & 63;
    // mode: the callers' fast regime (positive digits only).  emode: how a step
    // is evaluated here -- sign-symmetric, because %.14g / strtod and the
    // binade scaling are: a negative state in a fast decade (the balance a hot
    // key random-walks around zero after an allow, its last_refill rounded to
    // 100 us) steps with the decade arithmetic instead of a full
    // decimal conversion per step
    int32_t mode = fast_mode(D, E, profile);
    int32_t emode = fast_mode(D < 0 ? -D : D, E, profile);
    double Ps = 1.0, Rs = 1.0;
    if (emode != QM_NONE) mode_scale(emode, E, Ps, Rs);
    // the state as a double too (Dd == D while both are live; tb_dec_step
    // updates Dd alone and D follows when the general path needs it)
    double Dd = (double)D;
    bool d_stale = false;
    // add and th = min(capacity, n) of the next 64 positions in one vector load
    // each (lane k holds position q + k; the chain's are in its LDS ring): a
    // step costs its arithmetic, not a dependent memory round trip.  n and the
    // capacity themselves matter only when sum >= th (an allow or a clamp) or
    // the key has expired: below th the step denies without clamping whatever
    // they are, so only those steps load them (from HBM)
    double avec = 0.0, tvec = 0.0;
    double otok = 0.0;
    uint32_t odec = 0;
    uint32_t g0 = q;       // first position of the outputs collected in the lanes
    uint32_t k = 0;
    for (; q < lim && k < (uint32_t)CH_SERIAL && (force || (mode == QM_NONE && !(xd && xdec_fit(xd ? (int64_t)Dd : D, E))));
         k++) {
        const uint32_t kl = k & 63u;
        if (kl == 0) {
            if (k) {   // the previous 64 outputs
                a.tok[g0 + lane] = otok;
                a.dec[g0 + lane] = (uint8_t)odec;
            }
            g0 = q;
            const uint32_t pq = q + lane;
            avec = pq < lim ? add_at(pq) : 0.0;
            tvec = pq < lim ? th_at(pq) : 0.0;
        }
        const double add = __longlong_as_double(readlane_i64(__double_as_longlong(avec), kl));
        const bool alive = add == add;
        const double th = __longlong_as_double(readlane_i64(__double_as_longlong(tvec), kl));
        if (profile == PROFILE_REDIS7 && emode == QM_DEC && alive) {
            double tk;
            if (tb_dec_step(Dd, E, Ps, add, th, tk)) {
                otok = lane == kl ? tk : otok;
                odec = lane == kl ? (uint32_t)DEC_DENIED : odec;
                d_stale = true;
                force = false;
                mode = (Dd >= 1e13) ? QM_DEC : QM_NONE;   // E stays in the fast range
                q++;
                continue;
            }
        }
        if (d_stale) {
            D = (int64_t)Dd;
            d_stale = false;
        }
        TbEval v = tb_eval(emode, D, E, Ps, Rs, alive, alive ? add : 0.0, th, th, profile);
        if (!alive || v.clamped) {      // sum >= th or an expired key: the real n and capacity
            const int64_t nn = a.n[q];
            const double cap = cfgs[a.cfg[q]].limit_d;
            v = tb_eval(emode, D, E, Ps, Rs, alive, alive ? add : 0.0, cap, (double)nn, profile);
        }
        otok = lane == kl ? v.tokens : otok;
        odec = lane == kl ? (uint32_t)(v.allowed ? DEC_ALLOWED : DEC_DENIED) : odec;
        force = !xd && (v.allowed || v.clamped || !alive);
        const bool same = emode != QM_NONE && v.inrange;
        if (same) {
            D = v.Dact;                     // same decade / binade (sign may flip)
        } else {
            // a step out of a fast decade nearly always lands in a neighbouring
            // one: its 14 digits there from one exact scaled rounding (valid in
            // exactly one decade: the exact product >= 1e13 and the rounded
            // digits < 1e14), else the general %.14g decomposition
            bool nb = false;
            if (emode == QM_DEC) {
                const double at = v.tokens < 0.0 ? -v.tokens : v.tokens;
#pragma unroll
                for (int d = -1; d <= 1; d += 2) {
                    const int32_t k2 = 13 - (E + d);
                    if (nb || k2 < 1 || k2 > 22) continue;
                    const double P2 = d < 0 ? Ps * 10.0 : Ps / 10.0;     // exact powers of ten (k2 <= 22)
                    bool ge_lo;
                    const double Dn = round_scaled_Pd(at, P2, ge_lo);
                    if (at > 0.0 && ge_lo && Dn < (double)DEC_HI) {
                        D = v.tokens < 0.0 ? -(int64_t)Dn : (int64_t)Dn;
                        E = E + d;
                        Ps = P2;
                        Rs = 0.0;
                        nb = true;
                    }
                }
            }
            if (!nb) {
                const TbQ nq = tb_quant(v.tokens, profile);
                D = nq.D;
                E = nq.E;
                emode = fast_mode(D < 0 ? -D : D, E, profile);
                if (emode != QM_NONE) mode_scale(emode, E, Ps, Rs);
            }
        }
        Dd = (double)D;
        mode = fast_mode(D, E, profile);
        q++;
    }
    if (d_stale) D = (int64_t)Dd;
    if (k && lane < q - g0) {   // the last (partial) group of outputs
        a.tok[g0 + lane] = otok;
        a.dec[g0 + lane] = (uint8_t)odec;
    }
    return SerialOut{q, D, E, mode, k};
}

// TbPre::{add, th} from HBM, with the segment head's add computed at replay
struct HeadSrc {
    const double* a;
    const double* t;
    uint32_t j0;
    double add0;
    __device__ double add(uint32_t p) const { return p == j0 ? add0 : a[p]; }
    __device__ double th(uint32_t p) const { return t[p]; }
};

// A multi-decade span of a heavy segment's wave, out of line (as the
// chain's multi-decade work): from the exact stored state (D, E) off the fast
// decades, up to CH_TILE requests at p with outputs, in a window whose floor
// sits four decades below an upper bound of the span's states.  Returns the
// requests replayed (the first one that leaves the regime, or len) and the
// exact state before it in (D, E); 0 when no window fits.
struct XSpan {
    uint32_t brk;
    int32_t E;
    int64_t D;
};
__device__ XDEC_FN XSpan wave_span_x(HeadSrc src, uint32_t p, uint32_t len, int64_t D, int32_t E, ReqArgs a) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    XSpan o{0u, E, D};
    double sa = 0.0;
#pragma unroll
    for (int q = 0; q < K; q++) {
        const uint32_t i = lane * K + q;
        const double ad = i < len ? src.add(p + i) : 0.0;
        sa += fabs(ad) < 1e300 ? fabs(ad) : 0.0;
    }
    const double x0 = st_value(D, E, QM_NONE);
    const double mx = fabs(x0) + wave_reduce_f64(sa, 0.0, [](double x, double y) { return x + y; });
    if (!(mx < 1e12)) return o;
    const int Et = mx > 0.0 ? (int)floor(log10(mx)) : XDEC_FMIN + 4;
    const int F = max(Et - 4, XDEC_FMIN);
    if (F > XDEC_FMAX) return o;
    int64_t X0;
    if (!dec_to_win(D, E, QM_XDEC, F, X0)) return o;
    const XScale xs = xscale(F);
    int64_t Xe = X0;
    uint32_t iters = 0;
    const uint32_t brk = exact_span_x<true>(src, p, len, X0, xs, Xe, a, iters);
    if (brk > len) return o;   // (never) no convergence: the serial steps take over
    x_to_dec(Xe, F, o.D, o.E);
    o.brk = brk;
    return o;
}

// Replay one heavy (not huge) token-bucket segment [j0, j1) with ONE wave:
// exact_span over CH_TILE requests at a time, writing every result, and exact
// serial steps wherever a step leaves the regime.  No producers, no runs:
// for a few thousand requests this beats a block-wide chain round.
__device__ __attribute__((always_inline)) inline void wave_segment(TbEntry* e, uint32_t j0, uint32_t j1,
                                                                  const CfgDev* __restrict__ cfgs, int32_t profile,
                                                                  const ReqArgs& a, const TbPre& pre,
                                                                  uint32_t* eflags, uint32_t& iters) {
    const TbQ q0 = tb_quant(e->tok, profile);
    const HeadSrc src{pre.add, pre.th, j0, tb_head_add(e, j0, cfgs, profile, a)};
    int64_t D = q0.D;
    int32_t E = q0.E;
    int32_t mode = fast_mode(D, E, profile);
    uint32_t pos = j0;
    const bool xd = CH_XDEC && profile == PROFILE_REDIS7;
    bool exited = false;       // the last span stopped at a step that leaves the regime: a serial step next
    for (uint32_t guard = 0; pos < j1; guard++) {
        if (guard > 2u * (j1 - j0) + 8u) {        // each pass advances pos; never hang on it
            if ((threadIdx.x & 63) == 0) atomicOr(eflags, EF_INTERNAL | 0x100u);
            return;
        }
        if (mode != QM_NONE) {
            double P, R;
            mode_scale(mode, E, P, R);
            const uint32_t len = (j1 - pos) < CH_TILE ? (j1 - pos) : CH_TILE;
            int64_t Dq = D;
            const uint32_t brk = mode == QM_DEC ? exact_span<QM_DEC, true>(src, pos, len, D, 0, P, R, Dq, a, iters)
                                                : exact_span<QM_BIN, true>(src, pos, len, D, 0, P, R, Dq, a, iters);
            if (brk > len) {
                if ((threadIdx.x & 63) == 0) atomicOr(eflags, EF_INTERNAL | 0x200u);
                return;
            }
            D = readfirstlane_i64(Dq);
            pos += (uint32_t)__builtin_amdgcn_readfirstlane((int)brk);
            if (brk == len) continue;
        } else if (xd && !exited && xdec_fit(D, E)) {
            // off the fast decades (after an allow the balance random-walks
            // across zero and decades): a multi-decade span, not serial steps
            const uint32_t len = (j1 - pos) < CH_TILE ? (j1 - pos) : CH_TILE;
            const XSpan xo = wave_span_x(src, pos, len, D, E, a);
            const uint32_t brk = (uint32_t)__builtin_amdgcn_readfirstlane((int)xo.brk);
            if (brk) {
                D = readfirstlane_i64(xo.D);
                E = __builtin_amdgcn_readfirstlane(xo.E);
                mode = fast_mode(D, E, profile);
                pos += brk;
                exited = brk < len;
                continue;
            }
        }
        exited = false;
        const SerialOut so = serial_steps([&](uint32_t p) { return src.add(p); }, [&](uint32_t p) { return src.th(p); },
                                          pos, D, E, true, j1, j1, cfgs,
                                          profile, a, xd);
        // wave-uniform by construction; say so (the loop and its ballots stay uniform)
        pos = (uint32_t)__builtin_amdgcn_readfirstlane((int)so.q);
        D = readfirstlane_i64(so.D);
        E = __builtin_amdgcn_readfirstlane(so.E);
        mode = __builtin_amdgcn_readfirstlane(so.mode);
    }
    if ((threadIdx.x & 63) == 0) tb_store_end(e, tb_value(D, E, profile), j1 - 1, cfgs, profile, a);
}

// Replay one heavy fixed / sliding window segment [j0, j1) with ONE wave.
// Within a window run (consecutive requests of one window start ws) the
// reference's state transition is a prefix sum: INCRBY adds n to the current
// window key, whose TTL is set once at creation; SW's previous-window count is
// constant and its key's TTL is refreshed by every request
// (fixedwindow.go:21-27, slidingwindow.go:22-30).  So per run: the first
// request runs exactly (fw_step / sw_step on the exact state: key lookup,
// expiry, slot allocation), the rest are computed in parallel from a prefix
// sum of n and checked request by request against every assumption of that
// shortcut -- the current key alive, no INCRBY overflow, no TTL reset,
// the previous key's refresh chain.  A failed check (or a config change, a
// key in the spill, sub-second windows) continues serially from the first
// request not yet applied, on the exact state reached so far: the first
// request of a run has side effects on the spill table, so nothing is ever
// replayed twice.
__device__ __attribute__((always_inline)) inline void wave_win_segment(WinEntry* e, const Spill& S, uint32_t j0,
                                                                      uint32_t j1, const CfgDev* __restrict__ cfgs,
                                                                      int32_t profile, const ReqArgs& a,
                                                                      uint32_t* eflags) {
    constexpr int K = CH_K;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c0 = a.cfg[j0];
    const CfgDev& C = cfgs[c0];
    const bool sw = C.alg == ALG_SLIDING_WINDOW;
    WinState w = win_load(e);
    uint32_t ef = 0;
    bool ok = C.ttl_c > 0;
    uint32_t pos = j0;
    while (ok && pos < j1) {
        // first request of the run: exact
        const Req r0 = load_req(a, pos);
        if (r0.c != c0) { ok = false; break; }   // serial from pos
        const Out o0 = sw ? sw_step(w, S, r0.t, r0.n, r0.sms, C, profile, ef)
                          : fw_step(w, S, r0.t, r0.n, r0.sms, C, profile, ef);
        if (lane == 0) write_out(a, pos, o0);
        const int64_t wsn = window_start_ns(r0.t, C);
        const int64_t ws = floor_div(wsn, NS_PER_S), pws = ws - C.ttl_c;
        int ck = -1, pk = -1;
        for (int k = 0; k < 2; k++) {
            if (w.s[k].when == ABSENT) continue;
            if (w.s[k].ws == ws) ck = k;
            else if (sw && w.s[k].ws == pws) pk = k;
        }
        pos++;   // r0 is applied
        if (o0.decision == DEC_ERROR || ck < 0) { ok = false; break; }
        // the run's shortcut keeps the previous window's key in the entry; one
        // in the spill (per-key time went back) takes the serial path
        if (sw && pk < 0 && spill_lookup(S, w.key, w.nspill, pws)) { ok = false; break; }
        const int64_t when_c = w.s[ck].when;
        const int64_t cnt_p = pk >= 0 ? w.s[pk].cnt : 0;
        int64_t c_run = w.s[ck].cnt, sms_prev = r0.sms;
        bool p_alive = pk >= 0;
        bool run_end = false;
        while (ok && !run_end && pos < j1) {
            // K requests per lane; the run ends at the first other window / config
            const uint32_t off = lane * K;
            int64_t t[K], n[K], sm[K];
            bool same[K];
            uint32_t firstx = NO_STOP;
#pragma unroll
            for (int q = 0; q < K; q++) {
                const uint32_t j = pos + off + q;
                const bool v = j < j1;
                t[q] = v ? a.ts[j] : 0;
                n[q] = v ? a.n[j] : 0;
                sm[q] = v ? req_server_ms(a, j, t[q]) : 0;
                // window_start(t) == ws without two 64-bit divisions: W >= 1 s
                // here (ttl_c > 0), so windows whose starts differ also differ
                // in the key's second, and t is in r0's window iff it lies in
                // [wsn, wsn + W)
                same[q] = v && a.cfg[j] == c0 && t[q] >= wsn && t[q] - wsn < C.window;
                if (v && !same[q] && firstx == NO_STOP) firstx = off + q;
            }
            const uint32_t cend = wave_min_u32(firstx);            // run end in this chunk (relative)
            const uint32_t lim = min(min(cend, j1 - pos), (uint32_t)(64 * K));
            run_end = cend != NO_STOP;
            if (lim == 0) break;   // the run was r0 alone: nothing to carry
            // prefix sum of n (int64) inside the run, per-request checks
            int64_t ls = 0;
#pragma unroll
            for (int q = 0; q < K; q++)
                if (off + q < lim) ls += n[q];
            const int64_t li = wave_incl_scan_i64(ls);
            int64_t c = c_run + li - ls;                            // count before my first request
            int64_t sp = __shfl_up(sm[K - 1], 1);                   // server clock of my predecessor
            if (lane == 0) sp = sms_prev;
            bool bad = false, pdead = false;
            uint32_t pdead_at = NO_STOP;
#pragma unroll
            for (int q = 0; q < K; q++) {
                if (off + q >= lim) continue;
                bad |= incr_overflows(c, n[q]);
                const int64_t cur = c + n[q];
                bad |= (double)cur == (double)n[q];                 // would (re)set the TTL
                bad |= !key_alive(when_c, sm[q], profile);          // current key expired mid-run
                if (sw && !pdead && !key_alive(expire_when(C.ttl_p, sp), sm[q], profile)) {
                    pdead = true;
                    pdead_at = off + q;
                }
                sp = sm[q];
                c = cur;
            }
            if (__ballot(bad)) { ok = false; break; }   // serial from pos (this chunk)
            const uint32_t pd = wave_min_u32(pdead_at);             // first request that finds prev dead
            // outputs
            c = c_run + li - ls;
#pragma unroll
            for (int q = 0; q < K; q++) {
                if (off + q >= lim) continue;
                const int64_t cur = c + n[q];
                c = cur;
                Out o;
                o.tokens = 0.0;
                o.reset_at = wadd(wmul(ws, NS_PER_S), C.window);
                int64_t count;
                bool allowed;
                if (sw) {
                    const int64_t p = (p_alive && off + q < pd) ? go_f2i((double)cnt_p) : 0;
                    const int64_t cc = go_f2i((double)cur);
                    const int64_t elapsed = wsub(t[q], wmul(ws, NS_PER_S));
                    const double progress = (double)elapsed / (double)C.window;
                    double weighted = (double)p * (1.0 - progress);
                    weighted = weighted + (double)cc;
                    allowed = weighted <= C.limit_d;
                    count = go_f2i(weighted);
                } else {
                    count = go_f2i((double)cur);
                    allowed = count <= C.limit;
                }
                const int64_t rem = wsub(C.limit, count);
                o.remaining = rem < 0 ? 0 : rem;
                o.decision = allowed ? DEC_ALLOWED : DEC_DENIED;
                o.retry = allowed ? 0 : until_reset(o.reset_at, t[q]);
                write_out(a, pos + off + q, o);
            }
            // carry to the next chunk
            const uint32_t lastl = (lim - 1) / K, lastq = (lim - 1) % K;
            int64_t smv = sm[0];
#pragma unroll
            for (int q = 1; q < K; q++) smv = (uint32_t)q == lastq ? sm[q] : smv;
            sms_prev = readlane_i64(smv, lastl);
            c_run = readlane_i64(c, lastl);
            if (pd != NO_STOP) p_alive = false;
            pos += lim;
        }
        // the state after the run's applied requests
        w.s[ck].cnt = c_run;
        if (pk >= 0) w.s[pk].when = p_alive ? expire_when(C.ttl_p, sms_prev) : ABSENT;
    }
    if (lane == 0) {
        if (!ok) replay_win_steps(w, S, pos, j1, cfgs, profile, a, ef);
        win_store(e, w);
        if (ef) atomicOr(eflags, ef);
    }
}

// the chain's exact state (D, E, mode: its window's representation, or
// stored digits for QM_DEC / QM_NONE) into the representation of window w;
// false when it does not fit (then the state is left as it was)
__device__ inline bool st_convert(ChState& s, const ChWin& w, int32_t profile) {
    if (w.mode == QM_NONE) return false;
    if (w.mode == s.mode && w.E == s.E) return true;
    if (profile != PROFILE_REDIS7 || s.mode == QM_BIN || w.mode == QM_BIN) return false;
    int64_t Dd = s.D;
    int32_t Ed = s.E;
    if (s.mode == QM_XDEC) x_to_dec(s.D, s.E, Dd, Ed);
    int64_t out;
    if (!dec_to_win(Dd, Ed, w.mode, w.E, out)) return false;
    s.D = out;
    s.E = w.E;
    s.mode = w.mode;
    return true;
}

// The multi-decade windows' work out of line (ch_resolve_x, ch_plan_w,
// ch_produce_xw): it is the rarer path, and inlined into the chain kernel its
// registers crowded the one-decade path's -- the 9-wave block (168 VGPRs)
// spilled VGPRs into scratch inside the chain's loops, and an 8-wave block
// cost the heavy / light phases 15 % on FW uniform (profiles/r5_xdec_ab.txt).
// Called with the LDS state as an address-space-3 pointer, so their LDS
// accesses stay ds_* instructions; everything else by value.
typedef ChainShared __attribute__((address_space(3))) ChainLds;

__device__ XDEC_FN ChOutcome ch_resolve_x(ChainLds* shp, ChState s, XScale xs, ReqArgs a,
                                                          TbRuns runs, uint32_t* eflags, uint32_t iters,
                                                          uint32_t* dbg) {
    ChainShared& sh = *(ChainShared*)shp;
    ChOutcome o = ch_resolve<QM_XDEC>(sh, s, xs.P[0], 0.0, xs, a, runs, eflags, iters, dbg);
    o.iters = iters;
    return o;
}

#ifdef RL_PLAN_INLINE   // A/B: the plan inlined into the producers' round (no call)
#define PLAN_FN __attribute__((always_inline)) inline
#else
#define PLAN_FN XDEC_FN
#endif
struct XPlanW {
    int32_t mode;
    int32_t E;
    double vt;        // the calling producer's tile start estimate
};
__device__ PLAN_FN XPlanW ch_plan_w(ChainLds* shp, uint32_t first, uint32_t cnt, double v0,
                                                    uint32_t pw, uint32_t seq) {
    ChainShared& sh = *(ChainShared*)shp;
#ifdef RL_PLAN_SEQ   // A/B: every producer wave sums the whole window
    (void)seq;
    const XPlan pl = ch_plan(sh, first, cnt, v0);
#else
    const XPlan pl = ch_plan_par(sh, first, cnt, v0, pw, seq);
#endif
    return XPlanW{pl.mode, pl.E, pick(pl.vt, pw)};
}
__device__ XDEC_FN void ch_produce_xw(ChainLds* shp, uint32_t buf, uint32_t t, uint32_t pfirst,
                                                       uint32_t pcnt, int32_t F, double vt) {
    ChainShared& sh = *(ChainShared*)shp;
    const XScale xs = xscale(F);
    ch_produce_x(sh, buf, t, pfirst, pcnt, xs, vt);
}

// Replay one huge token-bucket segment [j0, j1) with the whole block.
template <bool LCFG>
__device__ __attribute__((always_inline)) inline void ch_segment(ChainShared& sh, TbEntry* e, uint32_t j0, uint32_t j1,
                                                                const CfgDev* __restrict__ cfgs, int32_t profile,
                                                                const ReqArgs& a, const TbPre& pre, uint32_t* eflags,
                                                                uint32_t* dbg, const TbRuns& runs, uint32_t& plan_seq) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t nrounds = 0, iters = 0, par = 0, nserial = 0;
    uint64_t cyc[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0;
#ifdef RL_STAMPS
    // dbg[70..79] (producer 0 / chain wave, segments >= 65536): producer cycles
    // of one-decade / multi-decade windows and their counts, chain resolve
    // cycles of one-decade / multi-decade windows and their counts
    uint64_t cx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t cplan = 0;   // producer 0: plan cycles (dbg[48])
    uint64_t cpcall = 0;  // of which in ch_plan_w calls (dbg[50]), npcall of them (dbg[49])
    uint32_t npcall = 0;
#endif
    (void)t0; (void)t1;
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
        s0.hot = j1 - j0 >= 65536u;
        sh.st[0] = s0;
        sh.spec[0].valid = 0u;
    }
    if (wave == (uint32_t)CH_LOADER) {
        ld_until(L, sh, j0, j0 + 2 * CH_W, j1, pre, lane);
        // the head's add comes from the table entry: into the ring and HBM
        // (k_tb_expand reads it there)
        if (lane == 0) {
            const double add0 = tb_head_add(e, j0, cfgs, profile, a);
            pre.add[j0] = add0;
            reinterpret_cast<double*>(&sh.r_add[ring_slot(j0 >> 1)])[j0 & 1u] = add0;
        }
    }
#ifdef RL_STAMPS
    if (tid < 2) sh.wk[tid] = 0;
    // pipeline model (chain wave, lane 0; cycles / 16): the finish times of the
    // producers' and the chain's work per round with two summary buffers (the
    // barrier schedule) and with three (producers one window further ahead)
    // (a wave's round work is measured from the previous barrier's exit, so
    // the round-top code every wave runs is in it)
    uint64_t gP = 0, gC = 0, fP = 0, fC = 0, fC2 = 0, bsum = 0, csum = 0, psum = 0, tr0 = 0, ttop = 0;
#endif
    lds_barrier();
#ifdef RL_STAMPS
    CH_T(tr0);
#endif
    const bool xd = CH_XDEC && profile == PROFILE_REDIS7;
    for (;;) {
        ChState s = sh.st[par];
        // A window is resolved in the representation the producers summarized
        // it in (sh.win): the chain's exact state at the window's start is
        // converted into it.  nofit: it did not fit -- at least one exact
        // serial step this round (progress whatever the plans say).
        bool nofit = false;
        {
            const ChSpec sp = sh.spec[par];
            if (sp.valid) {
                ChState t = s;
                if (s.ccnt == 0 && s.pfirst == sp.first &&
                    (xd ? st_convert(t, sh.win[sp.buf], profile) : (s.mode == QM_DEC && s.E == sp.E))) {
                    // the chain's exit ended where the producers guessed: their
                    // window is the next chain window
                    s.D = t.D;
                    s.E = t.E;
                    s.mode = t.mode;
                    s.cfirst = sp.first;
                    s.ccnt = sp.cnt;
                    s.cbuf = sp.buf;
                    s.pbuf = sp.buf ^ 1u;
                    s.pfirst = sp.first + sp.cnt;
                    if (dbg && threadIdx.x == 0) atomicAdd(&dbg[22], 1u);
                } else {
                    // the chain went elsewhere: tile[s.cbuf] does not hold its
                    // next window (the state is exact at s.cfirst / s.pfirst)
                    if (s.ccnt > 0) {
                        s.pfirst = s.cfirst;
                        s.ccnt = 0;
                    }
                    if (dbg && threadIdx.x == 0) {
                        atomicAdd(&dbg[23], 1u);
                        // why: the chain's exit ended [9] 1 or [10] 2-64 steps after
                        // the guess, [15] anything else
                        const uint32_t dd = s.pfirst - sp.first;
                        atomicAdd(&dbg[s.ccnt > 0 || s.pfirst <= sp.first || dd > 64u ? 15 : dd == 1u ? 9 : 10], 1u);
                    }
                }
            } else if (xd && s.ccnt > 0 && !st_convert(s, sh.win[s.cbuf], profile)) {
                s.pfirst = s.cfirst;
                s.ccnt = 0;
                nofit = true;
            }
        }
        if (s.ccnt == 0 && s.pfirst >= j1) break;                 // block-uniform
        const bool fits = s.mode != QM_NONE || (xd && xdec_fit(s.D, s.E));
        const uint32_t pcnt = (fits && !nofit && s.pfirst < j1) ? ((j1 - s.pfirst) < CH_W ? (j1 - s.pfirst) : CH_W)
                                                                 : 0u;
        // the scale (the decimal modes' reciprocal only where the chain
        // resolves a window: a division on every wave's round is ~1 % of the
        // producers' round)
        double P = 1.0, R = 1.0;
        if (s.mode == QM_BIN) mode_scale(s.mode, s.E, P, R);
        else if (s.mode != QM_NONE) P = rlq::pow10_exact(13 - s.E);
        nrounds++;
        CH_T(t0);
#ifdef RL_STAMPS
        ttop += t0 - tr0;   // the round top: from the barrier's exit to here
#endif
        if (ch_producer_index(wave) >= 0) {
            const uint32_t pw = (uint32_t)ch_producer_index(wave);
            ChSpec sp{0u, 0u, 0u, 0u, 0, 0.0};
            if (s.ccnt > 0 && s.mode == QM_DEC) sp = ch_predict(sh, s, P, R, j1, xd);
#ifdef RL_STAMPS
            CH_T(t1);
            cyc[1] += t1 - t0;          // producers: the exit guess
            cyc[2] += sp.valid;         // producers: windows guessed
#endif
            // the window to summarize and its representation
            ChainLds* const shl = (ChainLds*)&sh;
            XPlanW pl;
            pl.mode = QM_NONE;
            pl.E = 0;
            pl.vt = 0.0;
            uint32_t wf = 0, wc = 0;
            double dmax = (double)DEC_HI;
            if (sp.valid) {
                if (xd) {
#ifdef RL_STAMPS
                    uint64_t tq0, tq1;
                    CH_T(tq0);
#endif
                    pl = ch_plan_w(shl, sp.first, sp.cnt, sp.v0, pw, ++plan_seq);
#ifdef RL_STAMPS
                    CH_T(tq1);
                    cpcall += tq1 - tq0;
                    npcall++;
#endif
                    if (pl.mode == QM_NONE) sp.valid = 0u;
                } else {
                    pl.mode = QM_DEC;
                    pl.E = sp.E;
                }
                wf = sp.first;
                wc = sp.cnt;
            }
            if (!sp.valid && pcnt) {
                wf = s.pfirst;
                wc = pcnt;
                if (s.mode == QM_DEC || s.mode == QM_BIN) {
                    pl.mode = s.mode;
                    pl.E = s.E;
                    if (s.mode == QM_DEC && s.ccnt == CH_W) {
                        // bound on the window's states (the chain verifies it per
                        // tile): from the chain window's base, its nominal growth G
                        // plus the larger of 1.25 G and 1.5 x its peak above its
                        // start.  Round 4 took 2.25 G alone: one hot key's states
                        // climb ~4e-3 tokens per window under a +-2e-3 sawtooth of
                        // last_refill's rounding, which broke the bound in ~40 % of
                        // its tiles -- each then replayed exactly
                        double G = 0.0, pk = 0.0;
#pragma unroll
                        for (int t = 0; t < CH_NP; t++) {
                            pk = fmax(pk, G + sh.tile[s.cbuf][t].cmax);
                            G += sh.tile[s.cbuf][t].Sd;   // exact: |G| < 2^53
                        }
                        const double g = G > 0.0 ? G : 0.0;
                        dmax = fmin(dmax, (double)s.D + g + fmax(1.25 * g, 1.5 * pk) + 0x1p21);
                    }
                } else {
                    // after a multi-decade window or from a state off the fast
                    // decades: plan from the state's estimate at the window start
                    int64_t Xe = s.D;
                    if (s.ccnt > 0) {
                        const uint32_t nt = (s.ccnt + CH_TILE - 1) / CH_TILE;
#pragma unroll
                        for (int t = 0; t < CH_NP; t++) Xe += (uint32_t)t < nt ? sh.tile[s.cbuf][t].S : 0;
                    }
#ifdef RL_STAMPS
                    uint64_t tq0, tq1;
                    CH_T(tq0);
#endif
                    pl = ch_plan_w(shl, wf, wc, st_value(Xe, s.E, s.mode), pw, ++plan_seq);
#ifdef RL_STAMPS
                    CH_T(tq1);
                    cpcall += tq1 - tq0;
                    npcall++;
#endif
                }
            }
#ifdef RL_STAMPS
            uint64_t tpl;
            CH_T(tpl);
            cplan += tpl - t1;   // the plan (one-decade bound or multi-decade plan)
#endif
            if (pw == 0 && (threadIdx.x & 63) == 0) {
                sp.buf = s.pbuf;
                sh.spec[par ^ 1u] = sp;
                sh.win[s.pbuf] = ChWin{wc ? pl.mode : (int32_t)QM_NONE, pl.E};
                // dbg[64 / 65]: windows summarized multi-decade / one-decade
                if (dbg && wc) atomicAdd(&dbg[pl.mode == QM_XDEC ? 64 : 65], 1u);
            }
#ifdef RL_STAMPS
            uint64_t tp0;
            CH_T(tp0);
#endif
            if (wc && pl.mode == QM_XDEC) {
                ch_produce_xw(shl, s.pbuf, pw, wf, wc, pl.E, pl.vt);
            } else if (wc && pl.mode == QM_DEC) {
                ch_produce<QM_DEC>(sh, s.pbuf, pw, wf, wc, rlq::pow10_exact(13 - pl.E), dmax);
            } else if (wc && pl.mode == QM_BIN) {
                ch_produce<QM_BIN>(sh, s.pbuf, pw, wf, wc, P, (double)BIN_HI);
            }
            __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            CH_T(t1);
#ifdef RL_STAMPS
            if (wc) {
                const int xk = pl.mode == QM_XDEC ? 1 : 0;
                cx[xk] += t1 - tp0;
                cx[2 + xk] += 1;
            }
#endif
            cyc[0] += t1 - t0;
        } else if (wave == (uint32_t)CH_LOADER) {
            const uint32_t first = s.ccnt ? s.cfirst : s.pfirst;
            ld_until(L, sh, first, s.pfirst + 2 * CH_W, j1, pre, lane);
            CH_T(t1);
            cyc[0] += t1 - t0;
        } else {
            // ---- chain wave ----
            ChState nx;
            nx.hot = s.hot;
            nx.pbuf = s.pbuf ^ 1u;
            nx.cbuf = s.pbuf;
            ChOutcome o{CH_PARTIAL, s.pfirst, s.D};
            bool restart = true, force = nofit;
            if (s.ccnt > 0) {
                if (s.mode == QM_XDEC) {
                    const XScale xs = xscale(s.E);
                    const uint64_t tx0 = __builtin_amdgcn_s_memtime();
                    o = ch_resolve_x((ChainLds*)&sh, s, xs, a, runs, eflags, iters, dbg);
                    iters = o.iters;
                    // dbg[60..]: XDEC windows resolved, of them full, chain passes,
                    // shader cycles / 16 (diagnostics)
                    if (dbg && lane == 0) {
                        atomicAdd(&dbg[60], 1u);
                        atomicAdd(&dbg[61], o.kind == CH_FULL ? 1u : 0u);
                        atomicAdd(&dbg[63], (uint32_t)((__builtin_amdgcn_s_memtime() - tx0) >> 4));
                    }
                } else {
                    XScale xs;
                    xs.F = 0;
                    o = s.mode == QM_DEC ? ch_resolve<QM_DEC>(sh, s, P, 1.0 / P, xs, a, runs, eflags, iters, dbg)
                                         : ch_resolve<QM_BIN>(sh, s, P, R, xs, a, runs, eflags, iters, dbg);
                }
                if (dbg && lane == 0) atomicAdd(&dbg[3 + o.kind], 1u);
                CH_T(t1);
#ifdef RL_STAMPS
                cx[4 + (s.mode == QM_XDEC ? 1 : 0)] += t1 - t0;
                cx[6 + (s.mode == QM_XDEC ? 1 : 0)] += 1;
#endif
                cyc[o.kind == CH_FULL ? 0 : 1] += t1 - t0;
                t0 = t1;
                if (o.kind == CH_FULL) {
                    restart = false;
                    nx.D = o.D;                 // exact at s.pfirst (the window's representation)
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
                // fits no window (off the fast decades, and with multi-decade
                // windows also outside theirs) or the last step left the regime
                const uint32_t lim = (j1 - s.pfirst) < CH_W ? j1 : s.pfirst + CH_W;   // resident in the ring
                int64_t Dd = o.D;
                int32_t Ed = s.E;
                if (s.mode == QM_XDEC) x_to_dec(o.D, s.E, Dd, Ed);
                const SerialOut so = serial_steps([&](uint32_t p) { return ring_add(sh, p); },
                                                  [&](uint32_t p) { return ring_th(sh, p); }, o.q, Dd, Ed, force,
                                                  lim, j1, cfgs, profile, a, xd);
                nserial += so.steps;
                CH_T(t1);
                cyc[2] += t1 - t0;
                t0 = t1;
                nx.D = so.D;
                nx.E = so.E;
                nx.mode = so.mode;
                nx.cfirst = so.q;
                nx.ccnt = 0;
                nx.pfirst = so.q;
            }
            if (lane == 0) sh.st[par ^ 1u] = nx;
        }
        par ^= 1u;
        CH_T(t0);
#ifdef RL_STAMPS
        const uint32_t wr = (uint32_t)((t0 - tr0) >> 4);
        if (ch_producer_index(wave) >= 0 && lane == 0) atomicMax(&sh.wk[par], wr);
#endif
        lds_barrier();
        CH_T(t1);
        cyc[3] += t1 - t0;
#ifdef RL_STAMPS
        tr0 = t1;
        if (wave == 0 && lane == 0) {
            // producers of round r summarize window r, the chain of round r
            // resolves window r - 1; a buffer is free once its window is resolved
            const uint64_t pr = sh.wk[par], cr = wr;
            sh.wk[par] = 0;
            const uint64_t nP2 = max(gP, gC) + pr, nC2 = max(gC, gP) + cr;
            gP = nP2;
            gC = nC2;
            const uint64_t nP3 = max(fP, fC2) + pr, nC3 = max(fC, fP) + cr;
            fC2 = fC;
            fP = nP3;
            fC = nC3;
            bsum += max(pr, cr);
            csum += cr;
            psum += pr;
        }
#endif
    }
#ifdef RL_STAMPS
    // dbg[24 + 4 * role + k]: role 0 chain (full / stop rounds, serial, barrier),
    // 1 producer wave 1 (produce, -, -, barrier), 2 loader (load, -, -, barrier)
    if (lane == 0 && dbg && j1 - j0 >= 65536u) {
        dbg[40 + wave] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));   // HW_ID
        const uint32_t role = wave == 0 ? 0u : wave == 1 ? 1u : wave == (uint32_t)CH_LOADER ? 2u : 3u;
        if (role < 3)
            for (int k = 0; k < 4; k++) atomicAdd(&dbg[24 + 4 * role + k], (uint32_t)(cyc[k] >> 4));
        if (role == 1) {
            for (int k = 0; k < 4; k++) atomicAdd(&dbg[70 + k], (uint32_t)(k < 2 ? cx[k] >> 4 : cx[k]));
            atomicAdd(&dbg[48], (uint32_t)(cplan >> 4));
            atomicAdd(&dbg[49], npcall);
            atomicAdd(&dbg[50], (uint32_t)(cpcall >> 4));
        }
        if (role == 0) {
            for (int k = 4; k < 8; k++) atomicAdd(&dbg[70 + k], (uint32_t)(k < 6 ? cx[k] >> 4 : cx[k]));
            // dbg[82..86]: the pipeline model's two-buffer and three-buffer
            // finish, the sum of the rounds' max(producer, chain) work, and the
            // chain's and the slowest producer's work summed over the rounds
            atomicAdd(&dbg[82], (uint32_t)max(gP, gC));
            atomicAdd(&dbg[83], (uint32_t)max(fP, fC));
            atomicAdd(&dbg[84], (uint32_t)bsum);
            atomicAdd(&dbg[85], (uint32_t)csum);
            atomicAdd(&dbg[86], (uint32_t)psum);
            atomicAdd(&dbg[87], (uint32_t)(ttop >> 4));   // the chain wave's round tops
        }
    }
#endif
    if (tid == 0) {
        const ChState s = sh.st[par];
        int64_t Dd = s.D;
        int32_t Ed = s.E;
        if (s.mode == QM_XDEC) x_to_dec(s.D, s.E, Dd, Ed);
        tb_store_end(e, tb_value(Dd, Ed, profile), j1 - 1, cfgs, profile, a);
        if (dbg) {
            atomicAdd(&dbg[0], nrounds);
            atomicAdd(&dbg[1], iters);
            atomicMax(&dbg[2], nrounds);
            atomicAdd(&dbg[21], nserial);
        }
    }
    (void)eflags;
}

// Outputs of the multi-decade windows' runs (the chain lists them): one wave
// per run, exact_span_x with outputs from the run's exact start, checked
// against the end state the chain resolved.  A kernel of its own: inside
// k_tb_expand its registers halved that kernel's occupancy, which every
// batch's scan of the run starts pays for (mixed: 21 -> 38 us per batch,
// profiles/r5_xdec_ab.txt).
__global__ __launch_bounds__(256) void k_tb_expand_x(TbRuns runs, ReqArgs a, TbPre pre, uint32_t* eflags) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    const uint32_t n = *runs.xcnt;
    uint32_t iters = 0;
    for (uint32_t i = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < n; i += nw) {
        const uint32_t p = runs.xlist[i];
        const uint32_t len = runs.len[p];
        const int32_t F = runs.E[p] - XRUN;
        const int64_t D0 = runs.D0[p], D1 = runs.D1[p];
        const XScale xs = xscale(F);
        int64_t Dend = 0;
        const uint32_t brk = exact_span_x<true>(GlobSrc{pre.add, pre.th}, p, len, D0, xs, Dend, a, iters);
        if (lane == 0) {
            if (brk != len || Dend != D1) atomicOr(eflags, EF_INTERNAL);
            runs.len[p] = 0;
        }
    }
}

// Outputs of the committed runs: one wave per run, exact_span with outputs
// from the run's exact start state, checked against the state the chain
// resolved at the run's end.  Waves scan the batch in CH_TILE-position blocks and
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
            if (profile == PROFILE_REDIS7 && E >= XRUN - 100) {     // a multi-decade window's: k_tb_expand_x
                continue;
            } else if (profile == PROFILE_REDIS7) {
                mode_scale(QM_DEC, E, P, R);
                brk = exact_span<QM_DEC, true>(GlobSrc{pre.add, pre.th}, p, len, D0, 0, P, R, Dend, a, iters);
            } else {
                mode_scale(QM_BIN, E, P, R);
                brk = exact_span<QM_BIN, true>(GlobSrc{pre.add, pre.th}, p, len, D0, 0, P, R, Dend, a, iters);
            }
            if (lane == 0) {
                if (brk != len || Dend != D1) atomicOr(eflags, EF_INTERNAL);
                runs.len[p] = 0;
            }
        }
    }
}

// Phases 2 and 3 of the replay kernels: heavy token-bucket segments
// (wave_segment) and heavy window segments (wave_win_segment), one per wave,
// then light segments of any algorithm, one per thread, serial
// (replay_*_serial).  nhx: huge token-bucket segments taken here as heavy
// ones, ahead of them (k_replay_light; the chain kernel's phase 1 takes them
// otherwise).  s_u: a __shared__ word of the calling kernel.
__device__ __attribute__((always_inline)) inline void replay_rest(const uint32_t* __restrict__ sk, const SegLists& L,
                                                                 uint32_t* qctr, uint32_t win_base, TbEntry* tb,
                                                                 WinEntry* win, const Spill& spill,
                                                                 const CfgDev* __restrict__ cfgs, int32_t profile,
                                                                 const ReqArgs& a, const TbPre& pre, uint32_t* eflags,
                                                                 uint32_t* dbg, uint32_t& s_u, uint32_t nhx) {
    const uint32_t nheavy = L.count[0], nlight = L.count[1], nwin = L.count[2];
    {
        // heavy segments, HEAVY_G per claim: every wave's claim is an atomic on
        // ONE counter, which sustains only ~88 atomics/us -- with one segment
        // per claim, ten thousand short heavy segments (configs[0]'s keys)
        // spent longer queueing on the counter than replaying
        uint32_t iters = 0;
        const uint32_t nhw = nhx + nheavy + nwin;
        for (;;) {
            uint32_t u0 = 0;
            if ((threadIdx.x & 63) == 0) u0 = atomicAdd(&qctr[2], (uint32_t)HEAVY_G);
            u0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)u0);
            if (u0 >= nhw) break;
            const uint32_t u1 = min(u0 + (uint32_t)HEAVY_G, nhw);
            for (uint32_t u = u0; u < u1; u++) {
                if (u < nhx + nheavy) {
                    const SegRec sg = u < nhx ? L.list[3][u] : L.list[0][u - nhx];
#ifdef RL_STAMPS
                    const uint64_t th0 = __builtin_amdgcn_s_memrealtime();
#endif
                    wave_segment(&tb[sk[sg.j0]], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre, eflags, iters);
#ifdef RL_STAMPS
                    // the longest heavy segment's replay (dbg[56], ticks) and its length (dbg[57])
                    if ((threadIdx.x & 63) == 0 && dbg) {
                        const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memrealtime() - th0);
                        if (atomicMax(&dbg[56], dt) < dt) dbg[57] = sg.len;
                    }
#endif
                } else {
                    const SegRec sg = L.list[2][u - nhx - nheavy];
                    wave_win_segment(&win[sk[sg.j0] - win_base], spill, sg.j0, sg.j0 + sg.len, cfgs, profile, a,
                                     eflags);
                }
            }
        }
    }
    __syncthreads();
    const uint64_t t_light = __builtin_amdgcn_s_memrealtime();
#ifdef RL_STAMPS
    // the latest end of a block's heavy phase (dbg[53])
    if (threadIdx.x == 0 && dbg) atomicMax(&dbg[53], (uint32_t)t_light);
#endif
    for (;;) {
        if (threadIdx.x == 0) s_u = atomicAdd(&qctr[1], (uint32_t)blockDim.x);
        __syncthreads();
        const uint32_t u0 = s_u;
        __syncthreads();
        if (u0 >= nlight) break;
#ifdef RL_STAMPS
        // the latest light claim that got work (dbg[54])
        if (threadIdx.x == 0 && dbg) atomicMax(&dbg[54], (uint32_t)__builtin_amdgcn_s_memrealtime());
#endif
        const uint32_t u = u0 + threadIdx.x;
        if (u < nlight) {
            const SegRec sg = L.list[1][u];
            const uint32_t k0 = sk[sg.j0];
            // a key the batch inserted, alone in it: the absent state, unread
#ifdef RL_AB_ALLFRESH   // timing experiment only (wrong results): no table read in the light phase
            const bool fresh = sg.len == 1u;
#else
            const bool fresh = sg.len == 1u && a.fresh && a.fresh[sg.j0];
#endif
            if (k0 < win_base) replay_tb_serial(&tb[k0], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre, fresh);
            else replay_win_serial(&win[k0 - win_base], spill, sg.j0, sg.j0 + sg.len, cfgs, profile, a, eflags, fresh);
        }
    }
    if (threadIdx.x == 0 && dbg) {
        atomicMax(&dbg[12], (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_light));
        atomicMax(&dbg[14], (uint32_t)__builtin_amdgcn_s_memrealtime());
    }
}

// blocks past grid_base join only a batch with a long light phase (many
// distinct keys: every one a serial replay), or with many heavy segments
// (configs[0]'s 10k keys of ~100 requests, one per wave; light_min / 32 =
// m / 128 of them); otherwise they would only take CUs from the next batch's
// grouping, which then bounds the step
__device__ inline bool replay_joins(const SegLists& L, uint32_t grid_base, uint32_t light_min) {
    return blockIdx.x < grid_base || L.count[1] >= light_min || L.count[0] + L.count[2] >= light_min / 32u;
}

// The replay kernel.  Phase 1: huge token-bucket segments, one per block (the
// chain), longest first; then replay_rest.  The hot keys' blocks stay in
// phase 1 while the others drain phases 2-3.  h_huge: a host-mapped word, the
// batch's count of huge segments (the host launches k_replay_light when the
// last replay it saw had none).
template <bool LCFG>
__global__ __launch_bounds__(CH_BLOCK) void k_tb_chain(const uint32_t* __restrict__ sk, SegLists L, uint32_t* qctr,
                                                       uint32_t win_base, TbEntry* tb, WinEntry* win, Spill spill,
                                                       const CfgDev* __restrict__ gcfgs, uint32_t ncfg,
                                                       int32_t profile, ReqArgs a, TbPre pre, uint32_t* eflags,
                                                       uint32_t* dbg, TbRuns runs, uint32_t grid_base,
                                                       uint32_t light_min, uint32_t* h_huge) {
    __shared__ ChainShared sh;
    __shared__ uint32_t s_u;
    __shared__ CfgDev s_cfg[LCFG ? MAX_LCFG : 1];
    if (LCFG) {
        for (uint32_t c = threadIdx.x; c < ncfg; c += blockDim.x) s_cfg[c] = gcfgs[c];
        __syncthreads();
    }
    const CfgDev* cfgs = LCFG ? s_cfg : gcfgs;
    const uint32_t nhuge = L.count[3];
    if (blockIdx.x == 0 && threadIdx.x == 0 && h_huge) *(volatile uint32_t*)h_huge = nhuge;
    if (!replay_joins(L, grid_base, light_min)) return;
    if (threadIdx.x < (uint32_t)CH_NP) sh.plan_tag[threadIdx.x] = 0u;   // (the claim loop's barrier follows)
    uint32_t plan_seq = 0;   // ch_plan_par numbers (the same in every producer wave)
    // timeline (10 ns ticks, low 32 bits): dbg[13] = ~first block start,
    // dbg[14] = last block end, dbg[16/17] = longest segment start / end
    if (threadIdx.x == 0 && dbg) atomicMax(&dbg[13], ~(uint32_t)__builtin_amdgcn_s_memrealtime());
#ifdef RL_STAMPS
    // the replay's tail: the latest block start (dbg[51]; all four are 10-ns
    // realtime ticks, low 32 bits)
    if (threadIdx.x == 0 && dbg) atomicMax(&dbg[51], (uint32_t)__builtin_amdgcn_s_memrealtime());
#endif
    for (;;) {
        // claim the longest unclaimed huge segment (their list is short:
        // batch / 4096 at most), so the hottest key starts with the first
        // block.  The block reads the whole list at once (one entry per
        // thread, an argmax over the waves): one memory round trip, not one
        // per entry before the hot key's chain can start
        if (threadIdx.x == 0) s_u = atomicAdd(&qctr[0], 1u) < nhuge ? 0u : NO_STOP;
        __syncthreads();
        if (s_u == 0u) {
            __shared__ uint64_t s_best[CH_BLOCK / 64];
            for (;;) {
                uint64_t best = 0;   // (len << 32) | (~k): the longest, ties to the lowest k
                for (uint32_t k = threadIdx.x; k < nhuge; k += blockDim.x) {
                    const uint32_t len = L.list[3][k].len;
                    if (__hip_atomic_load(&L.claim[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
                        const uint64_t c = ((uint64_t)len << 32) | (uint32_t)~k;
                        best = c > best ? c : best;
                    }
                }
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(best, off);
                    best = o > best ? o : best;
                }
                if ((threadIdx.x & 63) == 0) s_best[threadIdx.x >> 6] = best;
                __syncthreads();
                if (threadIdx.x == 0) {
                    uint64_t b = 0;
                    for (int w = 0; w < CH_BLOCK / 64; w++) b = s_best[w] > b ? s_best[w] : b;
                    const uint32_t k = ~(uint32_t)b;
                    s_u = b == 0 ? NO_STOP : (atomicCAS(&L.claim[k], 0u, 1u) == 0u ? k : NO_STOP - 1u);
                }
                __syncthreads();
                if (s_u != NO_STOP - 1u) break;   // claimed one, or none is left; else another block won it: again
                __syncthreads();
            }
        }
        __syncthreads();
        const uint32_t u = s_u;
        __syncthreads();
        if (u == NO_STOP) break;
        const SegRec sg = L.list[3][u];
        const uint64_t t_seg = __builtin_amdgcn_s_memrealtime();
        ch_segment<LCFG>(sh, &tb[sk[sg.j0]], sg.j0, sg.j0 + sg.len, cfgs, profile, a, pre, eflags, dbg, runs,
                         plan_seq);
        __syncthreads();
        if (threadIdx.x == 0 && dbg) {
            const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
            if (atomicMax(&dbg[8], (uint32_t)(t_end - t_seg)) < (uint32_t)(t_end - t_seg)) {
                dbg[16] = (uint32_t)t_seg;
                dbg[17] = (uint32_t)t_end;
            }
        }
    }
    replay_rest(sk, L, qctr, win_base, tb, win, spill, cfgs, profile, a, pre, eflags, dbg, s_u, 0u);
}

// The replay kernel of a batch with no huge segment expected (the last
// replay the host saw had none: mixed, uniform and bursty traffic): phases 2-3
// only, in blocks of LT_BLOCK threads -- without the chain's 156 KB of LDS and
// its register budget, a CU holds 12 replay waves instead of 8.  A huge
// segment that arrives anyway is replayed as a heavy one (wave_segment:
// exact, one wave), and the host word makes the next batches take the chain
// kernel again.
#ifndef RL_LT_BLOCK
#define RL_LT_BLOCK 768
#endif
constexpr int LT_BLOCK = RL_LT_BLOCK;
template <bool LCFG>
__global__ __launch_bounds__(LT_BLOCK) void k_replay_light(const uint32_t* __restrict__ sk, SegLists L, uint32_t* qctr,
                                                           uint32_t win_base, TbEntry* tb, WinEntry* win, Spill spill,
                                                           const CfgDev* __restrict__ gcfgs, uint32_t ncfg,
                                                           int32_t profile, ReqArgs a, TbPre pre, uint32_t* eflags,
                                                           uint32_t* dbg, TbRuns runs, uint32_t grid_base,
                                                           uint32_t light_min, uint32_t* h_huge) {
    __shared__ uint32_t s_u;
    __shared__ CfgDev s_cfg[LCFG ? MAX_LCFG : 1];
    if (LCFG) {
        for (uint32_t c = threadIdx.x; c < ncfg; c += blockDim.x) s_cfg[c] = gcfgs[c];
        __syncthreads();
    }
    (void)runs;
    const CfgDev* cfgs = LCFG ? s_cfg : gcfgs;
    const uint32_t nhuge = L.count[3];
    if (blockIdx.x == 0 && threadIdx.x == 0 && h_huge) *(volatile uint32_t*)h_huge = nhuge;
    if (!replay_joins(L, grid_base, light_min)) return;
    if (threadIdx.x == 0 && dbg) atomicMax(&dbg[13], ~(uint32_t)__builtin_amdgcn_s_memrealtime());
    replay_rest(sk, L, qctr, win_base, tb, win, spill, cfgs, profile, a, pre, eflags, dbg, s_u, nhuge);
}

}  // namespace rl
