// rl_q14.h -- exact `tonumber(tostring(x))` of Redis 7's Lua 5.1 on CDNA4.
//
// The token-bucket script persists its state with tostring()
// (reference: internal/ratelimiter/tokenbucket.go:48), which Redis's Lua 5.1
// formats with sprintf("%.14g") (LUAI_NUMFFORMAT); the next call parses it back
// with tonumber() = strtod (tokenbucket.go:32-33).  glibc rounds both steps
// correctly (printf: round-half-even on the 14th digit; strtod: nearest-even),
// so the round trip is the pure function
//
//     q14(x) = RN_double( RNE_14_significant_digits( x ) ).
//
// This header computes it exactly, as __host__ __device__ code (the host
// instantiation is fuzzed against glibc in tests/, the device one against the
// oracle on the GPU):
//   * fast path, 1e-9 <= |x| < 1e35: one exact product (TwoProduct via fma) or
//     one exact division residual gives the 14-digit integer D and its rounding
//     direction; D / 10^k (or D * 10^k) is then a single correctly rounded IEEE
//     operation because D < 2^47 and 10^k (k <= 22) are exact doubles;
//   * wide path, 1e-345 < |x| < 1e-9 (normal doubles): 128-bit truncated
//     powers of five (rl_pow5.h) give D, and D * 10^j back to a double, with
//     a proven error bound; a result the bound cannot decide (never seen in
//     fuzzing: it needs a remainder within 2^-70 of a rounding midpoint) falls
//     through to
//   * slow path, everything else: fixed-width big-integer arithmetic.
// All code here must be compiled with -ffp-contract=off.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RL_HD __host__ __device__
#else
#include <math.h>
#define RL_HD
#endif
// Fast paths are forced inline: an out-of-line call on AMDGPU sets up a stack
// frame in scratch memory on every step.  The big-integer slow paths (rare:
// |x| < 1e-9 or >= 1e35) stay out of line so their arrays never touch the
// hot loop's registers.
#define RL_INLINE RL_HD inline __attribute__((always_inline))
#define RL_COLD RL_HD inline __attribute__((noinline))

namespace rlq {

#if defined(__HIPCC__)
// diagnostic: device calls of the big-integer slow paths (each costs
// hundreds of microseconds to milliseconds of one lane); read by
// rl_engine_debug_q14_slow
static __device__ unsigned long long q14_slow_calls;
#define RL_COUNT_SLOW() atomicAdd(&q14_slow_calls, 1ull)
#endif
#if !defined(__HIP_DEVICE_COMPILE__)
#undef RL_COUNT_SLOW
#define RL_COUNT_SLOW() ((void)0)
#endif

// 10^k, k in [0,22]: every partial product is a power of ten <= 1e22, hence exact.
RL_INLINE double pow10_exact(int k) {
    double p = 1.0;
    if (k & 1) p *= 1e1;
    if (k & 2) p *= 1e2;
    if (k & 4) p *= 1e4;
    if (k & 8) p *= 1e8;
    if (k & 16) p *= 1e16;
    return p;
}

RL_INLINE uint64_t dbits(double x) {
    union { double d; uint64_t u; } v; v.d = x; return v.u;
}
RL_INLINE double bitsd(uint64_t u) {
    union { double d; uint64_t u; } v; v.u = u; return v.d;
}

// floor(e2 * log10(2)) for |e2| <= 2000
RL_INLINE int floor_log10_pow2(int e2) { return (e2 * 78913) >> 18; }

// Round a * 10^k (a > 0, |k| <= 22, result < 2^47) to the nearest integer,
// ties to even, exactly; ge: the exact a * 10^k >= lo (an integer-valued
// double), which the rounded result cannot tell when it rounds up onto lo.
RL_INLINE int64_t round_scaled_ge(double a, int k, double lo, bool& ge) {
    double p, err;
    if (k >= 0) {
        double P = pow10_exact(k);
        p = a * P;
        err = __builtin_fma(a, P, -p);          // a*P == p + err exactly
    } else {
        double P = pow10_exact(-k);
        p = a / P;
        err = __builtin_fma(-p, P, a);          // a - p*P, exact; sign = direction
    }
    ge = (p > lo) || (p == lo && err >= 0.0);
    double d0 = floor(p);
    double f = p - d0;                           // exact (p has few fraction bits)
    int64_t D = (int64_t)d0;
    bool up;
    if (f > 0.5) up = true;
    else if (f < 0.5) up = false;
    else up = (err > 0.0) || (err == 0.0 && (D & 1));
    return D + (up ? 1 : 0);
}
RL_INLINE int64_t round_scaled(double a, int k) {
    bool ge;
    return round_scaled_ge(a, k, 0.0, ge);
}


// RNE(x * P) exactly, for x > 0, P = 10^k exact (k <= 22), x*P < 2^47
#include "rl_pow5.h"

// ---------------------------------------------------------------------------
// wide path (cold): 192-bit products with 128-bit powers of five
// ---------------------------------------------------------------------------
typedef unsigned __int128 u128;

// (w2:w1:w0) = m * (fhi:flo)
RL_INLINE void mul_64x128(uint64_t m, uint64_t fhi, uint64_t flo, uint64_t& w2, uint64_t& w1, uint64_t& w0) {
    const u128 a = (u128)m * flo, b = (u128)m * fhi;
    w0 = (uint64_t)a;
    const u128 mid = (a >> 64) + (u128)(uint64_t)b;
    w1 = (uint64_t)mid;
    w2 = (uint64_t)(b >> 64) + (uint64_t)(mid >> 64);
}

// RNE(W' * 2^-t) where the exact W' lies in [W, W + err), W = (w2:w1:w0),
// 64 <= t <= 191, err < 2^64: q = floor(W * 2^-t) (must fit 64 bits) and
// whether to round up.  False when [W, W + err) straddles the midpoint.
RL_INLINE bool round_shift192(uint64_t w2, uint64_t w1, uint64_t w0, int t, uint64_t err, uint64_t& q, bool& up) {
    if (t < 64 || t > 191) return false;
    const int s = t - 64;
    const u128 hi = ((u128)w2 << 64) | w1;
    const u128 qq = hi >> s;
    if ((uint64_t)(qq >> 64)) return false;
    q = (uint64_t)qq;
    // remainder R = (rh : w0), rh < 2^s; the midpoint 2^(t-1)
    const u128 rh = s ? (hi & (((u128)1 << s) - 1)) : 0;
    const u128 hh = s ? ((u128)1 << (s - 1)) : 0;
    const uint64_t hl = s ? 0 : (1ull << 63);
    const bool gt_half = rh > hh || (rh == hh && w0 > hl);          // R > half
    const uint64_t e0 = w0 + err;
    const u128 eh = rh + (e0 < w0 ? 1 : 0);                          // R + err = (eh : e0)
    const bool le_half = eh < hh || (eh == hh && e0 <= hl);          // R + err <= half
    if (gt_half) { up = true; return true; }
    if (le_half) { up = false; return true; }
    return false;
}

// RNE(m * 2^e * 10^k), k in [POW5_KMIN, POW5_KMAX], result < 2^62, and
// floor(m * 2^e * 10^k) in Dfloor
RL_INLINE bool round_scaled_wide(uint64_t m, int e, int k, int64_t& D, int64_t& Dfloor) {
    const Pow5 p = pow5_pos(k);                 // 5^k = (F + theta) 2^sh
    uint64_t w2, w1, w0, q;
    mul_64x128(m, p.hi, p.lo, w2, w1, w0);      // exact product in [W, W + m)
    bool up;
    if (!round_shift192(w2, w1, w0, -(p.sh + e + k), m, q, up)) return false;
    if (q >= (1ull << 62)) return false;
    D = (int64_t)(q + (up ? 1 : 0));
    Dfloor = (int64_t)q;
    return true;
}

// correctly rounded D * 10^-n (strtod), n in [POW5_KMIN, POW5_KMAX], 0 < D < 2^63;
// false when undecided or the result is not a normal double
RL_INLINE bool dec_value_wide(uint64_t D, int n, double& out) {
    const Pow5 p = pow5_neg(n);                 // 5^-n = (G + theta) 2^-sh
    uint64_t w2, w1, w0, q;
    mul_64x128(D, p.hi, p.lo, w2, w1, w0);      // exact product in [W, W + D)
    const int L = w2 ? 128 + 64 - __builtin_clzll(w2) : (w1 ? 64 + 64 - __builtin_clzll(w1) : 64 - __builtin_clzll(w0));
    int t = L - 53;
    bool up;
    if (!round_shift192(w2, w1, w0, t, D, q, up)) return false;
    q += up ? 1 : 0;
    if (q == (1ull << 53)) { q >>= 1; t++; }
    const int ex = t - p.sh - n;                // value = q * 2^ex, q in [2^52, 2^53)
    if (ex + 52 < -1022 || ex + 52 > 1023) return false;
    out = ldexp((double)q, ex);
    return true;
}

RL_INLINE int64_t round_scaled_P(double x, double P) {
    double p = x * P;
    double err = __builtin_fma(x, P, -p);
    double d0 = floor(p);
    double f = p - d0;
    int64_t D = (int64_t)d0;
    bool up = (f > 0.5) || (f == 0.5 && ((err > 0.0) || (err == 0.0 && (D & 1))));
    return D + (up ? 1 : 0);
}
RL_INLINE bool round_scaled_is(double x, double P, int64_t want) { return round_scaled_P(x, P) == want; }

// -------------------------------------------------------------------------
// slow path: fixed-width big integers (32-bit limbs, little endian)
// -------------------------------------------------------------------------
constexpr int BN_LIMBS = 40;   // 1280 bits: covers m*5^337*2^k and 5^295*2^1074

struct Big {
    uint32_t w[BN_LIMBS];
    int n;  // limbs in use
};

RL_HD inline void bn_set_u64(Big& b, uint64_t v) {
    for (int i = 0; i < BN_LIMBS; i++) b.w[i] = 0;
    b.w[0] = (uint32_t)v;
    b.w[1] = (uint32_t)(v >> 32);
    b.n = b.w[1] ? 2 : (b.w[0] ? 1 : 0);
}
RL_HD inline void bn_mul_small(Big& b, uint32_t m) {
    uint64_t carry = 0;
    for (int i = 0; i < b.n; i++) {
        uint64_t t = (uint64_t)b.w[i] * m + carry;
        b.w[i] = (uint32_t)t;
        carry = t >> 32;
    }
    if (carry) b.w[b.n++] = (uint32_t)carry;
}
RL_HD inline void bn_mul_pow5(Big& b, int k) {
    while (k >= 13) { bn_mul_small(b, 1220703125u); k -= 13; }   // 5^13
    uint32_t m = 1;
    while (k-- > 0) m *= 5;
    if (m != 1) bn_mul_small(b, m);
}
RL_HD inline void bn_shl(Big& b, int s) {
    if (b.n == 0 || s == 0) return;
    int ls = s >> 5, bs = s & 31;
    int nn = b.n + ls + 1;
    for (int i = nn - 1; i >= 0; i--) {
        int src = i - ls;
        uint32_t hi = (src >= 0 && src < b.n) ? b.w[src] : 0;
        uint32_t lo = (src - 1 >= 0 && src - 1 < b.n) ? b.w[src - 1] : 0;
        b.w[i] = bs ? (uint32_t)((hi << bs) | (lo >> (32 - bs))) : hi;
    }
    b.n = nn;
    while (b.n > 0 && b.w[b.n - 1] == 0) b.n--;
}
RL_HD inline void bn_shr1(Big& b) {
    for (int i = 0; i < b.n; i++) {
        uint32_t next = (i + 1 < b.n) ? b.w[i + 1] : 0;
        b.w[i] = (b.w[i] >> 1) | (next << 31);
    }
    while (b.n > 0 && b.w[b.n - 1] == 0) b.n--;
}
RL_HD inline int bn_cmp(const Big& a, const Big& b) {
    if (a.n != b.n) return a.n < b.n ? -1 : 1;
    for (int i = a.n - 1; i >= 0; i--)
        if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
}
RL_HD inline void bn_sub(Big& a, const Big& b) {   // a -= b, requires a >= b
    int64_t borrow = 0;
    for (int i = 0; i < a.n; i++) {
        int64_t t = (int64_t)a.w[i] - (i < b.n ? (int64_t)b.w[i] : 0) - borrow;
        borrow = t < 0;
        a.w[i] = (uint32_t)(t + (borrow ? ((int64_t)1 << 32) : 0));
    }
    while (a.n > 0 && a.w[a.n - 1] == 0) a.n--;
}
RL_HD inline int bn_bitlen(const Big& b) {
    if (b.n == 0) return 0;
    uint32_t top = b.w[b.n - 1];
    int l = 0;
    while (top) { l++; top >>= 1; }
    return (b.n - 1) * 32 + l;
}
RL_HD inline bool bn_is_zero(const Big& b) { return b.n == 0; }

// q = floor(N / Q) (q < 2^qbits), N <- remainder
RL_HD inline uint64_t bn_divmod_small_q(Big& N, const Big& Q, int qbits) {
    Big T = Q;
    bn_shl(T, qbits - 1);
    uint64_t q = 0;
    for (int b = qbits - 1; b >= 0; b--) {
        if (bn_cmp(T, N) <= 0) { bn_sub(N, T); q |= (uint64_t)1 << b; }
        bn_shr1(T);
    }
    return q;
}

// exact round(a * 10^k) to nearest-even integer (result < 2^48); a = m * 2^e
RL_COLD int64_t round_scaled_big(uint64_t m, int e, int k, int64_t* floor_out = nullptr) {
    Big N, Q;
    bn_set_u64(N, m);
    bn_set_u64(Q, 1);
    int s;
    if (k >= 0) { bn_mul_pow5(N, k); s = e + k; }
    else { bn_mul_pow5(Q, -k); s = e + k; }
    if (s >= 0) bn_shl(N, s); else bn_shl(Q, -s);
    uint64_t D = bn_divmod_small_q(N, Q, 50);
    if (floor_out) *floor_out = (int64_t)D;
    // compare 2*rem with Q
    bn_shl(N, 1);
    int c = bn_cmp(N, Q);
    if (c > 0 || (c == 0 && (D & 1))) D++;
    return (int64_t)D;
}

// correctly rounded q * 2^b (+ sticky) to double, subnormals included; q < 2^64
RL_HD inline double round_to_double(uint64_t q, int b, bool sticky) {
    if (q == 0) return 0.0;
    int L = 64 - __builtin_clzll(q);
    int lead = b + L - 1;
    int drop = (lead >= -1022) ? (L - 53) : (-1074 - b);
    if (drop <= 0) return ldexp((double)q, b);  // exact (sticky impossible by construction)
    uint64_t kept, rem, half;
    if (drop >= 64) {
        kept = 0;
        bool up = (drop == 64) && ((q >> 63) & 1) && ((q << 1) != 0 || sticky);
        return up ? ldexp(1.0, b + drop) : 0.0;
    }
    kept = q >> drop;
    rem = q & ((drop == 64) ? ~0ULL : (((uint64_t)1 << drop) - 1));
    half = (uint64_t)1 << (drop - 1);
    if (rem > half || (rem == half && (sticky || (kept & 1)))) kept++;
    return ldexp((double)kept, b + drop);
}

// correctly rounded D * 10^j (D < 2^48, any j in [-400, 400]) as strtod would
RL_COLD double dec_to_double_big(int64_t D, int j) {
    if (j < 0 && -j >= POW5_KMIN && -j <= POW5_KMAX && D > 0) {
        double v;
        if (dec_value_wide((uint64_t)D, -j, v)) return v;
    }
    RL_COUNT_SLOW();
    Big X;
    bn_set_u64(X, (uint64_t)D);
    if (j >= 0) {
        bn_mul_pow5(X, j);                      // value = X * 2^j
        int L = bn_bitlen(X);
        int sh = L > 64 ? L - 64 : 0;
        bool sticky = false;
        // extract the top 64 bits and a sticky bit
        Big T = X;
        for (int i = 0; i < sh; i++) { if (T.w[0] & 1) sticky = true; bn_shr1(T); }
        uint64_t top = (uint64_t)T.w[0] | ((uint64_t)T.w[1] << 32);
        return round_to_double(top, j + sh, sticky);
    }
    Big Q;
    bn_set_u64(Q, 1);
    bn_mul_pow5(Q, -j);                         // value = D / 5^-j * 2^j
    int t = 60 + bn_bitlen(Q) - bn_bitlen(X);   // quotient gets ~60 bits
    if (t < 0) t = 0;
    bn_shl(X, t);
    uint64_t q = bn_divmod_small_q(X, Q, 63);
    bool sticky = !bn_is_zero(X);
    return round_to_double(q, j - t, sticky);
}

// -------------------------------------------------------------------------
// q14
// -------------------------------------------------------------------------

// 14-significant-digit decimal of |x| (x finite, nonzero): |x| ~ D * 10^(E-13),
// D in [1e13, 1e14).  Returns false if the slow path was needed.
RL_INLINE bool dec14_fast(double a, int64_t& D, int& E) {
    int e2 = (int)((dbits(a) >> 52) & 0x7ff) - 1023;
    if (e2 < -1022) return false;                // subnormal: slow path
    int E0 = floor_log10_pow2(e2);
    if (E0 < -9 || E0 > 34) return false;
    const int64_t LO = 10000000000000LL, HI = 100000000000000LL;
    // a >= 10^(E0+1) exactly (a value just below it can ROUND onto 1e13 at
    // E0+1 digits, and its 14 digits are still those of decade E0)
    bool ge;
    int64_t D1 = round_scaled_ge(a, 12 - E0, (double)LO, ge);   // try E = E0 + 1
    if (ge) { D = D1; E = E0 + 1; return true; }
    int64_t D0 = round_scaled(a, 13 - E0);
    if (D0 >= HI) { D = LO; E = E0 + 1; }        // rounding carried into the next decade
    else { D = D0; E = E0; }
    return true;
}

struct Dec14 {
    int64_t D;
    int E;
};

// returned by value (registers): out-parameters of an out-of-line call would
// round-trip through scratch, and scratch loads share vmcnt with the caller's
// pending stores (every join after the call would wait for them)
RL_COLD Dec14 dec14_slow_v(double a) {
    int64_t D;
    int E;
    uint64_t bits = dbits(a);
    int ex = (int)((bits >> 52) & 0x7ff);
    uint64_t m = bits & ((1ULL << 52) - 1);
    int e;
    if (ex == 0) { e = -1074; } else { m |= 1ULL << 52; e = ex - 1075; }
    int L = 64 - __builtin_clzll(m);
    int e2 = e + L - 1;                           // a in [2^e2, 2^(e2+1))
    int E0 = floor_log10_pow2(e2);
    const int64_t LO = 10000000000000LL, HI = 100000000000000LL;
    if (ex != 0 && 12 - E0 >= POW5_KMIN && 13 - E0 <= POW5_KMAX) {
        int64_t D1, D0, F1, F0;
        if (round_scaled_wide(m, e, 12 - E0, D1, F1)) {
            if (F1 >= LO) return Dec14{D1, E0 + 1};   // a >= 10^(E0+1): exact, not rounded onto LO
            if (round_scaled_wide(m, e, 13 - E0, D0, F0)) {
                if (D0 >= HI) return Dec14{LO, E0 + 1};
                return Dec14{D0, E0};
            }
        }
    }
    RL_COUNT_SLOW();
    int64_t F1 = 0;
    int64_t D1 = round_scaled_big(m, e, 12 - E0, &F1);
    if (F1 >= LO) return Dec14{D1, E0 + 1};
    int64_t D0 = round_scaled_big(m, e, 13 - E0);
    if (D0 >= HI) { D = LO; E = E0 + 1; } else { D = D0; E = E0; }
    return Dec14{D, E};
}

RL_INLINE void dec14_slow(double a, int64_t& D, int& E) {
    Dec14 r = dec14_slow_v(a);
    D = r.D;
    E = r.E;
}

// strtod of D * 10^(E-13), D < 2^47
RL_INLINE double dec14_value(int64_t D, int E) {
    int j = E - 13;
    if (j >= -22 && j <= 22) {
        double d = (double)D;                     // exact
        return j >= 0 ? d * pow10_exact(j) : d / pow10_exact(-j);
    }
    return dec_to_double_big(D, j);
}

// tonumber(tostring(x)) in Redis 7's Lua 5.1
RL_INLINE double q14(double x) {
    if (x == 0.0 || !(x - x == 0.0)) return x;   // +-0, inf, nan round-trip unchanged
    double a = x < 0 ? -x : x;
    int64_t D;
    int E;
    if (!dec14_fast(a, D, E)) dec14_slow(a, D, E);
    double v = dec14_value(D, E);
    return x < 0 ? -v : v;
}

}  // namespace rlq
