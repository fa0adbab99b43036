/* Host check of div_p10 (csrc/rl_tb_chain.h): x / 10^k by five fma-based
 * operations with R = RN(10^-k) against IEEE division, for integer-valued x
 * below 2^47 (random, half of them in the decimal mode's [1e13, 1e14)) and
 * every k in [1, 22], plus the decade edges.  Usage: div_p10_check [samples per k]
 * Build: gcc -O2 -ffp-contract=off div_p10_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t st = 88172645463325252ull;
static uint64_t xs(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }

static double div_p10(double x, double P, double R) {
    const double q0 = x * R;
    const double q1 = fma(fma(-q0, P, x), R, q0);
    return fma(fma(-q1, P, x), R, q1);
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 60000000L;
    long bad = 0, tot = 0;
    double P = 1.0;
    for (int k = 1; k <= 22; k++) {
        P *= 10.0;
        const double R = 1.0 / P;
        const double edge[] = {0.0, 1.0, 1e13, 1e13 + 1, 1e14 - 1, 1e14, 140737488355327.0, 99999999999999.0};
        for (long i = 0; i < n + 8; i++) {
            double x;
            if (i < 8) x = edge[i];
            else {
                const uint64_t r = xs();
                x = (i & 1) ? (double)(10000000000000LL + (int64_t)(r % 90000000000000ull))
                            : (double)(r % 140737488355328ull);
                if (i & 2) x = -x;
            }
            const double a = div_p10(x, P, R), b = x / P;
            tot++;
            if (a != b || signbit(a) != signbit(b)) {
                if (bad < 10) printf("k=%d x=%.17g got %.17g want %.17g\n", k, x, a, b);
                bad++;
            }
        }
    }
    /* the multi-decade windows' reciprocals: RN(10^-e0) times an exact 10^k
     * (k <= 4), rounded -- within 2^-52 of 1 / 10^(e0 - k) */
    for (int e0 = 5; e0 <= 22; e0++) {
        double Pe = 1.0, Re;
        for (int i = 0; i < e0; i++) Pe *= 10.0;
        Re = 1.0 / Pe;
        double t = 1.0;
        for (int k = 0; k <= 4 && e0 - k >= 1; k++, t *= 10.0) {
            double Pk = 1.0;
            for (int i = 0; i < e0 - k; i++) Pk *= 10.0;
            const double R = Re * t;
            for (long i = 0; i < n / 8; i++) {
                const uint64_t r = xs();
                double x = (i & 1) ? (double)(10000000000000LL + (int64_t)(r % 90000000000000ull))
                                   : (double)(r % 140737488355328ull);
                if (i & 2) x = -x;
                const double a = div_p10(x, Pk, R), b = x / Pk;
                tot++;
                if (a != b || signbit(a) != signbit(b)) {
                    if (bad < 10) printf("e0=%d k=%d x=%.17g got %.17g want %.17g\n", e0, k, x, a, b);
                    bad++;
                }
            }
        }
    }
    printf("div_p10: %ld cases, %ld mismatches\n", tot, bad);
    return bad != 0;
}
