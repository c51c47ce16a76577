/* Exactness check of the kd-descent split distance with a per-ray reciprocal
 * (device_math.hpp div_by_rcp, the FD trace builds):
 *     y  = RN(1/b)                  once per ray and axis
 *     q0 = RN(a*y);  r = fma(-q0, b, a);  q = fma(r, y, q0)
 * claimed equal to RN(a/b) whenever 2^-40 <= |b| <= 2^40 and 2^-60 <= |q0| <= 2^60.
 * Every b significand (2^23) is tried, with random a and with a built so that
 * a/b sits next to a rounding midpoint (the hard cases), over a spread of
 * exponents.  x86-64 SSE float ops and fmaf are IEEE RN, like the GPU's.
 *   gcc -O2 -fopenmp -ffp-contract=off scripts/markstein_check.c -o /tmp/mc -lm && /tmp/mc [per_b]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline float fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}

int main(int argc, char **argv) {
    const int per_b = argc > 1 ? atoi(argv[1]) : 64;
    const float lo_q = ldexpf(1.f, -60), hi_q = ldexpf(1.f, 60);
    long long tested = 0, skipped = 0, bad = 0;
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : tested, skipped, bad)
    for (uint32_t m = 0; m < (1u << 23); m++) {
        uint64_t s = mix64(m + 1);
        for (int k = 0; k < per_b; k++) {
            s = mix64(s + k);
            const int eb = (int)(s % 81) - 40;                       /* b exponent in [-40, 40] */
            const uint32_t sb = (uint32_t)(s >> 8) & 1u;
            const float b = fbits((sb << 31) | ((uint32_t)(eb + 127) << 23) | m);
            float a;
            if (k & 1) {
                /* a/b next to a midpoint: take a random q, its midpoint with the next
                 * float, a = RN(mid * b) (double product rounded once to float) */
                const int eq = (int)((s >> 16) % 101) - 50;
                const float q = fbits(((uint32_t)(eq + 127) << 23) | ((uint32_t)(s >> 24) & 0x7fffffu));
                const double mid = ((double)q + (double)nextafterf(q, INFINITY)) * 0.5;
                a = (float)(mid * (double)b);
                if (s & (1ull << 60)) a = nextafterf(a, INFINITY);
                if (s & (1ull << 61)) a = nextafterf(a, -INFINITY);
            } else {
                const int ea = eb + (int)((s >> 16) % 101) - 50;
                if (ea < -100 || ea > 100) { skipped++; continue; }
                a = fbits(((uint32_t)(s >> 40) & 1u) << 31 | ((uint32_t)(ea + 127) << 23) |
                          ((uint32_t)(s >> 41) & 0x7fffffu));
            }
            const float y = 1.f / b;
            const float q0 = a * y;
            if (!(fabsf(q0) >= lo_q && fabsf(q0) <= hi_q)) { skipped++; continue; }
            const float r = fmaf(-q0, b, a);
            const float q = fmaf(r, y, q0);
            const float ref = a / b;
            tested++;
            if (ubits(q) != ubits(ref)) {
                if (bad < 10)
#pragma omp critical
                    fprintf(stderr, "MISMATCH a=%a b=%a q=%a ref=%a\n", a, b, q, ref);
                bad++;
            }
        }
    }
    printf("tested %lld skipped %lld mismatches %lld\n", tested, skipped, bad);
    return bad != 0;
}
