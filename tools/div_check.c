/* Check of ch_device.h divc(): x / c as q = RN(x * RN(1/c)), r = fma(-q, c, x), q2 = fma(r, rc, q),
 * q when r is +-0 or NaN -- against IEEE division, for the divisors the step kernels use and for
 * random divisors (the reciprocal then computed once by IEEE division, as for a loop-invariant c).
 * Usage: div_check [samples per divisor]   Prints one line per divisor and exits non-zero on any
 * mismatch.  Host C with the same fp64 fma semantics as the gfx950 v_fma_f64. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st[2] = {0x12345678abcdefULL, 0x9abcdef012345ULL};
static uint64_t rnd(void) {
    uint64_t s1 = st[0];
    const uint64_t s0 = st[1];
    st[0] = s0;
    s1 ^= s1 << 23;
    st[1] = s1 ^ s0 ^ (s1 >> 17) ^ (s0 >> 26);
    return st[1] + s0;
}
/* random sign and significand, exponent in [2^-60, 2^60) */
static double rd(void) {
    uint64_t b = rnd();
    const int e = (int)(rnd() % 120) - 60 + 1023;
    b = (b & 0x800FFFFFFFFFFFFFULL) | ((uint64_t)e << 52);
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static double divc(double x, double c, double rc) {
    const double q = x * rc, r = fma(-q, c, x), q2 = fma(r, rc, q);
    return (r == 0.0 || r != r) ? q : q2;
}
static int same(double a, double b) { return memcmp(&a, &b, 8) == 0 || (a != a && b != b); }

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000L;
    const double kEps = 0.1, kH = 0.2;
    const double cs[] = {0.027 /* kMass */, 1.4e-5, 2.17e-5 /* J */, 4 * 3.16e-10 /* 4 kf */, 0.2685 /* pwm scale */,
                         kEps, 1 - kH, (sqrt(1 + kEps * (1.2 * 1.2)) - 1) / kEps /* ra */, 1.0 / 60 /* dt */,
                         1.0 / 240, 0.4 + 1e-9, 0.3 + 1e-9, 3.5, 2 * (3.3 * 3.3), 2 * (0.2 * 0.2), 100.0, 16.0};
    long bad_total = 0;
    for (size_t k = 0; k < sizeof(cs) / sizeof(cs[0]); ++k) {
        const double c = cs[k], rc = 1.0 / c;
        long bad = 0;
        for (long i = 0; i < n; ++i) {
            const double x = rd();
            if (!same(divc(x, c, rc), x / c)) ++bad;
        }
        /* edge operands */
        const double edge[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 1.0, -1.0, c, -c};
        for (size_t j = 0; j < sizeof(edge) / sizeof(edge[0]); ++j)
            if (!same(divc(edge[j], c, rc), edge[j] / c)) ++bad;
        printf("c=%.17g bad=%ld\n", c, bad);
        bad_total += bad;
    }
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        const double a = rd(), b = rd();
        if (!same(divc(a, b, 1.0 / b), a / b)) ++bad;
    }
    printf("random divisors bad=%ld\n", bad);
    bad_total += bad;
    return bad_total != 0;
}
