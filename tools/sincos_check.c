/* Check of ch_device.h sincos_small(): the fdlibm __kernel_sin / __kernel_cos polynomials without
 * argument reduction, as the drone substep evaluates them for 0 <= x <= pi/8 (the exponential-map
 * half angle after btMultiBody's clamp), against glibc sin/cos.  Arguments are uniform in [0, pi/8],
 * scaled by 1e-3 and 1e-7 for a quarter each, plus the endpoints.
 * Also cos_0pi() (the bump's cos on [0, pi]: Cody-Waite reduction by pi/2, then these kernels) against
 * glibc cos over uniform arguments in [0, pi] plus the quadrant boundaries.
 * Usage: sincos_check [samples]   Prints the max ulp distance and exits non-zero above 1 ulp. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int32_t hiword(double x) { uint64_t u; memcpy(&u, &x, 8); return (int32_t)(u >> 32); }
static double from_hilo(int32_t hi, uint32_t lo) {
    uint64_t v = ((uint64_t)(uint32_t)hi << 32) | lo;
    double r; memcpy(&r, &v, 8); return r;
}
/* the device function, line for line (selects as in ch_device.h) */
static void sincos_small(double x, double* s, double* c) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    *s = x + v * (S1 + z * r);
    const double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const int ix = hiword(x) & 0x7fffffff;
    const double qx = ix > 0x3fe90000 ? 0.28125 : from_hilo(ix - 0x00200000, 0);
    const double big = (1.0 - qx) - ((0.5 * z - qx) - (z * rc - 0.0));
    const double small = 1.0 - (0.5 * z - (z * rc - 0.0));
    *c = ix < 0x3FD33333 ? small : big;
}
static double cos_0pi(double x) {
    const double PIO2_1 = 1.57079632673412561417e+00, PIO2_2 = 6.07710050630396597660e-11,
                 PIO2_3 = 2.02226624871116645580e-21, PIO2_3T = 8.47842766036889956997e-32;
    const double n = rint(x * 6.36619772367581382433e-01);
    const double r = (((x - n * PIO2_1) - n * PIO2_2) - n * PIO2_3) - n * PIO2_3T;
    double s, c;
    sincos_small(fabs(r), &s, &c);
    s = r < 0 ? -s : s;
    return n == 0.0 ? c : (n == 1.0 ? -s : -c);
}
static void sincos_pi(double x, double* s, double* c) {
    const double PIO2_1 = 1.57079632673412561417e+00, PIO2_2 = 6.07710050630396597660e-11,
                 PIO2_3 = 2.02226624871116645580e-21, PIO2_3T = 8.47842766036889956997e-32;
    const double n = rint(x * 6.36619772367581382433e-01);
    const double r = (((x - n * PIO2_1) - n * PIO2_2) - n * PIO2_3) - n * PIO2_3T;
    double sr, cr;
    sincos_small(fabs(r), &sr, &cr);
    sr = r < 0 ? -sr : sr;
    const int q = (int)n & 3;
    *s = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    *c = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}
static double ulps(double a, double b) {
    if (a == b) return 0;
    int e; frexp(b, &e);
    return fabs(a - b) / ldexp(1.0, e - 53);
}
int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 20000000;
    uint64_t st = 12345;
    double ms = 0, mc = 0;
    long ds = 0, dc = 0;
    const double lim = M_PI / 8;
    for (long i = 0; i < n + 2; ++i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        double x = (double)(st >> 11) * (1.0 / 9007199254740992.0) * lim;
        if (i % 4 == 1) x *= 1e-3; else if (i % 4 == 2) x *= 1e-7;
        if (i == n) x = 0.0; else if (i == n + 1) x = lim;
        double s, c;
        sincos_small(x, &s, &c);
        const double us = ulps(s, sin(x)), uc = ulps(c, cos(x));
        if (us > ms) ms = us;
        if (uc > mc) mc = uc;
        ds += s != sin(x); dc += c != cos(x);
    }
    printf("samples=%ld max_ulp_sin=%.3f max_ulp_cos=%.3f differ_sin=%ld differ_cos=%ld\n", n + 2, ms, mc, ds, dc);
    double mp = 0;
    long dp = 0;
    for (long i = 0; i < n + 4; ++i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        double x = (double)(st >> 11) * (1.0 / 9007199254740992.0) * M_PI;
        if (i == n) x = 0.0; else if (i == n + 1) x = M_PI; else if (i == n + 2) x = M_PI / 4; else if (i == n + 3) x = 3 * M_PI / 4;
        const double c = cos_0pi(x), ref = cos(x);
        const double u = ulps(c, ref);
        if (u > mp) mp = u;
        dp += c != ref;
    }
    printf("cos_0pi: samples=%ld max_ulp=%.3f differ=%ld\n", n + 4, mp, dp);
    double m2s = 0, m2c = 0;
    for (long i = 0; i < n + 5; ++i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        double x = ((double)(st >> 11) * (1.0 / 9007199254740992.0) * 2 - 1) * M_PI;
        if (i == n) x = -M_PI; else if (i == n + 1) x = M_PI; else if (i == n + 2) x = -M_PI / 2;
        else if (i == n + 3) x = 3 * M_PI / 4; else if (i == n + 4) x = -0.0;
        double s, c;
        sincos_pi(x, &s, &c);
        const double us = ulps(s, sin(x)), uc = ulps(c, cos(x));
        if (us > m2s) m2s = us;
        if (uc > m2c) m2c = uc;
    }
    printf("sincos_pi: samples=%ld max_ulp_sin=%.3f max_ulp_cos=%.3f\n", n + 5, m2s, m2c);
    return (ms <= 1.0 && mc <= 1.0 && mp <= 1.0 && m2s <= 1.0 && m2c <= 1.0) ? 0 : 1;
}
