/* Checks that  q0 = x r, q1 = fma(fma(-d, q0, x), r, q0), q2 = fma(fma(-d, q1, x), r, q1)
 * with r = RN(1/d) equals the IEEE quotient x / d bit for bit (Markstein: r
 * correctly rounded and q1 faithful => q2 = RN(x/d); no overflow/underflow).
 * Usage: div_exact N [d ...]  -- N random (x, d) pairs over wide exponent
 * ranges, then N random x per listed divisor d.  Prints mismatches; exit 1 if any. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9e3779b97f4a7c15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double unif(void) { return (rnd() >> 11) * 0x1.0p-53; }
static double rnd_mag(double lo_exp, double hi_exp) {   /* log-uniform magnitude */
  return pow(10.0, lo_exp + (hi_exp - lo_exp) * unif());
}
static double q2(double x, double d, double r) {
  double q0 = x * r;
  double q1 = fma(fma(-d, q0, x), r, q0);
  return fma(fma(-d, q1, x), r, q1);
}
static long check(double x, double d) {
  double r = 1.0 / d, a = x / d, b = q2(x, d, r);
  if (memcmp(&a, &b, 8) != 0 && !(a == 0 && b == 0)) {
    printf("mismatch x=%.17g d=%.17g exact=%.17g got=%.17g\n", x, d, a, b);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 1000000, bad = 0;
  for (long i = 0; i < n; ++i) {
    double d = rnd_mag(-6, 6) * ((rnd() & 1) ? 1 : -1);
    double x = rnd_mag(-12, 12) * ((rnd() & 1) ? 1 : -1);
    bad += check(x, d);
    /* random bit patterns of the mantissa at fixed exponents */
    uint64_t bx = (rnd() & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    uint64_t bd = (rnd() & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double xx, dd;
    memcpy(&xx, &bx, 8);
    memcpy(&dd, &bd, 8);
    bad += check(xx, dd);
  }
  for (int a = 2; a < argc; ++a) {
    double d = atof(argv[a]);
    for (long i = 0; i < n; ++i) {
      double x = (2.0 * unif() - 1.0) * fabs(d) * 1.5;
      bad += check(x, d);
      bad += check(nextafter(x, 0.0), d);
    }
  }
  printf("checked, mismatches: %ld\n", bad);
  return bad ? 1 : 0;
}
