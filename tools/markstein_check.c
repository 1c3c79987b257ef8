/* Check of the conductivity phase's s1 quotient (h9g_pair.h hk_fast):
 *   y = RN(1/b), q0 = RN(a y), e = RN(b * -q0 + a), q1 = RN(e y + q0)
 * against the IEEE quotient RN(a/b), for a, b in [2^-60, 2^60).
 * Markstein's theorem (y within half an ulp of 1/b, q0 within one ulp of
 * a/b, no under/overflow) says q1 = RN(a/b); this runs it:
 *   1. every significand of b in [1, 2), with random a in [1, 4) and a near
 *      the midpoints of RN(a/b) (the hard cases), PER a's per b;
 *   2. random a, b over the whole guarded exponent range;
 *   3. a control with y one ulp off RN(1/b), which must fail somewhere.
 * Build and run:  gcc -O2 -ffp-contract=off -o /tmp/mk tools/markstein_check.c -lm && /tmp/mk 64
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float fb(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static uint64_t s = 88172645463325252ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }

static float mk(float a, float b, float y) {
  const float q0 = a * y;
  return fmaf(fmaf(-b, q0, a), y, q0);
}

static long sweep(int per, int off) {
  long bad = 0;
  for (uint32_t mb = 0; mb < (1u << 23); mb++) {
    const float b = fb(0x3f800000u | mb);
    const float y = fb(bf(1.0f / b) + off);
    for (int k = 0; k < per; k++) {
      const uint64_t r = rnd();
      float a;
      if (k & 1) {
        a = fb(0x3f800000u | (uint32_t)(r & 0x7fffff)) * (((r >> 40) & 1) ? 2.0f : 1.0f);
      } else {                           /* a = RN(b * midpoint) + d ulps */
        const float q = fb(0x3f000000u + (uint32_t)(r % (0x40000000u - 0x3f000000u)));
        const double mid = (double)q + 0.5 * ((double)nextafterf(q, INFINITY) - (double)q);
        a = fb(bf((float)((double)b * mid)) + (int)((r >> 50) % 5) - 2);
      }
      if (bf(mk(a, b, y)) != bf(a / b)) bad++;
    }
  }
  return bad;
}

int main(int argc, char **argv) {
  const int per = argc > 1 ? atoi(argv[1]) : 16;
  const long b1 = sweep(per, 0);
  printf("1. b over [1,2) exhaustively x %d a: %ld mismatches in %lld\n", per, b1, (long long)per << 23);
  long b2 = 0, n2 = 200000000;
  for (long i = 0; i < n2; i++) {
    const uint64_t r = rnd();
    const float a = fb(0x21800000u + (uint32_t)(r % (0x5d800000u - 0x21800000u)));
    const float b = fb(0x21800000u + (uint32_t)((r >> 32) % (0x5d800000u - 0x21800000u)));
    if (bf(mk(a, b, 1.0f / b)) != bf(a / b)) b2++;
  }
  printf("2. a, b over [2^-60, 2^60): %ld mismatches in %ld\n", b2, n2);
  const long b3 = sweep(per, 1);
  printf("3. control, y one ulp above RN(1/b): %ld mismatches (must be > 0)\n", b3);
  return (b1 == 0 && b2 == 0 && b3 > 0) ? 0 : 1;
}
