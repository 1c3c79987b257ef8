// TEST INFRASTRUCTURE: checks hybrid9_amd/csrc/h9_math.h (host build of the
// device math) bit-for-bit against this machine's glibc expf/powf.
//   check_math expf_all            all 2^32 float inputs
//   check_math expf_rand N seed    N random inputs
//   check_math powf_rand N seed    N random (x, y) pairs from mixed ranges
//   check_math powf_special        grid of special / boundary values
// Exit status 0 iff no mismatch (NaN compares equal to NaN).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <omp.h>
#include "../../hybrid9_amd/csrc/h9_math.h"

static const uint64_t E2[32] = H9M_EXP2F_TAB_INIT;
static const double L2[32] = H9M_POWF_LOG2_TAB_INIT;
static const h9m::Tabs T = {E2, L2};

static inline bool same(float a, float b) {
  if (isnan(a) && isnan(b)) return true;
  uint32_t ua, ub; memcpy(&ua, &a, 4); memcpy(&ub, &b, 4);
  return ua == ub;
}
static inline uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static inline float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// The speculative powf of the fast substep (powf_nx, without glibc's test
// of y): whenever it leaves `special` clear its result must be glibc's.
static inline bool fast_ok(float x, float y, float ref) {
  bool sp = false;
  const float f = h9m::powf_nx<false>(x, y, T, sp);
  return sp || same(f, ref);
}

// x, y drawn from a mix of: raw bit patterns, the hot path's ranges
// (bases in (0, 3e6], exponents in [-12, 25]) and integer-valued y.
static void pair(uint64_t i, uint64_t seed, float *x, float *y) {
  uint64_t a = mix(seed * 0x9E3779B97F4A7C15ULL + 2 * i), b = mix(seed + 2 * i + 1);
  float u = (float)(a >> 40) * (1.0f / 16777216.0f), v = (float)(b >> 40) * (1.0f / 16777216.0f);
  switch ((a >> 8) & 7) {
    case 0: *x = bits((uint32_t)a); *y = bits((uint32_t)b); break;
    case 1: *x = bits((uint32_t)a & 0x7fffffffu); *y = -12.0f + 37.0f * v; break;
    case 2: *x = 0.005f + u; *y = -12.0f + 37.0f * v; break;
    case 3: *x = u; *y = 2.0f + 22.0f * v; break;
    case 4: *x = 1.0f + 4.0f * u; *y = -(0.5f + 0.4f * v); break;
    case 5: *x = u * 3.0e6f; *y = 0.33333334f; break;
    case 6: *x = 2.8f; *y = -2000.0f * v; break;
    default: *x = bits((uint32_t)a); *y = (float)((int)(b % 41) - 20); break;
  }
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  long long bad = 0, n = 0;
  const char *mode = argv[1];
  if (!strcmp(mode, "expf_all") || !strcmp(mode, "expf_rand")) {
    const bool all = !strcmp(mode, "expf_all");
    const long long N = all ? (1LL << 32) : atoll(argv[2]);
    const uint64_t seed = all ? 0 : strtoull(argv[3], 0, 10);
#pragma omp parallel for reduction(+ : bad) schedule(static, 1 << 16)
    for (long long i = 0; i < N; i++) {
      const uint32_t u = all ? (uint32_t)i : (uint32_t)mix(seed + (uint64_t)i);
      const float x = bits(u);
      const float a = h9m::expf(x, T), b = ::expf(x);
      if (!same(a, b)) {
        if (bad < 5) fprintf(stderr, "expf(%a): h9 %a glibc %a\n", x, a, b);
        bad++;
      }
    }
    n = N;
  } else if (!strcmp(mode, "powf_rand")) {
    const long long N = atoll(argv[2]);
    const uint64_t seed = strtoull(argv[3], 0, 10);
#pragma omp parallel for reduction(+ : bad) schedule(static, 1 << 16)
    for (long long i = 0; i < N; i++) {
      float x, y;
      pair((uint64_t)i, seed, &x, &y);
      const float a = h9m::powf(x, y, T), b = ::powf(x, y);
      if (!same(a, b) || !fast_ok(x, y, b)) {
        if (bad < 5) fprintf(stderr, "powf(%a, %a): h9 %a glibc %a\n", x, y, a, b);
        bad++;
      }
    }
    n = N;
  } else if (!strcmp(mode, "powf_special")) {
    const float sv[] = {0.0f, -0.0f, 1.0f, -1.0f, 2.0f, -2.0f, 0.5f, -0.5f, 3.0f, -3.0f,
                        INFINITY, -INFINITY, NAN, bits(0x7fa00000u), bits(1u), bits(0x807fffffu),
                        bits(0x00800000u), 0x1p-126f, 0x1.fffffep127f, -0x1.fffffep127f, 126.0f,
                        -126.0f, 149.0f, -149.0f, 150.0f, -150.0f, 0.33333334f, 1.0000001f,
                        0.99999994f, 2.8f, 1e-38f, 1e38f, 23.0f, 24.0f, 25.0f, 0.1f, 1e-3f};
    const int ns = sizeof(sv) / sizeof(sv[0]);
    for (int i = 0; i < ns; i++)
      for (int j = 0; j < ns; j++) {
        const float a = h9m::powf(sv[i], sv[j], T), b = ::powf(sv[i], sv[j]);
        if (!same(a, b) || !fast_ok(sv[i], sv[j], b)) {
          if (bad < 10) fprintf(stderr, "powf(%a, %a): h9 %a glibc %a\n", sv[i], sv[j], a, b);
          bad++;
        }
        n++;
      }
    // boundary sweep around the under/overflow thresholds of 2^(y log2 x)
    for (int k = 0; k < 2000000; k++) {
      const float x = 0.5f + (float)k * 1e-7f, y = -148.0f - (float)(k % 4000) * 1e-3f;
      const float a = h9m::powf(x, -y, T), b = ::powf(x, -y);
      const float c = h9m::powf(2.0f, y * 1.01f, T), d = ::powf(2.0f, y * 1.01f);
      if (!same(a, b) || !same(c, d) || !fast_ok(x, -y, b) || !fast_ok(2.0f, y * 1.01f, d)) bad++;
      n += 2;
    }
  } else {
    return 2;
  }
  printf("%s: %lld checked, %lld mismatches\n", mode, n, bad);
  return bad ? 1 : 0;
}
