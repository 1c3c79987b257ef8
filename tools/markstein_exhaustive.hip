// Exhaustive proof of the conductivity phase's s1 quotient (h9g_pair.h
// hk_fast, DESIGN.md §3 "Interface saturation by Markstein's correction"):
//
//   y = RN(1/b), q0 = RN(a y), e = RN(-b q0 + a), q1 = RN(e y + q0)
//
// equals the IEEE quotient RN(a/b) for EVERY pair of float significands,
// a, b in [1, 2): 2^46 pairs, about 20 s on one MI355X.
//
// Why significands suffice.  hk_fast sends any a or b outside [2^-60, 2^60)
// to the exact path.  Inside it, scaling a by 2^i and b by 2^j scales y by
// 2^-j, q0 and q1 by 2^(i-j) and e by 2^i, and no value leaves the normal
// range: |q| < 2^121, and e, when not zero, is a multiple of
// ulp(a) * ulp(b) / 2 >= 2^-107 (e = a - b q0 exactly once q1 is right; an
// fma never rounds its product, so a subnormal e*y is harmless).  Every
// rounding therefore happens at the same relative position as for the
// significands, and the result for (a 2^i, b 2^j) is the significand pair's
// result times 2^(i-j).  (ADVICE r03 pointed out that q0 = RN(a RN(1/b)) is
// not faithful by the textbook bound alone, so the sampling in
// tools/markstein_check.c did not prove the rule; this sweep does.)
//
// The control run uses y one ulp above RN(1/b) on a slice of b and must
// find mismatches (the check can fail).
//
// Build (here, no GPU needed):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/_build/markstein_exhaustive tools/markstein_exhaustive.hip
// Run (GPU box): tools/_build/markstein_exhaustive [b_lo b_hi [mode]]
// (significand indices of b, default the full 0 .. 2^23; tests/test_math.py
// runs a slice; mode 1 checks the refined hardware reciprocal instead)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define NA (1u << 23)          // a significands
#define ASPLIT 64              // threads per b
#define BCHUNK 8192            // b significands per launch: 8,192 waves

// mode 0: y = RN(1/b) (hk_fast's stored PF_ITS).  mode 1 (round 4, a
// candidate for runtime divisors): y = the hardware estimate v_rcp_f32(b)
// refined by one Newton step, y = fma(fma(-b, r, 1), r, r), then the same
// correction of q0 = RN(a y).
__global__ void __launch_bounds__(256) mk_kernel(uint32_t b0, uint32_t bend, int yoff, int mode, unsigned *cnt,
                                                 uint32_t *first) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t mb = b0 + t / ASPLIT;
  if (mb >= bend) return;
  const float b = __uint_as_float(0x3f800000u | mb);
  float y;
  if (mode == 1) {
    const float r = __builtin_amdgcn_rcpf(b);
    y = __builtin_fmaf(__builtin_fmaf(-b, r, 1.0f), r, r);
  } else {
    y = 1.0f / b;
  }
  y = __uint_as_float(__float_as_uint(y) + yoff);
  const uint32_t a0 = (t % ASPLIT) * (NA / ASPLIT);
  unsigned bad = 0;
  uint32_t fa = 0xffffffffu;
  for (uint32_t ma = a0; ma < a0 + NA / ASPLIT; ma++) {
    const float a = __uint_as_float(0x3f800000u | ma);
    const float q0 = a * y;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
    const float r = a / b;                         // correctly rounded (no fast-math)
    const bool ne = __float_as_uint(q1) != __float_as_uint(r);
    bad += ne ? 1u : 0u;
    fa = (ne && fa == 0xffffffffu) ? ma : fa;
  }
  cnt[t] = bad;                                    // vector stores only
  first[t] = fa;
}

// Mode 1 checks significands only, which is complete if the hardware
// reciprocal is scale-invariant: v_rcp_f32(b 2^k) = v_rcp_f32(b) 2^-k for
// every b significand and every k with b 2^k in [2^-60, 2^60), and odd in b
// (the corrections are exact under a sign change of a or b).  Counted here.
__global__ void __launch_bounds__(256) rcp_scale_kernel(unsigned *cnt) {
  const uint32_t mb = blockIdx.x * blockDim.x + threadIdx.x;
  if (mb >= NA) return;
  const float b = __uint_as_float(0x3f800000u | mb);
  const uint32_t r = __float_as_uint(__builtin_amdgcn_rcpf(b));
  unsigned bad = 0;
  for (int k = -60; k < 60; k++) {
    const float bk = __uint_as_float((uint32_t)((int)__float_as_uint(b) + (k << 23)));
    const uint32_t rk = __float_as_uint(__builtin_amdgcn_rcpf(bk));
    bad += rk != (uint32_t)((int)r - (k << 23)) ? 1u : 0u;
    // and sign symmetry, v_rcp_f32(-b) = -v_rcp_f32(b) (mk_div takes signed operands)
    bad += __float_as_uint(__builtin_amdgcn_rcpf(-bk)) != (rk ^ 0x80000000u) ? 1u : 0u;
  }
  cnt[mb] = bad;
}

static int run(uint32_t blo, uint32_t bhi, int yoff, int mode, unsigned long long *total, long long *ex_a,
               long long *ex_b) {
  const uint32_t nthr = BCHUNK * ASPLIT;
  unsigned *d_cnt = nullptr;
  uint32_t *d_first = nullptr;
  if (hipMalloc(&d_cnt, sizeof(unsigned) * nthr) != hipSuccess) return 1;
  if (hipMalloc(&d_first, sizeof(uint32_t) * nthr) != hipSuccess) return 1;
  unsigned *h_cnt = (unsigned *)malloc(sizeof(unsigned) * nthr);
  uint32_t *h_first = (uint32_t *)malloc(sizeof(uint32_t) * nthr);
  *total = 0;
  *ex_a = *ex_b = -1;
  int launches = 0;
  for (uint32_t b0 = blo; b0 < bhi; b0 += BCHUNK) {
    const uint32_t bend = b0 + BCHUNK < bhi ? b0 + BCHUNK : bhi;
    const uint32_t n = (bend - b0) * ASPLIT;
    mk_kernel<<<(n + 255) / 256, 256>>>(b0, bend, yoff, mode, d_cnt, d_first);
    if (hipGetLastError() != hipSuccess) return 1;
    if (hipMemcpy(h_cnt, d_cnt, sizeof(unsigned) * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    if (hipMemcpy(h_first, d_first, sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (uint32_t i = 0; i < n; i++) {
      *total += h_cnt[i];
      if (h_cnt[i] && *ex_a < 0) {
        *ex_a = h_first[i];
        *ex_b = b0 + i / ASPLIT;
      }
    }
    if (++launches % 128 == 0) {
      printf("  b significands %u .. %u: %llu mismatches so far\n", blo, bend, *total);
      fflush(stdout);
    }
  }
  hipFree(d_cnt);
  hipFree(d_first);
  free(h_cnt);
  free(h_first);
  return 0;
}

int main(int argc, char **argv) {
  const uint32_t blo = argc > 2 ? (uint32_t)strtoul(argv[1], nullptr, 0) : 0u;
  const uint32_t bhi = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 0) : NA;
  const int mode = argc > 3 ? atoi(argv[3]) : 0;
  if (blo >= bhi || bhi > NA || mode < 0 || mode > 1) {
    fprintf(stderr, "usage: %s [b_lo b_hi [mode]]  (0 <= b_lo < b_hi <= 2^23; mode 0 RN(1/b), 1 refined rcp)\n",
            argv[0]);
    return 2;
  }
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  unsigned long long bad = 0, ctl = 0;
  long long xa, xb, ca, cb;
  hipEventRecord(e0, 0);
  if (run(blo, bhi, 0, mode, &bad, &xa, &xb)) { fprintf(stderr, "HIP failure\n"); return 3; }
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const uint32_t cend = blo + 4096 < bhi ? blo + 4096 : bhi;   // control slice
  if (run(blo, cend, 1, mode, &ctl, &ca, &cb)) { fprintf(stderr, "HIP failure\n"); return 3; }
  unsigned long long rcp_bad = 0;
  if (mode == 1) {                     // scale invariance of v_rcp_f32 over the guarded range
    unsigned *d = nullptr;
    if (hipMalloc(&d, sizeof(unsigned) * NA) != hipSuccess) return 3;
    rcp_scale_kernel<<<NA / 256, 256>>>(d);
    unsigned *hb = (unsigned *)malloc(sizeof(unsigned) * NA);
    if (hipMemcpy(hb, d, sizeof(unsigned) * NA, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    for (uint32_t i = 0; i < NA; i++) rcp_bad += hb[i];
    free(hb);
    (void)hipFree(d);
  }
  const double pairs = (double)(bhi - blo) * NA;
  printf("markstein exhaustive (%s): b significands [%u, %u) x all 2^23 a significands = %.4g pairs, %.1f s\n",
         mode ? "y = v_rcp_f32(b) + one Newton step" : "y = RN(1/b)", blo, bhi, pairs, ms / 1e3);
  printf("  mismatches against the IEEE quotient: %llu", bad);
  if (bad) printf(" (first: a = 1 + %lld/2^23, b = 1 + %lld/2^23)", xa, xb);
  printf("\n  control (y one ulp above RN(1/b), b in [%u, %u)): %llu mismatches (must be > 0)\n", blo, cend, ctl);
  if (mode == 1)
    printf("  v_rcp_f32 scale invariance, every b significand x 2^k, k in [-60, 60): %llu exceptions (must be 0)\n",
           rcp_bad);
  return (bad == 0 && ctl > 0 && rcp_bad == 0) ? 0 : 1;
}
