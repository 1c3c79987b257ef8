// Microbenchmarks of the instruction classes the year kernel is made of, on
// MI355X: cycles per wave64 instruction for dependent chains (latency) and
// for K independent chains (issue), at W waves per SIMD; glibc-exact powf
// (h9_math.h powf_nx) and the divisions the substep uses.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/ubench.hip -o tools/_build/ubench
// Output: one line per (test, chains, waves/SIMD): ns per launch and shader
// cycles per instruction per SIMD (s_memtime deltas, averaged over waves).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../hybrid9_amd/csrc/h9_math.h"

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                           \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

static const uint64_t h_e2[32] = H9M_EXP2F_TAB_INIT;
static const double h_l2[32] = H9M_POWF_LOG2_TAB_INIT;

enum { T_F32FMA, T_F64FMA, T_CVT, T_POWF, T_POWF_LDS, T_DIV, T_RCP64DIV, T_EXPF, T_N };
static const char *names[T_N] = {"f32_fma", "f64_fma", "cvt_f32_f64", "powf_nx(gtab)", "powf_nx(lds)",
                                 "div_ieee_f32", "div_rcp64", "expf_nx(lds)"};

template <int T, int K>
__global__ void __launch_bounds__(256) bench(int iters, float seed, float *out, unsigned long long *cyc,
                                             const uint64_t *ge2, const double *gl2) {
  __shared__ uint64_t se2[32];
  __shared__ double sl2[32];
  if (threadIdx.x < 32) {
    se2[threadIdx.x] = ge2[threadIdx.x];
    sl2[threadIdx.x] = gl2[threadIdx.x];
  }
  __syncthreads();
  const h9m::Tabs tg{ge2, gl2}, tl{se2, sl2};
  float a[K];
  double d[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    a[k] = seed + 0.001f * (threadIdx.x & 7) + 0.01f * k;
    d[k] = a[k];
  }
  bool sp = false;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < K; k++) {
      if constexpr (T == T_F32FMA) {
#pragma unroll
        for (int r = 0; r < 16; r++) a[k] = __builtin_fmaf(a[k], 0.999f, 0.001f);
      } else if constexpr (T == T_F64FMA) {
#pragma unroll
        for (int r = 0; r < 16; r++) d[k] = __builtin_fma(d[k], 0.999, 0.001);
      } else if constexpr (T == T_CVT) {
#pragma unroll
        for (int r = 0; r < 8; r++) a[k] = (float)((double)a[k] * 1.0000001);
      } else if constexpr (T == T_POWF) {
        a[k] = h9m::powf_nx<false>(a[k], 0.83f, tg, sp) * 0.5f + 0.6f;
      } else if constexpr (T == T_POWF_LDS) {
        a[k] = h9m::powf_nx<false>(a[k], 0.83f, tl, sp) * 0.5f + 0.6f;
      } else if constexpr (T == T_DIV) {
        a[k] = 1.3f / (a[k] + 0.7f);
      } else if constexpr (T == T_RCP64DIV) {
        const double r = __builtin_amdgcn_rcp(d[k]);
        const double e = __builtin_fma(-d[k], r, 1.0);
        const double r1 = __builtin_fma(e, r, r);
        a[k] = (float)(1.3 * r1);
        d[k] = (double)a[k] + 0.7;
      } else if constexpr (T == T_EXPF) {
        a[k] = h9m::expf_nx(-a[k], tl, sp) + 0.2f;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = sp ? 1.0f : 0.0f;
#pragma unroll
  for (int k = 0; k < K; k++) s += a[k] + (float)d[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

template <int T, int K>
static void run(int waves_per_simd, int iters, const uint64_t *e2, const double *l2) {
  // 256 CUs x 4 SIMDs: blocks of 4 waves, `waves_per_simd` blocks per CU
  const int blocks = 256 * waves_per_simd, threads = 256;
  float *out;
  unsigned long long *cyc;
  CHK(hipMalloc(&out, sizeof(float) * blocks * threads));
  CHK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  bench<T, K><<<blocks, threads>>>(iters / 8, 0.7f, out, cyc, e2, l2);   // warm-up
  CHK(hipEventRecord(e0));
  bench<T, K><<<blocks, threads>>>(iters, 0.7f, out, cyc, e2, l2);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * blocks * 4);
  CHK(hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost));
  double avg = 0;
  for (int i = 0; i < blocks * 4; i++) avg += (double)h[i];
  avg /= blocks * 4;
  // operations per wave: iters x K x (16 for fma, 8 for cvt, 1 otherwise)
  const double per = (T == T_F32FMA || T == T_F64FMA) ? 16 : (T == T_CVT ? 8 : 1);
  const double nops = (double)iters * K * per;
  // s_memtime ticks at a fixed 100 MHz on gfx9? report both: cycles per op per wave and per SIMD (x waves)
  printf("%-16s K=%d W=%d  %8.3f ms  wave-ticks/op %8.3f  SIMD-ns/op %8.4f\n", names[T], K, waves_per_simd, ms,
         avg / nops, ms * 1e6 / (nops * waves_per_simd));
  free(h);
  CHK(hipFree(out));
  CHK(hipFree(cyc));
}

template <int T>
static void sweep(int iters, const uint64_t *e2, const double *l2) {
  for (int w = 1; w <= 4; w++) {
    run<T, 1>(w, iters, e2, l2);
    run<T, 2>(w, iters, e2, l2);
    run<T, 4>(w, iters, e2, l2);
  }
}

int main(int argc, char **argv) {
  uint64_t *e2;
  double *l2;
  CHK(hipMalloc(&e2, sizeof(h_e2)));
  CHK(hipMalloc(&l2, sizeof(h_l2)));
  CHK(hipMemcpy(e2, h_e2, sizeof(h_e2), hipMemcpyHostToDevice));
  CHK(hipMemcpy(l2, h_l2, sizeof(h_l2), hipMemcpyHostToDevice));
  int clk = 0;
  CHK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
  printf("clock attr %d kHz\n", clk);
  sweep<T_F32FMA>(4000, e2, l2);
  sweep<T_F64FMA>(4000, e2, l2);
  sweep<T_CVT>(4000, e2, l2);
  sweep<T_POWF>(8000, e2, l2);
  sweep<T_POWF_LDS>(8000, e2, l2);
  sweep<T_EXPF>(8000, e2, l2);
  sweep<T_DIV>(20000, e2, l2);
  sweep<T_RCP64DIV>(20000, e2, l2);
  return 0;
}
