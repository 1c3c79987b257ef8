// Issue cost of single VALU instruction classes on MI355X (gfx950): each
// lane runs 8 independent chains of one instruction (inline asm, so the
// compiler neither packs nor reorders them) at W = 1..4 waves per SIMD.
// Prints shader-clock ticks per instruction per SIMD (s_memtime deltas /
// W) and the clock the chip held (ticks / wall time).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_issue.hip -o tools/_build/ubench_issue
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                   \
  do {                                                           \
    hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));    \
      exit(1);                                                   \
    }                                                            \
  } while (0)

enum { I_FMA32, I_FMA64, I_MUL64, I_CVT64_32, I_CVT32_64, I_CNDMASK, I_ADDU32, I_LSHLADD64, I_RCP64, I_RCP32,
       I_PKFMA32, I_CMPCLASS, I_CND_SGPR, I_CMP_CND, I_MAXF32, I_DPP, I_CND_ONE, I_N };
static const char *names[I_N] = {"v_fma_f32", "v_fma_f64", "v_mul_f64", "v_cvt_f64_f32", "v_cvt_f32_f64",
                                 "v_cndmask_b32", "v_add_u32", "v_lshl_add_u64", "v_rcp_f64", "v_rcp_f32",
                                 "v_pk_fma_f32", "v_cmp_class_f32", "v_cndmask(s[0:1])", "v_cmp+v_cndmask", "v_max_f32",
                                 "v_mov_dpp", "1 cndmask/8 add"};

#define R8(X) X X X X X X X X

template <int I>
__global__ void __launch_bounds__(256) kern(int iters, unsigned long long *cyc, float *out) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
    if constexpr (I == I_FMA32) {
      asm volatile(R8("v_fma_f32 %0, %0, %0, %0\n v_fma_f32 %1, %1, %1, %1\n v_fma_f32 %2, %2, %2, %2\n "
                      "v_fma_f32 %3, %3, %3, %3\n v_fma_f32 %4, %4, %4, %4\n v_fma_f32 %5, %5, %5, %5\n "
                      "v_fma_f32 %6, %6, %6, %6\n v_fma_f32 %7, %7, %7, %7\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (I == I_FMA64) {
      asm volatile(R8("v_fma_f64 %0, %0, %0, %0\n v_fma_f64 %1, %1, %1, %1\n v_fma_f64 %2, %2, %2, %2\n "
                      "v_fma_f64 %3, %3, %3, %3\n v_fma_f64 %4, %4, %4, %4\n v_fma_f64 %5, %5, %5, %5\n "
                      "v_fma_f64 %6, %6, %6, %6\n v_fma_f64 %7, %7, %7, %7\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
    } else if constexpr (I == I_MUL64) {
      asm volatile(R8("v_mul_f64 %0, %0, %0\n v_mul_f64 %1, %1, %1\n v_mul_f64 %2, %2, %2\n "
                      "v_mul_f64 %3, %3, %3\n v_mul_f64 %4, %4, %4\n v_mul_f64 %5, %5, %5\n "
                      "v_mul_f64 %6, %6, %6\n v_mul_f64 %7, %7, %7\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
    } else if constexpr (I == I_CVT64_32) {
      asm volatile(R8("v_cvt_f64_f32 %0, %8\n v_cvt_f64_f32 %1, %9\n v_cvt_f64_f32 %2, %10\n "
                      "v_cvt_f64_f32 %3, %11\n v_cvt_f64_f32 %4, %12\n v_cvt_f64_f32 %5, %13\n "
                      "v_cvt_f64_f32 %6, %14\n v_cvt_f64_f32 %7, %15\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7)
                   : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7));
    } else if constexpr (I == I_CVT32_64) {
      asm volatile(R8("v_cvt_f32_f64 %0, %8\n v_cvt_f32_f64 %1, %9\n v_cvt_f32_f64 %2, %10\n "
                      "v_cvt_f32_f64 %3, %11\n v_cvt_f32_f64 %4, %12\n v_cvt_f32_f64 %5, %13\n "
                      "v_cvt_f32_f64 %6, %14\n v_cvt_f32_f64 %7, %15\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                   : "v"(d0), "v"(d1), "v"(d2), "v"(d3), "v"(d4), "v"(d5), "v"(d6), "v"(d7));
    } else if constexpr (I == I_CNDMASK) {
      asm volatile(R8("v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %2, vcc\n "
                      "v_cndmask_b32 %2, %2, %3, vcc\n v_cndmask_b32 %3, %3, %4, vcc\n "
                      "v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %5, %5, %6, vcc\n "
                      "v_cndmask_b32 %6, %6, %7, vcc\n v_cndmask_b32 %7, %7, %0, vcc\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)::"vcc");
    } else if constexpr (I == I_ADDU32) {
      asm volatile(R8("v_add_u32 %0, %0, %1\n v_add_u32 %1, %1, %2\n v_add_u32 %2, %2, %3\n "
                      "v_add_u32 %3, %3, %4\n v_add_u32 %4, %4, %5\n v_add_u32 %5, %5, %6\n "
                      "v_add_u32 %6, %6, %7\n v_add_u32 %7, %7, %0\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (I == I_LSHLADD64) {
      asm volatile(R8("v_lshl_add_u64 %0, %0, 3, %0\n v_lshl_add_u64 %1, %1, 3, %1\n "
                      "v_lshl_add_u64 %2, %2, 3, %2\n v_lshl_add_u64 %3, %3, 3, %3\n "
                      "v_lshl_add_u64 %4, %4, 3, %4\n v_lshl_add_u64 %5, %5, 3, %5\n "
                      "v_lshl_add_u64 %6, %6, 3, %6\n v_lshl_add_u64 %7, %7, 3, %7\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
    } else if constexpr (I == I_RCP64) {
      asm volatile(R8("v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n "
                      "v_rcp_f64 %4, %4\n v_rcp_f64 %5, %5\n v_rcp_f64 %6, %6\n v_rcp_f64 %7, %7\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
    } else if constexpr (I == I_RCP32) {
      asm volatile(R8("v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n "
                      "v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (I == I_PKFMA32) {
      asm volatile(R8("v_pk_fma_f32 %0, %0, %0, %0\n v_pk_fma_f32 %1, %1, %1, %1\n "
                      "v_pk_fma_f32 %2, %2, %2, %2\n v_pk_fma_f32 %3, %3, %3, %3\n "
                      "v_pk_fma_f32 %4, %4, %4, %4\n v_pk_fma_f32 %5, %5, %5, %5\n "
                      "v_pk_fma_f32 %6, %6, %6, %6\n v_pk_fma_f32 %7, %7, %7, %7\n")
                   : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3), "+v"(d4), "+v"(d5), "+v"(d6), "+v"(d7));
    } else if constexpr (I == I_CMPCLASS) {
      asm volatile(R8("v_cmp_class_f32 vcc, %0, %1\n v_cmp_class_f32 vcc, %1, %2\n "
                      "v_cmp_class_f32 vcc, %2, %3\n v_cmp_class_f32 vcc, %3, %4\n "
                      "v_cmp_class_f32 vcc, %4, %5\n v_cmp_class_f32 vcc, %5, %6\n "
                      "v_cmp_class_f32 vcc, %6, %7\n v_cmp_class_f32 vcc, %7, %0\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)::"vcc");
    } else if constexpr (I == I_CND_SGPR) {
      asm volatile("s_mov_b64 s[20:21], exec\n" R8("v_cndmask_b32_e64 %0, %0, %1, s[20:21]\n v_cndmask_b32_e64 %1, %1, %2, s[20:21]\n "
                      "v_cndmask_b32_e64 %2, %2, %3, s[20:21]\n v_cndmask_b32_e64 %3, %3, %4, s[20:21]\n "
                      "v_cndmask_b32_e64 %4, %4, %5, s[20:21]\n v_cndmask_b32_e64 %5, %5, %6, s[20:21]\n "
                      "v_cndmask_b32_e64 %6, %6, %7, s[20:21]\n v_cndmask_b32_e64 %7, %7, %0, s[20:21]\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)::"s20", "s21");
    } else if constexpr (I == I_CMP_CND) {
      asm volatile(R8("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n v_cmp_gt_f32 vcc, %2, %3\n "
                      "v_cndmask_b32 %2, %2, %3, vcc\n v_cmp_gt_f32 vcc, %4, %5\n v_cndmask_b32 %4, %4, %5, vcc\n "
                      "v_cmp_gt_f32 vcc, %6, %7\n v_cndmask_b32 %6, %6, %7, vcc\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)::"vcc");
    } else if constexpr (I == I_MAXF32) {
      asm volatile(R8("v_max_f32 %0, %0, %1\n v_max_f32 %1, %1, %2\n v_max_f32 %2, %2, %3\n "
                      "v_max_f32 %3, %3, %4\n v_max_f32 %4, %4, %5\n v_max_f32 %5, %5, %6\n "
                      "v_max_f32 %6, %6, %7\n v_max_f32 %7, %7, %0\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (I == I_DPP) {
      asm volatile(R8("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %2, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %4, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %5, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %6, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n "
                      "v_mov_b32_dpp %7, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if constexpr (I == I_CND_ONE) {
      asm volatile(R8("v_cndmask_b32 %0, %0, %1, vcc\n v_add_u32 %1, %1, %2\n v_add_u32 %2, %2, %3\n "
                      "v_add_u32 %3, %3, %4\n v_add_u32 %4, %4, %5\n v_add_u32 %5, %5, %6\n "
                      "v_add_u32 %6, %6, %7\n v_add_u32 %7, %7, %0\n")
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)::"vcc");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int I>
static void run(int W, int iters) {
  const int blocks = 256 * W;
  unsigned long long *cyc;
  float *out;
  CHK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4));
  CHK(hipMalloc(&out, sizeof(float) * blocks * 256));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  kern<I><<<blocks, 256>>>(iters, cyc, out);
  CHK(hipEventRecord(e0));
  kern<I><<<blocks, 256>>>(iters, cyc, out);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * blocks * 4);
  CHK(hipMemcpy(h, cyc, sizeof(unsigned long long) * blocks * 4, hipMemcpyDeviceToHost));
  double avg = 0;
  for (int i = 0; i < blocks * 4; i++) avg += (double)h[i];
  avg /= blocks * 4;
  const double n = (double)iters * 64;
  printf("%-16s W=%d  ticks/instr/SIMD %6.3f  (per wave %6.3f)  clock %.2f GHz  %.3f ms\n", names[I], W, avg / n / W,
         avg / n, avg / (ms * 1e6), ms);
  free(h);
  CHK(hipFree(cyc));
  CHK(hipFree(out));
}

template <int I>
static void sweep() {
  for (int W = 1; W <= 4; W++) run<I>(W, 20000);
}

int main(int argc, char **argv) {
  if (argc > 1) {
    sweep<I_CNDMASK>();
    sweep<I_CND_SGPR>();
    sweep<I_CMP_CND>();
    sweep<I_MAXF32>();
    sweep<I_DPP>();
    sweep<I_CND_ONE>();
    sweep<I_ADDU32>();
    return 0;
  }
  sweep<I_FMA32>();
  sweep<I_PKFMA32>();
  sweep<I_FMA64>();
  sweep<I_MUL64>();
  sweep<I_CVT64_32>();
  sweep<I_CVT32_64>();
  sweep<I_CNDMASK>();
  sweep<I_ADDU32>();
  sweep<I_LSHLADD64>();
  sweep<I_CMPCLASS>();
  sweep<I_RCP32>();
  sweep<I_RCP64>();
  return 0;
}
