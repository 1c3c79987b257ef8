// Accuracy of the gfx950 v_rcp_f64 estimate on every positive finite float
// divisor d (converted to double), and of one and two Newton steps from it
// (recip64, h9g_step.h).  Prints max |1 - d r| for each.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o tools/_rcp_probe tools/rcp_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ unsigned long long g_max[3];

__global__ void probe(uint32_t base, uint32_t count) {
  unsigned long long m0 = 0, m1 = 0, m2 = 0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += gridDim.x * blockDim.x) {
    const uint32_t u = base + k;
    const double d = (double)__builtin_bit_cast(float, u);
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    m0 = max(m0, (unsigned long long)__builtin_bit_cast(uint64_t, __builtin_fabs(e)));
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    m1 = max(m1, (unsigned long long)__builtin_bit_cast(uint64_t, __builtin_fabs(e)));
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    m2 = max(m2, (unsigned long long)__builtin_bit_cast(uint64_t, __builtin_fabs(e)));
  }
  atomicMax(&g_max[0], m0);
  atomicMax(&g_max[1], m1);
  atomicMax(&g_max[2], m2);
}

int main() {
  const uint32_t lo = 0x00000001u, hi = 0x7f7fffffu;   // positive subnormal .. largest finite
  unsigned long long z[3] = {0, 0, 0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_max), z, sizeof z) != hipSuccess) return 1;
  const uint32_t chunk = 1u << 28;
  for (uint64_t b = lo; b <= hi; b += chunk) {
    const uint32_t cnt = (uint32_t)((hi - b + 1) < chunk ? (hi - b + 1) : chunk);
    probe<<<8192, 256>>>((uint32_t)b, cnt);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
  }
  if (hipMemcpyFromSymbol(z, HIP_SYMBOL(g_max), sizeof z) != hipSuccess) return 3;
  const char *nm[3] = {"v_rcp_f64", "+1 Newton step", "+2 Newton steps"};
  for (int i = 0; i < 3; i++) {
    const double v = __builtin_bit_cast(double, z[i]);
    int ex = 0;
    frexp(v, &ex);
    printf("%-16s max |1 - d r| = %.6e (< 2^%d)\n", nm[i], v, ex);
  }
  return 0;
}
