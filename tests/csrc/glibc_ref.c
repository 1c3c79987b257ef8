/* TEST INFRASTRUCTURE: vectorised calls of this machine's glibc expf/powf
 * (the functions the reference calls), for checking the device math. */
#include <math.h>
void glibc_expf_v(int n, const float *x, float *out) {
  for (int i = 0; i < n; i++) out[i] = expf(x[i]);
}
void glibc_powf_v(int n, const float *x, const float *y, float *out) {
  for (int i = 0; i < n; i++) out[i] = powf(x[i], y[i]);
}
