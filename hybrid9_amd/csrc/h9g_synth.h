// h9g_synth.h -- synthetic HYBRID9 inputs, host + device.
// Bit-identical to hybrid9_amd/synth.py (see its docstring for the why):
// a splitmix64 counter hash per (seed, stream, key) and a fixed sequence
// of float32 operations (no transcendentals).  Compile -ffp-contract=off.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define H9S_HD __host__ __device__ __forceinline__
#else
#define H9S_HD static inline
#endif

namespace h9s {

enum : uint64_t {
  S_THETA_S = 10, S_KS = 11, S_LAMBDA = 12, S_PSI = 13, S_FMAX = 14,
  S_WET = 15, S_PCELL = 16, S_FORCING = 100
};

H9S_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

H9S_HD float u01(uint64_t seed, uint64_t stream, uint64_t key) {
  const uint64_t z = seed * 0x9E3779B97F4A7C15ULL + stream * 0xD1B54A32D192ED03ULL + key;
  return (float)(uint32_t)(mix64(z) >> 40) * (1.0f / 16777216.0f);
}

H9S_HD float fmax32(float a, float b) { return a > b ? a : b; }   // np.maximum (no NaN)
H9S_HD float fmin32(float a, float b) { return a < b ? a : b; }

// per-layer parameters of cell gid, layer l (0-based): 0.8 x column draw
// + 0.2 x layer draw (see synth.make_params)
H9S_HD float mixu(uint64_t seed, uint64_t stream, uint64_t gid, int l) {
  return 0.8f * u01(seed, stream, gid * 16u + 15u) + 0.2f * u01(seed, stream, gid * 16u + (uint64_t)l);
}

H9S_HD void params(uint64_t seed, uint64_t gid, int l, float *theta_s, float *hksat,
                   float *bsw, float *psi_s) {
  *theta_s = 0.30f + 0.30f * mixu(seed, S_THETA_S, gid, l);
  const float mk = mixu(seed, S_KS, gid, l);
  const float ks = 0.5f + 487.5f * (mk * mk);
  *hksat = (10.0f * ks) / 86400.0f;
  float lam = 0.10f + 0.40f * mixu(seed, S_LAMBDA, gid, l);
  lam = fmax32(lam, 1.0e-8f);
  *bsw = 1.0f / lam;
  const float psi = -80.0f + 75.0f * mixu(seed, S_PSI, gid, l);
  *psi_s = 10.0f * psi;
}

H9S_HD float fmax_param(uint64_t seed, uint64_t gid) {
  return 0.1f + 0.5f * u01(seed, S_FMAX, gid);
}

// the 7 forcing values of cell (gid, lat) on global day d (0 = 1 Jan 1901)
H9S_HD void forcing(uint64_t seed, uint64_t gid, float lat, int64_t d, float out[7]) {
  const uint64_t key = ((uint64_t)d << 32) | gid;
  const float alat = lat < 0.0f ? -lat : lat;
  const float hs = lat >= 0.0f ? -1.0f : 1.0f;
  const float f = (float)(d % 365) / 365.0f;
  const float fm = f - 0.5f;
  const float tri = 4.0f * (fm < 0.0f ? -fm : fm) - 1.0f;
  const float season = hs * tri;
  const float wet = u01(seed, S_WET, gid);
  const float pcell = 65000.0f + 38000.0f * u01(seed, S_PCELL, gid);
  const float tmean = 303.0f - 0.55f * alat;
  const float amp = 0.25f * alat;
  float tas = tmean + amp * season + 6.0f * (u01(seed, S_FORCING + 0, key) - 0.5f);
  tas = fmin32(fmax32(tas, 240.0f), 315.0f);
  float rlds = 250.0f + 2.5f * (tas - 273.0f) + 60.0f * (u01(seed, S_FORCING + 1, key) - 0.5f);
  rlds = fmin32(fmax32(rlds, 150.0f), 450.0f);
  float rsds = 180.0f + 100.0f * season * (alat / 80.0f) - alat +
               120.0f * (u01(seed, S_FORCING + 2, key) - 0.5f);
  rsds = fmin32(fmax32(rsds, 0.0f), 350.0f);
  const float warm = fmax32(0.0f, (tas - 240.0f) / 70.0f);
  const float huss = 1.0e-4f + 0.015f * u01(seed, S_FORCING + 3, key) * warm;
  const float ps = pcell + 800.0f * (u01(seed, S_FORCING + 4, key) - 0.5f);
  const float prain = 0.15f + 0.5f * wet;
  const float rate = 2.0e-4f * wet + 2.0e-5f;
  const float u2 = u01(seed, S_FORCING + 15, key);
  const float pr = (u01(seed, S_FORCING + 5, key) < prain) ? 3.0f * rate * (u2 * u2) : 0.0f;
  const float rhs = 10.0f + 90.0f * u01(seed, S_FORCING + 6, key);
  out[0] = tas; out[1] = rlds; out[2] = rsds; out[3] = huss;
  out[4] = ps; out[5] = pr; out[6] = rhs;
}

}  // namespace h9s
