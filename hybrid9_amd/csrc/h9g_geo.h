// h9g_geo.h -- layer geometry policies (compile-time default and runtime).
//
// Geometry (INIT.f90:202-204,252-263): zi(0:L+1) from driver.txt, dz, zc,
// dt = 86400/NISURF.  Two policies share one interface:
//   GeoC<L, NS>  the reference's driver.txt layers (L=8) / the config-5
//                layers (L=10) and NISURF as compile-time constants: every
//                geometry value folds into instruction literals (no SGPR
//                pressure, no spills of uniform values to VGPR lanes).
//   GeoR<L>      any zi / NISURF, read from kernel arguments.
//
// Both also provide RN64(1/d) of the geometry divisors (thk, dt, the node
// spacings zc(I+1)-zc(I)) for the exact double-reciprocal division of
// h9g_step.h (MathFast::divk).  (An all-f32 x*RN32(1/d) + one correction
// step was evaluated first and rejected: over all 2^32 inputs it is wrong
// for about half of the divisors.  See DESIGN.md.)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define H9K_HD __host__ __device__ __forceinline__
#else
#define H9K_HD inline __attribute__((always_inline))
#endif

namespace h9k {

// --- compile-time layer sets --------------------------------------------
template <int L> struct ZiDefault;
template <> struct ZiDefault<8> {           // driver.txt:17-26
  static constexpr float zi[10] = {0.0f, 45.0f, 91.0f, 166.0f, 289.0f, 493.0f,
                                   829.0f, 1383.0f, 2296.0f, 5000.0f};
};
template <> struct ZiDefault<10> {          // config 5 (synth.ZI_L10)
  static constexpr float zi[12] = {0.0f, 18.0f, 45.0f, 91.0f, 166.0f, 289.0f, 493.0f,
                                   829.0f, 1383.0f, 2296.0f, 3500.0f, 5000.0f};
};

template <int L, int NS>
struct GeoC {
  static constexpr bool kConst = true;
  static constexpr float zi_(int i) { return ZiDefault<L>::zi[i]; }
  static constexpr float dz_(int i) { return zi_(i) - zi_(i - 1); }
  static constexpr float zc_(int i) { return zi_(i) - dz_(i) / 2.0f; }
  H9K_HD float zi(int i) const { return zi_(i); }
  H9K_HD float dz(int i) const { return dz_(i); }
  H9K_HD float zc(int i) const { return zc_(i); }
  H9K_HD float zim(int i) const { return zi_(i) / 1000.0f; }         // zi(I)/1000
  H9K_HD float thk(int i) const { return dz_(i) * 1000.0f / 1.0E3f; } // dz*rhow/1e3
  static constexpr float dt_ = 86400.0f / (float)NS;
  static constexpr float den_(int i) { return zc_(i + 1) - zc_(i); }
  H9K_HD float dt() const { return dt_; }
  H9K_HD float den(int i) const { return den_(i); }              // zc(I+1)-zc(I)
  H9K_HD double rthk(int i) const { return 1.0 / (double)(dz_(i) * 1000.0f / 1.0E3f); }
  H9K_HD double rdz(int i) const { return 1.0 / (double)dz_(i); }
  H9K_HD double rdt() const { return 1.0 / (double)dt_; }
  H9K_HD double rden(int i) const { return 1.0 / (double)den_(i); }
};

template <int L>
struct GeoR {
  static constexpr bool kConst = false;
  float zi_[L + 2], dz_[L + 1], zc_[L + 1], zim_[L + 1], thk_[L + 1], den_[L + 1];
  float dt_;
  double rthk_[L + 1], rdz_[L + 1], rden_[L + 1], rdt_;
  H9K_HD float zi(int i) const { return zi_[i]; }
  H9K_HD float dz(int i) const { return dz_[i]; }
  H9K_HD float zc(int i) const { return zc_[i]; }
  H9K_HD float zim(int i) const { return zim_[i]; }
  H9K_HD float thk(int i) const { return thk_[i]; }
  H9K_HD float dt() const { return dt_; }
  H9K_HD float den(int i) const { return den_[i]; }
  H9K_HD double rthk(int i) const { return rthk_[i]; }
  H9K_HD double rdz(int i) const { return rdz_[i]; }
  H9K_HD double rdt() const { return rdt_; }
  H9K_HD double rden(int i) const { return rden_[i]; }
};

template <int L>
inline GeoR<L> make_geo_r(const float *zi, int nisurf) {
  GeoR<L> g;
  for (int i = 0; i <= L + 1; i++) g.zi_[i] = zi[i];
  g.dz_[0] = g.zc_[0] = g.zim_[0] = g.thk_[0] = 0.0f;
  for (int i = 1; i <= L; i++) g.dz_[i] = g.zi_[i] - g.zi_[i - 1];
  for (int i = 1; i <= L; i++) g.zc_[i] = g.zi_[i] - g.dz_[i] / 2.0f;
  for (int i = 1; i <= L; i++) g.zim_[i] = g.zi_[i] / 1000.0f;
  for (int i = 1; i <= L; i++) g.thk_[i] = g.dz_[i] * 1000.0f / 1.0E3f;
  g.dt_ = 86400.0f / (float)nisurf;
  g.den_[0] = g.den_[L] = 0.0f;
  for (int i = 1; i < L; i++) g.den_[i] = g.zc_[i + 1] - g.zc_[i];
  g.rthk_[0] = g.rdz_[0] = g.rden_[0] = g.rden_[L] = 0.0;
  for (int i = 1; i <= L; i++) g.rthk_[i] = 1.0 / (double)g.thk_[i];
  for (int i = 1; i <= L; i++) g.rdz_[i] = 1.0 / (double)g.dz_[i];
  for (int i = 1; i < L; i++) g.rden_[i] = 1.0 / (double)g.den_[i];
  g.rdt_ = 1.0 / (double)g.dt_;
  return g;
}

}  // namespace h9k
