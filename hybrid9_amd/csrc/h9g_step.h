// h9g_step.h -- per-cell HYDROLOGY substep and daily GROW update, written
// once for gfx950 device code and for a host build used only by the CPU
// test that pins this code against the oracle (tests/test_kernel_host.py).
//
//   hydrology_step  /root/reference/SOURCE/HYDROLOGY.f90:141-1283
//   grow_day        /root/reference/SOURCE/GROW.f90:55-201
//   day_consts      the parts of HYDROLOGY.f90:232-389 that depend only on
//                   the day's forcing and on LAI / LAI_litter (which only
//                   GROW changes, once a day): computed once per cell-day
//   CellInv         expressions of the soil parameters alone (e.g.
//                   one-one/bsw), computed once per cell and launch
//
// Bit-exactness rules (pinned by tests/test_gpu_parity.py and
// tests/test_kernel_host.py against the reference goldens and the oracle):
//   * float32 throughout, -ffp-contract=off, correctly rounded division;
//   * every reference expression keeps its Fortran left-to-right operation
//     order; a hoisted sub-expression is exactly one the reference
//     evaluates as a unit (a parenthesised term or a left-to-right prefix);
//   * MIN(a,b) = a<b?a:b, MAX(a,b) = a>b?a:b (flang's compare+select);
//   * EXP / real powers -> glibc-2.35-exact h9m::expf / h9m::powf.
// Layer arrays are 1-based (index 0 unused) and fully unrolled over the
// compile-time layer count L, so per-layer values live in registers; the
// data-dependent index jwt is resolved with unrolled compare/select chains.
//
// Speculate-then-verify: hydrology_step is instantiated with a math policy.
// MathFast runs glibc's main path only (h9m::*_nx, straight-line code) and
// records whether any input would have taken a special path; the caller
// then re-runs that lane's substep from the saved state with MathExact
// (full glibc special-case handling).  Results are therefore bit-identical
// to MathExact for every input, while the common case carries no per-call
// branches.
#pragma once
#include "h9_math.h"
#include "h9g_geo.h"

namespace h9k {

constexpr float zero = 0.0f, one = 1.0f;
constexpr float rhow = 1000.0f;
constexpr float gasc = 8.314510f;
constexpr float rgas = 0x1.1f0c7cp+8f;     // 1000*gasc/mair (SHARED.f90:335)
constexpr float deltx = 0x1.3738bcp-1f;    // bymrat - one   (SHARED.f90:351)
constexpr float stbo = 5.67E-8f;
constexpr float tf = 273.16f;
constexpr float smpmin = -1.0E8f;
constexpr float cp = 1010.0f;              // HYDROLOGY.f90:35
constexpr float watmin = 0.01f;            // HYDROLOGY.f90:135
constexpr float sla1 = 23.0E-3f;           // INIT.f90:154
constexpr float log_0p1 = -0x1.26bb1cp+1f; // LOG(0.1) as folded by flang

H9K_HD float MAXF(float a, float b) { return a > b ? a : b; }
H9K_HD float MINF(float a, float b) { return a < b ? a : b; }
H9K_HD float absf(float a) { return __builtin_fabsf(a); }

// Scheduling fence: stops the machine scheduler from interleaving the
// unrolled per-layer bodies (each a few powf with double-precision
// temporaries), which otherwise multiplies the live register set by L.
H9K_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// Makes a value opaque to the optimiser at this point, so address
// arithmetic derived from it is recomputed after it instead of being kept
// live (as 64-bit per-lane pointers) across the year loop.
template <class T>
H9K_HD void opaque(T &x) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(x));
#else
  (void)x;
#endif
}

// true if p holds for any active lane of the wave (host: p itself)
H9K_HD bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ballot_w64(p) != 0;
#else
  return p;
#endif
}

// ------------------------------------------------------------ math policies
H9K_HD bool is_subnormal(float q) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_classf(q, 0x090);     // -denormal | +denormal
#else
  const uint32_t u = __builtin_bit_cast(uint32_t, q) & 0x7fffffffu;
  return u != 0 && u < 0x00800000u;
#endif
}

// Reciprocal of a float divisor in double, |r - 1/d| <= 1.2 * 2^-53 |1/d|:
// hardware estimate + two Newton steps (each squares the error and adds
// <= 2^-53; two steps suffice from any estimate within 2^-14).
H9K_HD double recip64(float d) {
  const double dd = (double)d;
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(dd);
#else
  double r = 1.0 / dd;
#endif
  double e = __builtin_fma(-dd, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-dd, r, 1.0);
  r = __builtin_fma(r, e, r);
  return r;
}

// Division policy.  MathExact divides; MathFast computes RN32(RN64(x * r))
// from a double reciprocal r of the divisor d with relative error
// <= 2^-52.  That equals the correctly rounded x/d whenever the result is
// a normal float: a float quotient that is not itself a rounding midpoint
// lies at least 2^-49 (relative) away from every midpoint (x and d have
// 24-bit significands), and a normal-range quotient is never exactly a
// midpoint.  Subnormal results flag the substep for the exact re-run.
struct MathExact {
  static constexpr bool kExact = true;
  h9m::Tabs T;
  H9K_HD float expf(float x) { return h9m::expf(x, T); }
  H9K_HD float powf(float x, float y) { return h9m::powf(x, y, T); }
  H9K_HD float div(float x, float d, double) { return x / d; }
};
struct MathFast {
  static constexpr bool kExact = false;
  h9m::Tabs T;
  bool special;
  H9K_HD float expf(float x) { return h9m::expf_nx(x, T, special); }
  H9K_HD float powf(float x, float y) { return h9m::powf_nx(x, y, T, special); }
  H9K_HD float div(float x, float, double r) {
    const float q = (float)((double)x * r);
    special |= is_subnormal(q);
    return q;
  }
};

// ------------------------------------------------------------ cell data
// Per-cell values that are read (not updated) by the substep live in a
// "cell store": soil parameters, parameter-only sub-expressions (computed
// once per cell and launch, exact as the reference evaluates them),
// rootr, the day's constants and the substep rollback area.  On the device the store is the
// lane's column of a [field][64] LDS block; on the host (test build) it is
// a plain array.  Layout in floats:
// day-constant fields (HYDROLOGY.f90:232-389 terms fixed within a day)
enum : int {
  D_FORC = 0, D_DESAT, D_GAMMA, D_VDD, D_DG, D_RHOCP, D_A1, D_X, D_LAI2, D_PW28, D_RSCMIN,
  D_RAC, D_RAA, D_RAS, D_RAARAC, D_RAARAS, D_NUMC, D_NUMS, D_RA, D_DGRAS, D_DGRAC, D_DRR,
  D_DRG, D_RL, D_LIT, D_LIT1000, D_OK, D_N
};
static_assert(D_N == 27, "day-constant block size");
template <int L>
struct Lay {
  enum : int {
    TS = 0, HKS = L, BSW = 2 * L, PSI = 3 * L, FMAX = 4 * L,     // SHARED.f90:398-446
    NINVB = 4 * L + 1,    // -one/bsw  (HYDROLOGY.f90:939,964,980,1034,1079); the
                          // reference's one-one/bsw (:534,550,580) is one+NINVB exactly
    ITS = 5 * L + 1,      // one/(ts(I)+ts(I+1))    (:620-621)
    PTE = 6 * L + 1,      // psi*ts/(one-one/bsw)   (:535-536,554-555,581-582)
    C3 = 7 * L + 1,       // pte/(zi(I)-zi(I-1))    (:554-556)
    MH3 = 8 * L + 1,      // MINVAL(hksat(1:3))     (:458)
    TSDZ1 = 8 * L + 2,    // MAX(zero, theta_s(1)*dz(1))  (:1145-1147)
    ROOTR = 8 * L + 3,    // rootr_col(1..L), updated daily by GROW
    DAY = 9 * L + 3,      // D_* fields
    // substep rollback / exact-path exchange area
    SV_H2O = DAY + D_N, SV_SMP = SV_H2O + L, SV_ZWT = SV_SMP + L, SV_WA, SV_RNF, SV_ERR,
    N
  };
};

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) float lds_float;
// Device cell store: column `lane` of a [Lay<L>::N][64] LDS block.  The
// base pointer is "laundered" (made opaque to the optimiser) at phase
// boundaries so loads stay next to their uses instead of being hoisted
// into long-lived registers.
template <int L>
struct CellStore {
  lds_float *b;
  __device__ __forceinline__ float get(int f) const { return b[f * 64]; }
  __device__ __forceinline__ void set(int f, float x) const { b[f * 64] = x; }
  __device__ __forceinline__ void launder() { asm volatile("" : "+v"(b)); }
  __device__ __forceinline__ float day(int f) const { return get(Lay<L>::DAY + f); }
  __device__ __forceinline__ void set_day(int f, float x) const { set(Lay<L>::DAY + f, x); }
  __device__ __forceinline__ float root(int i) const { return get(Lay<L>::ROOTR + i - 1); }
  __device__ __forceinline__ void set_root(int i, float x) const { set(Lay<L>::ROOTR + i - 1, x); }
};
#else
typedef float lds_float;
template <int L>
struct CellStore {
  float *b;
  inline float get(int f) const { return b[f]; }
  inline void set(int f, float x) const { b[f] = x; }
  inline void launder() {}
  inline float day(int f) const { return get(Lay<L>::DAY + f); }
  inline void set_day(int f, float x) const { set(Lay<L>::DAY + f, x); }
  inline float root(int i) const { return get(Lay<L>::ROOTR + i - 1); }
  inline void set_root(int i, float x) const { set(Lay<L>::ROOTR + i - 1, x); }
};
#endif

template <int L>
struct St {            // persistent per-cell state (SHARED.f90), in registers
  float h2o[L + 1], smp[L + 1];
  float zwt, wa, LAI, LAI_litter, pm, pfm, plen, rdepth;
};

struct Day {           // HYBRID9.f90:168-184 + forcing read by HYDROLOGY
  float tak, rh, Rnet, PAR, forc_rain, lamb, huss, ps;
};

// Fill the parameter-derived fields of the store (params already stored).
template <int L, class G>
H9K_HD void cell_inv(const G &g, const CellStore<L> &cs) {
  typedef Lay<L> Y;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    const int ip = (L < i + 1) ? L : i + 1;
    const float ts = cs.get(Y::TS + i - 1), tsp = cs.get(Y::TS + ip - 1);
    const float bsw = cs.get(Y::BSW + i - 1), psi = cs.get(Y::PSI + i - 1);
    const float e = one - one / bsw;
    cs.set(Y::NINVB + i - 1, -one / bsw);
    cs.set(Y::ITS + i - 1, one / (ts + tsp));
    const float pte = psi * ts / e;
    cs.set(Y::PTE + i - 1, pte);
    cs.set(Y::C3 + i - 1, pte / (g.zi(i) - g.zi(i - 1)));
  }
  float mh = cs.get(Y::HKS + 0);
  if (cs.get(Y::HKS + 1) < mh) mh = cs.get(Y::HKS + 1);
  if (cs.get(Y::HKS + 2) < mh) mh = cs.get(Y::HKS + 2);
  cs.set(Y::MH3, mh);
  cs.set(Y::TSDZ1, MAXF(zero, (cs.get(Y::TS + 0) * g.dz(1))));
}

template <int L>
H9K_HD int jwt_of(float zwt, const float *zim) {
  // HYDROLOGY.f90:499-508: first I with zwt <= zi(I)/1000, jwt = I-1
  int jwt = L;
#pragma unroll
  for (int i = L; i >= 1; i--)
    if (zwt <= zim[i]) jwt = i - 1;
  return jwt;
}

// Day constants into the store (any store type with set_day).  M = MathExact
// (once per cell-day).
template <class CS, class M>
H9K_HD void day_consts(const Day &d, float LAI, float LAI_litter, const CS &cs, M &m) {
  const float tak = d.tak;
  cs.set_day(D_FORC, d.forc_rain);
  cs.set_day(D_OK, ((LAI > zero) && (d.PAR > zero)) ? one : zero);
  const float tsv = tak * (one + d.huss * deltx);                       // :232
  const float rho = d.ps / (rgas * tsv);                                // :236
  const float tc = tak - tf + 237.3f;
  const float ex = m.expf((17.27f * (tak - tf)) / tc);                  // :244,254
  float desatdT = (4098.0f * (0.6108f * ex)) / (tc * tc);
  desatdT = desatdT * 18.0f / (gasc * tak);                             // :247
  float esat = 0.6108f * ex;
  esat = esat * 18.0f / (gasc * tak);                                   // :255
  const float VDD = esat * (one - d.rh / 100.0f);                       // :259
  const float gamma = (cp * d.ps / (d.lamb * 0.622f)) * (18.0E-3f / (gasc * tak));  // :263
  cs.set_day(D_DESAT, desatdT);
  cs.set_day(D_GAMMA, gamma);
  cs.set_day(D_VDD, VDD);
  // :283-295 (beta enters per substep)
  cs.set_day(D_X, (1.0f / (d.PAR / (d.PAR + 300.0f))) * 400.0f);
  cs.set_day(D_LAI2, 2.0f * LAI);
  cs.set_day(D_PW28, m.powf(2.8f, -80.0f * MAXF(zero, VDD) / rho));
  cs.set_day(D_RSCMIN, 1.0f / ((LAI / 2.7f) * 0.9f / (rho * 1.0E3f / 18.0f)));
  // :302-318
  const float rac = (LAI > zero) ? 25.0f / (2.0f * LAI) : 1.0E6f;
  float raa, ras;
  if (LAI <= 4.0f) {
    raa = 0.25f * LAI * 42.0f + 0.25f * (4.0f - LAI) * 34.0f;
    ras = 0.25f * LAI * 128.0f + 0.25f * (4.0f - LAI) * 49.0f;
  } else {
    raa = 42.0f;
    ras = 128.0f;
  }
  cs.set_day(D_RAC, rac);
  cs.set_day(D_RAA, raa);
  cs.set_day(D_RAS, ras);
  // :326-330 litter factors
  cs.set_day(D_LIT, 10.0f + 1000.0f * LAI_litter);
  cs.set_day(D_LIT1000, 1000.0f * LAI_litter);
  // :335-389
  const float Rnet = d.Rnet;
  const float Rnets = Rnet * m.expf(-0.7f * LAI);
  const float G = 0.2f * Rnets;
  const float rhocp = rho * cp;
  const float A1 = desatdT * (Rnet - G);
  const float rcv = rhocp * VDD;
  const float raarac = raa + rac, raaras = raa + ras;
  const float dg = desatdT + gamma;
  cs.set_day(D_RHOCP, rhocp);
  cs.set_day(D_A1, A1);
  cs.set_day(D_RAARAC, raarac);
  cs.set_day(D_RAARAS, raaras);
  cs.set_day(D_NUMC, A1 + (rcv - desatdT * rac * (Rnets - G)) / raarac);
  cs.set_day(D_NUMS, A1 + (rcv - desatdT * ras * (Rnet - Rnets)) / raaras);
  cs.set_day(D_DG, dg);
  cs.set_day(D_RA, dg * raa);
  cs.set_day(D_DGRAS, dg * ras);
  cs.set_day(D_DGRAC, dg * rac);
  cs.set_day(D_DRR, desatdT * (Rnet - Rnets));
  cs.set_day(D_DRG, desatdT * (Rnets - G));
  cs.set_day(D_RL, rhow * d.lamb);
}

// One HYDROLOGY call.  Returns 0 or an H9G_ERR_* code.  theta (1..L)
// receives the end-of-step volumetric water (HYDROLOGY.f90:1233).
template <int L, class G, class M>
H9K_HD int hydrology_step(const G &g, CellStore<L> cs, St<L> &s, float *theta, float &rnf_sum,
                          float &errval, M &m) {
  typedef Lay<L> Y;
  const float dt = g.dt();
  constexpr double r1000 = 1.0 / 1000.0;
  float zim[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) zim[i] = g.zim(i);
  float *h2o = s.h2o, *smp = s.smp;
  cs.launder();
#define TS(i) cs.get(Y::TS + (i) - 1)
#define HKS(i) cs.get(Y::HKS + (i) - 1)
#define BSW(i) cs.get(Y::BSW + (i) - 1)
#define PSI(i) cs.get(Y::PSI + (i) - 1)
#define INV(F, i) cs.get(Y::F + (i) - 1)
#define EXPO(i) (one + cs.get(Y::NINVB + (i) - 1))
#define ROOT(i) cs.get(Y::ROOTR + (i) - 1)
#define DC(F) cs.get(Y::DAY + F)

  // :141-151
  float w0 = DC(D_FORC) * dt + s.wa;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    w0 = w0 + h2o[i];
    theta[i] = m.div(h2o[i], g.thk(i), g.rthk(i));
  }
  // :161-212
  const float qflx_top_soil = DC(D_FORC);
  const float hkdepth = one / 2.5f;
  const float fff = 1.0f / hkdepth;
  const float fsat = cs.get(Y::FMAX) * m.expf(-0.5f * fff * s.zwt);
  float qflx_surf = fsat * qflx_top_soil;
  const float frac_h2osfc = zero;
  // :269-276 (previous-step smp)
  float beta = zero;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    float b = one - m.div(smp[i] - g.zc(i), -150000.0f, 1.0 / -150000.0);
    b = MINF(one, b);
    b = MAXF(zero, b);
    beta = beta + ROOT(i) * b;
  }
  // :283-295
  float rsc;
  if ((DC(D_OK) != zero) && (beta > zero))
    rsc = DC(D_X) / (DC(D_LAI2) * beta * DC(D_PW28));
  else
    rsc = 1.0E6f;
  rsc = MAXF(rsc, DC(D_RSCMIN));
  // :325-331
  float rss;
  if (theta[1] <= 0.15f)
    rss = DC(D_LIT) * m.expf(0.3563f * 100.0f * (0.15f - theta[1]));
  else
    rss = (10.0f + DC(D_LIT1000) * (1.0f - theta[1] / TS(1)));
  // :344-389
  const float desatdT = DC(D_DESAT), gamma = DC(D_GAMMA);
  const float PMc = DC(D_NUMC) / (desatdT + gamma * (one + rsc / DC(D_RAARAC)));
  const float PMs = DC(D_NUMS) / (desatdT + gamma * (one + rss / DC(D_RAARAS)));
  const float Ra = DC(D_RA);
  const float Rs = DC(D_DGRAS) + gamma * rss;
  const float Rc = DC(D_DGRAC) + gamma * rsc;
  const float Cc = one / (one + Rc * Ra / (Rs * (Rc + Ra)));
  const float Cs = one / (one + Rs * Ra / (Rc * (Rs + Ra)));
  const float LE = Cc * PMc + Cs * PMs;
  const float VDD0 = DC(D_VDD) + (DC(D_A1) - DC(D_DG) * LE) * DC(D_RAA) / DC(D_RHOCP);
  const float LEc = (DC(D_DRR) + DC(D_RHOCP) * VDD0 / DC(D_RAC)) / (desatdT + gamma * (1.0f + rsc / DC(D_RAC)));
  const float LEs = (DC(D_DRG) + DC(D_RHOCP) * VDD0 / DC(D_RAS)) / (desatdT + gamma * (1.0f + rss / DC(D_RAS)));
  const float tran = LEc * 1.0E3f / DC(D_RL);
  float evg = LEs * 1.0E3f / DC(D_RL);
  // :396-400
  float em1 = m.div(g.dz(1) * (theta[1] - watmin), dt, g.rdt()) - tran * ROOT(1);
  em1 = MAXF(zero, em1);
  evg = MINF(em1, evg);
  // :426-478
  const float qflx_evap = evg;
  float qflx_in_soil = (one - frac_h2osfc) * (qflx_top_soil - qflx_surf);
  qflx_in_soil = qflx_in_soil - (one - frac_h2osfc) * qflx_evap;
  const float qinmax = (one - fsat) * cs.get(Y::MH3);
  const float qflx_infl_excess = MAXF(zero, qflx_in_soil - (one - frac_h2osfc) * qinmax);
  const float qflx_infl = qflx_in_soil - qflx_infl_excess;
  qflx_surf = qflx_surf + qflx_infl_excess;
  // :492-508
  float zwtmm = 1000.0f * s.zwt;
  const int jwt = jwt_of<L>(s.zwt, zim);
  cs.launder();
  // :517-567 equilibrium profile
  float zq[L + 2];
#pragma unroll
  for (int i = 1; i <= L; i++) {
    float vol_eq;
    if (zwtmm <= g.zi(i - 1)) {
      vol_eq = TS(i);
    } else {
      // (-psi + zwtmm - zi(I-1))/(-psi) ** (1-1/bsw): temp0 of both cases
      const float temp0 = m.powf((((-PSI(i)) + zwtmm - g.zi(i - 1)) / (-PSI(i))), EXPO(i));
      if ((zwtmm < g.zi(i)) && (zwtmm > g.zi(i - 1))) {
        const float tempi = one;
        const float voleq1 = INV(PTE, i) / (zwtmm - g.zi(i - 1)) * (tempi - temp0);
        vol_eq = m.div(voleq1 * (zwtmm - g.zi(i - 1)) + TS(i) * (g.zi(i) - zwtmm), g.dz(i),
                       g.rdz(i));
        vol_eq = MINF(TS(i), vol_eq);
        vol_eq = MAXF(vol_eq, zero);
      } else {
        const float tempi = m.powf(((-PSI(i) + zwtmm - g.zi(i)) / (-PSI(i))), EXPO(i));
        vol_eq = INV(C3, i) * (tempi - temp0);
        vol_eq = MAXF(vol_eq, 0.0f);
        vol_eq = MINF(TS(i), vol_eq);
      }
    }
    zq[i] = PSI(i) * m.powf(MAXF(vol_eq / TS(i), 0.01f), -BSW(i));
    zq[i] = MAXF(smpmin, zq[i]);
    sched_fence();
  }
  // :574-590 aquifer node when the water table is below the column
  zq[L + 1] = zero;
  if (jwt == L) {
    const float tempi = 1.0f;
    const float temp0 = m.powf(((-PSI(L) + zwtmm - g.zi(L)) / (-PSI(L))), EXPO(L));
    float ve = INV(PTE, L) / (zwtmm - g.zi(L)) * (tempi - temp0);
    ve = MAXF(ve, 0.0f);
    ve = MINF(TS(L), ve);
    const float z = PSI(L) * m.powf(MAXF(ve / TS(L), 0.01f), -BSW(L));
    zq[L + 1] = MAXF(smpmin, z);
  }
  cs.launder();
  // :598-639 conductivity and matric potential
  float hk[L + 1], dhkdw[L + 1], dsmpdw[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) {
    const int ip = (L < i + 1) ? L : i + 1;
    float s1 = 0.5f * (theta[i] + theta[ip]) / (0.5f * (TS(i) + TS(ip)));
    s1 = MINF(one, s1);
    const float s2 = HKS(i) * m.powf(s1, 2.0f * BSW(i) + 2.0f);
    hk[i] = s1 * s2;
    dhkdw[i] = (2.0f * BSW(i) + 3.0f) * s2 * INV(ITS, i);
    float s_node = MAXF(theta[i] / TS(i), 0.01f);
    s_node = MINF(one, s_node);
    float sm = PSI(i) * m.powf(s_node, -BSW(i));
    sm = MAXF(smpmin, sm);
    smp[i] = sm;
    dsmpdw[i] = (-BSW(i)) * sm / (s_node * TS(i));
    sched_fence();
  }
  // :645-650 aquifer node geometry
  const float zcA = 0.5f * (zwtmm + g.zc(L));
  const float dzA = (jwt < L) ? g.dz(L) : zwtmm - g.zc(L);
  cs.launder();
  // tridiagonal system, rows 1..L+1 (:661-799)
  float amx[L + 2], bmx[L + 2], cmx[L + 2], rmx[L + 2];
  {
    const float den = g.den(1);                     // zc(2)-zc(1)
    const double rden = g.rden(1);
    const float dzq = (zq[2] - zq[1]);
    const float num = (smp[2] - smp[1]) - dzq;
    const float qout = m.div(-hk[1] * num, den, rden);
    const float dqodw1 = m.div(-(-hk[1] * dsmpdw[1] + num * dhkdw[1]), den, rden);
    const float dqodw2 = m.div(-(hk[1] * dsmpdw[2] + num * dhkdw[1]), den, rden);
    rmx[1] = qflx_infl - qout - tran * ROOT(1);
    amx[1] = zero;
    bmx[1] = m.div(g.dz(1), dt, g.rdt()) + dqodw1;
    cmx[1] = dqodw2;
  }
#pragma unroll
  for (int i = 2; i <= L - 1; i++) {
    float den = g.den(i - 1);                       // zc(I)-zc(I-1)
    double rden = g.rden(i - 1);
    float dzq = zq[i] - zq[i - 1];
    float num = smp[i] - smp[i - 1] - dzq;
    const float qin = m.div(-hk[i - 1] * num, den, rden);
    const float dqidw0 = m.div(-(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]), den, rden);
    const float dqidw1 = m.div(-(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]), den, rden);
    den = g.den(i);                                 // zc(I+1)-zc(I)
    rden = g.rden(i);
    dzq = zq[i + 1] - zq[i];
    num = (smp[i + 1] - smp[i]) - dzq;
    const float qout = m.div(-hk[i] * num, den, rden);
    const float dqodw1 = m.div(-(-hk[i] * dsmpdw[i] + num * dhkdw[i]), den, rden);
    const float dqodw2 = m.div(-(hk[i] * dsmpdw[i + 1] + num * dhkdw[i]), den, rden);
    rmx[i] = qin - qout - tran * ROOT(i);
    amx[i] = -dqidw0;
    bmx[i] = m.div(g.dz(i), dt, g.rdt()) - dqidw1 + dqodw1;
    cmx[i] = dqodw2;
  }
  {
    constexpr int i = L;
    float den = g.den(i - 1);
    const double rden0 = g.rden(i - 1);
    float dzq = zq[i] - zq[i - 1];
    float num = smp[i] - smp[i - 1] - dzq;
    const float qin = m.div(-hk[i - 1] * num, den, rden0);
    const float dqidw0 = m.div(-(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]), den, rden0);
    const float dqidw1 = m.div(-(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]), den, rden0);
    amx[i] = -dqidw0;
    if (i > jwt) {                 // water table inside the column
      const float qout = zero, dqodw1 = zero;
      rmx[i] = qin - qout - tran * ROOT(i);
      bmx[i] = m.div(g.dz(i), dt, g.rdt()) - dqidw1 + dqodw1;
      cmx[i] = zero;
      rmx[i + 1] = zero;
      amx[i + 1] = zero;
      bmx[i + 1] = m.div(dzA, dt, g.rdt());
      cmx[i + 1] = zero;
    } else {                       // below: aquifer row
      float s_node = MAXF(0.5f * (one + theta[i] / TS(i)), 0.01f);
      s_node = MINF(one, s_node);
      float smp1 = PSI(i) * m.powf(s_node, -BSW(i));
      smp1 = MAXF(smpmin, smp1);
      const float dsmpdw1 = -BSW(i) * smp1 / (s_node * TS(i));
      den = zcA - g.zc(i);
      const double rden = recip64(den);
      dzq = zq[i + 1] - zq[i];
      num = smp1 - smp[i] - dzq;
      const float qout = m.div(-hk[i] * num, den, rden);
      const float dqodw1 = m.div(-(-hk[i] * dsmpdw[i] + num * dhkdw[i]), den, rden);
      const float dqodw2 = m.div(-(hk[i] * dsmpdw1 + num * dhkdw[i]), den, rden);
      rmx[i] = qin - qout - tran * ROOT(i);
      bmx[i] = m.div(g.dz(i), dt, g.rdt()) - dqidw1 + dqodw1;
      cmx[i] = dqodw2;
      const float qin1 = qout;
      const float dqidw0b = dqodw1;    // the same expression (:787-788 vs :769-770)
      const float dqidw1b = dqodw2;    // (:789-790 vs :771-772)
      const float qout1 = zero, dqodw1b = zero;
      rmx[i + 1] = qin1 - qout1;
      amx[i + 1] = -dqidw0b;
      bmx[i + 1] = m.div(dzA, dt, g.rdt()) - dqidw1b + dqodw1b;
      cmx[i + 1] = zero;
    }
  }
  // :806-837 Thomas algorithm
  if (bmx[1] == 0.0f) { errval = bmx[1]; return 1; }
  float dwat2[L + 2], GAM[L + 2];
  // each pivot's reciprocal serves both quotients of its row (MathFast)
  float BET = bmx[1];
  double rbet = recip64(BET);
  dwat2[1] = m.div(rmx[1], BET, rbet);
  int zero_pivot = 0;
#pragma unroll
  for (int i = 2; i <= L + 1; i++) {
    GAM[i] = m.div(cmx[i - 1], BET, rbet);
    BET = bmx[i] - amx[i] * GAM[i];
    if (BET == 0.0f && !zero_pivot) zero_pivot = i;
    rbet = recip64(BET);
    dwat2[i] = m.div(rmx[i] - amx[i] * dwat2[i - 1], BET, rbet);
  }
  if (zero_pivot) { errval = (float)zero_pivot; return 2; }
#pragma unroll
  for (int i = L; i >= 1; i--) dwat2[i] = dwat2[i] - GAM[i + 1] * dwat2[i + 1];
  // :845-850
#pragma unroll
  for (int i = 1; i <= L; i++) h2o[i] = h2o[i] + dwat2[i] * g.dz(i);
  cs.launder();
  // :856-904 recharge
  float qcharge;
  if (jwt < L) {
    float th_j = zero, ts_j = one, hks_j = zero, bsw_j = zero, smp_m = zero, zq_m = zero, zc_j = zero;
#pragma unroll
    for (int i = 1; i <= L; i++) {
      if (i == jwt + 1) { th_j = theta[i]; ts_j = TS(i); hks_j = HKS(i); bsw_j = BSW(i); }
      if (i == (jwt > 1 ? jwt : 1)) { smp_m = smp[i]; zq_m = zq[i]; }
      if (i == jwt) zc_j = g.zc(i);
    }
    const float wh_zwt = zero;
    const float s_node = MAXF(th_j / ts_j, 0.01f);
    const float s1 = MINF(one, s_node);
    const float ka = hks_j * m.powf(s1, 2.0f * bsw_j + 3.0f);
    const float smp1 = MAXF(smpmin, smp_m);
    const float wh = smp1 - zq_m;
    if (jwt == 0)
      qcharge = -ka * (wh_zwt - wh) / (zwtmm + one);
    else
      qcharge = -ka * (wh_zwt - wh) / ((zwtmm - zc_j) * 2.0f);
    qcharge = MAXF(-10.0f / dt, qcharge);
    qcharge = MINF(10.0f / dt, qcharge);
  } else {
    qcharge = m.div(dwat2[L + 1] * dzA, dt, g.rdt());
  }
  // :923-1009 water table from recharge.  The jwt recomputed at :923-931
  // equals the one above (zwt unchanged since :499).  Specific yields
  // s_y(I) (:963-965, :979-981) and rous (:937-940, = s_y(L)) for the
  // current zwtmm are evaluated once; all layers only if some lane of
  // the wave has its water table inside the column.
  float sy[L + 1];
  sy[L] = MAXF(TS(L) * (one - m.powf((one + zwtmm / (-PSI(L))), INV(NINVB, L))), 0.02f);
  if (any_lane(jwt < L)) {
#pragma unroll
    for (int i = 1; i <= L - 1; i++) {
      sy[i] = MAXF(TS(i) * (one - m.powf((one + zwtmm / (-PSI(i))), INV(NINVB, i))), 0.02f);
      sched_fence();
    }
  }
  float rous = sy[L];
  int jwt2 = jwt;
  if (jwt == L) {
    s.wa = s.wa + qcharge * dt;
    s.zwt = s.zwt - m.div(qcharge * dt, 1000.0f, r1000) / rous;
  } else {
    float qcharge_tot = qcharge * dt;
    if (qcharge_tot > zero) {          // rising: I = jwt+1 .. 1
      bool active = true;
#pragma unroll
      for (int i = L; i >= 1; i--) {
        if (active && i <= jwt + 1) {
          const float s_y = sy[i];
          float qcl = MINF(qcharge_tot, s_y * (zwtmm - g.zi(i - 1)));
          qcl = MAXF(qcl, zero);
          if (s_y > zero) s.zwt = s.zwt - m.div(qcl / s_y, 1000.0f, r1000);
          qcharge_tot = qcharge_tot - qcl;
          if (qcharge_tot <= zero) active = false;
        }
      }
    } else {                            // deepening: I = jwt+1 .. L
      bool active = true;
#pragma unroll
      for (int i = 1; i <= L; i++) {
        if (active && i >= jwt + 1) {
          const float s_y = sy[i];
          float qcl = MAXF(qcharge_tot, -s_y * (g.zi(i) - zwtmm));
          qcl = MINF(qcl, zero);
          qcharge_tot = qcharge_tot - qcl;
          if (qcharge_tot >= zero) {
            s.zwt = s.zwt - m.div(qcl / s_y, 1000.0f, r1000);
            active = false;
          } else {
            s.zwt = g.zi(i) / 1000.0f;
          }
        }
      }
      if (qcharge_tot > zero) s.zwt = s.zwt - m.div(qcharge_tot, 1000.0f, r1000) / rous;
    }
    jwt2 = jwt_of<L>(s.zwt, zim);
  }
  cs.launder();
  // :1015-1035 baseflow; s_y for the new zwtmm (:1077-1080) as above
  zwtmm = 1000.0f * s.zwt;
  float rsub_top = 5.5E-3f * m.expf(-fff * s.zwt);
  sy[L] = MAXF(TS(L) * (one - m.powf((one + zwtmm / (-PSI(L))), INV(NINVB, L))), 0.02f);
  if (any_lane(jwt2 < L)) {
#pragma unroll
    for (int i = 1; i <= L - 1; i++) {
      sy[i] = MAXF(TS(i) * (one - m.powf((one + zwtmm / (-PSI(i))), INV(NINVB, i))), 0.02f);
      sched_fence();
    }
  }
  rous = sy[L];
  // :1048-1118
  int jwt3 = jwt2;
  if (jwt2 == L) {
    s.wa = s.wa - rsub_top * dt;
    s.zwt = s.zwt + m.div(rsub_top * dt, 1000.0f, r1000) / rous;
    h2o[L] = h2o[L] + MAXF(0.0f, (s.wa - 5000.0f));
    s.wa = MINF(s.wa, 5000.0f);
  } else {
    float rsub_top_tot = -rsub_top * dt;
    if (rsub_top_tot > zero) { errval = rsub_top_tot; return 3; }
    bool active = true;
#pragma unroll
    for (int i = 1; i <= L; i++) {
      if (active && i >= jwt2 + 1) {
        const float s_y = sy[i];
        float rstl = MAXF(rsub_top_tot, -(s_y * (g.zi(i) - zwtmm)));
        rstl = MINF(rstl, zero);
        h2o[i] = h2o[i] + rstl;
        rsub_top_tot = rsub_top_tot - rstl;
        if (rsub_top_tot >= zero) {
          s.zwt = s.zwt - m.div(rstl / s_y, 1000.0f, r1000);
          active = false;
        } else {
          s.zwt = g.zi(i) / 1000.0f;
        }
      }
    }
    s.zwt = s.zwt - m.div(rsub_top_tot, 1000.0f, r1000) / rous;
    s.wa = s.wa + rsub_top_tot;
    jwt3 = jwt_of<L>(s.zwt, zim);
  }
  // :1122-1123
  s.zwt = MAXF(0.0f, s.zwt);
  s.zwt = MINF(80.0f, s.zwt);
  cs.launder();
  // :1131-1137 saturation excess, bottom-up bucket
#pragma unroll
  for (int i = L; i >= 2; i--) {
    const float cap = MAXF(0.01f, TS(i)) * g.dz(i);
    const float xsi = MAXF(h2o[i] - cap, zero);
    h2o[i] = MINF(cap, h2o[i]);
    h2o[i - 1] = h2o[i - 1] + xsi;
  }
  // :1144-1152
  const float xs1 = MAXF(MAXF(h2o[1], zero) - cs.get(Y::TSDZ1), zero);
  h2o[1] = MINF(cs.get(Y::TSDZ1), h2o[1]);
  const float qflx_rsub_sat = m.div(xs1, dt, g.rdt());
  // :1161-1174 watmin top-down
#pragma unroll
  for (int i = 1; i <= L - 1; i++) {
    float xs = zero;
    if (h2o[i] < watmin) {
      xs = watmin - h2o[i];
      if (i == jwt3) s.zwt = s.zwt + m.div(xs / MAXF(0.01f, TS(i)), 1000.0f, r1000);
    }
    h2o[i] = h2o[i] + xs;
    h2o[i + 1] = h2o[i + 1] - xs;
  }
  // :1180-1211 bottom layer from above
  float xs = zero;
  if (h2o[L] < watmin) {
    xs = watmin - h2o[L];
    bool active = true;
#pragma unroll
    for (int j = L - 1; j >= 1; j--) {
      if (active) {
        const float avail = MAXF(h2o[j] - watmin - xs, zero);
        if (avail >= xs) {
          h2o[L] = h2o[L] + xs;
          h2o[j] = h2o[j] - xs;
          xs = zero;
          active = false;
        } else {
          h2o[L] = h2o[L] + avail;
          h2o[j] = h2o[j] - avail;
          xs = xs - avail;
        }
      }
    }
  }
  h2o[L] = h2o[L] + xs;
  rsub_top = rsub_top - m.div(xs, dt, g.rdt());
  // :1221-1236
  float w1 = ((1.0f - frac_h2osfc) * (qflx_surf + evg + tran) + rsub_top + qflx_rsub_sat) * dt + s.wa;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    w1 = w1 + h2o[i];
    theta[i] = m.div(MAXF(h2o[i], 1.0E-6f), g.thk(i), g.rthk(i));
  }
  // :1244
  if (absf(w1 - w0) > 0.1f) { errval = w1 - w0; return 4; }
  // :1282-1283
  rnf_sum = rnf_sum + qflx_surf * dt;
  rnf_sum = rnf_sum + rsub_top * dt;
  return 0;
#undef TS
#undef HKS
#undef BSW
#undef PSI
#undef INV
#undef EXPO
#undef ROOT
#undef DC
}

// GROW.f90:55-201 (nplants = 1, iGPT = 1).  rootr(L+1) is zeroed by the
// caller's state write-back.
template <int L, class G, class M, class CS>
H9K_HD void grow_day(const G &g, float tas, St<L> &s, const CS &cs, float &npp, M &m) {
  float w_i = zero;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    float w = (-150000.0f - s.smp[i]) / (-150000.0f - (-50000.0f));
    w = MAXF(zero, w);
    w = MINF(one, w);
    w_i = w_i + cs.root(i) * w;
  }
  float fT;
  if ((tas - tf) > 18.0f) {
    const float a = absf(tas - tf - 18.0f) / 21.0f;
    fT = one - a * a;
  } else {
    const float a = absf(tas - tf - 18.0f) / 25.0f;
    fT = one - a * a;
    fT = MAXF(zero, fT);
    fT = MINF(one, fT);
  }
  const float grow_plant_mass = (1000.0f / 365.0f) * w_i * fT;
  const float grow_foliage_mass = grow_plant_mass / 3.3f;
  const float loss_plant_mass = (0.1f / 365.0f) * s.pm;
  float loss_foliage_mass = (1.0f / 365.0f) * s.pfm / MINF(one, MAXF(0.01f, w_i));
  if (w_i < 0.6f) loss_foliage_mass = 0.1f * s.pfm;
  const float dplant_mass = grow_plant_mass - loss_plant_mass;
  const float dplant_foliage_mass = grow_foliage_mass - loss_foliage_mass;
  s.pm = s.pm + dplant_mass;
  s.pfm = s.pfm + dplant_foliage_mass;
  s.plen = m.powf(400.0f * s.pm / 3.142E-3f, one / 3.0f);
  const float dLAI = dplant_foliage_mass * sla1;
  s.LAI = s.LAI + dLAI;
  s.LAI = MAXF(0.001f, s.LAI);
  s.LAI_litter = s.LAI_litter + MAXF(zero, dLAI);
  s.rdepth = 0.3f * s.plen;
  const float decay = m.expf(log_0p1 / (s.rdepth / 10.0f));
  // decay ** (zi(I)/10) is shared by rows I and I+1: 9 powf instead of 16
  float pw_prev = m.powf(decay, g.zi(0) / 10.0f);
#pragma unroll
  for (int i = 1; i <= L; i++) {
    const float pw = m.powf(decay, g.zi(i) / 10.0f);
    cs.set_root(i, zero + (1.0f - pw) - (1.0f - pw_prev));
    pw_prev = pw;
  }
  npp = zero + dplant_mass;
  s.LAI_litter = s.LAI_litter - 0.02f * s.LAI_litter;
}

// INIT.f90:707-811 for one cell (smp = 0).
template <int L, class G, class M>
H9K_HD void init_cell(const G &g, const float *ts, St<L> &s, float *rootr, float *h2o_ma, M &m) {
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = 0.4f * ts[i] * g.dz(i) * rhow / 1000.0f;
    h2o_ma[i] = 0.4f * 0.1f * g.dz(i) * rhow / 1000.0f;
    s.smp[i] = zero;
  }
  s.zwt = (g.zi(L) + 5000.0f) / 1000.0f;
  s.wa = 4000.0f;
  s.LAI_litter = 0.001f;
  s.pm = 1.0f;
  s.pfm = 0.0435f;
  s.plen = m.powf(400.0f * s.pm / 3.142E-3f, one / 3.0f);
  s.LAI = zero + s.pfm * sla1 / 1.0f;
  s.rdepth = 0.3f * s.plen;
  const float decay = m.expf(log_0p1 / (s.rdepth / 10.0f));
#pragma unroll
  for (int i = 1; i <= L; i++)
    rootr[i] = zero + (1.0f - m.powf(decay, g.zi(i) / 10.0f)) -
                 (1.0f - m.powf(decay, g.zi(i - 1) / 10.0f));
}

// Day driver variables (HYBRID9.f90:168-184) from the forcing of one day.
H9K_HD Day make_day(float tas, float rlds, float rsds, float huss, float ps, float pr, float rhs) {
  Day d;
  d.tak = tas;
  d.rh = rhs;
  d.Rnet = 0.92f * rsds + rlds - stbo * (tas * (tas * (tas * tas)));
  d.PAR = 0.92f * rsds * 2.3f;
  d.forc_rain = 1.0E3f * pr / rhow;
  d.lamb = ((2503.0f - 2.386f * (d.tak - tf))) * 1.0E3f;
  d.huss = huss;
  d.ps = ps;
  return d;
}

// Exact re-run of a substep (rare path), out of line so the hot path's
// register allocation does not carry a second copy of the substep.  State
// in and out goes through the store's SV_* area (no stack objects).
#if defined(__HIP_DEVICE_COMPILE__)
#define H9K_COLD __device__ __attribute__((noinline, cold))
#else
#define H9K_COLD static __attribute__((noinline, cold))
#endif
template <int L, class G>
H9K_COLD int substep_exact(const G *g, CellStore<L> cs, const uint64_t *e2, const double *l2) {
  typedef Lay<L> Y;
  St<L> s;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = cs.get(Y::SV_H2O + i - 1);
    s.smp[i] = cs.get(Y::SV_SMP + i - 1);
  }
  s.zwt = cs.get(Y::SV_ZWT);
  s.wa = cs.get(Y::SV_WA);
  float rnf = cs.get(Y::SV_RNF), errval = zero;
  float theta[L + 1];
  MathExact me{{e2, l2}};
  const int code = hydrology_step<L, G, MathExact>(*g, cs, s, theta, rnf, errval, me);
#pragma unroll
  for (int i = 1; i <= L; i++) {
    cs.set(Y::SV_H2O + i - 1, s.h2o[i]);
    cs.set(Y::SV_SMP + i - 1, s.smp[i]);
  }
  cs.set(Y::SV_ZWT, s.zwt);
  cs.set(Y::SV_WA, s.wa);
  cs.set(Y::SV_RNF, rnf);
  cs.set(Y::SV_ERR, errval);
  return code;
}

// One substep with speculate-then-verify math (see file comment).  The
// pre-step state is parked in the store rather than in registers.
template <int L, class G>
H9K_HD int substep(const G &g, CellStore<L> cs, St<L> &s, float *theta, float &rnf_sum,
                   float &errval, const h9m::Tabs &T) {
  typedef Lay<L> Y;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    cs.set(Y::SV_H2O + i - 1, s.h2o[i]);
    cs.set(Y::SV_SMP + i - 1, s.smp[i]);
  }
  cs.set(Y::SV_ZWT, s.zwt);
  cs.set(Y::SV_WA, s.wa);
  cs.set(Y::SV_RNF, rnf_sum);
  MathFast mf{T, false};
  int code = hydrology_step<L, G, MathFast>(g, cs, s, theta, rnf_sum, errval, mf);
  if (__builtin_expect(mf.special, 0)) {
    code = substep_exact<L, G>(&g, cs, T.exp2, T.log2);
    cs.launder();
#pragma unroll
    for (int i = 1; i <= L; i++) {
      s.h2o[i] = cs.get(Y::SV_H2O + i - 1);
      s.smp[i] = cs.get(Y::SV_SMP + i - 1);
      theta[i] = MAXF(s.h2o[i], 1.0E-6f) / g.thk(i);     // HYDROLOGY.f90:1233
    }
    s.zwt = cs.get(Y::SV_ZWT);
    s.wa = cs.get(Y::SV_WA);
    rnf_sum = cs.get(Y::SV_RNF);
    errval = cs.get(Y::SV_ERR);
  }
  return code;
}

// One calendar year for one cell: HYBRID9.f90:150-290.  The store holds
// the cell's parameters (cell_inv has run) and rootr.  forc points at the
// cell's tas of day 0; fday/fvar are the strides between days and between
// the 7 variables.  acc[r*astride], r < 12+L, accumulates the annual sums
// (:235-254) and finally receives the annual means (:263-290) in the
// order npp plant_mass rnf evap tas rlds rsds huss ps pr rhs theta(1..L)
// theta_total.  Returns 0 or the first STOP code (eday/estep/errval).
template <int L, class G>
H9K_HD int cell_year(const G &g, CellStore<L> cs, St<L> &s, const float *forc, size_t fday,
                     size_t fvar, int nt, int nisurf, int grow_on, float *acc, size_t astride,
                     int &eday, int &estep, float &errval, const h9m::Tabs &T) {
  enum { A_NPP = 0, A_PM, A_RNF, A_EVAP, A_TAS, A_RLDS, A_RSDS, A_HUSS, A_PS, A_PR, A_RHS,
         A_THETA, A_H2O = 11 + L };
  float *A = acc;
  const size_t as = astride;
  float rnf_sum = zero;
  float theta[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) theta[i] = zero;
#pragma unroll
  for (int k = 0; k < 12 + L; k++) A[k * as] = zero;
  float npp = zero;
  int code = 0;
  MathExact me{T};
  for (int day = 0; day < nt; day++) {
    cs.launder();
    opaque(A);
    const float *f = forc + (size_t)day * fday;
    opaque(f);
    const float tas = f[0 * fvar], rlds = f[1 * fvar], rsds = f[2 * fvar], huss = f[3 * fvar];
    const float ps = f[4 * fvar], pr = f[5 * fvar], rhs = f[6 * fvar];
    const Day d = make_day(tas, rlds, rsds, huss, ps, pr, rhs);     // :168-184
    day_consts(d, s.LAI, s.LAI_litter, cs, me);
    for (int ns = 0; ns < nisurf; ns++) {                            // :193-211
      code = substep<L, G>(g, cs, s, theta, rnf_sum, errval, T);
      if (code) { eday = day; estep = ns; break; }
    }
    if (code) return code;
    cs.launder();
    opaque(A);
    if (grow_on) grow_day<L, G, MathExact>(g, tas, s, cs, npp, me);  // :217
    A[A_TAS * as] = A[A_TAS * as] + tas;                              // :235-254
    A[A_RLDS * as] = A[A_RLDS * as] + rlds;
    A[A_RSDS * as] = A[A_RSDS * as] + rsds;
    A[A_HUSS * as] = A[A_HUSS * as] + huss;
    A[A_PS * as] = A[A_PS * as] + ps;
    A[A_PR * as] = A[A_PR * as] + pr;
    A[A_RHS * as] = A[A_RHS * as] + rhs;
    A[A_PM * as] = A[A_PM * as] + s.pm;
    A[A_NPP * as] = A[A_NPP * as] + npp;
    float h2o_sum = A[A_H2O * as];
#pragma unroll
    for (int i = 1; i <= L; i++) {
      A[(A_THETA + i - 1) * as] = A[(A_THETA + i - 1) * as] + theta[i];
      h2o_sum = h2o_sum + s.h2o[i];
    }
    A[A_H2O * as] = h2o_sum;
  }
  // :263-290 (npp_sum stays a sum; evap_sum is never accumulated)
  opaque(A);
  A[A_PM * as] = A[A_PM * as] / (float)nt;
  A[A_RNF * as] = rnf_sum / (float)(nt * nisurf);
  A[A_EVAP * as] = zero / (float)(nt * nisurf);
#pragma unroll
  for (int k = A_TAS; k <= A_H2O; k++) A[k * as] = A[k * as] / (float)nt;
  return 0;
}

}  // namespace h9k
