// h9g_step.h -- device restatement of the per-cell HYDROLOGY substep and
// the daily GROW update for gfx950, with the soil column in registers.
//
//   hydrology_step  /root/reference/SOURCE/HYDROLOGY.f90:141-1283
//   grow_day        /root/reference/SOURCE/GROW.f90:55-201
//
// Bit-exactness rules (same as the reference build, pinned by
// tests/test_gpu_parity.py against the oracle and tests/golden):
//   * float32 throughout, -ffp-contract=off, correctly rounded division;
//   * Fortran left-to-right evaluation order kept operation by operation;
//   * MIN(a,b) = a<b?a:b, MAX(a,b) = a>b?a:b (flang's compare+select);
//   * EXP / real powers -> h9m::expf / h9m::powf (glibc 2.35 bit-exact).
// Layer arrays are 1-based (index 0 unused) and fully unrolled over the
// compile-time layer count L, so every per-layer value lives in a VGPR;
// the only data-dependent index (jwt, the layer above the water table) is
// resolved with unrolled compare/select chains instead of indexed
// (scratch-memory) accesses.
#pragma once
#include "h9_math.h"

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

__device__ __forceinline__ float MAXF(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float MINF(float a, float b) { return a < b ? a : b; }

// Uniform layer geometry (INIT.f90:252-263), passed by value -> SGPRs.
template <int L>
struct Geo {
  float zi[L + 2];     // zi(0:L+1)
  float dz[L + 1];     // dz(1:L)    (dz(L+1) is per-step scratch)
  float zc[L + 1];     // zc(1:L)
  float zi_m[L + 1];   // zi(1:L)/1000 (water-table index test)
  float dt;
};

template <int L>
struct Par {           // per-cell soil parameters (SHARED.f90:398-429)
  float ts[L + 1], hks[L + 1], bsw[L + 1], psi[L + 1];
  float fmax;
};

template <int L>
struct St {            // per-cell persistent state (SHARED.f90)
  float h2o[L + 1], smp[L + 1], rootr[L + 1];
  float zwt, wa, LAI, LAI_litter, pm, pfm, plen, rdepth;
};

struct Day {           // HYBRID9.f90:168-184 + the forcing HYDROLOGY reads
  float tak, rh, Rnet, PAR, forc_rain, lamb, huss, ps;
};

template <int L>
__device__ __forceinline__ int jwt_of(float zwt, const Geo<L> &g) {
  // HYDROLOGY.f90:499-508: first I with zwt <= zi(I)/1000, jwt = I-1
  int jwt = L;
#pragma unroll
  for (int i = L; i >= 1; i--)
    if (zwt <= g.zi_m[i]) jwt = i - 1;
  return jwt;
}

// One HYDROLOGY call.  Returns 0 or an H9G_ERR_* code.  theta (1..L)
// receives the end-of-step volumetric water (HYDROLOGY.f90:1233).
template <int L>
__device__ __forceinline__ int hydrology_step(const Geo<L> &g, const Par<L> &p,
                                              const Day &d, St<L> &s, float *theta,
                                              float &rnf_sum, float &errval,
                                              const h9m::Tabs &T) {
  const float dt = g.dt;
  const float *zi = g.zi;
  const float *dz = g.dz;
  const float *zc = g.zc;
  const float *ts = p.ts, *hks = p.hks, *bsw = p.bsw, *psi = p.psi;
  float *h2o = s.h2o, *smp = s.smp;

  // :141-151
  float w0 = d.forc_rain * dt + s.wa;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    w0 = w0 + h2o[i];
    theta[i] = h2o[i] / (dz[i] * rhow / 1.0E3f);
  }
  // :161-212
  const float qflx_top_soil = d.forc_rain;
  const float hkdepth = one / 2.5f;
  const float fff = 1.0f / hkdepth;
  const float fsat = p.fmax * h9m::expf(-0.5f * fff * s.zwt, T);
  float qflx_surf = fsat * qflx_top_soil;
  const float frac_h2osfc = zero;
  // :232-263
  const float tak = d.tak;
  const float tsv = tak * (one + d.huss * deltx);
  const float rho = d.ps / (rgas * tsv);
  const float tc = tak - tf + 237.3f;
  const float ex = h9m::expf((17.27f * (tak - tf)) / tc, T);
  float desatdT = (4098.0f * (0.6108f * ex)) / (tc * tc);
  desatdT = desatdT * 18.0f / (gasc * tak);
  float esat = 0.6108f * ex;
  esat = esat * 18.0f / (gasc * tak);
  const float VDD = esat * (one - d.rh / 100.0f);
  const float gamma = (cp * d.ps / (d.lamb * 0.622f)) * (18.0E-3f / (gasc * tak));
  // :269-276 (previous-step smp)
  float beta = zero;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    float b = one - (smp[i] - zc[i]) / (-150000.0f);
    b = MINF(one, b);
    b = MAXF(zero, b);
    beta = beta + s.rootr[i] * b;
  }
  // :283-295
  const float LAI = s.LAI, PAR = d.PAR;
  float rsc;
  if ((LAI > zero) && (beta > zero) && (PAR > zero))
    rsc = (1.0f / (PAR / (PAR + 300.0f))) * 400.0f /
          (2.0f * LAI * beta * h9m::powf(2.8f, -80.0f * MAXF(zero, VDD) / rho, T));
  else
    rsc = 1.0E6f;
  rsc = MAXF(rsc, 1.0f / ((LAI / 2.7f) * 0.9f / (rho * 1.0E3f / 18.0f)));
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
  // :325-331
  float rss;
  if (theta[1] <= 0.15f)
    rss = (10.0f + 1000.0f * s.LAI_litter) * h9m::expf(0.3563f * 100.0f * (0.15f - theta[1]), T);
  else
    rss = (10.0f + 1000.0f * s.LAI_litter * (1.0f - theta[1] / ts[1]));
  // :335-389
  const float Rnet = d.Rnet;
  const float Rnets = Rnet * h9m::expf(-0.7f * LAI, T);
  const float G = 0.2f * Rnets;
  const float PMc = (desatdT * (Rnet - G) + (rho * cp * VDD - desatdT * rac * (Rnets - G)) /
                     (raa + rac)) / (desatdT + gamma * (one + rsc / (raa + rac)));
  const float PMs = (desatdT * (Rnet - G) + (rho * cp * VDD - desatdT * ras * (Rnet - Rnets)) /
                     (raa + ras)) / (desatdT + gamma * (one + rss / (raa + ras)));
  const float Ra = (desatdT + gamma) * raa;
  const float Rs = (desatdT + gamma) * ras + gamma * rss;
  const float Rc = (desatdT + gamma) * rac + gamma * rsc;
  const float Cc = one / (one + Rc * Ra / (Rs * (Rc + Ra)));
  const float Cs = one / (one + Rs * Ra / (Rc * (Rs + Ra)));
  const float LE = Cc * PMc + Cs * PMs;
  const float VDD0 = VDD + (desatdT * (Rnet - G) - (desatdT + gamma) * LE) * raa / (rho * cp);
  const float LEc = (desatdT * (Rnet - Rnets) + rho * cp * VDD0 / rac) /
                    (desatdT + gamma * (1.0f + rsc / rac));
  const float LEs = (desatdT * (Rnets - G) + rho * cp * VDD0 / ras) /
                    (desatdT + gamma * (1.0f + rss / ras));
  const float tran = LEc * 1.0E3f / (rhow * d.lamb);
  float evg = LEs * 1.0E3f / (rhow * d.lamb);
  // :396-400
  float em1 = dz[1] * (theta[1] - watmin) / dt - tran * s.rootr[1];
  em1 = MAXF(zero, em1);
  evg = MINF(em1, evg);
  // :426-478
  const float qflx_evap = evg;
  float qflx_in_soil = (one - frac_h2osfc) * (qflx_top_soil - qflx_surf);
  qflx_in_soil = qflx_in_soil - (one - frac_h2osfc) * qflx_evap;
  float mh = hks[1];
  if (hks[2] < mh) mh = hks[2];
  if (hks[3] < mh) mh = hks[3];
  const float qinmax = (one - fsat) * mh;
  const float qflx_infl_excess = MAXF(zero, qflx_in_soil - (one - frac_h2osfc) * qinmax);
  const float qflx_infl = qflx_in_soil - qflx_infl_excess;
  qflx_surf = qflx_surf + qflx_infl_excess;
  // :492-508
  float zwtmm = 1000.0f * s.zwt;
  int jwt = jwt_of<L>(s.zwt, g);
  // :517-567  equilibrium profile
  float zq[L + 2];
#pragma unroll
  for (int i = 1; i <= L; i++) {
    float vol_eq;
    const float e = one - one / bsw[i];
    if (zwtmm <= zi[i - 1]) {
      vol_eq = ts[i];
    } else {
      // (-psi + zwtmm - zi(I-1)) / (-psi)  ** (1 - 1/bsw): temp0 of both cases
      const float temp0 = h9m::powf((((-psi[i]) + zwtmm - zi[i - 1]) / (-psi[i])), e, T);
      if ((zwtmm < zi[i]) && (zwtmm > zi[i - 1])) {
        const float tempi = one;
        const float voleq1 = psi[i] * ts[i] / e / (zwtmm - zi[i - 1]) * (tempi - temp0);
        vol_eq = (voleq1 * (zwtmm - zi[i - 1]) + ts[i] * (zi[i] - zwtmm)) / (zi[i] - zi[i - 1]);
        vol_eq = MINF(ts[i], vol_eq);
        vol_eq = MAXF(vol_eq, zero);
      } else {
        const float tempi = h9m::powf(((-psi[i] + zwtmm - zi[i]) / (-psi[i])), e, T);
        vol_eq = psi[i] * ts[i] / e / (zi[i] - zi[i - 1]) * (tempi - temp0);
        vol_eq = MAXF(vol_eq, 0.0f);
        vol_eq = MINF(ts[i], vol_eq);
      }
    }
    zq[i] = psi[i] * h9m::powf(MAXF(vol_eq / ts[i], 0.01f), -bsw[i], T);
    zq[i] = MAXF(smpmin, zq[i]);
  }
  // :574-590  aquifer node when the water table is below the column
  zq[L + 1] = zero;
  if (jwt == L) {
    const float e = 1.0f - 1.0f / bsw[L];
    const float tempi = 1.0f;
    const float temp0 = h9m::powf(((-psi[L] + zwtmm - zi[L]) / (-psi[L])), e, T);
    float v = psi[L] * ts[L] / e / (zwtmm - zi[L]) * (tempi - temp0);
    v = MAXF(v, 0.0f);
    v = MINF(ts[L], v);
    float z = psi[L] * h9m::powf(MAXF(v / ts[L], 0.01f), -bsw[L], T);
    zq[L + 1] = MAXF(smpmin, z);
  }
  // :598-639  conductivity and matric potential
  float hk[L + 1], dhkdw[L + 1], dsmpdw[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) {
    const int ip = (L < i + 1) ? L : i + 1;
    float s1 = 0.5f * (theta[i] + theta[ip]) / (0.5f * (ts[i] + ts[ip]));
    s1 = MINF(one, s1);
    const float s2 = hks[i] * h9m::powf(s1, 2.0f * bsw[i] + 2.0f, T);
    hk[i] = s1 * s2;
    dhkdw[i] = (2.0f * bsw[i] + 3.0f) * s2 * (one / (ts[i] + ts[ip]));
    float s_node = MAXF(theta[i] / ts[i], 0.01f);
    s_node = MINF(one, s_node);
    float sm = psi[i] * h9m::powf(s_node, -bsw[i], T);
    sm = MAXF(smpmin, sm);
    smp[i] = sm;
    dsmpdw[i] = (-bsw[i]) * sm / (s_node * ts[i]);
  }
  // :645-650
  const float zcA = 0.5f * (zwtmm + zc[L]);
  const float dzA = (jwt < L) ? dz[L] : zwtmm - zc[L];
  // tridiagonal system, rows 1..L+1 (:661-799)
  float amx[L + 2], bmx[L + 2], cmx[L + 2], rmx[L + 2];
  {
    const float den = (zc[2] - zc[1]);
    const float dzq = (zq[2] - zq[1]);
    const float num = (smp[2] - smp[1]) - dzq;
    const float qout = -hk[1] * num / den;
    const float dqodw1 = -(-hk[1] * dsmpdw[1] + num * dhkdw[1]) / den;
    const float dqodw2 = -(hk[1] * dsmpdw[2] + num * dhkdw[1]) / den;
    rmx[1] = qflx_infl - qout - tran * s.rootr[1];
    amx[1] = zero;
    bmx[1] = dz[1] / dt + dqodw1;
    cmx[1] = dqodw2;
  }
#pragma unroll
  for (int i = 2; i <= L - 1; i++) {
    float den = zc[i] - zc[i - 1];
    float dzq = zq[i] - zq[i - 1];
    float num = smp[i] - smp[i - 1] - dzq;
    const float qin = -hk[i - 1] * num / den;
    const float dqidw0 = -(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]) / den;
    const float dqidw1 = -(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]) / den;
    den = zc[i + 1] - zc[i];
    dzq = zq[i + 1] - zq[i];
    num = (smp[i + 1] - smp[i]) - dzq;
    const float qout = -hk[i] * num / den;
    const float dqodw1 = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
    const float dqodw2 = -(hk[i] * dsmpdw[i + 1] + num * dhkdw[i]) / den;
    rmx[i] = qin - qout - tran * s.rootr[i];
    amx[i] = -dqidw0;
    bmx[i] = dz[i] / dt - dqidw1 + dqodw1;
    cmx[i] = dqodw2;
  }
  {
    const int i = L;
    float den = zc[i] - zc[i - 1];
    float dzq = zq[i] - zq[i - 1];
    float num = smp[i] - smp[i - 1] - dzq;
    const float qin = -hk[i - 1] * num / den;
    const float dqidw0 = -(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]) / den;
    const float dqidw1 = -(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]) / den;
    amx[i] = -dqidw0;
    if (i > jwt) {                 // water table inside the column
      const float qout = zero, dqodw1 = zero;
      rmx[i] = qin - qout - tran * s.rootr[i];
      bmx[i] = dz[i] / dt - dqidw1 + dqodw1;
      cmx[i] = zero;
      rmx[i + 1] = zero;
      amx[i + 1] = zero;
      bmx[i + 1] = dzA / dt;
      cmx[i + 1] = zero;
    } else {                       // below: aquifer row
      float s_node = MAXF(0.5f * (one + theta[i] / ts[i]), 0.01f);
      s_node = MINF(one, s_node);
      float smp1 = psi[i] * h9m::powf(s_node, -bsw[i], T);
      smp1 = MAXF(smpmin, smp1);
      const float dsmpdw1 = -bsw[i] * smp1 / (s_node * ts[i]);
      den = zcA - zc[i];
      dzq = zq[i + 1] - zq[i];
      num = smp1 - smp[i] - dzq;
      const float qout = -hk[i] * num / den;
      const float dqodw1 = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
      const float dqodw2 = -(hk[i] * dsmpdw1 + num * dhkdw[i]) / den;
      rmx[i] = qin - qout - tran * s.rootr[i];
      bmx[i] = dz[i] / dt - dqidw1 + dqodw1;
      cmx[i] = dqodw2;
      const float qin1 = qout;
      const float dqidw0b = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
      const float dqidw1b = -(hk[i] * dsmpdw1 + num * dhkdw[i]) / den;
      const float qout1 = zero, dqodw1b = zero;
      rmx[i + 1] = qin1 - qout1;
      amx[i + 1] = -dqidw0b;
      bmx[i + 1] = dzA / dt - dqidw1b + dqodw1b;
      cmx[i + 1] = zero;
    }
  }
  // :806-837 Thomas algorithm
  if (bmx[1] == 0.0f) { errval = bmx[1]; return 1; }
  float dwat2[L + 2], GAM[L + 2];
  float BET = bmx[1];
  dwat2[1] = rmx[1] / BET;
  bool zero_pivot = false;
#pragma unroll
  for (int i = 2; i <= L + 1; i++) {
    GAM[i] = cmx[i - 1] / BET;
    BET = bmx[i] - amx[i] * GAM[i];
    if (BET == 0.0f && !zero_pivot) { zero_pivot = true; errval = (float)i; }
    dwat2[i] = (rmx[i] - amx[i] * dwat2[i - 1]) / BET;
  }
  if (zero_pivot) return 2;
#pragma unroll
  for (int i = L; i >= 1; i--) dwat2[i] = dwat2[i] - GAM[i + 1] * dwat2[i + 1];
  // :845-850
#pragma unroll
  for (int i = 1; i <= L; i++) h2o[i] = h2o[i] + dwat2[i] * dz[i];
  // :856-904 recharge
  float qcharge;
  if (jwt < L) {
    float th_j = zero, ts_j = one, hks_j = zero, bsw_j = zero, smp_m = zero, zq_m = zero, zc_j = zero;
#pragma unroll
    for (int i = 1; i <= L; i++) {
      if (i == jwt + 1) { th_j = theta[i]; ts_j = ts[i]; hks_j = hks[i]; bsw_j = bsw[i]; }
      if (i == (jwt > 1 ? jwt : 1)) { smp_m = smp[i]; zq_m = zq[i]; }
      if (i == jwt) zc_j = zc[i];
    }
    const float wh_zwt = zero;
    const float s_node = MAXF(th_j / ts_j, 0.01f);
    const float s1 = MINF(one, s_node);
    const float ka = hks_j * h9m::powf(s1, 2.0f * bsw_j + 3.0f, T);
    const float smp1 = MAXF(smpmin, smp_m);
    const float wh = smp1 - zq_m;
    if (jwt == 0)
      qcharge = -ka * (wh_zwt - wh) / (zwtmm + one);
    else
      qcharge = -ka * (wh_zwt - wh) / ((zwtmm - zc_j) * 2.0f);
    qcharge = MAXF(-10.0f / dt, qcharge);
    qcharge = MINF(10.0f / dt, qcharge);
  } else {
    qcharge = dwat2[L + 1] * dzA / dt;
  }
  // :923-1009 water table update from recharge
  jwt = jwt_of<L>(s.zwt, g);
  float rous = ts[L] * (one - h9m::powf((one + zwtmm / (-psi[L])), (-one / bsw[L]), T));
  rous = MAXF(rous, 0.02f);
  if (jwt == L) {
    s.wa = s.wa + qcharge * dt;
    s.zwt = s.zwt - (qcharge * dt) / 1000.0f / rous;
  } else {
    float qcharge_tot = qcharge * dt;
    if (qcharge_tot > zero) {          // rising: I = jwt+1 .. 1
      bool active = true;
#pragma unroll
      for (int i = L; i >= 1; i--) {
        if (active && i <= jwt + 1) {
          float s_y = ts[i] * (one - h9m::powf((one + zwtmm / (-psi[i])), (-one / bsw[i]), T));
          s_y = MAXF(s_y, 0.02f);
          float qcl = MINF(qcharge_tot, s_y * (zwtmm - zi[i - 1]));
          qcl = MAXF(qcl, zero);
          if (s_y > zero) s.zwt = s.zwt - qcl / s_y / 1000.0f;
          qcharge_tot = qcharge_tot - qcl;
          if (qcharge_tot <= zero) active = false;
        }
      }
    } else {                            // deepening: I = jwt+1 .. L
      bool active = true;
#pragma unroll
      for (int i = 1; i <= L; i++) {
        if (active && i >= jwt + 1) {
          float s_y = ts[i] * (one - h9m::powf((one + zwtmm / (-psi[i])), (-one / bsw[i]), T));
          s_y = MAXF(s_y, 0.02f);
          float qcl = MAXF(qcharge_tot, -s_y * (zi[i] - zwtmm));
          qcl = MINF(qcl, zero);
          qcharge_tot = qcharge_tot - qcl;
          if (qcharge_tot >= zero) {
            s.zwt = s.zwt - qcl / s_y / 1000.0f;
            active = false;
          } else {
            s.zwt = zi[i] / 1000.0f;
          }
        }
      }
      if (qcharge_tot > zero) s.zwt = s.zwt - qcharge_tot / 1000.0f / rous;
    }
    jwt = jwt_of<L>(s.zwt, g);
  }
  // :1015-1035 baseflow
  zwtmm = 1000.0f * s.zwt;
  float rsub_top = 5.5E-3f * h9m::expf(-fff * s.zwt, T);
  rous = ts[L] * (one - h9m::powf((one + zwtmm / (-psi[L])), (-one / bsw[L]), T));
  rous = MAXF(rous, 0.02f);
  // :1048-1118
  if (jwt == L) {
    s.wa = s.wa - rsub_top * dt;
    s.zwt = s.zwt + (rsub_top * dt) / 1000.0f / rous;
    h2o[L] = h2o[L] + MAXF(0.0f, (s.wa - 5000.0f));
    s.wa = MINF(s.wa, 5000.0f);
  } else {
    float rsub_top_tot = -rsub_top * dt;
    if (rsub_top_tot > zero) { errval = rsub_top_tot; return 3; }
    bool active = true;
#pragma unroll
    for (int i = 1; i <= L; i++) {
      if (active && i >= jwt + 1) {
        float s_y = ts[i] * (one - h9m::powf((one + zwtmm / (-psi[i])), (-one / bsw[i]), T));
        s_y = MAXF(s_y, 0.02f);
        float rstl = MAXF(rsub_top_tot, -(s_y * (zi[i] - zwtmm)));
        rstl = MINF(rstl, zero);
        h2o[i] = h2o[i] + rstl;
        rsub_top_tot = rsub_top_tot - rstl;
        if (rsub_top_tot >= zero) {
          s.zwt = s.zwt - rstl / s_y / 1000.0f;
          active = false;
        } else {
          s.zwt = zi[i] / 1000.0f;
        }
      }
    }
    s.zwt = s.zwt - rsub_top_tot / 1000.0f / rous;
    s.wa = s.wa + rsub_top_tot;
    jwt = jwt_of<L>(s.zwt, g);
  }
  // :1122-1123
  s.zwt = MAXF(0.0f, s.zwt);
  s.zwt = MINF(80.0f, s.zwt);
  // :1131-1137 saturation excess, bottom-up bucket
#pragma unroll
  for (int i = L; i >= 2; i--) {
    const float cap = MAXF(0.01f, ts[i]) * dz[i];
    const float xsi = MAXF(h2o[i] - cap, zero);
    h2o[i] = MINF(cap, h2o[i]);
    h2o[i - 1] = h2o[i - 1] + xsi;
  }
  // :1144-1152
  const float xs1 = MAXF(MAXF(h2o[1], zero) - MAXF(zero, (ts[1] * dz[1])), zero);
  h2o[1] = MINF(MAXF(zero, ts[1] * dz[1]), h2o[1]);
  const float qflx_rsub_sat = xs1 / dt;
  // :1161-1174 watmin top-down
#pragma unroll
  for (int i = 1; i <= L - 1; i++) {
    float xs = zero;
    if (h2o[i] < watmin) {
      xs = watmin - h2o[i];
      if (i == jwt) s.zwt = s.zwt + xs / MAXF(0.01f, ts[i]) / 1000.0f;
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
  rsub_top = rsub_top - xs / dt;
  // :1221-1236
  float w1 = ((1.0f - frac_h2osfc) * (qflx_surf + evg + tran) + rsub_top + qflx_rsub_sat) * dt + s.wa;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    w1 = w1 + h2o[i];
    theta[i] = MAXF(h2o[i], 1.0E-6f) / (dz[i] * rhow / 1000.0f);
  }
  // :1244
  if (fabsf(w1 - w0) > 0.1f) { errval = w1 - w0; return 4; }
  // :1282-1283
  rnf_sum = rnf_sum + qflx_surf * dt;
  rnf_sum = rnf_sum + rsub_top * dt;
  return 0;
}

// GROW.f90:55-201 (nplants = 1, iGPT = 1).  rootr(L+1) is zeroed by the
// caller's state write-back.
template <int L>
__device__ __forceinline__ void grow_day(const Geo<L> &g, float tas, St<L> &s, float &npp,
                                         const h9m::Tabs &T) {
  float w_i = zero;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    float w = (-150000.0f - s.smp[i]) / (-150000.0f - (-50000.0f));
    w = MAXF(zero, w);
    w = MINF(one, w);
    w_i = w_i + s.rootr[i] * w;
  }
  float fT;
  if ((tas - tf) > 18.0f) {
    const float a = fabsf(tas - tf - 18.0f) / 21.0f;
    fT = one - a * a;
  } else {
    const float a = fabsf(tas - tf - 18.0f) / 25.0f;
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
  s.plen = h9m::powf(400.0f * s.pm / 3.142E-3f, one / 3.0f, T);
  const float dLAI = dplant_foliage_mass * sla1;
  s.LAI = s.LAI + dLAI;
  s.LAI = MAXF(0.001f, s.LAI);
  s.LAI_litter = s.LAI_litter + MAXF(zero, dLAI);
  s.rdepth = 0.3f * s.plen;
  const float decay = h9m::expf(log_0p1 / (s.rdepth / 10.0f), T);
  // decay ** (zi(I)/10) is shared by rows I and I+1: 9 powf instead of 16
  float pw_prev = h9m::powf(decay, g.zi[0] / 10.0f, T);
#pragma unroll
  for (int i = 1; i <= L; i++) {
    const float pw = h9m::powf(decay, g.zi[i] / 10.0f, T);
    s.rootr[i] = zero + (1.0f - pw) - (1.0f - pw_prev);
    pw_prev = pw;
  }
  npp = zero + dplant_mass;
  s.LAI_litter = s.LAI_litter - 0.02f * s.LAI_litter;
}

// INIT.f90:707-811 for one cell (smp = 0).
template <int L>
__device__ __forceinline__ void init_cell(const Geo<L> &g, const Par<L> &p, St<L> &s,
                                          float *h2o_ma, const h9m::Tabs &T) {
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = 0.4f * p.ts[i] * g.dz[i] * rhow / 1000.0f;
    h2o_ma[i] = 0.4f * 0.1f * g.dz[i] * rhow / 1000.0f;
    s.smp[i] = zero;
  }
  s.zwt = (g.zi[L] + 5000.0f) / 1000.0f;
  s.wa = 4000.0f;
  s.LAI_litter = 0.001f;
  s.pm = 1.0f;
  s.pfm = 0.0435f;
  s.plen = h9m::powf(400.0f * s.pm / 3.142E-3f, one / 3.0f, T);
  s.LAI = zero + s.pfm * sla1 / 1.0f;
  s.rdepth = 0.3f * s.plen;
  const float decay = h9m::expf(log_0p1 / (s.rdepth / 10.0f), T);
#pragma unroll
  for (int i = 1; i <= L; i++)
    s.rootr[i] = zero + (1.0f - h9m::powf(decay, g.zi[i] / 10.0f, T)) -
                 (1.0f - h9m::powf(decay, g.zi[i - 1] / 10.0f, T));
}

}  // namespace h9k
