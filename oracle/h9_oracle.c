/*
 * TEST INFRASTRUCTURE ONLY -- the CPU oracle (plain C restatement).
 * See h9_oracle.h.  Every block cites the reference line it restates.
 *
 * Evaluation-order rules followed throughout (pinned by tests/golden):
 *   - Fortran evaluates a*b/c*d left to right; C does the same.
 *   - MIN(a,b) -> (a < b ? a : b), MAX(a,b) -> (a > b ? a : b): flang
 *     lowers the intrinsics to compare+select in this argument order.
 *   - x**2 -> x*x; real**real -> powf; EXP -> expf; LOG(0.1) folded.
 *   - Arrays are 1-based here (index 0 unused) to mirror the Fortran.
 */
#include "h9_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define LM H9O_LMAX

static inline float MAXF(float a, float b) { return a > b ? a : b; }
static inline float MINF(float a, float b) { return a < b ? a : b; }

/* SHARED.f90:308-367, constants folded in float as flang does */
static const float zero = 0.0f, one = 1.0f;
static const float rhow = 1000.0f;
static const float gasc = 8.314510f;
static const float rgas = 0x1.1f0c7cp+8f;    /* 1000*gasc/mair   */
static const float deltx = 0x1.3738bcp-1f;   /* one/mrat - one   */
static const float stbo = 5.67E-8f;
static const float tf = 273.16f;
static const float smpmin = -1.0E8f;
static const float trunc_ = 1.0E-8f;
static const float cp = 1010.0f;            /* HYDROLOGY.f90:35  */
static const float watmin = 0.01f;          /* HYDROLOGY.f90:135 */
static const float sla1 = 23.0E-3f;         /* INIT.f90:154      */
static const float log_0p1 = -0x1.26bb1cp+1f; /* LOG(0.1), GROW.f90:176 */

typedef struct {
  int L;
  float dt;
  float zi[LM + 2];   /* zi(0:L+1) */
  float dz[LM + 2];   /* dz(1:L+1) from INIT; dz(L+1) rewritten per call */
  float zc[LM + 2];
} geom_t;

typedef struct {
  float theta_s[LM + 2], hksat[LM + 2], bsw[LM + 2], psi_s[LM + 2];
  float fmax;
} par_t;

typedef struct {
  float h2o[LM + 2], h2o_ma[LM + 2], smp[LM + 2], rootr[LM + 3];
  float zwt, wa, LAI, LAI_litter, pm, pfm, plen, rdepth;
} st_t;

typedef struct {  /* per-day driver variables, HYBRID9.f90:168-184 */
  float tak, rh, Rnet, PAR, forc_rain, lamb, huss, ps, tas;
} day_t;

int h9o_state_size(int L) { return 4 * L + 1 + 8; }

static void geom_init(geom_t *g, int L, int nisurf, const float *zi) {
  g->L = L;
  for (int i = 0; i <= L + 1; i++) g->zi[i] = zi[i];
  g->dt = 86400.0f / (float)nisurf;                   /* INIT.f90:214 */
  for (int i = 1; i <= L + 1; i++) g->dz[i] = g->zi[i] - g->zi[i - 1];
  for (int i = 1; i <= L + 1; i++) g->zc[i] = g->zi[i] - g->dz[i] / 2.0f;
}

static void load_par(par_t *p, const float *params, int ncell, int L, int c) {
  for (int i = 1; i <= L; i++) {
    p->theta_s[i] = params[0 * ncell * L + c * L + i - 1];
    p->hksat[i] = params[1 * ncell * L + c * L + i - 1];
    p->bsw[i] = params[2 * ncell * L + c * L + i - 1];
    p->psi_s[i] = params[3 * ncell * L + c * L + i - 1];
  }
  p->fmax = params[4 * ncell * L + c];
}

/* packed state <-> struct (refcase.state_fields order) */
static void load_st(st_t *s, const float *st, int ncell, int L, int c) {
  const float *q = st;
  for (int i = 1; i <= L; i++) s->h2o[i] = q[c * L + i - 1];
  q += ncell * L;
  for (int i = 1; i <= L; i++) s->h2o_ma[i] = q[c * L + i - 1];
  q += ncell * L;
  for (int i = 1; i <= L; i++) s->smp[i] = q[c * L + i - 1];
  q += ncell * L;
  for (int i = 1; i <= L + 1; i++) s->rootr[i] = q[c * (L + 1) + i - 1];
  q += ncell * (L + 1);
  s->zwt = q[c]; q += ncell;
  s->wa = q[c]; q += ncell;
  s->LAI = q[c]; q += ncell;
  s->LAI_litter = q[c]; q += ncell;
  s->pm = q[c]; q += ncell;
  s->pfm = q[c]; q += ncell;
  s->plen = q[c]; q += ncell;
  s->rdepth = q[c];
}

static void store_st(const st_t *s, float *st, int ncell, int L, int c) {
  float *q = st;
  for (int i = 1; i <= L; i++) q[c * L + i - 1] = s->h2o[i];
  q += ncell * L;
  for (int i = 1; i <= L; i++) q[c * L + i - 1] = s->h2o_ma[i];
  q += ncell * L;
  for (int i = 1; i <= L; i++) q[c * L + i - 1] = s->smp[i];
  q += ncell * L;
  for (int i = 1; i <= L + 1; i++) q[c * (L + 1) + i - 1] = s->rootr[i];
  q += ncell * (L + 1);
  q[c] = s->zwt; q += ncell;
  q[c] = s->wa; q += ncell;
  q[c] = s->LAI; q += ncell;
  q[c] = s->LAI_litter; q += ncell;
  q[c] = s->pm; q += ncell;
  q[c] = s->pfm; q += ncell;
  q[c] = s->plen; q += ncell;
  q[c] = s->rdepth;
}

/* INIT.f90:707-811 */
static void init_cell(st_t *s, const geom_t *g, const par_t *p) {
  const int L = g->L;
  memset(s, 0, sizeof(*s));
  for (int i = 1; i <= L; i++) {
    s->h2o[i] = 0.4f * p->theta_s[i] * g->dz[i] * rhow / 1000.0f;
    s->h2o_ma[i] = 0.4f * 0.1f * g->dz[i] * rhow / 1000.0f;
    s->smp[i] = zero;
  }
  s->zwt = (g->zi[L] + 5000.0f) / 1000.0f;
  s->wa = 4000.0f;
  s->LAI_litter = 0.001f;
  s->LAI = zero;
  for (int i = 1; i <= L + 1; i++) s->rootr[i] = zero;
  s->pm = 1.0f;
  s->pfm = 0.0435f;
  s->plen = powf(400.0f * s->pm / 3.142E-3f, one / 3.0f);
  s->LAI = s->LAI + s->pfm * sla1 / 1.0f;             /* plot_area = 1 */
  s->rdepth = 0.3f * s->plen;
  float decay = expf(log_0p1 / (s->rdepth / 10.0f));
  for (int i = 1; i <= L; i++)
    s->rootr[i] = s->rootr[i] + (1.0f - powf(decay, g->zi[i] / 10.0f)) -
                  (1.0f - powf(decay, g->zi[i - 1] / 10.0f));
}

int h9o_init_state(int ncell, int L, const float *zi, const float *params,
                   float *state) {
  if (ncell < 0 || L < 3 || L > LM) return H9O_ERR_ARGS;
  geom_t g;
  geom_init(&g, L, 48, zi);
  for (int c = 0; c < ncell; c++) {
    par_t p;
    st_t s;
    load_par(&p, params, ncell, L, c);
    init_cell(&s, &g, &p);
    store_st(&s, state, ncell, L, c);
  }
  return H9O_OK;
}

static int jwt_of(float zwt, const geom_t *g) {   /* HYDROLOGY.f90:499-508 */
  int jwt = g->L;
  for (int i = 1; i <= g->L; i++) {
    if (zwt <= (g->zi[i] / 1000.0f)) { jwt = i - 1; break; }
  }
  return jwt;
}

/* HYDROLOGY.f90:141-1283 for one cell and one substep.
 * theta[] (1-based) receives the end-of-step volumetric water
 * (HYDROLOGY.f90:1233) used by the day driver. */
static int hydrology(geom_t *g, const par_t *p, const day_t *d, st_t *s,
                     float *rnf_sum, float *theta, float *tran_o,
                     float *evg_o, float *errval) {
  const int L = g->L;
  const float dt = g->dt;
  const float *zi = g->zi, *dz = g->dz, *zc = g->zc;
  float *h2o = s->h2o, *smp = s->smp;
  const float *ts = p->theta_s, *hks = p->hksat, *bsw = p->bsw, *psi = p->psi_s;
  float theta_ma[LM + 2], eff_porosity[LM + 2], vol_eq[LM + 3], zq[LM + 3];
  float hk[LM + 2], dhkdw[LM + 2], dsmpdw[LM + 3];
  float qin[LM + 3], qout[LM + 3], dqidw0[LM + 3], dqidw1[LM + 3];
  float dqodw1[LM + 3], dqodw2[LM + 3], amx[LM + 3], bmx[LM + 3];
  float cmx[LM + 3], rmx[LM + 3], dwat2[LM + 3], GAM[LM + 3], rnff[LM + 3];
  int jwt;

  /* :141-151 */
  float w0 = d->forc_rain * dt + s->wa;
  for (int i = 1; i <= L; i++) {
    w0 = w0 + h2o[i];
    theta[i] = h2o[i] / (dz[i] * rhow / 1.0E3f);
    theta_ma[i] = s->h2o_ma[i] / (dz[i] * rhow / 1.0E3f);
  }
  (void)theta_ma;
  /* :161-212 */
  const float qflx_top_soil = d->forc_rain;
  const float hkdepth = one / 2.5f;
  const float fff = 1.0f / hkdepth;
  const float wtfact = p->fmax;
  const float fsat = wtfact * expf(-0.5f * fff * s->zwt);
  float qflx_surf = fsat * qflx_top_soil;
  const float frac_h2osfc = zero;
  /* :232-263 */
  const float tak = d->tak;
  const float tsv = tak * (one + d->huss * deltx);
  const float rho = d->ps / (rgas * tsv);
  const float ex = expf((17.27f * (tak - tf)) / (tak - tf + 237.3f));
  float desatdT = (4098.0f * (0.6108f * ex)) /
                  ((tak - tf + 237.3f) * (tak - tf + 237.3f));
  desatdT = desatdT * 18.0f / (gasc * tak);
  float esat = 0.6108f * ex;
  esat = esat * 18.0f / (gasc * tak);
  const float VDD = esat * (one - d->rh / 100.0f);
  const float gamma = (cp * d->ps / (d->lamb * 0.622f)) * (18.0E-3f / (gasc * tak));
  /* :269-276, previous-step smp */
  float beta_save = zero, beta;
  for (int i = 1; i <= L; i++) {
    beta = one - (smp[i] - zc[i]) / (-150000.0f);
    beta = MINF(one, beta);
    beta = MAXF(zero, beta);
    beta_save = beta_save + s->rootr[i] * beta;
  }
  beta = beta_save;
  /* :283-295 */
  const float LAI = s->LAI, PAR = d->PAR;
  float rsc;
  if ((LAI > zero) && (beta > zero) && (PAR > zero))
    rsc = (1.0f / (PAR / (PAR + 300.0f))) * 400.0f /
          (2.0f * LAI * beta * powf(2.8f, -80.0f * MAXF(zero, VDD) / rho));
  else
    rsc = 1.0E6f;
  rsc = MAXF(rsc, 1.0f / ((LAI / 2.7f) * 0.9f / (rho * 1.0E3f / 18.0f)));
  /* :302-318 */
  const float rac = (LAI > zero) ? 25.0f / (2.0f * LAI) : 1.0E6f;
  float raa, ras;
  if (LAI <= 4.0f) {
    raa = 0.25f * LAI * 42.0f + 0.25f * (4.0f - LAI) * 34.0f;
    ras = 0.25f * LAI * 128.0f + 0.25f * (4.0f - LAI) * 49.0f;
  } else {
    raa = 42.0f;
    ras = 128.0f;
  }
  /* :325-331 */
  float rss;
  if (theta[1] <= 0.15f)
    rss = (10.0f + 1000.0f * s->LAI_litter) * expf(0.3563f * 100.0f * (0.15f - theta[1]));
  else
    rss = (10.0f + 1000.0f * s->LAI_litter * (1.0f - theta[1] / ts[1]));
  /* :335-389 */
  const float Rnet = d->Rnet;
  const float Rnets = Rnet * expf(-0.7f * LAI);
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
  const float tran = LEc * 1.0E3f / (rhow * d->lamb);
  float evg = LEs * 1.0E3f / (rhow * d->lamb);
  /* :396-400 */
  float em1 = dz[1] * (theta[1] - watmin) / dt - tran * s->rootr[1];
  em1 = MAXF(zero, em1);
  evg = MINF(em1, evg);
  /* :426-478 */
  for (int i = 1; i <= L; i++) eff_porosity[i] = MAXF(0.01f, ts[i]);
  const float qflx_evap = evg;
  float qflx_in_soil = (one - frac_h2osfc) * (qflx_top_soil - qflx_surf);
  qflx_in_soil = qflx_in_soil - (one - frac_h2osfc) * qflx_evap;
  float mh = hks[1];                                   /* MINVAL(hksat(1:3)) */
  if (hks[2] < mh) mh = hks[2];
  if (hks[3] < mh) mh = hks[3];
  const float qinmax = (one - fsat) * mh;
  float qflx_infl_excess = MAXF(zero, qflx_in_soil - (one - frac_h2osfc) * qinmax);
  const float qflx_infl = qflx_in_soil - qflx_infl_excess;
  qflx_surf = qflx_surf + qflx_infl_excess;
  /* :492-508 */
  float zwtmm = 1000.0f * s->zwt;
  jwt = jwt_of(s->zwt, g);
  /* :517-567 */
  for (int i = 1; i <= L; i++) {
    if (zwtmm <= zi[i - 1]) {
      vol_eq[i] = ts[i];
    } else if ((zwtmm < zi[i]) && (zwtmm > zi[i - 1])) {
      const float tempi = one;
      const float temp0 = powf((((-psi[i]) + zwtmm - zi[i - 1]) / (-psi[i])), (one - one / bsw[i]));
      const float voleq1 = psi[i] * ts[i] / (one - one / bsw[i]) / (zwtmm - zi[i - 1]) * (tempi - temp0);
      vol_eq[i] = (voleq1 * (zwtmm - zi[i - 1]) + ts[i] * (zi[i] - zwtmm)) / (zi[i] - zi[i - 1]);
      vol_eq[i] = MINF(ts[i], vol_eq[i]);
      vol_eq[i] = MAXF(vol_eq[i], zero);
    } else {
      const float tempi = powf(((-psi[i] + zwtmm - zi[i]) / (-psi[i])), (1.0f - 1.0f / bsw[i]));
      const float temp0 = powf(((-psi[i] + zwtmm - zi[i - 1]) / (-psi[i])), (1.0f - 1.0f / bsw[i]));
      vol_eq[i] = psi[i] * ts[i] / (1.0f - 1.0f / bsw[i]) / (zi[i] - zi[i - 1]) * (tempi - temp0);
      vol_eq[i] = MAXF(vol_eq[i], 0.0f);
      vol_eq[i] = MINF(ts[i], vol_eq[i]);
    }
    zq[i] = psi[i] * powf(MAXF(vol_eq[i] / ts[i], 0.01f), -bsw[i]);
    zq[i] = MAXF(smpmin, zq[i]);
  }
  /* :574-590 */
  if (jwt == L) {
    const int i = L;
    const float tempi = 1.0f;
    const float temp0 = powf(((-psi[i] + zwtmm - zi[i]) / (-psi[i])), (1.0f - 1.0f / bsw[i]));
    vol_eq[i + 1] = psi[i] * ts[i] / (1.0f - 1.0f / bsw[i]) / (zwtmm - zi[i]) * (tempi - temp0);
    vol_eq[i + 1] = MAXF(vol_eq[i + 1], 0.0f);
    vol_eq[i + 1] = MINF(ts[i], vol_eq[i + 1]);
    zq[i + 1] = psi[i] * powf(MAXF(vol_eq[i + 1] / ts[i], 0.01f), -bsw[i]);
    zq[i + 1] = MAXF(smpmin, zq[i + 1]);
  }
  /* :598-639 */
  for (int i = 1; i <= L; i++) {
    const int ip = (L < i + 1) ? L : i + 1;
    float s1 = 0.5f * (theta[i] + theta[ip]) / (0.5f * (ts[i] + ts[ip]));
    s1 = MINF(one, s1);
    const float s2 = hks[i] * powf(s1, 2.0f * bsw[i] + 2.0f);
    hk[i] = s1 * s2;
    dhkdw[i] = (2.0f * bsw[i] + 3.0f) * s2 * (one / (ts[i] + ts[ip]));
    float s_node = MAXF(theta[i] / ts[i], 0.01f);
    s_node = MINF(one, s_node);
    smp[i] = psi[i] * powf(s_node, -bsw[i]);
    smp[i] = MAXF(smpmin, smp[i]);
    dsmpdw[i] = (-bsw[i]) * smp[i] / (s_node * ts[i]);
  }
  /* :645-650 (module scratch zc(L+1), dz(L+1)) */
  g->zc[L + 1] = 0.5f * (zwtmm + zc[L]);
  if (jwt < L) g->dz[L + 1] = dz[L];
  else g->dz[L + 1] = zwtmm - zc[L];
  /* :661-675 */
  {
    const int i = 1;
    qin[i] = qflx_infl;
    const float den = (zc[i + 1] - zc[i]);
    const float dzq = (zq[i + 1] - zq[i]);
    const float num = (smp[i + 1] - smp[i]) - dzq;
    qout[i] = -hk[i] * num / den;
    dqodw1[i] = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
    dqodw2[i] = -(hk[i] * dsmpdw[i + 1] + num * dhkdw[i]) / den;
    rmx[i] = qin[i] - qout[i] - tran * s->rootr[i];
    amx[i] = zero;
    bmx[i] = dz[i] / dt + dqodw1[i];
    cmx[i] = dqodw2[i];
  }
  /* :679-703 */
  for (int i = 2; i <= L - 1; i++) {
    float den = zc[i] - zc[i - 1];
    float dzq = zq[i] - zq[i - 1];
    float num = smp[i] - smp[i - 1] - dzq;
    qin[i] = -hk[i - 1] * num / den;
    dqidw0[i] = -(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]) / den;
    dqidw1[i] = -(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]) / den;
    den = zc[i + 1] - zc[i];
    dzq = zq[i + 1] - zq[i];
    num = (smp[i + 1] - smp[i]) - dzq;
    qout[i] = -hk[i] * num / den;
    dqodw1[i] = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
    dqodw2[i] = -(hk[i] * dsmpdw[i + 1] + num * dhkdw[i]) / den;
    rmx[i] = qin[i] - qout[i] - tran * s->rootr[i];
    amx[i] = -dqidw0[i];
    bmx[i] = dz[i] / dt - dqidw1[i] + dqodw1[i];
    cmx[i] = dqodw2[i];
  }
  /* :710-799 */
  {
    const int i = L;
    if (i > jwt) {
      const float den = zc[i] - zc[i - 1];
      const float dzq = zq[i] - zq[i - 1];
      const float num = smp[i] - smp[i - 1] - dzq;
      qin[i] = -hk[i - 1] * num / den;
      dqidw0[i] = -(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]) / den;
      dqidw1[i] = -(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]) / den;
      qout[i] = zero;
      dqodw1[i] = zero;
      rmx[i] = qin[i] - qout[i] - tran * s->rootr[i];
      amx[i] = -dqidw0[i];
      bmx[i] = dz[i] / dt - dqidw1[i] + dqodw1[i];
      cmx[i] = zero;
      rmx[i + 1] = zero;
      amx[i + 1] = zero;
      bmx[i + 1] = dz[i + 1] / dt;
      cmx[i + 1] = zero;
    } else {
      float s_node = MAXF(0.5f * (one + theta[i] / ts[i]), 0.01f);
      s_node = MINF(one, s_node);
      float smp1 = psi[i] * powf(s_node, -bsw[i]);
      smp1 = MAXF(smpmin, smp1);
      const float dsmpdw1 = -bsw[i] * smp1 / (s_node * ts[i]);
      float den = zc[i] - zc[i - 1];
      float dzq = zq[i] - zq[i - 1];
      float num = smp[i] - smp[i - 1] - dzq;
      qin[i] = -hk[i - 1] * num / den;
      dqidw0[i] = -(-hk[i - 1] * dsmpdw[i - 1] + num * dhkdw[i - 1]) / den;
      dqidw1[i] = -(hk[i - 1] * dsmpdw[i] + num * dhkdw[i - 1]) / den;
      den = zc[i + 1] - zc[i];
      dzq = zq[i + 1] - zq[i];
      num = smp1 - smp[i] - dzq;
      qout[i] = -hk[i] * num / den;
      dqodw1[i] = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
      dqodw2[i] = -(hk[i] * dsmpdw1 + num * dhkdw[i]) / den;
      rmx[i] = qin[i] - qout[i] - tran * s->rootr[i];
      amx[i] = -dqidw0[i];
      bmx[i] = dz[i] / dt - dqidw1[i] + dqodw1[i];
      cmx[i] = dqodw2[i];
      qin[i + 1] = qout[i];
      dqidw0[i + 1] = -(-hk[i] * dsmpdw[i] + num * dhkdw[i]) / den;
      dqidw1[i + 1] = -(hk[i] * dsmpdw1 + num * dhkdw[i]) / den;
      qout[i + 1] = zero;
      dqodw1[i + 1] = zero;
      rmx[i + 1] = qin[i + 1] - qout[i + 1];
      amx[i + 1] = -dqidw0[i + 1];
      bmx[i + 1] = dz[i + 1] / dt - dqidw1[i + 1] + dqodw1[i + 1];
      cmx[i + 1] = zero;
    }
  }
  /* :806-837 Thomas algorithm */
  if (bmx[1] == 0.0f) { *errval = bmx[1]; return H9O_ERR_TRIDIAG1; }
  float BET = bmx[1];
  dwat2[1] = rmx[1] / BET;
  for (int i = 2; i <= L + 1; i++) {
    GAM[i] = cmx[i - 1] / BET;
    BET = bmx[i] - amx[i] * GAM[i];
    if (BET == 0.0f) { *errval = (float)i; return H9O_ERR_TRIDIAG2; }
    dwat2[i] = (rmx[i] - amx[i] * dwat2[i - 1]) / BET;
  }
  for (int i = L; i >= 1; i--) dwat2[i] = dwat2[i] - GAM[i + 1] * dwat2[i + 1];
  /* :845-850 */
  for (int i = 1; i <= L; i++) h2o[i] = h2o[i] + dwat2[i] * dz[i];
  /* :856-904 */
  float qcharge;
  if (jwt < L) {
    const float wh_zwt = zero;
    const float s_node = MAXF(theta[jwt + 1] / ts[jwt + 1], 0.01f);
    const float s1 = MINF(one, s_node);
    const float ka = hks[jwt + 1] * powf(s1, 2.0f * bsw[jwt + 1] + 3.0f);
    const int jm = (jwt > 1) ? jwt : 1;
    const float smp1 = MAXF(smpmin, smp[jm]);
    const float wh = smp1 - zq[jm];
    if (jwt == 0)
      qcharge = -ka * (wh_zwt - wh) / (zwtmm + one);
    else
      qcharge = -ka * (wh_zwt - wh) / ((zwtmm - zc[jwt]) * 2.0f);
    qcharge = MAXF(-10.0f / dt, qcharge);
    qcharge = MINF(10.0f / dt, qcharge);
  } else {
    qcharge = dwat2[L + 1] * dz[L + 1] / dt;
  }
  /* :923-1009 */
  jwt = jwt_of(s->zwt, g);
  float rous = ts[L] * (one - powf((one + zwtmm / (-psi[L])), (-one / bsw[L])));
  rous = MAXF(rous, 0.02f);
  if (jwt == L) {
    s->wa = s->wa + qcharge * dt;
    s->zwt = s->zwt - (qcharge * dt) / 1000.0f / rous;
  } else {
    float qcharge_tot = qcharge * dt;
    if (qcharge_tot > zero) {
      for (int i = jwt + 1; i >= 1; i--) {
        float s_y = ts[i] * (one - powf((one + zwtmm / (-psi[i])), (-one / bsw[i])));
        s_y = MAXF(s_y, 0.02f);
        float qcl = MINF(qcharge_tot, s_y * (zwtmm - zi[i - 1]));
        qcl = MAXF(qcl, zero);
        if (s_y > zero) s->zwt = s->zwt - qcl / s_y / 1000.0f;
        qcharge_tot = qcharge_tot - qcl;
        if (qcharge_tot <= zero) break;
      }
    } else {
      for (int i = jwt + 1; i <= L; i++) {
        float s_y = ts[i] * (one - powf((one + zwtmm / (-psi[i])), (-one / bsw[i])));
        s_y = MAXF(s_y, 0.02f);
        float qcl = MAXF(qcharge_tot, -s_y * (zi[i] - zwtmm));
        qcl = MINF(qcl, zero);
        qcharge_tot = qcharge_tot - qcl;
        if (qcharge_tot >= zero) {
          s->zwt = s->zwt - qcl / s_y / 1000.0f;
          break;
        } else {
          s->zwt = zi[i] / 1000.0f;
        }
      }
      if (qcharge_tot > zero) s->zwt = s->zwt - qcharge_tot / 1000.0f / rous;
    }
    jwt = jwt_of(s->zwt, g);
  }
  /* :1015-1035 */
  zwtmm = 1000.0f * s->zwt;
  const float rsub_top_max = 5.5E-3f;
  float rsub_top = rsub_top_max * expf(-fff * s->zwt);
  rous = ts[L] * (one - powf((one + zwtmm / (-psi[L])), (-one / bsw[L])));
  rous = MAXF(rous, 0.02f);
  for (int i = 1; i <= L + 1; i++) rnff[i] = 0.0f;
  /* :1048-1118 */
  if (jwt == L) {
    s->wa = s->wa - rsub_top * dt;
    s->zwt = s->zwt + (rsub_top * dt) / 1000.0f / rous;
    h2o[L] = h2o[L] + MAXF(0.0f, (s->wa - 5000.0f));
    s->wa = MINF(s->wa, 5000.0f);
    rnff[L + 1] = rsub_top;
  } else {
    float rsub_top_tot = -rsub_top * dt;
    if (rsub_top_tot > zero) {
      *errval = rsub_top_tot;
      return H9O_ERR_RSUB_POS;
    } else {
      for (int i = jwt + 1; i <= L; i++) {
        float s_y = ts[i] * (one - powf((one + zwtmm / (-psi[i])), (-one / bsw[i])));
        s_y = MAXF(s_y, 0.02f);
        float rstl = MAXF(rsub_top_tot, -(s_y * (zi[i] - zwtmm)));
        rstl = MINF(rstl, zero);
        h2o[i] = h2o[i] + rstl;
        rnff[i] = -rstl;
        rsub_top_tot = rsub_top_tot - rstl;
        if (rsub_top_tot >= zero) {
          s->zwt = s->zwt - rstl / s_y / 1000.0f;
          break;
        } else {
          s->zwt = zi[i] / 1000.0f;
        }
      }
      s->zwt = s->zwt - rsub_top_tot / 1000.0f / rous;
      s->wa = s->wa + rsub_top_tot;
      rnff[L + 1] = rnff[L + 1] - rsub_top_tot;
    }
    jwt = jwt_of(s->zwt, g);
  }
  (void)rnff;
  /* :1122-1123 */
  s->zwt = MAXF(0.0f, s->zwt);
  s->zwt = MINF(80.0f, s->zwt);
  /* :1131-1137 */
  for (int i = L; i >= 2; i--) {
    const float xsi = MAXF(h2o[i] - eff_porosity[i] * dz[i], zero);
    h2o[i] = MINF(eff_porosity[i] * dz[i], h2o[i]);
    h2o[i - 1] = h2o[i - 1] + xsi;
  }
  /* :1144-1152 */
  const float xs1 = MAXF(MAXF(h2o[1], zero) - MAXF(zero, (ts[1] * dz[1])), zero);
  h2o[1] = MINF(MAXF(zero, ts[1] * dz[1]), h2o[1]);
  const float qflx_rsub_sat = xs1 / dt;
  /* :1161-1174 */
  float xs;
  for (int i = 1; i <= L - 1; i++) {
    if (h2o[i] < watmin) {
      xs = watmin - h2o[i];
      if (i == jwt) s->zwt = s->zwt + xs / eff_porosity[i] / 1000.0f;
    } else {
      xs = zero;
    }
    h2o[i] = h2o[i] + xs;
    h2o[i + 1] = h2o[i + 1] - xs;
  }
  /* :1180-1211 */
  if (h2o[L] < watmin) {
    xs = watmin - h2o[L];
    for (int j = L - 1; j >= 1; j--) {
      const float avail = MAXF(h2o[j] - watmin - xs, zero);
      if (avail >= xs) {
        h2o[L] = h2o[L] + xs;
        h2o[j] = h2o[j] - xs;
        xs = zero;
        break;
      } else {
        h2o[L] = h2o[L] + avail;
        h2o[j] = h2o[j] - avail;
        xs = xs - avail;
      }
    }
  } else {
    xs = zero;
  }
  h2o[L] = h2o[L] + xs;
  rsub_top = rsub_top - xs / dt;
  /* :1221-1236 */
  float w1 = ((1.0f - frac_h2osfc) * (qflx_surf + evg + tran) + rsub_top + qflx_rsub_sat) * dt + s->wa;
  for (int i = 1; i <= L; i++) {
    w1 = w1 + h2o[i];
    theta[i] = MAXF(h2o[i], 1.0E-6f) / (dz[i] * rhow / 1000.0f);
  }
  /* :1244-1274 */
  if (fabsf(w1 - w0) > 0.1f) { *errval = w1 - w0; return H9O_ERR_IMBALANCE; }
  /* :1282-1283 */
  *rnf_sum = *rnf_sum + qflx_surf * dt;
  *rnf_sum = *rnf_sum + rsub_top * dt;
  *tran_o = tran;
  *evg_o = evg;
  return H9O_OK;
}

/* GROW.f90:55-201 (nplants = 1, iGPT = 1) */
static void grow(const geom_t *g, const day_t *d, st_t *s, float *npp) {
  const int L = g->L;
  float w_i_save = zero, w_i;
  for (int i = 1; i <= L; i++) {
    w_i = (-150000.0f - s->smp[i]) / (-150000.0f - (-50000.0f));
    w_i = MAXF(zero, w_i);
    w_i = MINF(one, w_i);
    w_i_save = w_i_save + s->rootr[i] * w_i;
  }
  w_i = w_i_save;
  float fT;
  if ((d->tas - tf) > 18.0f) {
    const float a = fabsf(d->tas - tf - 18.0f) / 21.0f;
    fT = one - a * a;
  } else {
    const float a = fabsf(d->tas - tf - 18.0f) / 25.0f;
    fT = one - a * a;
    fT = MAXF(zero, fT);
    fT = MINF(one, fT);
  }
  for (int i = 1; i <= L + 1; i++) s->rootr[i] = zero;
  *npp = zero;
  const float grow_plant_mass = (1000.0f / 365.0f) * w_i * fT;
  const float grow_foliage_mass = grow_plant_mass / 3.3f;
  const float loss_plant_mass = (0.1f / 365.0f) * s->pm;
  float loss_foliage_mass = (1.0f / 365.0f) * s->pfm / MINF(one, MAXF(0.01f, w_i));
  if (w_i < 0.6f) loss_foliage_mass = 0.1f * s->pfm;
  const float dplant_mass = grow_plant_mass - loss_plant_mass;
  const float dplant_foliage_mass = grow_foliage_mass - loss_foliage_mass;
  s->pm = s->pm + dplant_mass;
  s->pfm = s->pfm + dplant_foliage_mass;
  s->plen = powf(400.0f * s->pm / 3.142E-3f, one / 3.0f);
  const float dLAI = dplant_foliage_mass * sla1;
  s->LAI = s->LAI + dLAI;
  s->LAI = MAXF(0.001f, s->LAI);
  s->LAI_litter = s->LAI_litter + MAXF(zero, dLAI);
  s->rdepth = 0.3f * s->plen;
  const float decay = expf(log_0p1 / (s->rdepth / 10.0f));
  for (int i = 1; i <= L; i++)
    s->rootr[i] = s->rootr[i] + (1.0f - powf(decay, g->zi[i] / 10.0f)) -
                  (1.0f - powf(decay, g->zi[i - 1] / 10.0f));
  *npp = *npp + dplant_mass;
  s->LAI_litter = s->LAI_litter - 0.02f * s->LAI_litter;
}

static int days_in_year(int y) {   /* INIT.f90:844-859 (Gregorian) */
  if (y % 4 != 0) return 365;
  if (y % 100 != 0) return 366;
  if (y % 400 != 0) return 365;
  return 366;
}

int h9o_run(int ncell, int L, int nisurf, int grow_on, int year0, int nyears,
            const float *zi, const float *params, const float *forcing,
            float *state, float *annual, int ntrace, const int *trace_cells,
            float *trace, int nthreads, h9o_error *err, int *cell_err) {
  if (ncell < 0 || L < 3 || L > LM || nisurf < 1 || nyears < 1) return H9O_ERR_ARGS;
  int ndays = 0;
  for (int y = 0; y < nyears; y++) ndays += days_in_year(year0 + y);
  const int nf = 12 + L;
  const int tw = 3 * L + 7;
  int first_code = 0, first_cell = ncell;
  h9o_error first = {0, -1, -1, -1, 0.0f};

#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1) if (nthreads != 1)
  for (int c = 0; c < ncell; c++) {
    geom_t g;
    geom_init(&g, L, nisurf, zi);
    par_t p;
    st_t s;
    load_par(&p, params, ncell, L, c);
    load_st(&s, state, ncell, L, c);
    float ts_sum = zero;
    for (int i = 1; i <= L; i++) ts_sum = ts_sum + p.theta_s[i];
    if (!(ts_sum > trunc_)) continue;          /* HYBRID9.f90:122-123 */
    int tslot = -1;
    for (int t = 0; t < ntrace; t++)
      if (trace_cells[t] == c) tslot = t;
    float *trow = (tslot >= 0 && trace) ? trace + (size_t)tslot * ndays * nisurf * tw : NULL;
    float theta[LM + 2] = {0};
    float npp = zero;
    int day = 0, code = 0;
    float errval = 0.0f;
    int eday = -1, estep = -1, edoy = -1;
    for (int y = 0; y < nyears && !code; y++) {
      const int nt = days_in_year(year0 + y);
      float npp_sum = zero, plant_mass_sum = zero, rnf_sum = zero, evap_sum = zero;
      float tas_sum = zero, rlds_sum = zero, rsds_sum = zero, huss_sum = zero;
      float ps_sum = zero, pr_sum = zero, rhs_sum = zero, h2osoi_sum_total = zero;
      float theta_sum[LM + 2];
      for (int i = 1; i <= L; i++) theta_sum[i] = zero;
      for (int dd = 0; dd < nt && !code; dd++, day++) {
        const size_t fo = (size_t)day * ncell + c;
        const size_t fv = (size_t)ndays * ncell;
        const float tas = forcing[0 * fv + fo], rlds = forcing[1 * fv + fo];
        const float rsds = forcing[2 * fv + fo], huss = forcing[3 * fv + fo];
        const float ps = forcing[4 * fv + fo], pr = forcing[5 * fv + fo];
        const float rhs = forcing[6 * fv + fo];
        day_t d;                                   /* HYBRID9.f90:168-184 */
        d.tas = tas;
        d.tak = tas;
        d.rh = rhs;
        d.Rnet = 0.92f * rsds + rlds - stbo * (tas * (tas * (tas * tas)));
        d.PAR = 0.92f * rsds * 2.3f;
        d.forc_rain = 1.0E3f * pr / rhow;
        d.lamb = ((2503.0f - 2.386f * (d.tak - tf))) * 1.0E3f;
        d.huss = huss;
        d.ps = ps;
        for (int ns = 0; ns < nisurf; ns++) {       /* :193-211 */
          float tran, evg;
          code = hydrology(&g, &p, &d, &s, &rnf_sum, theta, &tran, &evg, &errval);
          if (code) { eday = day; estep = ns; edoy = dd; break; }
          if (trow) {
            float *r = trow + ((size_t)day * nisurf + ns) * tw;
            for (int i = 0; i < L; i++) {
              r[i] = s.h2o[i + 1];
              r[L + i] = s.smp[i + 1];
              r[2 * L + i] = theta[i + 1];
            }
            r[3 * L + 0] = s.zwt;
            r[3 * L + 1] = s.wa;
            r[3 * L + 2] = tran;
            r[3 * L + 3] = evg;
            r[3 * L + 4] = rnf_sum;
            r[3 * L + 5] = s.LAI;
            r[3 * L + 6] = s.LAI_litter;
          }
        }
        if (code) break;
        if (grow_on) grow(&g, &d, &s, &npp);         /* :217 */
        tas_sum = tas_sum + tas;                      /* :235-254 */
        rlds_sum = rlds_sum + rlds;
        rsds_sum = rsds_sum + rsds;
        huss_sum = huss_sum + huss;
        ps_sum = ps_sum + ps;
        pr_sum = pr_sum + pr;
        rhs_sum = rhs_sum + rhs;
        plant_mass_sum = plant_mass_sum + s.pm;
        npp_sum = npp_sum + npp;
        for (int i = 1; i <= L; i++) {
          theta_sum[i] = theta_sum[i] + theta[i];
          h2osoi_sum_total = h2osoi_sum_total + s.h2o[i];
        }
      }
      if (code) break;
      float *a = annual + (size_t)y * nf * ncell;    /* :263-290 */
      a[0 * ncell + c] = npp_sum;
      a[1 * ncell + c] = plant_mass_sum / (float)nt;
      a[2 * ncell + c] = rnf_sum / (float)(nt * nisurf);
      a[3 * ncell + c] = evap_sum / (float)(nt * nisurf);
      a[4 * ncell + c] = tas_sum / (float)nt;
      a[5 * ncell + c] = rlds_sum / (float)nt;
      a[6 * ncell + c] = rsds_sum / (float)nt;
      a[7 * ncell + c] = huss_sum / (float)nt;
      a[8 * ncell + c] = ps_sum / (float)nt;
      a[9 * ncell + c] = pr_sum / (float)nt;
      a[10 * ncell + c] = rhs_sum / (float)nt;
      for (int i = 1; i <= L; i++) a[(10 + i) * ncell + c] = theta_sum[i] / (float)nt;
      a[(11 + L) * ncell + c] = h2osoi_sum_total / (float)nt;
    }
    store_st(&s, state, ncell, L, c);
    if (cell_err) {   /* every cell's STOP record: code, day of year, substep, value bits */
      cell_err[c] = code;
      cell_err[(size_t)ncell + c] = code ? edoy : 0;
      cell_err[2 * (size_t)ncell + c] = code ? estep : 0;
      memcpy(&cell_err[3 * (size_t)ncell + c], &errval, 4);
      if (!code) cell_err[3 * (size_t)ncell + c] = 0;
    }
    if (code) {
#pragma omp critical(h9o_err)
      {
        if (c < first_cell) {
          first_cell = c;
          first_code = code;
          first.code = code;
          first.cell = c;
          first.day = eday;
          first.substep = estep;
          first.value = errval;
        }
      }
    }
  }
  if (err) *err = first;
  return first_code;
}

/* ----------------------------------------------------------------------
 * LCLIM single-site path, HYBRID9.f90:353-478: per-substep forcing
 * (:428-445), the day-of-year LAI schedule (:380-417) as (LAI, a, b) rows
 * (NaN = no change; LAI_litter = LAI_litter + a - b), no GROW, and the
 * daily diagnostics of :464-469.  Layouts as h9g_run_site (include/h9g.h):
 * sub (nday*nisurf, 5, ncell), daily (nday, 2, ncell), lai (nday, 3, ncell),
 * diag out (nday, 11, ncell).  Pinned against oracle/_ref/h9ref's
 * lclim_mode through tests/golden/lclim_*.npz.
 * -------------------------------------------------------------------- */
int h9o_site(int ncell, int L, int nisurf, int nday, const float *zi, const float *params,
             const float *sub, const float *daily, const float *lai, float *state, float *diag,
             int nthreads, h9o_error *err) {
  if (ncell < 0 || L < 4 || L > LM || nisurf < 1 || nday < 1) return H9O_ERR_ARGS;
  const size_t n = (size_t)ncell;
  int first_code = 0, first_cell = ncell;
  h9o_error first = {0, -1, -1, -1, 0.0f};
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) if (nthreads != 1)
  for (int c = 0; c < ncell; c++) {
    geom_t g;
    geom_init(&g, L, nisurf, zi);
    par_t p;
    st_t s;
    load_par(&p, params, ncell, L, c);
    load_st(&s, state, ncell, L, c);
    float ts_sum = zero;
    for (int i = 1; i <= L; i++) ts_sum = ts_sum + p.theta_s[i];
    if (!(ts_sum > trunc_)) continue;
    float theta[LM + 2] = {0};
    float rnf_sum = zero, errval = 0.0f;
    int code = 0, eday = -1, estep = -1;
    for (int day = 0; day < nday && !code; day++) {
      const float *l = lai + (size_t)day * 3 * n + c;
      if (l[0] == l[0]) s.LAI = l[0];                                   /* :380-417 */
      if (l[n] == l[n]) s.LAI_litter = s.LAI_litter + l[n] - l[2 * n];
      float evap_day = zero, evap_grnd_day = zero;                      /* :421-422 */
      for (int ns = 0; ns < nisurf; ns++) {
        const float *v = sub + ((size_t)day * nisurf + ns) * 5 * n + c;
        day_t d;
        d.tak = v[0] + tf;                                              /* :430-439 */
        d.tas = d.tak;
        d.rh = v[n];
        d.Rnet = v[2 * n];
        d.PAR = v[3 * n];
        d.forc_rain = v[4 * n] / g.dt;
        d.lamb = ((2503.0f - 2.386f * (d.tak - tf))) * 1.0E3f;         /* :445 */
        d.huss = daily[(size_t)day * 2 * n + c];                        /* :377-378 */
        d.ps = daily[(size_t)day * 2 * n + n + c];
        float tran, evg;
        code = hydrology(&g, &p, &d, &s, &rnf_sum, theta, &tran, &evg, &errval);   /* :453 */
        if (code) { eday = day; estep = ns; break; }
        evap_day = evap_day + (evg + tran) * g.dt;                      /* :457-458 */
        evap_grnd_day = evap_grnd_day + evg * g.dt;
      }
      float *o = diag + (size_t)day * 11 * n + c;                       /* :464-469 */
      if (code) {
        for (int k = 0; k < 11; k++) o[k * n] = NAN;
        break;
      }
      o[0] = evap_day;
      o[n] = evap_grnd_day;
      for (int i = 1; i <= 4; i++) o[(1 + i) * n] = theta[i];
      o[6 * n] = s.h2o_ma[1] / (g.dz[1] * rhow / 1.0E3f);             /* HYDROLOGY.f90:149 */
      o[7 * n] = s.LAI;
      o[8 * n] = s.LAI_litter;
      o[9 * n] = zero;                                                  /* w_i, fT: no GROW */
      o[10 * n] = zero;
    }
    store_st(&s, state, ncell, L, c);
    if (code) {
#pragma omp critical(h9o_err)
      {
        if (c < first_cell) {
          first_cell = c;
          first_code = code;
          first.code = code;
          first.cell = c;
          first.day = eday;
          first.substep = estep;
          first.value = errval;
        }
      }
    }
  }
  if (err) *err = first;
  return first_code;
}

/* ----------------------------------------------------------------------
 * Soil parameter build, INIT.f90:575-631 (one soil layer) and :661-680
 * (Fmax), for the 0.5-degree cells gid (iy*nx+ix, row iy from the north).
 * Input fields are the 30" layers as read at INIT.f90:540-569: ny*60 rows
 * of nx*60 values, row-major (the Fortran (x1,y1) with x1 fastest).
 * Parity unpinned against the reference itself (INIT.f90 needs the
 * netCDF-Fortran library, absent here); tests/test_soil.py pins this
 * restatement with an independent numpy loop.
 * -------------------------------------------------------------------- */
void h9o_soil_layer(int nx, int ny, int ncell, const int64_t *gid, const float *ts_in,
                    const float *ks_in, const float *lm_in, const float *ps_in, float *theta_s,
                    float *hksat, float *bsw, float *psi_s) {
  const float zero = 0.0f, trunc = 1.0E-8f;     /* SHARED.f90:506 */
  const size_t W = (size_t)nx * 60;
  (void)ny;
  for (int c = 0; c < ncell; c++) {
    const int x = (int)(gid[c] % nx), y = (int)(gid[c] / nx);
    float ts = zero, ks = zero, lm = zero, ps = zero;   /* :575-578 */
    int j = 0;
    for (int x1 = x * 60; x1 < x * 60 + 60; x1++)       /* :582-592, x1 outer */
      for (int y1 = y * 60; y1 < y * 60 + 60; y1++) {
        const size_t k = (size_t)y1 * W + x1;
        if (ts_in[k] >= zero) {
          ts = ts + ts_in[k];
          ks = ks + ks_in[k];
          lm = lm + lm_in[k];
          ps = ps + ps_in[k];
          j = j + 1;
        }
      }
    if (j > 0) {                                         /* :593-598 */
      ts = ts / (float)j;
      ks = ks / (float)j;
      lm = lm / (float)j;
      ps = ps / (float)j;
    }
    theta_s[c] = ts / 1.0E3f;                            /* :613-628 */
    hksat[c] = 10.0f * ks / 86400.0f;
    float lambda = lm / 1.0E3f;
    psi_s[c] = 10.0f * ps;
    lambda = MAXF(lambda, trunc);
    bsw[c] = 1.0f / lambda;
  }
}

/* INIT.f90:661-680: Fmax of soiled cells from the 0.5-degree integer field
 * (missing -9999 -> global mean 3809), NaN elsewhere.  theta_s (ncell, L). */
void h9o_soil_fmax(int ncell, int L, const int64_t *gid, const int32_t *soil_tex,
                   const int32_t *fmax_in, const float *theta_s, float *fmax) {
  const float trunc = 1.0E-8f;
  for (int c = 0; c < ncell; c++) {
    float sum = 0.0f;
    for (int i = 0; i < L; i++) sum = sum + theta_s[(size_t)c * L + i];
    const int tex = soil_tex[gid[c]];
    if (tex > 0 && tex != 13 && sum > trunc) {
      int v = fmax_in[gid[c]];
      if (v == -9999) v = 3809;
      fmax[c] = (float)v / 10000.0f;
    } else {
      fmax[c] = NAN;
    }
  }
}
