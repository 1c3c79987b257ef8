// TEST INFRASTRUCTURE ONLY: a host (CPU) build of the GPU kernel body
// (hybrid9_amd/csrc/h9g_pair.h + h9g_step.h, one lane doing every layer:
// the code of the solo kernel and of the device exact re-run; the pair
// kernel differs only in which lane evaluates a layer), used by
// tests/test_kernel_host.py to pin the
// kernel's arithmetic against the oracle and the reference goldens without
// a GPU.  Never linked into the product library.
#include <stdint.h>
#include <string.h>
// exact re-runs: count, runs replaying from a snapshot taken before substep
// 0 of a later substep (several substeps replayed), substeps replayed
static long long g_exact[3];
#define H9G_EXACT_HOOK(k0, ns)                      \
  do {                                              \
    __atomic_add_fetch(&g_exact[0], 1, __ATOMIC_RELAXED); \
    if ((ns) > (k0)) __atomic_add_fetch(&g_exact[1], 1, __ATOMIC_RELAXED); \
    __atomic_add_fetch(&g_exact[2], (ns) - (k0) + 1, __ATOMIC_RELAXED); \
  } while (0)
#include "../../hybrid9_amd/csrc/h9g_geo.h"
#include "../../hybrid9_amd/csrc/h9g_step.h"
#include "../../hybrid9_amd/csrc/h9g_pair.h"

using namespace h9k;
static const uint64_t E2[32] = H9M_EXP2F_TAB_INIT;
static const double L2[32] = H9M_POWF_LOG2_TAB_INIT;

static int diy(int y) { return y % 4 ? 365 : (y % 100 ? 366 : (y % 400 ? 365 : 366)); }

template <int L, class G>
static int run_cells_pair(const G &g, int n, int nisurf, int grow_on, int year0, int nyears,
                          const float *par, const float *forc, float *st, float *ann, int *err) {
  const h9m::Tabs T = {E2, L2};
  int ndays = 0;
  for (int y = 0; y < nyears; y++) ndays += diy(year0 + y);
  int first = 0;
#pragma omp parallel for schedule(dynamic, 4)
  for (int c = 0; c < n; c++) {
    float store[FlatStore<L>::N], zt[zt_size<L>()];
    fill_zt<L>(g, zt);
    FlatStore<L> cs{store, zt};
    const SplitAll sp;
    St<L> s;
    for (int i = 1; i <= L; i++) {
      cs.set_lay(PF_TS, i, par[0 * n * L + c * L + i - 1]);
      cs.set_lay(PF_HKS, i, par[1 * n * L + c * L + i - 1]);
      cs.set_lay(PF_BSW, i, par[2 * n * L + c * L + i - 1]);
      cs.set_lay(PF_PSI, i, par[3 * n * L + c * L + i - 1]);
      s.h2o[i] = st[0 * n * L + c * L + i - 1];
      s.smp[i] = st[2 * n * L + c * L + i - 1];
      cs.set_lay(PF_ROOTR, i, st[3 * n * L + c * (L + 1) + i - 1]);
    }
    cs.set_sc(PS_FMAX, par[4 * n * L + c]);
    cell_inv_pair<L, G>(g, cs);
    float *q = st + (size_t)n * (4 * L + 1);
    s.zwt = q[c]; s.wa = q[n + c]; s.LAI = q[2 * n + c]; s.LAI_litter = q[3 * n + c];
    s.pm = q[4 * n + c]; s.pfm = q[5 * n + c]; s.plen = q[6 * n + c]; s.rdepth = q[7 * n + c];
    int d0 = 0;
    for (int y = 0; y < nyears; y++) {
      const int nt = diy(year0 + y);
      float a[12 + L];
      int eday = 0, estep = 0;
      float ev = 0;
      const int code = cell_year_pair<L, G>(g, cs, sp, s, forc + (size_t)d0 * n + c, (size_t)n,
                                            (size_t)ndays * n, nt, nisurf, grow_on, a, 1, eday,
                                            estep, ev, T);
      if (code) {
        err[4 * c] = code; err[4 * c + 1] = y; err[4 * c + 2] = eday; err[4 * c + 3] = estep;
#pragma omp atomic write
        first = code;
        break;
      }
      for (int r = 0; r < 12 + L; r++) ann[((size_t)y * (12 + L) + r) * n + c] = a[r];
      d0 += nt;
    }
    for (int i = 1; i <= L; i++) {
      st[0 * n * L + c * L + i - 1] = s.h2o[i];
      st[2 * n * L + c * L + i - 1] = s.smp[i];
      if (grow_on) st[3 * n * L + c * (L + 1) + i - 1] = cs.lay(PF_ROOTR, i);
    }
    if (grow_on) st[3 * n * L + c * (L + 1) + L] = 0.0f;
    q[c] = s.zwt; q[n + c] = s.wa; q[2 * n + c] = s.LAI; q[3 * n + c] = s.LAI_litter;
    q[4 * n + c] = s.pm; q[5 * n + c] = s.pfm; q[6 * n + c] = s.plen; q[7 * n + c] = s.rdepth;
  }
  return first;
}

// use_const_geo: 1 = the driver.txt / config-5 layer sets and NISURF 24|48
// as compile-time geometry (GeoC), 0 = runtime geometry (GeoR).
extern "C" int h9k_host_run(int n, int L, int nisurf, int grow_on, int year0, int nyears,
                            int use_const_geo, const float *zi, const float *par,
                            const float *forc, float *st, float *ann, int *err) {
  const bool cg = use_const_geo != 0;
#define RP(LL, G) return run_cells_pair<LL>(G, n, nisurf, grow_on, year0, nyears, par, forc, st, ann, err)
  if (L == 8) {
    if (cg && nisurf == 48) RP(8, (GeoC<8, 48>()));
    if (cg && nisurf == 24) RP(8, (GeoC<8, 24>()));
    RP(8, make_geo_r<8>(zi, nisurf));
  }
  if (cg && nisurf == 48) RP(10, (GeoC<10, 48>()));
  if (cg && nisurf == 24) RP(10, (GeoC<10, 24>()));
  RP(10, make_geo_r<10>(zi, nisurf));
#undef RP
}

// The LCLIM site path (cell_site of h9g_pair.h) on the host, same layouts as
// h9g_run_site; state in the oracle's packed layout (as h9k_host_run).
template <int L, class G>
static int run_site_cells(const G &g, int n, int nday, int nisurf, const float *par, const float *sub,
                          const float *daily, const float *lai, float *st, float *out, int *err) {
  const h9m::Tabs T = {E2, L2};
  int first = 0;
#pragma omp parallel for schedule(dynamic, 1)
  for (int c = 0; c < n; c++) {
    float store[FlatStore<L>::N], zt[zt_size<L>()];
    fill_zt<L>(g, zt);
    FlatStore<L> cs{store, zt};
    St<L> s;
    for (int i = 1; i <= L; i++) {
      cs.set_lay(PF_TS, i, par[0 * n * L + c * L + i - 1]);
      cs.set_lay(PF_HKS, i, par[1 * n * L + c * L + i - 1]);
      cs.set_lay(PF_BSW, i, par[2 * n * L + c * L + i - 1]);
      cs.set_lay(PF_PSI, i, par[3 * n * L + c * L + i - 1]);
      s.h2o[i] = st[0 * n * L + c * L + i - 1];
      s.smp[i] = st[2 * n * L + c * L + i - 1];
      cs.set_lay(PF_ROOTR, i, st[3 * n * L + c * (L + 1) + i - 1]);
    }
    cs.set_sc(PS_FMAX, par[4 * n * L + c]);
    cell_inv_pair<L, G>(g, cs);
    float *q = st + (size_t)n * (4 * L + 1);
    s.zwt = q[c]; s.wa = q[n + c]; s.LAI = q[2 * n + c]; s.LAI_litter = q[3 * n + c];
    s.pm = q[4 * n + c]; s.pfm = q[5 * n + c]; s.plen = q[6 * n + c]; s.rdepth = q[7 * n + c];
    int eday = 0, estep = 0;
    float ev = 0;
    const int code = cell_site<L, G>(g, cs, s, st[1 * n * L + c * L], sub + c, daily + c, lai + c, out + c,
                                     (size_t)n, nday, nisurf, eday, estep, ev, T);
    if (code) {
      err[4 * c] = code; err[4 * c + 1] = 0; err[4 * c + 2] = eday; err[4 * c + 3] = estep;
#pragma omp atomic write
      first = code;
    }
    for (int i = 1; i <= L; i++) {
      st[0 * n * L + c * L + i - 1] = s.h2o[i];
      st[2 * n * L + c * L + i - 1] = s.smp[i];
    }
    q[c] = s.zwt; q[n + c] = s.wa; q[2 * n + c] = s.LAI; q[3 * n + c] = s.LAI_litter;
  }
  return first;
}

extern "C" int h9k_host_site(int n, int L, int nisurf, int nday, int use_const_geo, const float *zi,
                             const float *par, const float *sub, const float *daily, const float *lai,
                             float *st, float *out, int *err) {
  const bool cg = use_const_geo != 0;
#define RS(LL, G) return run_site_cells<LL>(G, n, nday, nisurf, par, sub, daily, lai, st, out, err)
  if (L == 8) {
    if (cg && nisurf == 48) RS(8, (GeoC<8, 48>()));
    RS(8, make_geo_r<8>(zi, nisurf));
  }
  if (cg && nisurf == 48) RS(10, (GeoC<10, 48>()));
  RS(10, make_geo_r<10>(zi, nisurf));
#undef RS
}

// Exact re-run counters since the last call (then reset).
extern "C" void h9k_host_exact_stats(long long *out) {
  for (int i = 0; i < 3; i++) out[i] = __atomic_exchange_n(&g_exact[i], 0, __ATOMIC_RELAXED);
}
