// h9g_step.h -- the per-cell pieces of the HYBRID9 time step shared by the
// device kernels and by the host build that pins them against the oracle
// (tests/test_kernel_host.py):
//
//   day_consts   the parts of HYDROLOGY.f90:232-389 that depend only on the
//                day's forcing and on LAI / LAI_litter (which only GROW
//                changes, once a day): computed once per cell-day
//   grow_day     /root/reference/SOURCE/GROW.f90:55-201
//   init_cell    /root/reference/SOURCE/INIT.f90:707-811
//   make_day     /root/reference/SOURCE/HYBRID9.f90:168-184
//   MathExact / MathFast   the math policies of the substep (below)
//
// The HYDROLOGY substep itself (HYDROLOGY.f90:141-1283) is h9g_pair.h.
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
// Math policies: the substep is instantiated with one.  MathFast runs
// glibc's main path branch-free (h9m::*_nx) and redoes in place, in a rarely
// taken branch, any result whose input glibc sends down another path
// (deferred-check forms *_d / *_fix: one branch per group of independent
// operations).  MathExact evaluates glibc's full logic and divides.  Results
// are bit-identical either way.  Only a water-table loop that needs a third
// layer visit re-runs its substep, exactly, replaying the day from its
// snapshot (h9g_pair.h save_day / substep_exact_pair).
#pragma once
#include "h9_math.h"
#include "h9g_geo.h"

namespace h9k {

constexpr float zero = 0.0f, one = 1.0f;
// include/h9g.h H9G_ERR_NOSNAP (the host build does not include h9g.h)
constexpr int H9G_ERR_NOSNAP_K = 5;
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

#if defined(H9G_FASTMINMAX) && defined(__HIP_DEVICE_COMPILE__)   // experiment: v_max/v_min
H9K_HD float MAXF(float a, float b) { return __builtin_fmaxf(a, b); }
H9K_HD float MINF(float a, float b) { return __builtin_fminf(a, b); }
#else
H9K_HD float MAXF(float a, float b) { return a > b ? a : b; }
H9K_HD float MINF(float a, float b) { return a < b ? a : b; }
#endif
H9K_HD float absf(float a) { return __builtin_fabsf(a); }
// MIN/MAX with a NONZERO constant c, one VALU instead of compare + select:
//   MAXC(c, x) = flang's MAX(c, x) = c > x ? c : x.  For x NaN that is x, for
//     x == c it is x (the same bits, as c is not a zero): exactly IEEE
//     754-2019 maximum(c, x) (NaN-propagating; v_maximum3_f32 on gfx950);
//   MAXX(x, c) = MAX(x, c) = x > c ? x : c: c for x NaN, i.e. maxNum(x, c)
//     (v_max_f32).
// With c = 0 they would differ in the sign of a zero result, so zeros keep
// MAXF/MINF.  (A NaN's payload may differ; no result but a NaN depends on it.)
H9K_HD float MAXC(float c, float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_elementwise_maximum(c, x);
#else
  return MAXF(c, x);
#endif
}
H9K_HD float MINC(float c, float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_elementwise_minimum(c, x);
#else
  return MINF(c, x);
#endif
}
H9K_HD float MAXX(float x, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fmaxf(x, c);
#else
  return MAXF(x, c);
#endif
}

// Scheduling fence: stops the machine scheduler from interleaving the
// unrolled per-layer bodies (each a few powf with double-precision
// temporaries), which otherwise multiplies the live register set by L.
#ifndef H9G_FENCE_MASK
#define H9G_FENCE_MASK 0x100   // kinds allowed to cross (sched.barrier mask): LDS reads (round 3: 200.8 -> 200.3 ms)
#endif
H9K_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(H9G_NOFENCE)
  __builtin_amdgcn_sched_barrier(H9G_FENCE_MASK);
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

// Branch counters (measurement builds, -DH9G_COUNT_BRANCH; tools/isa_mix.py
// weighs the static mix with them): H9G_BR(k) counts the waves that enter
// site k ([k]) and their active lanes ([32 + k]).  Empty in product builds.
#if defined(H9G_COUNT_BRANCH)
__device__ unsigned long long h9g_branch_count[64];
#endif
#if defined(H9G_COUNT_BRANCH) && defined(__HIP_DEVICE_COMPILE__)
#define H9G_BR(k)                                                                   \
  do {                                                                              \
    const uint64_t em_ = __builtin_amdgcn_read_exec();                              \
    if (__lane_id() == (unsigned)__builtin_ctzll(em_)) {                            \
      atomicAdd(&h9g_branch_count[(k)], 1ull);                                      \
      atomicAdd(&h9g_branch_count[32 + (k)], (unsigned long long)__builtin_popcountll(em_)); \
    }                                                                               \
  } while (0)
#else
#define H9G_BR(k) ((void)0)
#endif
// Day-level water-table record (measurement builds, -DH9G_DUMP_AQ; tools/
// aq_sort.py designs the cell order from it): bit d of h9g_aq_bits[c][d/32]
// = the water table of cell c is below the column at the start of day d.
#if defined(H9G_DUMP_AQ)
__device__ unsigned *h9g_aq_bits;
__device__ const float *h9g_aq_base;   // the annual array: cell = acc - base
#endif
enum : int {   // H9G_BR sites
  BR_SUBSTEP = 0, BR_THETA, BR_QB, BR_EQX, BR_AQPOW, BR_AQS, BR_HKX, BR_TRIFLUX, BR_TRISWEEP, BR_RECH,
  BR_BASE, BR_WATMIN, BR_RERUN, BR_POWREDO, BR_DIVREDO, BR_EXPREDO, BR_POWFIX, BR_DIVFIX, BR_INL, BR_ANYAQ,
  BR_JWTCOL, BR_VISIT2, BR_SNAP, BR_EBX, BR_DAY, BR_N
};

// ------------------------------------------------------------ math policies
// A fast-division quotient that must re-run exactly: subnormal (RN32 of the
// double product may differ from the correctly rounded quotient there) or
// NaN (recip64 of a zero, infinite or NaN divisor is NaN; x/0 is not).
H9K_HD bool bad_quotient(float q) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_classf(q, 0x093);     // -denormal | +denormal | snan | qnan
#else
  const uint32_t u = __builtin_bit_cast(uint32_t, q) & 0x7fffffffu;
  return (u != 0 && u < 0x00800000u) || u > 0x7f800000u;
#endif
}

// x / d by the refined hardware reciprocal, y = fma(fma(-d, r, 1), r, r),
// r = v_rcp_f32(d), and Markstein's correction of RN(x y): the correctly
// rounded quotient for every pair of float significands
// (tools/markstein_exhaustive.hip mode 1), so whenever |x| and |d| lie in
// [2^-60, 2^60), where scaling by powers of two is exact; other operands
// (x = 0 among them) set bad, for the caller's exact path.  Six dependent
// operations against the IEEE division's nine.  (The host build uses the
// correctly rounded 1/d, mode 0 of the same proof.)
H9K_HD float mk_div(float x, float d, bool &bad) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float r = __builtin_amdgcn_rcpf(d);
#else
  const float r = 1.0f / d;
#endif
  const float y = __builtin_fmaf(__builtin_fmaf(-d, r, 1.0f), r, r);
  const float q0 = x * y;
  const float q = __builtin_fmaf(__builtin_fmaf(-d, q0, x), y, q0);
  const uint32_t ux = (__builtin_bit_cast(uint32_t, x) & 0x7fffffffu) - 0x21800000u;   // 2^-60
  const uint32_t ud = (__builtin_bit_cast(uint32_t, d) & 0x7fffffffu) - 0x21800000u;
  bad |= (ux > ud ? ux : ud) >= 0x5d800000u - 0x21800000u;                             // 2^60
  return q;
}

// Reciprocal of a float divisor in double, |r - 1/d| <= 1.2 * 2^-53 |1/d|:
// hardware estimate + two Newton steps (each squares the error and adds
// <= 2^-53; two steps suffice from any estimate within 2^-14).  NaN for
// d = 0, inf or NaN (the Newton residual is 0 * inf).
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
// midpoint.  Subnormal and NaN results flag the substep for the exact re-run.
struct MathExact {
  static constexpr bool kExact = true;
  h9m::Tabs T;
  H9K_HD float expf(float x) { return h9m::expf(x, T); }
  H9K_HD float powf(float x, float y) { return h9m::powf(x, y, T); }
  H9K_HD float div(float x, float d, double) { return x / d; }
  // deferred-check forms (MathFast): nothing to defer, never flagged
  H9K_HD float powf_d(float x, float y, bool &sp) {
    sp = false;
    return h9m::powf(x, y, T);
  }
  H9K_HD void powf_fix(float &, float, float, bool) {}
  H9K_HD float div_d(float x, float d, double) { return x / d; }
  H9K_HD bool div_bad(float) const { return false; }
  H9K_HD void div_fix(float &, float, float) {}
};
// The rare paths -- glibc's special cases of MathFast below and the exact
// re-run of a substep (h9g_pair.h) -- are inlined into the kernels, which
// make no calls.  Round 2 kept them out of line; the kernels' calls were
// miscompiled: a lane-mask SGPR stayed live across calls to the redo
// function, which overwrites it (tools/isa_calls.py).
#if defined(__HIP_DEVICE_COMPILE__) && defined(H9G_RARE_CALLS)
// reproducer of the round-2 miscompile: the rare paths out of
// line again; tools/isa_calls.py --live then finds SGPRs live across calls
// that the callee writes.  Never a product build.
#define H9K_RARE __device__ __attribute__((noinline, cold))
#elif defined(__HIP_DEVICE_COMPILE__)
#define H9K_RARE __device__ __forceinline__
#else
#define H9K_RARE static __attribute__((noinline, cold))
#endif

// glibc's full expf / powf: the in-place redo of MathFast (rare).
H9K_RARE float expf_redo(float x, const uint64_t *e2, const double *l2) { return h9m::expf(x, {e2, l2}); }
H9K_RARE float powf_redo(float x, float y, const uint64_t *e2, const double *l2) {
  return h9m::powf(x, y, {e2, l2});
}

struct MathFast {
  static constexpr bool kExact = false;
  h9m::Tabs T;
  bool special;             // set only by the water-table loops' third visit (visit_layers)
  unsigned redone = 0;      // results redone in place (read by the self tests only)
  // glibc's main path, branch-free; an input that glibc sends down another
  // path (|x| >= 88 for expf; for powf x not a positive normal number or
  // |y log2 x| >= 126, i.e. an under- or overflowing power such as the
  // conductivity power of a very dry layer) is recomputed in place with
  // glibc's full logic, in a branch that is rarely taken.  Round 1 re-ran
  // the whole substep on the exact path for these inputs instead; a column
  // that met one every substep made its wave, and so the kernel, up to
  // 2.6x slower.
  H9K_HD float expf(float x) {
    bool sp = false;
    float r = h9m::expf_nx(x, T, sp);
    if (__builtin_expect(sp, 0)) {
      H9G_BR(BR_EXPREDO);
      r = expf_redo(x, T.exp2, T.log2);
      redone++;
    }
    return r;
  }
  H9K_HD float powf(float x, float y) {
    bool sp = false;
    float r = h9m::powf_nx<false>(x, y, T, sp);
    if (__builtin_expect(sp, 0)) {
      H9G_BR(BR_POWREDO);
      r = powf_redo(x, y, T.exp2, T.log2);
      redone++;
    }
    return r;
  }
  // x / d from the double reciprocal r: RN32(x * r) is the correctly rounded
  // quotient whenever that is a normal or infinite float.  A
  // subnormal quotient (the tiny fluxes of a very dry column) or a NaN one
  // (d = 0, inf or NaN makes r NaN) is redone in place as the IEEE division.
  H9K_HD float div(float x, float d, double r) {
    float q = (float)((double)x * r);
    if (__builtin_expect(bad_quotient(q), 0)) {
      H9G_BR(BR_DIVREDO);
      q = x / d;
      redone++;
    }
    return q;
  }
  // Deferred checks.  A per-operation "redo if special" branch ends the
  // basic block, so the scheduler cannot interleave independent powers or
  // quotients and every one runs at its full dependency latency.  The _d
  // forms evaluate branch-free; a group of independent operations is then
  // followed by ONE rarely-taken branch (any flag set) in which _fix redoes
  // exactly the flagged results, as powf/div above would have:
  //   float a = m.powf_d(x0, y0, s0), b = m.powf_d(x1, y1, s1);
  //   if (__builtin_expect(s0 | s1, 0)) { m.powf_fix(a, x0, y0, s0); ... }
  H9K_HD float powf_d(float x, float y, bool &sp) {
    sp = false;
    return h9m::powf_nx<false>(x, y, T, sp);
  }
  H9K_HD void powf_fix(float &r, float x, float y, bool sp) {
    if (sp) {
      H9G_BR(BR_POWFIX);
      r = powf_redo(x, y, T.exp2, T.log2);
      redone++;
    }
  }
  H9K_HD float div_d(float x, float, double r) { return (float)((double)x * r); }
  H9K_HD bool div_bad(float q) const { return bad_quotient(q); }
  H9K_HD void div_fix(float &q, float x, float d) {
    if (bad_quotient(q)) {
      H9G_BR(BR_DIVFIX);
      q = x / d;
      redone++;
    }
  }
};

// ------------------------------------------------------------ cell data
// Day-constant fields (HYDROLOGY.f90:232-389 terms fixed within a day),
// stored per cell by day_consts through the store's set_day.
// The canopy/soil pairs (c, s) come first, c at odd D index: with the
// per-cell fields starting at an odd offset (h9g_pair.h PS_DAY) each pair
// shares one row of the pair store, c in the even lane's column, s in the
// odd lane's, so the pair-split energy balance reads its half with no select.
enum : int {
  D_FORC = 0,
  D_NUMC, D_NUMS, D_RAARAC, D_RAARAS, D_DGRAC, D_DGRAS, D_DRR, D_DRG, D_RAC, D_RAS,
  D_DESAT, D_GAMMA, D_VDD, D_DG, D_RHOCP, D_A1, D_X, D_LAI2, D_PW28, D_RSCMIN,
  D_RAA, D_RL, D_LIT1000, D_OK, D_N
};
// (10 + 1000 LAI_litter and dg*raa are re-evaluated where used, from
// D_LIT1000 and D_DG, D_RAA: same operations, one VALU each, one LDS row.)
static_assert(D_N == 25, "day-constant block size");
// Day constants that HYDROLOGY divides by, kept also as double reciprocals
// (recip64) by stores with kDayRecip (exact fast division, h9g_pair.h):
// the canopy/soil pairs DRP_* (raa+rac | raa+ras, rac | ras; day_rp(j, h))
// and the shared DR_* (day_r(k)).  2 * DR_N float fields.
enum : int { DRP_RAARA = 0, DRP_RA, DRP_N };
enum : int { DR_RHOCP = 0, DR_RL, DR_N1 };
enum : int { DR_N = 2 * DRP_N + DR_N1 };

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) float lds_float;
// Global-memory float: loads and stores through it cannot alias LDS, so
// they are not ordered against the store's LDS traffic (a generic pointer
// makes them flat_load/flat_store with a full wait after each).
typedef __attribute__((address_space(1))) float gbl_float;
#else
typedef float lds_float;
typedef float gbl_float;
#endif

// Loads of the forcing slab, which streams through L2 once per cell-day:
// with the non-temporal hint, so that it does not evict the L2-resident
// annual sums and day snapshots (config 2: HBM writes 4.9 -> 3.2 GB per
// launch; with the XCD-aware cell order 0.6 GB).
H9K_HD float ld_stream(const gbl_float *p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

template <int L>
struct St {            // persistent per-cell state (SHARED.f90), in registers
  float h2o[L + 1], smp[L + 1];
  float zwt, wa, LAI, LAI_litter, pm, pfm, plen, rdepth;
  int naq;             // substeps of the year with the water table below the column
                       // (not model state: the next year's cell order, h9g_sort_kernel)
};

struct Day {           // HYBRID9.f90:168-184 + forcing read by HYDROLOGY
  float tak, rh, Rnet, PAR, forc_rain, lamb, huss, ps;
};

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
  cs.set_day(D_DGRAS, dg * ras);
  cs.set_day(D_DGRAC, dg * rac);
  cs.set_day(D_DRR, desatdT * (Rnet - Rnets));
  cs.set_day(D_DRG, desatdT * (Rnets - G));
  cs.set_day(D_RL, rhow * d.lamb);
  if constexpr (CS::kDayRecip) {
    cs.set_day_rp(DRP_RAARA, 0, recip64(raarac));
    cs.set_day_rp(DRP_RAARA, 1, recip64(raaras));
    cs.set_day_rp(DRP_RA, 0, recip64(rac));
    cs.set_day_rp(DRP_RA, 1, recip64(ras));
    cs.set_day_r(DR_RHOCP, recip64(rhocp));
    cs.set_day_r(DR_RL, recip64(rhow * d.lamb));
  }
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



}  // namespace h9k
