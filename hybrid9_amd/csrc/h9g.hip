// h9g.hip -- MI355X (gfx950) implementation of the HYBRID9 per-cell
// time-stepping hot path behind the C-ABI of include/h9g.h.
//
// Kernel design:
//   * h9g_pair_kernel<L, G> (default): one launch runs one calendar year --
//     all days x NISURF substeps of HYDROLOGY plus the daily GROW -- for
//     every cell, time innermost as in the reference.  Two lanes per soil
//     column: the per-layer phases (equilibrium profile, conductivity and
//     matric potential; ~40 of the ~46 glibc-exact powf of a substep) are
//     split over the pair and exchanged by DPP, the rest runs in both
//     lanes.  22 columns per wave, 4 waves per workgroup: 3 waves on every
//     SIMD at 0.5 deg (767 workgroups, 768 slots).  The column's water
//     state lives in VGPRs, its read-mostly data (soil parameters and
//     their invariants, rootr, the day's constants) in the pair's two
//     columns of an LDS block, the day snapshot of the exact re-run in an
//     L2-resident global block.  HBM traffic per
//     cell-day is the 7 forcing values (coalesced, cell-fastest) plus the
//     annual sums (L2-resident): the SHARED-state contract of each substep
//     (376 B at L=8) never leaves the CU.
//   * h9g_solo_kernel<L, G> (at L = 10 chosen by column count, alone or
//     followed by the pair kernel on the remainder, l10_kind;
//     H9G_KERNEL=solo|pair|mixed overrides): one lane per column, the same
//     code with one lane doing every layer.
//   * glibc-exact expf/powf (h9_math.h) read their 32+16-entry tables from
//     LDS (per-lane indices, no scalar-cache serialisation).
//   * no MFMA: nothing here is GEMM-shaped.
//   * h9g_diag_kernel: deterministic FP64 reduction of global diagnostics
//     (the payload of the cross-GPU all-reduce).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/h9g.h"
#include "h9_math.h"
#include "h9g_geo.h"
#include "h9g_step.h"
#include "h9g_pair.h"
#include "h9g_synth.h"
#include "h9g_io.h"

using namespace h9k;
static_assert(H9G_ERR_NOSNAP_K == H9G_ERR_NOSNAP, "kernel and ABI error codes");

__constant__ uint64_t c_exp2tab[32] = H9M_EXP2F_TAB_INIT;
__constant__ double c_log2tab[32] = H9M_POWF_LOG2_TAB_INIT;
static const uint64_t h_exp2tab[32] = H9M_EXP2F_TAB_INIT;
static const double h_log2tab[32] = H9M_POWF_LOG2_TAB_INIT;

#define H9G_BLOCK 256
#define H9G_YBLOCK 64   // solo kernel: one wave per block (LDS cell stores)
// pair kernel: 22 columns (44 lanes) per wave, 4 waves per workgroup; the
// 0.5 deg grid is 767 workgroups = 3 waves on each of the 1,024 SIMDs
#define H9G_PCPW 22
#define H9G_PLANES (2 * H9G_PCPW)
#define H9G_PWAVES 4
#define NEVT 64
static size_t round_up(size_t x, size_t m) { return (x + m - 1) / m * m; }

// ---------------------------------------------------------------------------
// kernel arguments
// ---------------------------------------------------------------------------
struct KArgs {
  int ncell;       // row stride of every per-cell array
  int c0, cend;    // cells [c0, cend) of this launch
  int nt;          // days in the year
  int nisurf;
  int grow_on;
  size_t fvar;     // forcing variable stride (floats) = max_days * ncell
  const float *__restrict__ par;   // (4L+1) rows x ncell
  float *__restrict__ st;          // (4L+9) rows x ncell
  const float *__restrict__ forc;  // 7 x max_days x ncell (slot base)
  float *__restrict__ annual;      // (12+L) rows x ncell
  int *__restrict__ err;           // 4 rows x ncell: code, day, substep, value bits
  int *__restrict__ err_flag;
  unsigned *__restrict__ stamps;   // H9G_STAMPS builds: 8 phase cycle sums per wave
  float *__restrict__ sv;          // pair kernel: day snapshot, PairStore::GBLOCK bytes per workgroup
  const int *__restrict__ perm;    // lane slot -> cell (h9g_sort_kernel), or null: identity
  int sorted_io;                   // 1: forc and annual are in slot order (h9g_perm_forcing_kernel; round 4)
  int *__restrict__ hist;          // per cell: substeps of the year with the water table below the column
  unsigned *__restrict__ pace;     // pair kernel, Pacer mode 2: H9G_PACE_ROWS x 16 progress words
  unsigned epoch;                  // Pacer mode 2: launch tag
  int prio_mode;                   // Pacer mode: 0 none, 1 rotate, 2 pace
  // A second group of cells in the same launch (pair kernels; the cell-order
  // mode's re-runs of one decade riding in the next decade's year launches,
  // h9g_run_ordered).  Slots [c0, bend) are the first group; the waves from
  // slot `split` (a multiple of the wave's column count, >= bend) to cend
  // the second, with their own state and error rows, year length and no
  // sort history.  split == cend: no second group.
  int bend, split, nt2;
  float *__restrict__ st2;
  int *__restrict__ err2;
  size_t iostride;                 // row stride of forc and annual when sorted_io (slots)
  int raw;                         // 1: the annual rows are the running sums, undivided (the cell
                                   // order's day-1 probe, h9g_probe_cmp_kernel)
};

// XCD-aware workgroup order.  MI355X deals the workgroups of a launch
// round-robin to its 8 XCDs (workgroup b -> XCD b % 8), each with its own L2.
// Workgroup b works on the cells of virtual workgroup xcd_vwg(b), which makes
// each XCD's workgroups one contiguous range of cells: the forcing, annual
// sums and state lines an XCD touches are its own (no line fetched by two
// XCDs), and the per-year cell sort (h9g_sort_kernel) reorders cells only
// within an XCD's range.
#define H9G_NXCD 8
__host__ __device__ __forceinline__ unsigned xcd_vwg(unsigned b, unsigned nb) {
  const unsigned x = b % H9G_NXCD, q = nb / H9G_NXCD, r = nb % H9G_NXCD;
  return x * q + (x < r ? x : r) + b / H9G_NXCD;
}

__device__ __forceinline__ void load_tabs(uint64_t *e2, double *l2) {
  const int t = threadIdx.x;
  if (t < 32) {
    e2[t] = c_exp2tab[t];
    l2[t] = c_log2tab[t];
  }
  __syncthreads();
}

// Pair kernel (h9g_pair.h): two lanes per soil column, the per-layer powers
// split over the pair.  Same arguments, layouts and results as
// h9g_year_kernel.
// Waves per SIMD: 3 at L = 8 (168 VGPRs, 3 x 53 KB LDS per CU); 2 at L = 10,
// where 168 VGPRs spill ~90 registers into the substep loop.
template <int L>
constexpr int pair_waves() { return pair_resident<L>(); }

// C: columns (pairs) per wave: 22 (h9g_pair_kernel, h9g_pair2_kernel) or 11
// (h9g_pair11_kernel: 42 helper lanes, 2 rounds per phase at L = 10).
template <int L, class G, int R, int C = H9G_PCPW>
__device__ __forceinline__ void pair_body(const KArgs &a, const G &g) {
  typedef PairStore<L, 2 * C, R> PS;
  __shared__ uint64_t s_e2[32];
  __shared__ double s_l2[32];
  __shared__ float s_cell[H9G_PWAVES][PS::ROWS * 2 * C];   // [wave][row][lane]
  __shared__ float s_zt[zt_size<L>()];
  // the day snapshot addresses its global block by LDS byte offset
  // (PairStore::svw): every static LDS address must lie inside GBLOCK
  static_assert(sizeof(s_e2) + sizeof(s_l2) + sizeof(s_cell) + sizeof(s_zt) <= (size_t)PS::GBLOCK,
                "pair kernel LDS footprint exceeds the day-snapshot block");
  if (threadIdx.x == 0) fill_zt<L>(g, s_zt);
  load_tabs(s_e2, s_l2);
  const h9m::Tabs T = {s_e2, s_l2};
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // lanes 0..43: 22 pairs; 44..63: spare lanes, which join the pairs only in
  // the per-layer phases (Split2, hydrology_pair).  Spare lane 44 + j mirrors
  // pair lane 12 + j (mod the wave's pair lanes): its LDS column and
  // starting state, never stored to, so the substep code it runs masked-in
  // stays ordinary; a pure function of the lane, so nothing about it is
  // carried in registers.  Lanes 12..31 because an LDS read's lanes 32..63
  // share one cycle (bank = dword mod 32): their columns' banks are the 20
  // that pair lanes 32..43 leave free, so a mirrored read adds no conflict.
  const bool spare = lane >= 2 * C;
  if (spare && !PS::kSpare) return;
  const int h = lane & 1;
  const int slot0 = __builtin_amdgcn_readfirstlane(
      a.c0 + (int)(xcd_vwg(blockIdx.x, gridDim.x) * H9G_PWAVES + wave) * C);
  // the wave's group (wave-uniform: split is a multiple of C)
  const bool g2 = slot0 >= a.split;
  const int lim = g2 ? a.cend : a.bend;
  float *const st = g2 ? a.st2 : a.st;
  int *const err = g2 ? a.err2 : a.err;
  int *const hist = g2 ? nullptr : a.hist;
  const int nt = g2 ? a.nt2 : a.nt;
  const int ncol = min(C, lim - slot0);
  if (ncol <= 0) return;             // an empty wave
  const int pl = spare ? (lane - 2 * C + (C == H9G_PCPW ? 12 : 0)) % (2 * ncol) : lane;
  const int slot = slot0 + (pl >> 1);
  if (slot >= lim) return;           // both lanes of a pair leave together
  const int c = a.perm ? a.perm[slot] : slot;
  const int io = a.sorted_io ? slot : c;   // forcing and annual sums: slot order when sorted
  const int n = a.ncell;
  const size_t ios = a.sorted_io ? a.iostride : (size_t)n;

  int prow, pslot;
  pace_key(prow, pslot);
  PS cs{(lds_float *)&s_cell[wave][pl], (lds_float *)&s_cell[wave][pl & ~1], (const lds_float *)s_zt,
        a.sv + (size_t)blockIdx.x * (PS::GBLOCK / sizeof(float)),
        Pacer{a.pace + (size_t)prow * 16, a.epoch & 0xfffffu, pslot, a.prio_mode,
              (int)((blockIdx.x * (unsigned)PS::RESIDENT) / gridDim.x)},
        (lds_float *)&s_cell[wave][0]};
  const Split2 sp{h, lane, spare};
  St<L> s;
  if (!spare) {
#pragma unroll
    for (int p = 0; p < 4; p++)
#pragma unroll
      for (int t = 0; t < L / 2; t++) cs.set_slot(p, t, a.par[(size_t)(p * L + 2 * t + h) * n + c]);
    cs.set_sc(PS_FMAX, a.par[(size_t)(4 * L) * n + c]);
#pragma unroll
    for (int t = 0; t < L / 2; t++) cs.set_slot(PF_ROOTR, t, st[(size_t)(3 * L + 2 * t + h) * n + c]);
  }
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = st[(size_t)(0 * L + i - 1) * n + c];
    s.smp[i] = st[(size_t)(2 * L + i - 1) * n + c];
  }
  const size_t o8 = (size_t)(4 * L + 1) * n + c;
  s.zwt = st[o8 + 0 * (size_t)n];
  s.wa = st[o8 + 1 * (size_t)n];
  s.LAI = st[o8 + 2 * (size_t)n];
  s.LAI_litter = st[o8 + 3 * (size_t)n];
  s.pm = st[o8 + 4 * (size_t)n];
  s.pfm = st[o8 + 5 * (size_t)n];
  s.plen = st[o8 + 6 * (size_t)n];
  s.rdepth = st[o8 + 7 * (size_t)n];
  cs.launder();

  if (!spare) {
    // soil mask (HYBRID9.f90:122-123): SUM(theta_s) > trunc
    float ts_sum = zero;
#pragma unroll
    for (int i = 1; i <= L; i++) ts_sum = ts_sum + cs.lay(PF_TS, i);
    if (!(ts_sum > 1.0E-8f) || err[c] != 0) {
      if (h == 0)
#pragma unroll
        for (int r = 0; r < 12 + L; r++) a.annual[(size_t)r * ios + io] = __builtin_nanf("");
      return;
    }
    cell_inv_pair<L, G>(g, cs);
  }
  if (__builtin_amdgcn_ballot_w64(!spare) == 0) return;   // every pair masked out: the spare lanes leave too
  int eday = 0, estep = 0;
  float errval = 0.0f;
#if defined(H9G_STAMPS)
  StampProf pr{stamp_clock(), {0, 0, 0, 0, 0, 0, 0, 0}};
  const int code = cell_year_pair<L, G, Split2, PS, true>(g, cs, sp, s, (const gbl_float *)(a.forc + io), ios, a.fvar, nt,
                                                         a.nisurf, a.grow_on, (gbl_float *)(a.annual + io), ios, eday,
                                                         estep, errval, T, a.raw, pr);
  if (lane == 0 && a.stamps)
    for (int k = 0; k < 8; k++) a.stamps[(blockIdx.x * H9G_PWAVES + wave) * 8 + k] = pr.acc[k];
#else
  const int code = cell_year_pair<L, G>(g, cs, sp, s, (const gbl_float *)(a.forc + io), ios, a.fvar, nt, a.nisurf,
                                        a.grow_on, (gbl_float *)(a.annual + io), ios, eday, estep, errval, T, a.raw);
#endif
  if (spare || h != 0) return;       // the even lane writes the cell back
  int cw = c, iow = io;
  opaque(cw);
  opaque(iow);
  cs.launder();
  if (hist) hist[cw] = s.naq;
  const size_t ow = (size_t)(4 * L + 1) * n + cw;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    st[(size_t)(0 * L + i - 1) * n + cw] = s.h2o[i];
    st[(size_t)(2 * L + i - 1) * n + cw] = s.smp[i];
    if (a.grow_on) st[(size_t)(3 * L + i - 1) * n + cw] = cs.lay(PF_ROOTR, i);
  }
  if (a.grow_on) st[(size_t)(4 * L) * n + cw] = zero;   // rootr_col(Nlevgrnd)
  st[ow + 0 * (size_t)n] = s.zwt;
  st[ow + 1 * (size_t)n] = s.wa;
  st[ow + 2 * (size_t)n] = s.LAI;
  st[ow + 3 * (size_t)n] = s.LAI_litter;
  st[ow + 4 * (size_t)n] = s.pm;
  st[ow + 5 * (size_t)n] = s.pfm;
  st[ow + 6 * (size_t)n] = s.plen;
  st[ow + 7 * (size_t)n] = s.rdepth;
  if (code) {
    err[0 * (size_t)n + cw] = code;
    err[1 * (size_t)n + cw] = eday;
    err[2 * (size_t)n + cw] = estep;
    err[3 * (size_t)n + cw] = __builtin_bit_cast(int, errval);
    atomicOr(a.err_flag, 1);
#pragma unroll
    for (int r = 0; r < 12 + L; r++) a.annual[(size_t)r * ios + iow] = __builtin_nanf("");
  }
}

template <int L, class G>
__global__ void __launch_bounds__(64 * H9G_PWAVES)
    __attribute__((amdgpu_waves_per_eu(pair_waves<L>(), pair_waves<L>())))
h9g_pair_kernel(const KArgs a, const G g) {
  pair_body<L, G, pair_waves<L>()>(a, g);
}

// The pair kernel built for 2 waves per SIMD (round 4):
// 256 VGPRs, so the L = 10 substep does not spill (the 3-wave build spills
// 108 VGPRs and 118 SGPRs into a 296-B-per-lane scratch that reaches HBM),
// and 80 KB of LDS per workgroup, so every reciprocal field fits.  It trades
// a third of the resident waves for that; l10_kind picks it by shard size.
template <int L, class G>
__global__ void __launch_bounds__(64 * H9G_PWAVES) __attribute__((amdgpu_waves_per_eu(2, 2)))
h9g_pair2_kernel(const KArgs a, const G g) {
  pair_body<L, G, 2>(a, g);
}

// The pair kernel with 11 columns per wave (round 5): the 42
// lanes past the pairs help in the per-layer phases, which then take 2
// rounds instead of 5 at L = 10 (hydrology_pair helpers), and the wave's LDS
// block halves, so every reciprocal field fits at 3 waves per SIMD.  Twice
// the waves of 22-column ones for the same cells.  Measured on the 8-GPU
// config-5 shard (33,750 cells: 3,069 waves for 3,072 slots) it lost to
// pair2, so l10_kind never picks it; H9G_KERNEL=pair11
// selects it, and the GPU tests run it.
#define H9G_PCPW11 11
template <int L, class G>
__global__ void __launch_bounds__(64 * H9G_PWAVES) __attribute__((amdgpu_waves_per_eu(3, 3)))
h9g_pair11_kernel(const KArgs a, const G g) {
  pair_body<L, G, 3, H9G_PCPW11>(a, g);
}

// One column per wave (round 5): the 62 lanes past the pair help in the
// per-layer phases, which take one round each (hydrology_pair helpers), and
// the wave may hold every register (one wave per SIMD: no spills).  For the
// short lists of the cell-order re-runs (h9g_run_decade_ordered), whose
// years run as lone waves: a lone wave's year is latency-bound, and this
// cuts its per-layer rounds from 3 to 1 at L = 8 (from 5 to 1 at L = 10).
template <int L, class G>
__global__ void __launch_bounds__(64 * H9G_PWAVES) __attribute__((amdgpu_waves_per_eu(1, 1)))
h9g_pair1_kernel(const KArgs a, const G g) {
  pair_body<L, G, 1, 1>(a, g);
}


// Solo kernel: one lane per soil column running the generic code of
// h9g_pair.h with one lane doing every layer (SplitAll: two layers per
// scheduling region, tridiagonal rows eliminated as assembled).
template <int L, class G>
__global__ void __launch_bounds__(H9G_YBLOCK) __attribute__((amdgpu_waves_per_eu(2, 2)))
h9g_solo_kernel(const KArgs a, const G g) {
  typedef SoloStore<L> SS;
  __shared__ uint64_t s_e2[32];
  __shared__ double s_l2[32];
  __shared__ float s_cell[SS::ROWS * H9G_YBLOCK];
  __shared__ float s_zt[zt_size<L>()];
  if (threadIdx.x == 0) fill_zt<L>(g, s_zt);
  load_tabs(s_e2, s_l2);
  const h9m::Tabs T = {s_e2, s_l2};
  const int slot = a.c0 + (int)(xcd_vwg(blockIdx.x, gridDim.x) * blockDim.x + threadIdx.x);
  if (slot >= a.cend) return;
  const int c = a.perm ? a.perm[slot] : slot;
  const int io = a.sorted_io ? slot : c;
  const int n = a.ncell;
  const size_t ios = a.sorted_io ? a.iostride : (size_t)n;
  SS cs{(lds_float *)&s_cell[threadIdx.x], (const lds_float *)s_zt};
  const SplitAll sp;
  St<L> s;
#pragma unroll
  for (int p = 0; p < 4; p++)
#pragma unroll
    for (int i = 1; i <= L; i++) cs.set_lay(p, i, a.par[(size_t)(p * L + i - 1) * n + c]);
  cs.set_sc(PS_FMAX, a.par[(size_t)(4 * L) * n + c]);
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = a.st[(size_t)(0 * L + i - 1) * n + c];
    s.smp[i] = a.st[(size_t)(2 * L + i - 1) * n + c];
    cs.set_lay(PF_ROOTR, i, a.st[(size_t)(3 * L + i - 1) * n + c]);
  }
  const size_t o8 = (size_t)(4 * L + 1) * n + c;
  s.zwt = a.st[o8 + 0 * (size_t)n];
  s.wa = a.st[o8 + 1 * (size_t)n];
  s.LAI = a.st[o8 + 2 * (size_t)n];
  s.LAI_litter = a.st[o8 + 3 * (size_t)n];
  s.pm = a.st[o8 + 4 * (size_t)n];
  s.pfm = a.st[o8 + 5 * (size_t)n];
  s.plen = a.st[o8 + 6 * (size_t)n];
  s.rdepth = a.st[o8 + 7 * (size_t)n];
  cs.launder();
  float ts_sum = zero;
#pragma unroll
  for (int i = 1; i <= L; i++) ts_sum = ts_sum + cs.lay(PF_TS, i);
  if (!(ts_sum > 1.0E-8f) || a.err[c] != 0) {
#pragma unroll
    for (int r = 0; r < 12 + L; r++) a.annual[(size_t)r * ios + io] = __builtin_nanf("");
    return;
  }
  cell_inv_pair<L, G>(g, cs);
  int eday = 0, estep = 0;
  float errval = 0.0f;
  const int code = cell_year_pair<L, G, SplitAll, SS, false>(g, cs, sp, s, (const gbl_float *)(a.forc + io), ios, a.fvar,
                                                             a.nt, a.nisurf, a.grow_on, (gbl_float *)(a.annual + io),
                                                             ios, eday, estep, errval, T, a.raw);
  int cw = c, iow = io;
  opaque(cw);
  opaque(iow);
  cs.launder();
  if (a.hist) a.hist[cw] = s.naq;
  const size_t ow = (size_t)(4 * L + 1) * n + cw;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    a.st[(size_t)(0 * L + i - 1) * n + cw] = s.h2o[i];
    a.st[(size_t)(2 * L + i - 1) * n + cw] = s.smp[i];
    if (a.grow_on) a.st[(size_t)(3 * L + i - 1) * n + cw] = cs.lay(PF_ROOTR, i);
  }
  if (a.grow_on) a.st[(size_t)(4 * L) * n + cw] = zero;
  a.st[ow + 0 * (size_t)n] = s.zwt;
  a.st[ow + 1 * (size_t)n] = s.wa;
  a.st[ow + 2 * (size_t)n] = s.LAI;
  a.st[ow + 3 * (size_t)n] = s.LAI_litter;
  a.st[ow + 4 * (size_t)n] = s.pm;
  a.st[ow + 5 * (size_t)n] = s.pfm;
  a.st[ow + 6 * (size_t)n] = s.plen;
  a.st[ow + 7 * (size_t)n] = s.rdepth;
  if (code) {
    a.err[0 * (size_t)n + cw] = code;
    a.err[1 * (size_t)n + cw] = eday;
    a.err[2 * (size_t)n + cw] = estep;
    a.err[3 * (size_t)n + cw] = __builtin_bit_cast(int, errval);
    atomicOr(a.err_flag, 1);
#pragma unroll
    for (int r = 0; r < 12 + L; r++) a.annual[(size_t)r * ios + iow] = __builtin_nanf("");
  }
}

// The year's forcing in the year kernel's slot order (round 4, VERDICT r03
// #5): dst[v][d][s] = src[v][d][perm[s]].  With the cells re-ordered each
// year (h9g_sort_kernel), a wave's daily forcing loads by cell id scattered
// over its XCD's range, so the non-temporal loads of neighbouring lanes hit
// different lines: 4.45 GB fetched per config-2 launch for 0.69 GB of
// forcing (pmc_r03i.json).  One gather per year makes every wave's daily
// loads contiguous again.  XCD-aware like the year kernel: the launch range
// [c0, cend) is cut into the year kernel's workgroups of cpb slots, dealt to
// the XCDs as xcd_vwg deals them, and block L (XCD L % 8) copies PF_ROWS
// rows of one workgroup of XCD L % 8 -- so it reads only cells of its own
// XCD's range, which the sort never leaves.
#define H9G_PF_ROWS 32
// Source rows have stride n (a forcing slot, variables fvar apart); the
// slot-ordered copy has stride ds (variables dvar apart).
__global__ void __launch_bounds__(256) h9g_perm_forcing_kernel(int c0, int cend, int cpb, int nt, int n, size_t fvar,
                                                               size_t ds, size_t dvar, const int *__restrict__ perm,
                                                               const float *__restrict__ src, float *__restrict__ dst) {
  const unsigned nb = (unsigned)((cend - c0 + cpb - 1) / cpb), x = blockIdx.x % H9G_NXCD, j = blockIdx.x / H9G_NXCD;
  const unsigned q = nb / H9G_NXCD, r = nb % H9G_NXCD, cnt = q + (x < r ? 1u : 0u);
  const unsigned rows = 7u * (unsigned)nt, rgroups = (rows + H9G_PF_ROWS - 1) / H9G_PF_ROWS;
  if (cnt == 0 || j >= cnt * rgroups) return;
  const unsigned v = x * q + (x < r ? x : r) + j % cnt, r0 = (j / cnt) * H9G_PF_ROWS;
  for (unsigned t = threadIdx.x; t < (unsigned)cpb * H9G_PF_ROWS; t += blockDim.x) {
    const int s = c0 + (int)(v * (unsigned)cpb + t % (unsigned)cpb);
    const unsigned row = r0 + t / (unsigned)cpb;
    if (s >= cend || row >= rows) continue;
    const size_t v = row / (unsigned)nt, d = row % (unsigned)nt;
    dst[v * dvar + d * ds + s] = src[v * fvar + d * (size_t)n + perm[s]];
  }
}
static unsigned perm_forcing_blocks(int c0, int cend, int cpb, int nt) {
  const unsigned nb = (unsigned)((cend - c0 + cpb - 1) / cpb);
  const unsigned cmax = nb / H9G_NXCD + (nb % H9G_NXCD ? 1u : 0u);
  return H9G_NXCD * cmax * ((7u * (unsigned)nt + H9G_PF_ROWS - 1) / H9G_PF_ROWS);
}

// The annual sums of a sorted year kernel (slot order, rows of stride ss)
// back to cell order (rows of stride n): the m slots from s0 of the launch.
__global__ void __launch_bounds__(256) h9g_unperm_annual_kernel(int m, int n, int rows, int s0, size_t ss,
                                                                const int *__restrict__ perm,
                                                                const float *__restrict__ src, float *__restrict__ dst) {
  const int s = s0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (s >= s0 + m) return;
  const int c = perm[s];
  for (int r = blockIdx.y; r < rows; r += gridDim.y) dst[(size_t)r * n + c] = src[(size_t)r * ss + s];
}

// Cell-order mode (h9g_run_decade_ordered).  The reference's cell loop
// (HYBRID9.f90:120-295) leaves the module array smp (SHARED.f90:198) as the
// last cell's, and the next cell's first substep reads it in beta
// (HYDROLOGY.f90:270-275).  The m land cells (context order) form chains,
// one per reference rank (h9g_set_chains); position j starts a decade from
// the smp its predecessor pred[j] holds now, or, for a chain's first cell
// (first[j]), from what the chain's last cell pred[j] held when the decade
// started.  h9g_chain_kernel compares that with the smp the cell last
// started from (guess, L rows of n), takes it over where it differs and
// flags the cell for a re-run.  st: every cell's state at the decade's end
// as known now.  dirty (may be null): cells whose decade start changed after
// the first pass ran (h9g_settle_kernel), flagged whatever their input.
__global__ void __launch_bounds__(256) h9g_chain_kernel(int m, int n, int L, const int *__restrict__ chain,
                                                        const int *__restrict__ pred, const int *__restrict__ first,
                                                        const float *__restrict__ st, const float *__restrict__ st0,
                                                        float *__restrict__ guess, const int *__restrict__ dirty,
                                                        int *__restrict__ flag) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int k = chain[j];
  const float *src = first[j] ? st0 : st;
  const int p = pred[j];
  int differ = 0;
  for (int i = 0; i < L; i++) {
    const float v = src[(size_t)(2 * L + i) * n + p];
    differ |= __float_as_uint(v) != __float_as_uint(guess[(size_t)i * n + k]);
    guess[(size_t)i * n + k] = v;
  }
  flag[j] = differ | (dirty && dirty[k] ? 2 : 0);   // 1: input changed, 2: start changed
}

// The cell order's day-1 probe (round 6).  The input smp reaches a cell only
// through beta of its decade's first substep (HYDROLOGY.f90:270-275).  A
// cell whose input changed ran the day from its old and from its new input
// (one-day list launches from the decade's start, running sums undivided,
// KArgs::raw): if the two agree bit for bit at the day's end -- every state
// row, the STOP record and every running sum of the year's means -- the
// days after it and so the whole decade are the same from either input, and
// the cell needs no re-run (its trajectory is already the one its new input
// gives).  keep[j] = 1: they differ, the cell re-runs.
__global__ void __launch_bounds__(256) h9g_probe_cmp_kernel(int m, int n, int srows, int rows,
                                                            const int *__restrict__ list,
                                                            const float *__restrict__ stA, const float *__restrict__ stB,
                                                            const int *__restrict__ errA, const int *__restrict__ errB,
                                                            const float *__restrict__ annA,
                                                            const float *__restrict__ annB, int *__restrict__ keep) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int c = list[j];
  bool same = true;
  for (int r = 0; r < srows; r++)
    same &= __float_as_uint(stA[(size_t)r * n + c]) == __float_as_uint(stB[(size_t)r * n + c]);
  for (int r = 0; r < 4; r++) same &= errA[(size_t)r * n + c] == errB[(size_t)r * n + c];
  for (int r = 0; r < rows; r++)
    same &= __float_as_uint(annA[(size_t)r * n + c]) == __float_as_uint(annB[(size_t)r * n + c]);
  keep[j] = !same;
}

// Pipelined decades (h9g_run_ordered): decade D+1's first pass starts from
// every cell's state as known when decade D's first pass and year-1 re-run
// are done (st0); the cells D's later re-runs still change get their final
// D end state (fin, fin_err) here once D has settled, and are marked dirty.
// A dirty cell that has now STOPped (err0 != 0) leaves D+1: its state and
// STOP record go back into the context (st, err) and D+1's last-year
// checkpoint, and its annual means of D+1 (ny years of rows x n) are NaN.
__global__ void __launch_bounds__(256) h9g_settle_kernel(int n, int srows, int rows, int ny,
                                                         const float *__restrict__ fin, const int *__restrict__ fin_err,
                                                         float *__restrict__ st0, int *__restrict__ err0,
                                                         int *__restrict__ dirty, float *__restrict__ st,
                                                         int *__restrict__ err, float *__restrict__ ck_last,
                                                         int *__restrict__ eck_last, float *__restrict__ ann) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  bool same = true;
  for (int r = 0; r < srows; r++)
    same &= __float_as_uint(fin[(size_t)r * n + c]) == __float_as_uint(st0[(size_t)r * n + c]);
  for (int r = 0; r < 4; r++) same &= fin_err[(size_t)r * n + c] == err0[(size_t)r * n + c];
  if (same) return;
  for (int r = 0; r < srows; r++) st0[(size_t)r * n + c] = fin[(size_t)r * n + c];
  for (int r = 0; r < 4; r++) err0[(size_t)r * n + c] = fin_err[(size_t)r * n + c];
  dirty[c] = 1;
  if (err0[c] == 0) return;
  for (int r = 0; r < srows; r++) {
    st[(size_t)r * n + c] = st0[(size_t)r * n + c];
    ck_last[(size_t)r * n + c] = st0[(size_t)r * n + c];
  }
  for (int r = 0; r < 4; r++) {
    err[(size_t)r * n + c] = err0[(size_t)r * n + c];
    eck_last[(size_t)r * n + c] = err0[(size_t)r * n + c];
  }
  for (int y = 0; y < ny; y++)
    for (int r = 0; r < rows; r++) ann[((size_t)y * rows + r) * n + c] = __builtin_nanf("");
}

// Pass 0's input of every chain's first cell: the smp its chain's last cell
// holds when the decade starts (into the state and the guess).
__global__ void __launch_bounds__(256) h9g_chain_start_kernel(int m, int n, int L, const int *__restrict__ chain,
                                                              const int *__restrict__ pred, const int *__restrict__ first,
                                                              const float *__restrict__ st0, float *__restrict__ st,
                                                              float *__restrict__ guess) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m || !first[j]) return;
  const int k = chain[j], p = pred[j];
  for (int i = 0; i < L; i++) {
    const float v = st0[(size_t)(2 * L + i) * n + p];
    st[(size_t)(2 * L + i) * n + k] = v;
    guess[(size_t)i * n + k] = v;
  }
}

// The listed cells back to the decade's starting state (state rows and STOP
// record), starting from the smp in guess.
__global__ void __launch_bounds__(256) h9g_restart_kernel(int m, int n, int L, const int *__restrict__ list,
                                                          const float *__restrict__ st0, const int *__restrict__ err0,
                                                          const float *__restrict__ guess, float *__restrict__ st,
                                                          int *__restrict__ err) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int k = list[j];
  const int rows = 4 * L + 9;
  for (int r = 0; r < rows; r++) st[(size_t)r * n + k] = st0[(size_t)r * n + k];
  for (int i = 0; i < L; i++) st[(size_t)(2 * L + i) * n + k] = guess[(size_t)i * n + k];
  for (int r = 0; r < 4; r++) err[(size_t)r * n + k] = err0[(size_t)r * n + k];
}

// A re-run cell's trajectory against the one its last run took (ckpt: the
// state and STOP record at the end of the same year).  The state and the
// STOP record are everything a year carries into the next (the c4_spinup
// decade carry), so a cell whose end-of-year state equals the old one's bit
// for bit runs the rest of the decade exactly as it did: it leaves the
// re-run with the old run's end-of-decade state (ckpt_last), its later
// annual means stand, and keep[j] = 0.  Otherwise its new state becomes the
// checkpoint and it runs on (keep[j] = 1).
__global__ void __launch_bounds__(256) h9g_merge_kernel(int m, int n, int rows, const int *__restrict__ list,
                                                        float *__restrict__ st, int *__restrict__ err,
                                                        float *__restrict__ ckpt, int *__restrict__ eckpt,
                                                        const float *__restrict__ ckpt_last,
                                                        const int *__restrict__ eckpt_last, int *__restrict__ keep) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const int k = list[j];
  bool same = true;
  for (int r = 0; r < rows; r++)
    same &= __float_as_uint(st[(size_t)r * n + k]) == __float_as_uint(ckpt[(size_t)r * n + k]);
  for (int r = 0; r < 4; r++) same &= err[(size_t)r * n + k] == eckpt[(size_t)r * n + k];
  if (same) {
    for (int r = 0; r < rows; r++) st[(size_t)r * n + k] = ckpt_last[(size_t)r * n + k];
    for (int r = 0; r < 4; r++) err[(size_t)r * n + k] = eckpt_last[(size_t)r * n + k];
  } else {
    for (int r = 0; r < rows; r++) ckpt[(size_t)r * n + k] = st[(size_t)r * n + k];
    for (int r = 0; r < 4; r++) eckpt[(size_t)r * n + k] = err[(size_t)r * n + k];
  }
  keep[j] = !same;
}

// Cell order of the next year kernel: a stable counting sort of the cells
// by where their water table was over the last year, failed cells last.
// Cells are independent, so the order changes no result; it makes the 22
// columns of a wave take the same branches that depend on the layer holding
// the water table (jwt, HYDROLOGY.f90:499-508): the equilibrium-profile cases
// (:517-567), the aquifer node (:574-590, :737-741) for jwt = L, the recharge
// (:856-904) and the water-table and drainage loops (:923-1118) for jwt < L.
// A wave holding both kinds of column runs both.  Keys:
//   0 .. L-1   no substep of the last year below the column: the current jwt
//   L .. L+7   some: the fraction of the year's substeps below it, in eighths
//   L+8        every substep below the column
//   L+9        failed
// Without a last year (hist < 0) the current jwt decides (jwt = L: key L+8).
// Round 2 sorted by the current jwt alone; cells whose water table crosses
// the column's bottom during the year then sat in waves of both kinds
// (measured with H9G_COUNT_BRANCH at 1906-1907: 84% of the wave-substeps ran
// the aquifer node, 81% the recharge).  Block x sorts the slots of XCD x's
// workgroups of the year launch over [c0, cend) with cpb cells per workgroup
// (xcd_vwg), so no cell leaves its XCD's range.  list (may be null): the
// slots hold the cells list[c0 .. cend) instead of c0 .. cend (the cell
// order's re-run lists; round 6).
#define H9G_SORT_THREADS 512
template <int L, class G>
__global__ void __launch_bounds__(H9G_SORT_THREADS)
    h9g_sort_kernel(int n, int c0, int cend, int cpb, const float *__restrict__ st, const int *__restrict__ err,
                    const int *__restrict__ hist, int nsub, int *__restrict__ perm, const int *__restrict__ list,
                    const G g) {
  constexpr int NK = L + 10;
  constexpr int NTH = H9G_SORT_THREADS;
  __shared__ int cnt[NK][NTH];
  __shared__ int base[NK];
  const int t = threadIdx.x;
  const unsigned nb = (unsigned)((cend - c0 + cpb - 1) / cpb), x = blockIdx.x;
  const unsigned q = nb / H9G_NXCD, r = nb % H9G_NXCD;
  const int p0 = c0 + (int)(x * q + (x < r ? x : r)) * cpb;
  const int p1 = min(cend, p0 + (int)(q + (x < r ? 1u : 0u)) * cpb);
  const int m = p1 - p0;
  if (m <= 0) return;                      // (uniform per block)
  const int per = (m + NTH - 1) / NTH;
  const int b = p0 + t * per, e = min(p1, b + per);
  float zim[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) zim[i] = g.zim(i);
  const float *zwt = st + (size_t)(4 * L + 1) * n;
  auto key = [&](int c) -> int {
    if (err[c]) return L + 9;
    const int j = jwt_of<L>(zwt[c], zim);
    const int h = hist ? hist[c] : -1;
    if (h < 0 || nsub <= 0) return j < L ? j : L + 8;
    if (h == 0) return j < L ? j : L;
    if (h >= nsub) return L + 8;
    return L + (int)((long long)h * 8 / nsub);
  };
  int loc[NK];
#pragma unroll
  for (int k = 0; k < NK; k++) loc[k] = 0;
  for (int c = b; c < e; c++) {
    const int k = key(list ? list[c] : c);
#pragma unroll
    for (int j = 0; j < NK; j++) loc[j] += (j == k);
  }
#pragma unroll
  for (int k = 0; k < NK; k++) cnt[k][t] = loc[k];
  __syncthreads();
  if (t < NK) {                   // exclusive scan of each key's counts over the threads
    int sum = 0;
    for (int j = 0; j < NTH; j++) {
      const int v = cnt[t][j];
      cnt[t][j] = sum;
      sum += v;
    }
    base[t] = sum;
  }
  __syncthreads();
  if (t == 0) {
    int sum = 0;
    for (int k = 0; k < NK; k++) {
      const int v = base[k];
      base[k] = sum;
      sum += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NK; k++) loc[k] = base[k] + cnt[k][t];
  for (int c = b; c < e; c++) {
    const int cell = list ? list[c] : c;
    const int k = key(cell);
    int pos = 0;
#pragma unroll
    for (int j = 0; j < NK; j++)
      if (j == k) pos = loc[j]++;
    perm[p0 + pos] = cell;
  }
}

// LCLIM single-site kernel (HYBRID9.f90:339-480): one lane per site,
// cell_site of h9g_pair.h.  Parameters and state as the year kernels.
struct SiteArgs {
  int ncell, nday, nisurf;
  const float *__restrict__ par;
  float *__restrict__ st;
  const float *__restrict__ sub, *__restrict__ daily, *__restrict__ lai;
  float *__restrict__ out;
  int *__restrict__ err;
  int *__restrict__ err_flag;
};

template <int L, class G>
__global__ void __launch_bounds__(64) h9g_site_kernel(const SiteArgs a, const G g) {
  typedef SoloStore<L> SS;
  __shared__ uint64_t s_e2[32];
  __shared__ double s_l2[32];
  __shared__ float s_cell[SS::ROWS * 64];
  __shared__ float s_zt[zt_size<L>()];
  if (threadIdx.x == 0) fill_zt<L>(g, s_zt);
  load_tabs(s_e2, s_l2);
  const h9m::Tabs T = {s_e2, s_l2};
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.ncell) return;
  const int n = a.ncell;
  SS cs{(lds_float *)&s_cell[threadIdx.x], (const lds_float *)s_zt};
  St<L> s;
#pragma unroll
  for (int p = 0; p < 4; p++)
#pragma unroll
    for (int i = 1; i <= L; i++) cs.set_lay(p, i, a.par[(size_t)(p * L + i - 1) * n + c]);
  cs.set_sc(PS_FMAX, a.par[(size_t)(4 * L) * n + c]);
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = a.st[(size_t)(0 * L + i - 1) * n + c];
    s.smp[i] = a.st[(size_t)(2 * L + i - 1) * n + c];
    cs.set_lay(PF_ROOTR, i, a.st[(size_t)(3 * L + i - 1) * n + c]);
  }
  const float h2o_ma1 = a.st[(size_t)(1 * L) * n + c];
  const size_t o8 = (size_t)(4 * L + 1) * n + c;
  s.zwt = a.st[o8 + 0 * (size_t)n];
  s.wa = a.st[o8 + 1 * (size_t)n];
  s.LAI = a.st[o8 + 2 * (size_t)n];
  s.LAI_litter = a.st[o8 + 3 * (size_t)n];
  s.pm = a.st[o8 + 4 * (size_t)n];
  s.pfm = a.st[o8 + 5 * (size_t)n];
  s.plen = a.st[o8 + 6 * (size_t)n];
  s.rdepth = a.st[o8 + 7 * (size_t)n];
  float ts_sum = zero;
#pragma unroll
  for (int i = 1; i <= L; i++) ts_sum = ts_sum + cs.lay(PF_TS, i);
  if (!(ts_sum > 1.0E-8f) || a.err[c] != 0) {
    for (int d = 0; d < a.nday; d++)
      for (int r = 0; r < 11; r++) a.out[((size_t)d * 11 + r) * n + c] = __builtin_nanf("");
    return;
  }
  cell_inv_pair<L, G>(g, cs);
  int eday = 0, estep = 0;
  float errval = 0.0f;
  const int code = cell_site<L, G, SS>(g, cs, s, h2o_ma1, a.sub + c, a.daily + c, a.lai + c, a.out + c,
                                       (size_t)n, a.nday, a.nisurf, eday, estep, errval, T);
  const size_t ow = (size_t)(4 * L + 1) * n + c;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    a.st[(size_t)(0 * L + i - 1) * n + c] = s.h2o[i];
    a.st[(size_t)(2 * L + i - 1) * n + c] = s.smp[i];
  }
  a.st[ow + 0 * (size_t)n] = s.zwt;
  a.st[ow + 1 * (size_t)n] = s.wa;
  a.st[ow + 2 * (size_t)n] = s.LAI;
  a.st[ow + 3 * (size_t)n] = s.LAI_litter;
  if (code) {
    a.err[0 * (size_t)n + c] = code;
    a.err[1 * (size_t)n + c] = eday;
    a.err[2 * (size_t)n + c] = estep;
    a.err[3 * (size_t)n + c] = __builtin_bit_cast(int, errval);
    atomicOr(a.err_flag, 1);
    for (int d = eday; d < a.nday; d++)
      for (int r = 0; r < 11; r++) a.out[((size_t)d * 11 + r) * n + c] = __builtin_nanf("");
  }
}

template <int L, class G>
__global__ void __launch_bounds__(H9G_BLOCK) h9g_init_kernel(int ncell, const float *__restrict__ par,
                                                             float *__restrict__ st, const G g) {
  __shared__ uint64_t s_e2[32];
  __shared__ double s_l2[32];
  load_tabs(s_e2, s_l2);
  MathExact me{{s_e2, s_l2}};
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncell) return;
  const int n = ncell;
  float ts[L + 1];
  St<L> s;
  float h2o_ma[L + 1], rootr[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) ts[i] = par[(size_t)(i - 1) * n + c];
  init_cell<L, G, MathExact>(g, ts, s, rootr, h2o_ma, me);
#pragma unroll
  for (int i = 1; i <= L; i++) {
    st[(size_t)(0 * L + i - 1) * n + c] = s.h2o[i];
    st[(size_t)(1 * L + i - 1) * n + c] = h2o_ma[i];
    st[(size_t)(2 * L + i - 1) * n + c] = s.smp[i];
    st[(size_t)(3 * L + i - 1) * n + c] = rootr[i];
  }
  st[(size_t)(4 * L) * n + c] = zero;
  const size_t o8 = (size_t)(4 * L + 1) * n + c;
  st[o8 + 0 * (size_t)n] = s.zwt;
  st[o8 + 1 * (size_t)n] = s.wa;
  st[o8 + 2 * (size_t)n] = s.LAI;
  st[o8 + 3 * (size_t)n] = s.LAI_litter;
  st[o8 + 4 * (size_t)n] = s.pm;
  st[o8 + 5 * (size_t)n] = s.pfm;
  st[o8 + 6 * (size_t)n] = s.plen;
  st[o8 + 7 * (size_t)n] = s.rdepth;
}

// deterministic FP64 diagnostics: one block, fixed strided order + tree
__global__ void __launch_bounds__(1024) h9g_diag_kernel(int ncell, int L, const float *__restrict__ annual,
                                                        const float *__restrict__ st,
                                                        const int *__restrict__ err, double *__restrict__ out) {
  __shared__ double red[1024];
  double acc[H9G_NDIAG];
  for (int k = 0; k < H9G_NDIAG; k++) acc[k] = 0.0;
  const size_t n = ncell;
  const size_t o8 = (size_t)(4 * L + 1) * n;
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) {
    const float rnf = annual[2 * n + c];
    if (err[c] != 0) { acc[11] += 1.0; continue; }
    if (rnf != rnf) continue;                    // non-soil cell
    acc[0] += 1.0;
    acc[1] += (double)rnf;
    acc[2] += (double)annual[(size_t)(11 + L) * n + c];
    acc[3] += (double)st[o8 + 0 * n + c];
    acc[4] += (double)st[o8 + 1 * n + c];
    acc[5] += (double)annual[0 * n + c];
    acc[6] += (double)annual[1 * n + c];
    acc[7] += (double)st[o8 + 2 * n + c];
    acc[8] += (double)annual[11 * n + c];
    acc[9] += (double)annual[4 * n + c];
    acc[10] += (double)annual[9 * n + c];
  }
  for (int k = 0; k < H9G_NDIAG; k++) {
    red[threadIdx.x] = acc[k];
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[k] = red[0];
    __syncthreads();
  }
}

template <int L>
__global__ void __launch_bounds__(H9G_BLOCK) h9g_synth_params_kernel(int ncell, const int64_t *__restrict__ gid,
                                                                     uint64_t seed, float *__restrict__ par) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncell) return;
  const size_t n = ncell;
  const uint64_t g = (uint64_t)gid[c];
#pragma unroll
  for (int l = 0; l < L; l++) {
    float ts, hk, b, ps;
    h9s::params(seed, g, l, &ts, &hk, &b, &ps);
    par[(size_t)(0 * L + l) * n + c] = ts;
    par[(size_t)(1 * L + l) * n + c] = hk;
    par[(size_t)(2 * L + l) * n + c] = b;
    par[(size_t)(3 * L + l) * n + c] = ps;
  }
  par[(size_t)(4 * L) * n + c] = h9s::fmax_param(seed, g);
}

__global__ void __launch_bounds__(H9G_BLOCK) h9g_synth_forcing_kernel(int ncell, int nday, int day0,
                                                                      const int64_t *__restrict__ gid,
                                                                      const float *__restrict__ lat, uint64_t seed,
                                                                      size_t fvar, float *__restrict__ forc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const int d = blockIdx.y;
  if (c >= ncell || d >= nday) return;
  float v[7];
  h9s::forcing(seed, (uint64_t)gid[c], lat[c], (int64_t)day0 + d, v);
#pragma unroll
  for (int k = 0; k < 7; k++) forc[k * fvar + (size_t)d * ncell + c] = v[k];
}

// ---------------------------------------------------------------------------
// Soil parameter build, INIT.f90:575-631: each 0.5 deg
// cell of the context averages its 60x60 block of 30" pixels whose
// theta_s >= 0, then converts units.  The reference sums sequentially
// (x1 outer, y1 inner).  h9g_soil_kernel reads the block coalesced (a wave
// per pixel row) and reduces in a tree; that equals the sequential sum
// bit for bit whenever every contributing value is an integer of
// magnitude <= 4096 (the BNU fields are stored as scaled integers): all
// partial sums are then exact floats below 2^24.  Any other block is
// flagged and summed in the reference's order by h9g_soil_seq_kernel.
// ---------------------------------------------------------------------------
#define H9G_SWAVES 4
struct SoilOut {
  __device__ __forceinline__ static void store(float *par, int L, int layer, size_t n, int c, int v,
                                                float sum, int j) {
    float m = sum;
    if (j > 0) m = m / (float)j;                                  // INIT.f90:593-598
    float out;
    if (v == 0) out = m / 1.0E3f;                                 // theta_s      :613
    else if (v == 1) out = 10.0f * m / 86400.0f;                  // hksat        :614
    else if (v == 2) out = 1.0f / MAXF(m / 1.0E3f, 1.0E-8f);      // bsw          :615,624,628
    else out = 10.0f * m;                                         // psi_s        :616
    par[(size_t)(v * L + layer) * n + c] = out;
  }
};

__device__ __forceinline__ bool small_int(float v) { return v == __builtin_truncf(v) && __builtin_fabsf(v) <= 4096.0f; }

__global__ void __launch_bounds__(64 * H9G_SWAVES) h9g_soil_kernel(int nx, int ncell, const int64_t *__restrict__ gid,
                                                                  const float *__restrict__ ts,
                                                                  const float *__restrict__ ks,
                                                                  const float *__restrict__ lm,
                                                                  const float *__restrict__ ps, size_t pitch, int L,
                                                                  int layer, float *__restrict__ par,
                                                                  int *__restrict__ slow) {
  __shared__ float red[H9G_SWAVES][5];
  __shared__ int red_ok[H9G_SWAVES];
  const int c = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t g = gid[c];
  const int x = (int)(g % nx), y = (int)(g / nx);
  const size_t base = (size_t)y * 60 * pitch + (size_t)x * 60 + lane;
  float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f, sj = 0.0f;
  bool ok = true;
  if (lane < 60) {
#pragma unroll 5
    for (int r = wave; r < 60; r += H9G_SWAVES) {                 // one pixel row per wave
      const size_t i = base + (size_t)r * pitch;
      const float a = ts[i];
      if (a >= 0.0f) {                                            // :584
        const float b = ks[i], d = lm[i], e = ps[i];
        s0 += a; s1 += b; s2 += d; s3 += e; sj += 1.0f;
        ok = ok && small_int(a) && small_int(b) && small_int(d) && small_int(e);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {                              // wave tree (exact: see above)
    s0 += __shfl_xor(s0, o); s1 += __shfl_xor(s1, o); s2 += __shfl_xor(s2, o);
    s3 += __shfl_xor(s3, o); sj += __shfl_xor(sj, o);
  }
  const bool wok = __builtin_amdgcn_ballot_w64(!ok) == 0;
  if (lane == 0) {
    red[wave][0] = s0; red[wave][1] = s1; red[wave][2] = s2; red[wave][3] = s3; red[wave][4] = sj;
    red_ok[wave] = wok;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int v = threadIdx.x;
    bool all = true;
    float sum = 0.0f, cnt = 0.0f;
    for (int w = 0; w < H9G_SWAVES; w++) {
      all = all && red_ok[w];
      sum += red[w][v];
      cnt += red[w][4];
    }
    if (!all) {
      if (v == 0) slow[c] = 1;
    } else {
      SoilOut::store(par, L, layer, (size_t)ncell, c, v, sum, (int)cnt);
    }
  }
}

// The reference's order for the flagged blocks: thread (cell, variable).
__global__ void h9g_soil_seq_kernel(int nx, int ncell, const int64_t *__restrict__ gid, const float *__restrict__ ts,
                                    const float *__restrict__ ks, const float *__restrict__ lm,
                                    const float *__restrict__ ps, size_t pitch, int L, int layer,
                                    float *__restrict__ par, const int *__restrict__ slow) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = t >> 2, v = t & 3;
  if (c >= ncell || !slow[c]) return;
  const float *src = v == 0 ? ts : (v == 1 ? ks : (v == 2 ? lm : ps));
  const int64_t g = gid[c];
  const int x = (int)(g % nx), y = (int)(g / nx);
  float sum = 0.0f;
  int j = 0;
  for (int x1 = x * 60; x1 < x * 60 + 60; x1++)                  // :582-592, x1 outer
    for (int y1 = y * 60; y1 < y * 60 + 60; y1++) {
      const size_t i = (size_t)y1 * pitch + x1;
      if (ts[i] >= 0.0f) {
        sum = sum + src[i];
        j = j + 1;
      }
    }
  SoilOut::store(par, L, layer, (size_t)ncell, c, v, sum, j);
}

// Probe of the hardware ids pace_key decodes (h9g_pair.h): the
// pair kernel's launch shape and LDS footprint (dynamic LDS of the same size,
// so the same workgroups per CU), each wave's lane 0 arriving at a bounded
// barrier (s_sleep, at most `spin` shader cycles) and then recording
// HW_REG_HW_ID, HW_REG_XCC_ID and whether every wave had arrived, i.e. was
// resident at once.  out: 3 words per wave (blockIdx * waves + wave).
__global__ void __launch_bounds__(64 * H9G_PWAVES) h9g_pace_probe_kernel(unsigned *out, unsigned *arrive,
                                                                         unsigned total, long long spin) {
  extern __shared__ float pad[];
  if (threadIdx.x & 63) return;
  pad[threadIdx.x] = 0.0f;
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long t0 = clock64();
  unsigned seen = 0;
  while ((seen = __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < total &&
         clock64() - t0 < spin)
    __builtin_amdgcn_s_sleep(2);
  out[3 * w + 0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);           // HW_REG_HW_ID
  out[3 * w + 1] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;     // HW_REG_XCC_ID
  out[3 * w + 2] = seen >= total ? 1u : 0u;
}

// MathFast's division path with a device-computed reciprocal (recip64).
__global__ void h9g_div_kernel(int n, const float *x, const float *d, float *out, int *flag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  MathFast mf{{nullptr, nullptr}, false};
  out[i] = mf.div(x[i], d[i], recip64(d[i]));
  flag[i] = (mf.special || mf.redone) ? 1 : 0;     // 1: the quotient was redone as x / d
}

__global__ void h9g_math_kernel(int n, const float *x, const float *y, float *out) {
  __shared__ uint64_t s_e2[32];
  __shared__ double s_l2[32];
  load_tabs(s_e2, s_l2);
  const h9m::Tabs T = {s_e2, s_l2};
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = y ? h9m::powf(x[i], y[i], T) : h9m::expf(x[i], T);
}

// The year kernels' math (MathFast: glibc's main path, the rest redone in
// place); flag = 1 where it was redone.
__global__ void h9g_math_fast_kernel(int n, const float *x, const float *y, float *out, int *flag) {
  __shared__ uint64_t s_e2[32];
  __shared__ double s_l2[32];
  load_tabs(s_e2, s_l2);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  MathFast mf{{s_e2, s_l2}, false};
  out[i] = y ? mf.powf(x[i], y[i]) : mf.expf(x[i]);
  flag[i] = mf.redone ? 1 : 0;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct h9g_ctx {
  h9g_config cfg;
  int device = 0;
  int L = 8;
  size_t n = 0;
  hipStream_t sc = nullptr, sx = nullptr;      // compute, copy
  float *d_par = nullptr, *d_st = nullptr, *d_forc = nullptr, *d_ann = nullptr;
  int *d_err = nullptr, *d_errflag = nullptr;
  double *d_diag = nullptr;
  int64_t *d_gid = nullptr;
  float *d_lat = nullptr;
  std::vector<int> slot_days;
  std::vector<hipEvent_t> ev_copied, ev_consumed;
  hipEvent_t ev0[NEVT], ev1[NEVT];
  hipEvent_t ev_ext = nullptr, ev_diag = nullptr;   // h9g_get_diagnostics_async ordering
  int nev = 0;
  float last_ms = 0.0f;
  double total_ms = 0.0;
  int last_year = 0;
  int params_set = 0, state_set = 0, ran = 0;
  h9g_error last_err{};
  const char *kname = "";
  unsigned *d_stamps = nullptr;   // H9G_STAMPS builds only
  std::vector<int64_t> h_gid;     // grid ids of the cells (h9g_set_cells), for NetCDF ingest
  std::vector<float *> h_pin;     // per-slot pinned staging of the NetCDF prefetch
  std::vector<std::thread> prefetch;
  std::vector<int> prefetch_rc;
  unsigned soil_layers = 0;       // layers built by h9g_soil_layer (bit i = layer i)
  float soil_ms = 0.0f;           // device time of the last h9g_soil_layer
  int soil_slow = 0;              // cells of the last layer summed in the reference's order
  int *d_slow = nullptr;
  float *d_sv = nullptr;          // pair kernel day-snapshot blocks
  int *d_perm = nullptr;          // cell order of the year kernel (h9g_sort_kernel)
  int *d_perm2 = nullptr;         // a launch's second group as listed (sorted into d_perm)
  float *d_forc_s = nullptr;      // the year's forcing in slot order (h9g_perm_forcing_kernel)
  float *d_ann_s = nullptr;       // the year kernel's annual sums in slot order
  unsigned *d_aqbits = nullptr;   // H9G_DUMP_AQ builds: day-level water-table record of the last year
  int64_t dec_stats[4] = {0, 0, 0, 0};   // last h9g_run_decade_ordered (h9g_decade_stats)
  std::vector<int> chain_id;      // h9g_set_chains: reference rank (block) of every cell; empty = one chain
  std::vector<int64_t> dec_launches;   // last h9g_run_decade_ordered: cells of each re-run launch
  int *d_hist = nullptr;          // per cell: substeps of the last year below the column (-1: none)
  int hist_nsub = 0;              // substeps of that year
  unsigned *d_pace = nullptr;     // Pacer mode 2 progress rows (h9g_pair.h)
  unsigned epoch = 0;
  int prio_mode = -1;             // H9G_PRIO: 0 none, 1 rotate, 2 pace; -1 auto (pace_mode)
  int ncu = 256;
  int sort = 1;                   // H9G_SORT=0: identity order
  size_t sv_bytes = 0;
  int kind = 1;        // 1: h9g_pair_kernel, 2: h9g_solo_kernel, 3: both, 4: h9g_pair2_kernel (L = 10),
                       // 5: h9g_pair11_kernel, 6: h9g_pair1_kernel (H9G_KERNEL=pair|solo|mixed|pair2|pair11|
                       // pair1; default by L and the shard size, l10_kind)
  size_t n_solo = 0;   // kind 3: cells [0, n_solo) run on the solo kernel, the rest on the pair kernel
  size_t ios = 0;      // slots of the slot-ordered buffers (d_perm, d_forc_s, d_ann_s): twice the cells
  size_t stamp_words = 0;
  int ev_kind[NEVT] = {};         // kernel kind and cell-years of each timed launch
  int64_t ev_cells[NEVT] = {};
  double kstat[8][3] = {};        // per kernel kind: launches, cell-years, ms (h9g_launch_stats)
  struct OrdBufs *ord = nullptr;  // h9g_run_ordered's decade buffers
  int64_t ord_stats[9] = {};      // last ordered call (h9g_ordered_stats)
  int ord_probe = 1;              // the checks' day-1 probe (H9G_NO_PROBE: off)
  std::vector<int64_t> ord_passes;
};

static void ord_free(h9g_ctx *ctx);

#define HIPCHK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "h9g: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), \
              __FILE__, __LINE__);                                             \
      return H9G_EHIP;                                                         \
    }                                                                          \
  } while (0)

static int days_in_year(int y) {   // INIT.f90:844-859
  if (y % 4 != 0) return 365;
  if (y % 100 != 0) return 366;
  if (y % 400 != 0) return 365;
  return 366;
}

// Kernel variant for a context: compile-time geometry when zi is one of
// the built-in layer sets and NISURF is 24 or 48, runtime geometry otherwise.
enum GeoKind { GEO_R = 0, GEO_C24 = 24, GEO_C48 = 48 };

static GeoKind geo_kind(const h9g_config &c) {
  const float *zd = c.nlayers == 8 ? ZiDefault<8>::zi : ZiDefault<10>::zi;
  for (int i = 0; i <= c.nlayers + 1; i++)
    if (c.zi[i] != zd[i]) return GEO_R;
  if (c.nisurf == 24) return GEO_C24;
  if (c.nisurf == 48) return GEO_C48;
  return GEO_R;
}

// Launch a templated kernel K<L, G> with the context's geometry variant.
#if defined(H9G_ONLY_C2)
// A/B measurement builds (tools/build_variant.py --c2): the driver's config-2
// instantiation only (L = 8, driver.txt layers, NISURF = 48), ~1 minute
// instead of ~4 to build; any other configuration is refused.
#define H9G_DISPATCH(ctx, KERNEL, GRID, BLOCK, STREAM, ...)                          \
  do {                                                                               \
    if ((ctx)->L != 8 || geo_kind((ctx)->cfg) != GEO_C48) {                          \
      fprintf(stderr, "h9g: H9G_ONLY_C2 build runs config 2 only\n");                \
      return H9G_EINVAL;                                                             \
    }                                                                                \
    KERNEL<8, GeoC<8, 48>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<8, 48>());  \
  } while (0)
#else
#define H9G_DISPATCH(ctx, KERNEL, GRID, BLOCK, STREAM, ...)                          \
  do {                                                                               \
    const GeoKind gk_ = geo_kind((ctx)->cfg);                                        \
    if ((ctx)->L == 8) {                                                             \
      if (gk_ == GEO_C48)                                                            \
        KERNEL<8, GeoC<8, 48>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<8, 48>()); \
      else if (gk_ == GEO_C24)                                                       \
        KERNEL<8, GeoC<8, 24>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<8, 24>()); \
      else                                                                           \
        KERNEL<8, GeoR<8>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__,                  \
                                                       make_geo_r<8>((ctx)->cfg.zi, (ctx)->cfg.nisurf)); \
    } else {                                                                         \
      if (gk_ == GEO_C48)                                                            \
        KERNEL<10, GeoC<10, 48>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<10, 48>()); \
      else if (gk_ == GEO_C24)                                                       \
        KERNEL<10, GeoC<10, 24>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<10, 24>()); \
      else                                                                           \
        KERNEL<10, GeoR<10>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__,                \
                                                         make_geo_r<10>((ctx)->cfg.zi, (ctx)->cfg.nisurf)); \
    }                                                                                \
  } while (0)
#endif

// Launch a kernel that exists at L = 10 only (h9g_pair2_kernel).
#if defined(H9G_ONLY_C2)
#define H9G_DISPATCH_L10(ctx, KERNEL, GRID, BLOCK, STREAM, ...) \
  do {                                                          \
    fprintf(stderr, "h9g: H9G_ONLY_C2 build runs config 2 only\n"); \
    return H9G_EINVAL;                                          \
  } while (0)
#else
#define H9G_DISPATCH_L10(ctx, KERNEL, GRID, BLOCK, STREAM, ...)                         \
  do {                                                                              \
    const GeoKind gk_ = geo_kind((ctx)->cfg);                                       \
    if (gk_ == GEO_C48)                                                             \
      KERNEL<10, GeoC<10, 48>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<10, 48>()); \
    else if (gk_ == GEO_C24)                                                        \
      KERNEL<10, GeoC<10, 24>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__, GeoC<10, 24>()); \
    else                                                                            \
      KERNEL<10, GeoR<10>><<<GRID, BLOCK, 0, STREAM>>>(__VA_ARGS__,                 \
                                                       make_geo_r<10>((ctx)->cfg.zi, (ctx)->cfg.nisurf)); \
  } while (0)
#endif

#if defined(H9G_ISA_ONLY)
// tools/isa_pair.sh: device code of the config-2 pair kernel alone (ISA study)
#if defined(H9G_ISA_L10)
template __global__ void h9g_pair_kernel<10, GeoC<10, 24>>(const KArgs, const GeoC<10, 24>);
template __global__ void h9g_pair2_kernel<10, GeoC<10, 24>>(const KArgs, const GeoC<10, 24>);
template __global__ void h9g_pair11_kernel<10, GeoC<10, 24>>(const KArgs, const GeoC<10, 24>);
#else
template __global__ void h9g_pair1_kernel<8, GeoC<8, 48>>(const KArgs, const GeoC<8, 48>);
template __global__ void h9g_pair_kernel<8, GeoC<8, 48>>(const KArgs, const GeoC<8, 48>);
#endif
#else
static unsigned nblocks(size_t n) { return (unsigned)((n + H9G_BLOCK - 1) / H9G_BLOCK); }

extern "C" {

int h9g_abi_version(void) { return H9G_ABI_VERSION; }

int h9g_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int h9g_state_size(int nlayers) { return 4 * nlayers + 9; }

void h9g_destroy(h9g_ctx *ctx) {
  if (!ctx) return;
  for (auto &t : ctx->prefetch)
    if (t.joinable()) t.join();
  (void)hipSetDevice(ctx->device);
  if (ctx->sc) hipStreamSynchronize(ctx->sc);
  if (ctx->sx) hipStreamSynchronize(ctx->sx);
  (void)hipFree(ctx->d_par);
  (void)hipFree(ctx->d_st);
  (void)hipFree(ctx->d_forc);
  (void)hipFree(ctx->d_ann);
  (void)hipFree(ctx->d_err);
  (void)hipFree(ctx->d_sv);
  (void)hipFree(ctx->d_errflag);
  (void)hipFree(ctx->d_diag);
  (void)hipFree(ctx->d_gid);
  (void)hipFree(ctx->d_lat);
  (void)hipFree(ctx->d_stamps);
  (void)hipFree(ctx->d_slow);
  (void)hipFree(ctx->d_perm);
  (void)hipFree(ctx->d_perm2);
  (void)hipFree(ctx->d_forc_s);
  (void)hipFree(ctx->d_ann_s);
  (void)hipFree(ctx->d_hist);
  (void)hipFree(ctx->d_aqbits);
  (void)hipFree(ctx->d_pace);
  ord_free(ctx);
  for (auto e : ctx->ev_copied) hipEventDestroy(e);
  for (auto e : ctx->ev_consumed) hipEventDestroy(e);
  for (int i = 0; i < NEVT; i++) {
    (void)hipEventDestroy(ctx->ev0[i]);
    (void)hipEventDestroy(ctx->ev1[i]);
  }
  if (ctx->ev_ext) (void)hipEventDestroy(ctx->ev_ext);
  if (ctx->ev_diag) (void)hipEventDestroy(ctx->ev_diag);
  for (auto p : ctx->h_pin) (void)hipHostFree(p);
  if (ctx->sc) hipStreamDestroy(ctx->sc);
  if (ctx->sx) hipStreamDestroy(ctx->sx);
  delete ctx;
}

// Kernel for L = 10 (1: pair, 2: solo, 3: both).  They are bit-identical
// and differ in how n columns quantise into rounds of resident waves: the
// solo kernel (1-wave blocks, 1 wave/SIMD) packs 64 columns per wave, the
// pair kernel (88-column blocks, 3 waves/SIMD since round 3, pair_resident)
// 22; kind 3 runs the whole solo rounds and the pair kernel on the rest.
// Round 3 measured every strong-scaling shard of the config-5 grid
// (tools/l10_shards.py, profiles/r03e_l10_shards.txt, ms per year, pair /
// solo / mixed): 270,000 cells 537.7 / 618.6 / 538.1; 135,000 274.5 / 373.2 /
// 274.4; 67,500 130.1 / 246.5 / 130.4; 33,750 107.9 / 134.1 / 108.1.  The
// pair kernel is within noise of the best everywhere, so it is the choice;
// round 2's rounds model picked solo at 33,750 cells (24% slower there).
// Solo and mixed stay selectable (H9G_KERNEL) and are tested.  *n_solo:
// the whole solo rounds (kind 3 only).
// Round 4 adds the pair kernel built for 2 waves per SIMD (kind 4, 256
// VGPRs: no spills, every reciprocal): where the shard's pair workgroups fit
// one round of 2 per CU it is the faster one (33,750 cells: 98.1 vs 100.9 ms
// per year), and wherever they do not it needs an extra round (270,000 cells:
// 601.5 vs 505.8 ms), profiles/r04*_l10_shards.txt.
static int l10_kind(size_t n, int ncu, size_t *n_solo) {
  const size_t solo_round = (size_t)4 * ncu * H9G_YBLOCK;
  *n_solo = (n / solo_round) * solo_round;
  const size_t blocks = (n + (size_t)H9G_PCPW * H9G_PWAVES - 1) / ((size_t)H9G_PCPW * H9G_PWAVES);
  return blocks <= (size_t)2 * ncu ? 4 : 1;
}

// Device bytes a context of this configuration allocates: h9g_create's
// arrays plus what the first h9g_run_year / h9g_soil_layer allocate lazily
// (the pair kernel's per-workgroup day-snapshot blocks, the pacing rows, the
// soil build's slow-cell flags).
// Device bytes of the ordered mode's buffers for decades of up to ny years
// (h9g_config_bytes counts them with ny = 10).
static size_t ord_bytes(size_t n, size_t L, size_t ny) {
  const size_t srows = 4 * L + 9, rows = 12 + L;
  return 2 * (sizeof(float) * (srows + L + ny * (rows + srows)) * n + sizeof(int) * (4 + 4 * ny + 1) * n +
              sizeof(int) * 5 * (n + 1)) +
         sizeof(float) * srows * n + sizeof(int) * (4 * n + n + 1) +
         // the day-1 probe (OrdBufs): old inputs, two runs' state, sums and STOP rows, list, flags
         sizeof(float) * (L + 2 * srows + 2 * rows) * n + sizeof(int) * (8 * n + 2 * (n + 1));
}

size_t h9g_config_bytes(const h9g_config *cfg) {
  if (!cfg || cfg->ncell <= 0 || cfg->nlayers < 1 || cfg->max_days < 1 || cfg->nslots < 1) return 0;
  const size_t n = (size_t)cfg->ncell, L = (size_t)cfg->nlayers;
  const size_t ios = 2 * round_up(n, H9G_PCPW) + 64;
  // the largest launch's day-snapshot blocks: the 11-column kernel's over
  // every cell, or the one-column kernel's over H9G_PAIR1_MAX listed cells
  const size_t blocks = std::max((ios + (size_t)H9G_PCPW11 * H9G_PWAVES - 1) / ((size_t)H9G_PCPW11 * H9G_PWAVES),
                                 (size_t)1024 / H9G_PWAVES);
  // + the slot-ordered copies of a forcing slot and of the annual sums
  // (h9g_run_year, allocated on first use), the ordered mode's decade
  // buffers (h9g_run_ordered, decades of up to 10 years)
  return sizeof(float) * ((4 * L + 1) + (4 * L + 9) + 7 * (size_t)cfg->max_days * (size_t)cfg->nslots + (12 + L) + 1) * n +
         sizeof(float) * (7 * (size_t)cfg->max_days + 12 + L) * ios + sizeof(int) * 2 * ios +
         sizeof(int) * 6 * n + sizeof(int64_t) * n + sizeof(double) * H9G_NDIAG + sizeof(int) +
         blocks * PairStore<8, H9G_PLANES>::GBLOCK + sizeof(unsigned) * 16 * (size_t)H9G_PACE_ROWS +
         ord_bytes(n, L, 10);
}

// Free HBM h9g_create leaves beyond h9g_config_bytes (HIP runtime, RCCL
// buffers, allocation granularity), so that a configuration that passes the
// check at create time does not fail later inside h9g_run_year.
#define H9G_HEADROOM ((size_t)256 << 20)

static thread_local char g_create_reason[256];

static int config_fail(char *reason, int len, const char *msg) {
  if (reason && len > 0) snprintf(reason, (size_t)len, "%s", msg);
  return H9G_EINVAL;
}

// Host-only validation of a configuration (no GPU needed): 0 or H9G_EINVAL
// with a readable reason.  The slot count is bounded by memory, which
// h9g_create checks against the device's free HBM.
int h9g_config_check(const h9g_config *cfg, char *reason, int reason_len) {
  if (reason && reason_len > 0) reason[0] = 0;
  if (!cfg) return config_fail(reason, reason_len, "cfg is NULL");
  if (cfg->ncell <= 0) return config_fail(reason, reason_len, "ncell must be > 0");
  if (!(cfg->nlayers == 8 || cfg->nlayers == 10))
    return config_fail(reason, reason_len, "nlayers must be 8 or 10");
  if (cfg->nisurf < 1) return config_fail(reason, reason_len, "nisurf must be >= 1");
  if (cfg->max_days < 366) return config_fail(reason, reason_len, "max_days must be >= 366");
  if (cfg->nslots < 1 || cfg->nslots > H9G_MAX_SLOTS)
    return config_fail(reason, reason_len, "nslots must be in [1, H9G_MAX_SLOTS]");
  if ((size_t)cfg->ncell * 7 * (size_t)cfg->max_days > (size_t)INT32_MAX * 4)
    return config_fail(reason, reason_len, "ncell * max_days too large for one slot");
  for (int i = 1; i <= cfg->nlayers + 1; i++)
    if (!(cfg->zi[i] > cfg->zi[i - 1])) return config_fail(reason, reason_len, "zi must increase strictly");
  return 0;
}

const char *h9g_create_error(void) { return g_create_reason; }

h9g_ctx *h9g_create(const h9g_config *cfg, int device) {
  g_create_reason[0] = 0;
  if (h9g_config_check(cfg, g_create_reason, sizeof g_create_reason)) return nullptr;
  if (hipSetDevice(device) != hipSuccess) {
    snprintf(g_create_reason, sizeof g_create_reason, "hipSetDevice(%d) failed: no gfx950 GPU visible?", device);
    return nullptr;
  }
  {
    size_t free_b = 0, total_b = 0;
    const size_t need = h9g_config_bytes(cfg);
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && need + H9G_HEADROOM > free_b) {
      snprintf(g_create_reason, sizeof g_create_reason,
               "needs %.2f GB of device memory + %.2f GB headroom, %.2f GB free (reduce nslots=%d)", need / 1e9,
               H9G_HEADROOM / 1e9, free_b / 1e9, cfg->nslots);
      return nullptr;
    }
  }
  h9g_ctx *ctx = new h9g_ctx();
  ctx->cfg = *cfg;
  ctx->device = device;
  ctx->L = cfg->nlayers;
  ctx->n = (size_t)cfg->ncell;
  const size_t n = ctx->n;
  const int L = ctx->L;
  ctx->ios = 2 * round_up(n, H9G_PCPW) + 64;
  bool ok = hipStreamCreateWithFlags(&ctx->sc, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&ctx->sx, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&ctx->d_par, sizeof(float) * (4 * L + 1) * n) == hipSuccess &&
            hipMalloc(&ctx->d_st, sizeof(float) * (4 * L + 9) * n) == hipSuccess &&
            hipMalloc(&ctx->d_forc, sizeof(float) * 7 * (size_t)cfg->max_days * n * cfg->nslots) == hipSuccess &&
            hipMalloc(&ctx->d_ann, sizeof(float) * (12 + L) * n) == hipSuccess &&
            hipMalloc(&ctx->d_err, sizeof(int) * 4 * n) == hipSuccess &&
            hipMalloc(&ctx->d_errflag, sizeof(int)) == hipSuccess &&
            hipMalloc(&ctx->d_diag, sizeof(double) * H9G_NDIAG) == hipSuccess &&
            hipMalloc(&ctx->d_gid, sizeof(int64_t) * n) == hipSuccess &&
            hipMalloc(&ctx->d_lat, sizeof(float) * n) == hipSuccess &&
            hipMalloc(&ctx->d_perm, sizeof(int) * ctx->ios) == hipSuccess &&
            hipMalloc(&ctx->d_perm2, sizeof(int) * ctx->ios) == hipSuccess &&
            hipMalloc(&ctx->d_hist, sizeof(int) * n) == hipSuccess;
  if (ok) {
    ok = hipMemset(ctx->d_err, 0, sizeof(int) * 4 * n) == hipSuccess &&
         hipMemset(ctx->d_errflag, 0, sizeof(int)) == hipSuccess &&
         hipMemset(ctx->d_diag, 0, sizeof(double) * H9G_NDIAG) == hipSuccess &&
         hipMemset(ctx->d_ann, 0xff, sizeof(float) * (12 + L) * n) == hipSuccess &&
         hipMemset(ctx->d_hist, 0xff, sizeof(int) * n) == hipSuccess;
  }
  ctx->slot_days.assign(cfg->nslots, 0);
  ctx->h_pin.assign(cfg->nslots, nullptr);
  ctx->prefetch.resize(cfg->nslots);
  ctx->prefetch_rc.assign(cfg->nslots, 0);
  ctx->ev_copied.resize(cfg->nslots);
  ctx->ev_consumed.resize(cfg->nslots);
  for (int s = 0; ok && s < cfg->nslots; s++)
    ok = hipEventCreateWithFlags(&ctx->ev_copied[s], hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&ctx->ev_consumed[s], hipEventDisableTiming) == hipSuccess;
  for (int i = 0; ok && i < NEVT; i++)
    ok = hipEventCreate(&ctx->ev0[i]) == hipSuccess && hipEventCreate(&ctx->ev1[i]) == hipSuccess;
  if (ok)
    ok = hipEventCreateWithFlags(&ctx->ev_ext, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&ctx->ev_diag, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    snprintf(g_create_reason, sizeof g_create_reason, "device allocation failed (ncell=%d, nslots=%d)",
             cfg->ncell, cfg->nslots);
    fprintf(stderr, "h9g_create: %s\n", g_create_reason);
    h9g_destroy(ctx);
    return nullptr;
  }
  static const char *names[7][2][3] = {
      {{"", "", ""}, {"", "", ""}},
      {{"h9g_pair_kernel<8,GeoR>", "h9g_pair_kernel<8,GeoC<8,24>>", "h9g_pair_kernel<8,GeoC<8,48>>"},
       {"h9g_pair_kernel<10,GeoR>", "h9g_pair_kernel<10,GeoC<10,24>>", "h9g_pair_kernel<10,GeoC<10,48>>"}},
      {{"h9g_solo_kernel<8,GeoR>", "h9g_solo_kernel<8,GeoC<8,24>>", "h9g_solo_kernel<8,GeoC<8,48>>"},
       {"h9g_solo_kernel<10,GeoR>", "h9g_solo_kernel<10,GeoC<10,24>>", "h9g_solo_kernel<10,GeoC<10,48>>"}},
      {{"h9g_solo_kernel<8,GeoR>+h9g_pair_kernel<8,GeoR>", "h9g_solo_kernel<8,GeoC<8,24>>+h9g_pair_kernel<8,GeoC<8,24>>",
        "h9g_solo_kernel<8,GeoC<8,48>>+h9g_pair_kernel<8,GeoC<8,48>>"},
       {"h9g_solo_kernel<10,GeoR>+h9g_pair_kernel<10,GeoR>",
        "h9g_solo_kernel<10,GeoC<10,24>>+h9g_pair_kernel<10,GeoC<10,24>>",
        "h9g_solo_kernel<10,GeoC<10,48>>+h9g_pair_kernel<10,GeoC<10,48>>"}},
      {{"", "", ""},
       {"h9g_pair2_kernel<10,GeoR>", "h9g_pair2_kernel<10,GeoC<10,24>>", "h9g_pair2_kernel<10,GeoC<10,48>>"}},
      {{"h9g_pair11_kernel<8,GeoR>", "h9g_pair11_kernel<8,GeoC<8,24>>", "h9g_pair11_kernel<8,GeoC<8,48>>"},
       {"h9g_pair11_kernel<10,GeoR>", "h9g_pair11_kernel<10,GeoC<10,24>>", "h9g_pair11_kernel<10,GeoC<10,48>>"}},
      {{"h9g_pair1_kernel<8,GeoR>", "h9g_pair1_kernel<8,GeoC<8,24>>", "h9g_pair1_kernel<8,GeoC<8,48>>"},
       {"h9g_pair1_kernel<10,GeoR>", "h9g_pair1_kernel<10,GeoC<10,24>>", "h9g_pair1_kernel<10,GeoC<10,48>>"}}};
  // default: the pair kernel at L = 8; at L = 10 the kernel that needs less
  // time for this many columns (l10_kind)
  if (const char *se = getenv("H9G_SORT")) ctx->sort = atoi(se) != 0;
  if (const char *se = getenv("H9G_PRIO")) ctx->prio_mode = atoi(se);
  if (getenv("H9G_NO_PROBE")) ctx->ord_probe = 0;
  const char *kenv = getenv("H9G_KERNEL");
  int ncu = 256;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1)
    ncu = 256;
  ctx->ncu = ncu;
  // The XCD-aware orders (xcd_vwg, h9g_sort_kernel, h9g_perm_forcing_kernel)
  // assume H9G_NXCD = 8 XCDs dealt round-robin, i.e. the MI355X in SPX mode
  // (256 CUs).  Results never depend on it (every mapping is a permutation);
  // only the per-XCD L2 locality does.  Say so once if the device differs
  // (a CPX partition has one XCD of 32 CUs).
  if (ncu != 32 * H9G_NXCD) {
    static bool said = false;
    if (!said) {
      fprintf(stderr, "h9g: device %d has %d CUs, not %d: XCD-aware cell orders assume %d XCDs (SPX); results are "
                      "unaffected, L2 locality may not hold\n", device, ncu, 32 * H9G_NXCD, H9G_NXCD);
      said = true;
    }
  }
  if (kenv && strcmp(kenv, "solo") == 0)
    ctx->kind = 2;
  else if (kenv && strcmp(kenv, "pair") == 0)
    ctx->kind = 1;
  else if (kenv && strcmp(kenv, "pair2") == 0 && L == 10)
    ctx->kind = 4;
  else if (kenv && strcmp(kenv, "pair11") == 0)
    ctx->kind = 5;
  else if (kenv && strcmp(kenv, "pair1") == 0)   // the one-column kernel for every launch (tests, probes)
    ctx->kind = 6;
  else if (kenv && strcmp(kenv, "mixed") == 0) {
    // forced split (tests): H9G_SPLIT cells on the solo kernel, else the model's
    ctx->kind = 3;
    size_t ns = 0;
    (void)l10_kind(n, ncu, &ns);
    if (const char *sp = getenv("H9G_SPLIT")) ns = (size_t)strtoull(sp, nullptr, 10);
    ctx->n_solo = std::min(ns, n);
  } else if (L == 8)
    ctx->kind = 1;
  else
    ctx->kind = l10_kind(n, ncu, &ctx->n_solo);
  const GeoKind gk = geo_kind(*cfg);
  ctx->kname = names[ctx->kind][L == 8 ? 0 : 1][gk == GEO_R ? 0 : (gk == GEO_C24 ? 1 : 2)];
  return ctx;
}

// (L, ncell) layer-fastest host arrays -> device rows
int h9g_set_params(h9g_ctx *ctx, const float *theta_s, const float *hksat, const float *bsw,
                   const float *psi_s, const float *fmax) {
  if (!ctx || !theta_s || !hksat || !bsw || !psi_s || !fmax) return H9G_EINVAL;
  const size_t n = ctx->n;
  const int L = ctx->L;
  std::vector<float> rows((4 * L + 1) * n);
  const float *src[4] = {theta_s, hksat, bsw, psi_s};
  for (int k = 0; k < 4; k++)
    for (size_t c = 0; c < n; c++)
      for (int i = 0; i < L; i++) rows[(size_t)(k * L + i) * n + c] = src[k][c * L + i];
  memcpy(&rows[(size_t)(4 * L) * n], fmax, sizeof(float) * n);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(ctx->d_par, rows.data(), sizeof(float) * rows.size(), hipMemcpyHostToDevice, ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  ctx->params_set = 1;
  return 0;
}

// device rows -> (L, ncell) layer-fastest host arrays (h9g_set_params layout)
int h9g_get_params(h9g_ctx *ctx, float *theta_s, float *hksat, float *bsw, float *psi_s, float *fmax) {
  if (!ctx || !theta_s || !hksat || !bsw || !psi_s || !fmax) return H9G_EINVAL;
  const size_t n = ctx->n;
  const int L = ctx->L;
  std::vector<float> rows((4 * L + 1) * n);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemcpy(rows.data(), ctx->d_par, sizeof(float) * rows.size(), hipMemcpyDeviceToHost));
  float *dst[4] = {theta_s, hksat, bsw, psi_s};
  for (int k = 0; k < 4; k++)
    for (size_t c = 0; c < n; c++)
      for (int i = 0; i < L; i++) dst[k][c * L + i] = rows[(size_t)(k * L + i) * n + c];
  memcpy(fmax, &rows[(size_t)(4 * L) * n], sizeof(float) * n);
  return 0;
}

int h9g_init_state(h9g_ctx *ctx) {
  if (!ctx) return H9G_EINVAL;
  if (!ctx->params_set) return H9G_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  const int n = (int)ctx->n;
  H9G_DISPATCH(ctx, h9g_init_kernel, nblocks(n), H9G_BLOCK, ctx->sc, n, ctx->d_par, ctx->d_st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemsetAsync(ctx->d_err, 0, sizeof(int) * 4 * ctx->n, ctx->sc));
  HIPCHK(hipMemsetAsync(ctx->d_errflag, 0, sizeof(int), ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemsetAsync(ctx->d_hist, 0xff, sizeof(int) * ctx->n, ctx->sc));   // a new state has no last year
  ctx->hist_nsub = 0;
  ctx->state_set = 1;
  ctx->last_err = h9g_error{};
  return 0;
}

// packed (field-major, width-fastest) <-> device rows
static void widths(int L, int *w) {
  const int ws[12] = {L, L, L, L + 1, 1, 1, 1, 1, 1, 1, 1, 1};
  for (int k = 0; k < 12; k++) w[k] = ws[k];
}

int h9g_set_state(h9g_ctx *ctx, const float *packed) {
  if (!ctx || !packed) return H9G_EINVAL;
  const size_t n = ctx->n;
  int w[12];
  widths(ctx->L, w);
  std::vector<float> rows((size_t)h9g_state_size(ctx->L) * n);
  size_t off = 0, row = 0;
  for (int k = 0; k < 12; k++) {
    for (size_t c = 0; c < n; c++)
      for (int i = 0; i < w[k]; i++) rows[(row + i) * n + c] = packed[off + c * w[k] + i];
    off += n * w[k];
    row += w[k];
  }
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpyAsync(ctx->d_st, rows.data(), sizeof(float) * rows.size(), hipMemcpyHostToDevice, ctx->sc));
  HIPCHK(hipMemsetAsync(ctx->d_err, 0, sizeof(int) * 4 * n, ctx->sc));
  HIPCHK(hipMemsetAsync(ctx->d_errflag, 0, sizeof(int), ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemsetAsync(ctx->d_hist, 0xff, sizeof(int) * ctx->n, ctx->sc));   // a new state has no last year
  ctx->hist_nsub = 0;
  ctx->state_set = 1;
  ctx->last_err = h9g_error{};
  return 0;
}

int h9g_get_state(h9g_ctx *ctx, float *packed) {
  if (!ctx || !packed) return H9G_EINVAL;
  const size_t n = ctx->n;
  int w[12];
  widths(ctx->L, w);
  std::vector<float> rows((size_t)h9g_state_size(ctx->L) * n);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemcpy(rows.data(), ctx->d_st, sizeof(float) * rows.size(), hipMemcpyDeviceToHost));
  size_t off = 0, row = 0;
  for (int k = 0; k < 12; k++) {
    for (size_t c = 0; c < n; c++)
      for (int i = 0; i < w[k]; i++) packed[off + c * w[k] + i] = rows[(row + i) * n + c];
    off += n * w[k];
    row += w[k];
  }
  return 0;
}

float *h9g_forcing_slot(h9g_ctx *ctx, int slot) {
  if (!ctx || slot < 0 || slot >= ctx->cfg.nslots) return nullptr;
  return ctx->d_forc + (size_t)slot * 7 * ctx->cfg.max_days * ctx->n;
}

void *h9g_host_alloc(size_t bytes) {
  void *p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void h9g_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

// (7, nday, ncell) -> slot (7, max_days, ncell)
static int push_impl(h9g_ctx *ctx, int slot, int nday, const float *src, hipMemcpyKind kind, bool async) {
  if (!ctx || !src || slot < 0 || slot >= ctx->cfg.nslots || nday < 1 || nday > ctx->cfg.max_days)
    return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  float *dst = h9g_forcing_slot(ctx, slot);
  const size_t n = ctx->n;
  HIPCHK(hipStreamWaitEvent(ctx->sx, ctx->ev_consumed[slot], 0));
  HIPCHK(hipMemcpy2DAsync(dst, sizeof(float) * ctx->cfg.max_days * n, src, sizeof(float) * nday * n,
                          sizeof(float) * nday * n, 7, kind, ctx->sx));
  HIPCHK(hipEventRecord(ctx->ev_copied[slot], ctx->sx));
  if (!async) HIPCHK(hipStreamSynchronize(ctx->sx));
  ctx->slot_days[slot] = nday;
  return 0;
}

int h9g_push_forcing(h9g_ctx *ctx, int slot, int nday, const float *forcing, int async) {
  return push_impl(ctx, slot, nday, forcing, hipMemcpyHostToDevice, async != 0);
}

int h9g_push_forcing_device(h9g_ctx *ctx, int slot, int nday, const float *dev_forcing) {
  return push_impl(ctx, slot, nday, dev_forcing, hipMemcpyDeviceToDevice, true);
}

// Join the NetCDF prefetch thread of a slot (its copy is queued when it ends).
static int join_prefetch(h9g_ctx *ctx, int slot) {
  if (ctx->prefetch[slot].joinable()) ctx->prefetch[slot].join();
  const int rc = ctx->prefetch_rc[slot];
  ctx->prefetch_rc[slot] = 0;
  return rc;
}

// Columns per wave of a pair-kernel kind: 22, 11 (kind 5, h9g_pair11_kernel)
// or 1 (kind 6, h9g_pair1_kernel); 4 waves per workgroup.
// Launch-statistics row of the cell order's day-1 probes (h9g_launch_stats)
#define H9G_KIND_PROBE 7
static int pair_wave_cols(int kind) { return kind == 5 ? H9G_PCPW11 : (kind == 6 ? 1 : H9G_PCPW); }
static size_t pair_block_cells(int kind) { return (size_t)pair_wave_cols(kind) * H9G_PWAVES; }
// Workgroups of a pair-kernel kind resident per CU (= waves per SIMD).
static int pair_kind_resident(int kind) { return kind == 4 ? 2 : (kind == 6 ? 1 : pair_resident<8>()); }
// Lists of at most this many cells (the cell-order re-runs' tails) run on
// h9g_pair1_kernel: every workgroup resident at one wave per SIMD.
#define H9G_PAIR1_MAX 1024
// Pacer mode of a pair launch of `blocks` workgroups (h9g_pair.h Pacer): pace
// when all of them are resident at once (one round), else rotate -- a wave of
// a later round starts hundreds of days behind the waves it shares a SIMD with.
static int pace_mode(const h9g_ctx *ctx, int kind, size_t blocks) {
  if (ctx->prio_mode >= 0) return ctx->prio_mode;
  return blocks <= (size_t)ctx->ncu * pair_kind_resident(kind) ? 2 : 1;
}

// Whether a year launch of `base` cells on the context's kernel can carry k
// more cells in a second group for free: a pair kernel kind, and the extra
// waves fit the launch's last round of resident workgroups.
static bool g2_fits(const h9g_ctx *ctx, size_t base, size_t k) {
  if (k == 0 || !ctx->sort || !(ctx->kind == 1 || ctx->kind == 4 || ctx->kind == 5)) return false;
#if defined(H9G_DUMP_AQ)
  return false;
#endif
  const size_t C = (size_t)pair_wave_cols(ctx->kind), per = pair_block_cells(ctx->kind);
  if (round_up(base, C) + k > ctx->ios) return false;
  const size_t slots = (size_t)ctx->ncu * pair_kind_resident(ctx->kind);
  const size_t b1 = (base + per - 1) / per, b2 = (round_up(base, C) + k + per - 1) / per;
  return (b2 + slots - 1) / slots == (b1 + slots - 1) / slots;
}

// Fold the finished launches' HIP-event timings into the totals and the
// per-kernel-kind counts (synchronises the compute stream).
static int fold_events(h9g_ctx *ctx) {
  HIPCHK(hipStreamSynchronize(ctx->sc));
  for (int i = 0; i < ctx->nev; i++) {
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0[i], ctx->ev1[i]));
    ctx->total_ms += ms;
    ctx->last_ms = ms;
    const int k = ctx->ev_kind[i];
    ctx->kstat[k][0] += 1.0;
    ctx->kstat[k][1] += (double)ctx->ev_cells[i];
    ctx->kstat[k][2] += ms;
  }
  ctx->nev = 0;
  return 0;
}

// One year launch (run_year_impl).
struct YearSpec {
  int slot = 0, jyear = 0;
  const int *d_list = nullptr;   // null: every cell, in h9g_sort_kernel's order; else the m cells d_list[0..m)
  int m = 0;
  float *ann_dst = nullptr;      // list launches: their annual means into these rows (stride n, cell order)
  float *st = nullptr;           // the cells' state and STOP rows (null: the context's own)
  int *err = nullptr;
  bool bulk = false;             // a list launch that is a year of the context's cells (h9g_run_ordered's
                                 // first pass without the cells still re-running the decade before): the
                                 // context's kernel, sort history and diagnostics, as an every-cell launch
  // launches of a pair kernel (g2_fits): a second group of the k2 cells
  // h2[0..k2) (host) at year jyear2 from slot2, with state st2/err2, annual
  // means into ann2 (h9g_run_ordered: a decade's re-runs riding in the next
  // decade's years)
  const int *h2 = nullptr;
  int k2 = 0, slot2 = 0, jyear2 = 0;
  float *st2 = nullptr, *ann2 = nullptr;
  int *err2 = nullptr;
  // list launches: only the year's first `ndays` days (0: all), the annual
  // rows as undivided running sums (the cell order's day-1 probe)
  int ndays = 0;
  bool probe = false;
};

// The kernel of a list launch of m cells (the cell order's re-runs): the
// one-column kernel up to H9G_PAIR1_MAX cells (lone waves, one per SIMD);
// at L = 8 the 11-column kernel up to H9G_PAIR11_LIST cells, where its
// waves still fit about one round; else the context's pair kernel (the
// pair kernel for the mixed kind), never solo rounds.  Round 6,
// tools/list_sweep.py (config 2 / config 3, ms per year): 1,000 cells pair
// 132.7 / 67.7, pair11 119.7 / 61.3, pair1 97.4 / 50.2; 10,000 cells pair
// 132.5 / 67.9, pair11 120.0 / 62.3; 20,000 cells 133.6 / 68.5 against
// 136.3 / 70.3.
#define H9G_PAIR11_LIST 16384
static int list_kind(const h9g_ctx *ctx, int m) {
  if (ctx->kind == 2) return 2;
  if (m <= H9G_PAIR1_MAX && !getenv("H9G_NO_PAIR1")) return 6;
  if (ctx->L == 8 && ctx->kind == 1 && m <= H9G_PAIR11_LIST && !getenv("H9G_NO_PAIR11")) return 5;
  return ctx->kind == 3 ? 1 : ctx->kind;
}

static int run_year_impl(h9g_ctx *ctx, const YearSpec &ys) {
  const int *d_list = ys.d_list;
  const int m = ys.m;
  if (!ctx || ys.slot < 0 || ys.slot >= ctx->cfg.nslots || ys.jyear < 1861 || ys.jyear > 2299) return H9G_EINVAL;
  if (d_list && (m < 1 || (size_t)m > ctx->n || !ys.ann_dst)) return H9G_EINVAL;
  if (ys.bulk && (!d_list || ys.st || ctx->kind == 2 || ctx->kind == 3)) return H9G_EINVAL;
  if (ys.probe && (!d_list || ys.bulk || !ys.st || ys.k2 > 0 || ys.ndays < 1)) return H9G_EINVAL;
  const bool two = ys.k2 > 0;
  if (two && ((d_list && !ys.bulk) || !ys.h2 || !ys.st2 || !ys.err2 || !ys.ann2 || ys.slot2 < 0 ||
              ys.slot2 >= ctx->cfg.nslots || ys.jyear2 < 1861 || ys.jyear2 > 2299 ||
              !g2_fits(ctx, d_list ? (size_t)m : ctx->n, (size_t)ys.k2)))
    return H9G_EINVAL;
  if (!ctx->params_set || !ctx->state_set) return H9G_ESTATE;
#if defined(H9G_DUMP_AQ)
  if (d_list || ys.st) return H9G_EINVAL;   // (the record is indexed by the annual array's cell)
#endif
  if (const int prc = join_prefetch(ctx, ys.slot)) return prc;
  if (two)
    if (const int prc = join_prefetch(ctx, ys.slot2)) return prc;
  const int nt = ys.probe ? std::min(ys.ndays, days_in_year(ys.jyear)) : days_in_year(ys.jyear);
  const int nt2 = two ? days_in_year(ys.jyear2) : nt;
  if (ctx->slot_days[ys.slot] < nt || (two && ctx->slot_days[ys.slot2] < nt2)) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamWaitEvent(ctx->sc, ctx->ev_copied[ys.slot], 0));
  if (two) HIPCHK(hipStreamWaitEvent(ctx->sc, ctx->ev_copied[ys.slot2], 0));
  const int n = (int)ctx->n;
  const size_t ios = ctx->ios;
  KArgs a;
  a.ncell = n;
  a.c0 = 0;
  a.cend = d_list ? m : n;
  a.nt = nt;
  a.nisurf = ctx->cfg.nisurf;
  a.grow_on = ctx->cfg.grow_on;
  a.fvar = (size_t)ctx->cfg.max_days * ctx->n;
  a.par = ctx->d_par;
  a.st = ys.st ? ys.st : ctx->d_st;
  a.forc = h9g_forcing_slot(ctx, ys.slot);
  a.annual = ctx->d_ann;
  a.err = ys.err ? ys.err : ctx->d_err;
  a.err_flag = ctx->d_errflag;
  a.stamps = nullptr;
  a.sv = nullptr;
  a.perm = nullptr;
  a.sorted_io = 0;
  a.hist = ys.st ? nullptr : ctx->d_hist;   // sort history: the context's own cells only
  a.bend = a.split = a.cend;
  a.nt2 = nt;
  a.st2 = a.st;
  a.err2 = a.err;
  a.iostride = ios;
  a.raw = ys.probe ? 1 : 0;
  const int kind = d_list && !ys.bulk ? list_kind(ctx, m) : ctx->kind;
  const size_t ncells = d_list ? (size_t)m : ctx->n;
  // slot-ordered forcing and annual sums (row stride ios: the cells plus a
  // second group's slack)
  if (d_list || ctx->sort) {
    if (!ctx->d_forc_s) HIPCHK(hipMalloc(&ctx->d_forc_s, sizeof(float) * 7 * (size_t)ctx->cfg.max_days * ios));
    if (!ctx->d_ann_s) HIPCHK(hipMalloc(&ctx->d_ann_s, sizeof(float) * (12 + ctx->L) * ios));
  }
  const size_t dvar = (size_t)ctx->cfg.max_days * ios;
  // the second group from the first whole wave after the first group's
  // cells: its slots of d_perm (in h9g_sort_kernel's order over its own
  // state), then its year's forcing into them
  auto second_group = [&](int base, int pcpb) -> int {
    const int split = (int)round_up((size_t)base, (size_t)pair_wave_cols(kind));
    HIPCHK(hipMemcpyAsync(ctx->d_perm2 + split, ys.h2, sizeof(int) * ys.k2, hipMemcpyHostToDevice, ctx->sc));
    H9G_DISPATCH(ctx, h9g_sort_kernel, H9G_NXCD, H9G_SORT_THREADS, ctx->sc, n, split, split + ys.k2, pcpb, ys.st2,
                 ys.err2, ctx->d_hist, ctx->hist_nsub, ctx->d_perm, ctx->d_perm2);
    h9g_perm_forcing_kernel<<<perm_forcing_blocks(split, split + ys.k2, pcpb, nt2), 256, 0, ctx->sc>>>(
        split, split + ys.k2, pcpb, nt2, n, a.fvar, ios, dvar, ctx->d_perm, h9g_forcing_slot(ctx, ys.slot2),
        ctx->d_forc_s);
    HIPCHK(hipGetLastError());
    a.split = split;
    a.cend = split + ys.k2;
    a.nt2 = nt2;
    a.st2 = ys.st2;
    a.err2 = ys.err2;
    return 0;
  };
  if (d_list) {
    const int pcpb = kind == 2 ? H9G_YBLOCK : (int)pair_block_cells(kind);
    a.perm = d_list;
    if (ctx->sort && kind != 6) {
      // the list in h9g_sort_kernel's order (its waves' columns take the
      // same branches), into d_perm, free between every-cell launches
      H9G_DISPATCH(ctx, h9g_sort_kernel, H9G_NXCD, H9G_SORT_THREADS, ctx->sc, n, 0, m, pcpb, a.st, a.err, ctx->d_hist,
                   ctx->hist_nsub, ctx->d_perm, d_list);
      a.perm = ctx->d_perm;
    }
    h9g_perm_forcing_kernel<<<perm_forcing_blocks(0, m, pcpb, nt), 256, 0, ctx->sc>>>(
        0, m, pcpb, nt, n, a.fvar, ios, dvar, a.perm, a.forc, ctx->d_forc_s);
    HIPCHK(hipGetLastError());
    if (two)
      if (int r = second_group(m, pcpb)) return r;
    a.forc = ctx->d_forc_s;
    a.annual = ctx->d_ann_s;
    a.sorted_io = 1;
  } else if (ctx->sort) {             // per launch range and its workgroup size (h9g_sort_kernel)
    const int ns = (int)ctx->n_solo, pcpb = (int)pair_block_cells(ctx->kind);
    if (ctx->kind == 2) {
      H9G_DISPATCH(ctx, h9g_sort_kernel, H9G_NXCD, H9G_SORT_THREADS, ctx->sc, n, 0, n, H9G_YBLOCK, ctx->d_st, ctx->d_err,
                   ctx->d_hist, ctx->hist_nsub, ctx->d_perm, nullptr);
    } else if (ctx->kind == 3) {
      if (ns > 0)
        H9G_DISPATCH(ctx, h9g_sort_kernel, H9G_NXCD, H9G_SORT_THREADS, ctx->sc, n, 0, ns, H9G_YBLOCK, ctx->d_st,
                     ctx->d_err, ctx->d_hist, ctx->hist_nsub, ctx->d_perm, nullptr);
      if (ns < n)
        H9G_DISPATCH(ctx, h9g_sort_kernel, H9G_NXCD, H9G_SORT_THREADS, ctx->sc, n, ns, n, pcpb, ctx->d_st, ctx->d_err,
                     ctx->d_hist, ctx->hist_nsub, ctx->d_perm, nullptr);
    } else {
      H9G_DISPATCH(ctx, h9g_sort_kernel, H9G_NXCD, H9G_SORT_THREADS, ctx->sc, n, 0, n, pcpb, ctx->d_st, ctx->d_err,
                   ctx->d_hist, ctx->hist_nsub, ctx->d_perm, nullptr);
    }
    HIPCHK(hipGetLastError());
    a.perm = ctx->d_perm;
#if !defined(H9G_DUMP_AQ)                 // (that record is indexed by the annual array's cell)
    // forcing and annual sums in slot order for the year kernel, per launch
    // range with its workgroup size, as the sort above
    auto perm_range = [&](int c0, int cend, int cpb, int ntr, const float *src) {
      h9g_perm_forcing_kernel<<<perm_forcing_blocks(c0, cend, cpb, ntr), 256, 0, ctx->sc>>>(
          c0, cend, cpb, ntr, n, a.fvar, ios, dvar, ctx->d_perm, src, ctx->d_forc_s);
    };
    if (ctx->kind == 2) {
      perm_range(0, n, H9G_YBLOCK, nt, a.forc);
    } else if (ctx->kind == 3) {
      if (ns > 0) perm_range(0, ns, H9G_YBLOCK, nt, a.forc);
      if (ns < n) perm_range(ns, n, pcpb, nt, a.forc);
    } else {
      perm_range(0, n, pcpb, nt, a.forc);
    }
    HIPCHK(hipGetLastError());
    if (two)
      if (int r = second_group(n, pcpb)) return r;
    a.forc = ctx->d_forc_s;
    a.annual = ctx->d_ann_s;
    a.sorted_io = 1;
#endif
  }
  if (a.sorted_io) a.fvar = dvar;
  // workgroups of the launch (the pair part's, for the mixed kind)
  const size_t per_block = kind == 2 ? (size_t)H9G_YBLOCK : pair_block_cells(kind == 3 ? 1 : kind);
  const size_t blocks = kind == 3 ? (ctx->n - ctx->n_solo + per_block - 1) / per_block
                                  : ((size_t)a.cend + per_block - 1) / per_block;
  if (kind != 2) {
    // the pair kernels' day-snapshot blocks, one per workgroup of the launch
    const size_t need = std::max<size_t>(blocks, 1) * PairStore<8, H9G_PLANES>::GBLOCK;
    if (ctx->sv_bytes < need) {
      (void)hipFree(ctx->d_sv);
      ctx->d_sv = nullptr;
      ctx->sv_bytes = 0;
      HIPCHK(hipMalloc(&ctx->d_sv, need));
      ctx->sv_bytes = need;
    }
    a.sv = ctx->d_sv;
    if (!ctx->d_pace) {
      const size_t pb = sizeof(unsigned) * 16 * H9G_PACE_ROWS;
      HIPCHK(hipMalloc(&ctx->d_pace, pb));
      HIPCHK(hipMemsetAsync(ctx->d_pace, 0, pb, ctx->sc));
    }
  }
  a.pace = ctx->d_pace;
  a.epoch = ++ctx->epoch;
  a.prio_mode = pace_mode(ctx, kind == 3 ? 1 : kind, blocks);
#if defined(H9G_STAMPS)
  {  // one record of 8 words per wave of the launch
    const size_t words = (size_t)8 * H9G_PWAVES * (blocks + 1);
    if (ctx->stamp_words < words) {
      (void)hipFree(ctx->d_stamps);
      ctx->d_stamps = nullptr;
      HIPCHK(hipMalloc(&ctx->d_stamps, sizeof(unsigned) * words));
      ctx->stamp_words = words;
    }
    HIPCHK(hipMemsetAsync(ctx->d_stamps, 0, sizeof(unsigned) * words, ctx->sc));
    a.stamps = ctx->d_stamps;
  }
#endif
  if (ctx->nev >= NEVT)   // fold finished timings before reusing events
    if (int r = fold_events(ctx)) return r;
#if defined(H9G_DUMP_AQ)
  // the last year's record to $H9G_AQ_DUMP: year, n, then n x 12 words
  if (const char *path = getenv("H9G_AQ_DUMP"); path && ctx->d_aqbits && ctx->ran) {
    std::vector<unsigned> bits(12 * ctx->n);
    HIPCHK(hipStreamSynchronize(ctx->sc));
    HIPCHK(hipMemcpy(bits.data(), ctx->d_aqbits, sizeof(unsigned) * bits.size(), hipMemcpyDeviceToHost));
    if (FILE *f = fopen(path, "ab")) {
      const int hdr[2] = {ctx->last_year, (int)ctx->n};
      fwrite(hdr, sizeof(int), 2, f);
      fwrite(bits.data(), sizeof(unsigned), bits.size(), f);
      fclose(f);
    }
  }
  if (!ctx->d_aqbits) HIPCHK(hipMalloc(&ctx->d_aqbits, sizeof(unsigned) * 12 * ctx->n));
  HIPCHK(hipMemsetAsync(ctx->d_aqbits, 0, sizeof(unsigned) * 12 * ctx->n, ctx->sc));
  {
    const float *base = ctx->d_ann;
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(h9g_aq_bits), &ctx->d_aqbits, sizeof(void *), 0,
                                  hipMemcpyHostToDevice, ctx->sc));
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(h9g_aq_base), &base, sizeof(void *), 0, hipMemcpyHostToDevice,
                                  ctx->sc));
  }
#endif
  const int e = ctx->nev++;
  ctx->ev_kind[e] = ys.probe ? H9G_KIND_PROBE : kind;
  ctx->ev_cells[e] = (int64_t)ncells + (two ? ys.k2 : 0);
  HIPCHK(hipEventRecord(ctx->ev0[e], ctx->sc));
  if (kind == 2) {
    H9G_DISPATCH(ctx, h9g_solo_kernel, (unsigned)((ncells + H9G_YBLOCK - 1) / H9G_YBLOCK), H9G_YBLOCK,
                 ctx->sc, a);
  } else if (kind == 3) {
    // mixed (l10_kind): whole rounds of solo waves, then the pair kernel on the rest
    const size_t ns = ctx->n_solo;
    if (ns > 0) {
      a.c0 = 0;
      a.cend = a.bend = a.split = (int)ns;
      H9G_DISPATCH(ctx, h9g_solo_kernel, (unsigned)((ns + H9G_YBLOCK - 1) / H9G_YBLOCK), H9G_YBLOCK,
                   ctx->sc, a);
    }
    if (ns < ctx->n) {
      a.c0 = (int)ns;
      a.cend = a.bend = a.split = (int)ctx->n;
      H9G_DISPATCH(ctx, h9g_pair_kernel, (unsigned)blocks, 64 * H9G_PWAVES, ctx->sc, a);
    }
  } else if (kind == 4) {
    H9G_DISPATCH_L10(ctx, h9g_pair2_kernel, (unsigned)blocks, 64 * H9G_PWAVES, ctx->sc, a);
  } else if (kind == 5) {
    H9G_DISPATCH(ctx, h9g_pair11_kernel, (unsigned)blocks, 64 * H9G_PWAVES, ctx->sc, a);
  } else if (kind == 6) {
    H9G_DISPATCH(ctx, h9g_pair1_kernel, (unsigned)blocks, 64 * H9G_PWAVES, ctx->sc, a);
  } else {
    H9G_DISPATCH(ctx, h9g_pair_kernel, (unsigned)blocks, 64 * H9G_PWAVES, ctx->sc, a);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev1[e], ctx->sc));
  HIPCHK(hipEventRecord(ctx->ev_consumed[ys.slot], ctx->sc));
  if (two) HIPCHK(hipEventRecord(ctx->ev_consumed[ys.slot2], ctx->sc));
  if (a.sorted_io) {
    const unsigned rows = (unsigned)(12 + ctx->L);
    h9g_unperm_annual_kernel<<<dim3((unsigned)((ncells + 255) / 256), rows), 256, 0, ctx->sc>>>(
        (int)ncells, n, (int)rows, 0, ios, a.perm, ctx->d_ann_s, d_list ? ys.ann_dst : ctx->d_ann);
    if (two)
      h9g_unperm_annual_kernel<<<dim3((unsigned)((ys.k2 + 255) / 256), rows), 256, 0, ctx->sc>>>(
          ys.k2, n, (int)rows, a.split, ios, a.perm, ctx->d_ann_s, ys.ann2);
    HIPCHK(hipGetLastError());
  }
  if (!d_list || ys.bulk) {
    h9g_diag_kernel<<<1, 1024, 0, ctx->sc>>>((int)ctx->n, ctx->L, ctx->d_ann, ctx->d_st, ctx->d_err, ctx->d_diag);
    HIPCHK(hipGetLastError());
  }
  if (!ys.st) {
    ctx->last_year = ys.jyear;
    ctx->hist_nsub = nt * ctx->cfg.nisurf;
  }
  ctx->ran = 1;
  return 0;
}

int h9g_run_year(h9g_ctx *ctx, int slot, int jyear) {
  YearSpec ys;
  ys.slot = slot;
  ys.jyear = jyear;
  return run_year_impl(ctx, ys);
}

// ---------------------------------------------------------------------------
// The reference's own cell order (h9g_run_ordered, h9g_run_decade_ordered)
// ---------------------------------------------------------------------------
// One decade of the reference's loop (HYBRID9.f90:93-130) is a fixed point
// on the device.  Pass 0 runs every cell's years from its own smp.
// h9g_chain_kernel then gives every land cell the smp its predecessor now
// ends the decade with and flags the cells whose input changed; those
// re-run from the decade's starting state (h9g_restart_kernel), and the pass
// repeats until no input changes.  A cell's result depends on its
// predecessor's only through that smp, so when no input changes every cell
// has run from the input the reference gives it.  Position p of a chain is
// exact after pass p + 1 at the latest: at most m + 1 passes.
//
// A re-run stops early.  The input smp reaches a cell's decade only through
// beta of its first substep (HYDROLOGY.f90:270-275), and the perturbation
// it starts is rounded away within months in most cells: from then on the
// cell runs bit for bit as before.  Every run therefore checkpoints each
// cell's state and STOP record at every year end (ck), and after each
// re-run year h9g_merge_kernel drops the cells whose state is the
// checkpoint's again: they keep the old trajectory's later years and end
// state (and so the input their successor already has).  Pass 1 then costs
// about one year for most cells instead of ten.
//
// Decades overlap (round 6).  Decade D+1's first pass needs only every
// cell's own end state of D, which the first pass of D gives for every cell
// the re-runs leave alone; so it starts as soon as D's first pass and the
// re-run of year 1 (every cell whose input changed) are done.  D's
// remaining re-runs -- a tail of a few dozen cells whose perturbation
// lasts, run year by year -- ride as a second group of waves in D+1's year
// launches (KArgs::split, on their own state rows st2), in the slots the
// grid leaves free in the launch's last round of resident workgroups.  Once
// D has settled, the cells whose end of D differs from where D+1's first
// pass started them get their final state (h9g_settle_kernel) and are
// re-run in D+1's first check whatever their input.  Each decade's first
// pass, checkpoints and re-runs read only its own buffers (OrdDec), so D's
// tail and D+1's first pass are independent.
struct OrdDec {
  int y0 = 0, ny = 0, k0 = 0;            // first year, years, index of its first year in the call
  float *st0 = nullptr, *guess = nullptr, *ann = nullptr, *ck = nullptr;
  int *err0 = nullptr, *eck = nullptr, *dirty = nullptr;
  int *d_chain = nullptr, *d_pred = nullptr, *d_first = nullptr, *d_list = nullptr, *d_flag = nullptr;
  std::vector<int> chain, list, flag;
  int m = 0;
  enum { PASS0, CHECK, RERUN, SETTLED } phase = PASS0;
  int next_y = 0, np = 0;
};

struct OrdBufs {
  OrdDec d[2];
  float *st2 = nullptr;                  // the re-running cells' state and STOP rows
  int *err2 = nullptr;
  int *d_bulk = nullptr;                 // a first pass's cells when some are left out of it
  // the day-1 probe (h9g_probe_cmp_kernel): the inputs the checked cells'
  // trajectories started from, the probe list and its two runs
  float *gold = nullptr, *pst = nullptr, *pann = nullptr;
  int *perr = nullptr, *d_plist = nullptr, *d_pkeep = nullptr;
  int ny_cap = 0;
};

static void ord_free(h9g_ctx *ctx) {
  OrdBufs *o = ctx->ord;
  if (!o) return;
  for (OrdDec &D : o->d) {
    for (float *p : {D.st0, D.guess, D.ann, D.ck}) (void)hipFree(p);
    for (int *p : {D.err0, D.eck, D.dirty, D.d_chain, D.d_pred, D.d_first, D.d_list, D.d_flag}) (void)hipFree(p);
  }
  (void)hipFree(o->st2);
  (void)hipFree(o->err2);
  (void)hipFree(o->d_bulk);
  for (float *p : {o->gold, o->pst, o->pann}) (void)hipFree(p);
  for (int *p : {o->perr, o->d_plist, o->d_pkeep}) (void)hipFree(p);
  delete o;
  ctx->ord = nullptr;
}

static int ord_alloc(h9g_ctx *ctx, int ny) {
  if (ctx->ord && ctx->ord->ny_cap >= ny) return 0;
  ord_free(ctx);
  ctx->ord = new OrdBufs();
  OrdBufs *o = ctx->ord;
  const size_t n = ctx->n, L = (size_t)ctx->L, srows = (size_t)h9g_state_size(ctx->L), rows = 12 + L;
  bool ok = hipMalloc(&o->st2, sizeof(float) * srows * n) == hipSuccess &&
            hipMalloc(&o->err2, sizeof(int) * 4 * n) == hipSuccess &&
            hipMalloc(&o->d_bulk, sizeof(int) * (n + 1)) == hipSuccess &&
            hipMalloc(&o->gold, sizeof(float) * L * n) == hipSuccess &&
            hipMalloc(&o->pst, sizeof(float) * 2 * srows * n) == hipSuccess &&
            hipMalloc(&o->pann, sizeof(float) * 2 * rows * n) == hipSuccess &&
            hipMalloc(&o->perr, sizeof(int) * 2 * 4 * n) == hipSuccess &&
            hipMalloc(&o->d_plist, sizeof(int) * (n + 1)) == hipSuccess &&
            hipMalloc(&o->d_pkeep, sizeof(int) * (n + 1)) == hipSuccess;
  for (OrdDec &D : o->d) {
    ok = ok && hipMalloc(&D.st0, sizeof(float) * srows * n) == hipSuccess &&
         hipMalloc(&D.guess, sizeof(float) * L * n) == hipSuccess &&
         hipMalloc(&D.ann, sizeof(float) * (size_t)ny * rows * n) == hipSuccess &&
         hipMalloc(&D.ck, sizeof(float) * (size_t)ny * srows * n) == hipSuccess &&
         hipMalloc(&D.err0, sizeof(int) * 4 * n) == hipSuccess &&
         hipMalloc(&D.eck, sizeof(int) * (size_t)ny * 4 * n) == hipSuccess &&
         hipMalloc(&D.dirty, sizeof(int) * n) == hipSuccess;
    for (int **p : {&D.d_chain, &D.d_pred, &D.d_first, &D.d_list, &D.d_flag})
      ok = ok && hipMalloc(p, sizeof(int) * (n + 1)) == hipSuccess;
  }
  if (!ok) {
    ord_free(ctx);
    return H9G_ENOMEM;
  }
  o->ny_cap = ny;
  return 0;
}

// Work counters of the last ordered call (h9g_decade_stats, h9g_ordered_stats).
struct OrdStats {
  int64_t passes = 0, rerun_cells = 0, rerun_cell_years = 0, rerun_launches = 0;
  int64_t ticks = 0, ride_steps = 0, ride_cell_years = 0, alone_steps = 0, alone_cell_years = 0, excluded = 0;
  int64_t probed = 0, probe_kept = 0;
  std::vector<int64_t> launch_cells, dec_passes;
};

static float *ord_ck(const h9g_ctx *ctx, const OrdDec &D, int y) {
  return D.ck + (size_t)y * h9g_state_size(ctx->L) * ctx->n;
}
static int *ord_eck(const h9g_ctx *ctx, const OrdDec &D, int y) { return D.eck + (size_t)y * 4 * ctx->n; }
static float *ord_ann(const h9g_ctx *ctx, const OrdDec &D, int y) { return D.ann + (size_t)y * (12 + ctx->L) * ctx->n; }

// The decade's chains (h9g_set_chains) over its land cells that have not
// stopped when it starts (its final err0), in context order: predecessors
// are the previous land cell of the same chain, for a chain's first cell its
// last one.
static int ord_chain(h9g_ctx *ctx, OrdDec &D, const std::vector<char> &land) {
  const size_t n = ctx->n;
  std::vector<int> e0(n);
  HIPCHK(hipStreamSynchronize(ctx->sc));   // (the compute stream is non-blocking: hipMemcpy does not wait for it)
  HIPCHK(hipMemcpy(e0.data(), D.err0, sizeof(int) * n, hipMemcpyDeviceToHost));
  D.chain.clear();
  for (size_t c = 0; c < n; c++)
    if (land[c] && e0[c] == 0) D.chain.push_back((int)c);
  const int m = D.m = (int)D.chain.size();
  std::vector<int> pred(m), first(m), last_of, first_of;
  auto cid = [&](int j) { return ctx->chain_id.empty() ? 0 : ctx->chain_id[(size_t)D.chain[j]]; };
  for (int j = 0; j < m; j++) {
    const int c = cid(j);
    if ((int)last_of.size() <= c) {
      last_of.resize((size_t)c + 1, -1);
      first_of.resize((size_t)c + 1, -1);
    }
    if (last_of[(size_t)c] < 0) {
      first_of[(size_t)c] = j;
      first[j] = 1;
    } else {
      pred[j] = D.chain[last_of[(size_t)c]];
      first[j] = 0;
    }
    last_of[(size_t)c] = j;
  }
  for (int j = 0; j < m; j++)
    if (first[j]) pred[j] = D.chain[last_of[(size_t)cid(j)]];
  if (m > 0) {
    HIPCHK(hipMemcpy(D.d_chain, D.chain.data(), sizeof(int) * m, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D.d_pred, pred.data(), sizeof(int) * m, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(D.d_first, first.data(), sizeof(int) * m, hipMemcpyHostToDevice));
  }
  D.flag.assign((size_t)m + 1, 0);
  return 0;
}

// A check of decade D: every chain cell's input from its predecessor's end
// of the decade as known now (the last year's checkpoint); the flagged cells
// back to the decade's start on the re-run rows st2 (phase RERUN), or, with
// none flagged, D has settled.
// The day-1 probe of the cells in `cand` (their input changed, their start
// did not): each runs its decade's first day from the smp its trajectory
// started from (o->gold) and from its new one (D.guess); the cells whose two
// days differ are appended to D.list (h9g_probe_cmp_kernel).
static int ord_probe(h9g_ctx *ctx, OrdDec &D, const int32_t *slots, const std::vector<int> &cand, OrdStats &S) {
  OrdBufs *o = ctx->ord;
  const int n = (int)ctx->n, L = ctx->L, k = (int)cand.size();
  const int rows = 12 + L, srows = h9g_state_size(L);
  HIPCHK(hipMemcpyAsync(o->d_plist, cand.data(), sizeof(int) * k, hipMemcpyHostToDevice, ctx->sc));
  for (int v = 0; v < 2; v++) {
    float *st = o->pst + (size_t)v * srows * n;
    int *err = o->perr + (size_t)v * 4 * n;
    h9g_restart_kernel<<<(unsigned)((k + 255) / 256), 256, 0, ctx->sc>>>(k, n, L, o->d_plist, D.st0, D.err0,
                                                                        v ? D.guess : o->gold, st, err);
    HIPCHK(hipGetLastError());
    YearSpec ys;
    ys.slot = slots[D.k0];
    ys.jyear = D.y0;
    ys.d_list = o->d_plist;
    ys.m = k;
    ys.ann_dst = o->pann + (size_t)v * rows * n;
    ys.st = st;
    ys.err = err;
    ys.ndays = 1;
    ys.probe = true;
    if (int r = run_year_impl(ctx, ys)) return r;
  }
  h9g_probe_cmp_kernel<<<(unsigned)((k + 255) / 256), 256, 0, ctx->sc>>>(
      k, n, srows, rows, o->d_plist, o->pst, o->pst + (size_t)srows * n, o->perr, o->perr + (size_t)4 * n, o->pann,
      o->pann + (size_t)rows * n, o->d_pkeep);
  HIPCHK(hipGetLastError());
  std::vector<int> keep(k);
  HIPCHK(hipMemcpyAsync(keep.data(), o->d_pkeep, sizeof(int) * k, hipMemcpyDeviceToHost, ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  int kept = 0;
  for (int j = 0; j < k; j++)
    if (keep[j]) {
      D.list.push_back(cand[j]);
      kept++;
    }
  S.probed += k;
  S.probe_kept += kept;
  return 0;
}

static int ord_check(h9g_ctx *ctx, OrdDec &D, const int32_t *slots, bool use_dirty, OrdStats &S) {
  OrdBufs *o = ctx->ord;
  const int n = (int)ctx->n, L = ctx->L, m = D.m;
  D.list.clear();
  if (m > 0) {
    // the inputs the trajectories started from, for the probe
    HIPCHK(hipMemcpyAsync(o->gold, D.guess, sizeof(float) * L * n, hipMemcpyDeviceToDevice, ctx->sc));
    h9g_chain_kernel<<<(unsigned)((m + 255) / 256), 256, 0, ctx->sc>>>(m, n, L, D.d_chain, D.d_pred, D.d_first,
                                                                      ord_ck(ctx, D, D.ny - 1), D.st0, D.guess,
                                                                      use_dirty ? D.dirty : nullptr, D.d_flag);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(D.flag.data(), D.d_flag, sizeof(int) * m, hipMemcpyDeviceToHost, ctx->sc));
    HIPCHK(hipStreamSynchronize(ctx->sc));
    std::vector<int> cand;
    const bool probe = ctx->ord_probe;
    for (int j = 0; j < m; j++) {
      if (probe && D.flag[j] == 1)
        cand.push_back(D.chain[j]);
      else if (D.flag[j])
        D.list.push_back(D.chain[j]);
    }
    if (!cand.empty()) {
      if (int r = ord_probe(ctx, D, slots, cand, S)) return r;
      std::sort(D.list.begin(), D.list.end());
    }
  }
  if (D.list.empty()) {
    D.phase = OrdDec::SETTLED;
    return 0;
  }
  if (D.np > m + 1) return H9G_ESTATE;   // cannot happen (see above): a broken invariant, not a result
  const int k = (int)D.list.size();
  HIPCHK(hipMemcpy(D.d_list, D.list.data(), sizeof(int) * k, hipMemcpyHostToDevice));
  h9g_restart_kernel<<<(unsigned)((k + 255) / 256), 256, 0, ctx->sc>>>(k, n, L, D.d_list, D.st0, D.err0, D.guess,
                                                                      o->st2, o->err2);
  HIPCHK(hipGetLastError());
  S.rerun_cells += k;
  D.next_y = 0;
  D.phase = OrdDec::RERUN;
  return 0;
}

// After a re-run year of decade D's list: the cells back on their old
// trajectory leave the re-run (h9g_merge_kernel); at the decade's end, or
// with none left, the pass ends and a check follows.
static int ord_after_run(h9g_ctx *ctx, OrdDec &D, OrdStats &S) {
  OrdBufs *o = ctx->ord;
  const int n = (int)ctx->n, srows = h9g_state_size(ctx->L);
  const int k = (int)D.list.size(), y = D.next_y;
  h9g_merge_kernel<<<(unsigned)((k + 255) / 256), 256, 0, ctx->sc>>>(k, n, srows, D.d_list, o->st2, o->err2,
                                                                    ord_ck(ctx, D, y), ord_eck(ctx, D, y),
                                                                    ord_ck(ctx, D, D.ny - 1), ord_eck(ctx, D, D.ny - 1),
                                                                    D.d_flag);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(D.flag.data(), D.d_flag, sizeof(int) * k, hipMemcpyDeviceToHost, ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  S.rerun_cell_years += k;
  S.rerun_launches++;
  S.launch_cells.push_back(k);
  int kk = 0;
  for (int j = 0; j < k; j++)
    if (D.flag[j]) D.list[kk++] = D.list[j];
  D.list.resize(kk);
  if (kk > 0 && kk < k) HIPCHK(hipMemcpy(D.d_list, D.list.data(), sizeof(int) * kk, hipMemcpyHostToDevice));
  D.next_y = y + 1;
  if (kk == 0 || D.next_y == D.ny) {
    D.np++;
    D.phase = OrdDec::CHECK;
  }
  return 0;
}

// One re-run year of decade D's list as a launch of its own.
static int ord_run_alone(h9g_ctx *ctx, OrdDec &D, const int32_t *slots, OrdStats &S) {
  YearSpec ys;
  ys.slot = slots[D.k0 + D.next_y];
  ys.jyear = D.y0 + D.next_y;
  ys.d_list = D.d_list;
  ys.m = (int)D.list.size();
  ys.ann_dst = ord_ann(ctx, D, D.next_y);
  ys.st = ctx->ord->st2;
  ys.err = ctx->ord->err2;
  if (int r = run_year_impl(ctx, ys)) return r;
  S.alone_steps++;
  S.alone_cell_years += ys.m;
  return ord_after_run(ctx, D, S);
}

// Runs D's checks and re-runs until it has settled.
static int ord_settle(h9g_ctx *ctx, OrdDec &D, const int32_t *slots, OrdStats &S) {
  while (D.phase != OrdDec::SETTLED) {
    const int r = D.phase == OrdDec::CHECK ? ord_check(ctx, D, slots, false, S) : ord_run_alone(ctx, D, slots, S);
    if (r) return r;
  }
  return 0;
}

// D has settled: its annual means to the host, its first new STOP into the
// context's error record, and -- with a next decade N under way -- its end
// states into N's start (h9g_settle_kernel).
static int ord_finish(h9g_ctx *ctx, OrdDec &D, OrdDec *N, float *annual, int &stop_seen) {
  const size_t n = ctx->n;
  const int rows = 12 + ctx->L, srows = h9g_state_size(ctx->L);
  if (annual)
    HIPCHK(hipMemcpyAsync(annual + (size_t)D.k0 * rows * n, D.ann, sizeof(float) * (size_t)D.ny * rows * n,
                          hipMemcpyDeviceToHost, ctx->sc));
  if (!stop_seen && ctx->last_err.code == 0) {
    std::vector<int> e0(n), e1(4 * n);
    HIPCHK(hipMemcpyAsync(e0.data(), D.err0, sizeof(int) * n, hipMemcpyDeviceToHost, ctx->sc));
    HIPCHK(hipMemcpyAsync(e1.data(), ord_eck(ctx, D, D.ny - 1), sizeof(int) * 4 * n, hipMemcpyDeviceToHost, ctx->sc));
    HIPCHK(hipStreamSynchronize(ctx->sc));
    for (size_t c = 0; c < n; c++) {
      if (e1[c] == 0 || e0[c] != 0) continue;
      // the first cell in context order to STOP in this decade, in the first
      // year of the decade whose means it has not completed
      std::vector<float> npp(D.ny);
      for (int y = 0; y < D.ny; y++)
        HIPCHK(hipMemcpy(&npp[y], ord_ann(ctx, D, y) + c, sizeof(float), hipMemcpyDeviceToHost));
      int y = 0;
      while (y < D.ny - 1 && npp[y] == npp[y]) y++;
      ctx->last_err.code = e1[c];
      ctx->last_err.cell = (int)c;
      ctx->last_err.year = D.y0 + y;
      ctx->last_err.day = e1[n + c];
      ctx->last_err.substep = e1[2 * n + c];
      ctx->last_err.value = __builtin_bit_cast(float, e1[3 * n + c]);
      stop_seen = 1;
      break;
    }
  }
  if (N) {
    h9g_settle_kernel<<<(unsigned)((n + 255) / 256), 256, 0, ctx->sc>>>(
        (int)n, srows, rows, N->ny, ord_ck(ctx, D, D.ny - 1), ord_eck(ctx, D, D.ny - 1), N->st0, N->err0, N->dirty,
        ctx->d_st, ctx->d_err, ord_ck(ctx, *N, N->ny - 1), ord_eck(ctx, *N, N->ny - 1), N->ann);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(ctx->sc));
  return 0;
}

// Cells left out of a decade's first pass (still re-running the decade
// before): re-run in its first check whatever their input (dirty), and never
// merged back onto a first-pass trajectory they did not run (their
// checkpoints' STOP code -1, which no run produces).
__global__ void __launch_bounds__(256) h9g_exclude_kernel(int k, int n, int ny, const int *__restrict__ list,
                                                          int *__restrict__ dirty, int *__restrict__ eck) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  const int c = list[j];
  dirty[c] = 1;
  for (int y = 0; y < ny; y++) eck[(size_t)y * 4 * n + c] = -1;
}

// decades: (first year, years) of each decade the call runs, in order;
// their years' forcing in slots[0 .. sum of years).
static int run_ordered_impl(h9g_ctx *ctx, const int32_t *slots, int jyear0,
                            const std::vector<std::pair<int, int>> &decs, float *annual, int32_t *passes) {
  if (!ctx || !slots || decs.empty()) return H9G_EINVAL;
  int nyears = 0, nymax = 0;
  for (auto &d : decs) {
    nyears += d.second;
    nymax = std::max(nymax, d.second);
  }
  if (nyears < 1 || nymax > ctx->cfg.nslots) return H9G_EINVAL;
  for (int y = 0; y < nyears; y++)
    if (slots[y] < 0 || slots[y] >= ctx->cfg.nslots || jyear0 + y < 1861 || jyear0 + y > 2299) return H9G_EINVAL;
  {
    // every year its own slot: a decade's re-runs read their years' forcing
    // while the next decade's first pass reads its own
    std::vector<char> used((size_t)ctx->cfg.nslots, 0);
    for (int y = 0; y < nyears; y++)
      if (used[(size_t)slots[y]]++) return H9G_EINVAL;
  }
  if (!ctx->params_set || !ctx->state_set) return H9G_ESTATE;
  const size_t n = ctx->n;
  const int L = ctx->L, rows = 12 + L, srows = h9g_state_size(L);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  if (int r = ord_alloc(ctx, nymax)) return r;
  OrdBufs *o = ctx->ord;
  // land cells (HYBRID9.f90:122-123, summed in layer order as the year
  // kernels do)
  std::vector<char> land(n);
  {
    std::vector<float> ts((size_t)L * n);
    HIPCHK(hipMemcpy(ts.data(), ctx->d_par, sizeof(float) * ts.size(), hipMemcpyDeviceToHost));
    for (size_t c = 0; c < n; c++) {
      float sum = 0.0f;
      for (int i = 0; i < L; i++) sum = sum + ts[(size_t)i * n + c];
      land[c] = sum > 1.0E-8f;
    }
  }
  OrdStats S;
  int stop_seen = 0;
  OrdDec *P = nullptr;                     // the decade whose re-runs are still going
  int k0 = 0;
  for (size_t i = 0; i < decs.size(); i++) {
    OrdDec &D = o->d[i & 1];
    D.y0 = decs[i].first;
    D.ny = decs[i].second;
    D.k0 = k0;
    k0 += D.ny;
    D.phase = OrdDec::PASS0;
    D.np = 0;
    D.next_y = 0;
    D.list.clear();
    // the decade starts from the context's state as known now
    HIPCHK(hipMemcpyAsync(D.st0, ctx->d_st, sizeof(float) * srows * n, hipMemcpyDeviceToDevice, ctx->sc));
    HIPCHK(hipMemcpyAsync(D.err0, ctx->d_err, sizeof(int) * 4 * n, hipMemcpyDeviceToDevice, ctx->sc));
    HIPCHK(hipMemcpyAsync(D.guess, ctx->d_st + (size_t)2 * L * n, sizeof(float) * (size_t)L * n,
                          hipMemcpyDeviceToDevice, ctx->sc));
    HIPCHK(hipMemsetAsync(D.dirty, 0, sizeof(int) * n, ctx->sc));
    // the cells P is still re-running stay out of D's first pass: their end
    // of P, D's start, is not known yet (they re-run D in its first check);
    // the others form the first pass's list, and P's re-runs ride in its
    // launches in the slots this leaves
    std::vector<int> excl;
    if (P && P->phase == OrdDec::RERUN && !getenv("H9G_NO_EXCLUDE")) {
      excl = P->list;
      std::sort(excl.begin(), excl.end());
    }
    int nb = (int)n;
    if (!excl.empty()) {
      std::vector<int> bulk;
      bulk.reserve(n - excl.size());
      size_t e = 0;
      for (int c = 0; c < (int)n; c++) {
        if (e < excl.size() && excl[e] == c) {
          e++;
          continue;
        }
        bulk.push_back(c);
      }
      nb = (int)bulk.size();
      HIPCHK(hipMemcpy(o->d_bulk, bulk.data(), sizeof(int) * nb, hipMemcpyHostToDevice));
    }
    S.excluded += (int64_t)excl.size();
    // pass 0: each year one launch, P's re-runs riding along
    for (int y = 0; y < D.ny; y++) {
      YearSpec ys;
      ys.slot = slots[D.k0 + y];
      ys.jyear = D.y0 + y;
      if (!excl.empty()) {
        ys.d_list = o->d_bulk;
        ys.m = nb;
        ys.bulk = true;
        ys.ann_dst = ctx->d_ann;
      }
      const bool ride = P && P->phase == OrdDec::RERUN && g2_fits(ctx, (size_t)nb, P->list.size()) &&
                        !getenv("H9G_NO_RIDE");
      if (ride) {
        ys.h2 = P->list.data();
        ys.k2 = (int)P->list.size();
        ys.slot2 = slots[P->k0 + P->next_y];
        ys.jyear2 = P->y0 + P->next_y;
        ys.st2 = o->st2;
        ys.err2 = o->err2;
        ys.ann2 = ord_ann(ctx, *P, P->next_y);
      }
      if (int r = run_year_impl(ctx, ys)) return r;
      S.ticks++;
      HIPCHK(hipMemcpyAsync(ord_ann(ctx, D, y), ctx->d_ann, sizeof(float) * rows * n, hipMemcpyDeviceToDevice, ctx->sc));
      HIPCHK(hipMemcpyAsync(ord_ck(ctx, D, y), ctx->d_st, sizeof(float) * srows * n, hipMemcpyDeviceToDevice, ctx->sc));
      HIPCHK(hipMemcpyAsync(ord_eck(ctx, D, y), ctx->d_err, sizeof(int) * 4 * n, hipMemcpyDeviceToDevice, ctx->sc));
      if (ride) {
        S.ride_steps++;
        S.ride_cell_years += ys.k2;
        if (int r = ord_after_run(ctx, *P, S)) return r;
      }
      if (P && P->phase == OrdDec::CHECK)    // P's next pass starts in time for the next launch
        if (int r = ord_check(ctx, *P, slots, false, S)) return r;
    }
    D.np = 1;
    if (!excl.empty()) {
      HIPCHK(hipMemcpy(D.d_list, excl.data(), sizeof(int) * excl.size(), hipMemcpyHostToDevice));
      h9g_exclude_kernel<<<(unsigned)((excl.size() + 255) / 256), 256, 0, ctx->sc>>>((int)excl.size(), (int)n, D.ny,
                                                                                    D.d_list, D.dirty, D.eck);
      HIPCHK(hipGetLastError());
    }
    if (P) {                                 // P's remaining re-runs, then its end into D's start
      if (int r = ord_settle(ctx, *P, slots, S)) return r;
      if (int r = ord_finish(ctx, *P, &D, annual, stop_seen)) return r;
      S.dec_passes.push_back(P->np);
      S.passes += P->np;
    }
    // D's first check (its cells whose start changed flagged too) and the
    // year-1 re-run of every cell whose input changed
    if (int r = ord_chain(ctx, D, land)) return r;
    if (int r = ord_check(ctx, D, slots, true, S)) return r;
    if (D.phase == OrdDec::RERUN)
      if (int r = ord_run_alone(ctx, D, slots, S)) return r;
    if (D.phase == OrdDec::CHECK)
      if (int r = ord_check(ctx, D, slots, false, S)) return r;
    P = &D;
  }
  if (int r = ord_settle(ctx, *P, slots, S)) return r;
  if (int r = ord_finish(ctx, *P, nullptr, annual, stop_seen)) return r;
  S.dec_passes.push_back(P->np);
  S.passes += P->np;
  // the last decade's end: the context's state, STOP records and last-year means
  HIPCHK(hipMemcpyAsync(ctx->d_st, ord_ck(ctx, *P, P->ny - 1), sizeof(float) * srows * n, hipMemcpyDeviceToDevice,
                        ctx->sc));
  HIPCHK(hipMemcpyAsync(ctx->d_err, ord_eck(ctx, *P, P->ny - 1), sizeof(int) * 4 * n, hipMemcpyDeviceToDevice, ctx->sc));
  HIPCHK(hipMemcpyAsync(ctx->d_ann, ord_ann(ctx, *P, P->ny - 1), sizeof(float) * rows * n, hipMemcpyDeviceToDevice,
                        ctx->sc));
  h9g_diag_kernel<<<1, 1024, 0, ctx->sc>>>((int)n, L, ctx->d_ann, ctx->d_st, ctx->d_err, ctx->d_diag);
  HIPCHK(hipGetLastError());
  ctx->last_year = P->y0 + P->ny - 1;
  if (passes)
    for (size_t i = 0; i < S.dec_passes.size(); i++) passes[i] = (int32_t)S.dec_passes[i];
  ctx->dec_stats[0] = S.passes;
  ctx->dec_stats[1] = S.rerun_cells;
  ctx->dec_stats[2] = S.rerun_cell_years;
  ctx->dec_stats[3] = S.rerun_launches;
  ctx->dec_launches = S.launch_cells;
  const int64_t os[9] = {(int64_t)decs.size(), S.ticks, S.ride_steps, S.ride_cell_years, S.alone_steps,
                         S.alone_cell_years, S.excluded, S.probed, S.probe_kept};
  std::copy(os, os + 9, ctx->ord_stats);
  ctx->ord_passes = S.dec_passes;
  // the first STOP of the call (h9g_last_error) or one from before it
  return h9g_sync(ctx);
}

// The reference's decades (HYBRID9.f90:93-113: 1901-1910, 1911-1920, ...)
// cut to [jyear0, jyear0 + nyears).
static std::vector<std::pair<int, int>> ref_decades(int jyear0, int nyears) {
  std::vector<std::pair<int, int>> out;
  for (int y = jyear0, end = jyear0 + nyears; y < end;) {
    const int d = y - 1901, start = 1901 + 10 * (d >= 0 ? d / 10 : -((9 - d) / 10));
    const int e = std::min(start + 10, end);
    out.push_back({y, e - y});
    y = e;
  }
  return out;
}

int h9g_run_decade_ordered(h9g_ctx *ctx, const int32_t *slots, int jyear0, int nyears, float *annual, int32_t *passes) {
  if (nyears < 1) return H9G_EINVAL;
  return run_ordered_impl(ctx, slots, jyear0, {{jyear0, nyears}}, annual, passes);
}

int h9g_run_ordered(h9g_ctx *ctx, const int32_t *slots, int jyear0, int nyears, float *annual, int32_t *passes) {
  if (nyears < 1 || jyear0 < 1861) return H9G_EINVAL;
  return run_ordered_impl(ctx, slots, jyear0, ref_decades(jyear0, nyears), annual, passes);
}

int h9g_set_chains(h9g_ctx *ctx, const int32_t *chain) {
  if (!ctx) return H9G_EINVAL;
  if (!chain) {
    ctx->chain_id.clear();
    return 0;
  }
  for (size_t c = 0; c < ctx->n; c++)
    if (chain[c] < 0 || chain[c] >= (int32_t)ctx->n) {
      fprintf(stderr, "h9g_set_chains: cell %zu has chain id %d, not in [0, ncell): cells outside every reference "
                      "block (shard.reference_blocks gives -1) belong to no rank's run and must be left out of the "
                      "context\n", c, (int)chain[c]);
      return H9G_EINVAL;
    }
  ctx->chain_id.assign(chain, chain + ctx->n);
  return 0;
}

int h9g_decade_stats(h9g_ctx *ctx, int64_t *out, int n) {
  if (!ctx || !out || n < 1) return H9G_EINVAL;
  int m = 0;
  for (; m < n && m < 4; m++) out[m] = ctx->dec_stats[m];
  for (size_t i = 0; m < n && i < ctx->dec_launches.size(); i++) out[m++] = ctx->dec_launches[i];
  return m;
}

int h9g_ordered_stats(h9g_ctx *ctx, int64_t *out, int n) {
  if (!ctx || !out || n < 1) return H9G_EINVAL;
  int m = 0;
  for (; m < n && m < 9; m++) out[m] = ctx->ord_stats[m];
  for (size_t i = 0; m < n && i < ctx->ord_passes.size(); i++) out[m++] = ctx->ord_passes[i];
  return m;
}

int h9g_launch_stats(h9g_ctx *ctx, double *out, int n, int reset) {
  if (!ctx || !out || n < 1) return H9G_EINVAL;
  if (int r = fold_events(ctx)) return r;
  int m = 0;
  for (int k = 1; k <= H9G_KIND_PROBE; k++)
    for (int j = 0; j < 3 && m < n; j++) out[m++] = ctx->kstat[k][j];
  if (reset)
    for (auto &row : ctx->kstat) row[0] = row[1] = row[2] = 0.0;
  return m;
}

int h9g_sync(h9g_ctx *ctx) {
  if (!ctx) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sx));
  if (int r = fold_events(ctx)) return r;
#if defined(H9G_STAMPS)
  if (ctx->d_stamps && (ctx->kind == 1 || ctx->kind == 5 || ctx->kind == 6)) {   // mean shader cycles per wave and substep, by phase
    const size_t cw = (size_t)pair_wave_cols(ctx->kind), nw = (ctx->n + cw - 1) / cw;
    std::vector<unsigned> st(8 * nw);
    HIPCHK(hipMemcpy(st.data(), ctx->d_stamps, sizeof(unsigned) * 8 * nw, hipMemcpyDeviceToHost));
    double sum[8] = {0}, tot = 0;
    for (size_t w = 0; w < nw; w++)
      for (int k = 0; k < 8; k++) sum[k] += st[8 * w + k];
    const double steps = (double)nw * days_in_year(ctx->last_year) * ctx->cfg.nisurf;
    fprintf(stderr, "h9g stamps (cycles/wave/substep):");
    for (int k = 0; k < 8; k++) { fprintf(stderr, " p%d=%.0f", k, sum[k] / steps); tot += sum[k]; }
    fprintf(stderr, " total=%.0f\n", tot / steps);
    // load balance: per-wave totals (the kernel lasts as long as its slowest wave)
    std::vector<double> wt(nw, 0.0);
    for (size_t w = 0; w < nw; w++)
      for (int k = 0; k < 8; k++) wt[w] += st[8 * w + k];
    std::vector<double> ws(wt);
    std::sort(ws.begin(), ws.end());
    const double mean = tot / nw;
    fprintf(stderr, "h9g wave totals / mean: min %.3f p50 %.3f p90 %.3f p99 %.3f max %.3f\n", ws[0] / mean,
            ws[nw / 2] / mean, ws[nw * 9 / 10] / mean, ws[nw * 99 / 100] / mean, ws[nw - 1] / mean);
    // by blockIdx % 8 (workgroups are dealt round-robin to the 8 XCDs) and by wave in block (SIMD)
    double bx[8] = {0}, nx[8] = {0}, bs[4] = {0}, ns[4] = {0};
    for (size_t w = 0; w < nw; w++) {
      const size_t b = w / 4;
      bx[b % 8] += wt[w];
      nx[b % 8] += 1;
      bs[w % 4] += wt[w];
      ns[w % 4] += 1;
    }
    {  // phases of the slowest tenth of the waves against the fastest half
      const double cut90 = ws[nw * 9 / 10], cut50 = ws[nw / 2];
      double hi[8] = {0}, lo[8] = {0}, nh = 0, nl = 0;
      for (size_t w = 0; w < nw; w++) {
        if (wt[w] >= cut90) { nh++; for (int k = 0; k < 8; k++) hi[k] += st[8 * w + k]; }
        if (wt[w] <= cut50) { nl++; for (int k = 0; k < 8; k++) lo[k] += st[8 * w + k]; }
      }
      const double sub = (double)days_in_year(ctx->last_year) * ctx->cfg.nisurf;
      fprintf(stderr, "h9g slowest 10%% / fastest 50%% waves by phase (cycles/substep):");
      for (int k = 0; k < 8; k++) fprintf(stderr, " p%d %.0f/%.0f", k, hi[k] / nh / sub, lo[k] / nl / sub);
      fprintf(stderr, "\n");
    }
    {
      fprintf(stderr, "h9g mean wave total by slot decile:");
      for (int d = 0; d < 10; d++) {
        double a = 0, c = 0;
        for (size_t w = nw * d / 10; w < nw * (d + 1) / 10; w++) { a += wt[w]; c++; }
        fprintf(stderr, " %.3f", a / c / mean);
      }
      fprintf(stderr, "\n");
    }
    fprintf(stderr, "h9g mean wave total by block%%8:");
    for (int k = 0; k < 8; k++) fprintf(stderr, " %.3f", bx[k] / nx[k] / mean);
    fprintf(stderr, "  by wave-in-block:");
    for (int k = 0; k < 4; k++) fprintf(stderr, " %.3f", bs[k] / ns[k] / mean);
    fprintf(stderr, "\n");
  }
#endif
#if defined(H9G_COUNT_EXACT)
  {
    unsigned long long cnt = 0;
    HIPCHK(hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(h9g_exact_count), sizeof(cnt)));
    fprintf(stderr, "h9g exact re-runs (lanes, cumulative): %llu\n", cnt);
    std::vector<unsigned> w(1 << 16);
    HIPCHK(hipMemcpyFromSymbol(w.data(), HIP_SYMBOL(h9g_exact_wave), sizeof(unsigned) << 16));
    std::vector<std::pair<unsigned, int>> top;
    for (int i = 0; i < (1 << 16); i++)
      if (w[i]) top.push_back({w[i], i});
    std::sort(top.rbegin(), top.rend());
    fprintf(stderr, "h9g exact re-runs: %zu waves;", top.size());
    for (size_t k = 0; k < top.size() && k < 8; k++) fprintf(stderr, " w%d:%u", top[k].second, top[k].first);
    fprintf(stderr, "\n");
  }
#endif
#if defined(H9G_COUNT_BRANCH)
  {  // waves entering each H9G_BR site per wave-substep since the last sync, and their mean active lanes
    static const char *names[BR_N] = {"substep", "theta", "qb", "eq_exact", "aqpow", "aq_s", "hk_exact", "tri_flux",
                                      "tri_sweep", "recharge", "baseflow", "watmin", "rerun", "powf_redo",
                                      "div_redo", "expf_redo", "powf_fix", "div_fix", "inl", "any_aq", "jwt_col",
                                      "visit2", "snap", "eb_exact", "day"};
    unsigned long long c[64];
    HIPCHK(hipMemcpyFromSymbol(c, HIP_SYMBOL(h9g_branch_count), sizeof(c)));
    const double ws = c[BR_SUBSTEP] ? (double)c[BR_SUBSTEP] : 1.0;
    fprintf(stderr, "h9g branch counts (wave entries per wave-substep, mean lanes):");
    for (int k = 0; k < BR_N; k++)
      if (c[k]) fprintf(stderr, " %s=%.4g/%.1f", names[k], c[k] / ws, (double)c[32 + k] / c[k]);
    fprintf(stderr, "\n");
    memset(c, 0, sizeof(c));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(h9g_branch_count), c, sizeof(c)));
  }
#endif
  int flag = 0;
  HIPCHK(hipMemcpy(&flag, ctx->d_errflag, sizeof(int), hipMemcpyDeviceToHost));
  if (!flag) return 0;
  if (ctx->last_err.code == 0) {
    const size_t n = ctx->n;
    std::vector<int> e(4 * n);
    HIPCHK(hipMemcpy(e.data(), ctx->d_err, sizeof(int) * 4 * n, hipMemcpyDeviceToHost));
    for (size_t c = 0; c < n; c++) {
      if (e[c]) {        // lowest cell index first, as the reference's cell-outer loop
        ctx->last_err.code = e[c];
        ctx->last_err.cell = (int)c;
        ctx->last_err.year = ctx->last_year;
        ctx->last_err.day = e[n + c];
        ctx->last_err.substep = e[2 * n + c];
        ctx->last_err.value = __builtin_bit_cast(float, e[3 * n + c]);
        break;
      }
    }
  }
  return ctx->last_err.code;
}

int h9g_run_site(h9g_ctx *ctx, int nday, const float *sub, const float *daily, const float *lai, float *diag) {
  if (!ctx || nday <= 0 || !sub || !daily || !lai || !diag) return H9G_EINVAL;
  if (!ctx->params_set || !ctx->state_set) return H9G_ESTATE;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  const size_t n = ctx->n, ns = (size_t)ctx->cfg.nisurf;
  const size_t nsub = (size_t)nday * ns * 5 * n, nd = (size_t)nday * 2 * n, nl = (size_t)nday * 3 * n;
  const size_t nout = (size_t)nday * 11 * n;
  float *buf = nullptr;
  HIPCHK(hipMalloc(&buf, sizeof(float) * (nsub + nd + nl + nout)));
  SiteArgs a;
  a.ncell = (int)n;
  a.nday = nday;
  a.nisurf = ctx->cfg.nisurf;
  a.par = ctx->d_par;
  a.st = ctx->d_st;
  a.sub = buf;
  a.daily = buf + nsub;
  a.lai = buf + nsub + nd;
  a.out = buf + nsub + nd + nl;
  a.err = ctx->d_err;
  a.err_flag = ctx->d_errflag;
  int rc = 0;
  hipError_t e = hipMemcpy(buf, sub, sizeof(float) * nsub, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(buf + nsub, daily, sizeof(float) * nd, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(buf + nsub + nd, lai, sizeof(float) * nl, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    H9G_DISPATCH(ctx, h9g_site_kernel, (unsigned)((n + 63) / 64), 64, ctx->sc, a);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->sc);
  if (e == hipSuccess) e = hipMemcpy(diag, a.out, sizeof(float) * nout, hipMemcpyDeviceToHost);
  (void)hipFree(buf);
  if (e != hipSuccess) {
    fprintf(stderr, "h9g: h9g_run_site failed: %s\n", hipGetErrorString(e));
    return H9G_EHIP;
  }
  ctx->last_year = 0;      // error records of a site run: day counts from the start of the run
  ctx->ran = 1;
  rc = h9g_sync(ctx);
  return rc;
}

// Per-cell STOP records of the runs since the last state (re)set: 4 rows of
// ncell int32 -- code (0 = none), day, substep, bits of the float value.
int h9g_get_errors(h9g_ctx *ctx, int32_t *rec) {
  if (!ctx || !rec) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemcpy(rec, ctx->d_err, sizeof(int32_t) * 4 * ctx->n, hipMemcpyDeviceToHost));
  return 0;
}

int h9g_last_error(h9g_ctx *ctx, h9g_error *err) {
  if (!ctx || !err) return H9G_EINVAL;
  *err = ctx->last_err;
  return 0;
}

int h9g_get_annual(h9g_ctx *ctx, float *annual) {
  if (!ctx || !annual) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemcpy(annual, ctx->d_ann, sizeof(float) * (12 + ctx->L) * ctx->n, hipMemcpyDeviceToHost));
  return 0;
}

int h9g_get_diagnostics(h9g_ctx *ctx, double *host_out, double *dev_out) {
  if (!ctx) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  if (dev_out)
    HIPCHK(hipMemcpyAsync(dev_out, ctx->d_diag, sizeof(double) * H9G_NDIAG, hipMemcpyDeviceToDevice, ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  if (host_out) HIPCHK(hipMemcpy(host_out, ctx->d_diag, sizeof(double) * H9G_NDIAG, hipMemcpyDeviceToHost));
  return 0;
}

// Stream-ordered diagnostics hand-off for a cross-GPU all-reduce with no
// host synchronisation: the copy into dev_out waits for the work already
// queued on `stream` (e.g. last year's all-reduce still reading dev_out),
// and `stream` waits for the copy.  The next h9g_run_year queues behind it
// on the compute stream, so year k+1 runs while year k's all-reduce does.
int h9g_get_diagnostics_async(h9g_ctx *ctx, double *dev_out, void *stream) {
  if (!ctx || !dev_out) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipEventRecord(ctx->ev_ext, s));
  HIPCHK(hipStreamWaitEvent(ctx->sc, ctx->ev_ext, 0));
  HIPCHK(hipMemcpyAsync(dev_out, ctx->d_diag, sizeof(double) * H9G_NDIAG, hipMemcpyDeviceToDevice, ctx->sc));
  HIPCHK(hipEventRecord(ctx->ev_diag, ctx->sc));
  HIPCHK(hipStreamWaitEvent(s, ctx->ev_diag, 0));
  return 0;
}

int h9g_set_cells(h9g_ctx *ctx, const int64_t *gid, const float *lat) {
  if (!ctx || !gid || !lat) return H9G_EINVAL;
  ctx->h_gid.assign(gid, gid + ctx->n);
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipMemcpy(ctx->d_gid, gid, sizeof(int64_t) * ctx->n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(ctx->d_lat, lat, sizeof(float) * ctx->n, hipMemcpyHostToDevice));
  return 0;
}

int h9g_synth_params(h9g_ctx *ctx, uint64_t seed) {
  if (!ctx) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  const int n = (int)ctx->n;
  if (ctx->L == 8)
    h9g_synth_params_kernel<8><<<nblocks(n), H9G_BLOCK, 0, ctx->sc>>>(n, ctx->d_gid, seed, ctx->d_par);
  else
    h9g_synth_params_kernel<10><<<nblocks(n), H9G_BLOCK, 0, ctx->sc>>>(n, ctx->d_gid, seed, ctx->d_par);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(ctx->sc));
  ctx->params_set = 1;
  return 0;
}

int h9g_synth_forcing(h9g_ctx *ctx, int slot, uint64_t seed, int day0, int nday) {
  if (!ctx || slot < 0 || slot >= ctx->cfg.nslots || nday < 1 || nday > ctx->cfg.max_days || day0 < 0)
    return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  HIPCHK(hipStreamWaitEvent(ctx->sx, ctx->ev_consumed[slot], 0));
  dim3 grid(nblocks(ctx->n), (unsigned)nday);
  h9g_synth_forcing_kernel<<<grid, H9G_BLOCK, 0, ctx->sx>>>((int)ctx->n, nday, day0, ctx->d_gid, ctx->d_lat, seed,
                                                           (size_t)ctx->cfg.max_days * ctx->n,
                                                           h9g_forcing_slot(ctx, slot));
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ctx->ev_copied[slot], ctx->sx));
  ctx->slot_days[slot] = nday;
  return 0;
}

// Async PGF prefetch (READ_PGF.f90 on a host thread): days [t0, t0+nt) of
// the 7 NetCDF files are gathered for the context's cells (h9g_set_cells)
// into the slot's pinned staging buffer by the reader's thread pool, and
// copied into the slot on the copy stream in 8 day groups, each as soon as
// the pool has filled it (round 4: the copy overlaps the rest of the read
// instead of following it).  h9g_run_year on that slot joins the thread
// first, so the read of year y+1 overlaps the kernel of year y.
int h9g_nc_forcing_prefetch(h9g_ctx *ctx, int slot, const char *const *paths, int nx, int ny, int t0, int nt) {
  if (!ctx || slot < 0 || slot >= ctx->cfg.nslots || !paths || nt < 1 || nt > ctx->cfg.max_days || t0 < 0)
    return H9G_EINVAL;
  if (ctx->h_gid.size() != ctx->n) return H9G_ESTATE;
  for (int k = 0; k < H9G_NFORCING; k++)
    if (!paths[k]) return H9G_EINVAL;
  if (const int prc = join_prefetch(ctx, slot)) return prc;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t n = ctx->n;
  if (!ctx->h_pin[slot])
    HIPCHK(hipHostMalloc(&ctx->h_pin[slot], sizeof(float) * 7 * (size_t)ctx->cfg.max_days * n, hipHostMallocDefault));
  // the staging buffer may still feed the slot's previous copy
  HIPCHK(hipEventSynchronize(ctx->ev_copied[slot]));
  std::vector<std::string> p(paths, paths + H9G_NFORCING);
  ctx->slot_days[slot] = nt;
  ctx->prefetch[slot] = std::thread([ctx, slot, p, nx, ny, t0, nt]() {
    const char *pp[H9G_NFORCING];
    for (int k = 0; k < H9G_NFORCING; k++) pp[k] = p[k].c_str();
    if (hipSetDevice(ctx->device) != hipSuccess ||
        hipStreamWaitEvent(ctx->sx, ctx->ev_consumed[slot], 0) != hipSuccess) {
      ctx->prefetch_rc[slot] = H9G_EHIP;
      return;
    }
    const size_t n = ctx->n;
    float *dst = h9g_forcing_slot(ctx, slot), *src = ctx->h_pin[slot];
    std::atomic<int> hip_rc{0};
    std::mutex q;                      // one enqueuer at a time on the copy stream
    int rc = h9g_nc_read_groups(pp, nx, ny, (int)n, ctx->h_gid.data(), t0, nt, src, 8, [&](int d0, int d1) {
      std::lock_guard<std::mutex> g(q);
      // days [d0, d1) of the 7 variables: staging (7, nt, n) -> slot (7, max_days, n)
      if (hipSetDevice(ctx->device) != hipSuccess ||
          hipMemcpy2DAsync(dst + (size_t)d0 * n, sizeof(float) * ctx->cfg.max_days * n, src + (size_t)d0 * n,
                           sizeof(float) * nt * n, sizeof(float) * (size_t)(d1 - d0) * n, 7, hipMemcpyHostToDevice,
                           ctx->sx) != hipSuccess)
        hip_rc = H9G_EHIP;
    });
    if (rc == 0 && hip_rc) rc = hip_rc;
    if (rc == 0 && hipEventRecord(ctx->ev_copied[slot], ctx->sx) != hipSuccess) rc = H9G_EHIP;
    ctx->prefetch_rc[slot] = rc;
  });
  return 0;
}

// INIT.f90:575-631 for one soil layer (0-based) of the context's cells
// (h9g_set_cells).  ts, ks, lm, ps: the layer's 30" fields, (ny*60) rows of
// nx*60 values (row 0 north), device pointers if on_device else host
// (copied through a device staging buffer).  Writes the theta_s, hksat,
// bsw, psi_s rows of the parameters.
int h9g_soil_layer(h9g_ctx *ctx, int layer, const float *ts, const float *ks, const float *lm, const float *ps,
                   int nx, int ny, int on_device) {
  if (!ctx || layer < 0 || layer >= ctx->L || !ts || !ks || !lm || !ps || nx <= 0 || ny <= 0) return H9G_EINVAL;
  if (ctx->h_gid.size() != ctx->n) return H9G_ESTATE;
  for (auto g : ctx->h_gid)
    if (g < 0 || g >= (int64_t)nx * ny) return H9G_EINVAL;
  HIPCHK(hipSetDevice(ctx->device));
  const size_t pitch = (size_t)nx * 60, npix = pitch * (size_t)ny * 60;
  const float *src[4] = {ts, ks, lm, ps};
  float *stage = nullptr;
  if (!on_device) {
    HIPCHK(hipMalloc(&stage, sizeof(float) * 4 * npix));
    for (int k = 0; k < 4; k++) {
      HIPCHK(hipMemcpyAsync(stage + k * npix, src[k], sizeof(float) * npix, hipMemcpyHostToDevice, ctx->sc));
      src[k] = stage + k * npix;
    }
  }
  if (!ctx->d_slow) HIPCHK(hipMalloc(&ctx->d_slow, sizeof(int) * ctx->n));
  HIPCHK(hipMemsetAsync(ctx->d_slow, 0, sizeof(int) * ctx->n, ctx->sc));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  HIPCHK(hipEventRecord(e0, ctx->sc));
  const int n = (int)ctx->n;
  h9g_soil_kernel<<<n, 64 * H9G_SWAVES, 0, ctx->sc>>>(nx, n, ctx->d_gid, src[0], src[1], src[2], src[3], pitch,
                                                      ctx->L, layer, ctx->d_par, ctx->d_slow);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e1, ctx->sc));
  h9g_soil_seq_kernel<<<(4 * n + 255) / 256, 256, 0, ctx->sc>>>(nx, n, ctx->d_gid, src[0], src[1], src[2], src[3],
                                                               pitch, ctx->L, layer, ctx->d_par, ctx->d_slow);
  HIPCHK(hipGetLastError());
  std::vector<int> slow(ctx->n);
  HIPCHK(hipMemcpyAsync(slow.data(), ctx->d_slow, sizeof(int) * ctx->n, hipMemcpyDeviceToHost, ctx->sc));
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipEventElapsedTime(&ctx->soil_ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (stage) HIPCHK(hipFree(stage));
  ctx->soil_slow = 0;
  for (int v : slow) ctx->soil_slow += v != 0;
  ctx->soil_layers |= 1u << layer;
  return 0;
}

// INIT.f90:661-680 after every layer is built: Fmax of the soiled cells
// (soil_tex > 0, /= 13, SUM(theta_s) > trunc) from the 0.5 deg integer field
// (-9999 -> 3809), NaN elsewhere.  soil_tex, fmax: host (ny, nx) grids.
// The parameters are then complete (h9g_init_state may follow).
int h9g_soil_fmax(h9g_ctx *ctx, const int32_t *soil_tex, const int32_t *fmax, int nx, int ny) {
  if (!ctx || !soil_tex || !fmax || nx <= 0 || ny <= 0) return H9G_EINVAL;
  if (ctx->h_gid.size() != ctx->n || ctx->soil_layers != (1u << ctx->L) - 1) return H9G_ESTATE;
  const size_t n = ctx->n;
  const int L = ctx->L;
  HIPCHK(hipSetDevice(ctx->device));
  std::vector<float> ts((size_t)L * n), fm(n);
  HIPCHK(hipStreamSynchronize(ctx->sc));
  HIPCHK(hipMemcpy(ts.data(), ctx->d_par, sizeof(float) * L * n, hipMemcpyDeviceToHost));
  for (size_t c = 0; c < n; c++) {
    const int64_t g = ctx->h_gid[c];
    if (g < 0 || g >= (int64_t)nx * ny) return H9G_EINVAL;
    float sum = 0.0f;
    for (int i = 0; i < L; i++) sum = sum + ts[(size_t)i * n + c];
    const int tex = soil_tex[g];
    if (tex > 0 && tex != 13 && sum > 1.0E-8f) {
      int v = fmax[g];
      if (v == -9999) v = 3809;
      fm[c] = (float)v / 10000.0f;
    } else {
      fm[c] = __builtin_nanf("");
    }
  }
  HIPCHK(hipMemcpy(ctx->d_par + (size_t)(4 * L) * n, fm.data(), sizeof(float) * n, hipMemcpyHostToDevice));
  ctx->params_set = 1;
  return 0;
}

// Device time of the last h9g_soil_layer's block-average kernel, and the
// number of its cells that took the reference-order path.
float h9g_last_soil_ms(h9g_ctx *ctx) { return ctx ? ctx->soil_ms : 0.0f; }
int h9g_last_soil_slow(h9g_ctx *ctx) { return ctx ? ctx->soil_slow : -1; }

float h9g_last_kernel_ms(h9g_ctx *ctx) { return ctx ? ctx->last_ms : 0.0f; }

double h9g_total_kernel_ms(h9g_ctx *ctx, int reset) {
  if (!ctx) return 0.0;
  const double t = ctx->total_ms;
  if (reset) ctx->total_ms = 0.0;
  return t;
}

const char *h9g_kernel_name(h9g_ctx *ctx) { return ctx ? ctx->kname : ""; }

// (h9g_build_id is defined in h9g_io.cpp, the translation unit that is
// recompiled with every build.)

int h9g_math_selftest(int device, int n, const float *x, const float *y, float *out) {
  if (n <= 0 || !x || !out) return H9G_EINVAL;
  HIPCHK(hipSetDevice(device));
  float *dx = nullptr, *dy = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc(&dx, sizeof(float) * n));
  HIPCHK(hipMalloc(&dout, sizeof(float) * n));
  HIPCHK(hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice));
  if (y) {
    HIPCHK(hipMalloc(&dy, sizeof(float) * n));
    HIPCHK(hipMemcpy(dy, y, sizeof(float) * n, hipMemcpyHostToDevice));
  }
  h9g_math_kernel<<<(n + 255) / 256, 256>>>(n, dx, dy, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, sizeof(float) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dout);
  return 0;
}

int h9g_math_fast_selftest(int device, int n, const float *x, const float *y, float *out, int *flag) {
  if (n <= 0 || !x || !out || !flag) return H9G_EINVAL;
  HIPCHK(hipSetDevice(device));
  float *dx = nullptr, *dy = nullptr, *dout = nullptr;
  int *dflag = nullptr;
  HIPCHK(hipMalloc(&dx, sizeof(float) * n));
  HIPCHK(hipMalloc(&dout, sizeof(float) * n));
  HIPCHK(hipMalloc(&dflag, sizeof(int) * n));
  if (y) HIPCHK(hipMalloc(&dy, sizeof(float) * n));
  HIPCHK(hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice));
  if (y) HIPCHK(hipMemcpy(dy, y, sizeof(float) * n, hipMemcpyHostToDevice));
  h9g_math_fast_kernel<<<(n + 255) / 256, 256>>>(n, dx, dy, dout, dflag);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, sizeof(float) * n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(flag, dflag, sizeof(int) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dy);
  (void)hipFree(dout);
  (void)hipFree(dflag);
  return 0;
}

int h9g_pace_probe(int device, int nblocks, unsigned *out) {
  if (nblocks <= 0 || !out) return H9G_EINVAL;
  HIPCHK(hipSetDevice(device));
  const size_t nw = (size_t)nblocks * H9G_PWAVES;
  unsigned *dout = nullptr, *darr = nullptr;
  HIPCHK(hipMalloc(&dout, sizeof(unsigned) * 3 * nw));
  HIPCHK(hipMalloc(&darr, sizeof(unsigned)));
  HIPCHK(hipMemset(darr, 0, sizeof(unsigned)));
  const size_t lds = sizeof(float) * (size_t)PairStore<8, H9G_PLANES>::ROWS * H9G_PLANES * H9G_PWAVES +
                     sizeof(uint64_t) * 32 + sizeof(double) * 32 + sizeof(float) * zt_size<8>();
  h9g_pace_probe_kernel<<<nblocks, 64 * H9G_PWAVES, lds>>>(dout, darr, (unsigned)nw, 1ll << 29);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, sizeof(unsigned) * 3 * nw, hipMemcpyDeviceToHost));
  (void)hipFree(dout);
  (void)hipFree(darr);
  return 0;
}

int h9g_div_selftest(int device, int n, const float *x, const float *d, float *out, int *flag) {
  if (n <= 0 || !x || !d || !out || !flag) return H9G_EINVAL;
  HIPCHK(hipSetDevice(device));
  float *dx = nullptr, *dd = nullptr, *dout = nullptr;
  int *dflag = nullptr;
  HIPCHK(hipMalloc(&dx, sizeof(float) * n));
  HIPCHK(hipMalloc(&dd, sizeof(float) * n));
  HIPCHK(hipMalloc(&dout, sizeof(float) * n));
  HIPCHK(hipMalloc(&dflag, sizeof(int) * n));
  HIPCHK(hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dd, d, sizeof(float) * n, hipMemcpyHostToDevice));
  h9g_div_kernel<<<(n + 255) / 256, 256>>>(n, dx, dd, dout, dflag);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, sizeof(float) * n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(flag, dflag, sizeof(int) * n, hipMemcpyDeviceToHost));
  (void)hipFree(dx);
  (void)hipFree(dd);
  (void)hipFree(dout);
  (void)hipFree(dflag);
  return 0;
}

// Host build of the synthetic generator (CPU tests pin it to synth.py).
int h9g_synth_host(uint64_t seed, int nlayers, int ncell, const int64_t *gid, const float *lat, int day0,
                   int nday, float *params_out, float *forcing_out) {
  if (ncell < 0 || nlayers < 1 || nlayers > H9G_LMAX) return H9G_EINVAL;
  const size_t n = ncell;
  const int L = nlayers;
  if (params_out) {
    for (size_t c = 0; c < n; c++) {
      for (int l = 0; l < L; l++) {
        float ts, hk, b, ps;
        h9s::params(seed, (uint64_t)gid[c], l, &ts, &hk, &b, &ps);
        params_out[0 * n * L + c * L + l] = ts;
        params_out[1 * n * L + c * L + l] = hk;
        params_out[2 * n * L + c * L + l] = b;
        params_out[3 * n * L + c * L + l] = ps;
      }
      params_out[4 * n * L + c] = h9s::fmax_param(seed, (uint64_t)gid[c]);
    }
  }
  if (forcing_out) {
    for (int d = 0; d < nday; d++)
      for (size_t c = 0; c < n; c++) {
        float v[7];
        h9s::forcing(seed, (uint64_t)gid[c], lat[c], (int64_t)day0 + d, v);
        for (int k = 0; k < 7; k++) forcing_out[(size_t)k * nday * n + (size_t)d * n + c] = v[k];
      }
  }
  return 0;
}

int h9g_land_cells(int nx, int ny, int nland, uint64_t seed, int64_t *gid, float *lat) {
  if (nx <= 0 || ny <= 0 || nland <= 0 || nland > nx * ny || !gid || !lat) return H9G_EINVAL;
  const int64_t ng = (int64_t)nx * ny;
  std::vector<double> score(ng);
  for (int64_t g = 0; g < ng; g++) {
    const double iy = (double)(g / nx);
    const double la = 90.0 - (iy + 0.5) * (180.0 / ny);
    double c = (la + 10.0) / 70.0;
    c = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c);
    const double w = la < -60.0 ? 0.15 : (la > 80.0 ? 0.2 : 0.45 + 0.35 * c);
    score[g] = (double)h9s::u01(seed, 1, (uint64_t)g) * w;
  }
  std::vector<int64_t> idx(ng);
  for (int64_t g = 0; g < ng; g++) idx[g] = g;
  std::nth_element(idx.begin(), idx.begin() + nland, idx.end(), [&](int64_t a, int64_t b) {
    return score[a] > score[b] || (score[a] == score[b] && a < b);
  });
  std::sort(idx.begin(), idx.begin() + nland);
  const float dlat = (float)(180.0 / ny);
  for (int i = 0; i < nland; i++) {
    gid[i] = idx[i];
    lat[i] = (90.0f - dlat * 0.5f) - (float)(idx[i] / nx) * dlat;
  }
  return 0;
}

// Host build of the device math, for CPU checks of the shipped object.
float h9g_host_expf(float x) {
  const h9m::Tabs T = {h_exp2tab, h_log2tab};
  return h9m::expf(x, T);
}
float h9g_host_powf(float x, float y) {
  const h9m::Tabs T = {h_exp2tab, h_log2tab};
  return h9m::powf(x, y, T);
}

}  // extern "C"
#endif  // H9G_ISA_ONLY
