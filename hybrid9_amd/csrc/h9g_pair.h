// h9g_pair.h -- HYDROLOGY substep with two lanes per soil column.
//
// Why: the 0.5 deg grid has 67,420 land cells, i.e. 1,054 one-lane waves
// for 1,024 SIMDs.  One wave per SIMD leaves VALU issue and LDS latency
// exposed (a lone wave64 issues at most every 4 cycles; the SIMD can take
// one every 2), and the 30 surplus waves double up on 30 SIMDs and set the
// kernel time.  Giving each column two lanes ("a pair": lanes 2k, 2k+1 of
// a wave) halves the per-lane share of the work that is independent per
// layer -- the equilibrium profile zq (HYDROLOGY.f90:517-590), hydraulic
// conductivity and matric potential (:598-639) and the specific yields
// (:937-981), i.e. 40 of the ~46 glibc-exact powf of a substep -- and
// lets 22 columns per wave x 4-wave workgroups place exactly 3 waves on
// every SIMD (767 workgroups for 768 slots at 0.5 deg).
//
// Layer split: lane h (0 = even, 1 = odd) of a pair owns layers 2t+1+h,
// t = 0..L/2-1.  A per-layer phase evaluates the reference expression for
// the lane's own layers and swaps the results with the partner lane (DPP
// quad_perm [1,0,3,2]); everything else (energy balance, tridiagonal
// system, Thomas solve, drainage, ...) runs identically in both lanes.
// Every value is computed by exactly the reference expression, so the
// split changes no bit.
//
// One code path serves three builds through two policies:
//   Split2   device fast path: own layers per lane + DPP exchange;
//   SplitAll one lane computes every layer: the device exact re-run
//            (MathExact) and the host test build (tests/csrc/host_kernel.cpp).
// Stores: PairStore (device LDS, [row][lane] with the pair's layers
// interleaved over its two columns) and FlatStore (host, flat per cell).
#pragma once
#include "h9g_step.h"
#if !defined(__HIPCC__) && !defined(__HIP__)
#define __device__
#define __forceinline__ inline
#endif

#ifndef H9G_EXACT_HOOK
#define H9G_EXACT_HOOK(k0, ns)         // test builds: count the exact re-runs (tests/csrc/host_kernel.cpp)
#endif
#if defined(H9G_COUNT_EXACT)
__device__ unsigned long long h9g_exact_count;   // exact re-runs (lanes), measurement builds only
__device__ unsigned h9g_exact_wave[1 << 16];     // ... per wave (blockIdx * 4 + wave), pair kernel
#endif
namespace h9k {

// per-layer store fields (L entries each)
enum : int {
  PF_TS = 0, PF_HKS, PF_BSW, PF_PSI,   // soil parameters (SHARED.f90:398-429)
  PF_NINVB,                            // -one/bsw
  PF_ITS,                              // one/(ts(I)+ts(I+1))
  PF_PTE,                              // psi*ts/(one-one/bsw)
  PF_C3,                               // pte/(zi(I)-zi(I-1))
  PF_ROOTR,                            // rootr_col(1..L)
  PF_RPSI0, PF_RPSI1,                  // 1/(-psi), double (recip64) low, high word   (kRecip)
  PF_RTS0, PF_RTS1,                    // 1/theta_s, double                           (kRts)
  PF_SVH2O, PF_SVSMP,                  // day snapshot (sv_* of the store)
  PF_N
};
// per-cell fields
enum : int {
  PS_FMAX = 0, PS_MH3, PS_TSDZ1, PS_DAY,
  PS_LAI = PS_DAY + D_N,               // plant state, parked over the substeps (pair kernel)
  PS_LAIL, PS_PM, PS_PFM, PS_PLEN, PS_RDEPTH,
  PS_DR0,                              // day-constant reciprocals (kDayRecip): pairs
  PS_DRS = PS_DR0 + 4 * DRP_N,         //   (c.lo s.lo c.hi s.hi), then shared doubles (lo hi)
  PS_SVZWT = PS_DR0 + 2 * DR_N,        // day snapshot for the exact re-run (sv_* of the store)
  PS_SVWA, PS_SVRNF, PS_SVERR, PS_SVNS,
  PS_N
};
enum : int { SV_ZWT = 0, SV_WA, SV_RNF, SV_ERR, SV_NS };   // sv_sc fields (SV_NS: substep of the snapshot)
// canopy/soil pairs share a row, canopy in the even column (see D_NUMC)
static_assert((PS_DAY + D_NUMC) % 2 == 0 && (PS_DAY + D_RAARAC) % 2 == 0 && (PS_DAY + D_DGRAC) % 2 == 0 &&
                  (PS_DAY + D_DRR) % 2 == 0 && (PS_DAY + D_RAC) % 2 == 0 && PS_DR0 % 2 == 0,
              "pair fields must start a row");

#ifndef H9G_FE_EQ
#define H9G_FE_EQ 1   // fence interval of the equilibrium-profile slots (Split2::par)
#endif
#ifndef H9G_FE_HK
#define H9G_FE_HK 1   // ... of the conductivity / matric-potential slots
#endif
#ifndef H9G_FE2
#define H9G_FE2 1     // both, in the 2-wave build (PairStore R = 2)
#endif
#ifndef H9G_SPARE_FENCE
#define H9G_SPARE_FENCE 0      // rounds of the spare-lane phases followed by a scheduling fence (bit q)
#endif
#ifndef H9G_INL_LAST
// the in-layer case branch-free in the pairs' last-slot round (hydrology_pair;
// round 5: 182.7 -> 181.8 ms, three alternating pairs on one box)
#define H9G_INL_LAST 1
#endif
#ifndef H9G_EB_FAST
#define H9G_EB_FAST 1    // round 5: 182.2 -> 181.7 ms; the energy balance's quotients branch-free, runtime divisors by Markstein (hydrology_pair)
#endif
#ifndef H9G_HK_MDIV
#define H9G_HK_MDIV 1    // the conductivity phase's dsmpdw quotient by Markstein at L = 8 (hk_body; round 5: -0.3%; L = 10: +0.8%)
#endif
#ifndef H9G_INL_MDIV
#define H9G_INL_MDIV 0   // the in-layer case's PTE / (zw - zlo) by Markstein (eq_body) instead of recip64
#endif
#ifndef H9G_WT_DEFER
#define H9G_WT_DEFER 1   // the water-table loops' x/1000 flag the substep's exact re-run (hydrology_pair; round 5: -0.45%)
#endif
#ifndef H9G_AQ_FREE
#define H9G_AQ_FREE 0    // the aquifer node's second round and interface branch-free (hydrology_pair)
#endif
#ifndef H9G_SPARE_L10
#define H9G_SPARE_L10 0   // spare lanes in the 3-wave L = 10 build too (PairStore::kSpare)
#endif

template <int K>
struct FV {
  float v[K];
};

H9K_HD float sel(int h, float a, float b) { return h ? b : a; }
H9K_HD double seld(int h, double a, double b) { return h ? b : a; }

// value of the partner lane (lane ^ 1)
H9K_HD float pair_swap(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int x = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));
#else
  return v;
#endif
}

// value of the pair's even (E = 0) or odd (E = 1) lane, in both lanes (DPP
// quad_perm [0,0,2,2] / [1,1,3,3]): one instruction instead of pair_swap
// plus a select per lane
template <int E>
H9K_HD float pair_bcast(float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const int x = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(x, E ? 0xF5 : 0xA0, 0xF, 0xF, true));
#else
  return v;
#endif
}

// value of lane `src` of the wave (ds_bpermute: the LDS crossbar, no LDS
// storage); the spare lanes' operands and results (hydrology_pair)
H9K_HD float lane_get(float v, int src) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src << 2, __builtin_bit_cast(int, v)));
#else
  (void)src;
  return v;
#endif
}
H9K_HD int lane_geti(int v, int src) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ds_bpermute(src << 2, v);
#else
  (void)src;
  return v;
#endif
}

// A double kept as two float fields (low word, high word).
H9K_HD double join_d(float lo, float hi) {
  return __builtin_bit_cast(double, (uint64_t)__builtin_bit_cast(uint32_t, hi) << 32 |
                                        __builtin_bit_cast(uint32_t, lo));
}
H9K_HD float lo_d(double v) { return __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(uint64_t, v)); }
H9K_HD float hi_d(double v) {
  return __builtin_bit_cast(float, (uint32_t)(__builtin_bit_cast(uint64_t, v) >> 32));
}

// ------------------------------------------------------------------ stores
// Every store has the same interface: lay/set_lay (per-layer field p of
// layer i), sc/set_sc (per-cell field k), slot/set_slot (own layer t of a
// pair lane), day/set_day, the day reciprocals day_r/set_day_r, and the
// day snapshot sv_* (q = 0: h2osoi_liq, 1: smp; k = SV_*).  kRecip,
// kRts, kDayRecip say which reciprocal fields it holds (LDS budget).
template <int L>
struct FlatStore {                     // host: one flat array per cell
  static constexpr bool kRecip = true, kRts = true, kDayRecip = true, kRtsHK = true, kSpare = false;
  static constexpr int FE_EQ = 1, FE_HK = 1;
  static constexpr int N = PF_N * L + PS_N;
  float *b;
  const float *zt;                     // zi(0..L+1), then zi(0..L+1)/1000
  H9K_HD float zi(int i) const { return zt[i]; }
  H9K_HD float zim(int i) const { return zt[L + 2 + i]; }
  H9K_HD double rdz_t(int i) const { return join_d(zt[2 * (L + 2) + 2 * i], zt[2 * (L + 2) + 2 * i + 1]); }
  H9K_HD float lay(int p, int i) const { return b[p * L + i - 1]; }
  H9K_HD void set_lay(int p, int i, float v) const { b[p * L + i - 1] = v; }
  H9K_HD float sc(int k) const { return b[PF_N * L + k]; }
  H9K_HD void set_sc(int k, float v) const { b[PF_N * L + k] = v; }
  H9K_HD float slot(int p, int t) const { return b[p * L + 2 * t]; }   // unused (SplitAll)
  H9K_HD void set_slot(int p, int t, float v) const { b[p * L + 2 * t] = v; }
  H9K_HD void launder() {}
  H9K_HD float day(int f) const { return sc(PS_DAY + f); }
  H9K_HD void set_day(int f, float v) const { set_sc(PS_DAY + f, v); }
  H9K_HD double day_r(int k) const { return join_d(sc(PS_DRS + 2 * k), sc(PS_DRS + 2 * k + 1)); }
  H9K_HD void set_day_r(int k, double v) const {
    set_sc(PS_DRS + 2 * k, lo_d(v));
    set_sc(PS_DRS + 2 * k + 1, hi_d(v));
  }
  H9K_HD double day_rp(int j, int h) const { return join_d(sc(PS_DR0 + 4 * j + h), sc(PS_DR0 + 4 * j + 2 + h)); }
  H9K_HD void set_day_rp(int j, int h, double v) const {
    set_sc(PS_DR0 + 4 * j + h, lo_d(v));
    set_sc(PS_DR0 + 4 * j + 2 + h, hi_d(v));
  }
  H9K_HD float root(int i) const { return lay(PF_ROOTR, i); }
  H9K_HD void set_root(int i, float v) const { set_lay(PF_ROOTR, i, v); }
  H9K_HD float sv_lay(int q, int i) const { return lay(PF_SVH2O + q, i); }
  H9K_HD void sv_set_lay(int q, int i, float v) const { set_lay(PF_SVH2O + q, i, v); }
  H9K_HD float sv_sc(int k) const { return sc(PS_SVZWT + k); }
  H9K_HD void sv_set_sc(int k, float v) const { set_sc(PS_SVZWT + k, v); }
  H9K_HD void sv_sync() const {}
  H9K_HD void day_start(int) const {}
};

// Device: [row][S] LDS block per wave, S = lanes per wave.  Layer i of a
// per-layer field sits in row p*L/2 + (i-1)/2 of the pair's column
// (i-1)&1, so a lane's own layers are its own column's rows and any layer
// is a static offset from the pair's even column.  Per-cell fields are
// spread the same way over the two columns.  Both lanes of a pair store
// identical values to the same address where they both write.
//
// The day snapshot lives in global memory (L2-resident: 80 B per
// cell), in a per-workgroup block shaped like the LDS block: the byte
// offset of a value is its LDS address, so every snapshot store is
// `global_store v_lds_address, s_block + imm` with no address arithmetic.
// That leaves LDS room, within 3 workgroups per CU (75 rows per wave), for
// the reciprocal fields: 1/(-psi) at any L, 1/theta_s and the day
// reciprocals at L = 8 (75 rows; L = 10: 72 rows; the 2-wave build: all of
// them at L = 10 too, 89 rows).
// Issue priority of the waves sharing a SIMD (one from each of the CU's
// resident workgroups).  The SIMD arbitrates VALU issue by priority, then by
// wave age, so with equal priorities the oldest wave runs at its lone-wave
// rate, the youngest is starved, and the kernel ends on the youngest waves
// running alone (measured: the first-dispatched third of the waves took
// 0.82x the mean time, the last third 1.21x).
//   mode 1 (rotate): the top priority rotates over the resident rounds every
//     day, so the waves get equal issue shares (config 2: 283 -> 251 ms;
//     slowest wave 1.25 -> 1.09x the mean).  Rotating every 1, 4 or 16
//     substeps instead measured the same.
//   mode 2 (pace): each wave posts its day to a per-SIMD row in global memory
//     (keyed by the hardware XCC/SE/SH/CU/SIMD ids, tagged with the launch
//     epoch) and takes a priority equal to the number of waves on its SIMD
//     that are ahead of it, so the waves of a SIMD keep the same day and
//     finish together instead of one heavy wave finishing alone.
struct Pacer {
  unsigned *row;      // mode 2: this SIMD's 16 progress words
  unsigned epoch;     // mode 2: launch tag (20 bits)
  int me;             // mode 2: hardware wave slot (0..15)
  int mode;
  int round;          // mode 1: 0..resident-1, which of the CU's resident workgroups
  __device__ __forceinline__ static void set_prio(int p) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (p <= 0)
      __builtin_amdgcn_s_setprio(0);
    else if (p == 1)
      __builtin_amdgcn_s_setprio(1);
    else if (p == 2)
      __builtin_amdgcn_s_setprio(2);
    else
      __builtin_amdgcn_s_setprio(3);
#endif
  }
  __device__ __forceinline__ void day_start(int day, int resident) const {
#if defined(__HIP_DEVICE_COMPILE__)
    if (mode == 1) {
      set_prio((round + day) % resident);
    } else if (mode == 2) {
      const unsigned mine = (epoch << 12) | (unsigned)(day + 1);
      __hip_atomic_store(row + me, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int k = (int)(__lane_id() & 15);
      const unsigned v = __hip_atomic_load(row + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool ahead = k != me && (v >> 12) == (epoch & 0xfffffu) && (v & 0xfffu) > (unsigned)(day + 1);
      const uint64_t m = __builtin_amdgcn_ballot_w64(ahead);
      const unsigned slots = (unsigned)(m | (m >> 16) | (m >> 32) | (m >> 48)) & 0xffffu;
      set_prio(__builtin_popcount(slots));
    }
#endif
  }
};
// Key of the SIMD this wave runs on and its slot there (HW_REG_HW_ID:
// wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13; HW_REG_XCC_ID 3:0).
#define H9G_PACE_ROWS 16384
__device__ __forceinline__ void pace_key(int &row, int &slot) {
#if defined(__HIP_DEVICE_COMPILE__)
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
  slot = (int)(hw & 15u);
  row = (int)(((((xcc * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u + ((hw >> 8) & 15u)) * 4u) +
              ((hw >> 4) & 3u));
#else
  row = slot = 0;
#endif
}

// The L = 10 pair kernel runs 3 waves per SIMD like L = 8: without the
// per-layer double reciprocal of theta_s and the day constants' its LDS block
// fits three workgroups per CU (72 rows, 51.4 KB), and 168 VGPRs (config 5:
// 632 -> 535 ms per year against 2 waves/SIMD with every reciprocal,
// DESIGN.md §6).
template <int L>
constexpr int pair_resident() { return 3; }   // waves per SIMD (h9g.hip pair_waves)

// R = waves per SIMD the kernel is built for (its workgroups per CU): 3 (the
// default, 168 VGPRs, <= 53 KB LDS per workgroup) or 2 (round 4, L = 10:
// 256 VGPRs and 80 KB, so no spills and every reciprocal field; h9g.hip
// h9g_pair2_kernel).
template <int L, int S, int R = pair_resident<L>()>
struct PairStore {
  static constexpr int NT = L / 2;
  // LDS fields by layer count (3 workgroups per CU: at most 75 rows).  L = 8:
  // every reciprocal (75 rows).  L = 10 (5 rows per per-layer field): 1/(-psi)
  // (~15 divisions per substep) instead of the day constants' reciprocals (~5;
  // round 3: 533.6 -> 530.3 ms for config 5), no 1/theta_s (72 rows).  At
  // R = 2 every reciprocal fits at L = 10 too (89 rows).
  // (S = 22, the 11-column wave of h9g_pair11_kernel, leaves the LDS room for
  // every reciprocal at L = 10 and 3 workgroups per CU too: 89 rows, 31.3 KB)
  static constexpr bool kRecip = true, kRts = L <= 8 || R <= 2 || S <= 22, kDayRecip = L <= 8 || R <= 2 || S <= 22;
  // s_node of the conductivity phase from the stored 1/theta_s too (round 3:
  // no longer spills in the call-free kernel)
  static constexpr bool kRtsHK = kRts;
  static constexpr int NPF = kRecip ? (kRts ? PF_SVH2O : PF_RTS0) : PF_RPSI0;   // per-layer fields in LDS
  static constexpr int NPS = kDayRecip ? PS_SVZWT : PS_DR0; // per-cell fields in LDS
  static constexpr int ROWS = NPF * NT + (NPS + 1) / 2;
  static constexpr int GBLOCK = 65536;                      // bytes per workgroup (>= any LDS address)
  lds_float *self, *even;
  const lds_float *zt;                 // zi(0..L+1), then zi(0..L+1)/1000 (per block)
  float *svw;                          // this workgroup's day-snapshot block (global)
  static constexpr int RESIDENT = R;                        // workgroups per CU = waves per SIMD
  // fence intervals of the per-layer phases' slots (Split2::par_d): one slot
  // per scheduling region at 3 waves per SIMD (wider regions spill, DESIGN.md
  // §3); the 2-wave build has the registers for H9G_FE2 slots per region
  static constexpr int FE_EQ = R <= 2 ? H9G_FE2 : H9G_FE_EQ, FE_HK = R <= 2 ? H9G_FE2 : H9G_FE_HK;
  Pacer pace;
  lds_float *wb;                       // the wave's block (column 0): spare lanes' stolen slots
  static constexpr int LANES = S;
  // helper lanes in the per-layer phases (hydrology_pair): not in the 3-wave
  // L = 10 build of 22-column waves, whose registers they push further into
  // scratch
  static constexpr bool kSpare = H9G_SPARE_L10 || !(L >= 10 && R >= 3 && S >= 44);
  __device__ __forceinline__ void day_start(int day) const { pace.day_start(day, RESIDENT); }
  __device__ __forceinline__ float zi(int i) const { return zt[i]; }
  __device__ __forceinline__ float zim(int i) const { return zt[L + 2 + i]; }
  __device__ __forceinline__ double rdz_t(int i) const {
    return join_d(zt[2 * (L + 2) + 2 * i], zt[2 * (L + 2) + 2 * i + 1]);
  }
  __device__ __forceinline__ float lay(int p, int i) const {
    return even[(p * NT + ((i - 1) >> 1)) * S + ((i - 1) & 1)];
  }
  __device__ __forceinline__ void set_lay(int p, int i, float v) const {
    even[(p * NT + ((i - 1) >> 1)) * S + ((i - 1) & 1)] = v;
  }
  __device__ __forceinline__ float sc(int k) const { return even[(NPF * NT + (k >> 1)) * S + (k & 1)]; }
  __device__ __forceinline__ void set_sc(int k, float v) const {
    even[(NPF * NT + (k >> 1)) * S + (k & 1)] = v;
  }
  __device__ __forceinline__ float slot(int p, int t) const { return self[(p * NT + t) * S]; }
  __device__ __forceinline__ void set_slot(int p, int t, float v) const { self[(p * NT + t) * S] = v; }
  __device__ __forceinline__ void launder() {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(self), "+v"(even), "+v"(zt)::"memory");
#endif
  }
  __device__ __forceinline__ float day(int f) const { return sc(PS_DAY + f); }
  __device__ __forceinline__ void set_day(int f, float v) const { set_sc(PS_DAY + f, v); }
  __device__ __forceinline__ double day_r(int k) const {
    return join_d(sc(PS_DRS + 2 * k), sc(PS_DRS + 2 * k + 1));
  }
  __device__ __forceinline__ void set_day_r(int k, double v) const {
    set_sc(PS_DRS + 2 * k, lo_d(v));
    set_sc(PS_DRS + 2 * k + 1, hi_d(v));
  }
  __device__ __forceinline__ double day_rp(int j, int h) const {
    return join_d(sc(PS_DR0 + 4 * j + h), sc(PS_DR0 + 4 * j + 2 + h));
  }
  __device__ __forceinline__ void set_day_rp(int j, int h, double v) const {
    set_sc(PS_DR0 + 4 * j + h, lo_d(v));
    set_sc(PS_DR0 + 4 * j + 2 + h, hi_d(v));
  }
  // per-cell field k (even) + this lane's parity: the lane's own column of
  // the row holding fields k, k+1
  __device__ __forceinline__ float sc_own(int k) const { return self[(NPF * NT + (k >> 1)) * S]; }
  __device__ __forceinline__ double day_rp_own(int j) const {
    return join_d(sc_own(PS_DR0 + 4 * j), sc_own(PS_DR0 + 4 * j + 2));
  }
  __device__ __forceinline__ float root(int i) const { return lay(PF_ROOTR, i); }
  __device__ __forceinline__ void set_root(int i, float v) const { set_lay(PF_ROOTR, i, v); }
  // snapshot: rows q*NT + t (layers), 2*NT + k/2 (scalars) of the global block
  __device__ __forceinline__ float *gl(const lds_float *p, int off) const {
    return (float *)((char *)svw + (uint32_t)(size_t)p) + off;
  }
  __device__ __forceinline__ void sv_set_slot(int q, int t, float v) const { *gl(self, (q * NT + t) * S) = v; }
  __device__ __forceinline__ float sv_lay(int q, int i) const {
    return *gl(even, (q * NT + ((i - 1) >> 1)) * S + ((i - 1) & 1));
  }
  __device__ __forceinline__ void sv_set_lay(int q, int i, float v) const {
    *gl(even, (q * NT + ((i - 1) >> 1)) * S + ((i - 1) & 1)) = v;
  }
  __device__ __forceinline__ float sv_sc(int k) const { return *gl(even, (2 * NT + (k >> 1)) * S + (k & 1)); }
  __device__ __forceinline__ void sv_set_sc(int k, float v) const {
    *gl(even, (2 * NT + (k >> 1)) * S + (k & 1)) = v;
  }
  // before reading back what the wave stored (the exact re-run)
  __device__ __forceinline__ void sv_sync() const {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
#endif
  }
};

// Device, one lane per column ("solo"): column `lane` of a [row][64] block,
// every field in the lane's own column; no reciprocal fields, no parking
// (1054 waves = 5 blocks/CU), day snapshot in LDS.
template <int L>
struct SoloStore {
  static constexpr bool kRecip = false, kRts = false, kDayRecip = false, kRtsHK = false, kSpare = false;
  static constexpr int FE_EQ = 1, FE_HK = 1;
  static constexpr int NPF = PF_RPSI0 + 2;           // TS..ROOTR, SVH2O, SVSMP
  static constexpr int NPS = PS_LAI + 5;             // FMAX..DAY, SV*
  static constexpr int ROWS = NPF * L + NPS;
  lds_float *b;
  const lds_float *zt;
  H9K_HD static constexpr int pr(int p) { return p < PF_RPSI0 ? p : p - (PF_SVH2O - PF_RPSI0); }
  H9K_HD static constexpr int kr(int k) { return k < PS_LAI ? k : k - (PS_SVZWT - PS_LAI); }
  __device__ __forceinline__ float zi(int i) const { return zt[i]; }
  __device__ __forceinline__ float zim(int i) const { return zt[L + 2 + i]; }
  __device__ __forceinline__ double rdz_t(int i) const {
    return join_d(zt[2 * (L + 2) + 2 * i], zt[2 * (L + 2) + 2 * i + 1]);
  }
  __device__ __forceinline__ float lay(int p, int i) const { return b[(pr(p) * L + i - 1) * 64]; }
  __device__ __forceinline__ void set_lay(int p, int i, float v) const { b[(pr(p) * L + i - 1) * 64] = v; }
  __device__ __forceinline__ float sc(int k) const { return b[(NPF * L + kr(k)) * 64]; }
  __device__ __forceinline__ void set_sc(int k, float v) const { b[(NPF * L + kr(k)) * 64] = v; }
  __device__ __forceinline__ float slot(int p, int t) const { return b[(pr(p) * L + 2 * t) * 64]; }
  __device__ __forceinline__ void set_slot(int p, int t, float v) const { b[(pr(p) * L + 2 * t) * 64] = v; }
  __device__ __forceinline__ void launder() {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(b), "+v"(zt)::"memory");
#endif
  }
  __device__ __forceinline__ float day(int f) const { return sc(PS_DAY + f); }
  __device__ __forceinline__ void set_day(int f, float v) const { set_sc(PS_DAY + f, v); }
  __device__ __forceinline__ double day_r(int) const { return 0.0; }
  __device__ __forceinline__ void set_day_r(int, double) const {}
  __device__ __forceinline__ double day_rp(int, int) const { return 0.0; }
  __device__ __forceinline__ void set_day_rp(int, int, double) const {}
  __device__ __forceinline__ float root(int i) const { return lay(PF_ROOTR, i); }
  __device__ __forceinline__ void set_root(int i, float v) const { set_lay(PF_ROOTR, i, v); }
  __device__ __forceinline__ float sv_lay(int q, int i) const { return lay(PF_SVH2O + q, i); }
  __device__ __forceinline__ void sv_set_lay(int q, int i, float v) const { set_lay(PF_SVH2O + q, i, v); }
  __device__ __forceinline__ float sv_sc(int k) const { return sc(PS_SVZWT + k); }
  __device__ __forceinline__ void sv_set_sc(int k, float v) const { set_sc(PS_SVZWT + k, v); }
  __device__ __forceinline__ void sv_sync() const {}
  __device__ __forceinline__ void day_start(int) const {}
};

// Phase profiler (tools: H9G_STAMPS build only).  NoProf compiles away.
// flux(evg, tran) receives the substep's qflx_evap_grnd and
// qflx_tran_veg_col (HYDROLOGY.f90:388-400); only the site path keeps them.
struct NoProf {
#if defined(H9G_ISA_PHASES) && defined(__HIP_DEVICE_COMPILE__)
  template <int K>
  __device__ __forceinline__ void markk() { asm volatile("; h9g-phase %0" ::"i"(K)); }   // tools/isa_mix.py --phases
  H9K_HD void mark(int k) {
    switch (k) {
      case 0: markk<0>(); break;
      case 1: markk<1>(); break;
      case 2: markk<2>(); break;
      case 3: markk<3>(); break;
      case 4: markk<4>(); break;
      case 5: markk<5>(); break;
      case 6: markk<6>(); break;
      default: markk<7>(); break;
    }
  }
#else
  H9K_HD void mark(int) {}
#endif
  H9K_HD void flux(float, float) {}
};
struct FluxProf {
  float evg, tran;
  H9K_HD void mark(int) {}
  H9K_HD void flux(float e, float t) { evg = e; tran = t; }
};
#if defined(H9G_STAMPS)
H9K_HD uint64_t stamp_clock() {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_s_memtime();
#else
  return 0;
#endif
}
struct StampProf {                     // wave-uniform shader-clock deltas per phase
  uint64_t last;
  uint32_t acc[8];
  H9K_HD void mark(int k) {
    const uint64_t t = stamp_clock();
    acc[k] += (uint32_t)(t - last);
    last = t;
  }
  H9K_HD void flux(float, float) {}
};
#endif

// ---------------------------------------------------------------- policies
// One lane computes every layer.
struct SplitAll {
  static constexpr bool kSpare = false;
  H9K_HD constexpr bool act() const { return true; }
  H9K_HD SplitAll fresh() const { return *this; }
  template <class CS>
  H9K_HD float own(const CS &cs, int p, int t, int h) const { return cs.lay(p, 2 * t + 1 + h); }
  // out[2t+1+h] = f(t, h).f for every layer; K outputs per layer
  template <int NT, int K, int FE = 1, class F>
  H9K_HD void par(F f, float *const (&out)[K]) const {
#pragma unroll
    for (int t = 0; t < NT; t++) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const FV<K> r = f(t, h);
#pragma unroll
        for (int k = 0; k < K; k++) out[k][2 * t + 1 + h] = r.v[k];
      }
      sched_fence();
    }
  }
  // par with deferred checks: fast(t, h, bad) is branch-free and sets bad
  // when any of its results needs glibc's/IEEE's other path; exact(t, h)
  // (the body with in-place redos) then recomputes the layer.
  template <int NT, int K, int FE = 1, class FF, class FX>
  H9K_HD void par_d(FF fast, FX exact, float *const (&out)[K]) const {
#pragma unroll
    for (int t = 0; t < NT; t++) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        bool bad = false;
        FV<K> r = fast(t, h, bad);
        if (bad) r = exact(t, h);
#pragma unroll
        for (int k = 0; k < K; k++) out[k][2 * t + 1 + h] = r.v[k];
      }
      sched_fence();
    }
  }
  // r0 = f(0), r1 = f(1)
  template <int K, class F>
  H9K_HD void pick(F f, FV<K> &r0, FV<K> &r1) const {
    r0 = f(0);
    r1 = f(1);
  }
  H9K_HD bool pair_any(bool p) const { return p; }
  // per-cell field k + h of a canopy/soil pair (k even), the pair's day reciprocal
  template <class CS>
  H9K_HD float own_sc(const CS &cs, int k, int h) const { return cs.sc(k + h); }
  template <class CS>
  H9K_HD double own_day_rp(const CS &cs, int j, int h) const { return cs.day_rp(j, h); }
};

// Two lanes per column (device fast path); h = lane & 1.  The wave's lanes
// past the pairs (spare lanes, ln >= PairStore::LANES) take part only in the
// per-layer phases, where they evaluate the pairs' last slot (hydrology_pair)
// and are masked off everywhere else (act()).
struct Split2 {
  int h;
  int ln;                         // lane in the wave
  bool spare;
  static constexpr bool kSpare = true;
  H9K_HD bool act() const { return !spare; }
  H9K_HD Split2 fresh() const {   // h, opaque to the optimiser (hydrology_pair)
    Split2 r{h, ln, spare};
    opaque(r.h);
    return r;
  }
  // v of the even lane -> e, of the odd lane -> o, in both lanes: two DPP
  // broadcasts (round 3; round 2 swapped and selected per lane: one DPP
  // move and two selects, 214.5 -> 213.9 ms)
  H9K_HD void xchg(float v, float &e, float &o) const {
    e = pair_bcast<0>(v);
    o = pair_bcast<1>(v);
  }
  template <class CS>
  H9K_HD float own(const CS &cs, int p, int t, int) const { return cs.slot(p, t); }
  // FE: a scheduling fence after every FE slots (FE > 1 lets the scheduler
  // interleave FE slots' powers, at FE times the live temporaries)
  template <int NT, int K, int FE = 1, class F>
  H9K_HD void par(F f, float *const (&out)[K]) const {
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const FV<K> r = f(t, h);
#pragma unroll
      for (int k = 0; k < K; k++) xchg(r.v[k], out[k][2 * t + 1], out[k][2 * t + 2]);
      if ((t + 1) % FE == 0 || t == NT - 1) sched_fence();
    }
  }
  // par with the special-case checks of all NT slots deferred to one
  // rarely-taken branch after them (SplitAll::par_d): with no per-slot
  // branch the slots form one basic block, so the scheduler can interleave
  // FE slots' powers.  A lane with any flag recomputes its slots exactly.
  template <int NT, int K, int FE = 1, class FF, class FX>
  H9K_HD void par_d(FF fast, FX exact, float *const (&out)[K]) const {
    FV<K> r[NT];
    bool bad = false;
#pragma unroll
    for (int t = 0; t < NT; t++) {
      r[t] = fast(t, h, bad);
      if ((t + 1) % FE == 0 || t == NT - 1) sched_fence();
    }
    if (__builtin_expect(bad, 0)) {
#pragma unroll
      for (int t = 0; t < NT; t++) r[t] = exact(t, h);
    }
#pragma unroll
    for (int t = 0; t < NT; t++) {
#pragma unroll
      for (int k = 0; k < K; k++) xchg(r[t].v[k], out[k][2 * t + 1], out[k][2 * t + 2]);
    }
  }
  template <int K, class F>
  H9K_HD void pick(F f, FV<K> &r0, FV<K> &r1) const {
    const FV<K> r = f(h);
#pragma unroll
    for (int k = 0; k < K; k++) xchg(r.v[k], r0.v[k], r1.v[k]);
  }
  H9K_HD bool pair_any(bool p) const {
    const float f = p ? 1.0f : 0.0f;
    return (f + pair_swap(f)) != 0.0f;
  }
  template <class CS>
  H9K_HD float own_sc(const CS &cs, int k, int) const { return cs.sc_own(k); }
  template <class CS>
  H9K_HD double own_day_rp(const CS &cs, int j, int) const { return cs.day_rp_own(j); }
};

// Rollback copy of a per-layer state array (1-based v[1..L]).
template <int L, class CS>
H9K_HD void save_layers(const SplitAll &, const CS &cs, int q, const float *v) {
#pragma unroll
  for (int i = 1; i <= L; i++) cs.sv_set_lay(q, i, v[i]);
}
template <int L, class CS>
H9K_HD void save_layers(const Split2 &sp, const CS &cs, int q, const float *v) {
#pragma unroll
  for (int t = 0; t < L / 2; t++) cs.sv_set_slot(q, t, sel(sp.h, v[2 * t + 1], v[2 * t + 2]));
}

template <class CS>
H9K_HD void set_lay_d(const CS &cs, int p, int i, double v) {
  cs.set_lay(p, i, lo_d(v));
  cs.set_lay(p + 1, i, hi_d(v));
}
template <class CS>
H9K_HD double lay_d(const CS &cs, int p, int i) { return join_d(cs.lay(p, i), cs.lay(p + 1, i)); }

// x / d, from a stored double reciprocal of d when Use (MathFast::div,
// exact for normal quotients; MathExact divides), else divided.
template <bool Use, class M, class R>
H9K_HD float divr(M &m, float x, float d, R rget) {
  if constexpr (Use)
    return m.div(x, d, rget());
  else
    return x / d;
}

// divr with the check deferred (MathFast::div_d): bad |= the quotient
// needs the IEEE redo, done by divr_fix after the group.
template <bool Use, class M, class R>
H9K_HD float divr_d(M &m, float x, float d, R rget, bool &bad) {
  if constexpr (Use) {
    const float q = m.div_d(x, d, rget());
    bad |= m.div_bad(q);
    return q;
  } else {
    return x / d;
  }
}
template <bool Use, class M>
H9K_HD void divr_fix(M &m, float &q, float x, float d) {
  if constexpr (Use) m.div_fix(q, x, d);
}

// expf on glibc's main path, flagged (sp) when glibc takes another path
// (then M::expf recomputes); MathExact computes it exactly, never flagged.
template <class M>
H9K_HD float expf_fast(M &m, float x, bool &sp) {
  if constexpr (M::kExact)
    return m.expf(x);
  else
    return h9m::expf_nx(x, m.T, sp);
}

// Runs visit(k) for k = 0, 1, ... while it returns true (the reference's
// layer loops with EXIT).  The fast path (MathFast) unrolls two visits --
// the second only if some lane needs it -- and hands a third to the exact
// re-run; loops visit one layer 99.5% of the time and never three in the
// synthetic runs.  MathExact loops.
template <class M, class F>
H9K_HD void visit_layers(M &m, F visit) {
  if constexpr (M::kExact) {
    for (int k = 0;; k++)
      if (!visit(k)) break;
  } else {
    bool more = visit(0);
    if (any_lane(more)) {
      H9G_BR(BR_VISIT2);
      if (more) more = visit(1);
      m.special |= more;
    }
  }
}

// Runtime-indexable geometry table (zt_size(L) floats): zi(0..L+1), then
// zi(0..L+1)/1000 (the reference's zi(I)/1000.0, e.g. HYDROLOGY.f90:
// 499-508,998), then RN64(1/dz(I)) for I = 0..L+1 as (low, high) words
// (I = 0 unused).  A lane reads its own layers' values at a runtime index
// instead of keeping compile-time selects live in registers.
template <int L>
constexpr int zt_size() { return 4 * (L + 2); }
template <int L, class G, class T>
H9K_HD void fill_zt(const G &g, T *zt) {
#pragma unroll
  for (int i = 0; i <= L + 1; i++) {
    zt[i] = g.zi(i);
    zt[L + 2 + i] = g.zi(i) / 1000.0f;
    const double r = (i > 0 && i <= L) ? g.rdz(i) : 0.0;
    zt[2 * (L + 2) + 2 * i] = lo_d(r);
    zt[2 * (L + 2) + 2 * i + 1] = hi_d(r);
  }
}

// Parameter-only invariants (as cell_inv), into a pair/flat store.
template <int L, class G, class CS>
H9K_HD void cell_inv_pair(const G &g, const CS &cs) {
#pragma unroll
  for (int i = 1; i <= L; i++) {
    const int ip = (L < i + 1) ? L : i + 1;
    const float ts = cs.lay(PF_TS, i), tsp = cs.lay(PF_TS, ip);
    const float bsw = cs.lay(PF_BSW, i), psi = cs.lay(PF_PSI, i);
    const float e = one - one / bsw;
    cs.set_lay(PF_NINVB, i, -one / bsw);
    cs.set_lay(PF_ITS, i, one / (ts + tsp));
    const float pte = psi * ts / e;
    cs.set_lay(PF_PTE, i, pte);
    cs.set_lay(PF_C3, i, pte / (g.zi(i) - g.zi(i - 1)));
    if constexpr (CS::kRecip) set_lay_d(cs, PF_RPSI0, i, recip64(-psi));
    if constexpr (CS::kRts) set_lay_d(cs, PF_RTS0, i, recip64(ts));
  }
  float mh = cs.lay(PF_HKS, 1);
  if (cs.lay(PF_HKS, 2) < mh) mh = cs.lay(PF_HKS, 2);
  if (cs.lay(PF_HKS, 3) < mh) mh = cs.lay(PF_HKS, 3);
  cs.set_sc(PS_MH3, mh);
  cs.set_sc(PS_TSDZ1, MAXF(zero, (cs.lay(PF_TS, 1) * g.dz(1))));
}

// One HYDROLOGY call (/root/reference/SOURCE/HYDROLOGY.f90:141-1283) for
// one cell; every block cites the reference lines it restates.  Returns 0
// or an H9G_ERR_* code (the reference's STOP sites) with errval set;
// Under
// Split2 the per-layer phases are split over the pair (file comment).
// The end-of-step theta(1..L) of :1233 is left to the caller (end_theta).
template <int L, class G, class M, class SP, class CS, class PR = NoProf>
H9K_HD int hydrology_pair(const G &g, CS cs, const SP &sp0, St<L> &s, float &rnf_sum, float &errval,
                          M &m, PR &pr) {
  constexpr int NT = L / 2;
  // At L = 10 the lane parity is made opaque here, so that values that
  // depend only on it -- a lane's geometry-table offsets of its own layers,
  // one per slot -- are recomputed inside the substep (an add each) instead
  // of hoisted out of the year loop, spilled to scratch and reloaded behind
  // a vmcnt(0) in every slot (round 4: scratch ops in the L = 10 substep
  // loop 11.2 -> 6.7 per wave-substep, tools/isa_mix.py; at L = 8 nothing
  // is hoisted that way and the change would only add VALU).
  const SP sp = L >= 10 ? sp0.fresh() : sp0;
  const float dt = g.dt();
  constexpr double r1000 = 1.0 / 1000.0;
  float zim[L + 1];
#pragma unroll
  for (int i = 1; i <= L; i++) zim[i] = g.zim(i);
  float *h2o = s.h2o, *smp = s.smp;
  float theta[L + 1];
  cs.launder();
#define TS(i) cs.lay(PF_TS, i)
#define HKS(i) cs.lay(PF_HKS, i)
#define BSW(i) cs.lay(PF_BSW, i)
#define PSI(i) cs.lay(PF_PSI, i)
#define LAYF(F, i) cs.lay(F, i)
#define ROOT(i) cs.lay(PF_ROOTR, i)
#define DC(F) cs.sc(PS_DAY + F)
#define OWN(p) sp.own(cs, p, t, h)

  // :141-151
  float w0 = DC(D_FORC) * dt + s.wa;
  bool bad = false;                      // deferred checks (MathFast::div_d)
#pragma unroll
  for (int i = 1; i <= L; i++) {
    w0 = w0 + h2o[i];
    theta[i] = m.div_d(h2o[i], g.thk(i), g.rthk(i));
    bad |= m.div_bad(theta[i]);
  }
  if (__builtin_expect(bad, 0)) {
    H9G_BR(BR_THETA);
#pragma unroll
    for (int i = 1; i <= L; i++) m.div_fix(theta[i], h2o[i], g.thk(i));
  }
  // :161-212
  const float qflx_top_soil = DC(D_FORC);
  const float hkdepth = one / 2.5f;
  const float fff = 1.0f / hkdepth;
  const float fsat = cs.sc(PS_FMAX) * m.expf(-0.5f * fff * s.zwt);
  float qflx_surf = fsat * qflx_top_soil;
  const float frac_h2osfc = zero;
  // :269-276 (previous-step smp)
  float beta = zero;
  {
    // the terms rootr(i) * beta_i of the lane's own layers (the pair split:
    // round 3, 199.3 -> 197.3 ms), then the reference's sum over the layers
    // in order
    float rb[L + 1];
    float *const out[1] = {rb};
    auto qb_x = [&](int t, int h) __attribute__((always_inline)) {
      return sel(h, smp[2 * t + 1] - g.zc(2 * t + 1), smp[2 * t + 2] - g.zc(2 * t + 2));
    };
    auto term = [&](int t, int h, float q) __attribute__((always_inline)) {
      float b = one - q;
      b = MINC(one, b);
      b = MAXF(zero, b);
      return FV<1>{{sp.own(cs, PF_ROOTR, t, h) * b}};
    };
    sp.template par_d<NT, 1, NT>(
        [&](int t, int h, bool &bad) __attribute__((always_inline)) -> FV<1> {
          const float q = m.div_d(qb_x(t, h), -150000.0f, 1.0 / -150000.0);
          bad |= m.div_bad(q);
          return term(t, h, q);
        },
        [&](int t, int h) __attribute__((always_inline)) -> FV<1> {
          H9G_BR(BR_QB);
          return term(t, h, m.div(qb_x(t, h), -150000.0f, 1.0 / -150000.0));
        },
        out);
#pragma unroll
    for (int i = 1; i <= L; i++) beta = beta + rb[i];
  }
  // :325-331
  float rss;
  if (theta[1] <= 0.15f)
    rss = (10.0f + DC(D_LIT1000)) * m.expf(0.3563f * 100.0f * (0.15f - theta[1]));
  else
    rss = (10.0f + DC(D_LIT1000) * (1.0f - divr<CS::kRts>(m, theta[1], TS(1), [&]() { return lay_d(cs, PF_RTS0, 1); })));
  const float desatdT = DC(D_DESAT), gamma = DC(D_GAMMA);
  const float Ra = DC(D_DG) * DC(D_RAA);
  float rsc, tran, evg;
  bool eb_fast = false;
  if constexpr (H9G_EB_FAST && !M::kExact && (CS::kDayRecip || H9G_EB_FAST >= 2)) {
    // The energy balance's chain of quotients (:283-389) branch-free: the
    // day constants' by their stored double reciprocals (MathFast::div_d),
    // the runtime divisors by mk_div (Markstein's correction of the refined
    // v_rcp_f32 reciprocal, range-flagged).  Any flag on any lane of the
    // wave re-runs the block below exactly (wave-uniform: the pair exchanges
    // values).
    bool bad = false;
    auto mdiv = [&](float x, float d) __attribute__((always_inline)) { return mk_div(x, d, bad); };
    auto ddiv = [&](float x, float d, auto rget) __attribute__((always_inline)) {
      if constexpr (CS::kDayRecip) {   // the store has the day constants' double reciprocals
        const float q = m.div_d(x, d, rget());
        bad |= m.div_bad(q);
        return q;
      } else {
        return mdiv(x, d);
      }
    };
    // :283-295
    const bool open = (DC(D_OK) != zero) && (beta > zero);
    bool bo = bad;
    const float q_rsc = mdiv(DC(D_X), DC(D_LAI2) * beta * DC(D_PW28));
    bad = bo | (open && bad);
    float rscf = open ? q_rsc : 1.0E6f;
    rscf = MAXF(rscf, DC(D_RSCMIN));
    // :344-389
    FV<2> c2, s2;
    sp.template pick<2>(
        [&](int h) __attribute__((always_inline)) -> FV<2> {
          const float r = sel(h, rscf, rss);
          const float q = ddiv(r, sp.own_sc(cs, PS_DAY + D_RAARAC, h), [&]() { return sp.own_day_rp(cs, DRP_RAARA, h); });
          const float PM = mdiv(sp.own_sc(cs, PS_DAY + D_NUMC, h), desatdT + gamma * (one + q));
          const float R = sp.own_sc(cs, PS_DAY + D_DGRAC, h) + gamma * r;
          return FV<2>{{PM, R}};
        },
        c2, s2);
    FV<1> cc, cs1;
    sp.template pick<1>(
        [&](int h) __attribute__((always_inline)) -> FV<1> {
          const float Rh = sel(h, c2.v[1], s2.v[1]), Ro = sel(h, s2.v[1], c2.v[1]);
          return FV<1>{{mdiv(one, one + mdiv(Rh * Ra, Ro * (Rh + Ra)))}};
        },
        cc, cs1);
    const float LEf = cc.v[0] * c2.v[0] + cs1.v[0] * s2.v[0];
    const float VDD0f = DC(D_VDD) + ddiv((DC(D_A1) - DC(D_DG) * LEf) * DC(D_RAA), DC(D_RHOCP),
                                              [&]() { return cs.day_r(DR_RHOCP); });
    FV<1> ft, fe;
    sp.template pick<1>(
        [&](int h) __attribute__((always_inline)) -> FV<1> {
          const float r = sel(h, rscf, rss);
          const float d = sp.own_sc(cs, PS_DAY + D_RAC, h);
          auto rr = [&]() __attribute__((always_inline)) { return sp.own_day_rp(cs, DRP_RA, h); };
          const float LEh = mdiv(sp.own_sc(cs, PS_DAY + D_DRR, h) + ddiv(DC(D_RHOCP) * VDD0f, d, rr),
                                 desatdT + gamma * (1.0f + ddiv(r, d, rr)));
          return FV<1>{{ddiv(LEh * 1.0E3f, DC(D_RL), [&]() { return cs.day_r(DR_RL); })}};
        },
        ft, fe);
#if defined(H9G_FORCE_RERUN)   // test builds: the exact block in about one wave-substep of two
    bad |= (__builtin_bit_cast(uint32_t, theta[1]) & 15u) == 0;
#endif
    if (!__builtin_expect(any_lane(bad), 0)) {
      rsc = rscf;
      tran = ft.v[0];
      evg = fe.v[0];
      eb_fast = true;
    }
  }
  if (!eb_fast) {
  H9G_BR(BR_EBX);
  // :283-295
  if ((DC(D_OK) != zero) && (beta > zero))
    rsc = DC(D_X) / (DC(D_LAI2) * beta * DC(D_PW28));
  else
    rsc = 1.0E6f;
  rsc = MAXF(rsc, DC(D_RSCMIN));
  // :344-389.  The canopy (h = 0) and soil (h = 1) halves have the same
  // expressions on different operands: each lane of a pair evaluates one
  // (pick), reading its operands from its own column (D_NUMC comment).
  FV<2> ebc, ebs;                                       // {PM, R}: canopy, soil
  sp.template pick<2>(
      [&](int h) __attribute__((always_inline)) -> FV<2> {
        const float r = sel(h, rsc, rss);
        const float q = divr<CS::kDayRecip>(m, r, sp.own_sc(cs, PS_DAY + D_RAARAC, h),
                                            [&]() { return sp.own_day_rp(cs, DRP_RAARA, h); });
        const float PM = sp.own_sc(cs, PS_DAY + D_NUMC, h) / (desatdT + gamma * (one + q));
        const float R = sp.own_sc(cs, PS_DAY + D_DGRAC, h) + gamma * r;
        return FV<2>{{PM, R}};
      },
      ebc, ebs);
  const float PMc = ebc.v[0], Rc = ebc.v[1], PMs = ebs.v[0], Rs = ebs.v[1];
  FV<1> ccf, csf;                                       // Cc, Cs
  sp.template pick<1>(
      [&](int h) __attribute__((always_inline)) -> FV<1> {
        const float Rh = sel(h, Rc, Rs), Ro = sel(h, Rs, Rc);
        return FV<1>{{one / (one + Rh * Ra / (Ro * (Rh + Ra)))}};
      },
      ccf, csf);
  const float LE = ccf.v[0] * PMc + csf.v[0] * PMs;
  const float VDD0 = DC(D_VDD) + divr<CS::kDayRecip>(m, (DC(D_A1) - DC(D_DG) * LE) * DC(D_RAA), DC(D_RHOCP),
                                                     [&]() { return cs.day_r(DR_RHOCP); });
  FV<1> ftr, fev;                                       // tran, evg
  sp.template pick<1>(
      [&](int h) __attribute__((always_inline)) -> FV<1> {
        const float r = sel(h, rsc, rss);
        const float d = sp.own_sc(cs, PS_DAY + D_RAC, h);
        auto rr = [&]() __attribute__((always_inline)) { return sp.own_day_rp(cs, DRP_RA, h); };
        const float LEh = (sp.own_sc(cs, PS_DAY + D_DRR, h) + divr<CS::kDayRecip>(m, DC(D_RHOCP) * VDD0, d, rr)) /
                          (desatdT + gamma * (1.0f + divr<CS::kDayRecip>(m, r, d, rr)));
        return FV<1>{{divr<CS::kDayRecip>(m, LEh * 1.0E3f, DC(D_RL), [&]() { return cs.day_r(DR_RL); })}};
      },
      ftr, fev);
  tran = ftr.v[0];
  evg = fev.v[0];
  }
  // :396-400
  float em1 = m.div(g.dz(1) * (theta[1] - watmin), dt, g.rdt()) - tran * ROOT(1);
  em1 = MAXF(zero, em1);
  evg = MINF(em1, evg);
  pr.flux(evg, tran);
  // :426-478
  const float qflx_evap = evg;
  float qflx_in_soil = (one - frac_h2osfc) * (qflx_top_soil - qflx_surf);
  qflx_in_soil = qflx_in_soil - (one - frac_h2osfc) * qflx_evap;
  const float qinmax = (one - fsat) * cs.sc(PS_MH3);
  const float qflx_infl_excess = MAXF(zero, qflx_in_soil - (one - frac_h2osfc) * qinmax);
  const float qflx_infl = qflx_in_soil - qflx_infl_excess;
  qflx_surf = qflx_surf + qflx_infl_excess;
  // :492-508
  float zwtmm = 1000.0f * s.zwt;
  const int jwt = jwt_of<L>(s.zwt, zim);
  const bool aq = (jwt == L);
  cs.launder();
  pr.mark(1);

  // :517-567 equilibrium profile and :598-639 conductivity and matric
  // potential, own layers (independent phases)
  float zq[L + 2];
  float hk[L + 1], dhkdw[L + 1], dsmpdw[L + 1];
  {
    float *const outq[1] = {zq};
    float *const outk[4] = {hk, dhkdw, smp, dsmpdw};
    // exact: the reference expression with every special case redone in place
    auto eq_exact = [&](int t, int h) __attribute__((always_inline)) -> FV<1> {
          H9G_BR(BR_EQX);
          const int i0 = 2 * t + 1;                           // own layer il = i0 + h
          const int il = i0 + h;
          const float zlo = cs.zi(il - 1), zhi = cs.zi(il);   // zi(i-1), zi(i): geometry table
          const float ts = OWN(PF_TS), psi = OWN(PF_PSI);
          float vol_eq;
          if (zwtmm <= zlo) {
            vol_eq = ts;
          } else {
            const float expo = one + OWN(PF_NINVB);
            auto rp = [&]() __attribute__((always_inline)) {
              return join_d(OWN(PF_RPSI0), OWN(PF_RPSI1));
            };
            // temp0 and (below the layer) tempi are independent powers:
            // both bases, then both powers, each pair checked once.  With the
            // water table inside the layer tempi is not evaluated (its base
            // is replaced by 1, whose power is exactly 1 and never special).
            const bool inl = (zwtmm < zhi) && (zwtmm > zlo);
            const float n0 = ((-psi) + zwtmm - zlo), ni = (-psi + zwtmm - zhi);
            bool bq = false;
            float b0 = divr_d<CS::kRecip>(m, n0, -psi, rp, bq);
            float bi = divr_d<CS::kRecip>(m, ni, -psi, rp, bq);
            if (__builtin_expect(bq, 0)) {
              divr_fix<CS::kRecip>(m, b0, n0, -psi);
              divr_fix<CS::kRecip>(m, bi, ni, -psi);
            }
            bi = inl ? one : bi;
            bool s0, si;
            float temp0 = m.powf_d(b0, expo, s0);
            float tpi = m.powf_d(bi, expo, si);
            if (__builtin_expect(s0 | si, 0)) {
              m.powf_fix(temp0, b0, expo, s0);
              m.powf_fix(tpi, bi, expo, si);
            }
            if (inl) {
              const float tempi = one;
              const float voleq1 = OWN(PF_PTE) / (zwtmm - zlo) * (tempi - temp0);
              vol_eq = m.div(voleq1 * (zwtmm - zlo) + ts * (zhi - zwtmm), zhi - zlo, cs.rdz_t(il));   // dz(i)
              vol_eq = MINF(ts, vol_eq);
              vol_eq = MAXF(vol_eq, zero);
            } else {
              const float tempi = tpi;
              vol_eq = OWN(PF_C3) * (tempi - temp0);
              vol_eq = MAXF(vol_eq, 0.0f);
              vol_eq = MINF(ts, vol_eq);
            }
          }
          const float qv = divr<CS::kRts>(m, vol_eq, ts, [&]() { return join_d(OWN(PF_RTS0), OWN(PF_RTS1)); });
          float z = psi * m.powf(MAXX(qv, 0.01f), -OWN(PF_BSW));
          return FV<1>{{MAXC(smpmin, z)}};
    };
    // fast: the same values branch-free (all three cases evaluated, the
    // layer's selected); bad = some quotient or power of the selected case
    // needs its other path (then eq_exact recomputes the slot).  Bases of
    // cases not taken are replaced by 1 so they raise no flag.  eq_body is
    // the slot of layer il, with O(p) the slot's value of field p and zw the
    // water table (mm): a lane's own slot (eq_fast) or, on a spare lane,
    // another pair's last slot (below).
    // inl_all: evaluate the in-layer case for every lane, branch-free (the
    // round where the pairs evaluate their last slot, H9G_INL_LAST)
    auto eq_body = [&](int il, auto O, float zw, bool &bad, bool inl_all) __attribute__((always_inline)) -> FV<1> {
          const float zlo = cs.zi(il - 1), zhi = cs.zi(il);
          const float ts = O(PF_TS), psi = O(PF_PSI);
          const bool sat = zw <= zlo;
          const bool inl = (zw < zhi) && (zw > zlo);
          const float expo = one + O(PF_NINVB);
          auto rp = [&]() __attribute__((always_inline)) { return join_d(O(PF_RPSI0), O(PF_RPSI1)); };
          const float n0 = ((-psi) + zw - zlo), ni = (-psi + zw - zhi);
          float b0 = divr_d<CS::kRecip>(m, n0, -psi, rp, bad);
          float bi = divr_d<CS::kRecip>(m, ni, -psi, rp, bad);
          b0 = sat ? one : b0;
          bi = (sat || inl) ? one : bi;
          bool s0, si;
          const float temp0 = m.powf_d(b0, expo, s0);
          const float tpi = m.powf_d(bi, expo, si);
          bad |= s0 | si;
          // water table inside the layer (:530-543): at most one layer of a
          // column, so evaluated only in a slot where some lane of the wave
          // has it (a wave-uniform branch)
          float vin = zero;
          if (inl_all || any_lane(inl)) {
          H9G_BR(BR_INL);
          const float d0 = zw - zlo;
#if H9G_INL_MDIV
          bool bq = false;
          const float q1 = mk_div(O(PF_PTE), d0, bq);
#else
          const float q1 = m.div_d(O(PF_PTE), d0, recip64(d0));
          const bool bq = m.div_bad(q1);
#endif
          const float voleq1 = q1 * (one - temp0);
          vin = m.div_d(voleq1 * (zw - zlo) + ts * (zhi - zw), zhi - zlo, cs.rdz_t(il));
          bad |= inl && (bq | m.div_bad(vin));
          vin = MINF(ts, vin);
          vin = MAXF(vin, zero);
          }
          // water table below the layer (:548-558)
          float vbl = O(PF_C3) * (tpi - temp0);
          vbl = MAXF(vbl, 0.0f);
          vbl = MINF(ts, vbl);
          const float vol_eq = sat ? ts : (inl ? vin : vbl);
          const float qv = divr_d<CS::kRts>(m, vol_eq, ts, [&]() { return join_d(O(PF_RTS0), O(PF_RTS1)); }, bad);
          bool sz;
          const float z = psi * m.powf_d(MAXX(qv, 0.01f), -O(PF_BSW), sz);
          bad |= sz;
          return FV<1>{{MAXC(smpmin, z)}};
    };
    auto eq_fast = [&](int t, int h, bool &bad) __attribute__((always_inline)) -> FV<1> {
          return eq_body(2 * t + 1 + h, [&](int p) __attribute__((always_inline)) { return OWN(p); }, zwtmm, bad,
                         false);
    };
    auto hk_exact = [&](int t, int h) __attribute__((always_inline)) -> FV<4> {
          H9G_BR(BR_HKX);
          const int i0 = 2 * t + 1;
          const int ip1 = (L < i0 + 2) ? L : i0 + 2;          // ip of layer i0+1
          const float th = sel(h, theta[i0], theta[i0 + 1]);
          const float thp = sel(h, theta[i0 + 1], theta[ip1]);
          const float ts = OWN(PF_TS);
          const float tsp = sel(h, TS(i0 + 1), TS(ip1));
          float s1 = 0.5f * (th + thp) / (0.5f * (ts + tsp));
          s1 = MINC(one, s1);
          const float bsw = OWN(PF_BSW);
          float s_node = MAXX(divr<CS::kRtsHK>(m, th, ts, [&]() { return join_d(OWN(PF_RTS0), OWN(PF_RTS1)); }),
                              0.01f);
          s_node = MINC(one, s_node);
          // the two powers are independent: one deferred check
          const float ek = 2.0f * bsw + 2.0f, es = -bsw;
          bool sk, ss;
          float pk = m.powf_d(s1, ek, sk);
          float ps = m.powf_d(s_node, es, ss);
          if (__builtin_expect(sk | ss, 0)) {
            m.powf_fix(pk, s1, ek, sk);
            m.powf_fix(ps, s_node, es, ss);
          }
          const float s2 = OWN(PF_HKS) * pk;
          FV<4> r;
          r.v[0] = s1 * s2;
          r.v[1] = (2.0f * bsw + 3.0f) * s2 * OWN(PF_ITS);
          float sm = OWN(PF_PSI) * ps;
          sm = MAXC(smpmin, sm);
          r.v[2] = sm;
          r.v[3] = (-bsw) * sm / (s_node * ts);
          return r;
    };
    // the same, branch-free, flags deferred (par_d); hk_body as eq_body, with
    // the slot's operands theta(i), theta(ip), theta_s(ip) (ip = i + 1, at
    // most L) given
    auto hk_body = [&](auto O, float th, float thp, float tsp, bool &bad) __attribute__((always_inline)) -> FV<4> {
          const float ts = O(PF_TS);
          // s1 = RN(0.5a / 0.5b) = RN(a / b) (the halvings are exact for
          // normal a, b), from y = PF_ITS = RN(1/b) by Markstein's correction:
          // q0 = RN(a y), e = a - b q0 (exact), RN(q0 + e y) = RN(a / b) when
          // nothing under- or overflows.  a, b in [2^-60, 2^60) keeps q and e
          // normal; other operands flag the slot for hk_exact.  (The IEEE
          // division took 11 VALU in a chain of 9; tools/markstein_check.c.)
          const float sa = th + thp, sb = ts + tsp, its = O(PF_ITS);
          const float q0 = sa * its;
          float s1 = __builtin_fmaf(__builtin_fmaf(-sb, q0, sa), its, q0);
          const uint32_t ua = __builtin_bit_cast(uint32_t, sa) - 0x21800000u;   // 2^-60
          const uint32_t ub = __builtin_bit_cast(uint32_t, sb) - 0x21800000u;
          bad |= (ua > ub ? ua : ub) >= 0x5d800000u - 0x21800000u;             // 2^60
          s1 = MINC(one, s1);
          const float bsw = O(PF_BSW);
          float s_node = MAXX(divr_d<CS::kRtsHK>(m, th, ts, [&]() { return join_d(O(PF_RTS0), O(PF_RTS1)); }, bad),
                              0.01f);
          s_node = MINC(one, s_node);
          const float ek = 2.0f * bsw + 2.0f, es = -bsw;
          bool sk, ss;
          const float pk = m.powf_d(s1, ek, sk);
          const float ps = m.powf_d(s_node, es, ss);
          bad |= sk | ss;
          const float s2 = O(PF_HKS) * pk;
          FV<4> r;
          r.v[0] = s1 * s2;
          r.v[1] = (2.0f * bsw + 3.0f) * s2 * O(PF_ITS);
          float sm = O(PF_PSI) * ps;
          sm = MAXC(smpmin, sm);
          r.v[2] = sm;
          if constexpr (H9G_HK_MDIV && L <= 8)
            r.v[3] = mk_div((-bsw) * sm, s_node * ts, bad);   // dsmpdw, flagged for hk_exact
          else
            r.v[3] = (-bsw) * sm / (s_node * ts);
          return r;
    };
    auto hk_fast = [&](int t, int h, bool &bad) __attribute__((always_inline)) -> FV<4> {
          const int i0 = 2 * t + 1;
          const int ip1 = (L < i0 + 2) ? L : i0 + 2;
          return hk_body([&](int p) __attribute__((always_inline)) { return OWN(p); }, sel(h, theta[i0], theta[i0 + 1]),
                         sel(h, theta[i0 + 1], theta[ip1]), sel(h, TS(i0 + 1), TS(ip1)), bad);
    };
    if constexpr (SP::kSpare && CS::kSpare && !M::kExact) {
      // Helper lanes (round 4: "spare lanes"; round 5: any number of slots).
      // A wave's C pairs use S = 2C of its 64 lanes; the other H = 64 - S
      // lanes help in these two phases.  The phases take R = ceil(NT S / 64)
      // rounds instead of NT: in round q every pair lane evaluates its own
      // slot U + q (U = NT - R), and the helpers evaluate the first U slots of
      // all pair lanes, task tau = u S + k (slot u of pair lane k) on helper
      // S + tau % H in round tau / H, with k's operands by ds_bpermute
      // (fetched before the rounds) and its parameters from k's LDS column.
      // After the rounds pair lane k takes each helper result, and the flags
      // of that evaluation, from its helper.  The same expressions on the
      // same operands: no bit changes.  A flag on either side re-runs the
      // pair lane's slots exactly, as in par_d.
      //   L = 8,  C = 22: R = 3, U = 1 (round 4's spare lanes: NT - 1 rounds)
      //   L = 10, C = 11: R = 2, U = 3 (h9g_pair11_kernel, small L = 10 shards)
      // The helpers take the FIRST U slots (round 5): the water table lies in
      // layers L-1 or L in most columns, and the equilibrium profile's
      // in-layer case (a wave-uniform branch of ~20 VALU on the round's
      // critical path, :530-543) then runs in the one round where the pairs
      // evaluate their last slot, not in every round that holds a helper's
      // last slot of some pair (branch counts: 1.77 of 3 rounds with the
      // helpers on the last slot; config 2: 186.5 -> 183.7 ms).
      constexpr int S = CS::LANES, H = 64 - S;
      constexpr int R = (NT * S + 63) / 64, U = NT - R, TOT = U * S;
      static_assert(U >= 1 && TOT <= R * H, "the helpers cover the first U slots in R rounds");
      const bool st = sp.spare;
      const int hh = sp.h;
      // helper: its task in round q (idle helpers repeat the last task)
      auto tau_q = [&](int q) __attribute__((always_inline)) {
        const int t = q * H + (st ? sp.ln - S : 0);
        return t < TOT ? t : TOT - 1;
      };
      // pair lane: the helper lane of its slot u, and the round it ran in
      auto src_u = [&](int u) __attribute__((always_inline)) { return S + (u * S + sp.ln) % H; };
      auto qo_u = [&](int u) __attribute__((always_inline)) { return (u * S + sp.ln) / H; };
      // rounds that hold tasks of slot u, and slots that round q holds
      auto qlo = [](int u) constexpr { return (u * S) / H; };
      auto qhi = [](int u) constexpr { return ((u * S + S - 1) / H) < R - 1 ? (u * S + S - 1) / H : R - 1; };
      auto ulo = [](int q) constexpr { return (q * H) / S < U - 1 ? (q * H) / S : U - 1; };
      auto uhi = [](int q) constexpr { return (q * H + H - 1) / S < U - 1 ? (q * H + H - 1) / S : U - 1; };
      // a helper result of every round -> pair lane's slot u.  A ds_bpermute
      // must run in converged control flow: a lane reads only what active
      // lanes provide (a helpers-only fetch under `st ?` read zeros).
      auto back = [&](const float (&v)[R], int u) __attribute__((always_inline)) {
        const int src = src_u(u), qo = qo_u(u);
        float x = lane_get(v[qlo(u)], src);
#pragma unroll
        for (int q = qlo(u) + 1; q <= qhi(u); q++) {
          const float g = lane_get(v[q], src);
          x = qo == q ? g : x;
        }
        return x;
      };
      auto flags_back = [&](int fl) __attribute__((always_inline)) {
        bool any = false;
#pragma unroll
        for (int u = 0; u < U; u++) any |= ((lane_geti(fl, src_u(u)) >> qo_u(u)) & 1) != 0;
        return any;
      };
      {
        float zwk[R];
#pragma unroll
        for (int q = 0; q < R; q++) zwk[q] = lane_get(zwtmm, tau_q(q) % S);
        FV<1> r[NT];
        float rv[R];
        int fl = 0;
#pragma unroll
        for (int q = 0; q < R; q++) {
          const int tau = tau_q(q), k = tau % S, u = tau / S;
          const int t = U + q;
          const lds_float *o = st ? cs.wb + k + u * S : cs.self + t * S;
          bool b = false;
          r[t] = eq_body(st ? 2 * u + 1 + (k & 1) : 2 * t + 1 + hh,
                         [&](int p) __attribute__((always_inline)) { return o[p * NT * S]; },
                         st ? zwk[q] : zwtmm, b, H9G_INL_LAST && U + q == NT - 1);
          rv[q] = r[t].v[0];
          fl |= (b ? 1 : 0) << q;
          if ((H9G_SPARE_FENCE >> q) & 1) sched_fence();
        }
#pragma unroll
        for (int u = 0; u < U; u++) r[u].v[0] = back(rv, u);
        const bool bad = !st & ((fl != 0) | flags_back(fl));
        if (__builtin_expect(bad, 0)) {
#pragma unroll
          for (int t = 0; t < NT; t++) r[t] = eq_exact(t, hh);
        }
#pragma unroll
        for (int t = 0; t < NT; t++) sp.xchg(r[t].v[0], zq[2 * t + 1], zq[2 * t + 2]);
      }
      pr.mark(2);
      {
        // this lane's operands of its helper slots u (theta(i), theta(ip),
        // ip = i + 1 <= L as u <= NT - 2), and each helper's of its tasks
        float thu[U], thpu[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
          thu[u] = sel(hh, theta[2 * u + 1], theta[2 * u + 2]);
          thpu[u] = sel(hh, theta[2 * u + 2], theta[2 * u + 3]);
        }
        float thk[R], thpk[R];
#pragma unroll
        for (int q = 0; q < R; q++) {
          const int tau = tau_q(q), k = tau % S, u = tau / S;
          float a = lane_get(thu[ulo(q)], k), b = lane_get(thpu[ulo(q)], k);
#pragma unroll
          for (int w = ulo(q) + 1; w <= uhi(q); w++) {
            const float ga = lane_get(thu[w], k), gb = lane_get(thpu[w], k);
            a = u == w ? ga : a;
            b = u == w ? gb : b;
          }
          thk[q] = a;
          thpk[q] = b;
        }
        const lds_float *pe = cs.even + PF_TS * NT * S + (hh ? S : 1);           // TS(i + 1), TS(ip) of own slots
        FV<4> r[NT];
        float rv[4][R];
        int fl = 0;
#pragma unroll
        for (int q = 0; q < R; q++) {
          const int tau = tau_q(q), k = tau % S, u = tau / S;
          const int t = U + q;
          const lds_float *o = st ? cs.wb + k + u * S : cs.self + t * S;
          // TS(ip) of the slot: layer 2t+2 (odd column, row t) for the even
          // lane, 2t+3 (even column, row t+1) for the odd one; TS(L) (odd
          // column, row NT-1) in the last slot
          const lds_float *pt_h = cs.wb + ((k & 1) ? (k & ~1) + S : (k | 1)) + (PF_TS * NT + u) * S;
          const lds_float *pt_own = t == NT - 1 ? cs.even + 1 + (PF_TS * NT + NT - 1) * S : pe + t * S;
          const lds_float *pt = st ? pt_h : pt_own;
          bool b = false;
          r[t] = hk_body([&](int p) __attribute__((always_inline)) { return o[p * NT * S]; },
                         st ? thk[q] : sel(hh, theta[2 * t + 1], theta[2 * t + 2]),
                         st ? thpk[q] : sel(hh, theta[2 * t + 2], theta[2 * t + 3 <= L ? 2 * t + 3 : L]), *pt, b);
#pragma unroll
          for (int kk = 0; kk < 4; kk++) rv[kk][q] = r[t].v[kk];
          fl |= (b ? 1 : 0) << q;
          if ((H9G_SPARE_FENCE >> q) & 1) sched_fence();
        }
#pragma unroll
        for (int kk = 0; kk < 4; kk++)
#pragma unroll
          for (int u = 0; u < U; u++) r[u].v[kk] = back(rv[kk], u);
        const bool bad = !st & ((fl != 0) | flags_back(fl));
        if (__builtin_expect(bad, 0)) {
#pragma unroll
          for (int t = 0; t < NT; t++) r[t] = hk_exact(t, hh);
        }
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
          for (int kk = 0; kk < 4; kk++) sp.xchg(r[t].v[kk], outk[kk][2 * t + 1], outk[kk][2 * t + 2]);
      }
    } else {
      // (round 3: the two phases' slots interleaved in one region, twice the
      // independent powers per region, spilled 225 VGPRs: 214.5 vs 208.9 ms)
      sp.template par_d<NT, 1, CS::FE_EQ>(eq_fast, eq_exact, outq);
      pr.mark(2);
      sp.template par_d<NT, 4, CS::FE_HK>(hk_fast, hk_exact, outk);
    }
  }
  if constexpr (SP::kSpare) {
    if (!sp.act()) return 0;             // spare lanes: only the per-layer phases above
  }
  // First round of single powers, one per lane, chosen by where the lane's
  // water table is (jwt = L: below the column), with the lane's operands:
  //   below:  lane 0 temp0 of the aquifer node (:579-580), lane 1 the
  //           specific-yield power of layer L at this zwtmm (:937-940);
  //   inside: lane 0 the recharge conductivity's power (:874-877), lane 1
  //           the specific-yield power of layer jwt+1 (:963-981), both of
  //           the recharge section below, which reads only this substep's
  //           starting theta and zwt.
  // A wave holding columns of both kinds evaluates one round here instead of
  // one per kind (round 3).  The second aquifer round (zq(L+1) and smp1 of the
  // aquifer row, :581-590, :737-741) is read only by lanes below the column:
  // a wave with none skips it (wave-uniform); the deepening loop's rare
  // fall-through below the column evaluates s_y(L) itself for a lane inside.
  // (H9G_AQ_FREE: evaluated by every wave; lanes inside the column take
  // operands that make it an identity and raise no flag)
  const bool any_aq = H9G_AQ_FREE || any_lane(aq);
  const int jc = aq ? L : jwt + 1;            // the layer whose -psi divides
  float s1c = one, bsw_c = zero;              // recharge operands of layer jwt+1 (:866-873)
  if (any_lane(!aq)) {
    float th_j = zero;
#pragma unroll
    for (int i = 1; i <= L; i++)
      if (i == jc) th_j = theta[i];
    const float s_node =
        MAXX(divr<CS::kRts>(m, th_j, cs.lay(PF_TS, jc), [&]() { return lay_d(cs, PF_RTS0, jc); }), 0.01f);
    s1c = MINC(one, s_node);
    bsw_c = cs.lay(PF_BSW, jc);
  }
  FV<1> p0, p1;                               // lane 0's and lane 1's power
  sp.template pick<1>(
      [&](int h) __attribute__((always_inline)) -> FV<1> {
        const float npsi = -cs.lay(PF_PSI, jc);
        const float num = (aq && h == 0) ? (-PSI(L) + zwtmm - g.zi(L)) : zwtmm;
        bool sq = false, sw = false;
        float q = divr_d<CS::kRecip>(m, num, npsi, [&]() { return lay_d(cs, PF_RPSI0, jc); }, sq);
        const float ninv = cs.lay(PF_NINVB, jc);
        const float e = h ? ninv : (aq ? one + ninv : 2.0f * bsw_c + 3.0f);
        float w = m.powf_d(h ? one + q : (aq ? q : s1c), e, sw);
        if (__builtin_expect(sq | sw, 0)) {                  // one deferred check
          H9G_BR(BR_RECH);
          divr_fix<CS::kRecip>(m, q, num, npsi);
          w = m.powf(h ? one + q : (aq ? q : s1c), e);
        }
        return FV<1>{{w}};
      },
      p0, p1);
  const FV<1> pA = p0, pY = p1;
  FV<2> eA{{zero, zero}}, eS{{zero, zero}};
  if (any_aq) {
  H9G_BR(BR_ANYAQ);
  {
    const float d0 = aq ? (zwtmm - g.zi(L)) : one;
    float ve = LAYF(PF_PTE, L) / d0 * (1.0f - pA.v[0]);
    ve = MAXF(ve, 0.0f);
    ve = MINF(TS(L), ve);
    sp.template pick<2>(
        [&](int h) __attribute__((always_inline)) -> FV<2> {
          // the quotient's and the power's checks deferred to one branch
          // (round 2's d878d3e, backed out after a GPU fault that the calls
          // of the then out-of-line redo caused: DESIGN.md §3)
          const float xn = sel(h, ve, theta[L]);
          auto xof = [&](float q2) __attribute__((always_inline)) {
            float sn = MAXX(0.5f * (one + q2), 0.01f);
            sn = MINC(one, sn);
            const float x = sel(h, MAXX(q2, 0.01f), sn);
            return aq ? x : one;
          };
          bool sq = false, sw = false;
          float q2 = divr_d<CS::kRts>(m, xn, TS(L), [&]() { return lay_d(cs, PF_RTS0, L); }, sq);
          float x = xof(q2);
          float pw = m.powf_d(x, -BSW(L), sw);
          if (__builtin_expect(sq | sw, 0)) {
            H9G_BR(BR_AQS);
            divr_fix<CS::kRts>(m, q2, xn, TS(L));
            x = xof(q2);
            pw = m.powf(x, -BSW(L));
          }
          float z = PSI(L) * pw;
          z = MAXC(smpmin, z);
          return FV<2>{{z, -BSW(L) * z / (x * TS(L))}};
        },
        eA, eS);
  }
  }  // any_aq
  zq[L + 1] = aq ? eA.v[0] : zero;
  const float smp1 = eS.v[0], dsmpdw1 = eS.v[1];
  cs.launder();
  pr.mark(3);
  // :645-650 aquifer node geometry
  const float zcA = 0.5f * (zwtmm + g.zc(L));
  const float dzA = (jwt < L) ? g.dz(L) : zwtmm - g.zc(L);
  cs.launder();
  // Tridiagonal system rows 1..L+1 (:661-799), each row eliminated as soon
  // as it is assembled (Thomas forward sweep, :806-831).  The flux terms
  // of interface k are the reference's qout/dqodw1/dqodw2 of row k and,
  // bit for bit the same expressions, qin/dqidw0/dqidw1 of row k+1; they
  // are evaluated once.
  float dwat2[L + 2], GAM[L + 2];
  float BET = zero;
  double rbet = 0.0;
  int zero_pivot = 0;
  // Row i also evaluates the next row's GAM(i+1) = c(i) / BET(i) (the
  // reference's :827 of row i+1): it is independent of dwat2(i), so the two
  // quotients share one deferred check.
  auto row = [&](int i, float am, float bm, float cm, float rm) __attribute__((always_inline)) {
    float x;
    if (i == 1) {
      BET = bm;
      x = rm;
    } else {
      BET = bm - am * GAM[i];
      if (BET == 0.0f && !zero_pivot) zero_pivot = i;
      x = rm - am * dwat2[i - 1];
    }
    rbet = recip64(BET);
    dwat2[i] = m.div_d(x, BET, rbet);
    bool bad = m.div_bad(dwat2[i]);
    if (i <= L) {
      GAM[i + 1] = m.div_d(cm, BET, rbet);
      bad |= m.div_bad(GAM[i + 1]);
    }
    if (__builtin_expect(bad, 0)) {
      m.div_fix(dwat2[i], x, BET);
      if (i <= L) m.div_fix(GAM[i + 1], cm, BET);
    }
  };
  // Fast path (MathFast): every interface flux first (branch-free, one
  // deferred check, then the layer arrays die), then the forward sweep,
  // branch-free with its checks deferred to its end.  The two shapes of
  // rows L, L+1 (water table in the column or below it) are one set of
  // expressions with selected operands (a zero operand only where the
  // reference writes one too: x - 0, x + 0).  A flagged quotient, a zero
  // pivot or bm(1) = 0 re-runs the sweep exactly on the (exact) fluxes,
  // raising the reference's STOPs.  Measured: 234.3 -> 230.1 ms (config 2);
  // keeping the layer arrays live for a whole-block redo instead spilled
  // 55 VGPRs and measured 238.9 ms.
  bool tri_ok = false;
  if constexpr (!M::kExact) {
    bool bad = false, zp = false;
    float qo[L + 1], d1[L + 1], d2[L + 1];
    auto flux3_f = [&](float hki, float num, float dsi, float dsn, float dhk, float den, double rden, int k,
                       bool &b) __attribute__((always_inline)) {
      qo[k] = m.div_d(-hki * num, den, rden);
      d1[k] = m.div_d(-(-hki * dsi + num * dhk), den, rden);
      d2[k] = m.div_d(-(hki * dsn + num * dhk), den, rden);
      b |= m.div_bad(qo[k]) | m.div_bad(d1[k]) | m.div_bad(d2[k]);
    };
#pragma unroll
    for (int i = 1; i <= L - 1; i++)
      flux3_f(hk[i], (smp[i + 1] - smp[i]) - (zq[i + 1] - zq[i]), dsmpdw[i], dsmpdw[i + 1], dhkdw[i], g.den(i),
              g.rden(i), i, bad);
    qo[L] = d1[L] = d2[L] = zero;
    if (any_aq) {                      // aquifer interface (used when aq)
      const float den = zcA - g.zc(L);
      bool ba = false;
      flux3_f(hk[L], smp1 - smp[L] - (zq[L + 1] - zq[L]), dsmpdw[L], dsmpdw1, dhkdw[L], den, recip64(den), L, ba);
      bad |= aq && ba;
    }
    // fluxes made exact here, so the layer arrays die before the sweep
    if (__builtin_expect(bad, 0)) {
      H9G_BR(BR_TRIFLUX);
#pragma unroll
      for (int i = 1; i <= L; i++) {
        const bool a = i == L;
        const float num = a ? smp1 - smp[L] - (zq[L + 1] - zq[L]) : (smp[i + 1] - smp[i]) - (zq[i + 1] - zq[i]);
        const float dsn = a ? dsmpdw1 : dsmpdw[i < L ? i + 1 : L];
        const float den = a ? zcA - g.zc(L) : g.den(i);
        m.div_fix(qo[i], -hk[i] * num, den);
        m.div_fix(d1[i], -(-hk[i] * dsmpdw[i] + num * dhkdw[i]), den);
        m.div_fix(d2[i], -(hk[i] * dsn + num * dhkdw[i]), den);
      }
      bad = false;
    }
    auto row_f = [&](int i, float am, float bm, float cm, float rm) __attribute__((always_inline)) {
      float x;
      if (i == 1) {
        BET = bm;
        x = rm;
      } else {
        BET = bm - am * GAM[i];
        zp |= BET == 0.0f;
        x = rm - am * dwat2[i - 1];
      }
      const double rb = recip64(BET);
      dwat2[i] = m.div_d(x, BET, rb);
      bad |= m.div_bad(dwat2[i]);
      if (i <= L) {
        GAM[i + 1] = m.div_d(cm, BET, rb);
        bad |= m.div_bad(GAM[i + 1]);
      }
    };
    auto dzdt = [&](float dz) __attribute__((always_inline)) {
      const float q = m.div_d(dz, dt, g.rdt());
      bad |= m.div_bad(q);
      return q;
    };
    const float bm1 = dzdt(g.dz(1)) + d1[1];
    row_f(1, zero, bm1, d2[1], qflx_infl - qo[1] - tran * ROOT(1));
#pragma unroll
    for (int i = 2; i <= L - 1; i++)
      row_f(i, -d1[i - 1], dzdt(g.dz(i)) - d2[i - 1] + d1[i], d2[i], qo[i - 1] - qo[i] - tran * ROOT(i));
    row_f(L, -d1[L - 1], dzdt(g.dz(L)) - d2[L - 1] + (aq ? d1[L] : zero), aq ? d2[L] : zero,
          qo[L - 1] - (aq ? qo[L] : zero) - tran * ROOT(L));
    const float qA = dzdt(dzA);
    const float bmA = qA - d2[L] + zero;
    const float rmA = qo[L] - zero;
    row_f(L + 1, aq ? -d1[L] : zero, aq ? bmA : qA, zero, aq ? rmA : zero);
    if (__builtin_expect(bad | zp | (bm1 == 0.0f), 0)) {  // the exact sweep on the (exact) fluxes
      H9G_BR(BR_TRISWEEP);
      BET = zero;
      zero_pivot = 0;
      const float bm1x = m.div(g.dz(1), dt, g.rdt()) + d1[1];
      if (bm1x == 0.0f) { errval = bm1x; return 1; }                // :806-812
      row(1, zero, bm1x, d2[1], qflx_infl - qo[1] - tran * ROOT(1));
#pragma unroll
      for (int i = 2; i <= L - 1; i++)
        row(i, -d1[i - 1], m.div(g.dz(i), dt, g.rdt()) - d2[i - 1] + d1[i], d2[i], qo[i - 1] - qo[i] - tran * ROOT(i));
      if (!aq) {
        row(L, -d1[L - 1], m.div(g.dz(L), dt, g.rdt()) - d2[L - 1] + zero, zero, qo[L - 1] - zero - tran * ROOT(L));
        row(L + 1, zero, m.div(dzA, dt, g.rdt()), zero, zero);
      } else {
        row(L, -d1[L - 1], m.div(g.dz(L), dt, g.rdt()) - d2[L - 1] + d1[L], d2[L], qo[L - 1] - qo[L] - tran * ROOT(L));
        row(L + 1, -d1[L], m.div(dzA, dt, g.rdt()) - d2[L] + zero, zero, qo[L] - zero);
      }
      if (zero_pivot) { errval = (float)zero_pivot; return 2; }      // :818-825
    }
    tri_ok = true;
  }
  if (!tri_ok) {
  // qout, dqodw1, dqodw2 of one interface: independent quotients, one check.
  auto flux3 = [&](float hki, float num, float dsi, float dsn, float dhk, float den, double rden, float &qo,
                   float &d1, float &d2) __attribute__((always_inline)) {
    const float x0 = -hki * num, x1 = -(-hki * dsi + num * dhk), x2 = -(hki * dsn + num * dhk);
    qo = m.div_d(x0, den, rden);
    d1 = m.div_d(x1, den, rden);
    d2 = m.div_d(x2, den, rden);
    if (__builtin_expect(m.div_bad(qo) | m.div_bad(d1) | m.div_bad(d2), 0)) {
      m.div_fix(qo, x0, den);
      m.div_fix(d1, x1, den);
      m.div_fix(d2, x2, den);
    }
  };
  float q_prev, dq0_prev, dq1_prev;      // interface i-1
  {
    const float den = g.den(1);
    const double rden = g.rden(1);
    const float dzq = (zq[2] - zq[1]);
    const float num = (smp[2] - smp[1]) - dzq;
    float qout, dqodw1, dqodw2;
    flux3(hk[1], num, dsmpdw[1], dsmpdw[2], dhkdw[1], den, rden, qout, dqodw1, dqodw2);
    const float bm1 = m.div(g.dz(1), dt, g.rdt()) + dqodw1;
    if (bm1 == 0.0f) { errval = bm1; return 1; }                    // :806-812
    row(1, zero, bm1, dqodw2, qflx_infl - qout - tran * ROOT(1));
    q_prev = qout; dq0_prev = dqodw1; dq1_prev = dqodw2;
  }
#pragma unroll
  for (int i = 2; i <= L - 1; i++) {
    const float den = g.den(i);
    const double rden = g.rden(i);
    const float dzq = zq[i + 1] - zq[i];
    const float num = (smp[i + 1] - smp[i]) - dzq;
    float qout, dqodw1, dqodw2;
    flux3(hk[i], num, dsmpdw[i], dsmpdw[i + 1], dhkdw[i], den, rden, qout, dqodw1, dqodw2);
    row(i, -dq0_prev, m.div(g.dz(i), dt, g.rdt()) - dq1_prev + dqodw1, dqodw2,
        q_prev - qout - tran * ROOT(i));
    q_prev = qout; dq0_prev = dqodw1; dq1_prev = dqodw2;
  }
  {
    constexpr int i = L;
    if (i > jwt) {                 // water table inside the column
      const float qout = zero, dqodw1 = zero;
      row(i, -dq0_prev, m.div(g.dz(i), dt, g.rdt()) - dq1_prev + dqodw1, zero,
          q_prev - qout - tran * ROOT(i));
      row(i + 1, zero, m.div(dzA, dt, g.rdt()), zero, zero);
    } else {                       // below: aquifer row (smp1, dsmpdw1 from the pair split)
      const float den = zcA - g.zc(i);
      const double rden = recip64(den);
      const float dzq = zq[i + 1] - zq[i];
      const float num = smp1 - smp[i] - dzq;
      float qout, dqodw1, dqodw2;
      flux3(hk[i], num, dsmpdw[i], dsmpdw1, dhkdw[i], den, rden, qout, dqodw1, dqodw2);
      row(i, -dq0_prev, m.div(g.dz(i), dt, g.rdt()) - dq1_prev + dqodw1, dqodw2,
          q_prev - qout - tran * ROOT(i));
      const float qout1 = zero, dqodw1b = zero;
      row(i + 1, -dqodw1, m.div(dzA, dt, g.rdt()) - dqodw2 + dqodw1b, zero, qout - qout1);
    }
  }
  if (zero_pivot) { errval = (float)zero_pivot; return 2; }          // :818-825
  }  // !tri_ok
#pragma unroll
  for (int i = L; i >= 1; i--) dwat2[i] = dwat2[i] - GAM[i + 1] * dwat2[i + 1];
  // :845-850
#pragma unroll
  for (int i = 1; i <= L; i++) h2o[i] = h2o[i] + dwat2[i] * g.dz(i);
  cs.launder();
  pr.mark(4);
  // The specific yield s_y(I) = max(ts(I) (1 - (1 + zwtmm/(-psi(I)))^(-1/b(I))),
  // 0.02) (:963-965, :979-981, :1077-1080), for a layer i at runtime.
  auto s_y_base = [&](int i, float zmm) __attribute__((always_inline)) -> float {
    return one + divr<CS::kRecip>(m, zmm, -cs.lay(PF_PSI, i), [&]() { return lay_d(cs, PF_RPSI0, i); });
  };
  auto s_y_of = [&](int i, float pw) __attribute__((always_inline)) -> float {
    return MAXX(cs.lay(PF_TS, i) * (one - pw), 0.02f);
  };
  auto s_y_at = [&](int i, float zmm) __attribute__((always_inline)) -> float {
    return s_y_of(i, m.powf(s_y_base(i, zmm), cs.lay(PF_NINVB, i)));
  };
  // :856-904 recharge.  With the water table in the column, the power of
  // the recharge conductivity ka (:874-877) and the power of the first
  // layer the water-table loops below visit, s_y(jwt+1) at this zwtmm, are
  // independent: one lane of the pair evaluates each.
  float qcharge, sy_first = zero;
  if (jwt < L) {
    H9G_BR(BR_JWTCOL);
    // operands of layer jwt+1 (and jwt): the parameters by runtime-indexed
    // store reads, the register arrays by selects
    const int j1 = jwt + 1;
    const float hks_j = cs.lay(PF_HKS, j1);
    float smp_m = zero, zq_m = zero, zc_j = zero;
#pragma unroll
    for (int i = 1; i <= L; i++) {
      if (i == (jwt > 1 ? jwt : 1)) { smp_m = smp[i]; zq_m = zq[i]; }
      if (i == jwt) zc_j = g.zc(i);
    }
    const float wh_zwt = zero;
    // the two powers came from the first round above (p0, p1)
    sy_first = s_y_of(jwt + 1, p1.v[0]);
    const float ka = hks_j * p0.v[0];
    const float smp1m = MAXC(smpmin, smp_m);
    const float wh = smp1m - zq_m;
    if (jwt == 0)
      qcharge = -ka * (wh_zwt - wh) / (zwtmm + one);
    else
      qcharge = -ka * (wh_zwt - wh) / ((zwtmm - zc_j) * 2.0f);
    qcharge = MAXC(-10.0f / dt, qcharge);
    qcharge = MINC(10.0f / dt, qcharge);
  } else {
    qcharge = m.div(dwat2[L + 1] * dzA, dt, g.rdt());
  }
  // :923-1009 water table from recharge.  s_y(I) is evaluated for exactly
  // the layers the loops visit (usually one), at a runtime layer index (the
  // first visit's from the pick above); rous = s_y(L) of the pre-update
  // zwtmm came from the pair split of the equilibrium profile.
  float rous = MAXX(TS(L) * (one - pY.v[0]), 0.02f);
  // x / 1000 in the water-table loops, which run only for a substep that
  // started with the water table in the column (a day snapshot exists): a
  // quotient that needs the IEEE division (subnormal) asks for the exact
  // re-run of the substep instead of a redo branch in place (H9G_WT_DEFER)
  auto wdiv = [&](float x) __attribute__((always_inline)) {
    if constexpr (H9G_WT_DEFER && !M::kExact) {
      const float q = m.div_d(x, 1000.0f, r1000);
      m.special |= m.div_bad(q);
      return q;
    } else {
      return m.div(x, 1000.0f, r1000);
    }
  };
  int jwt2 = jwt;
  if (jwt == L) {
    s.wa = s.wa + qcharge * dt;
    s.zwt = s.zwt - m.div(qcharge * dt, 1000.0f, r1000) / rous;
  } else {
    float qcharge_tot = qcharge * dt;
    if (qcharge_tot > zero) {          // rising: I = jwt+1 .. 1
      visit_layers(m, [&](int k) __attribute__((always_inline)) -> bool {
        const int i = jwt + 1 - k;
        const float s_y = k == 0 ? sy_first : s_y_at(i, zwtmm);
        float qcl = MINF(qcharge_tot, s_y * (zwtmm - cs.zi(i - 1)));
        qcl = MAXF(qcl, zero);
        if (s_y > zero) s.zwt = s.zwt - wdiv(qcl / s_y);
        qcharge_tot = qcharge_tot - qcl;
        return !(qcharge_tot <= zero || i == 1);
      });
    } else {                            // deepening: I = jwt+1 .. L
      visit_layers(m, [&](int k) __attribute__((always_inline)) -> bool {
        const int i = jwt + 1 + k;
        const float s_y = k == 0 ? sy_first : s_y_at(i, zwtmm);
        float qcl = MAXF(qcharge_tot, -s_y * (cs.zi(i) - zwtmm));
        qcl = MINF(qcl, zero);
        qcharge_tot = qcharge_tot - qcl;
        if (qcharge_tot >= zero) {
          s.zwt = s.zwt - wdiv(qcl / s_y);
          return false;
        }
        s.zwt = cs.zim(i);
        return i != L;
      });
      if (qcharge_tot > zero) {
        if (!aq) rous = s_y_at(L, zwtmm);    // this lane's first round was the recharge's
        s.zwt = s.zwt - wdiv(qcharge_tot) / rous;
      }
    }
    jwt2 = jwt_of<L>(s.zwt, zim);
  }
  cs.launder();
  pr.mark(5);
  // :1015-1035 baseflow; s_y(L) for the new zwtmm (:1077-1080) on one lane
  // of the pair, the drainage loop's first layer s_y(jwt2+1) on the other
  zwtmm = 1000.0f * s.zwt;
  // rsub_top's exponential and the pair's power are independent: both
  // branch-free, one deferred check (before the pair exchange).
  float rsub_top;
  const int jd = jwt2 < L ? jwt2 + 1 : L;
  FV<1> pR, pD;
  sp.template pick<1>(
      [&](int h) __attribute__((always_inline)) -> FV<1> {
        const int i = h ? jd : L;
        bool se = false, sq = false, sw = false;
        float ex = expf_fast(m, -fff * s.zwt, se);
        const float nb = -cs.lay(PF_PSI, i);
        float q = divr_d<CS::kRecip>(m, zwtmm, nb, [&]() { return lay_d(cs, PF_RPSI0, i); }, sq);
        float w = m.powf_d(one + q, cs.lay(PF_NINVB, i), sw);
        if (__builtin_expect(se | sq | sw, 0)) {
          H9G_BR(BR_BASE);
          if (se) ex = m.expf(-fff * s.zwt);
          divr_fix<CS::kRecip>(m, q, zwtmm, nb);
          w = m.powf(one + q, cs.lay(PF_NINVB, i));
        }
        rsub_top = 5.5E-3f * ex;
        return FV<1>{{w}};
      },
      pR, pD);
  rous = s_y_of(L, pR.v[0]);
  const float sy_drain = s_y_of(jd, pD.v[0]);
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
    visit_layers(m, [&](int k) __attribute__((always_inline)) -> bool {   // I = jwt+1 .. L
      const int i = jwt2 + 1 + k;
      const float s_y = k == 0 ? sy_drain : s_y_at(i, zwtmm);
      float rstl = MAXF(rsub_top_tot, -(s_y * (cs.zi(i) - zwtmm)));
      rstl = MINF(rstl, zero);
#pragma unroll
      for (int j = 1; j <= L; j++) {    // h2o(I) = h2o(I) + rstl, I at runtime: a select per
        int hit = (j == i);             // layer (opaque, so it is not folded back into an
        opaque(hit);                    // indexed store that would demote h2o to scratch)
        h2o[j] = hit ? h2o[j] + rstl : h2o[j];
      }
      rsub_top_tot = rsub_top_tot - rstl;
      if (rsub_top_tot >= zero) {
        s.zwt = s.zwt - wdiv(rstl / s_y);
        return false;
      }
      s.zwt = cs.zim(i);
      return i != L;
    });
    s.zwt = s.zwt - wdiv(rsub_top_tot) / rous;
    s.wa = s.wa + rsub_top_tot;
    jwt3 = jwt_of<L>(s.zwt, zim);
  }
  // :1122-1123
  s.zwt = MAXF(0.0f, s.zwt);
  s.zwt = MINC(80.0f, s.zwt);
  cs.launder();
  pr.mark(6);
  // :1131-1137 saturation excess, bottom-up bucket
#pragma unroll
  for (int i = L; i >= 2; i--) {
    const float cap = MAXF(0.01f, TS(i)) * g.dz(i);
    const float xsi = MAXF(h2o[i] - cap, zero);
    h2o[i] = MINF(cap, h2o[i]);
    h2o[i - 1] = h2o[i - 1] + xsi;
  }
  // :1144-1152
  const float xs1 = MAXF(MAXF(h2o[1], zero) - cs.sc(PS_TSDZ1), zero);
  h2o[1] = MINF(cs.sc(PS_TSDZ1), h2o[1]);
  float qflx_rsub_sat = m.div_d(xs1, dt, g.rdt());   // checked with the watmin section's branch
  // :1161-1211 watmin.  With no layer below watmin every xs is zero and
  // every update below is an identity (x + 0 would change only x = -0, and
  // -0 < watmin), so a lane with no layer below watmin skips the section:
  // one rarely-taken branch instead of one per layer.
  bool low = false;
#pragma unroll
  for (int i = 1; i <= L; i++) low |= h2o[i] < watmin;
  if (__builtin_expect(low | m.div_bad(qflx_rsub_sat), 0)) {
  H9G_BR(BR_WATMIN);
  m.div_fix(qflx_rsub_sat, xs1, dt);
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
  }  // low
  // :1221-1236.  The end-of-step theta (:1233) is read only by the daily
  // sums after the day's last substep (the next substep recomputes theta
  // from h2osoi_liq, :141-151), so cell_year_pair evaluates it once a day.
  float w1 = ((1.0f - frac_h2osfc) * (qflx_surf + evg + tran) + rsub_top + qflx_rsub_sat) * dt + s.wa;
#pragma unroll
  for (int i = 1; i <= L; i++) w1 = w1 + h2o[i];
  pr.mark(7);
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
#undef LAYF
#undef ROOT
#undef DC
#undef OWN
}

// The day snapshot (sv_* of the store): the state at the start of substep
// SV_NS of the current day -- h2osoi_liq, smp, zwt, wa and the runoff sum.
// cell_year_pair writes it at most once a day, before the day's first
// substep with the water table in the column; the exact re-run below
// advances it.  Round 2 rewrote it before every substep (11 stores per lane
// per substep, 4.5 GB per config-2 launch written back from L2) although
// only the rare re-run reads it.
template <int L, class SP, class CS>
H9K_HD void save_day(const SP &sp, const CS &cs, const St<L> &s, float rnf_sum, int ns) {
  save_layers<L>(sp, cs, 0, s.h2o);
  save_layers<L>(sp, cs, 1, s.smp);
  cs.sv_set_sc(SV_ZWT, s.zwt);
  cs.sv_set_sc(SV_WA, s.wa);
  cs.sv_set_sc(SV_RNF, rnf_sum);
  cs.sv_set_sc(SV_NS, (float)ns);
}

// Exact re-run (rare path, out of line): from the snapshot (the state at
// the start of substep SV_NS of the day) through substep ns, one lane
// computing every layer with the full glibc special-case logic.  The fast
// path's substeps before ns are bit-identical to these, so replaying them
// reproduces its state exactly.  The snapshot then holds the state after ns.
template <int L, class G, class CS>
H9K_RARE int substep_exact_pair(const G *g, CS cs, const uint64_t *e2, const double *l2, int ns) {
  cs.sv_sync();
  St<L> s;
#pragma unroll
  for (int i = 1; i <= L; i++) {
    s.h2o[i] = cs.sv_lay(0, i);
    s.smp[i] = cs.sv_lay(1, i);
  }
  s.zwt = cs.sv_sc(SV_ZWT);
  s.wa = cs.sv_sc(SV_WA);
  float rnf = cs.sv_sc(SV_RNF), errval = zero;
  MathExact me{{e2, l2}};
  const SplitAll sa;
  NoProf np;
  int code = 0;
  H9G_EXACT_HOOK((int)cs.sv_sc(SV_NS), ns);
  for (int k = (int)cs.sv_sc(SV_NS); k <= ns && !code; k++)
    code = hydrology_pair<L, G, MathExact, SplitAll, CS>(*g, cs, sa, s, rnf, errval, me, np);
  cs.launder();
#pragma unroll
  for (int i = 1; i <= L; i++) {
    cs.sv_set_lay(0, i, s.h2o[i]);
    cs.sv_set_lay(1, i, s.smp[i]);
  }
  cs.sv_set_sc(SV_ZWT, s.zwt);
  cs.sv_set_sc(SV_WA, s.wa);
  cs.sv_set_sc(SV_RNF, rnf);
  cs.sv_set_sc(SV_ERR, errval);
  cs.sv_set_sc(SV_NS, (float)(ns + 1));
  cs.sv_sync();
  return code;
}

// Substep ns of the day on the fast path.  A pair re-runs (exactly, from the
// day snapshot) if either of its lanes needs a third water-table layer visit.
// `snapped`: the day snapshot was taken today, at or before this substep.
// Only a substep that starts with the water table in the column (jwt < L)
// can ask for the re-run -- the rising/deepening loops run only for jwt < L
// and the drainage loop only for jwt2 < L, where HYDROLOGY.f90 recomputes
// jwt2 only in the jwt < L branch (:995-1005), so a substep starting below
// the column keeps jwt2 = L -- and cell_year_pair snapshots before the
// first such substep of the day.  A request without a snapshot would replay
// another day's (or, after the yearly re-sort, another cell's) block: it is
// reported as H9G_ERR_NOSNAP instead (never raised by a correct
// build, tests/test_kernel_host.py forces it).
template <int L, class G, class SP, class CS, class PR>
H9K_HD int substep_pair(const G &g, CS cs, const SP &sp, St<L> &s, float &rnf_sum, float &errval,
                        const h9m::Tabs &T, PR &pr, int ns, bool snapped) {
  pr.mark(0);
  H9G_BR(BR_SUBSTEP);
#if defined(H9G_ISA_MARK) && defined(__HIP_DEVICE_COMPILE__)
  asm volatile("; h9g-substep");     // tools/isa_mix.py: once per substep
#endif
  MathFast mf{T, false};
#if defined(H9G_FORCE_RERUN)
  const bool in_column = s.zwt <= g.zim(L);   // the substeps that may re-run (cell_year_pair)
#elif defined(H9G_FORCE_RERUN_ANY)
  const bool in_column = true;                // test builds: also below the column (-> H9G_ERR_NOSNAP)
#endif
  int code = hydrology_pair<L, G, MathFast, SP, CS, PR>(g, cs, sp, s, rnf_sum, errval, mf, pr);
#if defined(H9G_FORCE_RERUN)
  // test builds: also re-run every H9G_FORCE_RERUN-th substep of a day that
  // could (the exact replay from the day snapshot must reproduce the fast
  // path's state)
  if (sp.act() && in_column && ns % H9G_FORCE_RERUN == H9G_FORCE_RERUN - 1) mf.special = true;
#elif defined(H9G_FORCE_RERUN_ANY)
  if (sp.act() && in_column && ns % H9G_FORCE_RERUN_ANY == H9G_FORCE_RERUN_ANY - 1) mf.special = true;
#endif
  if (__builtin_expect(sp.pair_any(mf.special), 0)) {
    H9G_BR(BR_RERUN);
    if (!snapped) {                          // no snapshot of today to replay from
      errval = (float)ns;
      return H9G_ERR_NOSNAP_K;
    }
#if defined(H9G_COUNT_EXACT) && defined(__HIP_DEVICE_COMPILE__)
    atomicAdd(&h9g_exact_count, 1ull);      // measurement builds only
    atomicAdd(&h9g_exact_wave[(blockIdx.x * 4 + (threadIdx.x >> 6)) & 0xffff], 1u);
#endif
    cs.launder();
    code = substep_exact_pair<L, G, CS>(&g, cs, T.exp2, T.log2, ns);
    cs.launder();
#pragma unroll
    for (int i = 1; i <= L; i++) {
      s.h2o[i] = cs.sv_lay(0, i);
      s.smp[i] = cs.sv_lay(1, i);
    }
    s.zwt = cs.sv_sc(SV_ZWT);
    s.wa = cs.sv_sc(SV_WA);
    rnf_sum = cs.sv_sc(SV_RNF);
    errval = cs.sv_sc(SV_ERR);
  }
  return code;
}

// One calendar year for one cell (HYBRID9.f90:150-290), as cell_year.
// Park = keep the plant state in the store over the substeps (register
// relief for the 168-VGPR pair kernel).
template <int L, class G, class SP, class CS, bool Park = true, class PR = NoProf>
H9K_HD int cell_year_pair(const G &g, CS cs, const SP &sp, St<L> &s, const gbl_float *forc, size_t fday,
                          size_t fvar, int nt, int nisurf, int grow_on, gbl_float *acc, size_t astride,
                          int &eday, int &estep, float &errval, const h9m::Tabs &T, int raw = 0,
                          PR &&pr = PR()) {
  enum { A_NPP = 0, A_PM, A_RNF, A_EVAP, A_TAS, A_RLDS, A_RSDS, A_HUSS, A_PS, A_PR, A_RHS,
         A_THETA, A_H2O = 11 + L };
  gbl_float *A = acc;
  const size_t as = astride;
  float rnf_sum = zero;
  // spare lanes (Split2) run only the substeps' per-layer phases: everything
  // here that stores is behind act()
  const bool act = sp.act();
  if (act) {
#pragma unroll
    for (int k = 0; k < 12 + L; k++) A[k * as] = zero;
  }
  // plant state parked in the store over the substeps (read by day_consts
  // and GROW only, once a day)
  auto park = [&]() __attribute__((always_inline)) {
    if constexpr (Park) {
      if (!act) return;
      cs.set_sc(PS_LAI, s.LAI);
      cs.set_sc(PS_LAIL, s.LAI_litter);
      cs.set_sc(PS_PM, s.pm);
      cs.set_sc(PS_PFM, s.pfm);
      cs.set_sc(PS_PLEN, s.plen);
      cs.set_sc(PS_RDEPTH, s.rdepth);
    }
  };
  park();
  float npp = zero;
  int code = 0;
  MathExact me{T};
  s.naq = 0;
  for (int day = 0; day < nt; day++) {
    cs.day_start(day);
    H9G_BR(BR_DAY);
#if defined(H9G_DUMP_AQ) && defined(__HIP_DEVICE_COMPILE__)
    if (act && h9g_aq_bits && s.zwt > g.zim(L)) {   // spare lanes hold a mirrored cell's stale zwt
      const size_t c = (size_t)((const float *)acc - h9g_aq_base);
      atomicOr(&h9g_aq_bits[c * 12 + day / 32], 1u << (day & 31));
    }
#endif
    cs.launder();
    opaque(A);
    const gbl_float *f = forc + (size_t)day * fday;
    opaque(f);
    if (act) {
      float fv[7];             // tas rlds rsds huss ps pr rhs
#pragma unroll
      for (int k = 0; k < 7; k++) fv[k] = ld_stream(f + k * fvar);
      const Day d = make_day(fv[0], fv[1], fv[2], fv[3], fv[4], fv[5], fv[6]);   // :168-184
      if constexpr (Park)
        day_consts(d, cs.sc(PS_LAI), cs.sc(PS_LAIL), cs, me);
      else
        day_consts(d, s.LAI, s.LAI_litter, cs, me);
      // :235-241, the forcing's running sums: they depend on the forcing
      // only, so they are added here, once the day's forcing is loaded, and
      // the forcing is read once a day (the reference adds them after the
      // substeps: the same values in the same order; a cell that STOPs has
      // NaN annual means either way)
      float a7[7];
#pragma unroll
      for (int k = 0; k < 7; k++) a7[k] = A[(A_TAS + k) * as];
#pragma unroll
      for (int k = 0; k < 7; k++) A[(A_TAS + k) * as] = a7[k] + fv[k];
    }
    bool snapped = false;
    for (int ns = 0; ns < nisurf; ns++) {                            // :193-211
      // the day snapshot, taken before the first substep of the day whose
      // water table is in the column (jwt < L): only such a substep visits
      // layers (:923-1118), so only it can need the exact re-run
      const bool in_column = s.zwt <= g.zim(L);
      s.naq += in_column ? 0 : 1;
      if (act && !snapped && in_column) {
        H9G_BR(BR_SNAP);
        save_day<L>(sp, cs, s, rnf_sum, ns);
        snapped = true;
      }
      code = substep_pair<L, G, SP, CS>(g, cs, sp, s, rnf_sum, errval, T, pr, ns, snapped);
      if (code) { eday = day; estep = ns; break; }
    }
    cs.launder();
    if constexpr (Park) {
      s.LAI = cs.sc(PS_LAI);
      s.LAI_litter = cs.sc(PS_LAIL);
      s.pm = cs.sc(PS_PM);
      s.pfm = cs.sc(PS_PFM);
      s.plen = cs.sc(PS_PLEN);
      s.rdepth = cs.sc(PS_RDEPTH);
    }
    if (code) return code;
    if (!act) continue;
    opaque(A);
    if (grow_on) {
      opaque(f);               // tas again (not kept live over the substeps)
      grow_day<L, G, MathExact>(g, ld_stream(f), s, cs, npp, me);       // :217
      park();
    }
    // :242-254.  All running sums are loaded before any is stored, so the
    // loads issue back to back (the compiler cannot prove the strided
    // fields distinct)
    auto later = [](int k) { return k != A_RNF && k != A_EVAP && (k < A_TAS || k > A_RHS); };
    float a[12 + L];
#pragma unroll
    for (int k = 0; k < 12 + L; k++)
      if (later(k)) a[k] = A[k * as];
    a[A_PM] = a[A_PM] + s.pm;
    a[A_NPP] = a[A_NPP] + npp;
    float h2o_sum = a[A_H2O];
#pragma unroll
    for (int i = 1; i <= L; i++) {
      const float theta = MAXF(s.h2o[i], 1.0E-6f) / g.thk(i);       // HYDROLOGY.f90:1233
      a[A_THETA + i - 1] = a[A_THETA + i - 1] + theta;
      h2o_sum = h2o_sum + s.h2o[i];
    }
    a[A_H2O] = h2o_sum;
#pragma unroll
    for (int k = 0; k < 12 + L; k++)
      if (later(k)) A[k * as] = a[k];
  }
  // :263-290
  if (!act) return 0;
  opaque(A);
  if (raw) {                   // the cell order's day-1 probe: the running sums themselves
    A[A_RNF * as] = rnf_sum;
    return 0;
  }
  A[A_PM * as] = A[A_PM * as] / (float)nt;
  A[A_RNF * as] = rnf_sum / (float)(nt * nisurf);
  A[A_EVAP * as] = zero / (float)(nt * nisurf);
#pragma unroll
  for (int k = A_TAS; k <= A_H2O; k++) A[k * as] = A[k * as] / (float)nt;
  return 0;
}

// LCLIM single-site days for one cell (HYBRID9.f90:353-478): per-substep
// forcing, the day-of-year LAI schedule, no GROW.  Every substep runs the
// exact path (MathExact, one lane for all layers): this is the one-site
// evaluation tool, not the grid path.  Layouts (n = cells, [row][cell]):
//   sub   (nday*nisurf, 5, n): tak (degC), rh, Rnet, PAR, ppt (mm per substep)  :428-439
//   daily (nday, 2, n): huss, ps                                                 :377-378
//   lai   (nday, 3, n): LAI, a, b -- LAI = LAI, LAI_litter = LAI_litter + a - b,
//         NaN = no change (the schedule of :380-417)
//   out   (nday, 11, n): evap_day, evap_grnd_day, theta(1:4), theta_ma(1), LAI,
//         LAI_litter, w_i, fT                                                    :464-469
// w_i and fT are GROW's and GROW never runs here: they are 0.
template <int L, class G, class CS>
H9K_HD int cell_site(const G &g, CS cs, St<L> &s, float h2o_ma1, const float *sub, const float *daily,
                     const float *lai, float *out, size_t n, int nday, int nisurf, int &eday, int &estep,
                     float &errval, const h9m::Tabs &T) {
  MathExact me{T};
  const SplitAll sp;
  FluxProf fx{zero, zero};
  float rnf_sum = zero;
  const float dt = g.dt();
  const float theta_ma1 = h2o_ma1 / g.thk(1);                         // HYDROLOGY.f90:149
  for (int day = 0; day < nday; day++) {
    const float *l = lai + (size_t)day * 3 * n;
    if (l[0] == l[0]) s.LAI = l[0];
    if (l[n] == l[n]) s.LAI_litter = s.LAI_litter + l[n] - l[2 * n];
    const float *dd = daily + (size_t)day * 2 * n;
    float evap_day = zero, evap_grnd_day = zero;
    for (int ns = 0; ns < nisurf; ns++) {
      const float *v = sub + ((size_t)day * nisurf + ns) * 5 * n;
      Day d;
      d.tak = v[0] + tf;
      d.rh = v[n];
      d.Rnet = v[2 * n];
      d.PAR = v[3 * n];
      d.forc_rain = v[4 * n] / dt;
      d.lamb = ((2503.0f - 2.386f * (d.tak - tf))) * 1.0E3f;        // :445
      d.huss = dd[0];
      d.ps = dd[n];
      day_consts(d, s.LAI, s.LAI_litter, cs, me);
      const int code = hydrology_pair<L, G, MathExact, SplitAll, CS, FluxProf>(g, cs, sp, s, rnf_sum, errval,
                                                                            me, fx);
      if (code) { eday = day; estep = ns; return code; }
      evap_day = evap_day + (fx.evg + fx.tran) * dt;                  // :457-458
      evap_grnd_day = evap_grnd_day + fx.evg * dt;
    }
    float *o = out + (size_t)day * 11 * n;
    o[0] = evap_day;
    o[n] = evap_grnd_day;
#pragma unroll
    for (int i = 1; i <= 4; i++) o[(1 + i) * n] = MAXF(s.h2o[i], 1.0E-6f) / g.thk(i);   // :1233
    o[6 * n] = theta_ma1;
    o[7 * n] = s.LAI;
    o[8 * n] = s.LAI_litter;
    o[9 * n] = zero;
    o[10 * n] = zero;
  }
  return 0;
}

}  // namespace h9k
