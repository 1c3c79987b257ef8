/*
 * h9g.h -- C-ABI of the MI355X HYBRID9 hot path (libh9g.so).
 *
 * Replaces the PGF cell loop of the reference driver
 *   /root/reference/SOURCE/HYBRID9.f90:120-295   (cell -> year -> day ->
 *   substep loop calling HYDROLOGY at :203 and GROW at :217)
 * which has no plugin/FFI surface of its own: HYDROLOGY and GROW take no
 * arguments and communicate through MODULE SHARED / CONTROL globals
 * (/root/reference/SOURCE/HYDROLOGY.f90:10-11, GROW.f90:11-12).  One call
 * of h9g_run_year advances every cell of a context through one calendar
 * year, exactly as one pass of HYBRID9.f90:130-291 does for one cell.
 *
 * Plain pointers and sizes only.  Host arrays use the reference's
 * Fortran layouts (SHARED.f90), with the land cells of a block compacted
 * into one dimension:
 *   per-layer arrays   A(L, ncell)     layer fastest   (SHARED.f90:398-429)
 *   per-cell arrays    A(ncell)                        (SHARED.f90:446-472)
 *   forcing            F(ncell, nday)  cell fastest, one array per variable
 *                      in READ_PGF.f90 order: tas rlds rsds huss ps pr rhs
 * The fortran/h9_gpu.f90 module binds every entry point with BIND(C).
 *
 * Semantics: h9g_run_decade_ordered is bit-identical to the reference as
 * it runs on one rank (its cells in order, the module array smp of
 * SHARED.f90:198 carried from cell to cell); h9g_run_year runs isolated
 * cells (every cell carries its own smp), bit-identical to the reference
 * harness run that way.
 * Threading: one host thread per context; contexts are not re-entrant;
 * one context per GPU.  All calls return 0 on success, a positive
 * H9G_ERR_* code for a reference STOP condition (details via
 * h9g_last_error) or a negative H9G_E* code for API/HIP failures.
 */
#ifndef H9G_H
#define H9G_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define H9G_ABI_VERSION 1
#define H9G_LMAX 10          /* soil layers supported: 8 (reference) or 10 */
#define H9G_NFORCING 7
#define H9G_NANNUAL_SCALARS 11
#define H9G_NDIAG 12
#define H9G_MAX_SLOTS 512   /* forcing slots per context; HBM bounds it too */

/* reference STOP sites (HYDROLOGY.f90) */
#define H9G_ERR_TRIDIAG1 1   /* :806-812  bmx(1) == 0            */
#define H9G_ERR_TRIDIAG2 2   /* :818-825  zero pivot             */
#define H9G_ERR_RSUB_POS 3   /* :1068-1072 rsub_top_tot > 0      */
#define H9G_ERR_IMBALANCE 4  /* :1244-1274 |w1 - w0| > 0.1 mm    */
/* not a reference STOP: the pair kernel's exact re-run was requested in a
 * substep with no day snapshot to replay from (an internal invariant,
 * DESIGN.md §3 "Day snapshot"; never raised by a correct build) */
#define H9G_ERR_NOSNAP 5
/* API / runtime failures */
#define H9G_EINVAL (-1)
#define H9G_EHIP (-2)
#define H9G_ENOMEM (-3)
#define H9G_ESTATE (-4)

typedef struct h9g_ctx h9g_ctx;

typedef struct {
  int32_t ncell;       /* land cells owned by this context (shard)          */
  int32_t nlayers;     /* L: 8 or 10 (SHARED.f90:294 nsoil_layers_max)      */
  int32_t nisurf;      /* substeps per day (driver.txt line 2, INIT.f90:183) */
  int32_t grow_on;     /* 1: CALL GROW daily (HYBRID9.f90:217); 0: frozen   */
  int32_t max_days;    /* forcing slot capacity in days (>= 366)            */
  int32_t nslots;      /* forcing slots (2 = double-buffered prefetch; up to
                          H9G_MAX_SLOTS resident years, bounded by free HBM) */
  float zi[H9G_LMAX + 2]; /* zi(0:L+1) mm (driver.txt:17-26, INIT.f90:202)  */
} h9g_config;

typedef struct {
  int32_t code;        /* H9G_ERR_* of the first failing cell (0: none)     */
  int32_t cell;        /* its 0-based index in the context                  */
  int32_t year;        /* calendar year                                     */
  int32_t day;         /* 0-based day of year (DOY-1)                       */
  int32_t substep;     /* 0-based NS-1                                      */
  float value;         /* w1-w0, pivot row, rsub_top_tot ...               */
} h9g_error;

/* --- lifetime -------------------------------------------------------- */
int h9g_abi_version(void);
int h9g_device_count(void);
/* Host-only validation of a configuration (needs no GPU): 0, or H9G_EINVAL
 * with a NUL-terminated reason in `reason` (may be NULL). */
int h9g_config_check(const h9g_config *cfg, char *reason, int reason_len);
/* Device bytes a context of this configuration allocates (0 if invalid). */
size_t h9g_config_bytes(const h9g_config *cfg);
/* Creates a context on HIP device `device`; NULL on failure, with the
 * reason (invalid field, free HBM short of h9g_config_bytes, no device)
 * in h9g_create_error() of the calling thread. */
h9g_ctx *h9g_create(const h9g_config *cfg, int device);
const char *h9g_create_error(void);
void h9g_destroy(h9g_ctx *ctx);

/* --- parameters and state (INIT.f90) ---------------------------------- */
/* theta_s, hksat, bsw, psi_s: (L, ncell); fmax: (ncell).  Units after
 * INIT.f90:611-631 (mm^3/mm^3, mm/s, -, mm). */
int h9g_set_params(h9g_ctx *ctx, const float *theta_s, const float *hksat,
                   const float *bsw, const float *psi_s, const float *fmax);
/* Initial state of INIT.f90:707-811 for every cell (smp = 0). */
int h9g_init_state(h9g_ctx *ctx);
/* Packed per-cell state, fields in this order, each (width, ncell) with
 * width-fastest:  h2osoi_liq(L) h2osoi_liq_ma(L) smp(L) rootr_col(L+1)
 * zwt wa LAI LAI_litter plant_mass plant_foliage_mass plant_length rdepth
 * -> h9g_state_size(L) = 4L+9 floats per cell. */
int h9g_state_size(int nlayers);
int h9g_set_state(h9g_ctx *ctx, const float *packed);
int h9g_get_state(h9g_ctx *ctx, float *packed);

/* --- forcing (READ_PGF.f90) ------------------------------------------ */
/* Copies nday days of forcing, 7 arrays of (ncell, nday) stacked as
 * (7, nday, ncell), into slot `slot`.  async=1 enqueues the copy on the
 * context's copy stream (host memory should be pinned, see
 * h9g_host_alloc); h9g_run_year orders itself after it. */
int h9g_push_forcing(h9g_ctx *ctx, int slot, int nday, const float *forcing,
                     int async);
/* Same from device memory (e.g. a slab already resident in HBM). */
int h9g_push_forcing_device(h9g_ctx *ctx, int slot, int nday,
                            const float *dev_forcing);
/* Device pointer of a slot (capacity max_days), for zero-copy producers. */
float *h9g_forcing_slot(h9g_ctx *ctx, int slot);
void *h9g_host_alloc(size_t bytes);   /* pinned host memory */
void h9g_host_free(void *p);

/* --- the hot path ----------------------------------------------------- */
/* Advance every cell through calendar year `jyear` (365/366 days by
 * INIT.f90:844-859) using the forcing in `slot` starting at its day 0.
 * Enqueued on the compute stream; returns after launch.  Errors are
 * reported by the next h9g_sync. */
int h9g_run_year(h9g_ctx *ctx, int slot, int jyear);
/* Wait for all work; returns the first STOP code raised, if any. */
int h9g_sync(h9g_ctx *ctx);
int h9g_last_error(h9g_ctx *ctx, h9g_error *err);
/* Every cell's STOP record since the state was last set: rec is 4 rows of
 * ncell int32 -- H9G_ERR_* code (0: none), 0-based day, substep, and the
 * bits of the float value the reference prints (failed cells stop; their
 * annual means are NaN). */
int h9g_get_errors(h9g_ctx *ctx, int32_t *rec);

/* --- the reference's own cell order (HYBRID9.f90:93-130) ---------------- */
/* Advances every cell through years jyear0 .. jyear0+nyears-1 (the forcing
 * of year jyear0+k in slots[k]) as ONE pass of the reference's decade loop
 * runs them on one rank (or on every rank of h9g_set_chains): the cell
 * loop (:120-295) visits the land cells in context order, and HYDROLOGY's
 * module array smp (SHARED.f90:198) is not per cell, so a land cell's
 * first substep reads in beta (HYDROLOGY.f90:270-275) the smp its
 * predecessor left behind; the first land cell reads what the last one
 * holds when the call starts (at a fresh start all smp are 0; the
 * reference leaves smp uninitialised, INIT.f90:109).  Call it once per
 * decade of the reference (1901-1910, 1911-1920, ...) with the rank's
 * cells in (y, x) order to reproduce the reference run bit for bit.
 * h9g_run_year's isolated-cell semantics (every cell its own smp) differ
 * from this by up to 4e-2 relative from the second decade on (DESIGN.md
 * §2).  Solved on the device: each pass re-runs the decade for the cells
 * whose input smp changed, until none does; a re-run cell leaves the pass
 * at the first year end where its state equals its previous run's (its
 * later years are then unchanged, bit for bit).  annual: (nyears, 12+L,
 * ncell) host (may be NULL); passes (may be NULL): decade passes run.
 * Synchronous; returns 0 or the STOP code of the first failing cell in
 * context order (h9g_last_error, with its year). */
int h9g_run_decade_ordered(h9g_ctx *ctx, const int32_t *slots, int jyear0,
                           int nyears, float *annual, int32_t *passes);
/* The reference's decade loop over several decades: years jyear0 ..
 * jyear0+nyears-1 (the forcing of year jyear0+k in slots[k], every year's
 * slot resident for the whole call) cut into the reference's decades
 * (1901-1910, 1911-1920, ...), each run as h9g_run_decade_ordered runs
 * one, with the same results bit for bit.  The years' slots must be
 * distinct (H9G_EINVAL otherwise).  The decades overlap on the
 * device: a decade's first pass starts as soon as the previous decade's
 * first pass and year-1 re-run are done, and that decade's remaining
 * re-runs ride in its year launches.  annual: (nyears,
 * 12+L, ncell) host (may be NULL); passes (may be NULL): one int32 per
 * decade.  A cell that STOPs leaves the later decades' chains (the
 * reference would end the program there; h9g_last_error reports the first
 * STOP in decade then context order).  Synchronous. */
int h9g_run_ordered(h9g_ctx *ctx, const int32_t *slots, int jyear0, int nyears,
                    float *annual, int32_t *passes);
/* Splits the context's cells into independent chains for
 * h9g_run_decade_ordered, one per reference MPI rank: chain[c] (ncell
 * int32, 0 <= id < ncell) is the rank whose block holds cell c (INIT.f90:
 * 271-274, 427-444; hybrid9_amd.shard.reference_blocks).  Each chain runs
 * its cells in context order, as that rank runs its block, so a context
 * holding several ranks' blocks reproduces them all at once.  NULL: one
 * chain (the default, a one-rank run). */
int h9g_set_chains(h9g_ctx *ctx, const int32_t *chain);
/* Work of the last h9g_run_decade_ordered: out[0..n) of passes, cells
 * re-run (summed over the passes), cell-years re-run, and year launches of
 * the re-runs (a re-run cell leaves at the first year end where its state
 * is its previous run's again), then the cells of each re-run launch in
 * order.  Returns the count written (<= 4 + launches). */
int h9g_decade_stats(h9g_ctx *ctx, int64_t *out, int n);
/* How the last ordered call overlapped its decades: out[0..n) of decades,
 * year launches of the first passes, re-run years that rode in them and
 * their cell-years, re-run years launched alone and their cell-years, cells
 * left out of a first pass (still re-running the decade before), cells the
 * checks' day-1 probe ran and those of them it kept for a re-run, then each
 * decade's passes.  Returns the count written. */
int h9g_ordered_stats(h9g_ctx *ctx, int64_t *out, int n);

/* --- LCLIM single-site path (HYBRID9.f90:339-480) ---------------------- */
/* Runs nday days of the site path for every cell of the context: per
 * substep forcing, a day-of-year LAI schedule, HYDROLOGY only (no GROW).
 * Replaces the LCLIM branch :339-480 (its CSV reads :353-439 are done by
 * the caller, e.g. hybrid9_amd.site.read_lclim).  Host arrays, [row][cell]:
 *   sub   (nday*nisurf, 5, ncell): tak (degC), rh (%), Rnet (W m-2),
 *         PAR, ppt (mm per substep)        -- LCLIM_array2 (22,25,14,16,35)
 *   daily (nday, 2, ncell): huss (kg/kg), ps (Pa)   -- LCLIM_array (5,6)
 *   lai   (nday, 3, ncell): (LAI, a, b): LAI = LAI, then
 *         LAI_litter = LAI_litter + a - b; NaN leaves a value unchanged
 *         (encodes the schedule of :380-417)
 *   diag  (nday, 11, ncell) out: evap_day, evap_grnd_day, theta(1:4),
 *         theta_ma(1), LAI, LAI_litter, w_i, fT (the daily line :464-469;
 *         w_i = fT = 0 as GROW does not run; NaN for masked/failed cells)
 * Synchronous.  Updates the state (h2osoi_liq, smp, zwt, wa, LAI,
 * LAI_litter).  Returns 0 or a STOP code (h9g_last_error: day counts
 * from the start of the run, year = 0). */
int h9g_run_site(h9g_ctx *ctx, int nday, const float *sub, const float *daily,
                 const float *lai, float *diag);

/* --- outputs (HYBRID9.f90:263-290) ------------------------------------ */
/* Annual means of the last year run, (12+L) rows of (ncell):
 * npp plant_mass rnf evap tas rlds rsds huss ps pr rhs theta(1..L)
 * theta_total  (axy_* of SHARED.f90:478-493, NaN for failed cells). */
int h9g_get_annual(h9g_ctx *ctx, float *annual);
/* Global diagnostics of the last year (FP64 sums over this context's
 * cells, deterministic order): see H9G_DIAG_* in DESIGN.md.  Intended
 * for an all-reduce across GPUs.  dev_out (may be NULL) receives a
 * device-side copy; host_out (may be NULL) a host copy. */
int h9g_get_diagnostics(h9g_ctx *ctx, double *host_out, double *dev_out);
/* Stream-ordered variant, no host synchronisation: copies the diagnostics
 * into device buffer dev_out after the work already queued on `stream` (a
 * hipStream_t, NULL = legacy default stream), and makes `stream` wait for
 * the copy -- e.g. the stream an RCCL all-reduce of dev_out runs on. */
int h9g_get_diagnostics_async(h9g_ctx *ctx, double *dev_out, void *stream);

/* --- synthetic inputs (hybrid9_amd/synth.py, bit-identical) ----------- */
/* Cells are identified by their grid id (iy*nx+ix) and latitude. */
int h9g_set_cells(h9g_ctx *ctx, const int64_t *gid, const float *lat);
/* The synthetic land mask (host): the nland grid ids of an nx x ny grid,
 * raster order, and their latitudes (synth.land_cells / cell_lat). */
int h9g_land_cells(int nx, int ny, int nland, uint64_t seed, int64_t *gid,
                   float *lat);
int h9g_synth_params(h9g_ctx *ctx, uint64_t seed);
int h9g_synth_forcing(h9g_ctx *ctx, int slot, uint64_t seed, int day0,
                      int nday);

/* --- NetCDF I/O (hybrid9_amd/csrc/h9g_io.cpp): reads netCDF-4 (HDF5,
 * through the image's libhdf5, loaded on first use) and classic CDF-1/2;
 * writes CDF-2 ------------------------------------------------------------ */
/* WRITE_NET_CDF_3DR.f90:93-263: annual means (h9g_get_annual layout, 12+L
 * rows of ncell) of the cells gid (grid ids iy*nx+ix, row iy from the
 * north) to axyYYYY.nc with the reference's dimensions, variable names,
 * units and NaN _FillValue; zc = layer centre depths (L).  Host only. */
int h9g_write_axy_nc(const char *path, int nx, int ny, int nlayers,
                     const float *zc, int ncell, const int64_t *gid,
                     const float *annual);
/* READ_PGF.f90 / READ_NET_CDF_3DR.f90: days [t0, t0+nt) of variable 4
 * (time, lat, lon) of the 7 PGF files (tas rlds rsds huss ps pr rhs)
 * gathered at the grid ids gid into out (7, nt, ncell).  Host only. */
int h9g_nc_forcing_read(const char *const *paths, int nx, int ny, int ncell,
                        const int64_t *gid, int t0, int nt, float *out);
/* NTIMES of a PGF file: length of its 'time' dimension. */
int h9g_nc_ntimes(const char *path);
/* Stage profile of the last completed forcing read (any thread, any
 * context): out[0..n) of, in order, wall s, serial setup s (headers and
 * chunk tables), pool threads, jobs, then thread-seconds summed over the
 * pool of pread, inflate + unshuffle, gather, and other layouts (classic
 * rows / H5Dread), then stored bytes read, bytes decoded, values gathered
 * and the pool's wall s.  Returns the count written (<= H9G_IO_NSTATS). */
#define H9G_IO_NSTATS 12
int h9g_nc_read_stats(double *out, int n);
/* The same read on a host thread into pinned memory, then an async copy
 * into `slot` (needs h9g_set_cells); h9g_run_year on the slot waits. */
int h9g_nc_forcing_prefetch(h9g_ctx *ctx, int slot, const char *const *paths,
                            int nx, int ny, int t0, int nt);

/* --- soil parameter build (INIT.f90:492-680) --------------------------- */
/* One soil layer (0-based) of the context's cells (h9g_set_cells): the
 * 60x60 block average of the layer's 30" fields theta_s (0.001 cm3/cm3),
 * k_s (cm/day), lambda (0.001), psi_s (cm) over pixels with theta_s >= 0,
 * and the unit conversions of INIT.f90:611-628.  Fields: (ny*60) rows of
 * nx*60 floats, row 0 north; device pointers if on_device, else host. */
int h9g_soil_layer(h9g_ctx *ctx, int layer, const float *ts, const float *ks,
                   const float *lm, const float *ps, int nx, int ny,
                   int on_device);
/* INIT.f90:661-680 once all layers are built: Fmax of the soiled cells
 * from the 0.5 deg integer grids soil_tex and fmax (ny, nx); completes the
 * parameters (replaces h9g_set_params). */
int h9g_soil_fmax(h9g_ctx *ctx, const int32_t *soil_tex, const int32_t *fmax,
                  int nx, int ny);
/* Device ms of the last soil layer's block-average kernel; number of its
 * cells summed in the reference's sequential order (non-integer data). */
float h9g_last_soil_ms(h9g_ctx *ctx);
int h9g_last_soil_slow(h9g_ctx *ctx);
/* Parameters back to the host, h9g_set_params layouts. */
int h9g_get_params(h9g_ctx *ctx, float *theta_s, float *hksat, float *bsw,
                   float *psi_s, float *fmax);

/* --- measurement ------------------------------------------------------ */
/* Device time (HIP events on the compute stream) of the last year kernel,
 * and of all year kernels since the last reset. */
float h9g_last_kernel_ms(h9g_ctx *ctx);
double h9g_total_kernel_ms(h9g_ctx *ctx, int reset);
const char *h9g_kernel_name(h9g_ctx *ctx);
/* Per kernel kind 1..6 (pair, solo, solo+pair, pair2, pair11, pair1 -- the
 * one-column kernel of short re-run lists), 3 doubles each: year launches,
 * cell-years and device ms since the last reset (synchronises); then row 7,
 * the cell order's one-day probe launches (launches, cells, ms).  Returns
 * the count written (<= 21). */
int h9g_launch_stats(h9g_ctx *ctx, double *out, int n, int reset);
/* Digest of the sources and compile flags of this library (16 hex digits;
 * hybrid9_amd/build.py build_id).  Profiles record it, and the bench
 * attaches counters only to the build they were measured on.  No GPU. */
const char *h9g_build_id(void);

/* --- self test of the device math (h9_math.h vs glibc) ---------------- */
/* out[i] = expf(x[i]) if y == NULL, else powf(x[i], y[i]), on device. */
int h9g_math_selftest(int device, int n, const float *x, const float *y,
                      float *out);
/* The same through the year kernels' math (glibc's main path; inputs that
 * glibc sends down another path are redone in place with its full logic,
 * flag[i] = 1 there). */
int h9g_math_fast_selftest(int device, int n, const float *x, const float *y,
                           float *out, int *flag);
/* out[i] = x[i]/d[i] through the kernel's fast exact division (double
 * reciprocal); flag[i] = 1 where the quotient was redone as
 * the IEEE division (subnormal or NaN quotient). */
int h9g_div_selftest(int device, int n, const float *x, const float *d,
                     float *out, int *flag);
/* Hardware ids as the pair kernel's issue pacer decodes them: nblocks
 * workgroups of the pair kernel's shape and LDS size; per wave out[3w..3w+2]
 * = HW_REG_HW_ID, HW_REG_XCC_ID, 1 if every wave was resident at once. */
int h9g_pace_probe(int device, int nblocks, unsigned *out);

#ifdef __cplusplus
}
#endif
#endif /* H9G_H */
