/*
 * TEST INFRASTRUCTURE ONLY -- the CPU oracle (plain C restatement).
 *
 * A line-by-line restatement, in C, of HYBRID9's per-cell hot path:
 *   HYDROLOGY  /root/reference/SOURCE/HYDROLOGY.f90:141-1283
 *   GROW       /root/reference/SOURCE/GROW.f90:55-201
 *   day driver /root/reference/SOURCE/HYBRID9.f90:120-290
 *   state init /root/reference/SOURCE/INIT.f90:707-811
 * calling glibc expf/powf exactly where the reference does (flang lowers
 * EXP and real powers to expf/powf; MIN/MAX to compare+select, see oracle/README.md).
 * Compiled with -ffp-contract=off (the reference executes no FMA).
 *
 * Pinned bit-for-bit against oracle/_ref/h9ref (the reference's own
 * HYDROLOGY/GROW) through tests/golden (see tests/test_oracle_golden.py).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, as the checker -- never as the product.
 *
 * Semantics: isolated-cell (each cell carries its own hidden smp).
 * Layouts: see oracle/refcase.py.  L <= H9O_LMAX soil layers.
 */
#ifndef H9_ORACLE_H
#include <stdint.h>
#define H9_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define H9O_LMAX 16
#define H9O_NANNUAL_SCALARS 11

/* STOP sites of the reference (HYDROLOGY.f90:806-825,1068-1072,1244-1274) */
enum { H9O_OK = 0, H9O_ERR_TRIDIAG1 = 1, H9O_ERR_TRIDIAG2 = 2,
       H9O_ERR_RSUB_POS = 3, H9O_ERR_IMBALANCE = 4, H9O_ERR_ARGS = 10 };

typedef struct {
  int code;      /* first failure, H9O_ERR_* */
  int cell;      /* 0-based cell index */
  int day;       /* 0-based day within the run */
  int substep;   /* 0-based substep */
  float value;   /* w1-w0, BET, ... */
} h9o_error;

/* floats per cell of the packed state (refcase.state_fields) */
int h9o_state_size(int L);

/* INIT.f90:707-811 initial state for every cell (smp = 0). */
int h9o_init_state(int ncell, int L, const float *zi, const float *params,
                   float *state);

/* Run nyears calendar years from year0 for every cell.
 *   zi       L+2 floats, zi(0:L+1)
 *   params   theta_s, hksat, bsw, psi_s (ncell*L each, layer-fastest), fmax
 *   forcing  (7, ndays, ncell), ndays = days in [year0, year0+nyears)
 *   state    in/out packed state (h9o_state_size(L) * ncell floats)
 *   annual   out (nyears, 12+L, ncell)
 *   trace    optional: for each of the ntrace cells, every substep,
 *            3L+7 floats (refcase.trace_width)
 *   nthreads OpenMP threads over cells (<=0: default)
 * Returns 0, or the first H9O_ERR_* (details in *err if non-NULL). */
int h9o_run(int ncell, int L, int nisurf, int grow_on, int year0, int nyears,
            const float *zi, const float *params, const float *forcing,
            float *state, float *annual, int ntrace, const int *trace_cells,
            float *trace, int nthreads, h9o_error *err,
            int *cell_err /* NULL, or 4 rows x ncell: STOP code, day of
                             year, substep, value bits (h9g_get_errors) */);

/* LCLIM single-site path (HYBRID9.f90:339-480), layouts of h9g_run_site:
 * sub (nday*nisurf, 5, ncell), daily (nday, 2, ncell), lai (nday, 3, ncell),
 * diag out (nday, 11, ncell); state in/out.  Returns 0 or the first STOP. */
int h9o_site(int ncell, int L, int nisurf, int nday, const float *zi, const float *params,
             const float *sub, const float *daily, const float *lai, float *state, float *diag,
             int nthreads, h9o_error *err);

/* Soil parameter build (INIT.f90:575-631 one layer, :661-680 Fmax). */
void h9o_soil_layer(int nx, int ny, int ncell, const int64_t *gid, const float *ts_in,
                    const float *ks_in, const float *lm_in, const float *ps_in, float *theta_s,
                    float *hksat, float *bsw, float *psi_s);
void h9o_soil_fmax(int ncell, int L, const int64_t *gid, const int32_t *soil_tex,
                   const int32_t *fmax_in, const float *theta_s, float *fmax);

#ifdef __cplusplus
}
#endif
#endif
