!======================================================================!
MODULE H9_GPU
!----------------------------------------------------------------------!
! ISO_C_BINDING interface of libh9g.so (include/h9g.h): the Fortran side
! of the drop-in boundary.  A HYBRID9 host replaces the cell loop of
! /root/reference/SOURCE/HYBRID9.f90:120-295 by one h9g_run_year call per
! simulated year (see INTEGRATION.md).  Arrays are passed by reference
! with the SHARED.f90 layouts: per-layer (L,ncell) layer-fastest,
! per-cell (ncell), forcing (ncell,nday) per variable stacked as
! (ncell,nday,7) in READ_PGF.f90 order tas rlds rsds huss ps pr rhs.
!----------------------------------------------------------------------!
USE, INTRINSIC :: ISO_C_BINDING
IMPLICIT NONE

INTEGER, PARAMETER :: H9G_LMAX = 10
INTEGER, PARAMETER :: H9G_NDIAG = 12
INTEGER, PARAMETER :: H9G_ERR_TRIDIAG1 = 1, H9G_ERR_TRIDIAG2 = 2
INTEGER, PARAMETER :: H9G_ERR_RSUB_POS = 3, H9G_ERR_IMBALANCE = 4
INTEGER, PARAMETER :: H9G_ERR_NOSNAP = 5   ! internal invariant, not a reference STOP

TYPE, BIND(C) :: h9g_config
  INTEGER(C_INT32_T) :: ncell, nlayers, nisurf, grow_on, max_days, nslots
  REAL(C_FLOAT) :: zi (0:H9G_LMAX+1)
END TYPE h9g_config

TYPE, BIND(C) :: h9g_error
  INTEGER(C_INT32_T) :: code, cell, year, day, substep
  REAL(C_FLOAT) :: value
END TYPE h9g_error

INTERFACE
  FUNCTION h9g_abi_version () BIND(C, NAME='h9g_abi_version')
    IMPORT :: C_INT
    INTEGER(C_INT) :: h9g_abi_version
  END FUNCTION
  FUNCTION h9g_device_count () BIND(C, NAME='h9g_device_count')
    IMPORT :: C_INT
    INTEGER(C_INT) :: h9g_device_count
  END FUNCTION
  FUNCTION h9g_create (cfg, device) BIND(C, NAME='h9g_create')
    IMPORT :: C_PTR, C_INT, h9g_config
    TYPE(h9g_config), INTENT(IN) :: cfg
    INTEGER(C_INT), VALUE :: device
    TYPE(C_PTR) :: h9g_create
  END FUNCTION
  FUNCTION h9g_config_check (cfg, reason, reason_len) BIND(C, NAME='h9g_config_check')
    IMPORT :: C_INT, C_CHAR, h9g_config
    TYPE(h9g_config), INTENT(IN) :: cfg
    CHARACTER(KIND=C_CHAR), INTENT(OUT) :: reason (*)
    INTEGER(C_INT), VALUE :: reason_len
    INTEGER(C_INT) :: h9g_config_check
  END FUNCTION
  FUNCTION h9g_config_bytes (cfg) BIND(C, NAME='h9g_config_bytes')
    IMPORT :: C_SIZE_T, h9g_config
    TYPE(h9g_config), INTENT(IN) :: cfg
    INTEGER(C_SIZE_T) :: h9g_config_bytes
  END FUNCTION
  FUNCTION h9g_create_error () BIND(C, NAME='h9g_create_error')
    IMPORT :: C_PTR
    TYPE(C_PTR) :: h9g_create_error
  END FUNCTION
  FUNCTION h9g_build_id () BIND(C, NAME='h9g_build_id')
    IMPORT :: C_PTR
    TYPE(C_PTR) :: h9g_build_id
  END FUNCTION
  SUBROUTINE h9g_destroy (ctx) BIND(C, NAME='h9g_destroy')
    IMPORT :: C_PTR
    TYPE(C_PTR), VALUE :: ctx
  END SUBROUTINE
  FUNCTION h9g_set_params (ctx, theta_s, hksat, bsw, psi_s, fmax) &
           BIND(C, NAME='h9g_set_params')
    IMPORT :: C_PTR, C_INT, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT), INTENT(IN) :: theta_s (*), hksat (*), bsw (*), psi_s (*), fmax (*)
    INTEGER(C_INT) :: h9g_set_params
  END FUNCTION
  FUNCTION h9g_init_state (ctx) BIND(C, NAME='h9g_init_state')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT) :: h9g_init_state
  END FUNCTION
  FUNCTION h9g_state_size (nlayers) BIND(C, NAME='h9g_state_size')
    IMPORT :: C_INT
    INTEGER(C_INT), VALUE :: nlayers
    INTEGER(C_INT) :: h9g_state_size
  END FUNCTION
  FUNCTION h9g_set_state (ctx, packed) BIND(C, NAME='h9g_set_state')
    IMPORT :: C_PTR, C_INT, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT), INTENT(IN) :: packed (*)
    INTEGER(C_INT) :: h9g_set_state
  END FUNCTION
  FUNCTION h9g_get_state (ctx, packed) BIND(C, NAME='h9g_get_state')
    IMPORT :: C_PTR, C_INT, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT), INTENT(OUT) :: packed (*)
    INTEGER(C_INT) :: h9g_get_state
  END FUNCTION
  FUNCTION h9g_push_forcing (ctx, slot, nday, forcing, async) &
           BIND(C, NAME='h9g_push_forcing')
    IMPORT :: C_PTR, C_INT, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: slot, nday, async
    REAL(C_FLOAT), INTENT(IN) :: forcing (*)
    INTEGER(C_INT) :: h9g_push_forcing
  END FUNCTION
  FUNCTION h9g_push_forcing_device (ctx, slot, nday, dev) &
           BIND(C, NAME='h9g_push_forcing_device')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx, dev
    INTEGER(C_INT), VALUE :: slot, nday
    INTEGER(C_INT) :: h9g_push_forcing_device
  END FUNCTION
  FUNCTION h9g_forcing_slot (ctx, slot) BIND(C, NAME='h9g_forcing_slot')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: slot
    TYPE(C_PTR) :: h9g_forcing_slot
  END FUNCTION
  FUNCTION h9g_host_alloc (bytes) BIND(C, NAME='h9g_host_alloc')
    IMPORT :: C_PTR, C_SIZE_T
    INTEGER(C_SIZE_T), VALUE :: bytes
    TYPE(C_PTR) :: h9g_host_alloc
  END FUNCTION
  SUBROUTINE h9g_host_free (p) BIND(C, NAME='h9g_host_free')
    IMPORT :: C_PTR
    TYPE(C_PTR), VALUE :: p
  END SUBROUTINE
  FUNCTION h9g_run_year (ctx, slot, jyear) BIND(C, NAME='h9g_run_year')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: slot, jyear
    INTEGER(C_INT) :: h9g_run_year
  END FUNCTION
  FUNCTION h9g_sync (ctx) BIND(C, NAME='h9g_sync')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT) :: h9g_sync
  END FUNCTION
  FUNCTION h9g_last_error (ctx, err) BIND(C, NAME='h9g_last_error')
    IMPORT :: C_PTR, C_INT, h9g_error
    TYPE(C_PTR), VALUE :: ctx
    TYPE(h9g_error), INTENT(OUT) :: err
    INTEGER(C_INT) :: h9g_last_error
  END FUNCTION
  FUNCTION h9g_get_annual (ctx, annual) BIND(C, NAME='h9g_get_annual')
    IMPORT :: C_PTR, C_INT, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT), INTENT(OUT) :: annual (*)
    INTEGER(C_INT) :: h9g_get_annual
  END FUNCTION
  FUNCTION h9g_get_diagnostics (ctx, host_out, dev_out) &
           BIND(C, NAME='h9g_get_diagnostics')
    IMPORT :: C_PTR, C_INT, C_DOUBLE
    TYPE(C_PTR), VALUE :: ctx, dev_out
    REAL(C_DOUBLE), INTENT(OUT) :: host_out (*)
    INTEGER(C_INT) :: h9g_get_diagnostics
  END FUNCTION
  FUNCTION h9g_get_errors (ctx, rec) BIND(C, NAME='h9g_get_errors')
    IMPORT :: C_PTR, C_INT, C_INT32_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT32_T), INTENT(OUT) :: rec (*)
    INTEGER(C_INT) :: h9g_get_errors
  END FUNCTION
  ! The reference's cell order over one decade (HYBRID9.f90:93-130: smp
  ! carried from cell to cell); annual (ncell, 12+L, nyears) in C order
  ! (nyears, 12+L, ncell).
  FUNCTION h9g_run_decade_ordered (ctx, slots, jyear0, nyears, annual, passes) &
           BIND(C, NAME='h9g_run_decade_ordered')
    IMPORT :: C_PTR, C_INT, C_INT32_T, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT32_T), INTENT(IN) :: slots (*)
    INTEGER(C_INT), VALUE :: jyear0, nyears
    REAL(C_FLOAT), INTENT(OUT) :: annual (*)
    INTEGER(C_INT32_T), INTENT(OUT) :: passes
    INTEGER(C_INT) :: h9g_run_decade_ordered
  END FUNCTION
  ! The same over several decades at once (every year's forcing resident),
  ! the decades overlapping on the device; passes: one per decade.
  FUNCTION h9g_run_ordered (ctx, slots, jyear0, nyears, annual, passes) &
           BIND(C, NAME='h9g_run_ordered')
    IMPORT :: C_PTR, C_INT, C_INT32_T, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT32_T), INTENT(IN) :: slots (*)
    INTEGER(C_INT), VALUE :: jyear0, nyears
    REAL(C_FLOAT), INTENT(OUT) :: annual (*)
    INTEGER(C_INT32_T), INTENT(OUT) :: passes (*)
    INTEGER(C_INT) :: h9g_run_ordered
  END FUNCTION
  FUNCTION h9g_ordered_stats (ctx, out, n) BIND(C, NAME='h9g_ordered_stats')
    IMPORT :: C_PTR, C_INT, C_INT64_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT64_T), INTENT(OUT) :: out (*)
    INTEGER(C_INT), VALUE :: n
    INTEGER(C_INT) :: h9g_ordered_stats
  END FUNCTION
  FUNCTION h9g_set_chains (ctx, chain) BIND(C, NAME='h9g_set_chains')
    IMPORT :: C_PTR, C_INT, C_INT32_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT32_T), INTENT(IN) :: chain (*)
    INTEGER(C_INT) :: h9g_set_chains
  END FUNCTION
  FUNCTION h9g_decade_stats (ctx, out, n) BIND(C, NAME='h9g_decade_stats')
    IMPORT :: C_PTR, C_INT, C_INT64_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT64_T), INTENT(OUT) :: out (*)
    INTEGER(C_INT), VALUE :: n
    INTEGER(C_INT) :: h9g_decade_stats
  END FUNCTION
  FUNCTION h9g_get_diagnostics_async (ctx, dev_out, stream) &
           BIND(C, NAME='h9g_get_diagnostics_async')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx, dev_out, stream
    INTEGER(C_INT) :: h9g_get_diagnostics_async
  END FUNCTION
  FUNCTION h9g_set_cells (ctx, gid, lat) BIND(C, NAME='h9g_set_cells')
    IMPORT :: C_PTR, C_INT, C_INT64_T, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT64_T), INTENT(IN) :: gid (*)
    REAL(C_FLOAT), INTENT(IN) :: lat (*)
    INTEGER(C_INT) :: h9g_set_cells
  END FUNCTION
  FUNCTION h9g_synth_params (ctx, seed) BIND(C, NAME='h9g_synth_params')
    IMPORT :: C_PTR, C_INT, C_INT64_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT64_T), VALUE :: seed
    INTEGER(C_INT) :: h9g_synth_params
  END FUNCTION
  FUNCTION h9g_synth_forcing (ctx, slot, seed, day0, nday) &
           BIND(C, NAME='h9g_synth_forcing')
    IMPORT :: C_PTR, C_INT, C_INT64_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: slot, day0, nday
    INTEGER(C_INT64_T), VALUE :: seed
    INTEGER(C_INT) :: h9g_synth_forcing
  END FUNCTION
  FUNCTION h9g_land_cells (nx, ny, nland, seed, gid, lat) &
           BIND(C, NAME='h9g_land_cells')
    IMPORT :: C_INT, C_INT64_T, C_FLOAT
    INTEGER(C_INT), VALUE :: nx, ny, nland
    INTEGER(C_INT64_T), VALUE :: seed
    INTEGER(C_INT64_T), INTENT(OUT) :: gid (*)
    REAL(C_FLOAT), INTENT(OUT) :: lat (*)
    INTEGER(C_INT) :: h9g_land_cells
  END FUNCTION
  ! NetCDF I/O (h9g_io.cpp): WRITE_NET_CDF_3DR.f90 / READ_PGF.f90
  FUNCTION h9g_write_axy_nc (path, nx, ny, nlayers, zc, ncell, gid, annual) &
      BIND(C, NAME='h9g_write_axy_nc')
    IMPORT :: C_INT, C_CHAR, C_FLOAT, C_INT64_T
    CHARACTER(KIND=C_CHAR), INTENT(IN) :: path (*)
    INTEGER(C_INT), VALUE :: nx, ny, nlayers, ncell
    REAL(C_FLOAT), INTENT(IN) :: zc (*), annual (*)
    INTEGER(C_INT64_T), INTENT(IN) :: gid (*)
    INTEGER(C_INT) :: h9g_write_axy_nc
  END FUNCTION
  FUNCTION h9g_nc_forcing_read (paths, nx, ny, ncell, gid, t0, nt, out) &
      BIND(C, NAME='h9g_nc_forcing_read')
    IMPORT :: C_INT, C_PTR, C_FLOAT, C_INT64_T
    TYPE(C_PTR), INTENT(IN) :: paths (*)
    INTEGER(C_INT), VALUE :: nx, ny, ncell, t0, nt
    INTEGER(C_INT64_T), INTENT(IN) :: gid (*)
    REAL(C_FLOAT) :: out (*)
    INTEGER(C_INT) :: h9g_nc_forcing_read
  END FUNCTION
  FUNCTION h9g_nc_ntimes (path) BIND(C, NAME='h9g_nc_ntimes')
    IMPORT :: C_INT, C_CHAR
    CHARACTER(KIND=C_CHAR), INTENT(IN) :: path (*)
    INTEGER(C_INT) :: h9g_nc_ntimes
  END FUNCTION
  FUNCTION h9g_nc_read_stats (out, n) BIND(C, NAME='h9g_nc_read_stats')
    IMPORT :: C_INT, C_DOUBLE
    REAL(C_DOUBLE), INTENT(OUT) :: out (*)
    INTEGER(C_INT), VALUE :: n
    INTEGER(C_INT) :: h9g_nc_read_stats
  END FUNCTION
  FUNCTION h9g_nc_forcing_prefetch (ctx, slot, paths, nx, ny, t0, nt) &
      BIND(C, NAME='h9g_nc_forcing_prefetch')
    IMPORT :: C_INT, C_PTR
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: slot, nx, ny, t0, nt
    TYPE(C_PTR), INTENT(IN) :: paths (*)
    INTEGER(C_INT) :: h9g_nc_forcing_prefetch
  END FUNCTION
  ! soil parameter build (INIT.f90:492-680)
  FUNCTION h9g_soil_layer (ctx, layer, ts, ks, lm, ps, nx, ny, on_device) &
      BIND(C, NAME='h9g_soil_layer')
    IMPORT :: C_INT, C_PTR, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: layer, nx, ny, on_device
    REAL(C_FLOAT), INTENT(IN) :: ts (*), ks (*), lm (*), ps (*)
    INTEGER(C_INT) :: h9g_soil_layer
  END FUNCTION
  FUNCTION h9g_soil_fmax (ctx, soil_tex, fmax, nx, ny) BIND(C, NAME='h9g_soil_fmax')
    IMPORT :: C_INT, C_PTR, C_INT32_T
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT32_T), INTENT(IN) :: soil_tex (*), fmax (*)
    INTEGER(C_INT), VALUE :: nx, ny
    INTEGER(C_INT) :: h9g_soil_fmax
  END FUNCTION
  FUNCTION h9g_last_soil_ms (ctx) BIND(C, NAME='h9g_last_soil_ms')
    IMPORT :: C_PTR, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT) :: h9g_last_soil_ms
  END FUNCTION
  FUNCTION h9g_last_soil_slow (ctx) BIND(C, NAME='h9g_last_soil_slow')
    IMPORT :: C_PTR, C_INT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT) :: h9g_last_soil_slow
  END FUNCTION
  FUNCTION h9g_get_params (ctx, theta_s, hksat, bsw, psi_s, fmax) BIND(C, NAME='h9g_get_params')
    IMPORT :: C_INT, C_PTR, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT) :: theta_s (*), hksat (*), bsw (*), psi_s (*), fmax (*)
    INTEGER(C_INT) :: h9g_get_params
  END FUNCTION
  ! LCLIM single-site path (HYBRID9.f90:339-480): sub (cells, 5, nday*NISURF),
  ! daily (cells, 2, nday), lai (cells, 3, nday), diag (cells, 11, nday)
  FUNCTION h9g_run_site (ctx, nday, sub, daily, lai, diag) BIND(C, NAME='h9g_run_site')
    IMPORT :: C_INT, C_PTR, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: nday
    REAL(C_FLOAT) :: sub (*), daily (*), lai (*), diag (*)
    INTEGER(C_INT) :: h9g_run_site
  END FUNCTION
  FUNCTION h9g_last_kernel_ms (ctx) BIND(C, NAME='h9g_last_kernel_ms')
    IMPORT :: C_PTR, C_FLOAT
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_FLOAT) :: h9g_last_kernel_ms
  END FUNCTION
  FUNCTION h9g_total_kernel_ms (ctx, reset) BIND(C, NAME='h9g_total_kernel_ms')
    IMPORT :: C_PTR, C_INT, C_DOUBLE
    TYPE(C_PTR), VALUE :: ctx
    INTEGER(C_INT), VALUE :: reset
    REAL(C_DOUBLE) :: h9g_total_kernel_ms
  END FUNCTION
  FUNCTION h9g_launch_stats (ctx, out, n, reset) BIND(C, NAME='h9g_launch_stats')
    IMPORT :: C_PTR, C_INT, C_DOUBLE
    TYPE(C_PTR), VALUE :: ctx
    REAL(C_DOUBLE), INTENT(OUT) :: out (*)
    INTEGER(C_INT), VALUE :: n, reset
    INTEGER(C_INT) :: h9g_launch_stats
  END FUNCTION
END INTERFACE

CONTAINS

  !--------------------------------------------------------------------!
  ! Print the reference's STOP diagnostics for the first failing cell
  ! and stop, as HYDROLOGY.f90:806-825,1068-1072,1244-1274 do.
  !--------------------------------------------------------------------!
  SUBROUTINE h9g_check_stop (ctx, rc)
    TYPE(C_PTR), INTENT(IN) :: ctx
    INTEGER(C_INT), INTENT(IN) :: rc
    TYPE(h9g_error) :: e
    INTEGER(C_INT) :: r
    IF (rc == 0) RETURN
    IF (rc < 0) THEN
      WRITE (*,*) 'h9g API/HIP failure, code ', rc
      STOP 'h9g failure'
    END IF
    r = h9g_last_error (ctx, e)
    SELECT CASE (e%code)
    CASE (H9G_ERR_TRIDIAG1)
      WRITE (*,*) 'Problem with tridiagonal 1.'
    CASE (H9G_ERR_TRIDIAG2)
      WRITE (*,*) 'Problem with tridiagonal 2.'
    CASE (H9G_ERR_RSUB_POS)
      WRITE (*,*) 'rsub_top_tot is positive in drainage'
      WRITE (*,*) 'HYBRID9 is stopping'
    CASE (H9G_ERR_NOSNAP)
      WRITE (*,*) 'h9g internal: exact re-run with no day snapshot'
    CASE DEFAULT
      WRITE (*,*) 'Problem in HYDROLOGY'
      WRITE (*,*) 'Water imbalance > 0.1 mm ', e%value
    END SELECT
    WRITE (*,*) 'DiTIME = ', e%day + 1
    WRITE (*,*) 'cell year substep ', e%cell + 1, e%year, e%substep + 1
    STOP
  END SUBROUTINE h9g_check_stop

END MODULE H9_GPU
!======================================================================!
