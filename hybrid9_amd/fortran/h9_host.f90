!======================================================================!
PROGRAM H9_HOST
!----------------------------------------------------------------------!
! MI355X host driver for HYBRID9's per-cell hot path.
!
! Restates the PGF path of /root/reference/SOURCE/HYBRID9.f90:81-333 with
! the cell loop (:120-295) replaced by the GPU: one h9g_run_year per
! simulated year advances every land cell (all days x NISURF substeps of
! HYDROLOGY, daily GROW), then the annual means (axy_*, :263-290) come
! back with h9g_get_annual.  Configuration keeps the reference surface:
! driver.txt is read with the same list-directed sequence as
! INIT.f90:181-204.  Inputs, since NetCDF/PGF/BNU are unavailable here:
!   input_mode = 'synth' : synthetic 0.5/0.25 deg land grid generated on
!                          the device (hybrid9_amd/synth.py bit-for-bit)
!   input_mode = 'case'  : a raw case directory (params.f32, forcing.f32,
!                          optional state0.f32, case.nml) -- the same files
!                          the reference harness oracle/_ref/h9ref reads
!   input_mode = 'pgf'   : forcing from the 7 PGF NetCDF files per decade
!                          (READ_PGF.f90 names <var>_pgfv2.1_<syr>_<eyr>.nc4
!                          in pgf_dir, netCDF classic), read on a host
!                          thread and copied while the previous year runs
!                          (h9g_nc_forcing_prefetch); synthetic soil
! chosen in the optional namelist file h9gpu.nml (/h9gpu/); nx, ny, nland
! override the synthetic grid.
!
! cell_order = 1 (default) runs the reference's own order: decade by
! decade (HYBRID9.f90:93-130), each land cell's first substep of a decade
! reading the smp its predecessor in (y, x) order left behind (HYDROLOGY.
! f90:270-275, SHARED.f90:198), through h9g_run_ordered -- bit for bit the
! reference on one rank.  Every year of a call is staged into its own slot
! and the call overlaps its decades on the device; ordered_decades > 0 cuts
! the run into calls of that many decades (HBM: 0.69 GB per 0.5 deg year),
! 0 (default) makes one call.  cell_order = 0: every cell its own smp
! (h9g_run_year per year, isolated-cell semantics, DESIGN.md §1).
!
! Usage:  h9_host [driver.txt] [h9gpu.nml]
! Outputs: <out_dir>/annual.f32 (ncell, 12+L, nyears),
!          <out_dir>/state_end.f32 (packed state, include/h9g.h) and, on a
!          grid (synth/pgf), <PATH_output>/axyYYYY.nc per year as
!          HYBRID9.f90:492-519 / WRITE_NET_CDF_3DR.f90 (nc_out = 1).
!----------------------------------------------------------------------!
USE, INTRINSIC :: ISO_C_BINDING
USE H9_GPU
IMPLICIT NONE

! --- driver.txt (INIT.f90:181-204) ---------------------------------------
CHARACTER (LEN = 200) :: PATH_output, LCLIM_filename, LSOIL_filename
INTEGER :: NISURF, iDEC_start, iDEC_end, syr, eyr, NYR_SPIN_UP
LOGICAL :: PGF, INTERACTIVE, LCLIM
REAL :: lon_w, lat_w, lon_c_w, lat_c_w
REAL(C_FLOAT) :: zi (0:H9G_LMAX+1)

! --- extension namelist ----------------------------------------------------
CHARACTER (LEN = 512) :: input_mode, case_dir, out_dir, pgf_dir
INTEGER :: nlayers, grow_on, device, grid, year0, nyears, nc_out, gnx, gny, gnland
INTEGER :: cell_order, ordered_decades
INTEGER(C_INT64_T) :: seed
NAMELIST /h9gpu/ input_mode, case_dir, out_dir, nlayers, grow_on, device, &
                 grid, year0, nyears, seed, pgf_dir, nc_out, gnx, gny, gnland, &
                 cell_order, ordered_decades
CHARACTER (LEN = 600, KIND = C_CHAR), TARGET :: pgf_file (7)
TYPE(C_PTR) :: pgf_ptr (7)
CHARACTER (LEN = *), PARAMETER :: pgf_var (7) = &
  (/ 'tas ', 'rlds', 'rsds', 'huss', 'ps  ', 'pr  ', 'rhs ' /)   ! READ_PGF.f90 order
REAL(C_FLOAT) :: zc (H9G_LMAX)
CHARACTER (LEN = 4) :: ydate

! --- case.nml of the harness (oracle/ref/h9ref_main.f90) -------------------
INTEGER :: ncell, state_override, ntrace, trace_cells (64), lclim_mode
NAMELIST /h9case/ ncell, NISURF, year0, nyears, grow_on, state_override, &
                  ntrace, trace_cells, lclim_mode, cell_order

TYPE(h9g_config) :: cfg
TYPE(C_PTR) :: ctx
INTEGER(C_INT) :: rc
INTEGER :: L, ndays, iyr, jyear, nt, d0, u, i, nslot, nland, nx, ny
INTEGER :: dsyr, deyr, ndec, k
INTEGER(C_INT32_T), ALLOCATABLE :: slots (:), passes (:)
LOGICAL :: have_driver, have_nml
CHARACTER (LEN = 512) :: arg
REAL(C_FLOAT), ALLOCATABLE :: theta_s (:,:), hksat (:,:), bsw (:,:), psi_s (:,:)
REAL(C_FLOAT), ALLOCATABLE :: Fmax (:), forcing (:,:,:), state (:), annual (:,:), annual_dec (:,:,:)
INTEGER(C_INT64_T), ALLOCATABLE :: gid (:)
REAL(C_FLOAT), ALLOCATABLE :: lat (:)
REAL(C_DOUBLE) :: diag (H9G_NDIAG)
TYPE(h9g_error) :: err
INTEGER :: time_BOY (2300-1860+1)

!----------------------------------------------------------------------!
! Defaults, then driver.txt and h9gpu.nml.
!----------------------------------------------------------------------!
input_mode = 'synth'; case_dir = ''; out_dir = '.'; pgf_dir = '.'
nlayers = 8; grow_on = 1; device = 0; grid = 1; year0 = 0; nyears = 0
nc_out = 1; gnx = 0; gny = 0; gnland = 0; cell_order = 1; ordered_decades = 0
PATH_output = '.'
seed = 20161123_C_INT64_T
NISURF = 48; iDEC_start = 1; iDEC_end = 1
zi = 0.0
zi (0:9) = (/ 0.0, 45.0, 91.0, 166.0, 289.0, 493.0, 829.0, 1383.0, 2296.0, 5000.0 /)

arg = 'driver.txt'
IF (COMMAND_ARGUMENT_COUNT () >= 1) CALL GET_COMMAND_ARGUMENT (1, arg)
INQUIRE (FILE = TRIM (arg), EXIST = have_driver)
IF (have_driver) CALL read_driver (TRIM (arg))
arg = 'h9gpu.nml'
IF (COMMAND_ARGUMENT_COUNT () >= 2) CALL GET_COMMAND_ARGUMENT (2, arg)
INQUIRE (FILE = TRIM (arg), EXIST = have_nml)
IF (have_nml) THEN
  OPEN (NEWUNIT = u, FILE = TRIM (arg), STATUS = 'OLD')
  READ (u, NML = h9gpu)
  CLOSE (u)
END IF

!----------------------------------------------------------------------!
! Calendar (INIT.f90:844-859).
!----------------------------------------------------------------------!
time_BOY (1) = 1
DO jyear = 1861, 2300
  IF (MOD (jyear-1,4) .NE. 0) THEN
    time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 365
  ELSE IF (MOD (jyear-1, 100) .NE. 0) THEN
    time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 366
  ELSE IF (MOD (jyear-1, 400) .NE. 0) THEN
    time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 365
  ELSE
    time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 366
  END IF
END DO

!----------------------------------------------------------------------!
! Inputs.
!----------------------------------------------------------------------!
state_override = 0
IF (TRIM (input_mode) == 'case') THEN
  ncell = 0; ntrace = 0; trace_cells = 0; lclim_mode = 0
  OPEN (NEWUNIT = u, FILE = TRIM (case_dir)//'/case.nml', STATUS = 'OLD')
  READ (u, NML = h9case)
  CLOSE (u)
  IF (lclim_mode /= 0) STOP 'h9_host: LCLIM cases run through h9g_run_site (hybrid9_amd.site)'

  nlayers = 8
  L = nlayers
  OPEN (NEWUNIT = u, FILE = TRIM (case_dir)//'/zi.f32', ACCESS = 'STREAM', &
        FORM = 'UNFORMATTED', STATUS = 'OLD')
  READ (u) zi (0:L+1)
  CLOSE (u)
  ALLOCATE (theta_s (L,ncell), hksat (L,ncell), bsw (L,ncell), psi_s (L,ncell))
  ALLOCATE (Fmax (ncell))
  OPEN (NEWUNIT = u, FILE = TRIM (case_dir)//'/params.f32', ACCESS = 'STREAM', &
        FORM = 'UNFORMATTED', STATUS = 'OLD')
  READ (u) theta_s, hksat, bsw, psi_s, Fmax
  CLOSE (u)
  ndays = time_BOY (year0+nyears-1859) - time_BOY (year0-1859)
  ALLOCATE (forcing (ncell, ndays, 7))
  OPEN (NEWUNIT = u, FILE = TRIM (case_dir)//'/forcing.f32', ACCESS = 'STREAM', &
        FORM = 'UNFORMATTED', STATUS = 'OLD')
  READ (u) forcing
  CLOSE (u)
ELSE
  ! synthetic land grid (SURVEY.md §8d): 0.5 deg = 67,420 cells, 0.25 deg
  ! = 270,000 cells with 10 layers
  IF (grid == 1) THEN
    nx = 720; ny = 360; nland = 67420
  ELSE
    nx = 1440; ny = 720; nland = 270000
  END IF
  IF (gnx > 0) nx = gnx
  IF (gny > 0) ny = gny
  IF (gnland > 0) nland = gnland
  ncell = nland
  L = nlayers
  IF (L == 10 .AND. grid == 1 .AND. gnx == 0) STOP 'h9_host: L=10 uses the 0.25 deg grid'
  IF (L == 10) zi (0:11) = (/ 0.0, 18.0, 45.0, 91.0, 166.0, 289.0, 493.0, &
                              829.0, 1383.0, 2296.0, 3500.0, 5000.0 /)
  ALLOCATE (gid (ncell), lat (ncell))
  rc = h9g_land_cells (nx, ny, nland, seed, gid, lat)
  IF (rc /= 0) STOP 'h9_host: h9g_land_cells failed'
  IF (year0 == 0) year0 = (iDEC_start - 1) * 10 + 1901        ! HYBRID9.f90:103
  IF (nyears == 0) THEN                                        ! HYBRID9.f90:109-113
    eyr = (iDEC_end - 1) * 10 + 1901 + MERGE (9, 1, iDEC_end < 12)
    nyears = eyr - year0 + 1
  END IF
END IF

! layer centre depths for the output (INIT.f90:252-263, zc_o)
DO i = 1, L
  zc (i) = zi (i) - (zi (i) - zi (i-1)) / 2.0
END DO

!----------------------------------------------------------------------!
! GPU context.
!----------------------------------------------------------------------!
nslot = 2                                  ! isolated cells: double-buffered years
IF (cell_order /= 0) THEN                  ! the reference's order: every year of a call resident
  nslot = nyears
  IF (ordered_decades > 0) nslot = MIN (nyears, 10 * ordered_decades)
END IF
cfg%ncell = ncell
cfg%nlayers = L
cfg%nisurf = NISURF
cfg%grow_on = grow_on
cfg%max_days = 366
cfg%nslots = nslot
cfg%zi = zi
IF (h9g_abi_version () /= 1) STOP 'h9_host: libh9g ABI mismatch'
IF (h9g_device_count () < 1) STOP 'h9_host: no GPU visible'
ctx = h9g_create (cfg, device)
IF (.NOT. C_ASSOCIATED (ctx)) STOP 'h9_host: h9g_create failed'

IF (TRIM (input_mode) == 'case') THEN
  CALL chk (h9g_set_params (ctx, theta_s, hksat, bsw, psi_s, Fmax))
  IF (state_override /= 0) THEN
    ALLOCATE (state (h9g_state_size (L) * ncell))
    OPEN (NEWUNIT = u, FILE = TRIM (case_dir)//'/state0.f32', ACCESS = 'STREAM', &
          FORM = 'UNFORMATTED', STATUS = 'OLD')
    READ (u) state
    CLOSE (u)
    CALL chk (h9g_set_state (ctx, state))
    DEALLOCATE (state)
  ELSE
    CALL chk (h9g_init_state (ctx))                ! INIT.f90:707-811
  END IF
ELSE
  CALL chk (h9g_set_cells (ctx, gid, lat))
  CALL chk (h9g_synth_params (ctx, seed))
  CALL chk (h9g_init_state (ctx))
END IF

!----------------------------------------------------------------------!
! Year loop: the GPU replaces HYBRID9.f90:120-295.  Forcing for year y+1
! is pushed (async) into the other slot while year y runs.
!----------------------------------------------------------------------!
ALLOCATE (annual (ncell, 12 + L))
OPEN (NEWUNIT = u, FILE = TRIM (out_dir)//'/annual.f32', ACCESS = 'STREAM', &
      FORM = 'UNFORMATTED', STATUS = 'REPLACE')
d0 = 1
IF (cell_order /= 0) THEN
  ! HYBRID9.f90:93-130: decade by decade (1901-1910, 1911-1920, ...), cut to
  ! [year0, year0 + nyears); a call's years staged into their slots, then
  ! the cells run in the reference's order, the decades overlapping
  ALLOCATE (annual_dec (ncell, 12 + L, nslot), slots (nslot), passes (nslot / 10 + 2))
  dsyr = year0
  DO WHILE (dsyr < year0 + nyears)
    ! the call's last year: ordered_decades whole decades on from dsyr's
    ! (FLOOR, not integer division, which truncates toward zero: before 1901
    ! the decades are 1891-1900, 1881-1890, ...)
    deyr = year0 + nyears - 1
    IF (ordered_decades > 0) &
      deyr = MIN (deyr, 1901 + 10 * (FLOOR (REAL (dsyr - 1901) / 10.0) + ordered_decades) - 1)
    ndec = deyr - dsyr + 1                   ! years of the call
    DO k = 1, ndec
      slots (k) = k - 1
      CALL stage (k - 1, dsyr + k - 1, d0)
      d0 = d0 + time_BOY (dsyr+k-1859) - time_BOY (dsyr+k-1-1859)
    END DO
    rc = h9g_run_ordered (ctx, slots, dsyr, ndec, annual_dec, passes)
    IF (rc < 0) CALL h9g_check_stop (ctx, rc)
    iyr = ndec
    IF (rc > 0) THEN                         ! a STOP: the reference ends in its decade,
      CALL chk (h9g_last_error (ctx, err))   ! after writing the decades before it
      iyr = 1901 + 10 * FLOOR (REAL (err%year - 1901) / 10.0) - dsyr
    END IF
    DO k = 1, iyr
      annual = annual_dec (:, :, k)
      CALL year_out (dsyr + k - 1)
    END DO
    CALL h9g_check_stop (ctx, rc)
    WRITE (*,'(A,I5,A,I5,A,12I3)') ' years', dsyr, ' -', deyr, ' in cell order: passes per decade', &
          passes (1:FLOOR (REAL (deyr - 1901) / 10.0) - FLOOR (REAL (dsyr - 1901) / 10.0) + 1)
    dsyr = deyr + 1
  END DO
ELSE
CALL stage (0, year0, d0)
DO iyr = 1, nyears
  jyear = year0 + iyr - 1
  nt = time_BOY (jyear+1-1859) - time_BOY (jyear-1859)
  CALL chk (h9g_run_year (ctx, MOD (iyr-1, nslot), jyear))
  IF (iyr < nyears) CALL stage (MOD (iyr, nslot), jyear + 1, d0 + nt)
  rc = h9g_sync (ctx)
  CALL h9g_check_stop (ctx, rc)
  CALL chk (h9g_get_annual (ctx, annual))
  CALL year_out (jyear)
  d0 = d0 + nt
END DO
END IF
CLOSE (u)
ALLOCATE (state (h9g_state_size (L) * ncell))
CALL chk (h9g_get_state (ctx, state))
OPEN (NEWUNIT = u, FILE = TRIM (out_dir)//'/state_end.f32', ACCESS = 'STREAM', &
      FORM = 'UNFORMATTED', STATUS = 'REPLACE')
WRITE (u) state
CLOSE (u)
CALL h9g_destroy (ctx)
WRITE (*,*) 'H9_HOST completed successfully'

CONTAINS

  ! One year's annual means to annual.f32 and axyYYYY.nc, and its line.
  SUBROUTINE year_out (y)
    INTEGER, INTENT(IN) :: y
    WRITE (u) annual
    IF (nc_out /= 0 .AND. TRIM (input_mode) /= 'case') THEN     ! HYBRID9.f90:503-513
      WRITE (ydate,'(I4)') y
      CALL chk (h9g_write_axy_nc (TRIM (PATH_output)//'/axy'//ydate//'.nc'//C_NULL_CHAR, nx, ny, L, &
                                  zc, ncell, gid, annual))
    END IF
    CALL chk (h9g_get_diagnostics (ctx, diag, C_NULL_PTR))    ! (in cell order: the decade's last year)
    WRITE (*,'(A,I5,A,I8,A,ES12.5,A,ES12.5,A,F9.1,A)') ' year', y, ' cells', NINT (diag (1)), &
          ' mean runoff', diag (2) / MAX (diag (1), 1.0D0), ' mm/s  mean soil water', &
          diag (3) / MAX (diag (1), 1.0D0), ' mm  (', h9g_last_kernel_ms (ctx), ' ms)'
  END SUBROUTINE year_out

  SUBROUTINE chk (r)
    INTEGER(C_INT), INTENT(IN) :: r
    IF (r /= 0) CALL h9g_check_stop (ctx, r)
  END SUBROUTINE chk

  ! Forcing of calendar year y into slot s (READ_PGF.f90 equivalent).
  SUBROUTINE stage (s, y, dfirst)
    INTEGER, INTENT(IN) :: s, y, dfirst
    INTEGER :: n
    INTEGER :: idec, dsyr, deyr, k
    CHARACTER (LEN = 9) :: decade
    n = time_BOY (y+1-1859) - time_BOY (y-1859)
    IF (TRIM (input_mode) == 'case') THEN
      CALL chk (h9g_push_forcing (ctx, s, n, forcing (:, dfirst:dfirst+n-1, :), 0))
    ELSE IF (TRIM (input_mode) == 'pgf') THEN
      ! decade files of READ_PGF.f90:22-106; day index within the file
      idec = (y - 1901) / 10 + 1
      dsyr = (idec - 1) * 10 + 1901
      deyr = MERGE (dsyr + 9, dsyr + 1, idec < 12)
      WRITE (decade,'(I4,A,I4)') dsyr, '_', deyr
      DO k = 1, 7
        pgf_file (k) = TRIM (pgf_dir)//'/'//TRIM (pgf_var (k))//'_pgfv2.1_'//decade//'.nc4'//C_NULL_CHAR
        pgf_ptr (k) = C_LOC (pgf_file (k))
      END DO
      CALL chk (h9g_nc_forcing_prefetch (ctx, s, pgf_ptr, nx, ny, &
                                         time_BOY (y-1859) - time_BOY (dsyr-1859), n))
    ELSE
      CALL chk (h9g_synth_forcing (ctx, s, seed, time_BOY (y-1859) - time_BOY (1901-1859), n))
    END IF
  END SUBROUTINE stage

  ! INIT.f90:181-204 list-directed read of driver.txt.
  SUBROUTINE read_driver (fname)
    CHARACTER (LEN = *), INTENT(IN) :: fname
    INTEGER :: v, k
    OPEN (NEWUNIT = v, FILE = fname, STATUS = 'OLD')
    READ (v,*) PATH_output
    READ (v,*) NISURF
    READ (v,*) PGF
    READ (v,*) iDEC_start
    READ (v,*) iDEC_end
    READ (v,*) INTERACTIVE
    READ (v,*) LCLIM
    READ (v,*) LCLIM_filename
    READ (v,*) LSOIL_filename
    READ (v,*) syr
    READ (v,*) eyr
    READ (v,*) NYR_SPIN_UP
    READ (v,*) lon_w
    READ (v,*) lat_w
    READ (v,*) lon_c_w
    READ (v,*) lat_c_w
    DO k = 0, 9
      READ (v,*) zi (k)
    END DO
    CLOSE (v)
    IF (.NOT. PGF) STOP 'h9_host: only the PGF path (HYBRID9.f90:87-337) is supported'
  END SUBROUTINE read_driver

END PROGRAM H9_HOST
!======================================================================!
