!======================================================================!
PROGRAM H9REF
!----------------------------------------------------------------------!
! TEST INFRASTRUCTURE ONLY -- never shipped, never timed as the product.
!
! Golden-vector harness around the UNMODIFIED reference subroutines
! HYDROLOGY (/root/reference/SOURCE/HYDROLOGY.f90) and GROW
! (/root/reference/SOURCE/GROW.f90), compiled from where they lie by
! oracle/Makefile together with the reference modules SHARED and
! CONTROL.  This file is our own code: it restates
!   * the state initialisation of INIT.f90:214,252-263,707-811,844-859
!   * the PGF cell/year/day/substep loop of HYBRID9.f90:120-290
! reading synthetic inputs from raw little-endian files instead of
! NetCDF (INIT.f90:473-680 and READ_PGF.f90 need libnetcdf, absent).
!
! Semantics pinned here (documented in DESIGN.md):
!   * isolated-cell: the module array smp (SHARED.f90:198) is reset to
!     0 (or to the per-cell smp of the state file) before each cell, so
!     results do not depend on cell order (SURVEY.md §7 hard part 3);
!   * one slab covers the whole run (READ_PGF decade slabs are an I/O
!     detail; iT is relative to the first simulated year);
!   * grow_on=0 skips CALL GROW (hydrology-only configs, as the LCLIM
!     path does at HYBRID9.f90:475).
!
! cell_order /= 0 instead runs the reference's own order and semantics:
! decade -> cell (y, x) -> year (HYBRID9.f90:93-130, decades 1901-1910,
! 1911-1920, ...), with the module array smp NOT reset between cells, so
! every cell's first substep of a decade computes beta (HYDROLOGY.f90:
! 270-275) from the smp its predecessor in cell order left behind
! (SHARED.f90:198).  The first land cell takes the smp the last land cell
! holds at the start (so from the second decade on, what it left behind;
! at a fresh start every smp is 0 -- the reference leaves smp
! uninitialised, INIT.f90:109).  The per-cell smp written to state_end is
! the smp each cell left behind at the end of its last decade.
!
! lclim_mode /= 0 restates instead the LCLIM single-site path of
! HYBRID9.f90:339-480: sub-daily forcing (tak, rh, Rnet, PAR, ppt per
! substep, :428-439), daily huss and ps (:377-378), the day-of-year LAI
! schedule (:380-417, given as (LAI, a, b): LAI = LAI; LAI_litter =
! LAI_litter + a - b), no GROW (:475), and the daily diagnostics of
! :464-469 (evap_day, evap_grnd_day, theta(1:4), theta_ma(1), LAI,
! LAI_litter, w_i, fT) instead of annual means.
!
! Files in <dir> (see oracle/README.md for the byte layout):
!   case.nml  namelist /h9case/
!   zi.f32    zi(0:Nlevgrnd)                       (Nlevgrnd+1 floats)
!   params.f32 theta_s,hksat,bsw,psi_s (L,ncell) then Fmax (ncell)
!   forcing.f32 tas,rlds,rsds,huss,ps,pr,rhs each (ncell,ndays)
!   state0.f32 (optional) full per-cell state, layout as state_end
! Outputs to <dir>: annual.f32, state_end.f32, trace.f32 (if ntrace>0)
!----------------------------------------------------------------------!
USE CONTROL
USE SHARED
IMPLICIT NONE

INTEGER :: ncell, year0, nyears, grow_on, state_override, ntrace, lclim_mode
INTEGER :: cell_order, dsyr, deyr
REAL, ALLOCATABLE :: lsub (:,:,:), lday (:,:,:), llai (:,:,:), out_day (:,:,:)
INTEGER :: trace_cells (64)
INTEGER :: ndays, iyr, itr, L, u, ios
LOGICAL :: do_trace
CHARACTER (LEN=1024) :: dir
REAL :: decay
REAL, ALLOCATABLE :: fz (:)
REAL, ALLOCATABLE :: out_ann (:,:,:)   ! (ncell, nfield, nyears)
REAL, ALLOCATABLE :: trace_buf (:)
! Annual sums (HYBRID9.f90:64-73)
REAL :: npp_sum, plant_mass_sum, tas_sum, rlds_sum, rsds_sum, huss_sum
REAL :: ps_sum, pr_sum, rhs_sum, h2osoi_sum_total
INTEGER :: nfield

NAMELIST /h9case/ ncell, NISURF, year0, nyears, grow_on, &
                  state_override, ntrace, trace_cells, lclim_mode, cell_order

CALL GET_COMMAND_ARGUMENT (1, dir)
IF (LEN_TRIM (dir) == 0) STOP 'usage: h9ref <casedir>'

ncell = 0; NISURF = 48; year0 = 1901; nyears = 1; grow_on = 1
state_override = 0; ntrace = 0; trace_cells = 0; lclim_mode = 0
cell_order = 0
OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/case.nml', STATUS='OLD')
READ (u, NML=h9case)
CLOSE (u)

!----------------------------------------------------------------------!
! Scratch / module allocations as INIT.f90:56-135.
!----------------------------------------------------------------------!
ALLOCATE (sla (nGPTs)); sla (1) = 23.0E-3
ALLOCATE (theta_sum (nsoil_layers_max))
ALLOCATE (qin (nsoil_layers_max+1), qout (nsoil_layers_max+1))
ALLOCATE (dsmpdw (nsoil_layers_max+1), dqodw1 (nsoil_layers_max+1))
ALLOCATE (dqodw2 (nsoil_layers_max+1), dhkdw (nsoil_layers_max))
ALLOCATE (dqidw0 (nsoil_layers_max+1), dqidw1 (nsoil_layers_max+1))
ALLOCATE (amx (nsoil_layers_max+1), bmx (nsoil_layers_max+1))
ALLOCATE (cmx (nsoil_layers_max+1), rmx (nsoil_layers_max+1))
ALLOCATE (dwat2 (nsoil_layers_max+1), dwat (nsoil_layers_max))
ALLOCATE (GAM (nsoil_layers_max+1))
ALLOCATE (zi (0:Nlevgrnd), dz (1:Nlevgrnd), zc_o (1:nsoil_layers_max))
ALLOCATE (zc (1:Nlevgrnd), smp (nsoil_layers_max))
ALLOCATE (zq (nsoil_layers_max+1), theta (nsoil_layers_max))
ALLOCATE (theta_ma (nsoil_layers_max), S (nsoil_layers_max))
ALLOCATE (vol_eq (nsoil_layers_max+1), eff_porosity (nsoil_layers_max))
ALLOCATE (hk (nsoil_layers_max), rnff (nsoil_layers_max+1))

!----------------------------------------------------------------------!
! Layer geometry (INIT.f90:202-204,252-263) and dt (INIT.f90:214).
!----------------------------------------------------------------------!
OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/zi.f32', ACCESS='STREAM', &
      FORM='UNFORMATTED', STATUS='OLD')
READ (u) zi (0:Nlevgrnd)
CLOSE (u)
dt = 86400.0 / FLOAT (NISURF)
DO I = 1, Nlevgrnd
  dz (I) = zi (I) - zi (I-1)
END DO
DO I = 1, Nlevgrnd
  zc (I) = zi (I) - dz (I) / 2.0
END DO
DO I = 1, nsoil_layers_max
  zc_o (I) = zc (I)
END DO

!----------------------------------------------------------------------!
! Calendar (INIT.f90:844-859).
!----------------------------------------------------------------------!
time_BOY (1) = 1
DO jyear = 1861, 2300
  IF (MOD (jyear-1,4) .NE. 0) THEN
    time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 365
  ELSE
    IF (MOD (jyear-1, 100) .NE. 0) THEN
      time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 366
    ELSE
      IF (MOD (jyear-1, 400) .NE. 0) THEN
        time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 365
      ELSE
        time_BOY (jyear-1859) = time_BOY (jyear-1859-1) + 366
      END IF
    END IF
  END IF
END DO
syr = year0
eyr = year0 + nyears - 1
iDEC_start = 1
NTIMES = time_BOY (eyr+1-1859) - time_BOY (syr-1859)
ndays = NTIMES

!----------------------------------------------------------------------!
! Per-cell arrays: the compacted land list is the x dimension.
!----------------------------------------------------------------------!
lon_c = ncell
lat_c = 1
L = nsoil_layers_max
ALLOCATE (plant_mass (nplants_max,lon_c,lat_c))
ALLOCATE (plant_foliage_mass (nplants_max,lon_c,lat_c))
ALLOCATE (plant_length (nplants_max,lon_c,lat_c))
ALLOCATE (rdepth (nplants_max,lon_c,lat_c))
ALLOCATE (nplants (lon_c,lat_c), LAI (lon_c,lat_c), LAI_litter (lon_c,lat_c))
ALLOCATE (rootr_col (1:Nlevgrnd,lon_c,lat_c))
ALLOCATE (Fmax (lon_c,lat_c))
! lon/lat are only printed by the reference's STOP diagnostics
! (HYDROLOGY.f90:810,823,1250): cell index and 0 here.
ALLOCATE (lon (lon_c), lat (lat_c))
DO I = 1, lon_c
  lon (I) = FLOAT (I)
END DO
lat = zero
my_id = 0
ALLOCATE (h2osoi_liq (L,lon_c,lat_c), h2osoi_liq_ma (L,lon_c,lat_c))
ALLOCATE (zwt (lon_c,lat_c), wa (lon_c,lat_c))
ALLOCATE (theta_s (L,lon_c,lat_c), theta_ma_s (L,lon_c,lat_c))
ALLOCATE (hksat (L,lon_c,lat_c), bsw (L,lon_c,lat_c), psi_s (L,lon_c,lat_c))
ALLOCATE (theta_m (L,lon_c,lat_c))
ALLOCATE (tas (lon_c,lat_c,NTIMES), rlds (lon_c,lat_c,NTIMES))
ALLOCATE (rsds (lon_c,lat_c,NTIMES), huss (lon_c,lat_c,NTIMES))
ALLOCATE (ps (lon_c,lat_c,NTIMES), pr (lon_c,lat_c,NTIMES))
ALLOCATE (rhs (lon_c,lat_c,NTIMES))

OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/params.f32', ACCESS='STREAM', &
      FORM='UNFORMATTED', STATUS='OLD')
READ (u) theta_s, hksat, bsw, psi_s, Fmax
CLOSE (u)
IF (lclim_mode == 0) THEN
  OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/forcing.f32', ACCESS='STREAM', &
        FORM='UNFORMATTED', STATUS='OLD')
  READ (u) tas, rlds, rsds, huss, ps, pr, rhs
  CLOSE (u)
ELSE
  ! lclim_sub.f32: (ncell, 5, NISURF*ndays): tak(degC) rh Rnet PAR ppt(mm/step)
  ! lclim_day.f32: (ncell, 2, ndays): huss ps;  lclim_lai.f32: (ncell, 3, ndays)
  ALLOCATE (lsub (lon_c, 5, NISURF*NTIMES), lday (lon_c, 2, NTIMES))
  ALLOCATE (llai (lon_c, 3, NTIMES), out_day (lon_c, 11, NTIMES))
  OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/lclim_sub.f32', ACCESS='STREAM', &
        FORM='UNFORMATTED', STATUS='OLD')
  READ (u) lsub
  CLOSE (u)
  OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/lclim_day.f32', ACCESS='STREAM', &
        FORM='UNFORMATTED', STATUS='OLD')
  READ (u) lday
  CLOSE (u)
  OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/lclim_lai.f32', ACCESS='STREAM', &
        FORM='UNFORMATTED', STATUS='OLD')
  READ (u) llai
  CLOSE (u)
  DO I = 1, NTIMES
    huss (:,1,I) = lday (:,1,I)
    ps (:,1,I) = lday (:,2,I)
  END DO
  tas = zero; rlds = zero; rsds = zero; pr = zero; rhs = zero
  out_day = zero
END IF

!----------------------------------------------------------------------!
! Initial state (INIT.f90:707-811), macroporosity 0.1 (INIT.f90:620).
!----------------------------------------------------------------------!
theta_ma_s = 0.1
theta_m = zero
h2osoi_liq = zero
h2osoi_liq_ma = zero
plant_mass = zero
zwt = zero
wa = zero
nlayers = nsoil_layers_max
DO y = 1, lat_c
  DO x = 1, lon_c
    DO I = 1, nsoil_layers_max
      h2osoi_liq (I,x,y) = 0.4 * theta_s (I,x,y) * dz (I) * rhow &
                           / 1000.0
      h2osoi_liq_ma (I,x,y) = 0.4 * theta_ma_s (I,x,y) * dz (I) * &
                              rhow / 1000.0
    END DO
    zwt (x,y) = (zi (nlayers) + 5000.0) / 1000.0
    wa (x,y) = 4000.0
    LAI_litter (x,y) = 0.001
    nplants (x,y) = 1
    LAI (x,y) = zero
    rootr_col (:,x,y) = zero
    DO K = 1, nplants (x,y)
      iGPT = 1
      plant_mass         (K,x,y) = 1.0
      plant_foliage_mass (K,x,y) = 0.0435
      plant_length (K,x,y) = (400.0 * plant_mass (K,x,y) / &
                             3.142E-3) ** (one / 3.0)
      LAI (x,y) = LAI (x,y) + &
                  plant_foliage_mass (K,x,y) * sla (iGPT) / plot_area
      rdepth (K,x,y) = 0.3 * plant_length (K,x,y)
      decay = EXP (LOG (0.1) / (rdepth (K,x,y) / 10.0))
      DO I = 1, nlayers
        rootr_col (I,x,y) = rootr_col (I,x,y) + &
                    (1.0 - decay ** (zi (I) / 10.0)) - &
                    (1.0 - decay ** (zi (I-1) / 10.0))
      END DO
    END DO
  END DO
END DO

!----------------------------------------------------------------------!
! Optional full-state override (edge-case fixtures).  smp0 keeps the
! per-cell hidden smp for the isolated-cell reset below.
!----------------------------------------------------------------------!
ALLOCATE (fz (L*lon_c))
fz = zero
IF (state_override /= 0) THEN
  OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/state0.f32', ACCESS='STREAM', &
        FORM='UNFORMATTED', STATUS='OLD')
  READ (u) h2osoi_liq, h2osoi_liq_ma, fz, rootr_col, zwt, wa, LAI, &
           LAI_litter, plant_mass, plant_foliage_mass, plant_length, rdepth
  CLOSE (u)
END IF

nfield = 12 + L
ALLOCATE (out_ann (lon_c, nfield, nyears))
out_ann = zero
ALLOCATE (trace_buf (3*L+7))
IF (ntrace > 0) THEN
  OPEN (NEWUNIT=itr, FILE=TRIM(dir)//'/trace.f32', ACCESS='STREAM', &
        FORM='UNFORMATTED', STATUS='REPLACE')
END IF
npp = zero

!----------------------------------------------------------------------!
! LCLIM single-site path, restating HYBRID9.f90:353-478 for every cell.
!----------------------------------------------------------------------!
IF (lclim_mode /= 0) THEN
DO y = 1, lat_c
  DO x = 1, lon_c
    IF (SUM (theta_s (:,x,y)) > trunc) THEN
      smp (:) = fz ((x-1)*L+1 : x*L)          ! isolated-cell semantics
      nlayers = nsoil_layers_max
      DO jyear = syr, eyr
        DO iTIME = time_BOY (jyear-1859), time_BOY (jyear+1-1859) - 1
          iT = iTIME-time_BOY(syr-1859) + 1
          IF (llai (x,1,iT) == llai (x,1,iT)) LAI (x,y) = llai (x,1,iT)          ! :380-417
          IF (llai (x,2,iT) == llai (x,2,iT)) &
            LAI_litter (x,y) = LAI_litter (x,y) + llai (x,2,iT) - llai (x,3,iT)
          evap_day = zero
          evap_grnd_day = zero
          DO NS = 1, NISURF
            tak  = lsub (x,1,(iT-1)*NISURF+NS) + tf                               ! :430-439
            rh   = lsub (x,2,(iT-1)*NISURF+NS)
            Rnet = lsub (x,3,(iT-1)*NISURF+NS)
            PAR  = lsub (x,4,(iT-1)*NISURF+NS)
            ppt  = lsub (x,5,(iT-1)*NISURF+NS) / dt
            forc_rain = ppt
            lamb = ((2503.0 - 2.386 * (tak - tf))) * 1.0E3                        ! :445
            CALL HYDROLOGY                                                         ! :453
            evap_day = evap_day + (qflx_evap_grnd + qflx_tran_veg_col) * dt        ! :457
            evap_grnd_day = evap_grnd_day + qflx_evap_grnd * dt                    ! :458
          END DO
          out_day (x, 1, iT) = evap_day                                           ! :464-469
          out_day (x, 2, iT) = evap_grnd_day
          out_day (x, 3:6, iT) = theta (1:4)
          out_day (x, 7, iT) = theta_ma (1)
          out_day (x, 8, iT) = LAI (x,y)
          out_day (x, 9, iT) = LAI_litter (x,y)
          out_day (x, 10, iT) = w_i
          out_day (x, 11, iT) = fT
        END DO
      END DO
      fz ((x-1)*L+1 : x*L) = smp (:)
    END IF
  END DO
END DO
OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/daily.f32', ACCESS='STREAM', &
      FORM='UNFORMATTED', STATUS='REPLACE')
WRITE (u) out_day
CLOSE (u)
ELSE

!----------------------------------------------------------------------!
! Hot loops, restating HYBRID9.f90:120-290 (PGF path).  Isolated-cell
! semantics run every year of a cell at once; cell_order runs the
! reference's decade loop (HYBRID9.f90:93-130) around the cell loop.
!----------------------------------------------------------------------!
DO x = 1, lon_c                               ! cell_order: chain start,
  IF (SUM (theta_s (:,x,1)) > trunc) smp (:) = fz ((x-1)*L+1 : x*L)   ! last land cell
END DO
dsyr = syr
DO WHILE (dsyr <= eyr)
IF (cell_order /= 0) THEN
  deyr = MIN (1901 + 10 * ((dsyr - 1901) / 10) + 9, eyr)
ELSE
  deyr = eyr
END IF
DO y = 1, lat_c
  DO x = 1, lon_c
    IF (SUM (theta_s (:,x,y)) > trunc) THEN
      do_trace = ANY (trace_cells (1:MAX(ntrace,1)) == x) .AND. ntrace > 0
      IF (cell_order == 0) smp (:) = fz ((x-1)*L+1 : x*L)   ! isolated-cell semantics
      nlayers = nsoil_layers_max
      DO jyear = dsyr, deyr
        npp_sum        = zero
        plant_mass_sum = zero
        rnf_sum  = zero
        evap_sum = zero
        tas_sum  = zero
        rlds_sum = zero
        rsds_sum = zero
        huss_sum = zero
        ps_sum   = zero
        pr_sum   = zero
        rhs_sum  = zero
        h2osoi_sum_total = zero
        theta_sum (:) = zero
        DO iTIME = time_BOY (jyear-1859), time_BOY (jyear+1-1859) - 1
          iT = iTIME-time_BOY(syr-1859) + 1
          DOY = iTIME - time_BOY (jyear-1859) + 1
          tak = tas (x,y,iT)
          rh = rhs (x,y,iT)
          Rnet = 0.92 * rsds (x,y,iT) + rlds (x,y,iT) - &
                 stbo * tas (x,y,iT) ** 4
          PAR = 0.92 * rsds (x,y,iT) * 2.3
          ppt = pr (x,y,iT)
          forc_rain = 1.0E3 * pr (x,y,iT) / rhow
          lamb = ((2503.0 - 2.386 * (tak - tf))) * 1.0E3
          evap_day = zero
          evap_grnd_day = zero
          DO NS = 1, NISURF
            CALL HYDROLOGY
            evap_day = evap_day + &
                       (qflx_evap_grnd + qflx_tran_veg_col) * dt
            evap_grnd_day = evap_grnd_day + qflx_evap_grnd * dt
            IF (do_trace) THEN
              trace_buf (1:L) = h2osoi_liq (1:L,x,y)
              trace_buf (L+1:2*L) = smp (1:L)
              trace_buf (2*L+1:3*L) = theta (1:L)
              trace_buf (3*L+1) = zwt (x,y)
              trace_buf (3*L+2) = wa (x,y)
              trace_buf (3*L+3) = qflx_tran_veg_col
              trace_buf (3*L+4) = qflx_evap_grnd
              trace_buf (3*L+5) = rnf_sum
              trace_buf (3*L+6) = LAI (x,y)
              trace_buf (3*L+7) = LAI_litter (x,y)
              WRITE (itr) trace_buf
            END IF
          END DO
          IF (grow_on /= 0) CALL GROW
          tas_sum  = tas_sum  + tas  (x,y,iT)
          rlds_sum = rlds_sum + rlds (x,y,iT)
          rsds_sum = rsds_sum + rsds (x,y,iT)
          huss_sum = huss_sum + huss (x,y,iT)
          ps_sum   = ps_sum   + ps   (x,y,iT)
          pr_sum   = pr_sum   + pr   (x,y,iT)
          rhs_sum  = rhs_sum  + rhs  (x,y,iT)
          DO K = 1, nplants (x,y)
            plant_mass_sum = plant_mass_sum + plant_mass (K,x,y)
          END DO
          npp_sum = npp_sum + npp
          DO I = 1, nlayers
            theta_sum (I) = theta_sum (I) + theta (I)
            h2osoi_sum_total = h2osoi_sum_total + h2osoi_liq (I,x,y)
          END DO
        END DO
        nt = (time_BOY (jyear + 1 - 1859) - 1) - &
             (time_BOY (jyear - 1859)) + 1
        iyr = jyear - syr + 1
        out_ann (x, 1, iyr) = npp_sum
        out_ann (x, 2, iyr) = plant_mass_sum / FLOAT (nt)
        out_ann (x, 3, iyr) = rnf_sum  / FLOAT (nt * NISURF)
        out_ann (x, 4, iyr) = evap_sum / FLOAT (nt * NISURF)
        out_ann (x, 5, iyr) = tas_sum  / FLOAT (nt)
        out_ann (x, 6, iyr) = rlds_sum / FLOAT (nt)
        out_ann (x, 7, iyr) = rsds_sum / FLOAT (nt)
        out_ann (x, 8, iyr) = huss_sum / FLOAT (nt)
        out_ann (x, 9, iyr) = ps_sum   / FLOAT (nt)
        out_ann (x,10, iyr) = pr_sum   / FLOAT (nt)
        out_ann (x,11, iyr) = rhs_sum  / FLOAT (nt)
        DO I = 1, nlayers
          out_ann (x, 11+I, iyr) = theta_sum (I) / FLOAT (nt)
        END DO
        out_ann (x, 12+L, iyr) = h2osoi_sum_total / FLOAT (nt)
      END DO
      fz ((x-1)*L+1 : x*L) = smp (:)
    END IF
  END DO
END DO
dsyr = deyr + 1
END DO   ! decades

IF (ntrace > 0) CLOSE (itr)

OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/annual.f32', ACCESS='STREAM', &
      FORM='UNFORMATTED', STATUS='REPLACE')
WRITE (u) out_ann
CLOSE (u)
END IF   ! lclim
OPEN (NEWUNIT=u, FILE=TRIM(dir)//'/state_end.f32', ACCESS='STREAM', &
      FORM='UNFORMATTED', STATUS='REPLACE', IOSTAT=ios)
WRITE (u) h2osoi_liq, h2osoi_liq_ma, fz, rootr_col, zwt, wa, LAI, &
          LAI_litter, plant_mass, plant_foliage_mass, plant_length, rdepth
CLOSE (u)

END PROGRAM H9REF
!======================================================================!
