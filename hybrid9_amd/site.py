"""LCLIM single-site path (HYBRID9.f90:339-480) around ``Context.run_site``.

The reference's second driver mode runs HYDROLOGY for one site from local
climate files: a daily CSV (``LCLIM_filename``, ``INIT.f90:189``) and one
sub-daily CSV per year, with a hard-coded day-of-year LAI schedule for the
Vaira grassland and GROW switched off.  This module holds the host side:
reading those CSVs into the arrays ``h9g_run_site`` takes, the schedule as
data, the spin-up loop, the daily CSV writer, and a synthetic site
generator (the Vaira files are not shipped with the reference).

Array layouts ([row][cell], cell fastest, as every h9g array):
  sub   (nday*nisurf, 5, ncell)  tak (degC), rh (%), Rnet (W m-2), PAR, ppt (mm/substep)
  daily (nday, 2, ncell)         huss (kg/kg), ps (Pa)
  lai   (nday, 3, ncell)         (LAI, a, b): LAI = LAI; LAI_litter = LAI_litter + a - b
  diag  (nday, 11, ncell)        DIAG_FIELDS
"""
from __future__ import annotations

import re
from pathlib import Path

import numpy as np

from . import synth

DIAG_FIELDS = ("evap_day", "evap_grnd_day", "theta1", "theta2", "theta3", "theta4",
               "theta_ma1", "LAI", "LAI_litter", "w_i", "fT")      # HYBRID9.f90:464-469
SUB_COLUMNS = (22, 25, 14, 16, 35)     # LCLIM_array2 columns of tak, rh, Rnet, PAR, ppt (:430-435)
DAILY_COLUMNS = (5, 6)                 # LCLIM_array columns of huss, ps (:377-378)
NAN = np.float32(np.nan)

# HYBRID9.f90:380-417: (day of year, new LAI, litter increment) where the
# increment is applied as LAI_litter = LAI_litter + a - b.
_VAIRA = {
    2002: [(1, 0.88, None), (59, 1.17, None), (79, 1.87, None), (94, 2.23, None),
           (108, 2.55, None), (122, 1.43, (2.55, 1.43)), (136, 0.001, (1.43, 0.001)),
           (357, 0.61, None)],
    2003: [(29, 0.96, None), (52, 1.58, None), (76, 1.82, None), (95, 2.63, None),
           (106, 2.52, (2.63, 2.52)), (120, 1.86, (2.52, 1.86)), (141, 0.76, (1.86, 0.76)),
           (158, 0.001, (0.76, 0.001))],
}


def lai_schedule(years, events=None) -> np.ndarray:
    """(nday, 3) schedule over the calendar years ``years``; ``events`` maps
    year -> [(doy, LAI or None, (a, b) or None)], default the reference's
    Vaira 2002/2003 schedule (other years: no change)."""
    events = _VAIRA if events is None else events
    rows = []
    for y in years:
        r = np.full((synth.days_in_year(y), 3), NAN, dtype=np.float32)
        for doy, lai, lit in events.get(y, []):
            if lai is not None:
                r[doy - 1, 0] = lai
            if lit is not None:
                r[doy - 1, 1:] = lit
        rows.append(r)
    return np.concatenate(rows)


def broadcast(a: np.ndarray, ncell: int) -> np.ndarray:
    """One site's (T, k) array -> (T, k, ncell)."""
    return np.ascontiguousarray(np.repeat(np.asarray(a, np.float32)[:, :, None], ncell, axis=2))


_SPLIT = re.compile(r"[,\s]+")


def _records(path, width: int):
    """Fortran list-directed READ (u,*) of ``width`` values per record after
    one header line (:352, :360): values separated by commas or blanks, the
    rest of a line is discarded."""
    out = []
    with open(path) as f:
        next(f)
        for line in f:
            v = [t for t in _SPLIT.split(line.strip()) if t]
            if not v:
                continue
            out.append([float(t) for t in v[:width]])
    return np.asarray(out, dtype=np.float64)


def read_lclim(daily_csv, subdaily_csvs, years, nisurf: int):
    """The files of :348-360 -> (sub (nday*nisurf, 5), daily (nday, 2)) of one
    site.  ``subdaily_csvs`` = one file per year (as the Vaira 2002/2003 files)."""
    nday = sum(synth.days_in_year(y) for y in years)
    d = _records(daily_csv, 7)                  # iDOY, LCLIM_array(1:6)
    if d.shape[0] < nday:
        raise ValueError(f"{daily_csv}: {d.shape[0]} days, need {nday}")
    daily = d[:nday, [c for c in DAILY_COLUMNS]].astype(np.float32)
    subs = []
    for y, path in zip(years, subdaily_csvs):
        r = _records(path, 37)
        need = synth.days_in_year(y) * nisurf
        if r.shape[0] < need or r.shape[1] < max(SUB_COLUMNS):
            raise ValueError(f"{path}: need {need} records of >= {max(SUB_COLUMNS)} values")
        subs.append(r[:need, [c - 1 for c in SUB_COLUMNS]])
    return np.concatenate(subs).astype(np.float32), daily


def run_lclim(ctx, sub, daily, lai, nloop: int = 1):
    """The spin-up loop of :341 (each pass re-reads the same years); the
    state carries over.  Returns the diagnostics of every pass, stacked
    (nloop*nday, 11, ncell), as the CSV of :464-469 accumulates them."""
    return np.concatenate([ctx.run_site(sub, daily, lai) for _ in range(nloop)])


def write_daily_csv(path, diag, years, cell: int = 0, nloop: int = 1):
    """The daily lines of :464-469 (jyear, DOY, 11 values, F10.4) of one cell."""
    with open(path, "w") as f:
        k = 0
        for _ in range(nloop):
            for y in years:
                for doy in range(1, synth.days_in_year(y) + 1):
                    v = ",".join("%10.4f" % x for x in diag[k, :, cell])
                    f.write("%5d,%5d,%s\n" % (y, doy, v))
                    k += 1


# -------------------------------------------------------------------------
# synthetic sites (the LCLIM files are not available): a Mediterranean
# annual cycle (wet winter, dry summer) with diurnal radiation, from
# synth.u01 (platform-independent bits, no transcendental calls).
# -------------------------------------------------------------------------
S_SITE = 300
F32 = np.float32


def _tri(x):
    """+1 at x = 0.5 (mod 1), -1 at x = 0."""
    x = (x - np.floor(x)).astype(np.float32)
    return (F32(1.0) - F32(4.0) * np.abs(x - F32(0.5))).astype(np.float32)


def synth_site(nsite: int, nday: int, nisurf: int, seed: int = synth.SEED, doy0: int = 0):
    """Synthetic sub-daily and daily site forcing: (sub (nday*nisurf, 5, nsite),
    daily (nday, 2, nsite))."""
    site = np.arange(nsite, dtype=np.uint64)
    t = np.arange(nday * nisurf, dtype=np.int64)
    day = t // nisurf
    key = (t.astype(np.uint64)[:, None] << np.uint64(16)) | site[None, :]
    dkey = (day[::nisurf].astype(np.uint64)[:, None] << np.uint64(16)) | site[None, :]
    u = lambda k, kk=key: synth.u01(seed, S_SITE + k, kk)                      # noqa: E731
    summer = _tri(((day + doy0) % 365).astype(np.float32) / F32(365.0) - F32(0.05))[:, None]
    hour = ((t % nisurf).astype(np.float32) + F32(0.5)) / F32(nisurf)
    noon = _tri(hour)[:, None]                                   # +1 at local noon
    sun = np.maximum(F32(0.0), F32(1.6) * noon - F32(0.6))       # daylight ~ 12 h
    tak = F32(14.0) + F32(9.0) * summer + F32(6.0) * noon + F32(3.0) * (u(0) - F32(0.5))
    rh = np.clip(F32(62.0) - F32(22.0) * summer - F32(18.0) * noon + F32(24.0) * (u(1) - F32(0.5)),
                 F32(5.0), F32(100.0))
    cloud = F32(0.55) + F32(0.45) * u(2)
    Rnet = F32(-45.0) + F32(620.0) * sun * (F32(0.75) + F32(0.25) * summer) * cloud
    PAR = F32(2100.0) * sun * (F32(0.75) + F32(0.25) * summer) * cloud
    wetday = synth.u01(seed, S_SITE + 5, dkey) < (F32(0.35) - F32(0.3) * _tri(
        ((np.arange(nday) + doy0) % 365).astype(np.float32) / F32(365.0) - F32(0.05))[:, None])
    wet = np.repeat(wetday, nisurf, axis=0)
    u3 = u(3)
    ppt = np.where(wet & (u(4) < F32(0.12)), F32(3.0) * u3 * u3, F32(0.0))
    sub = np.stack([tak, rh, Rnet, PAR, ppt], axis=1).astype(np.float32)
    warm = (F32(0.55) + F32(0.45) * summer[::nisurf])
    huss = F32(0.003) + F32(0.007) * warm * synth.u01(seed, S_SITE + 6, dkey)
    ps = F32(100200.0) + F32(900.0) * (synth.u01(seed, S_SITE + 7, dkey) - F32(0.5))
    daily = np.stack([huss, ps], axis=1).astype(np.float32)
    assert sub.shape == (nday * nisurf, 5, nsite) and daily.shape == (nday, 2, nsite)
    return sub, daily
