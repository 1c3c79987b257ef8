"""hybrid9_amd -- MI355X-native HYBRID9 per-cell hydrology/vegetation hot path.

Python host mirror of the C-ABI in ``include/h9g.h`` (``lib/libh9g.so``,
built by ``hybrid9_amd.build``).  The reference has no Python surface: its
only "interface" is the driver loop ``HYBRID9.f90:120-295`` around the
argument-less ``SUBROUTINE HYDROLOGY``/``GROW``.  ``Context`` exposes that
loop one calendar year at a time, with the reference's array layouts and
STOP conditions (raised as :class:`ReferenceStop` carrying the first failing
cell, like the reference's diagnostics block ``HYDROLOGY.f90:1244-1274``).

There is no CPU fallback: if the HIP library is missing or cannot reach a
GPU, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "lib" / "libh9g.so"
if os.environ.get("H9G_LIB"):          # alternative build (e.g. the H9G_STAMPS profiling build)
    LIB_PATH = Path(os.environ["H9G_LIB"]).resolve()
NFORCING = 7
NANNUAL_SCALARS = 11
NDIAG = 12
ANNUAL_SCALARS = ("npp", "plant_mass", "rnf", "evap", "tas", "rlds", "rsds",
                  "huss", "ps", "pr", "rhs")
DIAG_NAMES = ("cells", "rnf_sum", "theta_total_sum", "zwt_sum", "wa_sum",
              "npp_sum", "plant_mass_sum", "lai_sum", "theta1_sum", "tas_sum",
              "pr_sum", "failed_cells")
STOP_MESSAGES = {  # HYDROLOGY.f90 STOP sites
    1: "Problem with tridiagonal 1.",            # :806-812
    2: "Problem with tridiagonal 2.",            # :818-825
    3: "rsub_top_tot is positive in drainage",   # :1068-1072
    4: "Problem in HYDROLOGY: Water imbalance > 0.1 mm",  # :1244-1274
    5: "internal: exact re-run requested with no day snapshot",   # H9G_ERR_NOSNAP (not a reference STOP)
}
LMAX = 10
MAX_SLOTS = 512          # H9G_MAX_SLOTS


class H9GError(RuntimeError):
    """API / HIP failure (negative return codes)."""


class ReferenceStop(RuntimeError):
    """A cell hit one of the reference's STOP conditions."""

    def __init__(self, err: dict):
        self.err = err
        msg = STOP_MESSAGES.get(err["code"], f"code {err['code']}")
        super().__init__(f"{msg} cell={err['cell']} year={err['year']} "
                         f"day={err['day']} substep={err['substep']} value={err['value']}")


class _Config(C.Structure):
    _fields_ = [("ncell", C.c_int32), ("nlayers", C.c_int32), ("nisurf", C.c_int32),
                ("grow_on", C.c_int32), ("max_days", C.c_int32), ("nslots", C.c_int32),
                ("zi", C.c_float * (LMAX + 2))]


class _Error(C.Structure):
    _fields_ = [("code", C.c_int32), ("cell", C.c_int32), ("year", C.c_int32),
                ("day", C.c_int32), ("substep", C.c_int32), ("value", C.c_float)]


_lib = None
_FP = C.POINTER(C.c_float)
_DP = C.POINTER(C.c_double)
_I64P = C.POINTER(C.c_int64)


def lib() -> C.CDLL:
    """Load libh9g.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise H9GError(f"{LIB_PATH} not built: run `python -m hybrid9_amd.build` "
                       "(or __graft_entry__.build())")
    L = C.CDLL(str(LIB_PATH))
    vp = C.c_void_p
    sig = {
        "h9g_abi_version": (C.c_int, []),
        "h9g_device_count": (C.c_int, []),
        "h9g_create": (vp, [C.POINTER(_Config), C.c_int]),
        "h9g_create_error": (C.c_char_p, []),
        "h9g_config_check": (C.c_int, [C.POINTER(_Config), C.c_char_p, C.c_int]),
        "h9g_config_bytes": (C.c_size_t, [C.POINTER(_Config)]),
        "h9g_destroy": (None, [vp]),
        "h9g_set_params": (C.c_int, [vp, _FP, _FP, _FP, _FP, _FP]),
        "h9g_init_state": (C.c_int, [vp]),
        "h9g_state_size": (C.c_int, [C.c_int]),
        "h9g_set_state": (C.c_int, [vp, _FP]),
        "h9g_get_state": (C.c_int, [vp, _FP]),
        "h9g_push_forcing": (C.c_int, [vp, C.c_int, C.c_int, _FP, C.c_int]),
        "h9g_push_forcing_device": (C.c_int, [vp, C.c_int, C.c_int, vp]),
        "h9g_forcing_slot": (vp, [vp, C.c_int]),
        "h9g_host_alloc": (vp, [C.c_size_t]),
        "h9g_host_free": (None, [vp]),
        "h9g_run_year": (C.c_int, [vp, C.c_int, C.c_int]),
        "h9g_run_decade_ordered": (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int, C.c_int, _FP,
                                             C.POINTER(C.c_int32)]),
        "h9g_run_ordered": (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int, C.c_int, _FP, C.POINTER(C.c_int32)]),
        "h9g_decade_stats": (C.c_int, [vp, C.POINTER(C.c_int64), C.c_int]),
        "h9g_ordered_stats": (C.c_int, [vp, C.POINTER(C.c_int64), C.c_int]),
        "h9g_launch_stats": (C.c_int, [vp, _DP, C.c_int, C.c_int]),
        "h9g_set_chains": (C.c_int, [vp, C.POINTER(C.c_int32)]),
        "h9g_sync": (C.c_int, [vp]),
        "h9g_last_error": (C.c_int, [vp, C.POINTER(_Error)]),
        "h9g_get_errors": (C.c_int, [vp, C.POINTER(C.c_int32)]),
        "h9g_get_annual": (C.c_int, [vp, _FP]),
        "h9g_get_diagnostics": (C.c_int, [vp, _DP, vp]),
        "h9g_get_diagnostics_async": (C.c_int, [vp, vp, vp]),
        "h9g_set_cells": (C.c_int, [vp, _I64P, _FP]),
        "h9g_synth_params": (C.c_int, [vp, C.c_uint64]),
        "h9g_synth_forcing": (C.c_int, [vp, C.c_int, C.c_uint64, C.c_int, C.c_int]),
        "h9g_last_kernel_ms": (C.c_float, [vp]),
        "h9g_total_kernel_ms": (C.c_double, [vp, C.c_int]),
        "h9g_kernel_name": (C.c_char_p, [vp]),
        "h9g_build_id": (C.c_char_p, []),
        "h9g_math_selftest": (C.c_int, [C.c_int, C.c_int, _FP, _FP, _FP]),
        "h9g_div_selftest": (C.c_int, [C.c_int, C.c_int, _FP, _FP, _FP, C.POINTER(C.c_int)]),
        "h9g_pace_probe": (C.c_int, [C.c_int, C.c_int, C.POINTER(C.c_uint)]),
        "h9g_math_fast_selftest": (C.c_int, [C.c_int, C.c_int, _FP, _FP, _FP, C.POINTER(C.c_int)]),
        "h9g_synth_host": (C.c_int, [C.c_uint64, C.c_int, C.c_int, _I64P, _FP, C.c_int,
                                     C.c_int, _FP, _FP]),
        "h9g_land_cells": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_uint64, _I64P, _FP]),
        "h9g_write_axy_nc": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int, _FP, C.c_int, _I64P, _FP]),
        "h9g_nc_forcing_read": (C.c_int, [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_int, _I64P,
                                          C.c_int, C.c_int, _FP]),
        "h9g_nc_ntimes": (C.c_int, [C.c_char_p]),
        "h9g_nc_read_stats": (C.c_int, [C.POINTER(C.c_double), C.c_int]),
        "h9g_nc_forcing_prefetch": (C.c_int, [vp, C.c_int, C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                              C.c_int, C.c_int]),
        "h9g_soil_layer": (C.c_int, [vp, C.c_int, vp, vp, vp, vp, C.c_int, C.c_int, C.c_int]),
        "h9g_soil_fmax": (C.c_int, [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_int, C.c_int]),
        "h9g_last_soil_ms": (C.c_float, [vp]),
        "h9g_last_soil_slow": (C.c_int, [vp]),
        "h9g_get_params": (C.c_int, [vp, _FP, _FP, _FP, _FP, _FP]),
        "h9g_run_site": (C.c_int, [vp, C.c_int, _FP, _FP, _FP, _FP]),
        "h9g_host_expf": (C.c_float, [C.c_float]),
        "h9g_host_powf": (C.c_float, [C.c_float, C.c_float]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.h9g_abi_version() != 1:
        raise H9GError("libh9g ABI mismatch")
    _lib = L
    return L


def build_id() -> str:
    """Digest of the sources and flags the loaded libh9g.so was built from
    (hybrid9_amd/build.py build_id); needs no GPU."""
    return lib().h9g_build_id().decode()


def exported_symbols():
    """Names every C-ABI entry point declared in include/h9g.h."""
    import re
    hdr = (HERE.parent / "include" / "h9g.h").read_text()
    return sorted(set(re.findall(r"\b(h9g_[a-z_0-9]+)\s*\(", hdr)))


def _fp(a):
    return a.ctypes.data_as(_FP)


def _check(rc, what):
    if rc < 0:
        raise H9GError(f"{what} failed with {rc}")
    return rc


def days_in_year(y: int) -> int:
    """INIT.f90:844-859 calendar (Gregorian)."""
    if y % 4:
        return 365
    if y % 100:
        return 366
    if y % 400:
        return 365
    return 366


def state_size(L: int) -> int:
    return 4 * L + 9


def make_config(ncell: int, zi, *, nlayers: int = 8, nisurf: int = 48, grow_on: bool = True,
                max_days: int = 366, nslots: int = 2) -> _Config:
    """The ``h9g_config`` of a context, validated on the host by
    ``h9g_config_check`` (no GPU needed); raises ValueError with its reason."""
    zi = np.asarray(zi, dtype=np.float32)
    if zi.size != nlayers + 2:
        raise ValueError(f"zi must hold zi(0:L+1) = {nlayers + 2} values")
    cfg = _Config()
    cfg.ncell, cfg.nlayers, cfg.nisurf = int(ncell), int(nlayers), int(nisurf)
    cfg.grow_on, cfg.max_days, cfg.nslots = int(bool(grow_on)), int(max_days), int(nslots)
    for i, v in enumerate(zi):
        cfg.zi[i] = float(v)
    why = C.create_string_buffer(256)
    if lib().h9g_config_check(C.byref(cfg), why, 256):
        raise ValueError(f"invalid h9g_config: {why.value.decode()}")
    return cfg


def config_bytes(cfg: _Config) -> int:
    """Device bytes a context of ``cfg`` allocates (h9g_config_bytes)."""
    return int(lib().h9g_config_bytes(C.byref(cfg)))


class Context:
    """One GPU, one shard of land cells (C-ABI ``h9g_ctx``)."""

    def __init__(self, ncell: int, zi, *, nlayers: int = 8, nisurf: int = 48,
                 grow_on: bool = True, max_days: int = 366, nslots: int = 2,
                 device: int = 0):
        lb = lib()
        zi = np.asarray(zi, dtype=np.float32)
        if zi.size != nlayers + 2:
            raise ValueError(f"zi must hold zi(0:L+1) = {nlayers + 2} values")
        cfg = make_config(ncell, zi, nlayers=nlayers, nisurf=nisurf, grow_on=grow_on,
                          max_days=max_days, nslots=nslots)
        self._lib = lb
        self.ncell, self.L, self.nisurf, self.grow_on = int(ncell), int(nlayers), int(nisurf), bool(grow_on)
        self.zi = zi
        self.device = device
        self._keep = {}
        self._h = lb.h9g_create(C.byref(cfg), int(device))
        if not self._h:
            why = (lb.h9g_create_error() or b"").decode() or "unknown"
            raise H9GError(f"h9g_create failed (ncell={ncell}, L={nlayers}, nslots={nslots}, "
                           f"device={device}): {why}")

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.h9g_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- parameters & state -----------------------------------------------
    def set_params(self, params: dict):
        """params: theta_s, hksat, bsw, psi_s as (ncell, L); fmax (ncell)."""
        arrs = [np.ascontiguousarray(params[k], dtype=np.float32)
                for k in ("theta_s", "hksat", "bsw", "psi_s", "fmax")]
        for a in arrs[:4]:
            assert a.shape == (self.ncell, self.L), a.shape
        assert arrs[4].shape == (self.ncell,)
        _check(self._lib.h9g_set_params(self._h, *[_fp(a) for a in arrs]), "h9g_set_params")

    def get_params(self) -> dict:
        out = {k: np.empty((self.ncell, self.L), np.float32) for k in ("theta_s", "hksat", "bsw", "psi_s")}
        out["fmax"] = np.empty(self.ncell, np.float32)
        _check(self._lib.h9g_get_params(self._h, *[_fp(out[k]) for k in
                                                   ("theta_s", "hksat", "bsw", "psi_s", "fmax")]),
               "h9g_get_params")
        return out

    def soil_layer(self, layer: int, ts, ks, lm, ps, nx: int, ny: int):
        """INIT.f90:575-631 for one layer: 30" fields as (ny*60, nx*60) float32
        host arrays, or device pointers (ints, e.g. tensor.data_ptr())."""
        if all(isinstance(a, int) for a in (ts, ks, lm, ps)):
            ptrs, dev = [C.c_void_p(a) for a in (ts, ks, lm, ps)], 1
        else:
            arrs = [np.ascontiguousarray(a, dtype=np.float32) for a in (ts, ks, lm, ps)]
            for a in arrs:
                assert a.shape == (ny * 60, nx * 60), a.shape
            ptrs, dev = [a.ctypes.data_as(C.c_void_p) for a in arrs], 0
        _check(self._lib.h9g_soil_layer(self._h, layer, *ptrs, nx, ny, dev), "h9g_soil_layer")
        return float(self._lib.h9g_last_soil_ms(self._h)), int(self._lib.h9g_last_soil_slow(self._h))

    def soil_fmax(self, soil_tex, fmax, nx: int, ny: int):
        """INIT.f90:661-680 (0.5 deg integer grids (ny, nx)); completes the parameters."""
        t = np.ascontiguousarray(soil_tex, dtype=np.int32)
        f = np.ascontiguousarray(fmax, dtype=np.int32)
        assert t.size == f.size == nx * ny
        i32 = C.POINTER(C.c_int32)
        _check(self._lib.h9g_soil_fmax(self._h, t.ctypes.data_as(i32), f.ctypes.data_as(i32), nx, ny),
               "h9g_soil_fmax")

    def init_state(self):
        _check(self._lib.h9g_init_state(self._h), "h9g_init_state")

    def set_state(self, packed: np.ndarray):
        packed = np.ascontiguousarray(packed, dtype=np.float32)
        assert packed.size == state_size(self.L) * self.ncell
        _check(self._lib.h9g_set_state(self._h, _fp(packed)), "h9g_set_state")

    def get_state(self) -> np.ndarray:
        out = np.empty(state_size(self.L) * self.ncell, dtype=np.float32)
        _check(self._lib.h9g_get_state(self._h, _fp(out)), "h9g_get_state")
        return out

    # -- forcing ----------------------------------------------------------
    def push_forcing(self, slot: int, forcing: np.ndarray, async_: bool = False):
        """forcing: (7, nday, ncell) float32 in READ_PGF order."""
        forcing = np.ascontiguousarray(forcing, dtype=np.float32)
        assert forcing.shape[0] == NFORCING and forcing.shape[2] == self.ncell, forcing.shape
        self._keep[slot] = forcing        # async copies read it after return
        _check(self._lib.h9g_push_forcing(self._h, slot, forcing.shape[1], _fp(forcing),
                                          int(async_)), "h9g_push_forcing")

    def nc_prefetch(self, slot: int, paths, nx: int, ny: int, t0: int, nt: int):
        """Async PGF prefetch from NetCDF files (READ_PGF.f90) into `slot`:
        days [t0, t0+nt) of the 7 files, needs set_cells."""
        _check(self._lib.h9g_nc_forcing_prefetch(self._h, slot, _paths(paths), nx, ny, t0, nt),
               "h9g_nc_forcing_prefetch")

    def push_forcing_device(self, slot: int, nday: int, dev_ptr: int):
        _check(self._lib.h9g_push_forcing_device(self._h, slot, nday, C.c_void_p(dev_ptr)),
               "h9g_push_forcing_device")

    def set_cells(self, gid, lat):
        gid = np.ascontiguousarray(gid, dtype=np.int64)
        lat = np.ascontiguousarray(lat, dtype=np.float32)
        assert gid.size == lat.size == self.ncell
        _check(self._lib.h9g_set_cells(self._h, gid.ctypes.data_as(_I64P), _fp(lat)),
               "h9g_set_cells")

    def synth_params(self, seed: int):
        _check(self._lib.h9g_synth_params(self._h, C.c_uint64(seed)), "h9g_synth_params")

    def synth_forcing(self, slot: int, seed: int, day0: int, nday: int):
        _check(self._lib.h9g_synth_forcing(self._h, slot, C.c_uint64(seed), day0, nday),
               "h9g_synth_forcing")

    # -- hot path ---------------------------------------------------------
    def run_year(self, slot: int, jyear: int):
        _check(self._lib.h9g_run_year(self._h, slot, jyear), "h9g_run_year")

    def run_decade_ordered(self, slots, jyear0: int, raise_on_stop: bool = True, annual: bool = True):
        """One decade of the reference's own cell order (h9g_run_decade_ordered:
        smp carried from cell to cell, HYBRID9.f90:93-130); synchronous.
        Returns (annual (nyears, 12+L, ncell) or None, passes);
        self.decade_rc holds the STOP code."""
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        out = np.empty((sl.size, 12 + self.L, self.ncell), dtype=np.float32) if annual else None
        np_ = C.c_int32(0)
        rc = _check(self._lib.h9g_run_decade_ordered(self._h, sl.ctypes.data_as(C.POINTER(C.c_int32)), jyear0,
                                                     sl.size, _fp(out) if annual else None, C.byref(np_)),
                    "h9g_run_decade_ordered")
        self.decade_rc = rc
        if rc and raise_on_stop:
            raise ReferenceStop(self.last_error())
        return out, int(np_.value)

    def run_ordered(self, slots, jyear0: int, raise_on_stop: bool = True, annual: bool = True):
        """Years jyear0 .. jyear0+len(slots)-1 in the reference's own cell
        order, cut into its decades, which overlap on the device
        (h9g_run_ordered; bit-identical to run_decade_ordered per decade);
        synchronous.  Every year's slot must stay resident for the call.
        Returns (annual (nyears, 12+L, ncell) or None, passes per decade);
        self.decade_rc holds the STOP code."""
        sl = np.ascontiguousarray(slots, dtype=np.int32)
        out = np.empty((sl.size, 12 + self.L, self.ncell), dtype=np.float32) if annual else None
        np_ = (C.c_int32 * max(1, len(decades(jyear0, sl.size))))()
        rc = _check(self._lib.h9g_run_ordered(self._h, sl.ctypes.data_as(C.POINTER(C.c_int32)), jyear0, sl.size,
                                              _fp(out) if annual else None, np_), "h9g_run_ordered")
        self.decade_rc = rc
        if rc and raise_on_stop:
            raise ReferenceStop(self.last_error())
        return out, [int(v) for v in np_][:len(decades(jyear0, sl.size))]

    def ordered_stats(self) -> dict:
        """How the last ordered call overlapped its decades (h9g_ordered_stats)."""
        out = (C.c_int64 * 64)()
        m = _check(self._lib.h9g_ordered_stats(self._h, out, 64), "h9g_ordered_stats")
        keys = ("decades", "first_pass_launches", "rerun_years_riding", "rerun_cell_years_riding",
                "rerun_years_alone", "rerun_cell_years_alone", "cells_left_out_of_first_pass",
                "probed", "probe_kept")
        d = {k: int(out[i]) for i, k in enumerate(keys)}
        d["passes"] = [int(out[i]) for i in range(len(keys), m)]
        return d

    def launch_stats(self, reset: bool = False) -> dict:
        """Year launches per kernel kind since the last reset
        (h9g_launch_stats): launches, cell-years, device ms."""
        out = (C.c_double * 21)()
        m = _check(self._lib.h9g_launch_stats(self._h, out, 21, int(reset)), "h9g_launch_stats")
        names = ("pair", "solo", "mixed", "pair2", "pair11", "pair1", "probe")
        return {nm: dict(launches=int(out[3 * i]), cell_years=int(out[3 * i + 1]), ms=float(out[3 * i + 2]))
                for i, nm in enumerate(names) if 3 * i + 2 < m and out[3 * i] > 0}

    def set_chains(self, chain=None):
        """Independent cell-order chains, one per reference rank
        (h9g_set_chains; shard.reference_blocks gives the reference's).
        None: one chain."""
        if chain is None:
            _check(self._lib.h9g_set_chains(self._h, None), "h9g_set_chains")
            return
        ch = np.ascontiguousarray(chain, dtype=np.int32)
        assert ch.size == self.ncell
        _check(self._lib.h9g_set_chains(self._h, ch.ctypes.data_as(C.POINTER(C.c_int32))), "h9g_set_chains")

    def decade_stats(self) -> dict:
        """Work of the last run_decade_ordered (h9g_decade_stats)."""
        out = (C.c_int64 * 64)()
        m = _check(self._lib.h9g_decade_stats(self._h, out, 64), "h9g_decade_stats")
        return dict(passes=int(out[0]), rerun_cells=int(out[1]), rerun_cell_years=int(out[2]),
                    rerun_launches=int(out[3]), launch_cells=[int(out[i]) for i in range(4, m)])

    def run_site(self, sub, daily, lai, raise_on_stop: bool = True) -> np.ndarray:
        """LCLIM site path (HYBRID9.f90:339-480) over nday days, synchronous.

        sub (nday*nisurf, 5, ncell): tak (degC), rh, Rnet, PAR, ppt (mm per
        substep); daily (nday, 2, ncell): huss, ps; lai (nday, 3, ncell):
        (LAI, a, b), NaN = unchanged.  Returns the daily diagnostics
        (nday, 11, ncell), site.DIAG_FIELDS (NaN for masked/failed cells)."""
        daily = np.ascontiguousarray(daily, dtype=np.float32)
        nday = daily.shape[0]
        sub = np.ascontiguousarray(sub, dtype=np.float32)
        lai = np.ascontiguousarray(lai, dtype=np.float32)
        if (sub.shape != (nday * self.nisurf, 5, self.ncell) or daily.shape != (nday, 2, self.ncell)
                or lai.shape != (nday, 3, self.ncell)):
            raise ValueError("run_site: shapes must be sub (nday*nisurf, 5, ncell), "
                             "daily (nday, 2, ncell), lai (nday, 3, ncell)")
        out = np.empty((nday, 11, self.ncell), dtype=np.float32)
        rc = _check(self._lib.h9g_run_site(self._h, nday, _fp(sub), _fp(daily), _fp(lai), _fp(out)),
                    "h9g_run_site")
        if rc and raise_on_stop:
            raise ReferenceStop(self.last_error())
        self.site_rc = rc
        return out

    def sync(self, raise_on_stop: bool = True) -> int:
        rc = _check(self._lib.h9g_sync(self._h), "h9g_sync")
        if rc and raise_on_stop:
            raise ReferenceStop(self.last_error())
        return rc

    def last_error(self) -> dict:
        e = _Error()
        _check(self._lib.h9g_last_error(self._h, C.byref(e)), "h9g_last_error")
        return dict(code=e.code, cell=e.cell, year=e.year, day=e.day, substep=e.substep,
                    value=e.value)

    def get_errors(self) -> dict:
        """Every cell's STOP record: code (0: none), day, substep, value."""
        rec = np.empty((4, self.ncell), dtype=np.int32)
        _check(self._lib.h9g_get_errors(self._h, rec.ctypes.data_as(C.POINTER(C.c_int32))), "h9g_get_errors")
        return dict(code=rec[0].copy(), day=rec[1].copy(), substep=rec[2].copy(),
                    value=rec[3].view(np.float32).copy())

    def get_annual(self) -> np.ndarray:
        out = np.empty((12 + self.L, self.ncell), dtype=np.float32)
        _check(self._lib.h9g_get_annual(self._h, _fp(out)), "h9g_get_annual")
        return out

    def get_diagnostics(self, dev_ptr: int | None = None) -> np.ndarray:
        out = np.empty(NDIAG, dtype=np.float64)
        _check(self._lib.h9g_get_diagnostics(self._h, out.ctypes.data_as(_DP),
                                             C.c_void_p(dev_ptr) if dev_ptr else None),
               "h9g_get_diagnostics")
        return out

    def diagnostics_async(self, dev_ptr: int, stream: int | None):
        """Copy the diagnostics into device buffer dev_ptr, ordered on the
        hipStream_t `stream` (e.g. torch's current stream before an RCCL
        all-reduce) with no host synchronisation."""
        _check(self._lib.h9g_get_diagnostics_async(self._h, C.c_void_p(dev_ptr),
                                                   C.c_void_p(stream) if stream else None),
               "h9g_get_diagnostics_async")

    def last_kernel_ms(self) -> float:
        return float(self._lib.h9g_last_kernel_ms(self._h))

    def total_kernel_ms(self, reset: bool = False) -> float:
        return float(self._lib.h9g_total_kernel_ms(self._h, int(reset)))

    def kernel_name(self) -> str:
        return self._lib.h9g_kernel_name(self._h).decode()

    def kind_id(self) -> int:
        """The context's year kernel as h9g_launch_stats numbers it: 1 pair,
        2 solo, 3 solo rounds + pair, 4 pair2, 5 pair11, 6 pair1."""
        name = self.kernel_name()
        if "+" in name:
            return 3
        for prefix, k in (("h9g_solo_", 2), ("h9g_pair2_", 4), ("h9g_pair11_", 5), ("h9g_pair1_", 6)):
            if name.startswith(prefix):
                return k
        return 1


PGF_VARS = ("tas", "rlds", "rsds", "huss", "ps", "pr", "rhs")   # READ_PGF.f90 order


def _paths(paths):
    paths = [str(p).encode() for p in paths]
    if len(paths) != NFORCING:
        raise ValueError("need the 7 PGF files in READ_PGF order " + " ".join(PGF_VARS))
    return (C.c_char_p * NFORCING)(*paths)


def pgf_paths(directory, decade: str, suffix: str = "nc4"):
    """READ_PGF.f90:22-106 file names: <var>_pgfv2.1_<decade>.<suffix>."""
    return [str(Path(directory) / f"{v}_pgfv2.1_{decade}.{suffix}") for v in PGF_VARS]


def nc_ntimes(path) -> int:
    """NTIMES of a PGF file (its 'time' dimension, READ_NET_CDF_0D.f90)."""
    return _check(lib().h9g_nc_ntimes(str(path).encode()), "h9g_nc_ntimes")


IO_STATS = ("wall_s", "setup_s", "threads", "jobs", "pread_s", "inflate_s", "gather_s", "other_s",
            "bytes_read", "bytes_decoded", "values", "pool_wall_s")


def nc_read_stats() -> dict:
    """Stage profile of the last forcing read (h9g_nc_read_stats): wall and
    setup seconds, then thread-seconds per stage summed over the pool."""
    out = (C.c_double * len(IO_STATS))()
    m = _check(lib().h9g_nc_read_stats(out, len(IO_STATS)), "h9g_nc_read_stats")
    return {k: float(out[i]) for i, k in enumerate(IO_STATS[:m])}


def nc_forcing_read(paths, nx: int, ny: int, gid, t0: int, nt: int) -> np.ndarray:
    """Days [t0, t0+nt) of the 7 PGF files at grid ids gid -> (7, nt, ncell)."""
    gid = np.ascontiguousarray(gid, dtype=np.int64)
    out = np.empty((NFORCING, nt, gid.size), dtype=np.float32)
    _check(lib().h9g_nc_forcing_read(_paths(paths), nx, ny, gid.size, gid.ctypes.data_as(_I64P), t0, nt,
                                     _fp(out)), "h9g_nc_forcing_read")
    return out


def write_axy_nc(path, annual, gid, zc, nx: int = 720, ny: int = 360):
    """WRITE_NET_CDF_3DR.f90: one year of annual means (12+L, ncell) of the
    cells gid to axyYYYY.nc (netCDF classic, the reference's schema)."""
    annual = np.ascontiguousarray(annual, dtype=np.float32)
    gid = np.ascontiguousarray(gid, dtype=np.int64)
    zc = np.ascontiguousarray(zc, dtype=np.float32)
    L = annual.shape[0] - 12
    assert annual.shape[1] == gid.size and zc.size == L
    _check(lib().h9g_write_axy_nc(str(path).encode(), nx, ny, L, _fp(zc), gid.size,
                                  gid.ctypes.data_as(_I64P), _fp(annual)), "h9g_write_axy_nc")


def decades(year0: int, nyears: int):
    """The reference's decades (HYBRID9.f90:93-113: 1901-1910, 1911-1920,
    ...) cut to [year0, year0 + nyears): list of (first year, years)."""
    out, y, end = [], year0, year0 + nyears
    while y < end:
        e = min(1901 + 10 * ((y - 1901) // 10) + 10, end)
        out.append((y, e - y))
        y = e
    return out


def run_cell_order(*, zi, params, forcing, nisurf=48, year0=1901, nyears=1, grow_on=True,
                   state0: np.ndarray | None = None, device=0, chains=None, pipelined=True):
    """``run`` in the reference's own cell order (smp carried from cell to
    cell, cells in the given order; chains: a reference rank per cell, each
    rank its own chain, shard.reference_blocks).  pipelined: one
    ``Context.run_ordered`` over all the years (every year's forcing
    resident, the decades overlapping on the device); else decade by decade
    through ``Context.run_decade_ordered``.  Returns dict(annual, state, rc,
    err, errors, passes (per decade), work (decade_stats per call),
    overlap (ordered_stats, pipelined))."""
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    with Context(n, zi, nlayers=L, nisurf=nisurf, grow_on=grow_on, device=device,
                 nslots=nyears if pipelined else 10) as ctx:
        ctx.set_chains(chains)
        ctx.set_params(params)
        if state0 is None:
            ctx.init_state()
        else:
            ctx.set_state(state0)
        ann = np.full((nyears, 12 + L, n), np.nan, dtype=np.float32)
        d0, rc, err, passes, work = 0, 0, None, [], []
        if pipelined:
            for k in range(nyears):
                nt = days_in_year(year0 + k)
                ctx.push_forcing(k, forcing[:, d0:d0 + nt, :])
                d0 += nt
            a, passes = ctx.run_ordered(list(range(nyears)), year0, raise_on_stop=False)
            rc = ctx.decade_rc
            if not rc or len(decades(year0, nyears)) == 1:
                return dict(annual=a, state=ctx.get_state(), rc=rc, err=ctx.last_error() if rc else None,
                            errors=ctx.get_errors(), passes=passes, work=[ctx.decade_stats()],
                            overlap=ctx.ordered_stats())
    if pipelined:
        # a STOP: the reference program ends in that decade, while run_ordered
        # goes on with the other cells; the decade-by-decade form stops there
        return run_cell_order(zi=zi, params=params, forcing=forcing, nisurf=nisurf, year0=year0, nyears=nyears,
                              grow_on=grow_on, state0=state0, device=device, chains=chains, pipelined=False)
    with Context(n, zi, nlayers=L, nisurf=nisurf, grow_on=grow_on, device=device, nslots=10) as ctx:
        ctx.set_chains(chains)
        ctx.set_params(params)
        if state0 is None:
            ctx.init_state()
        else:
            ctx.set_state(state0)
        ann = np.full((nyears, 12 + L, n), np.nan, dtype=np.float32)
        d0, rc, err, passes, work = 0, 0, None, [], []
        for y0, ny in decades(year0, nyears):
            for k in range(ny):
                nt = days_in_year(y0 + k)
                ctx.push_forcing(k, forcing[:, d0:d0 + nt, :])
                d0 += nt
            a, p = ctx.run_decade_ordered(list(range(ny)), y0, raise_on_stop=False)
            ann[y0 - year0:y0 - year0 + ny] = a
            passes.append(p)
            work.append(ctx.decade_stats())
            rc = ctx.decade_rc
            if rc:
                err = ctx.last_error()
                break
        return dict(annual=ann, state=ctx.get_state(), rc=rc, err=err, errors=ctx.get_errors(), passes=passes,
                    work=work)


def run(*, zi, params, forcing, nisurf=48, year0=1901, nyears=1, grow_on=True,
        state0: np.ndarray | None = None, device=0, stop_on_error=True):
    """Run ``nyears`` years from ``year0`` for every cell (HYBRID9.f90:120-290).

    Same contract as ``oracle.port.run`` / ``oracle.refcase.run_case``:
    forcing is (7, ndays_total, ncell); returns dict(annual (nyears, 12+L,
    ncell), state (packed), rc, err, errors).  A cell reaching one of the
    reference's STOPs stops (NaN means); with stop_on_error the run ends
    after that year, as the reference program would, else the other cells
    go on.  ``errors`` holds every cell's STOP record (Context.get_errors)."""
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    with Context(n, zi, nlayers=L, nisurf=nisurf, grow_on=grow_on, device=device) as ctx:
        ctx.set_params(params)
        if state0 is None:
            ctx.init_state()
        else:
            ctx.set_state(state0)
        ann = np.full((nyears, 12 + L, n), np.nan, dtype=np.float32)
        d0, rc, err = 0, 0, None
        for y in range(nyears):
            nt = days_in_year(year0 + y)
            ctx.push_forcing(y % 2, forcing[:, d0:d0 + nt, :])
            ctx.run_year(y % 2, year0 + y)
            rc = ctx.sync(raise_on_stop=False)
            ann[y] = ctx.get_annual()
            d0 += nt
            if rc:
                err = ctx.last_error()
                if stop_on_error:
                    break
        return dict(annual=ann, state=ctx.get_state(), rc=rc, err=err, errors=ctx.get_errors())
