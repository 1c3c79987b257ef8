"""TEST INFRASTRUCTURE ONLY: ctypes binding of the C oracle (oracle/h9_oracle.c).

Used by tests/ (as the checker), __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

from . import refcase

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "libh9oracle.so"
_lib = None


class H9OError(C.Structure):
    _fields_ = [("code", C.c_int), ("cell", C.c_int), ("day", C.c_int),
                ("substep", C.c_int), ("value", C.c_float)]


def build():
    subprocess.run(["make", "-s", "-C", str(HERE), "port"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        f = C.POINTER(C.c_float)
        _lib.h9o_state_size.argtypes = [C.c_int]
        _lib.h9o_init_state.argtypes = [C.c_int, C.c_int, f, f, f]
        _lib.h9o_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                 f, f, f, f, f, C.c_int, C.POINTER(C.c_int), f,
                                 C.c_int, C.POINTER(H9OError), C.POINTER(C.c_int)]
        _lib.h9o_site.argtypes = [C.c_int] * 4 + [f] * 7 + [C.c_int, C.POINTER(H9OError)]
        i64 = C.POINTER(C.c_int64)
        _lib.h9o_soil_layer.argtypes = [C.c_int, C.c_int, C.c_int, i64, f, f, f, f, f, f, f, f]
        _lib.h9o_soil_fmax.argtypes = [C.c_int, C.c_int, i64, C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int32), f, f]
    return _lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def pack_params(params) -> np.ndarray:
    return np.concatenate([params[k].ravel() for k in ("theta_s", "hksat", "bsw", "psi_s")]
                          + [params["fmax"].ravel()]).astype(np.float32)


def init_state(params, zi) -> np.ndarray:
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    st = np.zeros(n * lib().h9o_state_size(L), dtype=np.float32)
    pp = pack_params(params)
    zi = np.ascontiguousarray(zi, dtype=np.float32)
    rc = lib().h9o_init_state(n, L, _fp(zi), _fp(pp), _fp(st))
    assert rc == 0
    return st


def run(*, zi, params, forcing, nisurf=48, year0=1901, nyears=1, grow_on=1,
        state0=None, trace_cells=(), nthreads=1):
    """Same contract as refcase.run_case; returns dict(annual, state, trace?, err)."""
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    zi = np.ascontiguousarray(zi, dtype=np.float32)
    if zi.size != L + 2:
        raise ValueError(f"zi must hold zi(0:L+1) = {L + 2} values, got {zi.size}")
    pp = pack_params(params)
    fo = np.ascontiguousarray(forcing, dtype=np.float32)
    if state0 is None:
        st = init_state(params, zi)
    else:
        st = refcase.pack_state(state0, L)
    ann = np.full((nyears, 12 + L, n), np.nan, dtype=np.float32)   # non-soil cells stay NaN (INIT.f90:402-414)
    ndays = fo.shape[1]
    tc = np.asarray(sorted(trace_cells), dtype=np.int32)
    tr = np.zeros((max(len(tc), 1), ndays * nisurf, refcase.trace_width(L)), dtype=np.float32)
    err = H9OError()
    rec = np.zeros((4, n), dtype=np.int32)
    rc = lib().h9o_run(n, L, nisurf, int(grow_on), year0, nyears, _fp(zi), _fp(pp), _fp(fo),
                       _fp(st), _fp(ann), len(tc), tc.ctypes.data_as(C.POINTER(C.c_int)),
                       _fp(tr), nthreads, C.byref(err), rec.ctypes.data_as(C.POINTER(C.c_int)))
    out = dict(annual=ann, state=refcase.unpack_state(st, n, L), rc=rc,
               err=dict(code=err.code, cell=err.cell, day=err.day, substep=err.substep,
                        value=err.value),
               errors=dict(code=rec[0], day=rec[1], substep=rec[2], value=rec[3].view(np.float32)))
    if len(tc):
        out["trace"] = tr
    return out


def decades(year0, nyears):
    """The reference's decades (HYBRID9.f90:93-113: 1901-1910, 1911-1920,
    ...) cut to [year0, year0 + nyears): list of (first year, years)."""
    out, y, end = [], year0, year0 + nyears
    while y < end:
        e = min(1901 + 10 * ((y - 1901) // 10) + 10, end)
        out.append((y, e - y))
        y = e
    return out


def run_cell_order(*, zi, params, forcing, nisurf=48, year0=1901, nyears=1, grow_on=1,
                   state0=None, chains=None):
    """The reference's own order (HYBRID9.f90:93-130): decade -> cell ->
    year, with smp (SHARED.f90:198) carried from cell to cell: a land cell's
    first substep of a decade reads the smp its predecessor in cell order
    left behind (HYDROLOGY.f90:270-275); the first land cell reads the smp
    the last land cell holds when the decade starts.  chains: a reference
    rank per cell (each rank its own chain, its cells in the given order).
    Restated on the C oracle one (cell, decade) at a time; same contract as
    run()."""
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    fo = np.ascontiguousarray(forcing, dtype=np.float32)
    st = refcase.unpack_state(init_state(params, zi) if state0 is None
                              else refcase.pack_state(state0, L), n, L)
    st = {k: np.array(v, copy=True) for k, v in st.items()}
    ann = np.full((nyears, 12 + L, n), np.nan, dtype=np.float32)
    # the soil mask (HYBRID9.f90:122-123), summed in layer order
    land =[c for c in range(n) if _mask_sum(params["theta_s"][c]) > np.float32(1.0e-8)]
    one = lambda a, c: a[c:c + 1]  # noqa: E731
    rc, err = 0, dict(code=0, cell=-1, day=-1, substep=-1, value=0.0)
    cid = np.zeros(n, np.int64) if chains is None else np.asarray(chains, np.int64)
    groups = [[c for c in land if cid[c] == r] for r in sorted(set(cid[land].tolist()))]
    day0 = 0
    for y0, ny in decades(year0, nyears):
        nd = sum(_days(y0 + k) for k in range(ny))
        carry = {}
        for grp in groups:
            carry[grp[0]] = st["smp"][grp[-1]].copy()     # the chain's first cell: its last one's smp
        prev = {}
        for grp in groups:
            for a_, b_ in zip(grp, grp[1:]):
                prev[b_] = a_
        for c in land:
            s1 = {k: one(v, c).copy() for k, v in st.items()}
            s1["smp"][0] = carry[c] if c in carry else st["smp"][prev[c]].copy()
            r = run(zi=zi, params={k: one(v, c) for k, v in params.items()},
                    forcing=np.ascontiguousarray(fo[:, day0:day0 + nd, c:c + 1]), nisurf=nisurf,
                    year0=y0, nyears=ny, grow_on=grow_on, state0=s1)
            for k in st:
                st[k][c] = r["state"][k][0]
            ann[y0 - year0:y0 - year0 + ny, :, c] = r["annual"][:, :, 0]
            if r["rc"] and not rc:
                rc = r["rc"]
                err = dict(r["err"], cell=c)
        day0 += nd
        if rc:
            break
    return dict(annual=ann, state=st, rc=rc, err=err)


def _mask_sum(ts):
    s = np.float32(0.0)
    for v in ts:
        s = np.float32(s + np.float32(v))
    return s


def _days(y):
    return 365 if y % 4 else (366 if y % 100 else (365 if y % 400 else 366))


def site(*, zi, params, sub, daily, lai, nisurf=48, state0=None, nthreads=1):
    """LCLIM site path restated (h9o_site); same contract as
    refcase.run_site_case; returns dict(daily, state, rc, err).  Masked and
    failed cells: NaN rows."""
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    zi = np.ascontiguousarray(zi, dtype=np.float32)
    pp = pack_params(params)
    st = init_state(params, zi) if state0 is None else refcase.pack_state(state0, L)
    sub = np.ascontiguousarray(sub, dtype=np.float32)
    daily = np.ascontiguousarray(daily, dtype=np.float32)
    lai = np.ascontiguousarray(lai, dtype=np.float32)
    nday = daily.shape[0]
    out = np.full((nday, 11, n), np.nan, dtype=np.float32)
    err = H9OError()
    rc = lib().h9o_site(n, L, nisurf, nday, _fp(zi), _fp(pp), _fp(sub), _fp(daily), _fp(lai),
                        _fp(st), _fp(out), nthreads, C.byref(err))
    return dict(daily=out, state=refcase.unpack_state(st, n, L), rc=rc,
                err=dict(code=err.code, cell=err.cell, day=err.day, substep=err.substep,
                         value=err.value))


def soil_layer(nx, ny, gid, ts, ks, lm, ps):
    """INIT.f90:575-631 restated (h9o_soil_layer): returns theta_s, hksat,
    bsw, psi_s of one layer for the cells gid."""
    gid = np.ascontiguousarray(gid, np.int64)
    a = [np.ascontiguousarray(x, np.float32) for x in (ts, ks, lm, ps)]
    out = [np.empty(gid.size, np.float32) for _ in range(4)]
    lib().h9o_soil_layer(nx, ny, gid.size, gid.ctypes.data_as(C.POINTER(C.c_int64)),
                         *[_fp(x) for x in a], *[_fp(o) for o in out])
    return out


def soil_fmax(gid, soil_tex, fmax_in, theta_s):
    """INIT.f90:661-680 restated (h9o_soil_fmax); theta_s (ncell, L)."""
    gid = np.ascontiguousarray(gid, np.int64)
    t = np.ascontiguousarray(soil_tex, np.int32).reshape(-1)
    fm = np.ascontiguousarray(fmax_in, np.int32).reshape(-1)
    ts = np.ascontiguousarray(theta_s, np.float32)
    out = np.empty(gid.size, np.float32)
    i32 = C.POINTER(C.c_int32)
    lib().h9o_soil_fmax(gid.size, ts.shape[1], gid.ctypes.data_as(C.POINTER(C.c_int64)),
                        t.ctypes.data_as(i32), fm.ctypes.data_as(i32), _fp(ts), _fp(out))
    return out
