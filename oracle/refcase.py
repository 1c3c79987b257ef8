"""TEST INFRASTRUCTURE ONLY: case files for the reference harness.

Writes/reads the raw little-endian case directory consumed by
``oracle/_ref/h9ref`` (built by ``oracle/Makefile`` from the unmodified
reference HYDROLOGY.f90/GROW.f90 plus our harness ``oracle/ref/h9ref_main.f90``)
and runs it.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.

Byte layouts (float32, Fortran column-major == numpy C-order reversed):
  params.f32   theta_s, hksat, bsw, psi_s as (ncell, L); fmax (ncell)
  forcing.f32  (7, ndays, ncell): tas, rlds, rsds, huss, ps, pr, rhs
  state*.f32   STATE_FIELDS below, each (ncell, width)
  annual.f32   (nyears, 12 + L, ncell), fields ANNUAL_FIELDS
  trace.f32    per traced substep: 3L+7 floats (TRACE_FIELDS)
"""
from __future__ import annotations

import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF_BIN = HERE / "_ref" / "h9ref"
REF_BIN_L10 = HERE / "_ref" / "h9ref_l10"     # nsoil_layers_max = 10 rebuild (make ref10)


def ref_bin(L: int) -> Path:
    """The reference harness built for L soil layers (8: as shipped;
    10: the parameter-only rebuild of SHARED.f90:294,300)."""
    if L == 8:
        return REF_BIN
    if L == 10:
        return REF_BIN_L10
    raise ValueError(f"no reference build for L={L}")

ANNUAL_SCALARS = ("npp", "plant_mass", "rnf", "evap", "tas", "rlds", "rsds",
                  "huss", "ps", "pr", "rhs")


def annual_fields(L: int):
    return list(ANNUAL_SCALARS) + [f"theta{i + 1}" for i in range(L)] + ["theta_total"]


def state_fields(L: int):
    """(name, width) in file order (HYBRID9 SHARED.f90 per-cell state)."""
    return [("h2osoi_liq", L), ("h2osoi_liq_ma", L), ("smp", L),
            ("rootr_col", L + 1), ("zwt", 1), ("wa", 1), ("LAI", 1),
            ("LAI_litter", 1), ("plant_mass", 1), ("plant_foliage_mass", 1),
            ("plant_length", 1), ("rdepth", 1)]


def trace_width(L: int) -> int:
    return 3 * L + 7


def pack_state(state: dict, L: int) -> np.ndarray:
    parts = []
    for name, w in state_fields(L):
        a = np.asarray(state[name], dtype=np.float32)
        parts.append(a.reshape(-1, w) if w > 1 else a.reshape(-1))
    return np.concatenate([p.ravel() for p in parts]).astype(np.float32)


def unpack_state(buf: np.ndarray, ncell: int, L: int) -> dict:
    out, off = {}, 0
    for name, w in state_fields(L):
        k = ncell * w
        a = buf[off:off + k]
        out[name] = a.reshape(ncell, w) if w > 1 else a.copy()
        off += k
    assert off == buf.size, (off, buf.size)
    return out


def write_case(d, *, zi, params, forcing=None, nisurf=48, year0=1901, nyears=1,
               grow_on=1, state0=None, trace_cells=(), site=None, cell_order=False):
    """cell_order: the reference's decade -> cell -> year order with smp
    carried from cell to cell (h9ref_main.f90 cell_order) instead of
    isolated-cell semantics."""
    if cell_order and trace_cells:
        raise ValueError("traces are per cell; cell_order interleaves them")
    d = Path(d)
    d.mkdir(parents=True, exist_ok=True)
    ncell = params["fmax"].size
    L = params["theta_s"].shape[1]
    if np.asarray(zi).size != L + 2:
        raise ValueError(f"zi must hold zi(0:L+1) = {L + 2} values, got {np.asarray(zi).size}")
    tc = list(trace_cells) or [0]
    nml = ("&h9case\n"
           f" ncell={ncell}, NISURF={nisurf}, year0={year0}, nyears={nyears},\n"
           f" grow_on={int(grow_on)}, state_override={int(state0 is not None)},\n"
           f" ntrace={len(trace_cells)}, trace_cells={','.join(str(c + 1) for c in tc)},\n"
           f" lclim_mode={int(site is not None)}, cell_order={int(bool(cell_order))}\n/\n")
    (d / "case.nml").write_text(nml)
    np.asarray(zi, dtype=np.float32).tofile(d / "zi.f32")
    np.concatenate([params[k].ravel() for k in ("theta_s", "hksat", "bsw", "psi_s")]
                   + [params["fmax"].ravel()]).astype(np.float32).tofile(d / "params.f32")
    if site is None:
        np.ascontiguousarray(forcing, dtype=np.float32).tofile(d / "forcing.f32")
    else:   # LCLIM mode (h9ref_main.f90): sub (T, 5, n), daily (nday, 2, n), lai (nday, 3, n)
        for k in ("sub", "daily", "lai"):
            np.ascontiguousarray(site[k], dtype=np.float32).tofile(d / f"lclim_{'day' if k == 'daily' else k}.f32")
    if state0 is not None:
        pack_state(state0, L).tofile(d / "state0.f32")


class RefStop(RuntimeError):
    """The reference executed one of its STOP statements (HYDROLOGY.f90)."""

    def __init__(self, stdout: str):
        self.stdout = stdout
        self.info = parse_stop(stdout)
        super().__init__(f"reference STOP: {self.info}")


def parse_stop(out: str) -> dict:
    """Fields printed by HYDROLOGY.f90:806-825 / 1068-1072 / 1245-1273."""
    info = {}
    lines = out.splitlines()
    for i, ln in enumerate(lines):
        t = ln.strip()
        if t.startswith("Water imbalance > 0.1 mm"):
            info["code"] = 4
            info["value"] = float(t.split()[-1])
        elif t.startswith("Problem with tridiagonal 1."):
            info["code"] = 1
        elif t.startswith("Problem with tridiagonal 2."):
            info["code"] = 2
        elif t.startswith("rsub_top_tot is positive"):
            info["code"] = 3
        elif t.startswith("DiTIME ="):
            info["day"] = int(t.split("=")[1]) - 1          # 0-based day of the year
        elif t.startswith("my_id x y"):
            info["cell"] = int(t.split()[-2]) - 1           # 0-based cell
    return info


def run_ref(d, timeout=3600, L=None):
    if L is None:
        L = np.fromfile(Path(d) / "zi.f32", dtype=np.float32).size - 2
    b = ref_bin(L)
    if not b.exists():
        raise FileNotFoundError(f"{b} missing: run `make -C oracle ref ref10`")
    r = subprocess.run([str(b), str(d)], capture_output=True, text=True,
                       timeout=timeout)
    if "Fortran STOP" in (r.stdout + r.stderr) or "Problem" in r.stdout:
        raise RefStop(r.stdout)
    if r.returncode != 0 or not ((Path(d) / "annual.f32").exists() or (Path(d) / "daily.f32").exists()):
        raise RuntimeError(f"h9ref failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    return r


def read_outputs(d, ncell, L, nyears, ntrace=0):
    d = Path(d)
    ann = np.fromfile(d / "annual.f32", dtype=np.float32).reshape(nyears, 12 + L, ncell)
    st = unpack_state(np.fromfile(d / "state_end.f32", dtype=np.float32), ncell, L)
    out = dict(annual=ann, state=st)
    if ntrace:
        tr = np.fromfile(d / "trace.f32", dtype=np.float32)
        out["trace"] = tr.reshape(ntrace, -1, trace_width(L))
    return out


def run_site_case(*, zi, params, sub, daily, lai, nisurf=48, year0=2002, nyears=2, state0=None):
    """LCLIM single-site path of the reference (HYBRID9.f90:339-480) through
    the harness: returns dict(daily (nday, 11, ncell), state)."""
    ncell = params["fmax"].size
    L = params["theta_s"].shape[1]
    with tempfile.TemporaryDirectory(prefix="h9ref_") as td:
        write_case(td, zi=zi, params=params, nisurf=nisurf, year0=year0, nyears=nyears,
                   grow_on=0, state0=state0, site=dict(sub=sub, daily=daily, lai=lai))
        run_ref(td)
        nday = np.asarray(daily).shape[0]
        out = np.fromfile(Path(td) / "daily.f32", dtype=np.float32).reshape(nday, 11, ncell)
        st = unpack_state(np.fromfile(Path(td) / "state_end.f32", dtype=np.float32), ncell, L)
        return dict(daily=out, state=st)


def run_case(**kw):
    """Write a case to a temp dir, run the reference harness, return outputs."""
    with tempfile.TemporaryDirectory(prefix="h9ref_") as td:
        write_case(td, **kw)
        run_ref(td)
        ncell = kw["params"]["fmax"].size
        L = kw["params"]["theta_s"].shape[1]
        return read_outputs(td, ncell, L, kw.get("nyears", 1),
                            len(kw.get("trace_cells", ())))
