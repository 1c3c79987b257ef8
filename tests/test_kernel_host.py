"""The GPU kernel body (hybrid9_amd/csrc/h9g_pair.h + h9g_step.h) compiled for the host
(tests/csrc/host_kernel.cpp, test-only) against the reference goldens and
the oracle, bit-for-bit -- both geometry policies (compile-time default
layers and runtime layers).  Lets the kernel's arithmetic be checked on
CPU; the GPU tests then check the device build."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from hybrid9_amd import synth
from oracle import port, refcase
from tests.conftest import golden_names, load_golden, same_bits
from tests.helpers import BUILD, ROOT

_lib = None


def _build_lib(extra):
    src = ROOT / "tests" / "csrc" / "host_kernel.cpp"
    out = BUILD / ("libhost_kernel%s.so" % ("_" + "_".join(f.strip("-D").lower().replace("=", "")
                                                          for f in extra) if extra else ""))
    deps = [src] + list((ROOT / "hybrid9_amd" / "csrc").glob("*.h"))
    if not out.exists() or out.stat().st_mtime < max(d.stat().st_mtime for d in deps):
        BUILD.mkdir(exist_ok=True)
        subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                        "-std=c++17", "-fPIC", "-shared", *extra, str(src), "-o", str(out)], check=True)
    return out


def lib():
    global _lib
    if _lib is None:
        src = ROOT / "tests" / "csrc" / "host_kernel.cpp"
        extra = os.environ.get("H9G_HOST_CFLAGS", "").split()   # e.g. kernel variant -D flags
        out = BUILD / ("libhost_kernel%s.so" % ("_" + "_".join(f.strip("-D").lower() for f in extra) if extra else ""))
        deps = [src] + list((ROOT / "hybrid9_amd" / "csrc").glob("*.h"))
        if not out.exists() or out.stat().st_mtime < max(d.stat().st_mtime for d in deps):
            BUILD.mkdir(exist_ok=True)
            subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                            "-std=c++17", "-fPIC", "-shared", *extra, str(src), "-o", str(out)], check=True)
        _lib = C.CDLL(str(out))
        fp = C.POINTER(C.c_float)
        _lib.h9k_host_run.argtypes = [C.c_int] * 7 + [fp, fp, fp, fp, fp, C.POINTER(C.c_int)]
    return _lib


def host_run(*, zi, params, forcing, nisurf, year0, nyears, grow_on, state0, const_geo, so=None):
    L = params["theta_s"].shape[1]
    n = params["fmax"].size
    zi = np.ascontiguousarray(zi, np.float32)
    pp = port.pack_params(params)
    fo = np.ascontiguousarray(forcing, np.float32)
    st = port.init_state(params, zi) if state0 is None else np.array(state0, np.float32)
    ann = np.zeros((nyears, 12 + L, n), np.float32)
    err = np.zeros(4 * n, np.int32)
    fp = C.POINTER(C.c_float)
    rc = (so or lib()).h9k_host_run(n, L, nisurf, int(grow_on), year0, nyears, int(const_geo),
                            zi.ctypes.data_as(fp), pp.ctypes.data_as(fp), fo.ctypes.data_as(fp),
                            st.ctypes.data_as(fp), ann.ctypes.data_as(fp),
                            err.ctypes.data_as(C.POINTER(C.c_int)))
    return dict(rc=rc, annual=ann, state=st, err=err.reshape(n, 4))


# const_geo: 1/0 = compile-time / runtime layer geometry
@pytest.mark.parametrize("const_geo", [1, 0])
@pytest.mark.parametrize("name", golden_names(kind=("synth", "explicit", "spinup")))
def test_kernel_body_matches_reference_golden(name, const_geo):
    meta, inp, exp = load_golden(name)
    out = host_run(const_geo=const_geo, **inp)
    assert out["rc"] == 0
    assert same_bits(out["annual"], exp["annual"])
    assert same_bits(out["state"], exp["state"])


@pytest.mark.parametrize("const_geo", [1, 0])
def test_kernel_body_reproduces_reference_stop(const_geo):
    meta, inp, _ = load_golden("stop_ns24")
    out = host_run(const_geo=const_geo, **inp)
    s = meta["stop"]
    assert out["rc"] == s["code"]
    c = s["cell"]
    assert out["err"][c, 0] == s["code"] and out["err"][c, 2] == s["day"]


@pytest.mark.parametrize("L,nisurf,grow", [(8, 48, 0), (8, 24, 1), (10, 24, 1), (10, 48, 0)])
def test_kernel_body_matches_oracle_random_cells(L, nisurf, grow):
    if L == 8:
        g = synth.land_cells()[7::389][:160]
        lat, zi = synth.cell_lat(g), synth.ZI_L8
    else:
        g = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)[11::1601][:160]
        lat, zi = synth.cell_lat(g, synth.NX025, synth.NY025), synth.ZI_L10
    p = synth.make_params(g, L)
    f = synth.make_forcing(g, lat, synth.year_day0(1903), 365 + 366)
    ref = port.run(zi=zi, params=p, forcing=f, nisurf=nisurf, year0=1903, nyears=2,
                   grow_on=grow, nthreads=8)
    out = host_run(zi=zi, params=p, forcing=f, nisurf=nisurf, year0=1903, nyears=2,
                   grow_on=grow, state0=None, const_geo=1)
    assert ref["rc"] == out["rc"] == 0
    assert same_bits(out["annual"], ref["annual"])
    assert same_bits(out["state"], refcase.pack_state(ref["state"], L))


def test_kernel_body_degenerate_exponents():
    """bsw = 1 makes 1-1/b zero (powf(x, 0) = 1 by glibc's special path,
    which the fast powf without its y test must reproduce)."""
    g = synth.land_cells()[5::997][:24]
    p = synth.make_params(g, 8)
    p["bsw"][::3, 2] = 1.0
    p["bsw"][1::5, 6] = 1.0
    f = synth.make_forcing(g, synth.cell_lat(g), synth.year_day0(1901), 365)
    ref = port.run(zi=synth.ZI_L8, params=p, forcing=f, nisurf=24, year0=1901, nyears=1,
                   grow_on=1, nthreads=8)
    out = host_run(zi=synth.ZI_L8, params=p, forcing=f, nisurf=24, year0=1901, nyears=1,
                   grow_on=1, state0=None, const_geo=1)
    assert ref["rc"] == out["rc"]
    assert same_bits(out["annual"], ref["annual"])
    assert same_bits(out["state"], refcase.pack_state(ref["state"], 8))


@pytest.mark.parametrize("name", ["edge", "c1_2yr_leap", "c4_spinup"])
def test_exact_rerun_replays_from_day_snapshot(name):
    """The exact re-run (a third water-table layer visit) replays from the
    day snapshot (h9g_pair.h save_day / substep_exact_pair) through its
    substep.  A test build forces a re-run at every 5th substep of a day, so
    each replays several substeps (the day snapshot is taken before the
    first substep that could re-run: water table in the column), and also
    re-runs right after a re-run of the same day; the result must still be
    the reference's bit for bit."""
    so = C.CDLL(str(_build_lib(["-DH9G_FORCE_RERUN=5"])))
    so.h9k_host_run.argtypes = lib().h9k_host_run.argtypes
    meta, inp, exp = load_golden(name)
    st = np.zeros(3, np.int64)
    so.h9k_host_exact_stats(st.ctypes.data_as(C.POINTER(C.c_longlong)))   # reset
    out = host_run(const_geo=1, so=so, **inp)
    so.h9k_host_exact_stats(st.ctypes.data_as(C.POINTER(C.c_longlong)))
    assert out["rc"] == 0
    assert same_bits(out["annual"], exp["annual"]) and same_bits(out["state"], exp["state"])
    runs, multi, replayed = st
    assert runs > 100 and multi > 0 and replayed > 4 * runs, st


def test_rerun_without_day_snapshot_is_reported():
    """an exact re-run requested in a substep that has no day
    snapshot (the water table started below the column, jwt = L) must not
    replay a stale snapshot block.  Such a request cannot arise (only a
    substep starting with jwt < L visits layers, h9g_pair.h substep_pair), so
    a test build forces one at every 5th substep regardless of where the
    water table is: every c1_10x10 cell starts below the column (INIT.f90:
    zwt = (zi(L) + 5000)/1000 m), so each must stop with H9G_ERR_NOSNAP on day
    0, substep 4, instead of running on."""
    so = C.CDLL(str(_build_lib(["-DH9G_FORCE_RERUN_ANY=5"])))
    so.h9k_host_run.argtypes = lib().h9k_host_run.argtypes
    meta, inp, exp = load_golden("c1_10x10")
    out = host_run(const_geo=1, so=so, **inp)
    assert out["rc"] == 5                                  # include/h9g.h H9G_ERR_NOSNAP
    err = out["err"]
    assert (err[:, 0] == 5).all() and (err[:, 1] == 0).all()
    assert (err[:, 2] == 0).all() and (err[:, 3] == 4).all()


@pytest.mark.parametrize("name", ["c1_2yr_leap", "c4_spinup"])
def test_exact_energy_balance_build(name):
    """The energy balance's exact block (h9g_pair.h, run when the branch-free
    block flags a quotient outside the Markstein range) as the whole path:
    a -DH9G_EB_FAST=0 build must give the reference's bits too."""
    so = C.CDLL(str(_build_lib(["-DH9G_EB_FAST=0"])))
    so.h9k_host_run.argtypes = lib().h9k_host_run.argtypes
    meta, inp, exp = load_golden(name)
    out = host_run(const_geo=1, so=so, **inp)
    assert out["rc"] == 0
    assert same_bits(out["annual"], exp["annual"]) and same_bits(out["state"], exp["state"])
