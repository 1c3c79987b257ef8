"""C-ABI surface: libh9g.so loads, exports every entry point that
include/h9g.h declares, and the Fortran ISO_C_BINDING module compiles and
links against it.  No compute without a GPU."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np

import hybrid9_amd as h
from hybrid9_amd import build

ROOT = Path(__file__).resolve().parents[1]


def test_library_builds_and_loads():
    build.build()
    lb = h.lib()
    assert lb.h9g_abi_version() == 1


def test_every_declared_symbol_is_exported():
    syms = h.exported_symbols()
    assert len(syms) >= 25
    nm = subprocess.run(["nm", "-D", "--defined-only", str(h.LIB_PATH)], capture_output=True,
                        text=True, check=True).stdout
    exported = set(re.findall(r"\b(h9g_[a-z_0-9]+)\b", nm))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    lb = C.CDLL(str(h.LIB_PATH))
    for s in syms:
        getattr(lb, s)


def test_state_size_and_bad_configs():
    lb = h.lib()
    assert lb.h9g_state_size(8) == 41 and lb.h9g_state_size(10) == 49
    cfg = h._Config()
    cfg.ncell, cfg.nlayers, cfg.nisurf, cfg.max_days, cfg.nslots = 10, 7, 48, 366, 2
    assert not lb.h9g_create(C.byref(cfg), 0)           # L must be 8 or 10
    cfg.nlayers = 8
    for i in range(10):
        cfg.zi[i] = float(i)
    cfg.zi[3] = 1.0                                       # non-monotone zi
    assert not lb.h9g_create(C.byref(cfg), 0)


def test_no_cpu_fallback_without_gpu():
    if h.lib().h9g_device_count() > 0:
        return
    try:
        h.Context(4, np.arange(10, dtype=np.float32))
    except h.H9GError as e:
        assert "h9g_create failed" in str(e)
    else:
        raise AssertionError("Context created without a GPU")


def test_device_code_makes_no_calls():
    """Every kernel of libh9g.so is call-free: the rare paths (glibc's special
    cases, the exact re-run) are inlined.  Calls from the kernels were
    miscompiled in round 2 -- a lane-mask SGPR stayed live across calls of the
    out-of-line redo function, which overwrites it (DESIGN.md §3,
    tools/isa_calls.py)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("isa_calls", Path(__file__).resolve().parents[1] / "tools" / "isa_calls.py")
    ic = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ic)
    calls = ic.calls_per_function(h.LIB_PATH)
    assert any("h9g_pair_kernel" in k for k in calls)
    assert {k: n for k, n in calls.items() if n} == {}
