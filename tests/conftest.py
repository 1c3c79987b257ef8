"""Shared test fixtures.  GPU tests are marked ``@pytest.mark.gpu``."""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
sys.path.insert(0, str(ROOT))


_CRASH_LOG = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long CPU test")
    # A fatal error (segfault, abort) in native code kills the interpreter
    # before pytest reports which test ran (one CPU run of six
    # died that way).  Every test's id is written, flushed, to
    # tests/_build/crash.log before it runs, and faulthandler dumps every
    # thread's Python stack into the same file, so the last id in it names
    # the test a crash happened in.
    global _CRASH_LOG
    import faulthandler
    d = ROOT / "tests" / "_build"
    d.mkdir(parents=True, exist_ok=True)
    _CRASH_LOG = open(d / "crash.log", "w", buffering=1)
    faulthandler.enable(file=_CRASH_LOG, all_threads=True)


def pytest_runtest_logstart(nodeid, location):
    if _CRASH_LOG is not None:
        import os
        _CRASH_LOG.write(f"== {nodeid}\n")
        _CRASH_LOG.flush()
        os.fsync(_CRASH_LOG.fileno())


def golden_names(kind=None):
    out = []
    for p in sorted(GOLDEN.glob("*.npz")):
        m = json.loads(str(np.load(p)["meta"]))
        if kind is None or m["kind"] in kind:
            out.append(p.stem)
    return out


def load_golden(name):
    """Returns (meta, inputs, expected) for a golden case.  Synthetic inputs
    are regenerated and checked against the stored sha256."""
    from hybrid9_amd import synth
    from tests.golden.make_golden import digest, packed_params, synth_inputs
    from oracle import refcase

    z = np.load(GOLDEN / f"{name}.npz")
    meta = json.loads(str(z["meta"]))
    L = meta["L"]
    n = meta["ncell"]
    if meta["kind"] in ("synth", "bench_stop", "cell_order"):
        gid = np.asarray(meta["gid"], dtype=np.int64)
        if meta.get("grid") == "025":           # 0.25 deg cells (config 5)
            from tests.golden.make_golden import l10_inputs
            p, f = l10_inputs(gid, meta["year0"], meta["nyears"], meta["seed"])
        else:
            p, f = synth_inputs(gid, meta["year0"], meta["nyears"], L, meta["seed"])
        assert digest(packed_params(p), f) == meta["input_sha256"], "synthetic inputs drifted"
        state0 = None
    elif meta["kind"] == "spinup":
        from tests.golden.make_golden import spinup_inputs
        gid = np.asarray(meta["gid"], dtype=np.int64)
        ns = meta["n_synth"]
        _, p, f, state0 = spinup_inputs(gid[:ns], gid[ns:], meta["year0"], meta["nyears"], L, meta["seed"])
        assert digest(packed_params(p), f, state0) == meta["input_sha256"], "spin-up inputs drifted"
    elif meta["kind"] == "l10":
        from tests.golden.make_golden import l10_inputs
        gid = np.asarray(meta["gid"], dtype=np.int64)
        p, f = l10_inputs(gid, meta["year0"], meta["nyears"], meta["seed"])
        assert digest(packed_params(p), f) == meta["input_sha256"], "L=10 inputs drifted"
        state0 = None
    else:
        pp = z["params"]
        p = {k: pp[i * n * L:(i + 1) * n * L].reshape(n, L)
             for i, k in enumerate(("theta_s", "hksat", "bsw", "psi_s"))}
        p["fmax"] = pp[4 * n * L:].copy()
        f = z["forcing"]
        state0 = z["state0"] if "state0" in z.files else None
    inputs = dict(zi=np.asarray(meta["zi"], np.float32), params=p, forcing=f,
                  nisurf=meta["nisurf"], year0=meta["year0"], nyears=meta["nyears"],
                  grow_on=meta["grow_on"], state0=state0)
    expected = {k: z[k] for k in ("annual", "state", "trace", "state_decade", "state_ok", "ok") if k in z.files}
    return meta, inputs, expected


def load_site_golden(name):
    """(meta, inputs, expected) of an LCLIM golden (tests/golden/make_golden.py
    lclim_case); inputs regenerated and checked against the stored sha256."""
    from tests.golden.make_golden import digest, packed_params, site_inputs

    z = np.load(GOLDEN / f"{name}.npz")
    meta = json.loads(str(z["meta"]))
    gid = np.asarray(meta["gid"], dtype=np.int64)
    years = tuple(range(meta["year0"], meta["year0"] + meta["nyears"]))
    ev = None if meta["events"] is None else {int(k): v for k, v in meta["events"].items()}
    p, sub, daily, lai = site_inputs(gid, meta["L"], meta["nisurf"], years, ev, meta["seed"],
                                     meta["soils"], meta["ppt_scale"])
    assert digest(packed_params(p), sub, daily, lai) == meta["input_sha256"], "site inputs drifted"
    inputs = dict(zi=np.asarray(meta["zi"], np.float32), params=p, sub=sub, daily=daily, lai=lai,
                  nisurf=meta["nisurf"])
    return meta, inputs, dict(daily=z["daily"], state=z["state"])


def same_bits(a, b):
    """Bit-for-bit equality of the IEEE bit patterns (+0 and -0 differ: 0 ULP
    means the same bits), except that any NaN equals any NaN (the payload of
    a NaN is not a value: the reference marks masked cells NaN)."""
    a = np.asarray(a)
    b = np.asarray(b)
    if a.shape != b.shape:
        return False
    t = np.result_type(a, b)
    if t.kind != "f":
        return bool(np.array_equal(a, b))
    a, b = a.astype(t), b.astype(t)          # f32 -> f64 is exact and keeps the sign of zero
    u = {2: np.uint16, 4: np.uint32, 8: np.uint64}[t.itemsize]
    return bool(np.all((a.view(u) == b.view(u)) | (np.isnan(a) & np.isnan(b))))


@pytest.fixture(scope="session")
def gpu_available():
    import hybrid9_amd as h
    return h.lib().h9g_device_count() > 0
