"""The host C/C++ under AddressSanitizer + UndefinedBehaviorSanitizer
(VERDICT r05 #7): the NetCDF ingest with its thread pool and the annual
writer (hybrid9_amd/csrc/h9g_io.cpp, the host part of libh9g.so), the C
oracle (oracle/h9_oracle.c, OpenMP) and the host build of the kernel body
(tests/csrc/host_kernel.cpp), linked into tests/csrc/san_driver.cpp and run
once each.  A sanitizer report aborts the driver (halt_on_error), so a
clean exit is the check.  The invariant these builds guard is the one the
kernel checks in every substep (HYDROLOGY.f90:1244-1274): no stray write
may reach a cell's state."""
from __future__ import annotations

import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

import hybrid9_amd as h
from hybrid9_amd import synth
from tests.helpers import BUILD, ROOT

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-O1"]
SRCS = [ROOT / "hybrid9_amd" / "csrc" / "h9g_io.cpp", ROOT / "oracle" / "h9_oracle.c",
        ROOT / "tests" / "csrc" / "host_kernel.cpp", ROOT / "tests" / "csrc" / "san_driver.cpp"]


def san_driver() -> Path:
    out = BUILD / "san_driver"
    deps = SRCS + list((ROOT / "hybrid9_amd" / "csrc").glob("*.h")) + [ROOT / "include" / "h9g.h",
                                                                    ROOT / "oracle" / "h9_oracle.h"]
    if out.exists() and out.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return out
    BUILD.mkdir(exist_ok=True)
    inc = [f"-I{ROOT / 'include'}", f"-I{ROOT / 'hybrid9_amd' / 'csrc'}"]
    objs = []
    for src in SRCS:
        obj = BUILD / f"san_{src.stem}.o"
        cc = ["gcc", "-std=c11"] if src.suffix == ".c" else ["g++", "-std=c++17"]
        subprocess.run([*cc, *SAN, "-ffp-contract=off", "-fno-fast-math", "-fopenmp", *inc, "-c", str(src),
                        "-o", str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run(["g++", *SAN, "-fopenmp", *objs, "-o", str(out), "-ldl", "-lpthread", "-lm"], check=True)
    return out


def _run(args, tmp_path):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", OMP_NUM_THREADS="4")
    r = subprocess.run([str(san_driver()), *map(str, args)], capture_output=True, text=True, env=env,
                       timeout=600, cwd=tmp_path)
    out = r.stdout + r.stderr
    assert "Sanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_sanitized_ingest_and_writer(tmp_path):
    from tests.test_netcdf import write_pgf_like
    rng = np.random.default_rng(11)
    nx, ny, nt = 30, 20, 12
    data = [rng.uniform(200, 300, (nt, ny, nx)).astype(np.float32) for _ in range(7)]
    d2, d4 = tmp_path / "cdf2", tmp_path / "nc4"
    d2.mkdir()
    d4.mkdir()
    for k, v in enumerate(h.PGF_VARS):
        write_pgf_like(d2, v, data[k], 2)
    nc4 = Path("/opt/conda/include/hdf5.h").exists()
    if nc4:
        from tests.helpers import write_nc4
        for k, v in enumerate(h.PGF_VARS):
            write_nc4(d4 / f"{v}_pgfv2.1_1901-1910.nc4", v, data[k], chunk=(2, 7, 9))
    gid = np.sort(rng.choice(nx * ny, 57, replace=False)).astype(np.int64)
    gid.tofile(tmp_path / "gid.i64")
    out = _run(["io", d2, d4 if nc4 else "-", nx, ny, nt, gid.size, tmp_path / "gid.i64",
                tmp_path / "axy1901.nc"], tmp_path)
    assert out.count("read ") == (6 if nc4 else 3)
    from scipy.io import netcdf_file
    with netcdf_file(tmp_path / "axy1901.nc", "r", mmap=False) as f:
        assert f.dimensions == {"latitude": ny, "longitude": nx, "layer_centre_depth": 8}


@pytest.mark.parametrize("case", ["synth", "stop_ns24"])
def test_sanitized_oracle_and_host_kernel(case, tmp_path):
    from oracle import port
    from tests.conftest import load_golden
    if case == "synth":
        gid = synth.land_cells()[::2811][:24].astype(np.int64)
        p = synth.make_params(gid, 8, synth.SEED)
        f = synth.make_forcing(gid, synth.cell_lat(gid), synth.year_day0(1901), 365, synth.SEED)
        zi, ns, grow = synth.ZI_L8, 24, 1
    else:
        _, inp, _ = load_golden(case)
        p, f, zi, ns, grow = inp["params"], inp["forcing"], inp["zi"], inp["nisurf"], inp["grow_on"]
    n = p["fmax"].size
    (tmp_path / "case.txt").write_text(f"{n} 8 {ns} {int(grow)} 1901 1\n")
    np.asarray(zi, np.float32).tofile(tmp_path / "zi.f32")
    port.pack_params(p).tofile(tmp_path / "params.f32")
    np.ascontiguousarray(f, np.float32).tofile(tmp_path / "forcing.f32")
    out = _run(["hydro", tmp_path], tmp_path)
    assert "bit-identical" in out
    if case == "stop_ns24":
        assert "oracle rc 0" not in out        # the reference's STOP, through both paths
