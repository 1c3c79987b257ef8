"""Fortran host (hybrid9_amd/fortran): the ISO_C_BINDING module and the
HYBRID9.f90-style driver compile with amdflang and link against the C-ABI;
on a GPU the driver reproduces the reference goldens end to end."""
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import hybrid9_amd as h
from oracle import refcase
from tests.conftest import load_golden, same_bits

ROOT = Path(__file__).resolve().parents[1]
FDIR = ROOT / "hybrid9_amd" / "fortran"
HOST = ROOT / "hybrid9_amd" / "lib" / "h9_host"


def _build():
    from hybrid9_amd import build
    build.build()
    if shutil.which("amdflang") is None and not Path("/opt/rocm/bin/amdflang").exists():
        pytest.skip("amdflang not available")
    subprocess.run(["make", "-s", "-C", str(FDIR)], check=True)
    return HOST


def test_fortran_host_builds_and_binds_every_entry_point():
    exe = _build()
    assert exe.exists()
    und = subprocess.run(["nm", "-u", str(exe)], capture_output=True, text=True).stdout
    src = (FDIR / "h9_gpu.f90").read_text()
    bound = set(__import__("re").findall(r"NAME='(h9g_[a-z_0-9]+)'", src))
    declared = set(h.exported_symbols()) - {"h9g_kernel_name", "h9g_math_selftest", "h9g_math_fast_selftest",
                                             "h9g_div_selftest", "h9g_pace_probe"}
    assert declared <= bound, sorted(declared - bound)
    for s in ("h9g_create", "h9g_run_year", "h9g_get_annual", "h9g_sync"):
        assert s in und


def test_fortran_host_reads_driver_txt(tmp_path):
    """driver.txt is read with the reference's list-directed sequence
    (INIT.f90:181-204); without a GPU the host stops cleanly."""
    exe = _build()
    drv = tmp_path / "driver.txt"
    drv.write_text("'/tmp/out' ! Path\n48 ! NISURF\n.T. ! PGF\n 1\n 1\n.F.\n .F.\n 'a'\n 'b'\n"
                   " 2002\n 2003\n 10\n-120.95\n 38.41\n 1\n 1\n" +
                   "".join(f"{v}\n" for v in (0.0, 45.0, 91.0, 166.0, 289.0, 493.0, 829.0,
                                               1383.0, 2296.0, 5000.0)))
    r = subprocess.run([str(exe), str(drv), str(tmp_path / "none.nml")], capture_output=True,
                       text=True, cwd=tmp_path, timeout=600)
    if h.lib().h9g_device_count() == 0:
        assert "no GPU visible" in r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1_10x10", "edge", "co_c1_30yr"])
def test_fortran_host_matches_reference_golden(tmp_path, name):
    exe = _build()
    meta, inp, exp = load_golden(name)
    n, L = meta["ncell"], meta["L"]
    st0 = None if inp["state0"] is None else refcase.unpack_state(inp["state0"], n, L)
    case = tmp_path / "case"
    # co_*: the reference's cell order (case.nml cell_order = 1: the host's
    # decade loop through h9g_run_decade_ordered); the others isolated cells
    refcase.write_case(case, zi=inp["zi"], params=inp["params"], forcing=inp["forcing"],
                       nisurf=inp["nisurf"], year0=inp["year0"], nyears=inp["nyears"],
                       grow_on=inp["grow_on"], state0=st0, cell_order=meta["kind"] == "cell_order")
    nml = tmp_path / "h9gpu.nml"
    nml.write_text(f"&h9gpu\n input_mode='case', case_dir='{case}', out_dir='{tmp_path}'\n/\n")
    r = subprocess.run([str(exe), str(tmp_path / "no_driver.txt"), str(nml)], capture_output=True,
                       text=True, timeout=600)
    assert "completed successfully" in r.stdout, r.stdout + r.stderr
    assert ("in cell order" in r.stdout) == (meta["kind"] == "cell_order")
    ann = np.fromfile(tmp_path / "annual.f32", np.float32).reshape(meta["nyears"], 12 + L, n)
    st = np.fromfile(tmp_path / "state_end.f32", np.float32)
    assert same_bits(ann, exp["annual"])
    assert same_bits(st, exp["state"])


@pytest.mark.gpu
def test_fortran_host_pgf_netcdf_mode(tmp_path):
    """The Fortran host's PGF path: forcing from decade netCDF-4 files named
    as READ_PGF.f90:22-106 (HDF5 chunk reads, async prefetch), annual output as axyYYYY.nc
    (HYBRID9.f90:503-513, WRITE_NET_CDF_3DR.f90); equal to the Python mirror
    fed the same forcing."""
    from scipy.io import netcdf_file
    from hybrid9_amd import synth
    from tests.helpers import nc4_writer_bin, write_nc4
    if nc4_writer_bin() is None:
        pytest.skip("no HDF5 headers to write netCDF-4 files")
    exe = _build()
    nx, ny, nland = 20, 10, 48
    gid = synth.land_cells(nx, ny, nland)
    lat = synth.cell_lat(gid, nx, ny)
    nt = sum(synth.days_in_year(1901 + k) for k in range(10))
    f = synth.make_forcing(gid, lat, 0, 366 + 365)          # the first two years suffice
    full = np.full((7, nt, ny * nx), np.float32(280.0))
    full[:, :f.shape[1]][:, :, gid] = f
    pgf = tmp_path / "pgf"
    pgf.mkdir()
    for k, v in enumerate(h.PGF_VARS):   # real netCDF-4 (HDF5): one chunk per day, shuffle + deflate
        write_nc4(pgf / f"{v}_pgfv2.1_1901_1910.nc4", v, full[k].reshape(nt, ny, nx))
    out = tmp_path / "out"
    out.mkdir()
    drv = tmp_path / "driver.txt"
    drv.write_text(f"'{out}'\n48\n.T.\n 1\n 1\n.F.\n .F.\n 'a'\n 'b'\n 1901\n 1902\n 0\n0.0\n0.0\n 1\n 1\n" +
                   "".join(f"{v}\n" for v in synth.ZI_L8[:10]))
    nml = tmp_path / "h9gpu.nml"
    # isolated cells (cell_order = 0), compared with h9g_run_year below
    nml.write_text(f"&h9gpu\n input_mode='pgf', pgf_dir='{pgf}', out_dir='{tmp_path}', grow_on=1,\n"
                   f" year0=1901, nyears=2, gnx={nx}, gny={ny}, gnland={nland}, cell_order=0\n/\n")
    r = subprocess.run([str(exe), str(drv), str(nml)], capture_output=True, text=True, timeout=600)
    assert "completed successfully" in r.stdout, r.stdout + r.stderr
    ann = np.fromfile(tmp_path / "annual.f32", np.float32).reshape(2, 20, nland)
    with h.Context(nland, synth.ZI_L8, nisurf=48) as ctx:      # the Python mirror, same inputs
        ctx.set_cells(gid, lat)
        ctx.synth_params(synth.SEED)
        ctx.init_state()
        ctx.push_forcing(0, f[:, :365])
        ctx.run_year(0, 1901)
        ctx.sync()
        a0 = ctx.get_annual()
        ctx.push_forcing(1, f[:, 365:365 + 365])
        ctx.run_year(1, 1902)
        ctx.sync()
        a1 = ctx.get_annual()
    assert same_bits(ann[0], a0) and same_bits(ann[1], a1)
    for y, a in ((1901, a0), (1902, a1)):
        with netcdf_file(out / f"axy{y}.nc", "r", mmap=False) as nc:
            assert same_bits(nc.variables["runoff"][:].reshape(-1)[gid], a[2])
            assert same_bits(nc.variables["soil_water"][:].reshape(-1)[gid], a[19])
