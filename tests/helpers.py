"""Test helpers: small native test tools built on demand into tests/_build."""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
BUILD = ROOT / "tests" / "_build"


def _build(src: Path, out: Path, cmd):
    if out.exists() and out.stat().st_mtime >= src.stat().st_mtime:
        return out
    BUILD.mkdir(exist_ok=True)
    subprocess.run(cmd, check=True)
    return out


def check_math_bin() -> Path:
    src = ROOT / "tests" / "csrc" / "check_math.cpp"
    out = BUILD / "check_math"
    hdr = ROOT / "hybrid9_amd" / "csrc" / "h9_math.h"
    if out.exists() and out.stat().st_mtime < hdr.stat().st_mtime:
        out.unlink()
    return _build(src, out, ["g++", "-O2", "-ffp-contract=off", "-fopenmp", "-std=c++17",
                             str(src), "-o", str(out), "-lm"])


_glibc = None


def glibc():
    global _glibc
    if _glibc is None:
        src = ROOT / "tests" / "csrc" / "glibc_ref.c"
        out = _build(src, BUILD / "libglibc_ref.so",
                     ["gcc", "-O2", "-fPIC", "-shared", str(src), "-o", str(BUILD / "libglibc_ref.so"), "-lm"])
        L = C.CDLL(str(out))
        fp = C.POINTER(C.c_float)
        L.glibc_expf_v.argtypes = [C.c_int, fp, fp]
        L.glibc_powf_v.argtypes = [C.c_int, fp, fp, fp]
        _glibc = L
    return _glibc


def glibc_expf(x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    fp = C.POINTER(C.c_float)
    glibc().glibc_expf_v(x.size, x.ctypes.data_as(fp), out.ctypes.data_as(fp))
    return out


def glibc_powf(x, y):
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    out = np.empty_like(x)
    fp = C.POINTER(C.c_float)
    glibc().glibc_powf_v(x.size, x.ctypes.data_as(fp), y.ctypes.data_as(fp), out.ctypes.data_as(fp))
    return out


def math_inputs(n=1 << 22, seed=7):
    """Random + hot-path-shaped (x, y) samples, incl. special values."""
    r = np.random.default_rng(seed)
    bits = r.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    xs = np.concatenate([bits,
                         r.uniform(-110, 90, n).astype(np.float32),
                         r.uniform(0.005, 1.0, n).astype(np.float32),
                         r.uniform(1.0, 5.0, n).astype(np.float32)])
    ys = np.concatenate([r.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32),
                         r.uniform(-12, 25, n).astype(np.float32),
                         r.uniform(-12, 25, n).astype(np.float32),
                         -r.uniform(0.5, 0.9, n).astype(np.float32)])
    sv = np.array([0.0, -0.0, 1.0, -1.0, 2.0, 0.5, np.inf, -np.inf, np.nan, 1e-45, 1e-38,
                   3e38, -3.0, 0.33333334, 2.8, 126.0, -150.0, 149.5], np.float32)
    gx, gy = np.meshgrid(sv, sv)
    return np.concatenate([xs, gx.ravel()]), np.concatenate([ys, gy.ravel()])


CONDA = Path("/opt/conda")


def nc4_writer_bin() -> Path | None:
    """tests/csrc/nc4_write.c against the image's HDF5 (None if absent)."""
    if not (CONDA / "include" / "hdf5.h").exists():
        return None
    src = ROOT / "tests" / "csrc" / "nc4_write.c"
    out = BUILD / "nc4_write"
    return _build(src, out, ["gcc", "-O1", f"-I{CONDA}/include", str(src), "-o", str(out),
                             f"-L{CONDA}/lib", f"-Wl,-rpath,{CONDA}/lib", "-lhdf5_hl", "-lhdf5"])


NC_FILL_FLOAT = np.float32(9.9692099683868690e+36)   # netCDF's default float fill (nc4_write.c)


def write_nc4(path: Path, var: str, data: np.ndarray, chunk=None, filters: str | None = None,
              skip: int | None = None) -> Path:
    """A netCDF-4 (HDF5) file with <var>(time, lat, lon) and its coordinate
    dimension scales (nc4_write.c); chunk (ct, cy, cx) and filters
    ("s" shuffle, "d" deflate, "f" fletcher32, "b" big-endian) default to one
    chunk per day, shuffle + deflate.  skip: a day whose time chunks are
    never written (they read as NC_FILL_FLOAT)."""
    exe = nc4_writer_bin()
    raw = path.with_suffix(".raw")
    np.ascontiguousarray(data, np.float32).tofile(raw)
    nt, ny, nx = data.shape
    extra = []
    if chunk is not None or filters is not None or skip is not None:
        ct, cy, cx = chunk if chunk is not None else (1, ny, nx)
        extra = [str(ct), str(cy), str(cx)] + ([filters if filters is not None else "sd"]
                                               if filters is not None or skip is not None else [])
        extra += [str(skip)] if skip is not None else []
    subprocess.run([str(exe), str(path), var, str(nt), str(ny), str(nx), str(raw), *extra], check=True)
    raw.unlink()
    return path
