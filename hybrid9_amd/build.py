"""Build the gfx950 HIP library ``hybrid9_amd/lib/libh9g.so`` in-tree.

``python -m hybrid9_amd.build`` (also called by ``__graft_entry__.build()``).
hipcc cross-compiles for gfx950 without a GPU.  Numerics flags are part of
the parity contract: ``-ffp-contract=off`` (the reference executes no FMA;
h9_math.h issues its FMAs explicitly) and HIP's default correctly-rounded
f32 division/sqrt and f32 denormal support are kept (no fast-math).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "csrc" / "h9g.hip"
SRC_IO = HERE / "csrc" / "h9g_io.cpp"       # host-only NetCDF I/O
DEPS = [SRC, SRC_IO, HERE / "csrc" / "h9_math.h", HERE / "csrc" / "h9g_step.h",
        HERE / "csrc" / "h9g_synth.h", HERE / "csrc" / "h9g_geo.h",
        HERE / "csrc" / "h9g_pair.h", HERE / "csrc" / "h9g_io.h",
        HERE.parent / "include" / "h9g.h"]
OUT = HERE / "lib" / "libh9g.so"
ARCH = os.environ.get("H9G_ARCH", "gfx950")

FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fhip-fp32-correctly-rounded-divide-sqrt", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-value"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and Path(c).exists():
            return c
    raise FileNotFoundError("hipcc not found")


def build_id(extra=()) -> str:
    """Digest of everything the library is compiled from: the sources, the
    flags and the target.  It is compiled into the library (h9g_build_id)
    and recorded with every profile (tools/pmc_summary.py), so bench.py
    attaches counters only to the build they were measured on."""
    import hashlib
    hs = hashlib.sha256()
    for d in DEPS:
        hs.update(d.name.encode() + b"\0" + d.read_bytes() + b"\0")
    hs.update(" ".join([ARCH, *FLAGS, *extra]).encode())
    return hs.hexdigest()[:16]


def id_flag(extra=()) -> str:
    return f'-DH9G_BUILD_ID="{build_id(extra)}"'


def up_to_date() -> bool:
    if not OUT.exists():
        return False
    t = OUT.stat().st_mtime
    return all(d.stat().st_mtime <= t for d in DEPS)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{r.stderr[-4000:]}")


def build(force: bool = False, verbose: bool = False, extra=()) -> Path:
    """Compiles the two translation units to objects (the device code, ~4
    minutes, and the host-only NetCDF I/O, seconds; each only when its own
    inputs changed, keyed by their digest) and links libh9g.so."""
    if not force and up_to_date():
        return OUT
    OUT.parent.mkdir(parents=True, exist_ok=True)
    obj = OUT.parent / "obj"
    obj.mkdir(exist_ok=True)
    import hashlib
    flags = [f"--offload-arch={ARCH}", *FLAGS, *extra]
    objs = []
    # h9g_build_id lives in the I/O unit: only it gets the digest flag
    for src, deps, idf in ((SRC, [d for d in DEPS if d != SRC_IO], []),
                           (SRC_IO, [SRC_IO, HERE / "csrc" / "h9g_io.h", DEPS[-1]], [id_flag(extra)])):
        flags_u = flags + idf
        hs = hashlib.sha256(" ".join(flags_u).encode())
        for d in deps:
            hs.update(d.read_bytes())
        o = obj / f"{src.stem}_{hs.hexdigest()[:16]}.o"
        if force or not o.exists():
            for old in obj.glob(f"{src.stem}_*.o"):
                old.unlink()
            tmp = o.with_suffix(".o.tmp")
            _run([hipcc(), *[f for f in flags_u if f != "-shared"], "-c", str(src), "-o", str(tmp)], verbose)
            os.replace(tmp, o)
        objs.append(str(o))
    tmp = OUT.with_suffix(".so.tmp")
    _run([hipcc(), f"--offload-arch={ARCH}", "-fPIC", "-shared", *objs, "-o", str(tmp)], verbose)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    p = build(force="--force" in sys.argv, verbose=True)
    print(p)
