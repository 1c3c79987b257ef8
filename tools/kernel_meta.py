#!/usr/bin/env python3
"""Register and scratch metadata of every kernel in a built libh9g.so,
read from its gfx950 code object (the numbers DESIGN.md quotes).

    python tools/kernel_meta.py [hybrid9_amd/lib/libh9g.so] [--all]

Extracts the .hip_fatbin section, unbundles the gfx950 code object with
clang-offload-bundler and reads the AMDHSA metadata note with llvm-readelf:
VGPRs, AGPRs, SGPRs, spilled VGPRs/SGPRs, private (scratch) bytes per lane
and static LDS bytes per workgroup.  Without --all only the year kernels
(pair, pair2, solo) are printed."""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
ROOT = Path(__file__).resolve().parents[1]


def code_object(lib: Path, tmp: Path) -> Path:
    fat = tmp / "fat.bin"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib), str(tmp / "x.so")],
                   check=True)
    co = tmp / "gfx950.co"
    subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                    f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
    return co


def kernels(co: Path) -> list[dict]:
    notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], capture_output=True, text=True,
                           check=True).stdout
    out, cur = [], None
    keys = {".name": "name", ".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
            ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill",
            ".private_segment_fixed_size": "private_bytes", ".group_segment_fixed_size": "lds_bytes"}
    for line in notes.splitlines():
        m = re.match(r"\s*-?\s*(\.[a-z_]+):\s*(.+)$", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == ".args":
            continue
        if k == ".name" and not v.startswith("_Z") and cur is not None and "name" in cur:
            continue
        if k == ".group_segment_fixed_size" and (cur is None or "lds_bytes" in cur):
            cur = {}
            out.append(cur)
        if k in keys and cur is not None:
            cur[keys[k]] = v if k == ".name" else int(v)
    return [k for k in out if "name" in k]


def demangle(names: list[str]) -> list[str]:
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines() if r.returncode == 0 else names


def main() -> None:
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = Path(pos[0]) if pos else ROOT / "hybrid9_amd" / "lib" / "libh9g.so"
    with tempfile.TemporaryDirectory() as t:
        ks = kernels(code_object(lib, Path(t)))
    names = demangle([k["name"] for k in ks])
    print(f"{lib.name}: {len(ks)} kernels")
    print(f"{'kernel':60s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'VGPR spill':>10s} {'SGPR spill':>10s} "
          f"{'private B':>9s} {'LDS B':>7s}")
    for k, nm in sorted(zip(ks, names), key=lambda x: x[1]):
        if "--all" not in sys.argv and not re.search(r"h9g_(pair|pair1|pair2|pair11|solo)_kernel", nm):
            continue
        short = nm.replace("h9k::", "").replace("(KArgs, ", "(")
        print(f"{short[:60]:60s} {k.get('vgpr', 0):5d} {k.get('agpr', 0):5d} {k.get('sgpr', 0):5d} "
              f"{k.get('vgpr_spill', 0):10d} {k.get('sgpr_spill', 0):10d} {k.get('private_bytes', 0):9d} "
              f"{k.get('lds_bytes', 0):7d}")


if __name__ == "__main__":
    main()
