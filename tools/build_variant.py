"""Build an A/B variant of libh9g: hybrid9_amd/lib/libh9g_<tag>.so with extra
hipcc flags (e.g. -DH9G_STAMPS, -mllvm ...).  Usage:
    python tools/build_variant.py <tag> [--c2] [flags...]
Several variants build in parallel when started as separate processes.
The variants are measurement builds; the product is libh9g.so."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from hybrid9_amd import build as hb  # noqa: E402


def main() -> None:
    tag, extra = sys.argv[1], sys.argv[2:]
    if "--c2" in extra:      # config-2 instantiation only (h9g.hip H9G_ONLY_C2): ~1 min
        extra = [e for e in extra if e != "--c2"] + ["-DH9G_ONLY_C2"]
    out = hb.OUT.with_name(f"libh9g_{tag}.so")
    cmd = [hb.hipcc(), f"--offload-arch={hb.ARCH}", *hb.FLAGS, *extra, hb.id_flag(extra), str(hb.SRC),
           str(hb.SRC_IO), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(f"{tag}: hipcc failed\n{r.stderr[-3000:]}")
    print(f"{tag}: {out}")


if __name__ == "__main__":
    main()
