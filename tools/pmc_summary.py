#!/usr/bin/env python3
"""Summarise a tools/prof.sh output dir into profiles/pmc_<tag>.json and copy
the rocprofv3 --stats kernel table to profiles/<tag>_kernel_stats.csv.

The summary records the build_id of the library the profiled bench runs
loaded (every pass must agree); bench.py attaches a summary's counters only
to a library of the same build_id.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a coalesced streaming read, so it is doubled."""
import csv
import json
import shutil
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def counters(d: Path, kernel: str):
    out = defaultdict(list)
    for f in d.glob("*/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                out[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}, {k: len(v) for k, v in out.items()}


def bench_build_ids(d: Path):
    """The build_id of the library each pass's bench.py run loaded (its JSON
    line, roofline.build_id): the profile belongs to that build only."""
    ids = {}
    for log in sorted(d.glob("*.log")):
        for line in log.read_text(errors="replace").splitlines():
            if line.startswith("{") and '"metric"' in line:
                try:
                    ids[log.stem] = json.loads(line)["roofline"].get("build_id")
                except Exception:
                    pass
    return ids


def main(tag, workload="config2", kernel="h9g_"):
    d = ROOT / "gpurun_out" / f"prof_{tag}"
    ids = bench_build_ids(d)
    if not ids or len(set(ids.values())) != 1 or None in ids.values():
        raise SystemExit(f"passes of prof_{tag} ran different or unknown builds: {ids}")
    build = next(iter(ids.values()))
    stats = list(csv.DictReader(open(d / "kt" / "kt_kernel_stats.csv")))
    ks = max((r for r in stats if kernel in r["Name"]), key=lambda r: float(r["TotalDurationNs"]))
    c, n = counters(d, ks["Name"].split("(")[0].replace("void ", ""))
    avg_ns = float(ks["AverageNs"])
    fetch = 2.0 * c["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in c else None
    write = c["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in c else None
    waves = c.get("SQ_WAVES")
    res = {
        "tag": tag, "workload": workload, "kernel": ks["Name"], "build_id": build,
        "kernel_stats": f"profiles/{tag}_kernel_stats.csv",
        "source": f"rocprofv3 --pmc (separate FETCH_SIZE / WRITE_SIZE passes), profiles/pmc_{tag}.json",
        "kernel_avg_ns_rocprof": avg_ns, "launches": int(ks["Calls"]),
        "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
        "hbm_bytes_per_launch": (fetch or 0) + (write or 0) if fetch is not None else None,
        "hbm_GBps_measured": ((fetch or 0) + (write or 0)) / (avg_ns * 1e-9) / 1e9 if fetch else None,
        "counters_per_launch": c,
    }
    if waves:
        res["per_wave"] = {k: v / waves for k, v in c.items() if k.startswith("SQ_INSTS")}
    (ROOT / "profiles" / f"pmc_{tag}.json").write_text(json.dumps(res, indent=1))
    shutil.copy(d / "kt" / "kt_kernel_stats.csv", ROOT / "profiles" / f"{tag}_kernel_stats.csv")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
