"""Which cells of a bench workload reach a reference STOP, and where.

Runs the bench's synthetic years (1901 + 0..nyears-1, seed SEED + rank 0)
through the product path on cuda:0 and writes every failed cell's global id
and STOP record to a JSON file, for tests/golden/make_stop_cells.py to
reproduce with the reference.  Usage (GPU box):
    python tools/find_stops.py [--workload config2] [--years 25] [--out gpurun_out/stops.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config2")
    ap.add_argument("--years", type=int, default=25)
    ap.add_argument("--out", default="gpurun_out/stops.json")
    a = ap.parse_args()
    import bench
    import hybrid9_amd as h
    from hybrid9_amd import synth
    pl = bench.plan(a.workload, 0, a.years, 1, 0, False, None)
    gid, lat = pl["gid"], pl["lat"]
    ctx = h.Context(gid.size, pl["zi"], nlayers=pl["L"], nisurf=pl["ns"], grow_on=pl["grow_on"], nslots=2)
    ctx.set_cells(gid, lat)
    ctx.synth_params(pl["seed"])
    ctx.init_state()
    first = {}
    for k, y in enumerate(pl["years"]):
        ctx.synth_forcing(k % 2, pl["seed"], synth.year_day0(y), synth.days_in_year(y))
        ctx.run_year(k % 2, y)
        ctx.sync(raise_on_stop=False)
        rec = ctx.get_errors()
        for c in np.nonzero(rec["code"])[0]:
            if int(c) not in first:
                first[int(c)] = dict(index=int(c), gid=int(gid[c]), year=y, code=int(rec["code"][c]),
                                     day=int(rec["day"][c]), substep=int(rec["substep"][c]),
                                     value=float(rec["value"][c]))
                print("STOP", first[int(c)], flush=True)
    out = dict(workload=a.workload, seed=pl["seed"], years=[pl["years"][0], pl["years"][-1]],
               ncell=int(gid.size), stops=sorted(first.values(), key=lambda r: r["index"]))
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
