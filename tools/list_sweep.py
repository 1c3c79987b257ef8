"""Year time of the cell order's re-run lists by size and kernel: k cells of
a workload's grid on a context of their own, one warm-up year, then one
timed year per kernel choice (H9G_KERNEL).  The lists of h9g_run_ordered
run at these sizes (config 2's tail is ~100 cells, the GROW-on
configurations' ~30% of the grid).

    python tools/list_sweep.py [workload] [sizes,...] [kernels,...]
"""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import hybrid9_amd as h  # noqa: E402
from hybrid9_amd import synth  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "config3"
sizes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1000,4000,10000,20000").split(",")]
kinds = (sys.argv[3] if len(sys.argv) > 3 else "pair,pair11,pair1").split(",")
pl = bench.plan(wl, 0, 2)
for k in sizes:
    idx = [(j * 7919) % pl["gid"].size for j in range(k)]
    gid, lat = pl["gid"][idx], pl["lat"][idx]
    row = [f"{wl} k={k}"]
    for kind in kinds:
        if kind == "pair1" and k > 4096:
            continue
        os.environ["H9G_KERNEL"] = kind
        with h.Context(k, pl["zi"], nlayers=pl["L"], nisurf=pl["ns"], grow_on=pl["grow_on"], nslots=2) as ctx:
            ctx.set_cells(gid, lat)
            ctx.synth_params(pl["seed"])
            ctx.init_state()
            for slot, y in enumerate(pl["slot_year"]):
                ctx.synth_forcing(slot, pl["seed"], synth.year_day0(y), synth.days_in_year(y))
            ctx.run_year(0, 1901)
            ctx.sync(raise_on_stop=False)
            ctx.run_year(1, 1902)
            ctx.sync(raise_on_stop=False)
            row.append(f"{kind} {ctx.last_kernel_ms():.1f} ms")
    print(" | ".join(row), flush=True)
