"""Per-year kernel time of a workload over a run of years (state carried).
Usage: python tools/year_probe.py <workload> <nyears>   (H9G_LIB selects a build)"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import hybrid9_amd as h  # noqa: E402
from hybrid9_amd import synth  # noqa: E402

wl, ny = sys.argv[1], int(sys.argv[2])
pl = bench.plan(wl, 0, ny)
ctx = h.Context(pl["gid"].size, pl["zi"], nlayers=pl["L"], nisurf=pl["ns"], grow_on=pl["grow_on"],
                nslots=pl["nslots"])
ctx.set_cells(pl["gid"], pl["lat"])
ctx.synth_params(pl["seed"])
ctx.init_state()
for slot, y in enumerate(pl["slot_year"]):
    ctx.synth_forcing(slot, pl["seed"], synth.year_day0(y), synth.days_in_year(y))
ctx.sync()
for s, y in enumerate(pl["years"]):
    ctx.run_year(pl["slot_of_step"][s], y)
    ctx.sync(raise_on_stop=False)
    d = ctx.get_diagnostics()
    print(f"{wl} {y} {ctx.last_kernel_ms():7.1f} ms  failed {int(d[11])}  lai {d[7] / d[0]:.3f}  "
          f"zwt {d[3] / d[0]:.3f}  theta1 {d[8] / d[0]:.4f}", flush=True)
