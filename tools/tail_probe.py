"""The cell order's re-run tail in isolation: N cells of the config-2 grid
on a context of their own, each simulated year one launch, timed per year.
With H9G_KERNEL=pair1 every launch runs the one-column kernel that the tail
runs on (lone waves, one per SIMD); with an H9G_STAMPS build (H9G_LIB) the
sync prints the phase cycles per wave-substep.

    python tools/tail_probe.py [ncell] [years]     (env: H9G_KERNEL, H9G_LIB)
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import hybrid9_amd as h  # noqa: E402
from hybrid9_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
ny = int(sys.argv[2]) if len(sys.argv) > 2 else 6
pl = bench.plan("config2", 0, ny)
idx = [(k * 7919) % pl["gid"].size for k in range(n)]      # cells spread over the grid
gid, lat = pl["gid"][idx], pl["lat"][idx]
ctx = h.Context(n, pl["zi"], nlayers=pl["L"], nisurf=pl["ns"], grow_on=pl["grow_on"], nslots=pl["nslots"])
ctx.set_cells(gid, lat)
ctx.synth_params(pl["seed"])
ctx.init_state()
for slot, y in enumerate(pl["slot_year"]):
    ctx.synth_forcing(slot, pl["seed"], synth.year_day0(y), synth.days_in_year(y))
ctx.sync()
print(f"tail probe: {n} cells, kernel {ctx.kernel_name()}", flush=True)
for s, y in enumerate(pl["years"]):
    ctx.run_year(pl["slot_of_step"][s], y)
    ctx.sync(raise_on_stop=False)
    print(f"{y} {ctx.last_kernel_ms():8.2f} ms  ({ctx.last_kernel_ms() / (synth.days_in_year(y) * pl['ns']) * 1e3:.2f} "
          f"us per substep)", flush=True)
