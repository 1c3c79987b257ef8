"""Year-kernel time vs cell count and kernel choice (occupancy probe).
Usage: python tools/occ_probe.py kernel:ncell ...  (kernel = pair|solo)"""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import hybrid9_amd as h  # noqa: E402
from hybrid9_amd import synth  # noqa: E402

land = synth.land_cells()
for arg in sys.argv[1:]:
    k, n = arg.split(":")
    n = int(n)
    os.environ["H9G_KERNEL"] = k
    g = land[:n] if n <= land.size else land[(h.np.arange(n) % land.size)]
    ctx = h.Context(n, synth.ZI_L8, nlayers=8, nisurf=48, grow_on=False, nslots=1)
    ctx.set_cells(g, synth.cell_lat(g))
    ctx.synth_params(synth.SEED)
    ctx.init_state()
    ctx.synth_forcing(0, synth.SEED, 0, 365)
    ctx.sync()
    ms = []
    for y in range(3):
        ctx.run_year(0, 1901)
        ctx.sync(raise_on_stop=False)
        ms.append(ctx.last_kernel_ms())
    print(f"{k:5s} n={n:6d} {ctx.kernel_name():32s} ms/year " + " ".join(f"{m:.1f}" for m in ms), flush=True)
    ctx.close()
