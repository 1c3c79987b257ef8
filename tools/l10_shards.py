#!/usr/bin/env python3
"""Time one 0.25 deg, L=10 year (config 5) per kernel on the shard sizes of
strong scaling over 1/2/4/8 GPUs (h9g.hip l10_kind picks between them).

    python3 tools/l10_shards.py [--years 1]
    python3 tools/l10_shards.py --ordered      (the reference's cell order)

--ordered: per shard, the decades 1911-1930 in the reference's own cell
order (one h9g_run_ordered call, after 1901-1910 untimed), the shard one chain (one
reference rank's block): ms per simulated year, and how the time splits
between the year launches of the first pass (with the re-runs riding in
them), the year-1 re-run and the one-column tail launches.
"""
import argparse
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--years", type=int, default=1)
    ap.add_argument("--ordered", action="store_true")
    args = ap.parse_args()
    if args.ordered:
        return ordered()
    import hybrid9_amd as h
    from hybrid9_amd import synth
    from hybrid9_amd.shard import shard_slice
    gid = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
    lat = synth.cell_lat(gid, synth.NX025, synth.NY025)
    for world in [int(w) for w in os.environ.get("L10_WORLDS", "1,2,4,8").split(",")]:
        sl = shard_slice(gid.size, 0, world)
        g, la = gid[sl], lat[sl]
        row = [f"N={world} cells={g.size}"]
        for k in os.environ.get("L10_KINDS", "pair,pair2,pair11,solo,mixed,auto").split(","):
            if k == "auto":
                os.environ.pop("H9G_KERNEL", None)
            else:
                os.environ["H9G_KERNEL"] = k
            with h.Context(g.size, synth.ZI_L10, nlayers=10, nisurf=24, grow_on=True,
                           nslots=1 + args.years) as ctx:
                ctx.set_cells(g, la)
                ctx.synth_params(synth.SEED)
                ctx.init_state()
                for s in range(1 + args.years):
                    ctx.synth_forcing(s, synth.SEED, synth.year_day0(1901 + s), synth.days_in_year(1901 + s))
                ctx.run_year(0, 1901)
                ctx.sync(raise_on_stop=False)
                ctx.total_kernel_ms(reset=True)
                t0 = time.perf_counter()
                for s in range(args.years):
                    ctx.run_year(1 + s, 1902 + s)
                ctx.sync(raise_on_stop=False)
                wall = (time.perf_counter() - t0) * 1e3 / args.years
                kms = ctx.total_kernel_ms(reset=True) / args.years
                row.append(f"{k}={ctx.kernel_name()} {kms:.1f} ms (wall {wall:.1f})")
        print(" | ".join(row), flush=True)


def ordered():
    import hybrid9_amd as h
    from hybrid9_amd import synth
    from hybrid9_amd.shard import shard_slice
    gid = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
    lat = synth.cell_lat(gid, synth.NX025, synth.NY025)
    years = list(range(1901, 1931))
    for world in [int(w) for w in os.environ.get("L10_WORLDS", "1,2,4,8").split(",")]:
        sl = shard_slice(gid.size, 0, world)
        g, la = gid[sl], lat[sl]
        with h.Context(g.size, synth.ZI_L10, nlayers=10, nisurf=24, grow_on=True, nslots=len(years)) as ctx:
            ctx.set_cells(g, la)
            ctx.synth_params(synth.SEED)
            ctx.init_state()
            for s, y in enumerate(years):
                ctx.synth_forcing(s, synth.SEED, synth.year_day0(y), synth.days_in_year(y))
            ctx.sync()
            ctx.run_ordered(list(range(10)), 1901, raise_on_stop=False, annual=False)
            ctx.launch_stats(reset=True)
            t0 = time.perf_counter()
            ctx.run_ordered(list(range(10, 30)), 1911, raise_on_stop=False, annual=False)
            wall = (time.perf_counter() - t0) * 1e3 / 20
            ls = ctx.launch_stats(reset=True)
            st, ov = ctx.decade_stats(), ctx.ordered_stats()
            parts = ", ".join(f"{k} {v['launches']} x {v['ms'] / v['launches']:.1f} ms" for k, v in ls.items())
            print(f"N={world} cells={g.size} kernel={ctx.kernel_name()}: {wall:.1f} ms per year in cell order "
                  f"({parts}); re-run launches {st['launch_cells']}; riding {ov['rerun_years_riding']} "
                  f"years / {ov['rerun_cell_years_riding']} cell-years; passes {ov['passes']}", flush=True)


if __name__ == "__main__":
    main()
