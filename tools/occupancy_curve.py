#!/usr/bin/env python3
"""Config-2 pair kernel (0.5 deg, L=8, NISURF=48) timed at 1, 2 and 3 resident
waves per SIMD and at 2 rounds of 3: the first cells of the 0.5 deg land list
(the last size repeats the list, cells are independent), 22 columns per wave,
4-wave workgroups, one workgroup per CU per round of 256.  Shows how far the
SIMD's throughput rises with the waves that share it (latency hiding).

    python3 tools/occupancy_curve.py [--years 1]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

COLS_PER_WG = 88          # 4 waves x 22 columns (h9g.hip pair kernel)
Y0 = 1905                 # warm-up year; timed from 1906 as the driver's bench


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--years", type=int, default=1)
    args = ap.parse_args()
    import torch
    import hybrid9_amd as h
    from hybrid9_amd import synth
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    gid_all = synth.land_cells(synth.NX05, synth.NY05, synth.NLAND05)
    lat_all = synth.cell_lat(gid_all, synth.NX05, synth.NY05)
    base = None
    for w in (1, 2, 3, 6):
        n = w * ncu * COLS_PER_WG
        idx = np.arange(n) % gid_all.size
        g, la = gid_all[idx], lat_all[idx]
        with h.Context(g.size, synth.ZI_L8, nlayers=8, nisurf=48, grow_on=False,
                       nslots=1 + args.years) as ctx:
            ctx.set_cells(g, la)
            ctx.synth_params(synth.SEED)
            ctx.init_state()
            for s in range(1 + args.years):
                ctx.synth_forcing(s, synth.SEED, synth.year_day0(Y0 + s), synth.days_in_year(Y0 + s))
            ctx.run_year(0, Y0)
            ctx.sync(raise_on_stop=False)
            ctx.total_kernel_ms(reset=True)
            t0 = time.perf_counter()
            for s in range(args.years):
                ctx.run_year(1 + s, Y0 + 1 + s)
            ctx.sync(raise_on_stop=False)
            wall = (time.perf_counter() - t0) * 1e3 / args.years
            kms = ctx.total_kernel_ms(reset=True) / args.years
        per_wave = kms / w
        base = base or per_wave
        print(f"waves/SIMD={w} cells={n} kernel={kms:.1f} ms (wall {wall:.1f}) "
              f"ms per wave-slot={per_wave:.1f} SIMD throughput x{base / per_wave:.2f} vs 1 wave",
              flush=True)


if __name__ == "__main__":
    main()
