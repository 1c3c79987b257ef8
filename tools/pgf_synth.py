#!/usr/bin/env python3
"""Synthetic PGF v2.1 netCDF-4 files for measuring forcing ingest
(READ_PGF.f90:22-109, READ_NET_CDF_3DR.f90:43-98), and a timing of
``h9g_nc_forcing_read`` on them.

The files hold the bench's own synthetic forcing (``synth.make_forcing``,
bit-identical to the device generator ``h9g_synth_forcing``) at the land
cells of the 0.5 deg grid and 1e20 over the ocean, in the on-disk form of a
PGF file: <var>(time, lat, lon) float32, one chunk per day, shuffle +
deflate level 4, with time/lat/lon dimension scales (tests/csrc/nc4_write.c).
A year run from these files must therefore give the same bits as one run
from the device generator (``bench.py --forcing nc4`` checks that).

    python tools/pgf_synth.py write DIR [--year 1901] [--days 366]
    python tools/pgf_synth.py read DIR [--days 365] [--threads N] [--shard K/N]
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import hybrid9_amd as h  # noqa: E402
from hybrid9_amd import synth  # noqa: E402

OCEAN = np.float32(1.0e20)


def decade_of(year: int) -> str:
    d0 = (year - 1) // 10 * 10 + 1
    return f"{d0}-{d0 + 9}"


def write_year(directory, year: int = 1901, ndays: int = 366, seed: int = synth.SEED,
               nx: int = synth.NX05, ny: int = synth.NY05, nland: int = synth.NLAND05) -> list[str]:
    """The 7 files of one year (days from year's Jan 1), READ_PGF names."""
    from tests.helpers import write_nc4
    d = Path(directory)
    d.mkdir(parents=True, exist_ok=True)
    g = synth.land_cells(nx, ny, nland)
    f = synth.make_forcing(g, synth.cell_lat(g, nx, ny), synth.year_day0(year), ndays, seed)
    paths = h.pgf_paths(d, decade_of(year))

    def one(k: int) -> str:
        full = np.full((ndays, ny * nx), OCEAN, np.float32)
        full[:, g] = f[k]
        return str(write_nc4(Path(paths[k]), h.PGF_VARS[k], full.reshape(ndays, ny, nx)))

    with ThreadPoolExecutor(max_workers=7) as ex:
        return list(ex.map(one, range(h.NFORCING)))


def time_read(paths, ndays: int, gid, nx: int = synth.NX05, ny: int = synth.NY05, reps: int = 2) -> dict:
    ts, stats = [], []
    out = None
    for _ in range(reps):
        t = time.perf_counter()
        out = h.nc_forcing_read(paths, nx, ny, gid, 0, ndays)
        ts.append(time.perf_counter() - t)
        stats.append(h.nc_read_stats())
    best = int(np.argmin(ts))
    return dict(seconds=ts[best], all=ts, out=out, stats=stats[best])


def stage_report(s: dict) -> str:
    """One line per stage of h9g_nc_read_stats: thread-seconds, share of
    the pool (wall x threads) and per-thread rate."""
    pool = s["pool_wall_s"] * s["threads"]
    busy = s["pread_s"] + s["inflate_s"] + s["gather_s"] + s["other_s"]
    lines = [f"  wall {s['wall_s']:.3f} s = setup {s['setup_s']:.3f} s + pool {s['pool_wall_s']:.3f} s "
             f"x {s['threads']:.0f} threads, {s['jobs']:.0f} jobs; busy {busy / max(pool, 1e-12):.2f} of the pool"]
    for k, what, b in (("pread_s", "stored bytes", s["bytes_read"]), ("inflate_s", "decoded bytes", s["bytes_decoded"]),
                       ("gather_s", "values", s["values"]), ("other_s", "", 0)):
        if s[k] <= 0:
            continue
        rate = f", {b / s[k] / 1e9:.2f} G{what} per thread-s" if b else ""
        lines.append(f"  {k[:-2]:8s} {s[k]:7.3f} thread-s ({s[k] / max(pool, 1e-12):.2f} of the pool){rate}")
    return "\n".join(lines)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["write", "read"])
    ap.add_argument("dir")
    ap.add_argument("--year", type=int, default=1901)
    ap.add_argument("--days", type=int, default=366)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--shard", default="0/1", help="K/N: the K-th of N contiguous cell shards")
    ap.add_argument("--check", action="store_true", help="compare with synth.make_forcing")
    a = ap.parse_args()
    if a.mode == "write":
        t = time.perf_counter()
        ps = write_year(a.dir, a.year, a.days)
        sz = sum(os.path.getsize(p) for p in ps)
        print(f"wrote {len(ps)} files, {sz / 1e9:.2f} GB, {time.perf_counter() - t:.1f} s")
        return
    if a.threads:
        os.environ["H9G_IO_THREADS"] = str(a.threads)
    g = synth.land_cells()
    k, n = (int(x) for x in a.shard.split("/"))
    from hybrid9_amd.shard import shard_slice
    sl = shard_slice(g.size, k, n)
    gs = g[sl]
    paths = h.pgf_paths(a.dir, decade_of(a.year))
    r = time_read(paths, a.days, gs)
    print(f"h9g_nc_forcing_read: {a.days} days x {gs.size} cells (shard {a.shard}): "
          f"{r['seconds']:.3f} s (runs {', '.join(f'{x:.3f}' for x in r['all'])}), "
          f"{a.days * 365.0 / a.days:.0f}-day year: {r['seconds'] * 365.0 / a.days:.3f} s")
    print(stage_report(r["stats"]))
    if a.check:
        ref = synth.make_forcing(gs, synth.cell_lat(gs), synth.year_day0(a.year), a.days)
        ok = np.array_equal(ref.view(np.uint32), r["out"].view(np.uint32))
        print("bit-equal to synth.make_forcing:", ok)
        if not ok:
            sys.exit(1)


if __name__ == "__main__":
    main()
