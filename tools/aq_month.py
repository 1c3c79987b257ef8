#!/usr/bin/env python3
"""Offline replay of a re-sort within the year: would
splitting h9g_run_year into monthly launches, with h9g_sort_kernel re-keyed
between them, cut the wave-days whose 22 columns hold both kinds of water
table (below the column: the aquifer node; inside it: the recharge and
water-table loops, HYDROLOGY.f90:499-508,574-590,856-1118)?

    python tools/aq_month.py gpurun_out/aq_<tag>.bin

Reads the day-level record of the H9G_DUMP_AQ build (tools/aq_sort.py
read()).  For every month m >= 1 of every year after the first, each key is
computed from what a sort at the start of month m could know -- the record
of the current year up to that day and the last year's -- and the mixed
wave-days are counted over month m's days only, with the cells cut into
waves exactly as h9g_sort_kernel does (aq_sort.mixed).  The yearly key the
product uses ("fraction/8" of the last year) is scored on the same days."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
from aq_sort import mixed, read  # noqa: E402


def frac_bucket(frac, nb=8):
    return np.where(frac == 0, 0, np.where(frac == 1, nb + 1, 1 + np.minimum(nb - 1, (frac * nb).astype(np.int64))))


def month_edges(nt):
    return [len(a) for a in np.array_split(np.arange(nt), 12)]


def main():
    recs = read(sys.argv[1])
    rows = {}
    for (py, prev), (y, cur) in zip(recs, recs[1:]):
        if prev.shape[0] != cur.shape[0]:
            continue
        nt = cur.shape[1]
        e = np.concatenate([[0], np.cumsum(month_edges(nt))])
        yearly = frac_bucket(prev.mean(axis=1))
        for m in range(1, 12):
            d0, d1 = e[m], e[m + 1]
            days = cur[:, d0:d1]
            last = cur[:, e[m - 1]:d0]                      # the month before
            last30 = cur[:, max(0, d0 - 30):d0]
            keys = {
                "yearly: last year's fraction/8 (product)": yearly,
                "month start state": cur[:, d0].astype(np.int64),
                "last month's fraction/8": frac_bucket(last.mean(axis=1)),
                "last month's fraction/8 + start state": frac_bucket(last.mean(axis=1)) * 2 + cur[:, d0],
                "start state + last year's fraction/8": cur[:, d0].astype(np.int64) * 16 + yearly,
                "last 30 days /8 + last year's /8": frac_bucket(last30.mean(axis=1)) * 16 + yearly,
            }
            for name, k in keys.items():
                rows.setdefault(name, []).append((mixed(days, k)[0], d1 - d0, y))
            rows.setdefault("floor: this month's own fraction/32", []).append(
                (mixed(days, frac_bucket(days.mean(axis=1), 32))[0], d1 - d0, y))
    print(f"years {[y for y, _ in recs]}; months 2-12 of each year after the first; mixed wave-days (weighted by days)")
    years = sorted({int(r[2]) for v in rows.values() for r in v})
    print(f"  {'key':42s} {'all':>6s} " + " ".join(f"{y:>6d}" for y in years))
    for name, v in rows.items():
        v = np.array(v)
        per = [np.average(v[v[:, 2] == y, 0], weights=v[v[:, 2] == y, 1]) for y in years]
        print(f"  {name:42s} {np.average(v[:, 0], weights=v[:, 1]):6.3f} " + " ".join(f"{x:6.3f}" for x in per))


if __name__ == "__main__":
    main()
