#!/usr/bin/env python3
"""Design the year kernel's cell order offline from a day-level record of
where each cell's water table was (H9G_DUMP_AQ build; h9g.hip h9g_sync writes
it to $H9G_AQ_DUMP: per year the year, n, then n x 12 words, bit d = water
table below the column at the start of day d).

    python tools/aq_sort.py gpurun_out/aq.bin

For every year after the first, each candidate key is computed from what the
sort kernel knows at the start of that year (the last year's record and the
current state), the cells are sorted stably within each XCD's range exactly
as h9g_sort_kernel orders them (xcd_vwg ranges of 88-cell workgroups), cut
into 22-column waves, and the script reports the fraction of wave-days whose
wave holds cells of both kinds (its substeps run both the aquifer node and
the recharge branches)."""
from __future__ import annotations

import sys

import numpy as np

PCPW, PWAVES, NXCD = 22, 4, 8


def read(path):
    raw = np.fromfile(path, dtype=np.uint32)
    recs, o = [], 0
    while o < raw.size:
        year, n = int(raw[o]), int(raw[o + 1])
        bits = raw[o + 2:o + 2 + 12 * n].reshape(n, 12)
        o += 2 + 12 * n
        nt = 366 if (year % 4 == 0 and (year % 100 != 0 or year % 400 == 0)) else 365
        days = np.unpackbits(bits.view(np.uint8).reshape(n, 48), axis=1, bitorder="little")[:, :nt].astype(bool)
        recs.append((year, days))
    return recs


def ranges(n):
    per = PCPW * PWAVES
    nb = (n + per - 1) // per
    q, r = divmod(nb, NXCD)
    out = []
    for x in range(NXCD):
        p0 = (x * q + min(x, r)) * per
        p1 = min(n, p0 + (q + (1 if x < r else 0)) * per)
        if p1 > p0:
            out.append((p0, p1))
    return out


def mixed(days, key):
    """fraction of wave-days with both kinds, and of wave-days with each kind"""
    n = days.shape[0]
    tot = mix = anyaq = anycol = 0
    for p0, p1 in ranges(n):
        idx = np.arange(p0, p1)
        order = idx[np.lexsort((idx, key[p0:p1]))]
        for w0 in range(0, order.size, PCPW):
            d = days[order[w0:w0 + PCPW]]
            a = d.any(axis=0)
            c = (~d).any(axis=0)
            tot += d.shape[1]
            mix += int((a & c).sum())
            anyaq += int(a.sum())
            anycol += int(c.sum())
    return mix / tot, anyaq / tot, anycol / tot


def keys(prev, cur):
    """candidate keys for the year `cur` from the last year's record"""
    nt = prev.shape[1]
    frac = prev.sum(axis=1) / nt
    start = cur[:, 0]
    k = {}
    k["index"] = np.zeros(prev.shape[0], dtype=np.int64)
    k["start state"] = start.astype(np.int64)
    fb = np.where(frac == 0, 0, np.where(frac == 1, 9, 1 + np.minimum(7, (frac * 8).astype(np.int64))))
    k["fraction/8"] = fb
    k["fraction/32"] = np.where(frac == 0, 0, np.where(frac == 1, 33, 1 + np.minimum(31, (frac * 32).astype(np.int64))))
    # monthly majority pattern, lexicographic (month 0 most significant)
    m = np.array_split(np.arange(nt), 12)
    pat = np.zeros(prev.shape[0], dtype=np.int64)
    for j, dd in enumerate(m):
        pat |= (prev[:, dd].mean(axis=1) > 0.5).astype(np.int64) << (11 - j)
    k["monthly pattern"] = pat
    # fraction bucket, then the day of the year the water table last dropped below
    # the column (phase of the oscillation), in 16ths
    drop = np.argmax(prev[:, ::-1] & ~np.roll(prev, 1, axis=1)[:, ::-1], axis=1)
    phase = ((nt - 1 - drop) * 16 // nt)
    k["fraction/8 + phase/16"] = fb * 16 + np.where((fb > 0) & (fb < 9), phase, 0)
    # monthly pattern ordered by fraction first
    k["fraction/8 + monthly"] = fb * 4096 + np.where((fb > 0) & (fb < 9), pat, 0)
    # 24 half-month majority bits
    m24 = np.array_split(np.arange(nt), 24)
    p24 = np.zeros(prev.shape[0], dtype=np.int64)
    for j, dd in enumerate(m24):
        p24 |= (prev[:, dd].mean(axis=1) > 0.5).astype(np.int64) << (23 - j)
    k["half-month pattern"] = p24
    # the current state first, then the last year's fraction
    k["start + fraction/8"] = start.astype(np.int64) * 16 + fb
    return k


def main():
    recs = read(sys.argv[1])
    print("years:", [y for y, _ in recs])
    res = {}
    for (py, prev), (y, cur) in zip(recs, recs[1:]):
        if prev.shape[0] != cur.shape[0]:
            continue
        for name, key in keys(prev, cur).items():
            res.setdefault(name, []).append(mixed(cur, key))
    for name, v in res.items():
        v = np.array(v)
        print(f"{name:28s} mixed {v[:, 0].mean():.3f}  any_aq {v[:, 1].mean():.3f}  any_col {v[:, 2].mean():.3f}"
              f"   per year {' '.join(f'{x:.3f}' for x in v[:, 0])}")



def oracle_bound(path):
    """lower bound-ish: keys from the year's own record (not available to the sort)"""
    recs = read(path)
    for y, cur in recs[1:]:
        frac = cur.mean(axis=1)
        fb = np.where(frac == 0, 0, np.where(frac == 1, 33, 1 + np.minimum(31, (frac * 32).astype(np.int64))))
        # exact pattern, lexicographic on the day bits (first day most significant)
        order_key = np.lexsort(tuple(cur[:, d] for d in range(cur.shape[1] - 1, -1, -1)))
        rank = np.empty_like(order_key)
        rank[order_key] = np.arange(order_key.size)
        # 1-D embedding: mean aq day index (centre of the aq time)
        tcent = (cur * np.arange(cur.shape[1])).sum(axis=1) / np.maximum(1, cur.sum(axis=1))
        print(y, "own fraction/32 %.3f" % mixed(cur, fb)[0], " own pattern %.3f" % mixed(cur, rank)[0],
              " own fraction/8+centre %.3f" % mixed(cur, np.minimum(8, (frac * 8).astype(np.int64)) * 1000
                                                   + tcent.astype(np.int64))[0])


if __name__ == "__main__":
    main()
