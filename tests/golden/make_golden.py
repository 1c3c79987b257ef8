#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE itself.

Runs ``oracle/_ref/h9ref`` -- the unmodified reference HYDROLOGY.f90 /
GROW.f90 / SHARED.f90 / CONTROL.f90 compiled by ``make -C oracle ref`` --
on synthetic inputs and stores inputs (or their checksums) and outputs.
Needs /root/reference (build container only); the fixtures are data and
travel with the repo.

    python tests/golden/make_golden.py            # all cases

Each npz holds: meta (json string), annual (nyears, 12+L, ncell),
state (packed, refcase.state_fields), optionally trace (ntrace, nsteps, 3L+7)
and, for cases with hand-built inputs, params / forcing / state0.
Synthetic cases store the sha256 of their inputs instead; tests regenerate
them with hybrid9_amd.synth and check the digest first.
"""
from __future__ import annotations

import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from hybrid9_amd import synth  # noqa: E402
from oracle import refcase  # noqa: E402

OUT = Path(__file__).resolve().parent
TRACE_STEPS = 96          # keep the first two days of per-substep traces


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def synth_inputs(gid, year0, nyears, L=8, seed=synth.SEED):
    lat = synth.cell_lat(gid)
    p = synth.make_params(gid, L, seed)
    nd = sum(synth.days_in_year(year0 + k) for k in range(nyears))
    f = synth.make_forcing(gid, lat, synth.year_day0(year0), nd, seed)
    return p, f


def packed_params(p):
    return np.concatenate([p[k].ravel() for k in ("theta_s", "hksat", "bsw", "psi_s")]
                          + [p["fmax"].ravel()]).astype(np.float32)


def save(name, meta, out, extra=None):
    d = dict(meta=np.array(json.dumps(meta)), annual=out["annual"],
             state=refcase.pack_state(out["state"], meta["L"]))
    if "trace" in out:
        d["trace"] = out["trace"][:, :TRACE_STEPS, :]
    if extra:
        d.update(extra)
    np.savez_compressed(OUT / f"{name}.npz", **d)
    print(f"{name}: {meta['ncell']} cells x {meta['nyears']} yr, "
          f"{(OUT / f'{name}.npz').stat().st_size / 1e3:.0f} kB")


def synth_case(name, gid, *, year0=1901, nyears=1, nisurf=48, grow_on=1, trace=()):
    gid = np.asarray(gid, dtype=np.int64)
    p, f = synth_inputs(gid, year0, nyears)
    out = refcase.run_case(zi=synth.ZI_L8, params=p, forcing=f, nisurf=nisurf, year0=year0,
                           nyears=nyears, grow_on=grow_on, trace_cells=trace)
    meta = dict(name=name, kind="synth", seed=synth.SEED, gid=gid.tolist(), L=8,
                ncell=int(gid.size), year0=year0, nyears=nyears, nisurf=nisurf,
                grow_on=grow_on, zi=synth.ZI_L8.tolist(), trace_cells=list(trace),
                input_sha256=digest(packed_params(p), f),
                generator="oracle/_ref/h9ref (reference HYDROLOGY.f90/GROW.f90, amdflang -O2)")
    save(name, meta, out)


def independent_layer_params(gid, L=8, seed=synth.SEED):
    """The generator's first version: every layer drawn independently.  Such
    columns can have extreme layer contrasts that make the reference STOP on
    its water-balance check (kept only to build the STOP fixture)."""
    F32 = np.float32
    gid = np.asarray(gid, dtype=np.uint64)
    key = gid[:, None] * np.uint64(16) + np.arange(L, dtype=np.uint64)[None, :]
    u = lambda s, k: synth.u01(seed, s, k)  # noqa: E731
    ks = F32(0.5) + F32(487.5) * u(synth.S_KS, key)
    lam = np.maximum(F32(0.10) + F32(0.40) * u(synth.S_LAMBDA, key), F32(1e-8))
    return dict(theta_s=(F32(0.30) + F32(0.30) * u(synth.S_THETA_S, key)).astype(F32),
                hksat=((F32(10.0) * ks) / F32(86400.0)).astype(F32),
                bsw=(F32(1.0) / lam).astype(F32),
                psi_s=(F32(10.0) * (F32(-80.0) + F32(75.0) * u(synth.S_PSI, key))).astype(F32),
                fmax=(F32(0.1) + F32(0.5) * u(synth.S_FMAX, gid)).astype(F32))


def stop_case(name, gid, *, year0=1901, nisurf=24, grow_on=1):
    """Explicit inputs on which the reference executes a STOP: the fixture
    is the STOP site and the values the reference prints."""
    gid = np.asarray(gid, dtype=np.int64)
    p = independent_layer_params(gid)
    f = synth.make_forcing(gid, synth.cell_lat(gid), synth.year_day0(year0), 365)
    try:
        refcase.run_case(zi=synth.ZI_L8, params=p, forcing=f, nisurf=nisurf, year0=year0,
                         nyears=1, grow_on=grow_on)
    except refcase.RefStop as e:
        info = e.info
    else:
        raise SystemExit(f"{name}: expected a reference STOP")
    meta = dict(name=name, kind="stop", L=8, ncell=int(gid.size), year0=year0, nyears=1,
                nisurf=nisurf, grow_on=grow_on, zi=synth.ZI_L8.tolist(), stop=info,
                generator="oracle/_ref/h9ref STOP output")
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)),
                        params=packed_params(p), forcing=f)
    print(f"{name}: reference STOP {info}")


def edge_case():
    """Hand-built states and forcing that drive every branch of HYDROLOGY
    and GROW the synthetic climate rarely reaches (see meta['cells'])."""
    L = 8
    zi = synth.ZI_L8
    dz = np.diff(zi)[:L]
    base = synth.land_cells()[::4211][:16].astype(np.int64)
    p, f = synth_inputs(base, 1901, 1)
    n = base.size
    st = refcase.unpack_state(np.zeros(n * (4 * L + 9), np.float32), n, L)
    # INIT.f90:707-811 defaults, then per-cell overrides
    from oracle import port
    st = refcase.unpack_state(port.init_state(p, zi), n, L)
    ts = p["theta_s"]
    desc = []

    def setc(c, what, **kv):
        for k, v in kv.items():
            st[k][c] = v
        desc.append(f"{c}: {what}")

    setc(0, "water table at surface (jwt=0), wet column", zwt=0.02,
         h2osoi_liq=(0.95 * ts[0] * dz).astype(np.float32))
    setc(1, "water table in layer 3 (jwt=2)", zwt=0.12)
    setc(2, "water table in layer 8 (jwt=7)", zwt=1.5)
    setc(3, "water table exactly at zi(8)/1000", zwt=np.float32(2296.0) / np.float32(1000.0))
    setc(4, "saturated column", zwt=0.5, h2osoi_liq=(ts[4] * dz).astype(np.float32))
    setc(5, "very dry and hot, no rain (theta(1)<=0.15, watmin)",
         h2osoi_liq=(0.03 * ts[5] * dz).astype(np.float32))
    f[5, :, 5] = 0.0
    f[0, :, 5] += 12.0
    setc(6, "dense canopy LAI>4", LAI=5.0, plant_foliage_mass=5.0 / 23.0e-3)
    setc(7, "very negative smp (w_i<0.6 foliage loss)",
         smp=np.full(L, -1.2e5, np.float32))
    f[5, :, 8] *= 30.0
    desc.append("8: heavy rain x30 (infiltration excess, rising water table)")
    setc(9, "water table near the 80 m clamp", zwt=79.5)
    setc(10, "aquifer near its 5000 mm cap", wa=4995.0, zwt=2.5)
    f[5, :, 10] *= 10.0
    setc(11, "no canopy, no litter, no light (rsc/rac 1e6 branches)", LAI=0.0, LAI_litter=0.0,
         plant_foliage_mass=0.0)
    f[2, :, 11] = 0.0
    f[0, :, 12] = np.minimum(f[0, :, 12], 250.0) - 5.0
    desc.append("12: cold (fT clipping)")
    f[0, :, 13] = np.maximum(f[0, :, 13], 296.0) + 2.0
    desc.append("13: hot, tas-tf>18 fT branch")
    p["hksat"][14, :3] = 1.0e-5
    f[5, :, 14] *= 15.0
    desc.append("14: tight topsoil + heavy rain (qinmax limits infiltration)")
    setc(15, "bottom layers near watmin", h2osoi_liq=np.array(
        [5, 5, 5, 5, 3, 0.02, 0.011, 0.0105], np.float32) * np.float32(1.0))
    state0 = refcase.pack_state(st, L)
    out = refcase.run_case(zi=zi, params=p, forcing=f, nisurf=48, year0=1901, nyears=1,
                           grow_on=1, state0=st, trace_cells=(0, 8, 15))
    meta = dict(name="edge", kind="explicit", L=L, ncell=n, year0=1901, nyears=1, nisurf=48,
                grow_on=1, zi=zi.tolist(), trace_cells=[0, 8, 15], cells=desc,
                generator="oracle/_ref/h9ref (reference HYDROLOGY.f90/GROW.f90, amdflang -O2)")
    save("edge", meta, out, extra=dict(params=packed_params(p), forcing=f, state0=state0))


# Config 4 spin-up cells with hand-set initial states / parameters /
# rainfall (state field overrides, pr multiplier), applied to synthetic inputs
SPINUP_EDGES = [
    ("water table at the surface, wet column", dict(zwt=0.02, wet=0.95), 1.0),
    ("water table in layer 3", dict(zwt=0.12), 1.0),
    ("water table in layer 8", dict(zwt=1.5), 1.0),
    ("saturated column", dict(zwt=0.5, wet=1.0), 1.0),
    ("very dry, no rain", dict(wet=0.03), 0.0),
    ("heavy rain x20: rising water table", dict(), 20.0),
    ("aquifer near its 5000 mm cap, rain x10", dict(wa=4995.0, zwt=2.5), 10.0),
    ("tight topsoil, rain x15 (qinmax)", dict(tight=1), 15.0),
]


def spinup_inputs(gid_syn, gid_edge, year0, nyears, L=8, seed=synth.SEED):
    """Inputs of the config-4 spin-up golden: synthetic cells gid_syn from
    the initial state of INIT.f90:707-811, then the SPINUP_EDGES cells."""
    from oracle import port
    gid = np.concatenate([gid_syn, gid_edge]).astype(np.int64)
    p, f = synth_inputs(gid, year0, nyears, L, seed)
    n0 = gid_syn.size
    dz = np.diff(synth.ZI_L8)[:L]
    for k, (_, ov, prs) in enumerate(SPINUP_EDGES):
        if ov.get("tight"):
            p["hksat"][n0 + k, :3] = np.float32(1.0e-5)
        f[5, :, n0 + k] *= np.float32(prs)
    st = refcase.unpack_state(port.init_state(p, synth.ZI_L8), gid.size, L)
    for k, (_, ov, _) in enumerate(SPINUP_EDGES):
        c = n0 + k
        if "zwt" in ov:
            st["zwt"][c] = np.float32(ov["zwt"])
        if "wa" in ov:
            st["wa"][c] = np.float32(ov["wa"])
        if "wet" in ov:
            st["h2osoi_liq"][c] = (np.float32(ov["wet"]) * p["theta_s"][c] * dz).astype(np.float32)
    return gid, p, f, refcase.pack_state(st, L)


def spinup_case(name="c4_spinup", year0=1901, nyears=20, decade=10):
    """Config 4 (30-year spin-up) restated small: 24 cells, NS = 48, GROW on,
    run as two decades with the state carried across, as HYBRID9.f90:93-130
    carries it across its decade loop.  The reference is run over all years
    at once and decade by decade; both must agree bit for bit (the packed
    state is the whole per-cell state).  Stores the annual means of every
    year, the state at the decade boundary and at the end."""
    land = synth.land_cells()
    gsyn, gedge = land[::4211][:16], land[2000::8000][:len(SPINUP_EDGES)]
    gid, p, f, st0 = spinup_inputs(gsyn, gedge, year0, nyears)
    kw = dict(zi=synth.ZI_L8, params=p, nisurf=48, grow_on=1)
    whole = refcase.run_case(forcing=f, year0=year0, nyears=nyears, state0=refcase.unpack_state(st0, gid.size, 8),
                             **kw)
    nd1 = sum(synth.days_in_year(year0 + k) for k in range(decade))
    d1 = refcase.run_case(forcing=f[:, :nd1], year0=year0, nyears=decade,
                          state0=refcase.unpack_state(st0, gid.size, 8), **kw)
    d2 = refcase.run_case(forcing=f[:, nd1:], year0=year0 + decade, nyears=nyears - decade,
                          state0=d1["state"], **kw)
    assert np.array_equal(np.concatenate([d1["annual"], d2["annual"]]), whole["annual"], equal_nan=True)
    assert np.array_equal(refcase.pack_state(d2["state"], 8), refcase.pack_state(whole["state"], 8))
    meta = dict(name=name, kind="spinup", seed=synth.SEED, gid=gid.tolist(), n_synth=int(gsyn.size),
                edges=[e[0] for e in SPINUP_EDGES], L=8, ncell=int(gid.size), year0=year0, nyears=nyears,
                decade=decade, nisurf=48, grow_on=1, zi=synth.ZI_L8.tolist(),
                input_sha256=digest(packed_params(p), f, st0),
                generator="oracle/_ref/h9ref (reference HYDROLOGY.f90/GROW.f90, amdflang -O2), "
                          "whole run == decade-by-decade run")
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)), annual=whole["annual"],
                        state=refcase.pack_state(whole["state"], 8),
                        state_decade=refcase.pack_state(d1["state"], 8))
    print(f"{name}: {gid.size} cells x {nyears} yr, {(OUT / f'{name}.npz').stat().st_size / 1e3:.0f} kB")


def l10_inputs(gid, year0, nyears, seed=synth.SEED):
    """Config 5 synthetic inputs: 0.25 deg cells, 10 soil layers."""
    lat = synth.cell_lat(gid, synth.NX025, synth.NY025)
    p = synth.make_params(gid, 10, seed)
    nd = sum(synth.days_in_year(year0 + k) for k in range(nyears))
    return p, synth.make_forcing(gid, lat, synth.year_day0(year0), nd, seed)


def l10_case(name="c5_l10_sample", year0=1901, nyears=2, nisurf=24):
    """Config 5 (0.25 deg, L = 10, NS = 24, GROW on) pinned to the reference:
    oracle/_ref/h9ref_l10 is the unmodified HYDROLOGY.f90/GROW.f90 built
    with nsoil_layers_max = 10, Nlevgrnd = 11 (make -C oracle ref10).
    Cells: a sample of the 0.25 deg land grid plus land cell 773, whose
    soil column reaches the water-imbalance STOP (HYDROLOGY.f90:1244) in
    1901 (found by running the C oracle over all 270,000 cells).  The
    reference STOPs the whole program there, so the STOP cell runs alone:
    the fixture holds its STOP record and NaN means, the others' outputs."""
    land = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
    stop_idx = [773]
    sample = [i for i in range(977, land.size, 5413)][:48]
    idx = sample + stop_idx
    gid = land[idx].astype(np.int64)
    p, f = l10_inputs(gid, year0, nyears)
    ok = np.array([i not in stop_idx for i in idx])
    sub = lambda a: {k: v[ok] for k, v in a.items()}  # noqa: E731
    out = refcase.run_case(zi=synth.ZI_L10, params=sub(p), forcing=np.ascontiguousarray(f[:, :, ok]),
                           nisurf=nisurf, year0=year0, nyears=nyears, grow_on=1)
    n, L = gid.size, 10
    annual = np.full((nyears, 12 + L, n), np.nan, np.float32)
    annual[:, :, ok] = out["annual"]
    stops = []
    for c in np.where(~ok)[0]:
        one = {k: v[c:c + 1] for k, v in p.items()}
        try:
            refcase.run_case(zi=synth.ZI_L10, params=one, forcing=np.ascontiguousarray(f[:, :, c:c + 1]),
                             nisurf=nisurf, year0=year0, nyears=nyears, grow_on=1)
        except refcase.RefStop as e:
            stops.append(dict(cell=int(c), **{k: e.info[k] for k in ("code", "day", "value")}))
        else:
            raise SystemExit(f"{name}: cell {c} was expected to STOP")
    meta = dict(name=name, kind="l10", seed=synth.SEED, gid=gid.tolist(), L=L, ncell=int(n), year0=year0,
                nyears=nyears, nisurf=nisurf, grow_on=1, zi=synth.ZI_L10.tolist(), stops=stops,
                input_sha256=digest(packed_params(p), f),
                generator="oracle/_ref/h9ref_l10 (reference HYDROLOGY.f90/GROW.f90 with "
                          "nsoil_layers_max=10, Nlevgrnd=11; amdflang -O2)")
    st = refcase.pack_state(out["state"], L)
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)), annual=annual,
                        state_ok=st, ok=ok)
    print(f"{name}: {n} cells x {nyears} yr, STOPs {stops}, {(OUT / f'{name}.npz').stat().st_size / 1e3:.0f} kB")


def bench_stop_case(name="c2_bench_stop", year0=1901, nyears=10, nisurf=48):
    """The config-2 bench's own STOP.  Over the driver's years (1901-1925,
    seed SEED, GROW off) one of the 67,420 synthetic land cells reaches the
    water-imbalance STOP (HYDROLOGY.f90:1244) in 1910: land index 20735,
    gid 53140, found on the GPU by tools/find_stops.py
    (profiles/stops_config2_r02.json).  The reference runs that cell alone
    from 1901 and must STOP at the same place; three other cells of the
    same grid run alongside it in a second reference run and must not."""
    land = synth.land_cells()
    stop_idx, other = 20735, [20734, 20736, 41000]
    idx = other + [stop_idx]
    gid = land[idx].astype(np.int64)
    p, f = synth_inputs(gid, year0, nyears)
    n = gid.size
    ok = np.arange(n) < len(other)
    sub = lambda a: {k: v[ok] for k, v in a.items()}  # noqa: E731
    out = refcase.run_case(zi=synth.ZI_L8, params=sub(p), forcing=np.ascontiguousarray(f[:, :, ok]),
                           nisurf=nisurf, year0=year0, nyears=nyears, grow_on=0)
    annual = np.full((nyears, 20, n), np.nan, np.float32)
    annual[:, :, ok] = out["annual"]
    one = {k: v[n - 1:] for k, v in p.items()}
    try:
        refcase.run_case(zi=synth.ZI_L8, params=one, forcing=np.ascontiguousarray(f[:, :, n - 1:]),
                         nisurf=nisurf, year0=year0, nyears=nyears, grow_on=0)
    except refcase.RefStop as e:
        stops = [dict(e.info, cell=n - 1)]
    else:
        raise SystemExit(f"{name}: land cell {stop_idx} was expected to STOP")
    meta = dict(name=name, kind="bench_stop", seed=synth.SEED, gid=gid.tolist(), L=8, ncell=int(n),
                year0=year0, nyears=nyears, nisurf=nisurf, grow_on=0, zi=synth.ZI_L8.tolist(), stops=stops,
                input_sha256=digest(packed_params(p), f),
                generator="oracle/_ref/h9ref (reference HYDROLOGY.f90/GROW.f90, amdflang -O2)")
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)), annual=annual,
                        state_ok=refcase.pack_state(out["state"], 8), ok=ok)
    print(f"{name}: {n} cells x {nyears} yr, STOPs {stops}")


def rel_bound(a, b):
    """max |a - b| / |b| over finite b != 0, and the cells where a and b
    differ in any bit (NaN == NaN)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    ok = np.isfinite(b) & (b != 0)
    r = np.abs(a[ok] - b[ok]) / np.abs(b[ok])
    return float(r.max()) if r.size else 0.0


def cell_order_case(name, gid, *, year0=1901, nyears=30, nisurf=48, grow_on=1, split=None, L=8):
    """The reference as it really runs: h9ref's cell_order
    mode, decade -> cell -> year with smp carried from cell to cell
    (HYBRID9.f90:93-130, HYDROLOGY.f90:270-275, SHARED.f90:198), cells in
    the reference's (y, x) order.  Also records, as data, how far the
    isolated-cell contract (every cell its own smp) sits from it, and
    (split) how far the reference itself moves when its cells are cut into
    two ranks (two chains, INIT.f90:271-274)."""
    gid = np.asarray(gid, dtype=np.int64)
    p, f = synth_inputs(gid, year0, nyears) if L == 8 else l10_inputs(gid, year0, nyears)
    zi = synth.ZI_L8 if L == 8 else synth.ZI_L10
    kw = dict(zi=zi, params=p, forcing=f, nisurf=nisurf, year0=year0, nyears=nyears,
              grow_on=grow_on)
    co = refcase.run_case(cell_order=True, **kw)
    iso = refcase.run_case(**kw)
    ai, ac = iso["annual"], co["annual"]
    fields = refcase.annual_fields(L)
    pick = [fields.index(k) for k in ["rnf", "theta_total"] + [f"theta{i + 1}" for i in range(L)]]
    diff_cells = np.any(np.any(ai.view(np.uint32) != ac.view(np.uint32), axis=0), axis=0)
    first_year = [int(year0 + np.argmax(np.any(ai[:, :, c].view(np.uint32) != ac[:, :, c].view(np.uint32), axis=1)))
                  for c in np.where(diff_cells)[0]]
    iso_bound = dict(
        annual=rel_bound(ai[:, pick, :], ac[:, pick, :]),
        **{k: rel_bound(iso["state"][k], co["state"][k]) for k in ("h2osoi_liq", "zwt", "wa")},
        cells_differing=int(diff_cells.sum()),
        first_decade_bitwise=bool(np.array_equal(ai[:min(nyears, 10)].view(np.uint32),
                                                 ac[:min(nyears, 10)].view(np.uint32))),
        first_year_hist={str(y): first_year.count(y) for y in sorted(set(first_year))})
    split_bound = None
    if split:
        half = gid.size // 2
        parts = []
        for sl in (slice(0, half), slice(half, gid.size)):
            parts.append(refcase.run_case(cell_order=True, zi=zi,
                                          params={k: v[sl] for k, v in p.items()},
                                          forcing=np.ascontiguousarray(f[:, :, sl]), nisurf=nisurf, year0=year0,
                                          nyears=nyears, grow_on=grow_on)["annual"])
        a2 = np.concatenate(parts, axis=2)
        split_bound = dict(annual=rel_bound(a2[:, pick, :], ac[:, pick, :]),
                           cells_differing=int(np.any(np.any(a2.view(np.uint32) != ac.view(np.uint32), axis=0),
                                                      axis=0).sum()))
    meta = dict(name=name, kind="cell_order", seed=synth.SEED, gid=gid.tolist(), L=L, ncell=int(gid.size),
                year0=year0, nyears=nyears, nisurf=nisurf, grow_on=grow_on, zi=zi.tolist(),
                grid="05" if L == 8 else "025",
                input_sha256=digest(packed_params(p), f), isolated_vs_cell_order=iso_bound,
                two_ranks_vs_one=split_bound,
                generator=f"oracle/_ref/{refcase.ref_bin(L).name} cell_order=1 (reference HYDROLOGY.f90/GROW.f90"
                          f"{'' if L == 8 else ' with nsoil_layers_max=10, Nlevgrnd=11'}, amdflang -O2; "
                          "decade -> cell -> year, smp carried between cells)")
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)), annual=ac,
                        state=refcase.pack_state(co["state"], L))
    print(f"{name}: {gid.size} cells x {nyears} yr, isolated vs cell order {iso_bound}, two ranks {split_bound}, "
          f"{(OUT / f'{name}.npz').stat().st_size / 1e3:.0f} kB")


def cell_order_blocks_case(name, gid, nx, ny, num_procs, *, year0=1901, nyears=20, nisurf=48, grow_on=1):
    """The reference on num_procs MPI ranks: the cells gid (row-major ids of
    an nx x ny grid, ascending) cut into the reference's blocks
    (shard.reference_blocks, INIT.f90:271-274,427-444), every block run by
    its own h9ref process in cell order -- ranks never communicate, so each
    is one independent chain (HYBRID9.f90:120-295)."""
    from hybrid9_amd.shard import reference_blocks
    gid = np.asarray(gid, dtype=np.int64)
    p, f = synth_inputs(gid, year0, nyears)
    L = 8
    loc = (gid // synth.NX05 - gid[0] // synth.NX05) * nx + (gid % synth.NX05 - gid[0] % synth.NX05)
    rank = reference_blocks(loc, nx, ny, num_procs)
    assert (rank >= 0).all() and np.all(np.diff(loc) > 0)
    ann = np.full((nyears, 12 + L, gid.size), np.nan, np.float32)
    st = {}
    for r in sorted(set(rank.tolist())):
        sel = np.where(rank == r)[0]
        out = refcase.run_case(cell_order=True, zi=synth.ZI_L8, params={k: v[sel] for k, v in p.items()},
                               forcing=np.ascontiguousarray(f[:, :, sel]), nisurf=nisurf, year0=year0,
                               nyears=nyears, grow_on=grow_on)
        ann[:, :, sel] = out["annual"]
        for k, v in out["state"].items():
            st.setdefault(k, np.zeros((gid.size,) + v.shape[1:], v.dtype))[sel] = v
    one = refcase.run_case(cell_order=True, zi=synth.ZI_L8, params=p, forcing=f, nisurf=nisurf, year0=year0,
                           nyears=nyears, grow_on=grow_on)["annual"]
    fields = refcase.annual_fields(L)
    pick = [fields.index(k) for k in ["rnf", "theta_total"] + [f"theta{i + 1}" for i in range(L)]]
    vs_one = dict(annual=rel_bound(ann[:, pick, :], one[:, pick, :]),
                  cells_differing=int(np.any(np.any(ann.view(np.uint32) != one.view(np.uint32), axis=0),
                                             axis=0).sum()))
    meta = dict(name=name, kind="cell_order", seed=synth.SEED, gid=gid.tolist(), L=L, ncell=int(gid.size),
                year0=year0, nyears=nyears, nisurf=nisurf, grow_on=grow_on, zi=synth.ZI_L8.tolist(),
                input_sha256=digest(packed_params(p), f), grid=[nx, ny], num_procs=num_procs,
                rank=rank.tolist(), blocks_vs_one_rank=vs_one,
                generator="oracle/_ref/h9ref cell_order=1, one process per reference block "
                          "(reference HYDROLOGY.f90/GROW.f90, amdflang -O2)")
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)), annual=ann,
                        state=refcase.pack_state(st, L))
    print(f"{name}: {gid.size} cells in {len(set(rank.tolist()))} blocks x {nyears} yr, vs one rank {vs_one}")


def cell_order_stop_case(name="co_stop", year0=1901, nisurf=24, grow_on=1):
    """A reference STOP inside the reference's own cell order: stop_ns24's
    hand-built soils run by h9ref's cell_order mode (smp carried from cell to
    cell).  The fixture is the STOP the reference prints (site, cell, day,
    value); the inputs are stop_ns24's, regenerated here."""
    land = synth.land_cells()
    gid = np.asarray(land[263::527][90:98], dtype=np.int64)
    p = independent_layer_params(gid)
    f = synth.make_forcing(gid, synth.cell_lat(gid), synth.year_day0(year0), 365)
    try:
        refcase.run_case(cell_order=True, zi=synth.ZI_L8, params=p, forcing=f, nisurf=nisurf, year0=year0,
                         nyears=1, grow_on=grow_on)
    except refcase.RefStop as e:
        info = e.info
    else:
        raise SystemExit(f"{name}: expected a reference STOP")
    meta = dict(name=name, kind="cell_order_stop", L=8, ncell=int(gid.size), year0=year0, nyears=1,
                nisurf=nisurf, grow_on=grow_on, zi=synth.ZI_L8.tolist(), stop=info, gid=gid.tolist(),
                input_sha256=digest(packed_params(p), f),
                generator="oracle/_ref/h9ref cell_order=1 STOP output")
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)),
                        params=packed_params(p), forcing=f)
    print(f"{name}: reference STOP in cell order {info}")


def main_cell_order_configs():
    """The ordered mode on the configurations the bench quotes it on
    (VERDICT r05 #2): config 2 (0.5 deg, GROW off, NS=48) on a row band over
    1901-1930, so the bench's timed decades are covered, and config 5
    (0.25 deg, L = 10, NS = 24, GROW on) on a row band over 1901-1920."""
    land = synth.land_cells()
    rows = land // synth.NX05
    cell_order_case("co_c2_band", land[(rows >= 130) & (rows < 138)], nyears=30, grow_on=0)
    l4 = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
    r4 = l4 // synth.NX025
    cell_order_case("co_c5_band", l4[(r4 >= 300) & (r4 < 304)], nyears=20, nisurf=24, grow_on=1, L=10)


def main_cell_order():
    g10 = np.array([(80 + j) * synth.NX05 + 400 + i for j in range(10) for i in range(10)])
    # config 1's grid over three decades (1901-1930)
    cell_order_case("co_c1_30yr", g10, nyears=30, split=True)
    # a contiguous 0.5 deg row band (rows 150-157: 2,022 land cells) over two decades
    land = synth.land_cells()
    rows = land // synth.NX05
    cell_order_case("co_band", land[(rows >= 150) & (rows < 158)], nyears=20)
    # config 1's grid as the reference runs it on 4 MPI ranks (2 x 2 blocks of 5 x 5)
    cell_order_blocks_case("co_c1_blocks4", g10, 10, 10, 4)
    cell_order_stop_case()
    main_cell_order_configs()


def site_inputs(gid, L, nisurf, years, events, seed=synth.SEED, soils="synth", ppt_scale=1.0):
    """Synthetic LCLIM site inputs (hybrid9_amd.site): soils of the land
    cells gid (soils="independent": independent_layer_params), site forcing
    (precipitation x ppt_scale), the day-of-year LAI schedule."""
    from hybrid9_amd import site
    p = synth.make_params(gid, L, seed) if soils == "synth" else independent_layer_params(gid, L, seed)
    nd = sum(synth.days_in_year(y) for y in years)
    sub, daily = site.synth_site(gid.size, nd, nisurf, seed, doy0=0)
    sub[:, 4, :] *= np.float32(ppt_scale)
    lai = site.broadcast(site.lai_schedule(years, events), gid.size)
    return p, sub, daily, lai


def lclim_case(name, gid, *, L=8, nisurf=48, years=(2002, 2003), events=None, stop=False,
               soils="synth", ppt_scale=1.0):
    """LCLIM single-site path (HYBRID9.f90:339-480) through the harness's
    lclim_mode; events=None is the reference's Vaira LAI schedule.  stop:
    the reference is expected to STOP; the fixture is what it prints."""
    gid = np.asarray(gid, dtype=np.int64)
    zi = synth.ZI_L8 if L == 8 else synth.ZI_L10
    p, sub, daily, lai = site_inputs(gid, L, nisurf, years, events, soils=soils, ppt_scale=ppt_scale)
    ev = None if events is None else {str(k): v for k, v in events.items()}
    try:
        out = refcase.run_site_case(zi=zi, params=p, sub=sub, daily=daily, lai=lai, nisurf=nisurf,
                                    year0=years[0], nyears=len(years))
        info = None
    except refcase.RefStop as e:
        if not stop:
            raise
        info = e.info
    if stop:
        if info is None:
            raise SystemExit(f"{name}: expected a reference STOP")
        out = dict(daily=np.zeros(0, np.float32), state=None)
    meta = dict(name=name, kind="lclim_stop" if stop else "lclim", stop=info, seed=synth.SEED,
                gid=gid.tolist(), L=L,
                ncell=int(gid.size), year0=years[0], nyears=len(years), nisurf=nisurf, grow_on=0,
                zi=zi.tolist(), events=ev, soils=soils, ppt_scale=ppt_scale, input_sha256=digest(packed_params(p), sub, daily, lai),
                generator="oracle/_ref/h9ref lclim_mode (reference HYDROLOGY.f90, amdflang -O2)")
    st = np.zeros(0, np.float32) if stop else refcase.pack_state(out["state"], L)
    np.savez_compressed(OUT / f"{name}.npz", meta=np.array(json.dumps(meta)), daily=out["daily"],
                        state=st)
    print(f"{name}: {gid.size} sites x {len(years)} yr, {(OUT / f'{name}.npz').stat().st_size / 1e3:.0f} kB")


# LAI schedule with litter moves on several days (lclim_ns24)
LCLIM_EVENTS_2004 = {2004: [(10, 0.5, None), (60, 1.9, None), (100, 2.8, (0.2, 0.05)),
                            (150, 1.1, (2.8, 1.1)), (200, 0.001, (1.1, 0.001)),
                            (250, None, (0.0, 0.5)), (300, 0.4, None), (366, 0.7, (0.3, 0.3))]}


def main_lclim():
    land = synth.land_cells()
    # the reference's Vaira configuration: 2002-2003, half-hourly, its LAI schedule
    lclim_case("lclim_vaira", land[1000::9000][:6])
    # NS=24, a leap year, another schedule (the reference's CONTROL.f90
    # fixes nsoil_layers_max = 8: L=10 is checked against the C oracle)
    g5 = land[4321::7000][:5]
    lclim_case("lclim_ns24", g5, nisurf=24, years=(2004,), events=LCLIM_EVENTS_2004)
    # a water-imbalance STOP (HYDROLOGY.f90:1244): hand-built soils, 10x rain
    lclim_case("lclim_stop", land[263::527][90:98], nisurf=24, years=(2004,),
               events=LCLIM_EVENTS_2004, stop=True, soils="independent", ppt_scale=10.0)


def main():
    if not refcase.REF_BIN.exists():
        sys.exit("build the reference harness first: make -C oracle ref")
    g10 = np.array([(80 + j) * synth.NX05 + 400 + i for j in range(10) for i in range(10)])
    land = synth.land_cells()
    # config 1: 10x10 synthetic land grid, one year daily, NS=48, GROW on
    synth_case("c1_10x10", g10, trace=(0, 37, 99))
    # config 1 over a leap-year boundary, two years (1903-1904)
    synth_case("c1_2yr_leap", g10[::6], year0=1903, nyears=2)
    # config 2 sample: 0.5 deg global land cells, hydrology only
    synth_case("c2_sample", land[::527][:128], grow_on=0, trace=(5,))
    # config 3 sample: NS=24, GROW on
    synth_case("c3_sample", land[263::527][:128], nisurf=24)
    # a reference STOP (water imbalance > 0.1 mm at NS=24) on hand-built soils
    stop_case("stop_ns24", land[263::527][90:98], nisurf=24)
    edge_case()
    main_lclim()
    spinup_case()
    l10_case()
    bench_stop_case()
    main_cell_order()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        globals()[sys.argv[1]]()
    else:
        main()
