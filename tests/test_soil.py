"""Soil parameter build: INIT.f90:575-631 (60x60 block
average of the 30" BNU layers over pixels with theta_s >= 0, then unit
conversions) and :661-680 (Fmax of soiled cells, -9999 -> 3809).

The reference cannot run here (INIT.f90 needs netCDF-Fortran), so parity
is unpinned against the reference itself: the C restatement
(oracle/h9_oracle.c h9o_soil_layer/h9o_soil_fmax) is pinned to an
independent numpy loop written from INIT.f90 (same order of additions),
and the GPU kernels (hybrid9_amd/csrc/h9g.hip h9g_soil_kernel /
h9g_soil_seq_kernel) are checked bit for bit against the restatement.
Fixtures: synthetic 30" fields in the BNU storage units (scaled integers,
plus fractional fields for the sequential-order path) and missing pixels
(< 0)."""
import numpy as np
import pytest

import hybrid9_amd as h
from hybrid9_amd import synth
from oracle import port
from tests.conftest import same_bits

NX, NY = 12, 6


def fields30(rng, nx=NX, ny=NY, integer=True, missing=0.03):
    shape = (ny * 60, nx * 60)
    ts = rng.integers(300, 600, shape).astype(np.float32)        # 0.001 cm3/cm3
    ks = rng.integers(5, 4000, shape).astype(np.float32)         # cm/day
    lm = rng.integers(100, 500, shape).astype(np.float32)        # 0.001
    ps = -rng.integers(5, 80, shape).astype(np.float32)          # cm
    if not integer:
        ks = ks + rng.uniform(0, 1, shape).astype(np.float32)
        ps = ps - rng.uniform(0, 1, shape).astype(np.float32)
    ts[rng.uniform(0, 1, shape) < missing] = -1.0
    ts[:60, :60] = -9999.0                                       # an all-missing block (j = 0)
    return ts, ks, lm, ps


def numpy_layer(x, y, ts, ks, lm, ps):
    """INIT.f90:575-631 for one cell, loop by loop."""
    z = np.float32(0)
    s = [z, z, z, z]
    j = 0
    for x1 in range(x * 60, x * 60 + 60):
        for y1 in range(y * 60, y * 60 + 60):
            if ts[y1, x1] >= z:
                s = [s[0] + ts[y1, x1], s[1] + ks[y1, x1], s[2] + lm[y1, x1], s[3] + ps[y1, x1]]
                j += 1
    if j > 0:
        s = [v / np.float32(j) for v in s]
    lam = max(s[2] / np.float32(1.0e3), np.float32(1.0e-8))
    return (s[0] / np.float32(1.0e3), np.float32(10.0) * s[1] / np.float32(86400.0),
            np.float32(1.0) / lam, np.float32(10.0) * s[3])


def test_oracle_soil_layer_matches_numpy_loop():
    rng = np.random.default_rng(5)
    for integer in (True, False):
        f = fields30(rng, integer=integer)
        gid = np.array([0, 1, 13, 40, NX * NY - 1], np.int64)
        got = port.soil_layer(NX, NY, gid, *f)
        for k, g in enumerate(gid):
            exp = numpy_layer(int(g % NX), int(g // NX), *f)
            for v in range(4):
                assert got[v][k].tobytes() == np.float32(exp[v]).tobytes(), (g, v)
    # the all-missing block: sums stay zero, lambda -> trunc
    assert got[0][0] == 0 and got[2][0] == np.float32(1.0) / np.float32(1.0e-8)


def test_oracle_soil_fmax_rules():
    gid = np.arange(6, dtype=np.int64)
    tex = np.array([1, 0, 13, 5, 5, 5], np.int32)
    fm = np.array([1234, 1234, 1234, -9999, 0, 5000], np.int32)
    ts = np.full((6, 8), 0.05, np.float32)
    ts[4] = 0.0                                                  # SUM(theta_s) <= trunc
    out = port.soil_fmax(gid, tex, fm, ts)
    exp = [np.float32(1234) / np.float32(10000), np.nan, np.nan, np.float32(3809) / np.float32(10000),
           np.nan, np.float32(0.5)]
    np.testing.assert_array_equal(out, np.array(exp, np.float32))


def _oracle_params(gid, layers, soil_tex, fmax_in):
    L = len(layers)
    out = {k: np.empty((gid.size, L), np.float32) for k in ("theta_s", "hksat", "bsw", "psi_s")}
    for i, f in enumerate(layers):
        r = port.soil_layer(NX, NY, gid, *f)
        for k, v in zip(("theta_s", "hksat", "bsw", "psi_s"), r):
            out[k][:, i] = v
    out["fmax"] = port.soil_fmax(gid, soil_tex, fmax_in, out["theta_s"])
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("integer", [True, False])
def test_gpu_soil_build_matches_oracle(integer):
    """Both GPU paths (tree reduction on integer data, the reference's
    sequential order otherwise) bit for bit against the restatement, then a
    year of the hot path on the built parameters against the oracle."""
    rng = np.random.default_rng(11)
    L = 8
    gid = np.sort(rng.choice(NX * NY, 40, replace=False)).astype(np.int64)
    gid[0] = 0                                                   # includes the all-missing block
    layers = [fields30(rng, integer=integer) for _ in range(L)]
    soil_tex = rng.integers(0, 14, NX * NY).astype(np.int32)
    fmax_in = rng.integers(1000, 6000, NX * NY).astype(np.int32)
    fmax_in[::7] = -9999
    exp = _oracle_params(gid, layers, soil_tex, fmax_in)
    lat = synth.cell_lat(gid, NX, NY)
    with h.Context(gid.size, synth.ZI_L8, nisurf=48, grow_on=True) as ctx:
        ctx.set_cells(gid, lat)
        for i, f in enumerate(layers):
            ms, slow = ctx.soil_layer(i, *f, NX, NY)
            # fractional data: every block with a contributing pixel takes the
            # sequential path (cell 0 is the all-missing block)
            assert slow == (0 if integer else gid.size - 1)
        ctx.soil_fmax(soil_tex, fmax_in, NX, NY)
        got = ctx.get_params()
        for k in ("theta_s", "hksat", "bsw", "psi_s"):
            assert got[k].tobytes() == exp[k].tobytes(), k
        assert same_bits(got["fmax"], exp["fmax"])
        ctx.init_state()
        forcing = synth.make_forcing(gid, lat, 0, 365)
        ctx.push_forcing(0, forcing)
        ctx.run_year(0, 1901)
        rc = ctx.sync(raise_on_stop=False)
        ann = ctx.get_annual()
    ref = port.run(zi=synth.ZI_L8, params=exp, forcing=forcing, nisurf=48, year0=1901, nyears=1,
                   grow_on=1, nthreads=16)
    assert rc == ref["rc"]
    assert same_bits(ann, ref["annual"][0])     # cells without soil texture: NaN Fmax -> NaN fields
