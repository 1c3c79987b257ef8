"""HIP path (libh9g.so, through the C-ABI) against the reference goldens and
the CPU oracle.  Bit-for-bit: the north-star tolerance is 1e-6 relative,
and the implementation is bit-exact, so every comparison here compares IEEE
bit patterns (conftest.same_bits: +0 and -0 differ; any NaN equals any NaN).
Runs on an MI355X only."""
import numpy as np
import pytest

import hybrid9_amd as h
from hybrid9_amd import shard, synth
from oracle import port, refcase
from tests.conftest import golden_names, load_golden, same_bits

pytestmark = pytest.mark.gpu

NTHREADS = 16   # oracle threads on the GPU box (its CPU share)


def _gpu_run(inp, L):
    n = inp["params"]["fmax"].size
    return h.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"],
                 nisurf=inp["nisurf"], year0=inp["year0"], nyears=inp["nyears"],
                 grow_on=bool(inp["grow_on"]), state0=inp["state0"])


@pytest.mark.parametrize("kernel", ["pair", "pair11", "pair1", "solo", "mixed"])
@pytest.mark.parametrize("name", golden_names(kind=("synth", "explicit", "spinup")))
def test_gpu_matches_reference_golden(name, kernel, monkeypatch):
    """The year kernels (two lanes per column = the default, with 22, 11 or
    1 column per wave -- the last is the cell order's kernel for short
    re-run lists; one lane), and two in one run (cells [0, 37) on the solo
    kernel, the rest on pair)."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    monkeypatch.setenv("H9G_SPLIT", "37")
    meta, inp, exp = load_golden(name)
    out = _gpu_run(inp, meta["L"])
    assert out["rc"] == 0, out["err"]
    assert same_bits(out["annual"], exp["annual"])
    assert same_bits(out["state"], exp["state"])


@pytest.mark.parametrize("kernel", ["pair", "pair11", "pair1", "solo"])
@pytest.mark.parametrize("name", golden_names(kind=("stop",)))
def test_gpu_reproduces_reference_stop(name, kernel, monkeypatch):
    monkeypatch.setenv("H9G_KERNEL", kernel)
    meta, inp, _ = load_golden(name)
    out = _gpu_run(inp, meta["L"])
    s = meta["stop"]
    assert out["rc"] == s["code"]
    e = out["err"]
    assert (e["cell"], e["day"], e["year"]) == (s["cell"], s["day"], meta["year0"])
    assert f"{e['value']:.9g}" == f"{s['value']:.9g}"


def test_config4_spinup_decades_carry_state():
    """Config 4 (30-year spin-up) restated on 24 cells: the reference's
    decade loop (HYBRID9.f90:93-130) carries every cell's state from one
    decade's forcing slab to the next.  Here each decade is its own context
    and the state crosses through h9g_get_state / h9g_set_state; the annual
    means of all 20 years and the state at the boundary and at the end are
    the reference's, bit for bit."""
    meta, inp, exp = load_golden("c4_spinup")
    dec = meta["decade"]
    nd1 = sum(h.days_in_year(meta["year0"] + k) for k in range(dec))
    common = dict(zi=inp["zi"], params=inp["params"], nisurf=inp["nisurf"], grow_on=bool(inp["grow_on"]))
    d1 = h.run(forcing=inp["forcing"][:, :nd1], year0=meta["year0"], nyears=dec, state0=inp["state0"], **common)
    assert d1["rc"] == 0, d1["err"]
    assert same_bits(d1["state"], exp["state_decade"])
    d2 = h.run(forcing=inp["forcing"][:, nd1:], year0=meta["year0"] + dec, nyears=meta["nyears"] - dec,
               state0=d1["state"], **common)
    assert d2["rc"] == 0, d2["err"]
    assert same_bits(np.concatenate([d1["annual"], d2["annual"]]), exp["annual"])
    assert same_bits(d2["state"], exp["state"])


@pytest.mark.parametrize("kernel", ["pair", "pair2", "pair11", "pair1", "solo", "mixed"])
def test_config5_l10_matches_reference_golden(kernel, monkeypatch):
    """Config 5 (0.25 deg, L = 10, NS = 24, GROW) against the reference
    rebuilt with nsoil_layers_max = 10: every annual mean (NaN for the cell
    that STOPs), the failed-cell set and its STOP record, and the end state
    of the other cells, bit for bit, over 2 years."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    monkeypatch.setenv("H9G_SPLIT", "17")
    meta, inp, exp = load_golden("c5_l10_sample")
    ok = exp["ok"]
    out = h.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"], nisurf=inp["nisurf"],
                year0=inp["year0"], nyears=inp["nyears"], grow_on=True, stop_on_error=False)
    assert same_bits(out["annual"], exp["annual"])
    e = out["errors"]
    assert np.array_equal(np.nonzero(e["code"])[0], [s["cell"] for s in meta["stops"]])
    for s in meta["stops"]:
        c = s["cell"]
        assert (e["code"][c], e["day"][c]) == (s["code"], s["day"])
        assert f"{e['value'][c]:.9g}" == f"{s['value']:.9g}"
    st = refcase.unpack_state(out["state"], meta["ncell"], meta["L"])
    st = {k: v[ok] for k, v in st.items()}
    assert same_bits(refcase.pack_state(st, meta["L"]), exp["state_ok"])


@pytest.mark.parametrize("kernel", ["pair", "solo"])
def test_gpu_reproduces_bench_stop(kernel, monkeypatch):
    """The config-2 bench's own STOP (land cell 20735 reaches the
    water-imbalance STOP on day 92 of 1910 in the driver's run): the product
    path over 1901-1910 stops that cell where the reference does, with the
    reference's record, and the three other cells match it bit for bit."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    meta, inp, exp = load_golden("c2_bench_stop")
    ok = exp["ok"]
    out = h.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"], nisurf=inp["nisurf"],
                year0=inp["year0"], nyears=inp["nyears"], grow_on=False, stop_on_error=False)
    (s,) = meta["stops"]
    c = s["cell"]
    e = out["errors"]
    assert np.array_equal(np.nonzero(e["code"])[0], [c])
    assert (e["code"][c], e["day"][c]) == (s["code"], s["day"])
    assert e["value"][c] == np.float32(s["value"])                 # printed by the reference to 8 digits
    assert out["err"]["year"] == meta["year0"] + meta["nyears"] - 1
    assert same_bits(out["annual"][:, :, ok], exp["annual"][:, :, ok])
    st = refcase.unpack_state(out["state"], meta["ncell"], meta["L"])
    st = {k: v[ok] for k, v in st.items()}
    assert same_bits(refcase.pack_state(st, meta["L"]), exp["state_ok"])


@pytest.mark.parametrize("kernel", ["pair", "pair11", "pair1", "solo"])
def test_gpu_nan_parameter_cells_match_oracle(kernel, monkeypatch):
    """Cells with missing soil data (NaN Fmax, a NaN layer parameter) run
    the year with NaN state, so every deferred special-case check of the
    substep flags and every redo path runs, in the same waves as normal
    cells.  A round-2 rewrite of one such path faulted the GPU only on such
    cells; this covers all of them against the oracle."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    meta, inp, _ = load_golden("c1_10x10")
    p = {k: v.copy() for k, v in inp["params"].items()}
    p["fmax"][::7] = np.nan
    p["psi_s"][3::11, 2] = np.nan
    p["hksat"][5::13, 0] = np.nan
    p["bsw"][8::17, 6] = np.nan
    gpu = h.run(zi=inp["zi"], params=p, forcing=inp["forcing"], nisurf=48, year0=1901, nyears=1,
                grow_on=True, stop_on_error=False)
    ref = port.run(zi=inp["zi"], params=p, forcing=inp["forcing"], nisurf=48, year0=1901, nyears=1,
                   grow_on=1, nthreads=NTHREADS)
    assert np.isnan(ref["annual"][0]).any(axis=0).sum() > 20
    assert np.array_equal(gpu["errors"]["code"], ref["errors"]["code"])
    assert same_bits(gpu["annual"], ref["annual"])
    assert same_bits(gpu["state"], refcase.pack_state(ref["state"], meta["L"]))


def test_reference_stop_raises():
    meta, inp, _ = load_golden("stop_ns24")
    n = meta["ncell"]
    with h.Context(n, inp["zi"], nisurf=inp["nisurf"]) as ctx:
        ctx.set_params(inp["params"])
        ctx.init_state()
        ctx.push_forcing(0, inp["forcing"])
        ctx.run_year(0, 1901)
        with pytest.raises(h.ReferenceStop, match="Water imbalance"):
            ctx.sync()


def _full_grid_gpu(gid, L, nisurf, grow_on, year0, nyears, seed=synth.SEED, nx=synth.NX05,
                   ny=synth.NY05, raise_on_stop=True):
    """Whole grid on the GPU with inputs generated on the device."""
    lat = synth.cell_lat(gid, nx, ny)
    zi = synth.ZI_L8 if L == 8 else synth.ZI_L10
    anns = []
    with h.Context(gid.size, zi, nlayers=L, nisurf=nisurf, grow_on=grow_on) as ctx:
        ctx.set_cells(gid, lat)
        ctx.synth_params(seed)
        ctx.init_state()
        for y in range(nyears):
            nt = synth.days_in_year(year0 + y)
            ctx.synth_forcing(y % 2, seed, synth.year_day0(year0 + y), nt)
            ctx.run_year(y % 2, year0 + y)
            ctx.sync(raise_on_stop=raise_on_stop)
            anns.append(ctx.get_annual())
        state = ctx.get_state()
        diag = ctx.get_diagnostics()
        if not raise_on_stop:
            return np.stack(anns), state, diag, ctx.get_errors()
    return np.stack(anns), state, diag


def _oracle_sample(gid, sample, L, nisurf, grow_on, year0, nyears, nx=synth.NX05, ny=synth.NY05):
    g = gid[sample]
    lat = synth.cell_lat(g, nx, ny)
    p = synth.make_params(g, L)
    nd = sum(synth.days_in_year(year0 + k) for k in range(nyears))
    f = synth.make_forcing(g, lat, synth.year_day0(year0), nd)
    zi = synth.ZI_L8 if L == 8 else synth.ZI_L10
    return port.run(zi=zi, params=p, forcing=f, nisurf=nisurf, year0=year0, nyears=nyears,
                    grow_on=grow_on, nthreads=NTHREADS)


def test_config2_full_grid_sampled_against_oracle():
    """0.5 deg global land (67,420 cells), 1 year, NS=48, hydrology only:
    every sampled cell bit-identical to the oracle; the global FP64
    diagnostics equal the host restatement over all cells."""
    gid = synth.land_cells()
    ann, st, diag = _full_grid_gpu(gid, 8, 48, False, 1901, 1)
    rng = np.random.default_rng(1)
    sample = np.sort(rng.choice(gid.size, 192, replace=False))
    ref = _oracle_sample(gid, sample, 8, 48, 0, 1901, 1)
    assert ref["rc"] == 0
    assert same_bits(ann[:, :, sample], ref["annual"])
    got = refcase.unpack_state(st, gid.size, 8)
    for k, v in ref["state"].items():
        assert same_bits(got[k][sample], v), k
    hd = shard.host_diagnostics(ann[0], got)
    assert diag[0] == gid.size and diag[11] == 0
    np.testing.assert_allclose(diag, hd, rtol=1e-12, atol=0)


def test_config4_full_grid_30_years_sampled_against_oracle():
    """Config 4 at its full size: the 0.5 deg grid (67,420 cells) spun up
    over 1901-1930 (NS=48, GROW on) with the state carried in the device
    context, 64 sampled cells bit-identical to the oracle after 30 years
    (every year's annual means and the end state; c4_spinup pins the oracle
    to the reference over 20 years with a decade carry)."""
    gid = synth.land_cells()
    ann, st, _ = _full_grid_gpu(gid, 8, 48, True, 1901, 30)
    rng = np.random.default_rng(4)
    sample = np.sort(rng.choice(gid.size, 64, replace=False))
    ref = _oracle_sample(gid, sample, 8, 48, 1, 1901, 30)
    assert ref["rc"] == 0
    assert same_bits(ann[:, :, sample], ref["annual"])
    got = refcase.unpack_state(st, gid.size, 8)
    for k, v in ref["state"].items():
        assert same_bits(got[k][sample], v), k


@pytest.mark.parametrize("kernel", ["pair", "pair2", "pair11", "solo", "mixed"])
def test_config5_l10_quarter_degree_sample(kernel, monkeypatch):
    """10 soil layers (config 5) on 0.25 deg cells, NS=24, GROW on, the
    year kernels (pair at 3 and at 2 waves per SIMD, solo) and the mixed
    launch (h9g.hip l10_kind picks by shard size), against the C restatement
    on 2,048 cells.  The
    restatement is itself pinned at L=10 to the reference's own L=10 build
    (oracle/_ref/h9ref_l10: SHARED.f90:294,300 set to 10/11) by the golden
    c5_l10_sample, which test_config5_l10_matches_reference_golden runs here."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    monkeypatch.setenv("H9G_SPLIT", "1001")
    land = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
    # a 2048-cell sample plus land cell 773, which reaches the reference's
    # water-imbalance STOP in 1901 (tests/golden/c5_l10_sample.npz)
    gid = np.sort(np.concatenate([land[::97][:2047], land[773:774]]))
    ann, st, _, errs = _full_grid_gpu(gid, 10, 24, True, 1901, 2, nx=synth.NX025, ny=synth.NY025,
                                      raise_on_stop=False)
    ref = _oracle_sample(gid, np.arange(gid.size), 10, 24, 1, 1901, 2, synth.NX025, synth.NY025)
    # every field, NaN for the failed cells, and the same failed-cell set,
    # STOP codes, days, substeps and values
    assert same_bits(ann, ref["annual"])
    re = ref["errors"]
    assert np.count_nonzero(re["code"]) >= 1
    for k in ("code", "day", "substep"):
        assert np.array_equal(errs[k], re[k]), k
    assert same_bits(errs["value"], re["value"])
    ok = re["code"] == 0
    got = refcase.unpack_state(st, gid.size, 10)
    for k, v in ref["state"].items():
        assert same_bits(got[k][ok], v[ok]), k


def test_shard_invariance_and_determinism():
    """Isolated-cell semantics: results are identical for any split of the
    cells into contexts (GPUs) and across repeated runs."""
    gid = synth.land_cells()[::31][:1500]
    ann_full, st_full, _ = _full_grid_gpu(gid, 8, 48, True, 1901, 2)
    ann_again, st_again, _ = _full_grid_gpu(gid, 8, 48, True, 1901, 2)
    assert same_bits(ann_full, ann_again) and same_bits(st_full, st_again)
    parts = []
    for r in range(3):
        sl = shard.shard_slice(gid.size, r, 3)
        a, _, _ = _full_grid_gpu(gid[sl], 8, 48, True, 1901, 2)
        parts.append(a)
    assert same_bits(np.concatenate(parts, axis=2), ann_full)


@pytest.mark.parametrize("L,nisurf,kernel", [(8, 48, "pair"), (10, 24, "pair2"), (8, 48, "pair11"),
                                             (10, 24, "pair11")])
def test_spare_lanes_in_ragged_waves(L, nisurf, kernel, monkeypatch):
    """The helper lanes of a pair-kernel wave (20 with 22 columns, 42 with
    11) evaluate the pairs' first layer slots and mirror a pair lane
    elsewhere (h9g.hip pair_body).  Waves with 1, 3, 9 and 22 + 1 columns
    (the mirror wraps; a second, one-column wave) give the same bits for
    every cell as the same cells inside a 1,500-cell run of full waves."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    gid = synth.land_cells()[::31][:1500]
    ann_all, st_all, _ = _full_grid_gpu(gid, L, nisurf, True, 1901, 2)
    for lo, n in ((0, 1), (5, 3), (101, 9), (700, 23)):
        ann, st, _ = _full_grid_gpu(gid[lo:lo + n], L, nisurf, True, 1901, 2)
        assert same_bits(ann, ann_all[:, :, lo:lo + n]), (lo, n)
        part, full = refcase.unpack_state(st, n, L), refcase.unpack_state(st_all, gid.size, L)
        for k in part:
            assert same_bits(part[k], full[k][lo:lo + n]), (lo, n, k)


def test_masked_waves_with_spare_lanes(monkeypatch):
    """Cells outside the soil mask (SUM(theta_s) <= trunc, HYBRID9.f90:
    122-123) leave the pair kernel at once; two whole waves of them (cells
    0..43 in the identity cell order, H9G_SORT=0) leave their spare lanes
    with no pair to serve, and those leave too.  The masked cells' annual
    means are NaN, and every other cell is the reference's golden, bit for
    bit."""
    monkeypatch.setenv("H9G_KERNEL", "pair")
    monkeypatch.setenv("H9G_SORT", "0")
    meta, inp, exp = load_golden("c1_10x10")
    p = {k: v.copy() for k, v in inp["params"].items()}
    p["theta_s"][:44] = 0.0
    out = h.run(zi=inp["zi"], params=p, forcing=inp["forcing"], nisurf=inp["nisurf"], year0=inp["year0"],
                nyears=inp["nyears"], grow_on=bool(inp["grow_on"]), state0=inp["state0"], stop_on_error=False)
    assert np.isnan(out["annual"][:, :, :44]).all()
    assert same_bits(out["annual"][:, :, 44:], exp["annual"][:, :, 44:])


@pytest.mark.parametrize("kernel", ["pair", "solo"])
def test_cell_order_invariance(kernel, monkeypatch):
    """The per-year cell order (h9g_sort_kernel: keyed from year 2 on by the
    fraction of the last year's substeps with the water table below the
    column) changes no bit: 8 years of 1,500 grid cells, sorted against the
    identity order (H9G_SORT=0), annual fields and state."""
    monkeypatch.setenv("H9G_KERNEL", kernel)
    gid = synth.land_cells()[::31][:1500]
    ann_s, st_s, _ = _full_grid_gpu(gid, 8, 48, False, 1901, 8)
    monkeypatch.setenv("H9G_SORT", "0")
    ann_i, st_i, _ = _full_grid_gpu(gid, 8, 48, False, 1901, 8)
    assert same_bits(ann_s, ann_i) and same_bits(st_s, st_i)


def test_async_prefetch_pipeline():
    """Double-buffered forcing (pinned host ring, copy stream) gives the
    same results as synchronous pushes over a multi-year run."""
    meta, inp, exp = load_golden("c1_2yr_leap")
    n = meta["ncell"]
    f = inp["forcing"]
    d0 = synth.days_in_year(1903)
    with h.Context(n, inp["zi"], nisurf=48) as ctx:
        ctx.set_params(inp["params"])
        ctx.init_state()
        ctx.push_forcing(0, f[:, :d0], async_=True)
        ctx.push_forcing(1, f[:, d0:], async_=True)
        ctx.run_year(0, 1903)
        ctx.run_year(1, 1904)
        ctx.sync()
        ann = ctx.get_annual()
        st = ctx.get_state()
    assert same_bits(ann, exp["annual"][1])
    assert same_bits(st, exp["state"])


@pytest.mark.parametrize("fmt", ["cdf2", "nc4"])
def test_netcdf_prefetch_pipeline(tmp_path, fmt):
    """READ_PGF path from NetCDF files: the async prefetch (host thread ->
    pinned staging -> copy stream, h9g_nc_forcing_prefetch) of two years of
    PGF-layout files gives the same results as pushing the same forcing
    directly, and the annual output written as axyYYYY.nc reads back equal.
    Both the classic CDF-2 layout and netCDF-4 (HDF5, chunked + deflate, as
    PGF v2.1 ships; READ_NET_CDF_3DR.f90:95-97)."""
    from scipy.io import netcdf_file
    from tests.helpers import write_nc4
    from tests.test_netcdf import write_pgf_like
    nx, ny, nland = 24, 12, 60
    gid, lat = synth.land_cells(nx, ny, nland), None
    lat = synth.cell_lat(gid, nx, ny)
    params = synth.make_params(gid, 8)
    nt = synth.days_in_year(1903) + synth.days_in_year(1904)
    f = synth.make_forcing(gid, lat, synth.year_day0(1903), nt)          # (7, nt, ncell)
    full = np.full((7, nt, ny * nx), np.float32(250.0))
    full[:, :, gid] = f
    if fmt == "nc4":
        paths = [write_nc4(tmp_path / f"{v}_pgfv2.1_1901-1910.nc4", v, full[k].reshape(nt, ny, nx))
                 for k, v in enumerate(h.PGF_VARS)]
        assert open(paths[0], "rb").read(4) == b"\x89HDF"
    else:
        paths = [write_pgf_like(tmp_path, v, full[k].reshape(nt, ny, nx), 2) for k, v in enumerate(h.PGF_VARS)]
    d0 = synth.days_in_year(1903)

    def run(prefetch):
        with h.Context(nland, synth.ZI_L8, nisurf=48) as ctx:
            ctx.set_cells(gid, lat)
            ctx.set_params(params)
            ctx.init_state()
            if prefetch:
                ctx.nc_prefetch(0, paths, nx, ny, 0, d0)
                ctx.nc_prefetch(1, paths, nx, ny, d0, nt - d0)
            else:
                ctx.push_forcing(0, f[:, :d0])
                ctx.push_forcing(1, f[:, d0:])
            ctx.run_year(0, 1903)
            ctx.run_year(1, 1904)
            ctx.sync()
            return ctx.get_annual(), ctx.get_state()

    a1, s1 = run(True)
    a0, s0 = run(False)
    assert same_bits(a1, a0) and same_bits(s1, s0)
    out = tmp_path / "axy1904.nc"
    zc = np.array([synth.ZI_L8[i] - (synth.ZI_L8[i] - synth.ZI_L8[i - 1]) / np.float32(2)
                   for i in range(1, 9)], np.float32)
    h.write_axy_nc(out, a1, gid, zc, nx, ny)
    with netcdf_file(out, "r", mmap=False) as nc:
        assert same_bits(nc.variables["runoff"][:].reshape(-1)[gid], a1[2])
        assert same_bits(nc.variables["soil_water_layers"][:].reshape(-1, 8)[gid], a1[11:19].T)
