"""LCLIM single-site path (HYBRID9.f90:339-480).

Goldens come from the reference's own HYDROLOGY.f90 driven through the
harness's lclim_mode (tests/golden/make_golden.py lclim_case).  CPU tests
pin the C restatement (oracle h9o_site) and the kernel body built for the
host against them.  GPU tests run h9g_run_site through the C-ABI.  Every
comparison is bit-exact.  The reference fixes nsoil_layers_max = 8
(CONTROL.f90), so L = 10 is checked against the pinned C restatement.
"""
import ctypes as C

import numpy as np
import pytest

from hybrid9_amd import site, synth
from oracle import port, refcase
from tests.conftest import load_site_golden, same_bits

NAMES = ("lclim_vaira", "lclim_ns24")


def _events_l10():
    from tests.golden.make_golden import LCLIM_EVENTS_2004
    return LCLIM_EVENTS_2004


def _l10_inputs(nisurf=24, nsite=6):
    from tests.golden.make_golden import site_inputs
    gid = synth.land_cells()[777::9000][:nsite]
    p, sub, daily, lai = site_inputs(gid, 10, nisurf, (2004,), _events_l10())
    return dict(zi=synth.ZI_L10, params=p, sub=sub, daily=daily, lai=lai, nisurf=nisurf)


# ---------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", NAMES)
def test_oracle_site_matches_reference_golden(name):
    meta, inp, exp = load_site_golden(name)
    out = port.site(**inp, nthreads=4)
    assert out["rc"] == 0
    assert same_bits(out["daily"], exp["daily"])
    assert same_bits(refcase.pack_state(out["state"], meta["L"]), exp["state"])


def test_oracle_site_reproduces_reference_stop():
    meta, inp, _ = load_site_golden("lclim_stop")
    out = port.site(**inp)
    s = meta["stop"]
    assert (out["rc"], out["err"]["cell"], out["err"]["day"]) == (s["code"], s["cell"], s["day"])
    assert f"{out['err']['value']:.8g}" == f"{s['value']:.8g}"


def _host_site(inp, const_geo):
    from tests.test_kernel_host import lib
    lb = lib()
    fp = C.POINTER(C.c_float)
    lb.h9k_host_site.argtypes = [C.c_int] * 5 + [fp] * 7 + [C.POINTER(C.c_int)]
    p = inp["params"]
    L, n = p["theta_s"].shape[1], p["fmax"].size
    zi = np.ascontiguousarray(inp["zi"], np.float32)
    pp = port.pack_params(p)
    st = port.init_state(p, zi)
    nday = inp["daily"].shape[0]
    out = np.full((nday, 11, n), np.nan, np.float32)
    err = np.zeros(4 * n, np.int32)
    a = [np.ascontiguousarray(inp[k], np.float32) for k in ("sub", "daily", "lai")]
    rc = lb.h9k_host_site(n, L, inp["nisurf"], nday, const_geo, zi.ctypes.data_as(fp),
                          pp.ctypes.data_as(fp), *[x.ctypes.data_as(fp) for x in a],
                          st.ctypes.data_as(fp), out.ctypes.data_as(fp),
                          err.ctypes.data_as(C.POINTER(C.c_int)))
    return rc, out, st


@pytest.mark.parametrize("const_geo", [1, 0])
@pytest.mark.parametrize("name", NAMES)
def test_kernel_body_site_matches_reference_golden(name, const_geo):
    meta, inp, exp = load_site_golden(name)
    rc, out, st = _host_site(inp, const_geo)
    assert rc == 0
    assert same_bits(out, exp["daily"])
    assert same_bits(st, exp["state"])


def test_kernel_body_site_l10_matches_oracle():
    inp = _l10_inputs()
    ref = port.site(**inp, nthreads=4)
    assert ref["rc"] == 0
    for cg in (1, 0):
        rc, out, st = _host_site(inp, cg)
        assert rc == 0
        assert same_bits(out, ref["daily"])
        assert same_bits(st, refcase.pack_state(ref["state"], 10))


def test_vaira_lai_schedule():
    """HYBRID9.f90:380-417 as data: LAI set on the listed days, litter moved
    by (a - b) on the days that also drop LAI."""
    s = site.lai_schedule([2002, 2003])
    assert s.shape == (730, 3)
    lai_days = np.flatnonzero(~np.isnan(s[:, 0]))
    assert lai_days.tolist() == [0, 58, 78, 93, 107, 121, 135, 356,
                                 365 + 28, 365 + 51, 365 + 75, 365 + 94, 365 + 105, 365 + 119,
                                 365 + 140, 365 + 157]
    assert np.isclose(s[121, 0], 1.43) and tuple(s[121, 1:]) == (np.float32(2.55), np.float32(1.43))
    assert np.isnan(s[0, 1]) and np.isnan(s[365 + 28, 1])
    litter_days = np.flatnonzero(~np.isnan(s[:, 1]))
    assert litter_days.tolist() == [121, 135, 365 + 105, 365 + 119, 365 + 140, 365 + 157]


def test_read_lclim_csv_columns(tmp_path):
    """The CSV reader takes LCLIM_array (5,6) and LCLIM_array2 (22,25,14,16,35)
    after one header line, as the list-directed READs of :352-435."""
    ns, years = 4, [2001]
    nd = 365
    rng = np.random.default_rng(3)
    dvals = rng.normal(size=(nd, 6)).astype(np.float32)
    with open(tmp_path / "daily.csv", "w") as f:
        f.write("DOY,evap,pr,tas,rhs,huss,ps,extra\n")
        for d in range(nd):
            f.write(f"{d + 1}," + ",".join(repr(float(v)) for v in dvals[d]) + ",99\n")
    svals = rng.normal(size=(nd * ns, 37)).astype(np.float32)
    with open(tmp_path / "sub2001.csv", "w") as f:
        f.write(",".join(f"c{i}" for i in range(37)) + "\n")
        for r in svals:
            f.write(" , ".join(repr(float(v)) for v in r) + "\n")
    sub, daily = site.read_lclim(tmp_path / "daily.csv", [tmp_path / "sub2001.csv"], years, ns)
    assert np.array_equal(daily, dvals[:, [4, 5]])
    assert np.array_equal(sub, svals[:, [21, 24, 13, 15, 34]])


def test_daily_csv_format(tmp_path):
    diag = np.arange(365 * 11, dtype=np.float32).reshape(365, 11, 1) / 7
    site.write_daily_csv(tmp_path / "d.csv", diag, [1999])
    lines = (tmp_path / "d.csv").read_text().splitlines()
    assert len(lines) == 365
    f = lines[3].split(",")
    assert len(f) == 13 and f[0] == " 1999" and f[1] == "    4"
    assert all(len(x) == 10 for x in f[2:])              # F10.4
    assert float(f[2]) == pytest.approx(diag[3, 0, 0], abs=1e-4)


def test_synthetic_site_forcing_is_plausible():
    sub, daily = site.synth_site(4, 365, 48)
    tak, rh, rnet, par, ppt = (sub[:, k, :] for k in range(5))
    assert -10 < tak.min() and tak.max() < 40
    assert rh.min() >= 5 and rh.max() <= 100
    assert (par >= 0).all() and (ppt >= 0).all()
    annual_mm = ppt.sum(0)
    assert ((annual_mm > 200) & (annual_mm < 1500)).all()
    assert (daily[:, 1, :] > 9.9e4).all()


# ---------------------------------------------------------------- GPU
def _gpu_site(inp, state0=None, nloop=1):
    import hybrid9_amd as h
    p = inp["params"]
    L, n = p["theta_s"].shape[1], p["fmax"].size
    with h.Context(n, inp["zi"], nlayers=L, nisurf=inp["nisurf"], grow_on=False) as ctx:
        ctx.set_params(p)
        if state0 is None:
            ctx.init_state()
        else:
            ctx.set_state(state0)
        diag = site.run_lclim(ctx, inp["sub"], inp["daily"], inp["lai"], nloop=nloop)
        return diag, ctx.get_state()


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_site_matches_reference_golden(name):
    meta, inp, exp = load_site_golden(name)
    diag, st = _gpu_site(inp)
    assert same_bits(diag, exp["daily"])
    assert same_bits(st, exp["state"])


@pytest.mark.gpu
def test_gpu_site_reproduces_reference_stop():
    import hybrid9_amd as h
    meta, inp, _ = load_site_golden("lclim_stop")
    with pytest.raises(h.ReferenceStop) as ei:
        _gpu_site(inp)
    e, s = ei.value.err, meta["stop"]
    assert (e["code"], e["cell"], e["day"]) == (s["code"], s["cell"], s["day"])
    assert f"{e['value']:.8g}" == f"{s['value']:.8g}"


@pytest.mark.gpu
def test_gpu_site_l10_and_spinup_match_oracle():
    """10 layers (runtime geometry at NS=24) and two spin-up passes
    (:341, the state carried over) against the C restatement."""
    inp = _l10_inputs()
    ref1 = port.site(**inp, nthreads=8)
    ref2 = port.site(**inp, state0=ref1["state"], nthreads=8)
    diag, st = _gpu_site(inp, nloop=2)
    nd = inp["daily"].shape[0]
    assert same_bits(diag[:nd], ref1["daily"])
    assert same_bits(diag[nd:], ref2["daily"])
    assert same_bits(st, refcase.pack_state(ref2["state"], 10))
