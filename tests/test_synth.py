"""Synthetic inputs: numpy generator == the C++ generator in libh9g (host
build of hybrid9_amd/csrc/h9g_synth.h, also used on device)."""
import numpy as np

import hybrid9_amd as h
from hybrid9_amd import synth


def test_land_mask_size_and_order():
    g = synth.land_cells()
    assert g.size == synth.NLAND05 == 67_420
    assert np.all(np.diff(g) > 0)                     # raster order, unique
    assert g.min() >= 0 and g.max() < synth.NX05 * synth.NY05


def test_calendar_matches_init_f90():
    # INIT.f90:844-859: time_BOY(1)=1 (1860); 1901-01-01 = iTIME 14976
    t = synth.time_boy()
    assert t[0] == 1
    assert t[1901 - 1860] == 14976
    assert [synth.days_in_year(y) for y in (1900, 1901, 1904, 2000)] == [365, 365, 366, 366]
    assert synth.year_day0(1902) == 365


def test_numpy_equals_cpp_generator():
    g = synth.land_cells()[::613][:110].astype(np.int64)
    lat = synth.cell_lat(g)
    for L in (8, 10):
        p = synth.make_params(g, L)
        f = synth.make_forcing(g, lat, 1460, 40)
        n = g.size
        pp = np.zeros(4 * n * L + n, np.float32)
        ff = np.zeros((7, 40, n), np.float32)
        rc = h.lib().h9g_synth_host(synth.SEED, L, n, g.ctypes.data_as(h._I64P), h._fp(lat),
                                    1460, 40, h._fp(pp), h._fp(ff))
        assert rc == 0
        ref = np.concatenate([p[k].ravel() for k in ("theta_s", "hksat", "bsw", "psi_s")]
                             + [p["fmax"]])
        assert np.array_equal(pp, ref)
        assert np.array_equal(ff, f)


def test_forcing_ranges():
    g = synth.land_cells()[::97]
    f = synth.make_forcing(g, synth.cell_lat(g), 0, 365)
    lo = [240, 150, 0, 1e-4, 6e4, 0, 10]
    hi = [315, 450, 350, 0.0152, 1.04e5, 1e-3, 100]
    for v in range(7):
        assert f[v].min() >= lo[v] and f[v].max() <= hi[v], synth.FORCING_VARS[v]
    assert 0.3 < (f[5] == 0).mean() < 0.9            # dry days
