"""NetCDF I/O of the hot path (hybrid9_amd/csrc/h9g_io.cpp, SURVEY.md §8f
rows 1-2), host-only entry points of libh9g.so checked against scipy's
independent netCDF-classic implementation:

* h9g_write_axy_nc restates WRITE_NET_CDF_3DR.f90:93-263 (dimensions,
  coordinate variables INIT.f90:142-145/262, variable names, units, NaN
  _FillValue, (z,lon,lat) soil layers);
* h9g_nc_forcing_read restates READ_PGF.f90 + READ_NET_CDF_3DR.f90 (variable
  4 of each of the 7 files, dims (time, lat, lon), 'time' = NTIMES), for
  record ('time' unlimited) and fixed layouts, CDF-1 and CDF-2.
The reference ships no netCDF files, so the fixtures are written here with
scipy in the reference's layout."""
from pathlib import Path

import numpy as np
import pytest
from scipy.io import netcdf_file

import hybrid9_amd as h
from hybrid9_amd import synth

NX, NY = 16, 8


def _annual(L, n, rng):
    a = rng.uniform(0.1, 300.0, (12 + L, n)).astype(np.float32)
    a[:, 1] = np.nan                       # a non-soil land cell (INIT.f90:402-414)
    return a


@pytest.mark.parametrize("L", [8, 10])
def test_axy_writer_matches_reference_schema(tmp_path, L):
    rng = np.random.default_rng(3)
    gid = np.sort(rng.choice(NX * NY, 23, replace=False)).astype(np.int64)
    ann = _annual(L, gid.size, rng)
    zi = synth.ZI_L8 if L == 8 else synth.ZI_L10
    zc = np.array([zi[i] - (zi[i] - zi[i - 1]) / np.float32(2) for i in range(1, L + 1)], np.float32)
    p = tmp_path / "axy1901.nc"
    h.write_axy_nc(p, ann, gid, zc, NX, NY)
    with netcdf_file(p, "r", mmap=False) as f:
        assert f.dimensions == {"latitude": NY, "longitude": NX, "layer_centre_depth": L}
        names = ["latitude", "longitude", "layer_centre_depth", "net primary production", "plant mass",
                 "runoff", "evaporation", "temperature", "specific_humidity", "air_pressure",
                 "precipitation", "relative_humidity", "soil_water", "soil_water_layers"]
        assert list(f.variables) == names
        units = {"latitude": b"degrees_north", "longitude": b"degrees_east", "layer_centre_depth": b"mm",
                 "net primary production": b"g[DM]/m^2/yr", "plant mass": b"g[DM]", "runoff": b"mm/s",
                 "evaporation": b"mm/s", "temperature": b"K", "specific_humidity": b"kg[water]/kg[air]",
                 "air_pressure": b"Pa", "precipitation": b"kg/m^2/s", "relative_humidity": b"percent",
                 "soil_water": b"mm", "soil_water_layers": b"mm^3/mm^3"}
        for k, u in units.items():
            assert f.variables[k].units == u, k
            assert f.variables[k].typecode() == "f"
        for k in names[3:]:
            assert np.isnan(f.variables[k]._FillValue)
        dlat, dlon = np.float32(180.0 / NY), np.float32(360.0 / NX)
        np.testing.assert_array_equal(f.variables["latitude"][:],
                                      (np.float32(90) - dlat / 2) - np.arange(NY, dtype=np.float32) * dlat)
        np.testing.assert_array_equal(f.variables["longitude"][:],
                                      (np.float32(-180) + dlon / 2) + np.arange(NX, dtype=np.float32) * dlon)
        np.testing.assert_array_equal(f.variables["layer_centre_depth"][:], zc)
        rows = {"net primary production": 0, "plant mass": 1, "runoff": 2, "evaporation": 3,
                "temperature": 4, "specific_humidity": 7, "air_pressure": 8, "precipitation": 9,
                "relative_humidity": 10, "soil_water": 11 + L}
        land = np.zeros(NX * NY, bool)
        land[gid] = True
        for k, r in rows.items():
            v = f.variables[k][:].reshape(-1)
            assert v.shape == (NX * NY,)
            np.testing.assert_array_equal(v[gid], ann[r])          # NaN == NaN here
            assert np.isnan(v[~land]).all()
        layers = f.variables["soil_water_layers"][:]
        assert layers.shape == (NY, NX, L)
        np.testing.assert_array_equal(layers.reshape(NX * NY, L)[gid], ann[11:11 + L].T)
        assert np.isnan(layers.reshape(NX * NY, L)[~land]).all()


def test_axy_writer_half_degree_coordinates(tmp_path):
    """INIT.f90:142,145: lon_all(x) = -179.75 + (x-1)*0.5, lat_all(y) = 89.75 - (y-1)*0.5."""
    p = tmp_path / "axy.nc"
    h.write_axy_nc(p, np.zeros((20, 1), np.float32), np.array([0]), np.arange(8, dtype=np.float32), 720, 360)
    with netcdf_file(p, "r", mmap=False) as f:
        lat, lon = f.variables["latitude"][:], f.variables["longitude"][:]
        assert lat[0] == np.float32(89.75) and lat[-1] == np.float32(-89.75)
        assert lon[0] == np.float32(-179.75) and lon[-1] == np.float32(179.75)
        np.testing.assert_array_equal(lon, np.float32(-179.75) + np.arange(720, dtype=np.float32) * np.float32(0.5))


def write_pgf_like(d, var, data, version, record=True):
    """A PGF-layout file: variables lon, lat, time, <var>(time, lat, lon)."""
    nt, ny, nx = data.shape
    with netcdf_file(d / f"{var}.nc", "w", version=version) as f:
        if record:                       # scipy: the unlimited dimension comes first
            f.createDimension("time", None)
        f.createDimension("lon", nx)
        f.createDimension("lat", ny)
        if not record:
            f.createDimension("time", nt)
        f.createVariable("lon", "f", ("lon",))[:] = np.arange(nx, dtype=np.float32)
        f.createVariable("lat", "f", ("lat",))[:] = np.arange(ny, dtype=np.float32)
        t = f.createVariable("time", "d", ("time",))
        t[:] = np.arange(nt, dtype=np.float64)
        t.units = "days since 1860-01-01 00:00:00"
        v = f.createVariable(var, "f", ("time", "lat", "lon"))
        v[:] = data
        v.units = "K"
    return d / f"{var}.nc"


@pytest.mark.parametrize("version,record", [(1, True), (2, True), (2, False)])
def test_forcing_reader_matches_scipy(tmp_path, version, record):
    rng = np.random.default_rng(version)
    nt = 40
    data = [rng.uniform(0, 1, (nt, NY, NX)).astype(np.float32) for _ in range(7)]
    paths = [write_pgf_like(tmp_path, v, data[k], version, record) for k, v in enumerate(h.PGF_VARS)]
    assert h.nc_ntimes(paths[0]) == nt
    gid = rng.choice(NX * NY, 37, replace=False).astype(np.int64)
    got = h.nc_forcing_read(paths, NX, NY, gid, 5, 30)
    for k in range(7):
        np.testing.assert_array_equal(got[k], data[k].reshape(nt, -1)[5:35][:, gid])


def test_forcing_reader_rejects_bad_inputs(tmp_path):
    data = np.zeros((4, NY, NX), np.float32)
    paths = [write_pgf_like(tmp_path, v, data, 2) for v in h.PGF_VARS]
    gid = np.arange(3, dtype=np.int64)
    with pytest.raises(h.H9GError):
        h.nc_forcing_read(paths, NX, NY, gid, 2, 5)          # past NTIMES
    with pytest.raises(h.H9GError):
        h.nc_forcing_read(paths, NX + 1, NY, gid, 0, 2)      # wrong grid
    with pytest.raises(h.H9GError):
        h.nc_forcing_read(paths[:6] + [tmp_path / "missing.nc"], NX, NY, gid, 0, 2)


@pytest.mark.skipif(not Path("/opt/conda/include/hdf5.h").exists(), reason="no HDF5 in this image")
def test_forcing_reader_netcdf4_equals_cdf2(tmp_path):
    """PGF v2.1 ships netCDF-4 (HDF5) files; READ_NET_CDF_3DR.f90:95-97 reads
    days of <var>(time, lat, lon).  The same data written as netCDF-4 (HDF5
    dimension-scale layout, chunked + deflate, tests/csrc/nc4_write.c) and
    as CDF-2 read back identically, gathered at the same cells."""
    from tests.helpers import write_nc4
    rng = np.random.default_rng(4)
    nt = 33
    data = [rng.uniform(200, 300, (nt, NY, NX)).astype(np.float32) for _ in range(7)]
    d4, d2 = tmp_path / "nc4", tmp_path / "cdf2"
    d4.mkdir()
    d2.mkdir()
    p4 = [write_nc4(d4 / f"{v}_pgfv2.1_1901-1910.nc4", v, data[k]) for k, v in enumerate(h.PGF_VARS)]
    p2 = [write_pgf_like(d2, v, data[k], 2) for k, v in enumerate(h.PGF_VARS)]
    assert open(p4[0], "rb").read(4) == b"\x89HDF"
    assert h.nc_ntimes(p4[0]) == nt
    gid = rng.choice(NX * NY, 41, replace=False).astype(np.int64)
    got4 = h.nc_forcing_read(p4, NX, NY, gid, 3, 25)
    got2 = h.nc_forcing_read(p2, NX, NY, gid, 3, 25)
    assert np.array_equal(got4, got2)
    for k in range(7):
        np.testing.assert_array_equal(got4[k], data[k].reshape(nt, -1)[3:28][:, gid])
    with pytest.raises(h.H9GError):
        h.nc_forcing_read(p4, NX, NY, gid, 20, 20)            # past NTIMES
    with pytest.raises(h.H9GError):
        h.nc_forcing_read(p4, NX, NY + 2, gid, 0, 2)          # wrong grid


@pytest.mark.skipif(not Path("/opt/conda/include/hdf5.h").exists(), reason="no HDF5 in this image")
@pytest.mark.parametrize("chunk,filters", [
    ((1, NY, NX), "sd"),       # PGF v2.1: a chunk per day, shuffle + deflate (direct chunk path)
    ((4, 5, 7), "sd"),         # chunks spanning days, partial chunks at every edge
    ((3, NY, NX), "d"),        # deflate only
    ((2, 4, NX), ""),          # no filter
    ((5, 3, 4), "sdb"),        # a big-endian field
    ((2, NY, 8), "sdf"),       # fletcher32: not decoded directly, H5Dread fallback
])
def test_forcing_reader_netcdf4_chunk_layouts(tmp_path, chunk, filters, monkeypatch):
    """h9g_nc_forcing_read's netCDF-4 path (round 4): the chunk table is read
    once through HDF5, then the chunks holding the cells are read with pread
    and inflated/unshuffled on a host thread pool outside HDF5; layouts it
    does not decode go through H5Dread.  Every layout returns the written
    values at the cells, for one thread and for several, and for a day range
    that starts and ends inside multi-day chunks."""
    from tests.helpers import write_nc4
    rng = np.random.default_rng(11)
    nt = 17
    data = [rng.uniform(200, 300, (nt, NY, NX)).astype(np.float32) for _ in range(7)]
    paths = [write_nc4(tmp_path / f"{v}_pgfv2.1_1901-1910.nc4", v, data[k], chunk, filters)
             for k, v in enumerate(h.PGF_VARS)]
    gid = np.sort(rng.choice(NX * NY, 29, replace=False)).astype(np.int64)[::-1].copy()   # any order
    exp = np.stack([data[k].reshape(nt, -1)[2:15][:, gid] for k in range(7)])
    for threads in ("1", "5"):
        monkeypatch.setenv("H9G_IO_THREADS", threads)
        got = h.nc_forcing_read(paths, NX, NY, gid, 2, 13)
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), threads
    # cells of one latitude row only (a rank's band: READ_NET_CDF_3DR.f90:95-97)
    row = np.arange(3 * NX + 2, 3 * NX + 9, dtype=np.int64)
    got = h.nc_forcing_read(paths, NX, NY, row, 0, nt)
    assert np.array_equal(got, np.stack([data[k].reshape(nt, -1)[:, row] for k in range(7)]))


@pytest.mark.skipif(not Path("/opt/conda/include/hdf5.h").exists(), reason="no HDF5 in this image")
@pytest.mark.parametrize("chunk", [(1, NY, NX), (4, 5, 7)])
def test_forcing_reader_netcdf4_unwritten_chunk(tmp_path, chunk, monkeypatch):
    """A time chunk that was never written has no entry in the chunk table
    (ADVICE r04): the reader must return the fill value there, as H5Dread /
    nf90_get_var do, not what the output buffer held before.  The file of
    one variable misses the chunks of day 6; the days read span it."""
    from tests.helpers import NC_FILL_FLOAT, write_nc4
    rng = np.random.default_rng(12)
    nt = 17
    data = [rng.uniform(200, 300, (nt, NY, NX)).astype(np.float32) for _ in range(7)]
    paths = [write_nc4(tmp_path / f"{v}_pgfv2.1_1901-1910.nc4", v, data[k], chunk, "sd", skip=6 if k == 3 else None)
             for k, v in enumerate(h.PGF_VARS)]
    gid = np.sort(rng.choice(NX * NY, 29, replace=False)).astype(np.int64)
    exp = np.stack([data[k].reshape(nt, -1)[2:15][:, gid] for k in range(7)])
    ct = chunk[0]
    for t in range(2, 15):
        if t // ct == 6 // ct:
            exp[3, t - 2] = NC_FILL_FLOAT
    for threads in ("1", "5"):
        monkeypatch.setenv("H9G_IO_THREADS", threads)
        got = h.nc_forcing_read(paths, NX, NY, gid, 2, 13)
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), threads


@pytest.mark.skipif(not Path("/opt/conda/include/hdf5.h").exists(), reason="no HDF5 in this image")
def test_synthetic_pgf_files_round_trip(tmp_path):
    """tools/pgf_synth.py (the files bench.py --forcing nc4 reads each step)
    holds the bench's own synthetic forcing at the land cells: read back
    through h9g_nc_forcing_read it is bit-equal to synth.make_forcing."""
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
    import pgf_synth
    from hybrid9_amd import synth
    nx, ny, nland = 24, 12, 90
    paths = pgf_synth.write_year(tmp_path, 1903, 40, nx=nx, ny=ny, nland=nland)
    assert [Path(p).name for p in paths] == [f"{v}_pgfv2.1_1901-1910.nc4" for v in h.PGF_VARS]
    g = synth.land_cells(nx, ny, nland)
    got = h.nc_forcing_read(paths, nx, ny, g, 0, 40)
    exp = synth.make_forcing(g, synth.cell_lat(g, nx, ny), synth.year_day0(1903), 40)
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))
