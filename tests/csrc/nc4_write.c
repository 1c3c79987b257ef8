/* TEST HELPER: writes a netCDF-4 file the way libnetcdf lays one out in
 * HDF5 -- coordinate variables time(time), lat(lat), lon(lon) made HDF5
 * dimension scales, and one chunked, deflated float field
 * <name>(time, lat, lon) with those scales attached -- so the HDF5 read
 * path of h9g_io.cpp is tested on the on-disk form of a PGF v2.1 file
 * (READ_NET_CDF_3DR.f90:95-97 reads it with nf90_get_var).
 *   nc4_write <path> <name> <nt> <ny> <nx> <raw float32 file (nt*ny*nx)>
 *             [ct cy cx [filters [skip]]]
 * Optional: the chunk shape (default 1, ny, nx: one chunk per day) and the
 * filters, letters of "s" shuffle, "d" deflate 4, "f" fletcher32, "b" a
 * big-endian field (default "sd"), so every layout the reader's direct
 * chunk path and its H5Dread fallback take can be written; skip: a day
 * whose time chunks are never written (left unallocated, so they read as
 * the fill value, netCDF's NC_FILL_FLOAT, as libnetcdf sets it).
 * Built by tests/test_netcdf.py: gcc ... -lhdf5_hl -lhdf5 (/opt/conda). */
#include <hdf5.h>
#include <hdf5_hl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static hid_t coord(hid_t f, const char *name, hsize_t n, const float *v) {
  hid_t sp = H5Screate_simple(1, &n, NULL);
  hid_t d = H5Dcreate2(f, name, H5T_IEEE_F32LE, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
  H5Dwrite(d, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, v);
  H5DSset_scale(d, name);
  H5Sclose(sp);
  return d;
}

int main(int argc, char **argv) {
  if (argc != 7 && argc != 10 && argc != 11 && argc != 12) return 2;
  const hsize_t nt = atoi(argv[3]), ny = atoi(argv[4]), nx = atoi(argv[5]);
  float *data = malloc(sizeof(float) * nt * ny * nx);
  FILE *in = fopen(argv[6], "rb");
  if (!in || fread(data, sizeof(float), nt * ny * nx, in) != nt * ny * nx) return 3;
  fclose(in);
  hid_t fapl = H5Pcreate(H5P_FILE_ACCESS);
  H5Pset_libver_bounds(fapl, H5F_LIBVER_EARLIEST, H5F_LIBVER_LATEST);
  hid_t fcpl = H5Pcreate(H5P_FILE_CREATE);
  H5Pset_link_creation_order(fcpl, H5P_CRT_ORDER_TRACKED | H5P_CRT_ORDER_INDEXED);
  hid_t f = H5Fcreate(argv[1], H5F_ACC_TRUNC, fcpl, fapl);
  float *tv = malloc(sizeof(float) * nt), *yv = malloc(sizeof(float) * ny), *xv = malloc(sizeof(float) * nx);
  for (hsize_t i = 0; i < nt; i++) tv[i] = (float)i;
  for (hsize_t i = 0; i < ny; i++) yv[i] = 90.0f - (i + 0.5f) * 180.0f / ny;
  for (hsize_t i = 0; i < nx; i++) xv[i] = -180.0f + (i + 0.5f) * 360.0f / nx;
  hid_t dt = coord(f, "time", nt, tv), dy = coord(f, "lat", ny, yv), dx = coord(f, "lon", nx, xv);
  hsize_t dims[3] = {nt, ny, nx}, chunk[3] = {1, ny, nx};
  const char *filt = argc >= 11 ? argv[10] : "sd";
  const long skip = argc == 12 ? atol(argv[11]) : -1;
  if (argc >= 10) {
    chunk[0] = atoi(argv[7]);
    chunk[1] = atoi(argv[8]);
    chunk[2] = atoi(argv[9]);
  }
  hid_t sp = H5Screate_simple(3, dims, NULL);
  hid_t dcpl = H5Pcreate(H5P_DATASET_CREATE);
  H5Pset_chunk(dcpl, 3, chunk);
  for (const char *c = filt; *c; c++) {
    if (*c == 's') H5Pset_shuffle(dcpl);
    if (*c == 'd') H5Pset_deflate(dcpl, 4);
    if (*c == 'f') H5Pset_fletcher32(dcpl);
  }
  const float fill = 9.9692099683868690e+36f;
  H5Pset_fill_value(dcpl, H5T_NATIVE_FLOAT, &fill);
  const hid_t ftype = strchr(filt, 'b') ? H5T_IEEE_F32BE : H5T_IEEE_F32LE;
  hid_t dv = H5Dcreate2(f, argv[2], ftype, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT);
  if (skip < 0) {
    H5Dwrite(dv, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, data);
  } else {                         // day by day, none of the skipped day's time chunk
    const hsize_t one[3] = {1, ny, nx};
    hid_t ms = H5Screate_simple(3, one, NULL);
    for (hsize_t t = 0; t < nt; t++) {
      if (t / chunk[0] == (hsize_t)skip / chunk[0]) continue;
      const hsize_t start[3] = {t, 0, 0};
      H5Sselect_hyperslab(sp, H5S_SELECT_SET, start, NULL, one, NULL);
      H5Dwrite(dv, H5T_NATIVE_FLOAT, ms, sp, H5P_DEFAULT, data + t * ny * nx);
    }
    H5Sclose(ms);
  }
  H5DSattach_scale(dv, dt, 0);
  H5DSattach_scale(dv, dy, 1);
  H5DSattach_scale(dv, dx, 2);
  H5Dclose(dv);
  H5Dclose(dt);
  H5Dclose(dy);
  H5Dclose(dx);
  H5Sclose(sp);
  H5Pclose(dcpl);
  H5Fclose(f);
  return 0;
}
