// h9g_io.cpp -- NetCDF I/O of the hot path's inputs and outputs (host C++,
// part of libh9g.so), SURVEY.md §8f rows 1-2:
//
//   * forcing ingest, /root/reference/SOURCE/READ_PGF.f90:22-109 and
//     READ_NET_CDF_3DR.f90:43-98: one file per PGF variable (tas rlds rsds
//     huss ps pr rhs), the variable's 4th netCDF variable (varid = 4,
//     READ_PGF.f90:30) with dims (time, lat, lon) -- Fortran (lon,lat,time)
//     -- and NTIMES from the 'time' dimension (READ_NET_CDF_3DR.f90:48-52).
//     h9g_nc_forcing_read gathers the land cells of a context for a range
//     of days; h9g_nc_forcing_prefetch does it on a host thread into pinned
//     memory and queues the copy into a forcing slot (async PGF prefetch).
//   * annual output, WRITE_NET_CDF_3DR.f90:93-263: axyYYYY.nc with the same
//     dimensions (latitude, longitude, layer_centre_depth), coordinate
//     variables, variable names, units and NaN _FillValue.
//
// Formats.  Input: netCDF-4 (HDF5) files -- what PGF v2.1 ships and what
// READ_NET_CDF_3DR.f90 opens -- read through the HDF5 C library (1.10, in
// /opt/conda/lib of this image; loaded with dlopen on first use, so
// libh9g.so has no link-time dependency on it), and netCDF "classic"
// (CDF-1) and 64-bit-offset (CDF-2) files, read directly (a big-endian
// header followed by the variables' data; record variables interleaved per
// record).  There is no libnetcdf in the image.  Output: CDF-2 with the
// reference's schema (the reference writes netCDF-4, NF90_NETCDF4 at
// WRITE_NET_CDF_3DR.f90:93), readable by every netCDF tool and by
// scipy.io.netcdf_file.
#include <dlfcn.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <mutex>
#include <type_traits>
#include <string>
#include <sched.h>
#include <thread>
#include <vector>

#include "../../include/h9g.h"
#include "h9g_io.h"

namespace {

enum { NC_BYTE = 1, NC_CHAR = 2, NC_SHORT = 3, NC_INT = 4, NC_FLOAT = 5, NC_DOUBLE = 6 };
enum { TAG_DIM = 0x0A, TAG_VAR = 0x0B, TAG_ATT = 0x0C };

int type_size(int t) {
  switch (t) {
    case NC_BYTE: case NC_CHAR: return 1;
    case NC_SHORT: return 2;
    case NC_INT: case NC_FLOAT: return 4;
    case NC_DOUBLE: return 8;
  }
  return 0;
}
size_t pad4(size_t n) { return (n + 3) & ~(size_t)3; }

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

// Stage times of the last forcing read (h9g_nc_read_stats): thread-seconds
// summed over the pool, so that a stage's share of the pool is its sum over
// (wall x threads).
std::mutex g_stats_lock;
double g_stats[H9G_IO_NSTATS];

// ------------------------------------------------------------------ reader
struct NcVar {
  std::string name;
  std::vector<int> dims;
  int type = 0;
  uint64_t vsize = 0, begin = 0;
  bool record = false;
};

struct NcReader {
  FILE *f = nullptr;
  int version = 0;
  uint64_t numrecs = 0, recsize = 0;
  std::vector<std::string> dim_names;
  std::vector<uint64_t> dim_len;
  int rec_dim = -1;
  std::vector<NcVar> vars;
  std::vector<unsigned char> hdr;
  size_t pos = 0;
  bool ok = true;

  ~NcReader() {
    if (f) fclose(f);
  }
  uint32_t u32() {
    if (pos + 4 > hdr.size()) { ok = false; return 0; }
    const unsigned char *p = &hdr[pos];
    pos += 4;
    return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3];
  }
  uint64_t u64() {
    const uint64_t hi = u32();
    return hi << 32 | u32();
  }
  std::string name() {
    const uint32_t n = u32();
    if (!ok || pos + n > hdr.size()) { ok = false; return ""; }
    std::string s((const char *)&hdr[pos], n);
    pos += pad4(n);
    return s;
  }
  void skip_atts() {
    const uint32_t tag = u32(), n = u32();
    if (tag == 0 && n == 0) return;
    if (tag != TAG_ATT) { ok = false; return; }
    for (uint32_t a = 0; a < n && ok; a++) {
      name();
      const int t = (int)u32();
      const uint32_t nel = u32();
      pos += pad4((size_t)nel * type_size(t));
    }
  }
  bool open(const char *path) {
    f = fopen(path, "rb");
    if (!f) return false;
    hdr.resize(1 << 16);
    size_t got = fread(hdr.data(), 1, hdr.size(), f);
    // grow until the header parses (headers are small; PGF: < 4 KiB)
    for (;;) {
      hdr.resize(got);
      pos = 0;
      ok = true;
      if (parse()) return true;
      if (got < (size_t)1 << 16 || hdr.size() > ((size_t)1 << 26)) return false;
      const size_t want = hdr.size() * 4;
      hdr.resize(want);
      fseek(f, 0, SEEK_SET);
      got = fread(hdr.data(), 1, want, f);
    }
  }
  bool parse() {
    if (hdr.size() < 8 || memcmp(hdr.data(), "CDF", 3) != 0) return false;
    version = hdr[3];
    if (version != 1 && version != 2) return false;
    pos = 4;
    numrecs = u32();
    uint32_t tag = u32(), n = u32();
    dim_names.clear();
    dim_len.clear();
    rec_dim = -1;
    if (tag == TAG_DIM) {
      for (uint32_t d = 0; d < n && ok; d++) {
        dim_names.push_back(name());
        dim_len.push_back(u32());
        if (dim_len.back() == 0) rec_dim = (int)d;
      }
    } else if (tag != 0 || n != 0) {
      return false;
    }
    skip_atts();                                  // global attributes
    tag = u32();
    n = u32();
    vars.clear();
    if (tag == TAG_VAR) {
      for (uint32_t v = 0; v < n && ok; v++) {
        NcVar var;
        var.name = name();
        const uint32_t nd = u32();
        for (uint32_t k = 0; k < nd && ok; k++) var.dims.push_back((int)u32());
        skip_atts();
        var.type = (int)u32();
        var.vsize = u32();
        var.begin = version == 2 ? u64() : u32();
        var.record = !var.dims.empty() && var.dims[0] == rec_dim;
        vars.push_back(var);
      }
    } else if (tag != 0 || n != 0) {
      return false;
    }
    if (!ok) return false;
    recsize = 0;
    int nrecvars = 0;
    for (auto &v : vars)
      if (v.record) { recsize += v.vsize; nrecvars++; }
    if (nrecvars == 1) {                          // a single record variable is not padded
      for (auto &v : vars)
        if (v.record) {
          uint64_t sz = type_size(v.type);
          for (size_t k = 1; k < v.dims.size(); k++) sz *= dim_len[v.dims[k]];
          recsize = sz;
        }
    }
    return true;
  }
  uint64_t dim_of(const NcVar &v, size_t k) const {
    const int d = v.dims[k];
    return d == rec_dim ? numrecs : dim_len[d];
  }
  // float data of v at first-dimension index t (all remaining dims)
  bool read_slice(const NcVar &v, uint64_t t, float *out) {
    if (v.type != NC_FLOAT || v.dims.empty()) return false;
    uint64_t n = 1;
    for (size_t k = 1; k < v.dims.size(); k++) n *= dim_of(v, k);
    const uint64_t off = v.record ? v.begin + t * recsize : v.begin + t * n * 4;
    if (fseeko(f, (off_t)off, SEEK_SET) != 0) return false;
    if (fread(out, 4, n, f) != n) return false;
    uint32_t *u = (uint32_t *)out;
    for (uint64_t i = 0; i < n; i++) u[i] = __builtin_bswap32(u[i]);
    return true;
  }
  const NcVar *find(const char *nm) const {
    for (auto &v : vars)
      if (v.name == nm) return &v;
    return nullptr;
  }
  int dim_index(const char *nm) const {
    for (size_t d = 0; d < dim_names.size(); d++)
      if (dim_names[d] == nm) return (int)d;
    return -1;
  }
};

// ------------------------------------------------------- netCDF-4 (HDF5)
// A netCDF-4 file is an HDF5 file whose variables are datasets in the root
// group and whose dimensions are HDF5 dimension scales.  Only the HDF5 C
// API entry points below are used (1.10 ABI: hid_t is 64-bit).
typedef int64_t hid_t_;
typedef unsigned long long hsize_t_;

struct H5Api {
  bool ok = false;
  int (*open)(void);
  int (*eset_auto2)(hid_t_, void *, void *);
  hid_t_ (*fopen)(const char *, unsigned, hid_t_);
  int (*fclose)(hid_t_);
  long (*lget_name_by_idx)(hid_t_, const char *, int, int, hsize_t_, char *, size_t, hid_t_);
  int (*lexists)(hid_t_, const char *, hid_t_);
  hid_t_ (*dopen2)(hid_t_, const char *, hid_t_);
  int (*dclose)(hid_t_);
  hid_t_ (*dget_space)(hid_t_);
  hid_t_ (*dget_type)(hid_t_);
  int (*tget_class)(hid_t_);
  int (*tclose)(hid_t_);
  int (*sget_simple_extent_ndims)(hid_t_);
  int (*sget_simple_extent_dims)(hid_t_, hsize_t_ *, hsize_t_ *);
  int (*sselect_hyperslab)(hid_t_, int, const hsize_t_ *, const hsize_t_ *, const hsize_t_ *, const hsize_t_ *);
  hid_t_ (*screate_simple)(int, const hsize_t_ *, const hsize_t_ *);
  int (*sclose)(hid_t_);
  int (*dread)(hid_t_, hid_t_, hid_t_, hid_t_, hid_t_, void *);
  hid_t_ *native_float;
  // chunk table of a dataset (HDF5 >= 1.10.5): the direct chunk path below
  bool chunks = false;
  hid_t_ (*dget_create_plist)(hid_t_);
  int (*pget_layout)(hid_t_);
  int (*pget_chunk)(hid_t_, int, hsize_t_ *);
  int (*pget_nfilters)(hid_t_);
  int (*pget_filter2)(hid_t_, unsigned, unsigned *, size_t *, unsigned *, size_t, char *, unsigned *);
  int (*pclose)(hid_t_);
  size_t (*tget_size)(hid_t_);
  int (*tget_order)(hid_t_);
  int (*dget_num_chunks)(hid_t_, hid_t_, hsize_t_ *);
  int (*dget_chunk_info)(hid_t_, hid_t_, hsize_t_, hsize_t_ *, unsigned *, uint64_t *, hsize_t_ *);
};

const H5Api &h5() {
  static H5Api a;
  static std::once_flag once;
  std::call_once(once, []() {
    void *h = nullptr;
    for (const char *lib : {"libhdf5.so.103", "libhdf5.so", "/opt/conda/lib/libhdf5.so.103", "/opt/conda/lib/libhdf5.so"})
      if ((h = dlopen(lib, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) return;
    bool ok = true;
    auto get = [&](auto &fp, const char *name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      ok = ok && fp;
    };
    get(a.open, "H5open");
    get(a.eset_auto2, "H5Eset_auto2");
    get(a.fopen, "H5Fopen");
    get(a.fclose, "H5Fclose");
    get(a.lget_name_by_idx, "H5Lget_name_by_idx");
    get(a.lexists, "H5Lexists");
    get(a.dopen2, "H5Dopen2");
    get(a.dclose, "H5Dclose");
    get(a.dget_space, "H5Dget_space");
    get(a.dget_type, "H5Dget_type");
    get(a.tget_class, "H5Tget_class");
    get(a.tclose, "H5Tclose");
    get(a.sget_simple_extent_ndims, "H5Sget_simple_extent_ndims");
    get(a.sget_simple_extent_dims, "H5Sget_simple_extent_dims");
    get(a.sselect_hyperslab, "H5Sselect_hyperslab");
    get(a.screate_simple, "H5Screate_simple");
    get(a.sclose, "H5Sclose");
    get(a.dread, "H5Dread");
    a.native_float = (hid_t_ *)dlsym(h, "H5T_NATIVE_FLOAT_g");
    ok = ok && a.native_float && a.open() >= 0;
    if (ok) a.eset_auto2(0, nullptr, nullptr);     // H5E_DEFAULT: no error stack printing
    a.ok = ok;
    if (ok) {
      get(a.dget_create_plist, "H5Dget_create_plist");
      get(a.pget_layout, "H5Pget_layout");
      get(a.pget_chunk, "H5Pget_chunk");
      get(a.pget_nfilters, "H5Pget_nfilters");
      get(a.pget_filter2, "H5Pget_filter2");
      get(a.pclose, "H5Pclose");
      get(a.tget_size, "H5Tget_size");
      get(a.tget_order, "H5Tget_order");
      get(a.dget_num_chunks, "H5Dget_num_chunks");
      get(a.dget_chunk_info, "H5Dget_chunk_info");
      a.chunks = ok;
    }
  });
  return a;
}

// HDF5 signature at offset 0 (or a user block of 512, 1024, 2048 bytes)
bool is_hdf5(const char *path) {
  static const unsigned char sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  bool yes = false;
  for (long off : {0L, 512L, 1024L, 2048L}) {
    unsigned char b[8];
    if (fseek(f, off, SEEK_SET) != 0 || fread(b, 1, 8, f) != 8) break;
    if (memcmp(b, sig, 8) == 0) { yes = true; break; }
  }
  fclose(f);
  return yes;
}

constexpr int H5T_FLOAT_CLASS = 1, H5T_INTEGER_CLASS = 0;

// One (time, lat, lon) field of a netCDF-4 file.  READ_PGF.f90:30 reads
// variable 4; in a PGF file that is the only 3-D numeric variable (the
// others are the time/lat/lon coordinates), which is what is looked for.
struct H5Field {
  const H5Api &a = h5();
  hid_t_ file = -1, dset = -1, space = -1;
  hsize_t_ dims[3] = {0, 0, 0};
  ~H5Field() {
    if (space >= 0) a.sclose(space);
    if (dset >= 0) a.dclose(dset);
    if (file >= 0) a.fclose(file);
  }
  bool open(const char *path) {
    if (!a.ok || (file = a.fopen(path, 0u /* H5F_ACC_RDONLY */, 0)) < 0) return false;
    char name[256];
    for (hsize_t_ i = 0;; i++) {
      if (a.lget_name_by_idx(file, ".", 0 /* H5_INDEX_NAME */, 0 /* H5_ITER_INC */, i, name, sizeof name, 0) < 0)
        return false;
      const hid_t_ d = a.dopen2(file, name, 0);
      if (d < 0) continue;                          // a group, not a variable
      const hid_t_ sp = a.dget_space(d), ty = a.dget_type(d);
      const int cls = a.tget_class(ty);
      a.tclose(ty);
      if (a.sget_simple_extent_ndims(sp) == 3 && (cls == H5T_FLOAT_CLASS || cls == H5T_INTEGER_CLASS)) {
        a.sget_simple_extent_dims(sp, dims, nullptr);
        dset = d;
        space = sp;
        return true;
      }
      a.sclose(sp);
      a.dclose(d);
    }
  }
  // rows [y0, y0+ny) of day t, row-major, converted to float by HDF5
  bool read_rows(hsize_t_ t, hsize_t_ y0, hsize_t_ ny, float *out) {
    const hsize_t_ start[3] = {t, y0, 0}, count[3] = {1, ny, dims[2]}, mdim[1] = {ny * dims[2]};
    if (a.sselect_hyperslab(space, 0 /* H5S_SELECT_SET */, start, nullptr, count, nullptr) < 0) return false;
    const hid_t_ mem = a.screate_simple(1, mdim, nullptr);
    const int rc = a.dread(dset, *a.native_float, mem, space, 0, out);
    a.sclose(mem);
    return rc >= 0;
  }
};

// NTIMES of a netCDF-4 file: the 'time' dimension (its coordinate
// variable), else the first dimension of the field
long h5_ntimes(const char *path) {
  const H5Api &a = h5();
  if (!a.ok) return -1;
  const hid_t_ f = a.fopen(path, 0u, 0);
  if (f < 0) return -1;
  long n = -1;
  if (a.lexists(f, "time", 0) > 0) {
    const hid_t_ d = a.dopen2(f, "time", 0);
    if (d >= 0) {
      const hid_t_ sp = a.dget_space(d);
      hsize_t_ dd[4];
      if (a.sget_simple_extent_ndims(sp) == 1 && a.sget_simple_extent_dims(sp, dd, nullptr) == 1) n = (long)dd[0];
      a.sclose(sp);
      a.dclose(d);
    }
  }
  a.fclose(f);
  if (n < 0) {
    H5Field fld;
    if (fld.open(path)) n = (long)fld.dims[0];
  }
  return n;
}

// ------------------------------------------- direct chunk reads (round 4)
// The PGF netCDF-4 files are chunked, shuffled and deflated float fields.
// Reading them day by day through H5Dread (round 3) runs every chunk's
// inflate inside HDF5, whose global lock serialises the threads of a
// thread-safe build (this image's 1.10.6 is one): 53 s per 0.5 deg year in
// an 8-core container.  Instead the chunk table (file address,
// stored size, filter mask of each chunk) is read once through HDF5, and
// the chunks the context's cells fall in are then read with pread, inflated
// (libdeflate, else zlib) and unshuffled on a pool of host threads outside
// HDF5.  Any other layout (a non-float or fletcher32-checked field, a filter
// other than shuffle/deflate) takes the H5Dread path.
struct Inflate {
  bool ok = false;
  void *(*alloc)(void) = nullptr;                                        // libdeflate
  int (*zlib)(void *, const void *, size_t, void *, size_t, size_t *) = nullptr;
  void (*release)(void *) = nullptr;
  int (*uncompress)(unsigned char *, unsigned long *, const unsigned char *, unsigned long) = nullptr;   // zlib
};
const Inflate &inflater() {
  static Inflate z;
  static std::once_flag once;
  std::call_once(once, []() {
    for (const char *lib : {"libdeflate.so.0", "/opt/conda/lib/libdeflate.so.0"})
      if (void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL)) {
        z.alloc = reinterpret_cast<void *(*)(void)>(dlsym(h, "libdeflate_alloc_decompressor"));
        z.zlib = reinterpret_cast<int (*)(void *, const void *, size_t, void *, size_t, size_t *)>(
            dlsym(h, "libdeflate_zlib_decompress"));
        z.release = reinterpret_cast<void (*)(void *)>(dlsym(h, "libdeflate_free_decompressor"));
        if (z.alloc && z.zlib && z.release) { z.ok = true; return; }
        z.alloc = nullptr;
        z.zlib = nullptr;
        z.release = nullptr;
      }
    for (const char *lib : {"libz.so.1", "/opt/conda/lib/libz.so.1"})
      if (void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL)) {
        z.uncompress = reinterpret_cast<int (*)(unsigned char *, unsigned long *, const unsigned char *,
                                                unsigned long)>(dlsym(h, "uncompress"));
        if (z.uncompress) { z.ok = true; return; }
      }
  });
  return z;
}
// zlib stream `in` -> exactly n_out bytes; st: per-thread libdeflate state
bool inflate_exact(void *&st, const unsigned char *in, size_t n_in, unsigned char *out, size_t n_out) {
  const Inflate &z = inflater();
  if (z.zlib) {
    if (!st) st = z.alloc();
    size_t got = 0;
    return st && z.zlib(st, in, n_in, out, n_out, &got) == 0 && got == n_out;
  }
  if (!z.uncompress) return false;
  unsigned long got = n_out;
  return z.uncompress(out, &got, in, n_in) == 0 && got == n_out;
}

struct Chunked {               // a (time, lat, lon) field stored as filtered chunks
  hsize_t_ dims[3] = {0, 0, 0}, cd[3] = {0, 0, 0};
  int nfilt = 0;
  int filt[8] = {0};           // pipeline order (applied in this order on write)
  bool be = false;
  struct Ch {
    hsize_t_ c[3];
    uint64_t addr, size;
    unsigned mask;
  };
  std::vector<Ch> ch;
  // true if the field's chunks can be read and decoded directly
  bool load(const char *path) {
    const H5Api &a = h5();
    if (!a.ok || !a.chunks) return false;
    H5Field fld;
    if (!fld.open(path)) return false;
    for (int i = 0; i < 3; i++) dims[i] = fld.dims[i];
    const hid_t_ ty = a.dget_type(fld.dset);
    const bool f32 = a.tget_class(ty) == H5T_FLOAT_CLASS && a.tget_size(ty) == 4;
    be = a.tget_order(ty) == 1;                   // H5T_ORDER_BE
    a.tclose(ty);
    if (!f32) return false;
    const hid_t_ pl = a.dget_create_plist(fld.dset);
    if (pl < 0) return false;
    bool ok = a.pget_layout(pl) == 2 /* H5D_CHUNKED */ && a.pget_chunk(pl, 3, cd) == 3;
    nfilt = ok ? a.pget_nfilters(pl) : -1;
    ok = ok && nfilt >= 0 && nfilt <= 8;
    for (int i = 0; ok && i < nfilt; i++) {
      unsigned flags = 0, cdv[8], fcfg = 0;
      size_t ncd = 8;
      char nm[32];
      filt[i] = a.pget_filter2(pl, (unsigned)i, &flags, &ncd, cdv, sizeof nm, nm, &fcfg);
      ok = filt[i] == 1 /* H5Z_FILTER_DEFLATE */ || filt[i] == 2 /* H5Z_FILTER_SHUFFLE */;
    }
    a.pclose(pl);
    if (!ok || !inflater().ok) return false;
    hsize_t_ n = 0;
    // (1.10.6 rejects H5S_ALL here: pass the dataset's own dataspace)
    if (a.dget_num_chunks(fld.dset, fld.space, &n) < 0) return false;
    ch.resize((size_t)n);
    for (hsize_t_ i = 0; i < n; i++) {
      Ch &c = ch[(size_t)i];
      hsize_t_ sz = 0;
      if (a.dget_chunk_info(fld.dset, fld.space, i, c.c, &c.mask, &c.addr, &sz) < 0) return false;
      c.size = sz;
    }
    return true;
  }
  size_t chunk_bytes() const { return (size_t)(cd[0] * cd[1] * cd[2]) * 4; }
  // Decodes a chunk.  The values end in *data: 4-byte elements, either
  // plain or, when the last filter to undo is the shuffle, still as the
  // shuffle's 4 byte planes -- the gather then reads each wanted element
  // from the planes (value()), so only the cells' values are ever
  // reassembled (a quarter of a 0.5 deg day).  raw and tmp are scratch.
  struct View {
    const unsigned char *p;
    size_t ne;
    bool planes, be;
    float value(size_t e) const {
      uint32_t u;
      if (planes)
        u = (uint32_t)p[e] | (uint32_t)p[ne + e] << 8 | (uint32_t)p[2 * ne + e] << 16 | (uint32_t)p[3 * ne + e] << 24;
      else
        memcpy(&u, p + 4 * e, 4);
      if (be) u = __builtin_bswap32(u);
      float f;
      memcpy(&f, &u, 4);
      return f;
    }
  };
  bool decode(int fd, const Ch &c, std::vector<unsigned char> &raw, std::vector<unsigned char> &tmp, View &out,
              void *&zst, double *t_stage) const {
    const size_t nb = chunk_bytes();
    raw.resize((size_t)c.size);
    const double ta = now_s();
    if (pread(fd, raw.data(), (size_t)c.size, (off_t)c.addr) != (ssize_t)c.size) return false;
    const double tb = now_s();
    t_stage[0] += tb - ta;
    struct Tail {                                 // the rest is inflate / unshuffle time
      double t0, *acc;
      ~Tail() { *acc += now_s() - t0; }
    } tail{tb, t_stage + 1};
    std::vector<unsigned char> *cur = &raw, *spare = &tmp;
    bool planes = false;
    for (int i = nfilt - 1; i >= 0; i--) {        // undo the pipeline in reverse
      if (c.mask & (1u << i)) continue;           // filter skipped for this chunk
      if (planes) {                               // a filter below the shuffle: reassemble first
        spare->resize(nb);
        const View v{cur->data(), nb / 4, true, false};
        for (size_t e = 0; e < nb / 4; e++) {
          const float f = v.value(e);
          memcpy(spare->data() + 4 * e, &f, 4);
        }
        std::swap(cur, spare);
        planes = false;
      }
      if (filt[i] == 1) {
        spare->resize(nb);
        if (!inflate_exact(zst, cur->data(), cur->size(), spare->data(), nb)) return false;
        std::swap(cur, spare);
      } else {
        if (cur->size() != nb) return false;
        planes = true;
      }
    }
    if (cur->size() != nb) return false;
    out = View{cur->data(), nb / 4, planes, be};
    return true;
  }
};

// Host threads of the ingest pool: $H9G_IO_THREADS, else the CPUs this
// process may run on (its affinity mask: the lease), at most
// $OMP_NUM_THREADS when that is set (the MI355X boxes set it to a GPU's
// share, 16), else at most 16.
int io_threads() {
  if (const char *e = getenv("H9G_IO_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return v;
  }
  unsigned hc = std::thread::hardware_concurrency();
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) hc = (unsigned)CPU_COUNT(&set);
  unsigned cap = 16;
  if (const char *e = getenv("OMP_NUM_THREADS"))
    if (atoi(e) > 0) cap = (unsigned)atoi(e);
  return (int)std::max(1u, std::min(cap, hc ? hc : 1u));
}

// Runs job(i, worker) for i in [0, n) on the pool; false if any job failed.
template <class F>
bool run_pool(size_t n, F job) {
  const int nt = (int)std::min<size_t>((size_t)io_threads(), std::max<size_t>(n, 1));
  std::atomic<size_t> next{0};
  std::atomic<bool> ok{true};
  auto work = [&](int w) {
    for (size_t i; ok.load(std::memory_order_relaxed) && (i = next.fetch_add(1)) < n;)
      if (!job(i, w)) ok = false;
  };
  std::vector<std::thread> th;
  for (int w = 1; w < nt; w++) th.emplace_back(work, w);
  work(0);
  for (auto &t : th) t.join();
  return ok;
}

// ------------------------------------------------------------------ writer
struct Att {
  std::string name;
  int type;
  std::vector<unsigned char> be;   // big-endian payload
  uint32_t nel;
};
struct WVar {
  std::string name;
  std::vector<int> dims;
  std::vector<Att> atts;
  uint64_t nel = 0, begin = 0;
};

struct Buf {
  std::vector<unsigned char> b;
  void u32(uint32_t x) {
    unsigned char c[4] = {(unsigned char)(x >> 24), (unsigned char)(x >> 16), (unsigned char)(x >> 8),
                          (unsigned char)x};
    b.insert(b.end(), c, c + 4);
  }
  void u64(uint64_t x) {
    u32((uint32_t)(x >> 32));
    u32((uint32_t)x);
  }
  void pad() {
    while (b.size() % 4) b.push_back(0);
  }
  void name(const std::string &s) {
    u32((uint32_t)s.size());
    b.insert(b.end(), s.begin(), s.end());
    pad();
  }
};

Att text_att(const char *name, const char *v) {
  Att a{name, NC_CHAR, {}, (uint32_t)strlen(v)};
  a.be.assign(v, v + strlen(v));
  return a;
}
Att float_att(const char *name, float v) {
  Att a{name, NC_FLOAT, {}, 1};
  uint32_t u;
  memcpy(&u, &v, 4);
  a.be = {(unsigned char)(u >> 24), (unsigned char)(u >> 16), (unsigned char)(u >> 8), (unsigned char)u};
  return a;
}

// CDF-2 file with fixed-size float variables; data(v, out) fills v's values.
template <class F>
int write_cdf2(const char *path, const std::vector<std::pair<std::string, uint32_t>> &dims,
               std::vector<WVar> &vars, F data) {
  auto header = [&]() {
    Buf h;
    h.b = {'C', 'D', 'F', 2};
    h.u32(0);                                    // numrecs
    h.u32(TAG_DIM);
    h.u32((uint32_t)dims.size());
    for (auto &d : dims) {
      h.name(d.first);
      h.u32(d.second);
    }
    h.u32(0);                                    // no global attributes
    h.u32(0);
    h.u32(TAG_VAR);
    h.u32((uint32_t)vars.size());
    for (auto &v : vars) {
      h.name(v.name);
      h.u32((uint32_t)v.dims.size());
      for (int d : v.dims) h.u32((uint32_t)d);
      if (v.atts.empty()) {
        h.u32(0);
        h.u32(0);
      } else {
        h.u32(TAG_ATT);
        h.u32((uint32_t)v.atts.size());
        for (auto &a : v.atts) {
          h.name(a.name);
          h.u32((uint32_t)a.type);
          h.u32(a.nel);
          h.b.insert(h.b.end(), a.be.begin(), a.be.end());
          h.pad();
        }
      }
      h.u32(NC_FLOAT);
      const uint64_t vs = pad4(v.nel * 4);
      h.u32(vs > 0xffffffffu ? 0xffffffffu : (uint32_t)vs);
      h.u64(v.begin);
    }
    return h;
  };
  Buf h = header();                              // sizes first, then the real begins
  uint64_t off = h.b.size();
  for (auto &v : vars) {
    v.begin = off;
    off += pad4(v.nel * 4);
  }
  h = header();
  FILE *f = fopen(path, "wb");
  if (!f) return H9G_EINVAL;
  bool ok = fwrite(h.b.data(), 1, h.b.size(), f) == h.b.size();
  std::vector<float> tmp;
  for (size_t k = 0; ok && k < vars.size(); k++) {
    tmp.assign(vars[k].nel, 0.0f);
    data(k, tmp.data());
    uint32_t *u = (uint32_t *)tmp.data();
    for (uint64_t i = 0; i < vars[k].nel; i++) u[i] = __builtin_bswap32(u[i]);
    ok = fwrite(tmp.data(), 4, vars[k].nel, f) == vars[k].nel;
  }
  ok = (fclose(f) == 0) && ok;
  return ok ? 0 : H9G_EINVAL;
}

}  // namespace

// --------------------------------------------------------------- C-ABI
extern "C" {

#ifndef H9G_BUILD_ID
#define H9G_BUILD_ID "unknown"
#endif
// Digest of the sources and flags this library was compiled from
// (hybrid9_amd/build.py build_id); profiles record it, bench.py matches it.
// Defined here, in the translation unit compiled last and in seconds, so
// the device code's object is reused when only this digest changes.
const char *h9g_build_id(void) { return H9G_BUILD_ID; }

// WRITE_NET_CDF_3DR.f90: one year of annual means of the cells `gid`
// (grid ids iy*nx+ix, latitude row iy from the north, INIT.f90:142-145) to
// a CDF-2 file; every other grid cell is the NaN fill.
int h9g_write_axy_nc(const char *path, int nx, int ny, int nlayers, const float *zc, int ncell,
                     const int64_t *gid, const float *annual) {
  if (!path || nx <= 0 || ny <= 0 || nlayers < 1 || nlayers > H9G_LMAX || ncell < 0 || (ncell && (!gid || !annual)))
    return H9G_EINVAL;
  const int L = nlayers;
  for (int c = 0; c < ncell; c++)
    if (gid[c] < 0 || gid[c] >= (int64_t)nx * ny) return H9G_EINVAL;
  const float nan = std::nanf("");
  // dims in definition order (WRITE_NET_CDF_3DR.f90:101-103)
  const std::vector<std::pair<std::string, uint32_t>> dims = {
      {"latitude", (uint32_t)ny}, {"longitude", (uint32_t)nx}, {"layer_centre_depth", (uint32_t)L}};
  enum { D_LAT = 0, D_LON = 1, D_Z = 2 };
  // (name, units, annual row) of the 2-D fields (:53-77, :142-180)
  struct F2 { const char *name, *units; int row; };
  const F2 f2[] = {{"net primary production", "g[DM]/m^2/yr", 0},
                   {"plant mass", "g[DM]", 1},
                   {"runoff", "mm/s", 2},
                   {"evaporation", "mm/s", 3},
                   {"temperature", "K", 4},
                   {"specific_humidity", "kg[water]/kg[air]", 7},
                   {"air_pressure", "Pa", 8},
                   {"precipitation", "kg/m^2/s", 9},
                   {"relative_humidity", "percent", 10},
                   {"soil_water", "mm", 11 + L}};
  std::vector<WVar> vars;
  vars.push_back({"latitude", {D_LAT}, {text_att("units", "degrees_north")}, (uint64_t)ny});
  vars.push_back({"longitude", {D_LON}, {text_att("units", "degrees_east")}, (uint64_t)nx});
  vars.push_back({"layer_centre_depth", {D_Z}, {text_att("units", "mm")}, (uint64_t)L});
  for (const F2 &v : f2)
    vars.push_back({v.name, {D_LAT, D_LON}, {text_att("units", v.units), float_att("_FillValue", nan)},
                    (uint64_t)nx * ny});
  vars.push_back({"soil_water_layers", {D_LAT, D_LON, D_Z},
                  {text_att("units", "mm^3/mm^3"), float_att("_FillValue", nan)}, (uint64_t)nx * ny * L});
  const float dlon = 360.0f / (float)nx, dlat = 180.0f / (float)ny;
  return write_cdf2(path, dims, vars, [&](size_t k, float *out) {
    const uint64_t n = vars[k].nel;
    if (k == 0) {                                // INIT.f90:145 lat_all(y) = 89.75 - (y-1)*0.5
      for (int y = 0; y < ny; y++) out[y] = (90.0f - 0.5f * dlat) - (float)y * dlat;
    } else if (k == 1) {                         // INIT.f90:142 lon_all(x) = -179.75 + (x-1)*0.5
      for (int x = 0; x < nx; x++) out[x] = (-180.0f + 0.5f * dlon) + (float)x * dlon;
    } else if (k == 2) {                         // zc_o (INIT.f90:262)
      for (int i = 0; i < L; i++) out[i] = zc ? zc[i] : nan;
    } else if (k < 3 + sizeof(f2) / sizeof(f2[0])) {
      for (uint64_t i = 0; i < n; i++) out[i] = nan;
      const int row = f2[k - 3].row;
      for (int c = 0; c < ncell; c++) out[gid[c]] = annual[(size_t)row * ncell + c];
    } else {                                     // soil_water_layers (lat, lon, z)
      for (uint64_t i = 0; i < n; i++) out[i] = nan;
      for (int c = 0; c < ncell; c++)
        for (int i = 0; i < L; i++) out[(size_t)gid[c] * L + i] = annual[(size_t)(11 + i) * ncell + c];
    }
  });
}

// READ_PGF.f90 + READ_NET_CDF_3DR.f90 for the cells of a context: days
// [t0, t0+nt) of the 7 files (READ_PGF order tas rlds rsds huss ps pr rhs),
// variable 4 of each (dims time, lat, lon), gathered at the grid ids gid
// into out (7, nt, ncell).  Like the reference, which reads only its rank's
// block (READ_NET_CDF_3DR.f90:95-97), only the rows spanning the cells are
// decoded.  All work runs on one pool of host threads (io_threads):
//   netCDF-4  one job per stored chunk holding any of the cells: pread, then
//             inflate/unshuffle outside HDF5 (Chunked), then the gather;
//             other layouts: one job per file through H5Dread, row band only
//   classic   one job per (file, day): pread of the row band, byte swap of
//             the gathered values.
int h9g_nc_forcing_read(const char *const *paths, int nx, int ny, int ncell, const int64_t *gid, int t0,
                        int nt, float *out) {
  return h9g_nc_read_groups(paths, nx, ny, ncell, gid, t0, nt, out, 1, nullptr);
}

}  // extern "C"

// The read of h9g_nc_forcing_read, reporting progress: the days are split
// into ngroups consecutive groups, and done(d0, d1) is called (on a pool
// thread, once per group, in any order) as soon as days [d0, d1) (relative
// to t0) of all 7 variables are in `out` -- h9g_nc_forcing_prefetch queues
// each group's copy to the device then, so the copies overlap the rest of
// the read.  Jobs are issued in day order.
int h9g_nc_read_groups(const char *const *paths, int nx, int ny, int ncell, const int64_t *gid, int t0, int nt,
                       float *out, int ngroups, const std::function<void(int, int)> &done) {
  if (!paths || nx <= 0 || ny <= 0 || ncell <= 0 || !gid || t0 < 0 || nt < 1 || !out) return H9G_EINVAL;
  const double tstart = now_s();
  ngroups = std::max(1, std::min(ngroups, nt));
  int64_t ymin = ny, ymax = -1;
  for (int c = 0; c < ncell; c++) {
    if (gid[c] < 0 || gid[c] >= (int64_t)nx * ny) return H9G_EINVAL;
    ymin = std::min<int64_t>(ymin, gid[c] / nx);
    ymax = std::max<int64_t>(ymax, gid[c] / nx);
  }
  const size_t plane = (size_t)nx * ny;
  struct Src {
    int kind = 0;            // 1 chunked netCDF-4, 2 other netCDF-4, 3 classic
    int fd = -1;
    Chunked ck;
    NcReader nc;
    const NcVar *v = nullptr;
    ~Src() {
      if (fd >= 0) close(fd);
    }
  };
  std::vector<Src> src(H9G_NFORCING);
  for (int k = 0; k < H9G_NFORCING; k++) {        // headers and chunk tables (HDF5 calls: serial)
    Src &s = src[(size_t)k];
    if (!paths[k]) return H9G_EINVAL;
    if (is_hdf5(paths[k])) {
      if (s.ck.load(paths[k])) {
        s.kind = 1;
        if ((s.fd = open(paths[k], O_RDONLY)) < 0) return H9G_EINVAL;
      } else {
        H5Field fld;
        if (!fld.open(paths[k])) return H9G_EINVAL;
        for (int i = 0; i < 3; i++) s.ck.dims[i] = fld.dims[i];
        s.kind = 2;
      }
      if (s.ck.dims[1] != (hsize_t_)ny || s.ck.dims[2] != (hsize_t_)nx || (hsize_t_)(t0 + nt) > s.ck.dims[0])
        return H9G_EINVAL;
      continue;
    }
    NcReader &r = s.nc;
    if (!r.open(paths[k]) || r.vars.empty()) return H9G_EINVAL;
    // varid = 4 (READ_PGF.f90:30) when it is the (time, lat, lon) float
    // field, as in the PGF files; otherwise the file's only such field
    const int dt = r.dim_index("time");
    auto is_field = [&](const NcVar &x) { return x.type == NC_FLOAT && x.dims.size() == 3 && x.dims[0] == dt; };
    const NcVar *pv = &r.vars[r.vars.size() >= 4 ? 3 : 0];
    if (!is_field(*pv))
      for (auto &x : r.vars)
        if (is_field(x)) { pv = &x; break; }
    if (pv->type != NC_FLOAT || pv->dims.size() != 3 || pv->dims[0] != dt || r.dim_of(*pv, 1) != (uint64_t)ny ||
        r.dim_of(*pv, 2) != (uint64_t)nx || (uint64_t)(t0 + nt) > r.dim_of(*pv, 0))
      return H9G_EINVAL;
    s.v = pv;
    s.kind = 3;
    if ((s.fd = open(paths[k], O_RDONLY)) < 0) return H9G_EINVAL;
  }
  // jobs: (file, chunk) for chunked files, (file, day) for classic, (file)
  // otherwise; d0..d1: the days (relative to t0) a job fills
  struct Job { int k; size_t i; int d0, d1; };
  std::vector<Job> jobs;
  // cells by chunk column (per chunked file's chunk shape; usually shared)
  struct Cols {
    hsize_t_ cy = 0, cx = 0;
    size_t nbx = 0;
    std::vector<std::vector<std::pair<int, uint32_t>>> cells;   // (cell, offset in the chunk's plane)
  };
  std::vector<Cols> cols(H9G_NFORCING);
  for (int k = 0; k < H9G_NFORCING; k++) {
    Src &s = src[(size_t)k];
    if (s.kind == 1) {
      Cols &cl = cols[(size_t)k];
      cl.cy = s.ck.cd[1];
      cl.cx = s.ck.cd[2];
      cl.nbx = (size_t)((nx + cl.cx - 1) / cl.cx);
      cl.cells.resize(cl.nbx * (size_t)((ny + cl.cy - 1) / cl.cy));
      for (int c = 0; c < ncell; c++) {
        const hsize_t_ y = (hsize_t_)(gid[c] / nx), x = (hsize_t_)(gid[c] % nx);
        cl.cells[(size_t)(y / cl.cy) * cl.nbx + (size_t)(x / cl.cx)].push_back(
            {c, (uint32_t)((y % cl.cy) * cl.cx + x % cl.cx)});
      }
      const size_t j0 = jobs.size();
      for (size_t i = 0; i < s.ck.ch.size(); i++) {
        const auto &ch = s.ck.ch[i];
        if (ch.c[0] + s.ck.cd[0] <= (hsize_t_)t0 || ch.c[0] >= (hsize_t_)(t0 + nt)) continue;
        if (!cl.cells[(size_t)(ch.c[1] / cl.cy) * cl.nbx + (size_t)(ch.c[2] / cl.cx)].empty()) {
          const int d0 = (int)std::max<hsize_t_>(ch.c[0], (hsize_t_)t0) - t0;
          const int d1 = (int)std::min<hsize_t_>(ch.c[0] + s.ck.cd[0], (hsize_t_)(t0 + nt)) - t0;
          jobs.push_back({k, i, d0, d1});
        }
      }
      // The chunk table lists only the chunks that were written.  A chunk
      // holding cells of the days asked for that was never written (its
      // values are the fill value) has no entry: then the file is read
      // through H5Dread, which fills it, as the reference's nf90_get_var
      // does.  Entries are unique by their coordinates, so
      // the count decides.
      size_t cols_used = 0;
      for (const auto &v : cl.cells) cols_used += !v.empty();
      const size_t tchunks = (size_t)((hsize_t_)(t0 + nt - 1) / s.ck.cd[0] - (hsize_t_)t0 / s.ck.cd[0] + 1);
      if (jobs.size() - j0 != tchunks * cols_used) {
        jobs.resize(j0);
        s.kind = 2;
        jobs.push_back({k, 0, 0, nt});
      }
    } else if (s.kind == 3) {
      for (int t = 0; t < nt; t++) jobs.push_back({k, (size_t)t, t, t + 1});
    } else {
      jobs.push_back({k, 0, 0, nt});
    }
  }
  std::stable_sort(jobs.begin(), jobs.end(), [](const Job &a, const Job &b) { return a.d0 < b.d0; });
  // day groups [gd(g), gd(g+1)) and the jobs each still waits for
  auto gd = [&](int g) { return (int)((long long)nt * g / ngroups); };
  auto group_of = [&](int d) {                     // the group holding day d
    int g = (int)((long long)d * ngroups / nt);
    while (g + 1 < ngroups && gd(g + 1) <= d) g++;
    while (g > 0 && gd(g) > d) g--;
    return g;
  };
  std::vector<std::atomic<int>> pending((size_t)ngroups);
  for (auto &p : pending) p = 0;
  for (const Job &jb : jobs)
    for (int g = group_of(jb.d0); g <= group_of(jb.d1 - 1); g++) pending[(size_t)g]++;
  // a group no job fills (cannot happen with every file covering every
  // day; kept so that a prefetch never waits on a copy nobody queues)
  for (int g = 0; g < ngroups; g++)
    if (pending[(size_t)g] == 0 && done) done(gd(g), gd(g + 1));
  const int nw = io_threads();
  struct Scratch {
    std::vector<unsigned char> raw, tmp;
    std::vector<float> vals;
    void *z = nullptr;
    double t[4] = {0, 0, 0, 0};          // pread, inflate + unshuffle, gather, other layouts (s)
    double bytes_in = 0, bytes_out = 0, values = 0, jobs = 0;
  };
  std::vector<Scratch> scr((size_t)nw);
  std::mutex h5lock;                                // kind 2 goes through HDF5
  auto finish = [&](const Job &jb) {
    for (int g = group_of(jb.d0); g <= group_of(jb.d1 - 1); g++)
      if (--pending[(size_t)g] == 0 && done) done(gd(g), gd(g + 1));
  };
  auto one = [&](const Job &jb, Scratch &sc) -> bool {
    Src &s = src[(size_t)jb.k];
    if (s.kind == 1) {
      const auto &ch = s.ck.ch[jb.i];
      Chunked::View v;
      if (!s.ck.decode(s.fd, ch, sc.raw, sc.tmp, v, sc.z, sc.t)) return false;
      const double tg = now_s();
      const Cols &cl = cols[(size_t)jb.k];
      const auto &cells = cl.cells[(size_t)(ch.c[1] / cl.cy) * cl.nbx + (size_t)(ch.c[2] / cl.cx)];
      const size_t cplane = (size_t)(cl.cy * cl.cx);
      const hsize_t_ ta = std::max<hsize_t_>(ch.c[0], (hsize_t_)t0);
      const hsize_t_ tb = std::min<hsize_t_>(ch.c[0] + s.ck.cd[0], (hsize_t_)(t0 + nt));
      for (hsize_t_ t = ta; t < tb; t++) {
        const size_t e0 = (size_t)(t - ch.c[0]) * cplane;
        float *o = out + ((size_t)jb.k * nt + (size_t)(t - (hsize_t_)t0)) * ncell;
        for (const auto &p : cells) o[p.first] = v.value(e0 + p.second);
      }
      sc.t[2] += now_s() - tg;
      sc.bytes_in += (double)ch.size;
      sc.bytes_out += (double)s.ck.chunk_bytes();
      sc.values += (double)cells.size() * (double)(tb - ta);
      return true;
    }
    const double to = now_s();
    struct Tail {
      double t0, *acc;
      ~Tail() { *acc += now_s() - t0; }
    } tail{to, sc.t + 3};
    if (s.kind == 3) {                              // classic: rows [ymin, ymax] of day t0 + i
      const NcReader &r = s.nc;
      const NcVar &v = *s.v;
      const uint64_t t = (uint64_t)t0 + jb.i;
      const uint64_t off = (v.record ? v.begin + t * r.recsize : v.begin + t * plane * 4) + (uint64_t)ymin * nx * 4;
      const size_t nb = (size_t)(ymax - ymin + 1) * nx * 4;
      sc.raw.resize(nb);
      if (pread(s.fd, sc.raw.data(), nb, (off_t)off) != (ssize_t)nb) return false;
      const uint32_t *u = (const uint32_t *)sc.raw.data();
      uint32_t *o = (uint32_t *)(out + ((size_t)jb.k * nt + jb.i) * ncell);
      const size_t base = (size_t)ymin * nx;
      for (int c = 0; c < ncell; c++) o[c] = __builtin_bswap32(u[(size_t)gid[c] - base]);
      return true;
    }
    // netCDF-4 of another layout: H5Dread of the row band, day by day
    std::lock_guard<std::mutex> g(h5lock);
    H5Field fld;
    if (!fld.open(paths[jb.k])) return false;
    const hsize_t_ nyb = (hsize_t_)(ymax - ymin + 1);
    sc.vals.resize((size_t)nyb * nx);
    for (int t = 0; t < nt; t++) {
      if (!fld.read_rows((hsize_t_)(t0 + t), (hsize_t_)ymin, nyb, sc.vals.data())) return false;
      float *o = out + ((size_t)jb.k * nt + t) * ncell;
      const size_t base = (size_t)ymin * nx;
      for (int c = 0; c < ncell; c++) o[c] = sc.vals[(size_t)gid[c] - base];
    }
    return true;
  };
  const double tpool = now_s();
  const bool ok = run_pool(jobs.size(), [&](size_t j, int w) -> bool {
    Scratch &sc = scr[(size_t)w % scr.size()];
    if (!one(jobs[j], sc)) return false;
    sc.jobs += 1;
    finish(jobs[j]);
    return true;
  });
  const double tend = now_s();
  for (auto &sc : scr)
    if (sc.z && inflater().release) inflater().release(sc.z);
  {
    std::lock_guard<std::mutex> g(g_stats_lock);
    double st[H9G_IO_NSTATS] = {tend - tstart, tpool - tstart,
                                (double)std::min<size_t>((size_t)nw, std::max<size_t>(jobs.size(), 1)), 0, 0, 0, 0,
                                0, 0, 0, 0, tend - tpool};
    for (auto &sc : scr) {
      st[3] += sc.jobs;
      for (int i = 0; i < 4; i++) st[4 + i] += sc.t[i];
      st[8] += sc.bytes_in;
      st[9] += sc.bytes_out;
      st[10] += sc.values;
    }
    memcpy(g_stats, st, sizeof st);
  }
  return ok ? 0 : H9G_EINVAL;
}

extern "C" {

int h9g_nc_read_stats(double *out, int n) {
  if (!out || n < 1) return H9G_EINVAL;
  std::lock_guard<std::mutex> g(g_stats_lock);
  const int m = std::min(n, (int)H9G_IO_NSTATS);
  memcpy(out, g_stats, sizeof(double) * (size_t)m);
  return m;
}

// NTIMES of a PGF file (READ_NET_CDF_0D.f90: the 'time' dimension).
int h9g_nc_ntimes(const char *path) {
  if (path && is_hdf5(path)) {
    const long n = h5_ntimes(path);
    return n < 0 ? H9G_EINVAL : (int)n;
  }
  NcReader r;
  if (!path || !r.open(path)) return H9G_EINVAL;
  const int d = r.dim_index("time");
  if (d < 0) return H9G_EINVAL;
  return d == r.rec_dim ? (int)r.numrecs : (int)r.dim_len[d];
}

}  // extern "C"
