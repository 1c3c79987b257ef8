// The host C/C++ of the product and its checkers under AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_sanitize.py).  Built
// with g++/gcc -fsanitize=address,undefined from the same sources as
// libh9g.so's host part and the checkers:
//   hybrid9_amd/csrc/h9g_io.cpp   the NetCDF reader (threaded inflate pool)
//                                 and the axyYYYY.nc writer
//   oracle/h9_oracle.c            the C restatement (OpenMP over cells)
//   tests/csrc/host_kernel.cpp    the kernel body built for the host
// Modes:
//   san_driver io <cdf2 dir> <nc4 dir|-> <nx> <ny> <nt> <ncell> <gid.i64> <out.nc>
//     reads days [1, nt-1) of the 7 PGF files of both directories with 1, 3
//     and 8 pool threads (they must agree value for value), prints the stage
//     profile, writes the gathered first day as an annual file
//   san_driver hydro <case dir>
//     runs the oracle (4 threads) and the host kernel body on the case
//     (n L nisurf grow_on year0 nyears in case.txt; zi, params, forcing as
//     raw float32) and checks that they agree bit for bit
// Any sanitizer report aborts with a non-zero exit (halt_on_error).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "h9g.h"
extern "C" {
#include "../../oracle/h9_oracle.h"
}

extern "C" int h9k_host_run(int n, int L, int nisurf, int grow_on, int year0, int nyears, int use_const_geo,
                            const float *zi, const float *par, const float *forc, float *st, float *ann, int *err);

static const char *kVars[7] = {"tas", "rlds", "rsds", "huss", "ps", "pr", "rhs"};

template <class T>
static std::vector<T> slurp(const std::string &path, size_t n) {
  std::vector<T> v(n);
  FILE *f = fopen(path.c_str(), "rb");
  if (!f || fread(v.data(), sizeof(T), n, f) != n) {
    fprintf(stderr, "san_driver: cannot read %zu values from %s\n", n, path.c_str());
    exit(2);
  }
  fclose(f);
  return v;
}

static int io_mode(int argc, char **argv) {
  if (argc != 10) return 2;
  const std::string d2 = argv[2], d4 = argv[3];
  const int nx = atoi(argv[4]), ny = atoi(argv[5]), nt = atoi(argv[6]), n = atoi(argv[7]);
  const std::vector<int64_t> gid = slurp<int64_t>(argv[8], (size_t)n);
  std::vector<std::string> p2, p4;
  for (const char *v : kVars) {
    p2.push_back(d2 + "/" + v + ".nc");
    p4.push_back(d4 + "/" + v + "_pgfv2.1_1901-1910.nc4");
  }
  std::vector<const char *> c2, c4;
  for (auto &s : p2) c2.push_back(s.c_str());
  for (auto &s : p4) c4.push_back(s.c_str());
  const int t0 = 1, cnt = nt - 2;
  std::vector<float> ref;
  for (const char *threads : {"1", "3", "8"}) {
    setenv("H9G_IO_THREADS", threads, 1);
    for (int form = 0; form < (d4 == "-" ? 1 : 2); form++) {
      std::vector<float> out((size_t)7 * cnt * n, -1.0f);
      const int rc = h9g_nc_forcing_read(form ? c4.data() : c2.data(), nx, ny, n, gid.data(), t0, cnt, out.data());
      if (rc) {
        fprintf(stderr, "san_driver: read (%s, %s threads) failed: %d\n", form ? "nc4" : "cdf2", threads, rc);
        return 1;
      }
      if (ref.empty()) ref = out;
      if (memcmp(ref.data(), out.data(), sizeof(float) * ref.size()) != 0) {
        fprintf(stderr, "san_driver: %s read with %s threads differs\n", form ? "nc4" : "cdf2", threads);
        return 1;
      }
      double st[H9G_IO_NSTATS];
      const int m = h9g_nc_read_stats(st, H9G_IO_NSTATS);
      printf("read %s threads=%s: %d stats, wall %.4f s, threads %.0f, jobs %.0f\n", form ? "nc4" : "cdf2", threads,
             m, st[0], st[2], st[3]);
    }
  }
  if (h9g_nc_ntimes(c2[0]) != nt) return 1;
  // a bad request must fail cleanly, not read out of bounds
  std::vector<float> bad((size_t)7 * nt * n);
  if (h9g_nc_forcing_read(c2.data(), nx, ny, n, gid.data(), nt - 1, 5, bad.data()) == 0) return 1;
  // the first gathered day as 12+L annual rows (L = 8) through the writer
  const int L = 8;
  std::vector<float> ann((size_t)(12 + L) * n);
  for (int r = 0; r < 12 + L; r++)
    for (int c = 0; c < n; c++) ann[(size_t)r * n + c] = ref[(size_t)(r % 7) * cnt * n + c];
  std::vector<float> zc(L);
  for (int i = 0; i < L; i++) zc[i] = 10.0f * (float)(i + 1);
  const int rc = h9g_write_axy_nc(argv[9], nx, ny, L, zc.data(), n, gid.data(), ann.data());
  printf("write %s: %d\n", argv[9], rc);
  return rc ? 1 : 0;
}

static int hydro_mode(int argc, char **argv) {
  if (argc != 3) return 2;
  const std::string d = argv[2];
  int n, L, ns, grow, year0, ny;
  {
    FILE *f = fopen((d + "/case.txt").c_str(), "r");
    if (!f || fscanf(f, "%d %d %d %d %d %d", &n, &L, &ns, &grow, &year0, &ny) != 6) return 2;
    fclose(f);
  }
  int nd = 0;
  for (int y = year0; y < year0 + ny; y++) nd += (y % 4 == 0 && (y % 100 != 0 || y % 400 == 0)) ? 366 : 365;
  const std::vector<float> zi = slurp<float>(d + "/zi.f32", (size_t)L + 2);
  const std::vector<float> par = slurp<float>(d + "/params.f32", (size_t)(4 * L + 1) * n);
  const std::vector<float> forc = slurp<float>(d + "/forcing.f32", (size_t)7 * nd * n);
  const size_t ss = (size_t)h9o_state_size(L) * n;
  std::vector<float> st_o(ss), st_k(ss);
  if (h9o_init_state(n, L, zi.data(), par.data(), st_o.data())) return 1;
  st_k = st_o;
  std::vector<float> ann_o((size_t)ny * (12 + L) * n), ann_k(ann_o.size());
  std::vector<int> cerr((size_t)4 * n), kerr((size_t)4 * n);
  h9o_error e{};
  const int ro = h9o_run(n, L, ns, grow, year0, ny, zi.data(), par.data(), forc.data(), st_o.data(), ann_o.data(), 0,
                         nullptr, nullptr, 4, &e, cerr.data());
  const int rk = h9k_host_run(n, L, ns, grow, year0, ny, 0, zi.data(), par.data(), forc.data(), st_k.data(),
                              ann_k.data(), kerr.data());
  const bool same = ro == rk && memcmp(ann_o.data(), ann_k.data(), sizeof(float) * ann_o.size()) == 0 &&
                    memcmp(st_o.data(), st_k.data(), sizeof(float) * ss) == 0;
  printf("hydro: %d cells x %d yr, oracle rc %d, host kernel rc %d, %s\n", n, ny, ro, rk,
         same ? "bit-identical" : "DIFFER");
  return same ? 0 : 1;
}

int main(int argc, char **argv) {
  if (argc >= 2 && strcmp(argv[1], "io") == 0) return io_mode(argc, argv);
  if (argc >= 2 && strcmp(argv[1], "hydro") == 0) return hydro_mode(argc, argv);
  fprintf(stderr, "usage: san_driver io ... | san_driver hydro <case dir>\n");
  return 2;
}
