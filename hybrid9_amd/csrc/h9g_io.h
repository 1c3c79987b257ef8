// h9g_io.h -- internal interface of h9g_io.cpp used by h9g.hip (not ABI).
#pragma once
#include <stdint.h>

#include <functional>

// h9g_nc_forcing_read with progress: done(d0, d1) once days [d0, d1)
// (relative to t0) of all 7 variables are in out, for ngroups consecutive
// day groups (any order, on a pool thread).
int h9g_nc_read_groups(const char *const *paths, int nx, int ny, int ncell, const int64_t *gid, int t0, int nt,
                       float *out, int ngroups, const std::function<void(int, int)> &done);
