"""Sharding of land cells over GPUs.

The reference decomposes the globe into sqrt(P) x sqrt(P) equal blocks, one
per MPI rank, and the ranks never communicate during compute
(``INIT.f90:271-274,427-456``; ``HYBRID9.f90:120-295``).  Cells are
independent under isolated-cell semantics, so there a shard is a contiguous
range of the compacted land-cell list -- balanced, unlike square blocks that
leave ocean-only ranks idle.  In the reference's own cell order a block is
one chain, so a rank takes whole blocks (``blocks_of_rank``).  The only
cross-GPU traffic is the all-reduce of the FP64 global diagnostics
(``h9g_get_diagnostics``) once per year or per ordered call.
"""
from __future__ import annotations

import numpy as np

from . import DIAG_NAMES


def shard_slice(n: int, rank: int, world: int) -> slice:
    """Contiguous balanced range of ``n`` cells for ``rank`` of ``world``."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return slice(lo, lo + base + (1 if rank < extra else 0))


def reference_blocks(gid, nx: int, ny: int, num_procs: int) -> np.ndarray:
    """The reference rank (MPI block) of every grid id ``gid`` (iy * nx + ix,
    0-based) for ``num_procs`` ranks, as INIT.f90 assigns them: an
    nb x nb grid of blocks, nb = NINT(SQRT(num_procs)), of lon_c = nx / nb by
    lat_c = ny / nb cells (:271-274), numbered along longitude first
    (:427-444: chunk(x, y), i_block + 1 every lon_c columns, i_block_s + nb
    every lat_c rows).  Cells past nb * lon_c or nb * lat_c belong to no
    block (-1): the reference never runs them.  Within a block the
    reference visits its cells in (y, x) order (HYBRID9.f90:120-121), i.e.
    ascending grid id, which is the order of synth.land_cells."""
    g = np.asarray(gid, dtype=np.int64)
    nb = int(np.rint(np.sqrt(np.float32(num_procs))))
    if nb < 1:
        raise ValueError("num_procs must be >= 1")
    lon_c, lat_c = nx // nb, ny // nb
    iy, ix = g // nx, g % nx
    bx, by = ix // lon_c, iy // lat_c
    r = by * nb + bx
    return np.where((bx < nb) & (by < nb), r, -1).astype(np.int32)


def blocks_of_rank(blocks, rank: int, world: int) -> np.ndarray:
    """The cells (indices into ``blocks``, ascending) a GPU rank takes in the
    reference's cell order: whole reference blocks (``reference_blocks``),
    block b to rank b mod world.  A block is one chain of the reference's
    order (one MPI rank's cell loop, HYBRID9.f90:120-295), so the ranks'
    chains are independent and no collective joins them; cells outside
    every block (-1) belong to no rank.  Give the rank's context
    ``h9g_set_chains`` with the blocks' ids."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    b = np.asarray(blocks)
    return np.where((b >= 0) & (b % world == rank))[0]


def weak_seed(base_seed: int, rank: int) -> int:
    """Weak scaling: every rank simulates a full land grid with its own seed."""
    return base_seed + rank


def host_diagnostics(annual: np.ndarray, state_rows_end: dict, failed=None) -> np.ndarray:
    """FP64 restatement of h9g_diag_kernel for one year (testing / CPU ranks).

    annual: (12+L, ncell) annual means; state_rows_end: dict with zwt, wa, LAI
    (ncell) at the end of the year; failed: bool mask of cells that stopped."""
    L = annual.shape[0] - 12
    n = annual.shape[1]
    failed = np.zeros(n, bool) if failed is None else np.asarray(failed, bool)
    ok = (~failed) & np.isfinite(annual[2])
    d = np.zeros(len(DIAG_NAMES), np.float64)
    a = annual.astype(np.float64)
    d[0] = ok.sum()
    d[1] = a[2, ok].sum()
    d[2] = a[11 + L, ok].sum()
    d[3] = np.asarray(state_rows_end["zwt"], np.float64)[ok].sum()
    d[4] = np.asarray(state_rows_end["wa"], np.float64)[ok].sum()
    d[5] = a[0, ok].sum()
    d[6] = a[1, ok].sum()
    d[7] = np.asarray(state_rows_end["LAI"], np.float64)[ok].sum()
    d[8] = a[11, ok].sum()
    d[9] = a[4, ok].sum()
    d[10] = a[9, ok].sum()
    d[11] = failed.sum()
    return d
