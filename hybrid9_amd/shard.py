"""Sharding of land cells over GPUs.

The reference decomposes the globe into sqrt(P) x sqrt(P) equal blocks, one
per MPI rank, and the ranks never communicate during compute
(``INIT.f90:271-274,427-456``; ``HYBRID9.f90:120-295``).  Cells are
independent under isolated-cell semantics, so here a shard is a contiguous
range of the compacted land-cell list -- balanced, unlike square blocks that
leave ocean-only ranks idle.  The only cross-GPU traffic is the all-reduce of
the FP64 global diagnostics (``h9g_get_diagnostics``) once per year.
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
