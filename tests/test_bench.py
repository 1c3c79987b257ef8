"""bench.py's host side on CPU: the driver's exact invocations map to
valid context configurations that fit one MI355X, the forcing ring keeps
every year's length, and the N > 1 per-year exchange (stream-ordered
diagnostics hand-off + all-reduce) runs under gloo at world size 2."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
import hybrid9_amd as h
from hybrid9_amd import synth

HBM_BYTES = 288e9


@pytest.mark.parametrize("workload", sorted(bench.WORKLOADS))
@pytest.mark.parametrize("wk", [(5, 20), (1, 3), (0, 30), (10, 100)])
def test_driver_configs_are_valid(workload, wk):
    W, K = wk
    pl = bench.plan(workload, W, K)
    cfg = h.make_config(pl["gid"].size, pl["zi"], nlayers=pl["L"], nisurf=pl["ns"],
                        grow_on=pl["grow_on"], nslots=pl["nslots"])
    assert 1 <= pl["nslots"] <= bench.RING_MAX
    # the forcing ring plus everything else fits well inside one GPU
    assert h.config_bytes(cfg) < 0.6 * HBM_BYTES
    assert len(pl["slot_of_step"]) == W + K
    for s, y in enumerate(pl["years"]):
        assert y == 1901 + s
        slot = pl["slot_of_step"][s]
        assert 0 <= slot < pl["nslots"]
        assert synth.days_in_year(pl["slot_year"][slot]) == synth.days_in_year(y)
    if W + K <= pl["nslots"]:
        assert pl["slot_of_step"] == list(range(W + K))     # every year its own forcing


def test_driver_default_invocation_config2():
    """The driver runs `bench.py --gpus 1 --steps 20 --warmup 5` (round 1 crashed
    on it: nslots = 25 > 8)."""
    pl = bench.plan("config2", 5, 20)
    assert pl["nslots"] == 25 and pl["gid"].size == synth.NLAND05
    h.make_config(pl["gid"].size, pl["zi"], nlayers=8, nisurf=48, grow_on=False, nslots=25)


def test_config4_spinup_is_thirty_distinct_years():
    wl = bench.WORKLOADS["config4"]
    pl = bench.plan("config4", wl["warmup"], wl["steps"])
    assert pl["years"][0] == 1901 and pl["years"][-1] == 1930
    assert pl["nslots"] == 30 and pl["slot_year"] == pl["years"]
    assert pl["grow_on"] and pl["ns"] == 48 and pl["L"] == 8


def test_config_check_reasons():
    zi = synth.ZI_L8
    with pytest.raises(ValueError, match="nslots"):
        h.make_config(100, zi, nslots=h.MAX_SLOTS + 1)
    with pytest.raises(ValueError, match="nlayers"):
        h.make_config(100, np.arange(11, dtype=np.float32), nlayers=9)
    with pytest.raises(ValueError, match="zi"):
        h.make_config(100, zi[::-1].copy())
    with pytest.raises(ValueError, match="ncell"):
        h.make_config(0, zi)
    cfg = h.make_config(67420, zi, nslots=25)
    # 25 resident years of forcing dominate: 7 x 366 x 67,420 x 4 B each
    assert 25 * 7 * 366 * 67420 * 4 < h.config_bytes(cfg) < 1.01 * 25 * 7 * 366 * 67420 * 4 + 50e6


class StubCtx:
    """Stands in for h9g_ctx on CPU: run_year records the years, and
    diagnostics_async writes this rank's FP64 diagnostics into the buffer."""

    def __init__(self, rank):
        self.rank, self.years, self.ms = rank, [], 0.0

    def run_year(self, slot, y):
        self.years.append((slot, y))
        self.ms += 1.0

    def diag(self):
        y = self.years[-1][1]
        return np.arange(h.NDIAG, dtype=np.float64) * (self.rank + 1) + y

    def diagnostics_async(self, ptr, stream):
        assert stream is None
        d = self.diag()
        ctypes.memmove(ptr, d.ctypes.data, d.nbytes)

    def total_kernel_ms(self, reset=False):
        ms = self.ms
        if reset:
            self.ms = 0.0
        return ms


def _worker(rank, world, port_no, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port_no)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pl = bench.plan("config2", 2, 3, world=world, rank=rank)
    ctx = StubCtx(rank)
    exchange, buf = bench.make_exchange(ctx, torch, dist, world, "cpu")
    elapsed = bench.timed_steps(ctx, pl, exchange, lambda: dist.barrier())
    q.put((rank, ctx.years, buf.numpy().copy(), elapsed, pl["seed"], pl["n_total"]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_world2_gloo_bench_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port_no = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port_no, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    last = 1901 + 4
    want = sum(np.arange(h.NDIAG, dtype=np.float64) * (r + 1) + last for r in range(2))
    for rank, years, buf, elapsed, seed, n_total in res:
        assert years == [(s, 1901 + s) for s in range(5)]
        np.testing.assert_array_equal(buf, want)        # all-reduced sum of both ranks
        assert seed == synth.SEED + rank                 # weak scaling: a grid per rank
        assert n_total == 2 * synth.NLAND05
        assert elapsed >= 0
