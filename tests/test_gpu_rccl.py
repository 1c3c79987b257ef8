"""The multi-GPU hand-off on one MI355X: bench.py's per-year exchange
(h9g_get_diagnostics_async on torch's current stream, then an RCCL
all-reduce, torch.distributed "nccl") at world size 1, pipelined exactly as
the bench runs it -- no host synchronisation between years, the next
year's kernel queued while the all-reduce runs.  Every year's reduced
buffer must equal that year's diagnostics from a synchronous re-run and
the FP64 host sum of the per-cell fields (the reference's ranks are
independent, INIT.f90:271-274; the all-reduce is this port's only
collective)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_diagnostics_exchange_world1():
    import torch
    import torch.distributed as dist

    import bench
    import hybrid9_amd as h
    from hybrid9_amd import shard, synth
    from oracle import refcase

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        W, K = 1, 3
        pl = bench.plan("config2", W, K)
        n = 8800                                         # 100 pair workgroups of the 0.5 deg grid
        gid, lat = pl["gid"][:n], pl["lat"][:n]
        ctx = h.Context(n, pl["zi"], nlayers=8, nisurf=48, grow_on=False, nslots=W + K, device=0)
        ctx.set_cells(gid, lat)
        ctx.synth_params(pl["seed"])
        for slot, y in enumerate(pl["slot_year"]):
            ctx.synth_forcing(slot, pl["seed"], synth.year_day0(y), synth.days_in_year(y))
        ctx.init_state()
        ctx.sync()
        exchange, buf = bench.diag_exchange(ctx, torch, dist, "cuda:0")
        stream = torch.cuda.current_stream()
        snaps = []
        for s in range(W + K):                           # pipelined, as bench.timed_steps
            ctx.run_year(pl["slot_of_step"][s], pl["years"][s])
            exchange()
            snaps.append(buf.clone())                    # on torch's stream, after the all-reduce
        stream.synchronize()
        ctx.sync()
        got = [t.cpu().numpy() for t in snaps]
        # the same years again, synchronously
        ctx.init_state()
        for s in range(W + K):
            ctx.run_year(pl["slot_of_step"][s], pl["years"][s])
            ctx.sync()
            want = ctx.get_diagnostics()
            st = refcase.unpack_state(ctx.get_state(), n, 8)
            hd = shard.host_diagnostics(ctx.get_annual(), st)
            assert want[0] == n and want[11] == 0
            np.testing.assert_array_equal(got[s], want)
            np.testing.assert_allclose(got[s], hd, rtol=1e-12, atol=0)
        assert len({float(g[1]) for g in got}) == W + K  # distinct years, not one buffer read K times
        ctx.close()
    finally:
        dist.destroy_process_group()
