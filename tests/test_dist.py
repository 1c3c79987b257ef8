"""Multi-GPU path on CPU: world_size 2 over gloo.  Cells are sharded in
contiguous ranges (hybrid9_amd.shard), each rank advances its shard
(here with the CPU oracle, standing in for its GPU), and the per-year FP64
diagnostics are all-reduced -- the only collective of the path.  The
reduced diagnostics must equal those of one process over all cells, and
the concatenated shard outputs must equal the unsharded run bit-for-bit."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hybrid9_amd import shard, synth
from oracle import port


def _inputs():
    g = synth.land_cells()[::211][:96]
    p = synth.make_params(g)
    f = synth.make_forcing(g, synth.cell_lat(g), 0, 365)
    return g, p, f


def _worker(rank, world, port_no, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port_no)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g, p, f = _inputs()
    sl = shard.shard_slice(g.size, rank, world)
    out = port.run(zi=synth.ZI_L8, params={k: v[sl] for k, v in p.items()},
                   forcing=np.ascontiguousarray(f[:, :, sl]), nisurf=48, grow_on=0, nthreads=2)
    d = torch.from_numpy(shard.host_diagnostics(out["annual"][0], out["state"]))
    dist.all_reduce(d)
    gathered = [None] * world
    dist.all_gather_object(gathered, out["annual"])
    if rank == 0:
        q.put((d.numpy(), np.concatenate(gathered, axis=2)))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_slices_cover_exactly():
    for n in (1, 7, 67420):
        for w in (1, 2, 3, 8):
            idx = np.concatenate([np.arange(n)[shard.shard_slice(n, r, w)] for r in range(w)])
            assert np.array_equal(idx, np.arange(n))
            sizes = [shard.shard_slice(n, r, w).stop - shard.shard_slice(n, r, w).start
                     for r in range(w)]
            assert max(sizes) - min(sizes) <= 1


def test_world2_gloo_allreduce_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port_no = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port_no, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    d2, ann2 = q.get(timeout=600)
    for pr in procs:
        pr.join(timeout=600)
        assert pr.exitcode == 0
    g, p, f = _inputs()
    one = port.run(zi=synth.ZI_L8, params=p, forcing=f, nisurf=48, grow_on=0, nthreads=4)
    d1 = shard.host_diagnostics(one["annual"][0], one["state"])
    np.testing.assert_allclose(d2, d1, rtol=1e-13)
    assert d2[0] == g.size
    assert np.array_equal(ann2, one["annual"])


# --------------------------------------------------------------------------
# the reference's own cell order over two ranks
# --------------------------------------------------------------------------
CO_YEARS = 10        # the golden's first decade: the rank split shows there already


def _co_worker(rank, world, port_no, q):
    """Rank `rank` takes whole reference blocks of co_c1_blocks4
    (shard.blocks_of_rank: block b to rank b mod world), each block one chain
    (h9g_set_chains' semantics), and runs them in the reference's order on
    the C oracle standing in for its GPU; rank 0 gathers the cells."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port_no)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests.conftest import load_golden
    meta, inp, _ = load_golden("co_c1_blocks4")
    blocks = np.asarray(meta["rank"])
    mine = shard.blocks_of_rank(blocks, rank, world)
    nd = sum(synth.days_in_year(1901 + k) for k in range(CO_YEARS))
    out = port.run_cell_order(zi=inp["zi"], params={k: v[mine] for k, v in inp["params"].items()},
                              forcing=np.ascontiguousarray(inp["forcing"][:, :nd, mine]), nisurf=inp["nisurf"],
                              year0=inp["year0"], nyears=CO_YEARS, grow_on=inp["grow_on"], chains=blocks[mine])
    gathered = [None] * world
    dist.all_gather_object(gathered, (mine, out["annual"], out["rc"]))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gloo_cell_order_blocks_match_reference():
    """Two ranks, each with two of the reference's four MPI blocks: the union
    of their outputs is the reference's 4-process run (golden co_c1_blocks4)
    bit for bit, with no collective between the chains."""
    from tests.conftest import load_golden, same_bits
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port_no = _free_port()
    procs = [ctx.Process(target=_co_worker, args=(r, 2, port_no, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=600)
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    meta, _, exp = load_golden("co_c1_blocks4")
    ann = np.full((CO_YEARS,) + exp["annual"].shape[1:], np.nan, np.float32)
    seen = np.zeros(meta["ncell"], int)
    for mine, a, rc in gathered:
        assert rc == 0
        ann[:, :, mine] = a
        seen[mine] += 1
    assert (seen == 1).all()                      # every cell on exactly one rank
    assert same_bits(ann, exp["annual"][:CO_YEARS])


def test_blocks_of_rank_partition():
    b = np.array([-1, 0, 1, 2, 3, 3, 2, 1, 0, -1, 4])
    got = [shard.blocks_of_rank(b, r, 3) for r in range(3)]
    assert np.array_equal(np.sort(np.concatenate(got)), np.where(b >= 0)[0])
    assert all(len(set(b[g] % 3)) == 1 for g in got)
