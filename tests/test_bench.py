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
    # 25 resident years of forcing dominate: 7 x 366 x 67,420 x 4 B each, plus
    # the slot-ordered copy of one year with room for a second group of cells
    # (h9g_perm_forcing_kernel, twice the cells) and the cell order's buffers
    # for two decades in flight (h9g_run_ordered: start state, checkpoints and
    # annual means of 10 years each, and the day-1 probe's rows: ~6.4 KB per cell)
    fixed = 27 * 7 * 366 * 67420 * 4
    assert fixed + 2 * 10 * (41 + 20) * 4 * 67420 < h.config_bytes(cfg) < 1.01 * fixed + 60e6 + 6.5e3 * 67420


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


class StubOrderedCtx(StubCtx):
    """The cell order's calls (bench.ordered_years): run_ordered records the
    years of each call; the stats are those of an empty call."""

    def run_ordered(self, slots, year0, raise_on_stop=True, annual=True):
        for k, s in enumerate(slots):
            self.years.append((s, year0 + k))
        self.ms += len(slots)
        return None, [1] * len(h.decades(year0, len(slots)))

    def decade_stats(self):
        return dict(passes=1, rerun_cells=0, rerun_cell_years=0, rerun_launches=0, launch_cells=[])

    def ordered_stats(self):
        return dict(decades=1, passes=[1])

    def launch_stats(self, reset=False):
        return {}


def _worker_cell(rank, world, port_no, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port_no)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, K = bench.decade_aligned(5, 20)
    pl = bench.plan("config2", W, K, world=world, rank=rank)
    ctx = StubOrderedCtx(rank)
    exchange, buf = bench.make_exchange(ctx, torch, dist, world, "cpu")
    work = []
    elapsed = bench.timed_steps(ctx, pl, exchange, lambda: dist.barrier(), "cell", work)
    q.put((rank, ctx.years, buf.numpy().copy(), elapsed, len(work), W, K))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gloo_bench_cell_order():
    """The driver's command at world size 2 in the default (cell) order:
    the warm-up rounded to whole decades (1901-1910 untimed), then 1911-1930
    as one h9g_run_ordered call per rank between two barriers, and the
    diagnostics all-reduced after each call."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port_no = _free_port()
    procs = [ctx.Process(target=_worker_cell, args=(r, 2, port_no, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0
    want = sum(np.arange(h.NDIAG, dtype=np.float64) * (r + 1) + 1930 for r in range(2))
    for rank, years, buf, elapsed, ncalls, W, K in res:
        assert (W, K) == (10, 20)
        assert [y for _, y in years] == list(range(1901, 1931))
        assert ncalls == 1                               # the timed call's stats only
        np.testing.assert_array_equal(buf, want)
        assert elapsed >= 0
    with pytest.raises(SystemExit):
        bench.decade_aligned(5, 15)                      # a cut decade is refused


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


def _pmc(root, tag, build, workload="config2", kernel="void h9g_pair_kernel<8, h9k::GeoC<8, 48> >(KArgs, h9k::GeoC<8, 48>)"):
    import json
    (root / "profiles").mkdir(exist_ok=True)
    (root / "profiles" / f"pmc_{tag}.json").write_text(json.dumps(
        {"tag": tag, "workload": workload, "kernel": kernel, "build_id": build,
         "kernel_stats": f"profiles/{tag}_kernel_stats.csv", "hbm_bytes_per_launch": 1e9,
         "kernel_avg_ns_rocprof": 2e8, "counters_per_launch": {"SQ_INSTS_VALU": 1e11}}))


def test_counters_attach_only_to_their_build(tmp_path):
    """load_traffic attaches a summary of the workload and kernel only if it
    was measured on this build (the r02f line cited the r02e
    counters), the latest such, whatever later tags of other builds exist."""
    k = "h9g_pair_kernel<8,GeoC<8,48>>"
    assert bench.load_traffic("config2", k, "aaaa", root=tmp_path) == (None, None)
    _pmc(tmp_path, "r03a", "aaaa")
    _pmc(tmp_path, "r03b", "bbbb")
    _pmc(tmp_path, "r03c", "aaaa", workload="config3")
    pmc, stale = bench.load_traffic("config2", k, "bbbb", root=tmp_path)
    assert stale is None and pmc["tag"] == "r03b"
    # build aaaa gets its own r03a counters, though r03b is later
    pmc, stale = bench.load_traffic("config2", k, "aaaa", root=tmp_path)
    assert stale is None and pmc["tag"] == "r03a"
    # a build with no summary gets none, and the latest tag is reported
    assert bench.load_traffic("config2", k, "cccc", root=tmp_path) == (None, "r03b")
    assert bench.load_traffic("config2", k, None, root=tmp_path) == (None, "r03b")
    assert bench.load_traffic("config3", k, "aaaa", root=tmp_path)[0]["tag"] == "r03c"
    assert bench.load_traffic("config2", "h9g_solo_kernel<8,GeoC<8,48>>", "bbbb", root=tmp_path) == (None, None)
    assert bench.valu_roofline(None, 0.2) is None


def test_build_id_is_the_source_digest():
    """The loaded library reports the digest of the sources and flags it was
    built from (a stale .so would report another id)."""
    from hybrid9_amd import build as hb
    bid = h.build_id()
    assert len(bid) == 16 and int(bid, 16) >= 0
    assert bid == hb.build_id()
    assert hb.build_id(["-DX"]) != bid


def test_pmc_summary_requires_one_build(tmp_path, monkeypatch):
    """tools/pmc_summary.py refuses a profile whose passes ran different
    builds, and records the build of one that did not."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location("pmc_summary", bench.ROOT / "tools" / "pmc_summary.py")
    ps = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ps)
    d = tmp_path / "gpurun_out" / "prof_t1"
    (d / "kt").mkdir(parents=True)
    line = lambda b: json.dumps({"metric": "m", "roofline": {"build_id": b}})
    (d / "kt.log").write_text("x\n" + line("aaaa") + "\n")
    (d / "sq1.log").write_text(line("bbbb") + "\n")
    monkeypatch.setattr(ps, "ROOT", tmp_path)
    with pytest.raises(SystemExit, match="different or unknown builds"):
        ps.main("t1")
    (d / "sq1.log").write_text(line("aaaa") + "\n")
    name = "void h9g_pair_kernel<8, h9k::GeoC<8, 48> >(KArgs, h9k::GeoC<8, 48>)"
    (d / "kt" / "kt_kernel_stats.csv").write_text(
        "Name,Calls,TotalDurationNs,AverageNs\n\"%s\",3,600000000,200000000\n" % name)
    (d / "sq1").mkdir()
    (d / "sq1" / "x_counter_collection.csv").write_text(
        "Kernel_Name,Counter_Name,Counter_Value\n\"%s\",SQ_INSTS_VALU,100\n\"%s\",SQ_WAVES,2\n" % (name, name))
    (tmp_path / "profiles").mkdir()
    ps.main("t1")
    out = json.loads((tmp_path / "profiles" / "pmc_t1.json").read_text())
    assert out["build_id"] == "aaaa" and out["kernel_stats"] == "profiles/t1_kernel_stats.csv"
    assert out["counters_per_launch"]["SQ_INSTS_VALU"] == 100
