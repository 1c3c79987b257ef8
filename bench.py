#!/usr/bin/env python3
"""HYBRID9 hot-path benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload config2]

A *step* is one simulated calendar year for every land cell of the GPU:
365/366 days x NISURF substeps of HYDROLOGY (+ daily GROW when enabled).
By default (``--order cell``, round 6) the years run in the reference's own
order -- decade -> cell -> year, smp carried from cell to cell
(HYBRID9.f90:93-130), bit-identical to the reference -- as one
``h9g_run_ordered`` call over whole reference decades: the untimed warm-up
is rounded up to whole decades (``--warmup 5`` runs 1901-1910) and the
timed years must be whole decades (``--steps 20``: 1911-1930).
``--order isolated`` times ``h9g_run_year`` launches (every cell its own
smp, the contract of rounds 1-5; it misses the reference by up to 4e-2,
DESIGN.md §2); the default run reports it under ``isolated``.  The FP64
diagnostics are all-reduced across GPUs over RCCL (torch.distributed
"nccl") after each call (cell order) or year (isolated).
Inputs (soil parameters, a distinct forcing year per step) are generated on
the device and resident in HBM before the timed region.  Weak scaling (the
default): each rank simulates the full synthetic land grid with its own seed;
``--strong`` shards one fixed grid over the ranks instead.
Rank 0 prints one JSON line.

``value`` = cell-steps/s over all ranks (cells x days x NISURF x K / max
rank time; re-runs of the cell order are overhead, not counted).
``roofline.achieved`` = the SURVEY.md §8d algorithmic bytes of the
per-substep SHARED-state contract (4(10L+14) B/cell-step) per launch of the
dominant kernel (the pair kernel: the cell order's year launches and their
riding re-runs, and its year-1 re-runs) / the launch's device time from HIP
events on the kernel's stream.
``cpu_baseline`` times the reference itself (oracle/_ref/h9ref: unmodified
HYDROLOGY.f90 compiled with amdflang) on a bounded sample of the same
workload, one process per host core, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "grid-cell-steps/sec at 0.5° global (1/2/4/8 GPUs) + achieved HBM GB/s"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak: 1024 SIMDs x 2.4 GHz; a SIMD-32 takes a wave64 f32/i32
# VALU instruction every 2 cycles when >= 2 waves interleave (one wave alone:
# every 4), MI355X_MICROARCH.md constants table.  f64 arithmetic runs at half
# that rate (78.6 vs 157.3 TF/s vector peak) and transcendentals at a
# quarter, so a kernel's issue floor depends on its instruction mix:
# VALU_CYCLES gives the SIMD cycles per wave64 instruction of each
# rocprofv3 SQ_INSTS_VALU_* class; the rest of SQ_INSTS_VALU costs 2.
VALU_PEAK_GIPS = 1024 * 2.4 / 2
SIMD_HZ = 1024 * 2.4e9
VALU_CYCLES = {"SQ_INSTS_VALU_ADD_F64": 4, "SQ_INSTS_VALU_MUL_F64": 4, "SQ_INSTS_VALU_FMA_F64": 4,
               "SQ_INSTS_VALU_TRANS_F64": 8, "SQ_INSTS_VALU_TRANS_F32": 4, "SQ_INSTS_VALU_INT64": 4}

WORKLOADS = {
    # BASELINE.json configs[1]: the metric's config (fits one GPU)
    "config2": dict(desc="0.5deg global synthetic land, 67,420 cells/GPU, daily forcing, "
                         "NISURF=48, hydrology-only (GROW off), L=8",
                    grid="05", nlayers=8, nisurf=48, grow_on=False),
    "config3": dict(desc="0.5deg global synthetic land, 67,420 cells/GPU, NISURF=24, "
                         "HYDROLOGY+GROW coupled, L=8",
                    grid="05", nlayers=8, nisurf=24, grow_on=True),
    # BASELINE.json configs[3]: the 30-year spin-up 1901-1930, state carried
    # from year to year as HYBRID9.f90:93-130 carries it across its decade
    # loop; every year's forcing is distinct and resident (30 x 691 MB).
    # Default run: no warmup, the 30 years timed (`--steps` / `--warmup`
    # override).  Weak scaling: 67,420 cells per GPU.
    "config4": dict(desc="0.5deg global synthetic land, 67,420 cells/GPU, 30-year spin-up "
                         "1901-1930, NISURF=48, HYDROLOGY+GROW, L=8",
                    grid="05", nlayers=8, nisurf=48, grow_on=True, steps=30, warmup=0),
    "config5": dict(desc="0.25deg global synthetic land, 270,000 cells, 10 layers, NISURF=24, "
                         "GROW on",
                    grid="025", nlayers=10, nisurf=24, grow_on=True),
}
RING_MAX = 32                   # resident forcing years (a multiple of 4: leap-year period)
SLOT_BUDGET = 120e9             # bytes of HBM the resident forcing years may take


def bytes_per_cell_step(L: int) -> int:
    """reads 8 per-layer arrays + 5 scalars + 7 forcing,
    writes 2 per-layer arrays + 2 scalars -> 4 (10 L + 14) bytes."""
    return 4 * (10 * L + 14)


def dist_setup(n_gpus: int):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}; launch N>1 with torchrun")
    torch = dist = None
    try:
        import torch  # noqa: F811
        import torch.distributed as dist  # noqa: F811
    except Exception:                        # torch is plumbing only
        if world > 1:
            raise
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")      # RCCL over xGMI on ROCm
    return rank, world, local, torch, dist


def barrier_sync(ctx, torch, dist, world):
    # a cell reaching one of the reference's STOPs (synthetic L=10 cells can)
    # is marked failed and NaN, as the error record says; the others go on
    ctx.sync(raise_on_stop=False)
    if torch is not None and torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()


def cpu_baseline(workload: dict, seed: int) -> dict:
    """The reference (oracle/_ref/h9ref, or h9ref_l10 for 10 layers) on a
    bounded sample of the same workload: P processes x C cells x 1 year,
    like `mpirun -np P` without MPI (the reference's ranks never
    communicate during compute)."""
    from hybrid9_amd import synth
    from oracle import refcase

    P = int(os.environ.get("H9_CPU_PROCS", os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    P = max(1, min(P, os.cpu_count() or 1, 64))
    L, ns, grow = workload["nlayers"], workload["nisurf"], int(workload["grow_on"])
    C = int(os.environ.get("H9_CPU_CELLS", "2048" if L == 8 else "1024"))
    ref_bin = refcase.ref_bin(L)
    kind = "reference" if ref_bin.exists() else "port"
    if workload["grid"] == "05":
        land, zi, lat_of = synth.land_cells(), synth.ZI_L8, (lambda g: synth.cell_lat(g))
    else:
        land = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
        zi, lat_of = synth.ZI_L10, (lambda g: synth.cell_lat(g, synth.NX025, synth.NY025))
    assert zi.size == L + 2
    nt = synth.days_in_year(1901)
    tmp = Path(tempfile.mkdtemp(prefix="h9cpu_"))
    dirs = []
    for i in range(P):
        g = land[(i * 7919) % (land.size - C):][:C]
        p = synth.make_params(g, L, seed)
        f = synth.make_forcing(g, lat_of(g), 0, nt, seed)
        d = tmp / f"p{i}"
        if kind == "reference":
            refcase.write_case(d, zi=zi, params=p, forcing=f, nisurf=ns, grow_on=grow)
        dirs.append((d, p, f))
    t0 = time.perf_counter()
    if kind == "reference":
        procs = [subprocess.Popen([str(ref_bin), str(d)], stdout=subprocess.PIPE,
                                  stderr=subprocess.STDOUT) for d, _, _ in dirs]
        outs = [pr.communicate()[0].decode() for pr in procs]
        wall = time.perf_counter() - t0
        ok = all(pr.returncode == 0 and "STOP" not in o for pr, o in zip(procs, outs))
    else:
        from oracle import port
        for d, p, f in dirs[:1]:
            port.run(zi=zi, params=p, forcing=f, nisurf=ns, grow_on=grow, nthreads=1)
        wall = time.perf_counter() - t0
        P = 1
        ok = True
    steps = P * C * nt * ns
    subprocess.run(["rm", "-rf", str(tmp)])
    return {"value": steps / wall, "unit": "cell-steps/s", "cores": P, "kind": kind, "host": host_cpu(),
            "sample": f"{'reference HYDROLOGY.f90 (amdflang -O2)' if kind == 'reference' else 'C port'}"
                      f"{'' if L == 8 else ' rebuilt with nsoil_layers_max=10'}"
                      f" x {P} processes x {C} cells x 1 yr ({ns} substeps/day, GROW "
                      f"{'on' if grow else 'off'}, L={L}) = {steps:.3e} cell-steps in {wall:.1f} s"
                      f"{'' if ok else ' (a sample process STOPped)'}"}


def host_cpu() -> dict:
    """The box's host CPU as this process sees it: os.cpu_count(), the
    affinity mask's size (the lease) and the model (/proc/cpuinfo)."""
    model = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"cpu_count": os.cpu_count(), "usable": usable, "model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def load_traffic(workload_name: str, kernel: str, build: str | None = None, root: Path = ROOT):
    """The PMC summary (profiles/pmc_<tag>.json, tools/prof.sh +
    tools/pmc_summary.py) of this workload and kernel instantiation measured
    on this build (the loaded library's h9g_build_id; the latest such tag).
    Returns (summary, None), or (None, stale_tag) with the latest tag of any
    build when none matches -- counters of another build are never attached
    to this run's timing."""
    def norm(k):
        k = k.replace("void ", "").replace("h9k::", "").replace(" ", "")
        return k.split("(")[0]
    latest = match = None
    for p in sorted((root / "profiles").glob("pmc_*.json")):     # tags sort by round/version
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get("workload") == workload_name and norm(d.get("kernel", "")) == norm(kernel):
            latest = d
            if build is not None and d.get("build_id") == build:
                match = d
    if match is not None:
        return match, None
    return None, (latest.get("tag") if latest is not None else None)


def valu_roofline(pmc, launch_s: float):
    """The kernel's real bound, VALU issue, from the
    rocprofv3 SQ counters of the same kernel and workload: `achieved` wave
    instructions per second against the 2-cycle issue peak, and `floor_ms`
    = the launch time if every SIMD issued the measured instruction mix at
    its class costs (VALU_CYCLES) back to back; frac_of_mix = floor / time."""
    cnt = (pmc or {}).get("counters_per_launch") or {}
    n_valu = cnt.get("SQ_INSTS_VALU")
    if not n_valu:
        return None
    out = {"achieved": n_valu / launch_s / 1e9, "peak": VALU_PEAK_GIPS,
           "unit": "G wave-VALU-instructions/s", "frac": n_valu / launch_s / 1e9 / VALU_PEAK_GIPS,
           "insts_per_launch": n_valu,
           "source": "rocprofv3 --pmc SQ_INSTS_VALU*, profiles/pmc_%s.json" % pmc.get("tag")}
    if all(k in cnt for k in VALU_CYCLES):
        typed = sum(cnt[k] for k in VALU_CYCLES)
        cyc = sum(cnt[k] * c for k, c in VALU_CYCLES.items()) + 2 * (n_valu - typed)
        out["mix_cycles_per_launch"] = cyc
        out["floor_ms"] = cyc / SIMD_HZ * 1e3
        out["frac_of_mix"] = cyc / SIMD_HZ / launch_s
        out["mix"] = {k: cnt[k] for k in VALU_CYCLES}
    return out


class HostFed:
    """--host-fed: the PCIe-inclusive variant of the step.  The device-made
    synthetic forcing years are copied once to pinned host memory; in the
    timed loop each step pushes its year with h9g_push_forcing (async copy
    stream, READ_PGF's slab) into one of two slots, the next year's copy
    overlapping the current kernel (ev_consumed orders slot reuse).  The
    first push of the timed region is not overlapped."""

    def __init__(self, ctx, h, ncell, years, W):
        import ctypes as C
        from hybrid9_amd import synth
        self.ctx, self.lib, self.C = ctx, h.lib(), C
        self.hip = C.CDLL("libamdhip64.so")
        self.years, self.W, self.ncell = years, W, ncell
        self.nday = [synth.days_in_year(y) for y in years]
        self.bufs, self.arrs = [], []
        max_days = 366
        for s, nd in enumerate(self.nday):
            nb = 7 * nd * ncell * 4
            ptr = self.lib.h9g_host_alloc(nb)
            if not ptr:
                raise RuntimeError("h9g_host_alloc failed")
            src = self.lib.h9g_forcing_slot(ctx._h, s)
            # slot layout (7, max_days, ncell) -> host (7, nd, ncell)
            rc = self.hip.hipMemcpy2D(C.c_void_p(ptr), C.c_size_t(nd * ncell * 4), C.c_void_p(src),
                                      C.c_size_t(max_days * ncell * 4), C.c_size_t(nd * ncell * 4),
                                      C.c_size_t(7), C.c_int(2))
            if rc != 0:
                raise RuntimeError(f"hipMemcpy2D D2H failed ({rc})")
            self.bufs.append(ptr)
            self.arrs.append(np.ctypeslib.as_array((C.c_float * (7 * nd * ncell)).from_address(ptr))
                             .reshape(7, nd, ncell))
        self.bytes = 0
        self.k = 0

    def step(self, s):
        """Step s of the run (year 1901 + s): its forcing, host year
        s % R (R = 4 or fewer source years, the leap-year period), goes to
        slot k % 2 (k-th call); the next step's year is pushed behind it."""
        R = len(self.arrs)
        slot = self.k % 2
        if self.k == 0 or self.k == self.W:       # first push of warmup / of the timed region
            self.ctx.push_forcing(slot, self.arrs[s % R], async_=True)
            self.bytes += self.arrs[s % R].nbytes
        if self.k + 1 != self.W:                   # prefetch the next year behind this kernel
            self.ctx.push_forcing(1 - slot, self.arrs[(s + 1) % R], async_=True)
            self.bytes += self.arrs[(s + 1) % R].nbytes
        self.k += 1
        return slot

    def describe(self):
        return {"forcing_bytes_per_year": int(self.arrs[-1].nbytes), "slots": 2,
                "copy": "h9g_push_forcing async, pinned host memory, copy stream overlapped with the kernel"}

    def close(self):
        self.arrs = []
        for p in self.bufs:
            self.lib.h9g_host_free(p)
        self.bufs = []


class NcFed:
    """--forcing nc4: the config-3 "async PGF prefetch" path from files.
    Synthetic PGF netCDF-4 files of one year (0.5 deg, per-day chunks,
    shuffle + deflate, tools/pgf_synth.py) are written before the timed
    region; every step reads its year's days from them with
    h9g_nc_forcing_prefetch (host thread pool: direct chunk reads, inflate,
    gather; then an async copy into the slot) into one of two slots, the next
    year's read overlapping the current kernel.  The first read of the timed
    region is not overlapped.  Every year reads the same file year (its
    days 0..nday-1), so only year 1 matches the device-generated run."""

    def __init__(self, ctx, W, directory, gid):
        sys.path.insert(0, str(ROOT / "tools"))
        import pgf_synth
        import hybrid9_amd as h
        self.ctx, self.W = ctx, W
        t = time.perf_counter()
        self.paths = pgf_synth.write_year(directory, 1901, 366)
        self.write_s = time.perf_counter() - t
        self.bytes = sum(os.path.getsize(p) for p in self.paths)
        self.k = 0
        self.nx, self.ny = 720, 360
        # a synchronous read of one year, for the ingest rate alone
        t = time.perf_counter()
        h.nc_forcing_read(self.paths, self.nx, self.ny, np.asarray(gid, np.int64), 0, 365)
        self.read_s = time.perf_counter() - t
        self.read_stages = h.nc_read_stats()           # h9g_nc_read_stats of that read

    def step(self, s):
        from hybrid9_amd import synth
        y, slot = 1901 + s, self.k % 2
        nd = synth.days_in_year(y)
        if self.k == 0 or self.k == self.W:
            self.ctx.nc_prefetch(slot, self.paths, self.nx, self.ny, 0, nd)
        self.ctx.run_year(slot, y)                       # joins this slot's read first
        if self.k + 1 != self.W:
            self.ctx.nc_prefetch(1 - slot, self.paths, self.nx, self.ny, 0, synth.days_in_year(y + 1))
        self.k += 1

    def describe(self):
        import hybrid9_amd as h
        return {"source": "synthetic PGF v2.1 netCDF-4 files (one chunk per day, shuffle + deflate 4)",
                "file_bytes_per_year": int(self.bytes), "write_s": self.write_s,
                "read_s_per_year_sync": self.read_s, "read_stages": self.read_stages,
                "io_threads": self.read_stages.get("threads"), "host": host_cpu(),
                "slots": 2, "reader": "h9g_nc_forcing_prefetch (direct chunk reads, libdeflate, host pool)"}


def plan(workload: str, W: int, K: int, world: int = 1, rank: int = 0, strong: bool = False,
         seed: int | None = None) -> dict:
    """Everything a rank's run is made of, decided on the host (no GPU):
    its cells, the years of the W + K steps and the forcing ring.

    Step s simulates calendar year 1901 + s.  Its forcing sits in slot
    s % R of a ring of R = min(W + K, RING_MAX, HBM budget) resident
    years, generated before the timed region; with R a multiple of 4 (or
    every step its own slot) each slot's year has the same length as every
    year that reuses it.  When W + K > R a later year re-reads the synthetic
    forcing of the year R earlier (its state is different, so the work is
    not repeated)."""
    from hybrid9_amd import synth
    wl = WORKLOADS[workload]
    L, ns = wl["nlayers"], wl["nisurf"]
    if wl["grid"] == "05":
        gid = synth.land_cells()
        lat = synth.cell_lat(gid)
        zi = synth.ZI_L8
    else:
        gid = synth.land_cells(synth.NX025, synth.NY025, synth.NLAND025)
        lat = synth.cell_lat(gid, synth.NX025, synth.NY025)
        zi = synth.ZI_L10
    n_total = gid.size
    base = seed if seed is not None else synth.SEED
    if strong:
        # strong scaling: one fixed grid, contiguous balanced
        # shards of the land-cell list; parameters and forcing are keyed by
        # the global cell id, so the shards are exactly the unsharded cells
        from hybrid9_amd.shard import shard_slice
        sl = shard_slice(gid.size, rank, world)
        gid, lat = gid[sl], lat[sl]
        rseed = base
    else:
        rseed = base + rank                       # weak scaling
        n_total = world * gid.size
    nsteps = W + K
    if nsteps < 1:
        raise ValueError("--steps + --warmup must be >= 1")
    slot_bytes = 7 * 366 * gid.size * 4
    cap = max(4, min(RING_MAX, int(SLOT_BUDGET // slot_bytes)) // 4 * 4)
    R = nsteps if nsteps <= cap else cap
    years = [1901 + s for s in range(nsteps)]
    slot_year = years[:R]
    slot_of_step = [s % R for s in range(nsteps)]
    for s, y in enumerate(years):
        assert synth.days_in_year(slot_year[slot_of_step[s]]) == synth.days_in_year(y), (s, y)
    return dict(workload=workload, wl=wl, L=L, ns=ns, grow_on=wl["grow_on"], zi=zi, gid=gid, lat=lat,
                seed=rseed, n_total=n_total, years=years, nslots=R, slot_year=slot_year,
                slot_of_step=slot_of_step, W=W, K=K)


def make_exchange(ctx, torch, dist, world: int, device: str):
    """The per-year cross-GPU step: this rank's FP64 diagnostics into a
    device buffer, stream-ordered behind the year kernel with no host
    synchronisation (h9g_get_diagnostics_async), then all-reduced (RCCL
    over xGMI; gloo on CPU in the tests).  Returns (exchange, buffer)."""
    if world <= 1:
        return None, None
    return diag_exchange(ctx, torch, dist, device)


def diag_exchange(ctx, torch, dist, device: str):
    """make_exchange's step for any world size (tests run it at world size 1
    over RCCL on one GPU)."""
    import hybrid9_amd as h
    buf = torch.zeros(h.NDIAG, dtype=torch.float64, device=device)
    on_gpu = device.startswith("cuda")

    def exchange():
        stream = torch.cuda.current_stream().cuda_stream if on_gpu else None
        ctx.diagnostics_async(buf.data_ptr(), stream)
        dist.all_reduce(buf)
    return exchange, buf


def ordered_years(ctx, pl: dict, s0: int, s1: int, exchange, work: list) -> None:
    """Steps s0 .. s1-1, whole reference decades (HYBRID9.f90:93-130), as
    one h9g_run_ordered call: the decades overlap on the device and every
    year's forcing stays resident."""
    if s1 <= s0:
        return
    ctx.run_ordered([pl["slot_of_step"][k] for k in range(s0, s1)], pl["years"][s0], raise_on_stop=False,
                    annual=False)
    work.append(dict(ctx.decade_stats(), overlap=ctx.ordered_stats(), years=s1 - s0))
    if exchange:
        exchange()


def decade_aligned(W: int, K: int) -> tuple[int, int]:
    """The cell order's warm-up and timed years: the warm-up rounded up to
    whole decades from 1901; the timed years must be whole decades, since a
    cut decade is not the reference's order (a cell's successor would start
    from its smp in the middle of the decade)."""
    if K < 10 or K % 10:
        raise SystemExit(f"--order cell times whole reference decades: --steps {K} is not a multiple of 10 "
                         "(use --order isolated for other counts)")
    return (W + 9) // 10 * 10, K


def isolated_line(ctx, pl: dict, ns: int, sync, W: int = 5, K: int = 20) -> dict:
    """The isolated-cell contract (h9g_run_year: every cell its own smp,
    rounds 1-5's `value`) on the same cells after the main measurement: the
    state re-initialised, W years untimed, K timed.  Secondary: it misses
    the reference's order by up to 4e-2."""
    from hybrid9_amd import synth
    ctx.init_state()
    W, K = min(W, len(pl["years"]) - 1), min(K, len(pl["years"]))
    W = min(W, len(pl["years"]) - K)
    sub = dict(pl, W=W, K=K, years=pl["years"][:W + K], slot_of_step=pl["slot_of_step"][:W + K])
    ctx.launch_stats(reset=True)
    el = timed_steps(ctx, sub, None, sync, "isolated")
    kern_ms = ctx.total_kernel_ms(reset=True)
    d = ctx.get_diagnostics()
    failed = int(round(float(d[11])))
    steps = sum(synth.days_in_year(y) for y in sub["years"][W:]) * ns
    n = pl["gid"].size
    algo = (n - failed) * steps / K * bytes_per_cell_step(pl["L"])
    return {"value": (n - failed) * steps / el, "unit": "cell-steps/s",
            "years": f"{sub['years'][W]}-{sub['years'][-1]} timed ({W} untimed)",
            "ms_per_step": el / K * 1e3, "kernel_ms_per_launch": kern_ms / K,
            "roofline_frac": algo / (kern_ms / K / 1e3) / 1e9 / HBM_PEAK_GBS,
            "semantics": "isolated cells (h9g_run_year, every cell its own smp): not the reference's order, "
                         "up to 4e-2 relative from it (DESIGN.md §2)"}


def timed_steps(ctx, pl: dict, exchange, sync, order: str = "isolated", work: list | None = None) -> float:
    """W untimed warmup years, then K timed years between two `sync`s
    (barrier + device synchronisation).  Returns the elapsed seconds.
    order "cell": the W and K years each as one h9g_run_ordered call
    (ordered_years; `work` collects each call's stats); both whole decades."""
    W, K = pl["W"], pl["K"]
    if order == "cell":
        work = [] if work is None else work
        ordered_years(ctx, pl, 0, W, exchange, [])
        sync()
        ctx.total_kernel_ms(reset=True)
        if hasattr(ctx, "launch_stats"):
            ctx.launch_stats(reset=True)
        t0 = time.perf_counter()
        ordered_years(ctx, pl, W, W + K, exchange, work)
        sync()
        return time.perf_counter() - t0
    for s in range(W):
        ctx.run_year(pl["slot_of_step"][s], pl["years"][s])
        if exchange:
            exchange()
    sync()
    ctx.total_kernel_ms(reset=True)
    t0 = time.perf_counter()
    for s in range(W, W + K):
        ctx.run_year(pl["slot_of_step"][s], pl["years"][s])
        if exchange:
            exchange()
    sync()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed years (cell order: whole decades, default 20; isolated: default 3; config4: 30)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed years (cell order: rounded up to whole decades, default 10; isolated: default "
                         "1; config4: 0)")
    ap.add_argument("--workload", default="config2", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: shard one fixed grid over the ranks (default: weak, "
                         "a full grid per rank with seed + rank)")
    ap.add_argument("--host-fed", action="store_true",
                    help="PCIe-inclusive rate: every step's forcing year is copied from pinned host "
                         "memory (async, double-buffered; isolated order); reported in DESIGN.md, never as `value`")
    ap.add_argument("--order", choices=["isolated", "cell"], default=None,
                    help="cell (default): the reference's own cell order (h9g_run_ordered over whole decades, "
                         "smp carried from cell to cell, bit-identical to the reference); isolated: every cell "
                         "its own smp (h9g_run_year per year; the default with --host-fed / --forcing nc4)")
    ap.add_argument("--no-isolated-line", action="store_true",
                    help="skip the secondary measurement of the isolated-cell contract (the default cell-order "
                         "run at N=1 adds it: 1901-1905 untimed, 1906-1925 timed, reported under `isolated`, "
                         "never as `value`)")
    ap.add_argument("--forcing", choices=["device", "nc4"], default="device",
                    help="nc4: every step's forcing is read from synthetic PGF netCDF-4 files through "
                         "h9g_nc_forcing_prefetch (ingest-inclusive, isolated order; DESIGN.md, never as `value`)")
    args = ap.parse_args()
    if args.forcing == "nc4" and (args.host_fed or WORKLOADS[args.workload]["grid"] != "05"):
        raise SystemExit("--forcing nc4: 0.5 deg workloads only, not with --host-fed")
    streamed = args.host_fed or args.forcing != "device"
    if args.order is None:
        args.order = "isolated" if streamed else "cell"
    if args.order == "cell" and streamed:
        raise SystemExit("--order cell: resident device forcing only (every year of a call stays resident)")
    wl = WORKLOADS[args.workload]
    if args.order == "cell":
        K = args.steps if args.steps is not None else wl.get("steps", 20)
        W_req = args.warmup if args.warmup is not None else wl.get("warmup", 10)
        W, K = decade_aligned(W_req, K)
    else:
        K = args.steps if args.steps is not None else wl.get("steps", 3)
        W_req = W = args.warmup if args.warmup is not None else wl.get("warmup", 1)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launched without torchrun: start one rank per GPU as child processes
        # (no GPU has been touched in this process) and exit with their code
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
               f"--master-port={os.environ.get('MASTER_PORT', '29517')}", str(Path(__file__).resolve())]
        raise SystemExit(subprocess.call(cmd + sys.argv[1:]))

    rank, world, local, torch, dist = dist_setup(args.gpus)
    import hybrid9_amd as h
    from hybrid9_amd import synth

    pl = plan(args.workload, W, K, world, rank, args.strong, args.seed)
    L, ns, gid, lat = pl["L"], pl["ns"], pl["gid"], pl["lat"]
    n_total, seed, years = pl["n_total"], pl["seed"], pl["years"]
    host_fed = None
    nslots = pl["nslots"]
    if args.host_fed:
        nslots = max(2, min(4, W + K))            # 2 push slots + up to 4 source years
    if args.forcing == "nc4":
        nslots = 2
    ctx = h.Context(gid.size, pl["zi"], nlayers=L, nisurf=ns, grow_on=wl["grow_on"],
                    nslots=nslots, device=local if world > 1 else 0)
    ctx.set_cells(gid, lat)
    ctx.synth_params(seed)
    ctx.init_state()
    src_years = pl["slot_year"] if not args.host_fed else years[:nslots]
    nc_fed = None
    if args.forcing == "nc4":
        nc_fed = NcFed(ctx, W, tempfile.mkdtemp(prefix="h9pgf_"), gid)
        pl = dict(pl, slot_of_step=[None] * (W + K))
    else:
        for slot, y in enumerate(src_years):       # forcing resident in HBM
            ctx.synth_forcing(slot, seed, synth.year_day0(y), synth.days_in_year(y))
    ctx.sync()

    if args.host_fed:
        host_fed = HostFed(ctx, h, gid.size, src_years, W)
        pl = dict(pl, slot_of_step=[None] * (W + K))

    device = f"cuda:{local}" if world > 1 else "cpu"
    exchange, diag_t = make_exchange(ctx, torch, dist, world, device)

    class _Fed:                                      # --host-fed: push, then run
        def __init__(self, c):
            self.c = c

        def run_year(self, _slot, y):
            self.c.run_year(host_fed.step(y - 1901), y)

        def total_kernel_ms(self, reset=False):
            return self.c.total_kernel_ms(reset)

    class _NcFed(_Fed):                              # --forcing nc4: read, then run
        def run_year(self, _slot, y):
            nc_fed.step(y - 1901)

    def sync():
        barrier_sync(ctx, torch, dist, world)

    runner = _Fed(ctx) if host_fed else (_NcFed(ctx) if nc_fed else ctx)
    work = []
    elapsed = timed_steps(runner, pl, exchange, sync, args.order, work)
    kern_ms = ctx.total_kernel_ms(reset=True)
    launches = ctx.launch_stats(reset=True)
    # the dominant kernel's launches: in cell order the context's pair kernel
    # (every year launch of the first passes, with the re-runs riding in them,
    # and the year-1 re-runs); the one-column kernel of short re-run lists
    # is reported beside it
    kname = ctx.kernel_name()
    main_kind = {1: "pair", 2: "solo", 3: "mixed", 4: "pair2", 5: "pair11", 6: "pair1"}[ctx.kind_id()]
    if args.order == "cell" and main_kind in launches:
        ml = launches[main_kind]
        n_launch, launch_ms, cy_launch = ml["launches"], ml["ms"], ml["cell_years"] / max(1, ml["launches"])
    else:
        n_launch, launch_ms, cy_launch = K, kern_ms, None
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, launch_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, launch_ms = float(t[0]), float(t[1]), float(t[2])
        diag = diag_t.cpu().numpy()
    else:
        diag = ctx.get_diagnostics()

    # cells that hit a reference STOP stop computing: count only the others
    # (diag is the all-reduced sum over ranks for N > 1)
    failed = int(round(float(diag[11])))
    steps_per_cell = sum(synth.days_in_year(y) * ns for y in years[W:])
    cell_steps_rank = (n_total - failed) / world * steps_per_cell
    value = (n_total - failed) * steps_per_cell / elapsed
    launch_s = launch_ms / 1e3 / n_launch
    if cy_launch is None:
        algo_bytes_launch = cell_steps_rank / K * bytes_per_cell_step(L)
    else:      # cell-years of an average launch x the timed years' mean substeps per cell-year
        algo_bytes_launch = cy_launch * steps_per_cell / K * bytes_per_cell_step(L)
    achieved = algo_bytes_launch / launch_s / 1e9
    build = h.build_id()
    pmc, stale = load_traffic(args.workload, ctx.kernel_name(), build)
    traffic = None
    if pmc and pmc.get("hbm_bytes_per_launch"):
        traffic = pmc["hbm_bytes_per_launch"] / launch_s / 1e9
    valu = valu_roofline(pmc, launch_s)

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "cell-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W_req,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (hybrid9_amd.synth seed %d%s, generated on device; PGF/BNU "
                "datasets are not available offline)" % (synth.SEED if args.seed is None else args.seed,
                                                         "" if args.strong else "+rank"),
        "config": {"workload": f"{args.workload}: {wl['desc']}", "cells_per_gpu": int(gid.size),
                   "cells_total": int(n_total),
                   "nlayers": L, "nisurf": ns, "grow": wl["grow_on"],
                   "years_per_step": 1,
                   "years": f"{years[W]}-{years[-1]} timed" + (f", {years[0]}-{years[W - 1]} untimed" if W else ""),
                   "order": args.order,
                   "forcing_slots": nslots,
                   "parallelism": f"dp{world} (cell shards, RCCL all-reduce "
                   "of FP64 diagnostics per year)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "kernel_ms_per_launch": launch_s * 1e3, "launches": n_launch,
                     "cell_years_per_launch": cy_launch if cy_launch is not None else (n_total - failed) / world,
                     "algorithmic_bytes_per_launch": algo_bytes_launch,
                     "traffic_source": (pmc or {}).get("source"), "valu": valu,
                     "build_id": build, "traffic_stale": stale,
                     "kernel_stats": (pmc or {}).get("kernel_stats"),
                     "rocprof_ms_per_launch": ((pmc or {}).get("kernel_avg_ns_rocprof") or 0) / 1e6 or None},
        "cpu_baseline": None,
        "diagnostics_last_year": {k: float(v) for k, v in zip(h.DIAG_NAMES, diag)},
        "cells_stopped": failed,
        "order": args.order,
        "semantics": ("the reference's own order: decade -> cell -> year, smp carried from cell to cell "
                      "(HYBRID9.f90:93-130), bit-identical to the reference (DESIGN.md §2)"
                      if args.order == "cell" else
                      "isolated cells (every cell its own smp): not the reference's order (DESIGN.md §2)"),
        "kernel_ms_total": kern_ms,
        "launches": launches,
    }
    if args.order == "cell":
        out["cell_order"] = {"calls": work,
                             "rerun_cell_years_per_cell_year": sum(w["rerun_cell_years"] for w in work) /
                             max(1.0, float(gid.size * K)),
                             "warmup_years_run": W}
        if (world == 1 and not args.no_isolated_line and len(pl["years"]) >= 25):
            out["isolated"] = isolated_line(ctx, pl, ns, sync)
    if host_fed is not None:
        out["host_fed"] = host_fed.describe()
        host_fed.close()
    if nc_fed is not None:
        out["forcing"] = nc_fed.describe()
        out["data"] = "synthetic forcing read from netCDF-4 files each step (tools/pgf_synth.py)"
        subprocess.run(["rm", "-rf", str(Path(nc_fed.paths[0]).parent)])
    ctx.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline and host_fed is None and nc_fed is None:
        out["cpu_baseline"] = cpu_baseline(wl, synth.SEED)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
