"""The reference as it really runs: decade -> cell -> year with the module
array smp carried from cell to cell (HYBRID9.f90:93-130, HYDROLOGY.f90:
270-275, SHARED.f90:198).

Goldens ``co_*`` come from oracle/_ref/h9ref's cell_order mode (the
unmodified reference HYDROLOGY/GROW).  Their metadata records, as data from
the reference itself, how far the isolated-cell contract of h9g_run_year
sits from them.  The product reproduces the reference's order exactly with
h9g_run_decade_ordered (GPU tests); the C oracle's restatement of that
order is pinned here on the CPU.
"""
from __future__ import annotations

import numpy as np
import pytest

from tests.conftest import load_golden, same_bits

FIELDS_CHECKED = "rnf, theta_total, theta(1..L)"


def pick(L):
    from oracle import refcase
    f = refcase.annual_fields(L)
    return [f.index(k) for k in ["rnf", "theta_total"] + [f"theta{i + 1}" for i in range(L)]]


def rel_bound(a, b):
    from tests.golden.make_golden import rel_bound as rb
    return rb(a, b)


def test_decades_follow_the_reference():
    import hybrid9_amd as h
    from oracle import port
    for f in (h.decades, port.decades):
        assert f(1901, 30) == [(1901, 10), (1911, 10), (1921, 10)]
        assert f(1905, 12) == [(1905, 6), (1911, 6)]
        assert f(1911, 1) == [(1911, 1)]


def test_isolated_contract_departs_from_the_reference_order():
    """The measured bound the north star's 1e-6 is about: the isolated-cell
    oracle (bit-identical to h9g_run_year) against the reference's own order
    over three decades.  Deterministic, so it equals the record exactly."""
    from oracle import port
    meta, inp, exp = load_golden("co_c1_30yr")
    rec = meta["isolated_vs_cell_order"]
    iso = port.run(nthreads=8, **inp)
    assert iso["rc"] == 0
    a, b = iso["annual"], exp["annual"]
    p = pick(meta["L"])
    assert rel_bound(a[:, p, :], b[:, p, :]) == rec["annual"]
    assert rec["annual"] > 1e-6            # the isolated contract misses the north star's 1e-6 ...
    assert same_bits(a[:10], b[:10]) and rec["first_decade_bitwise"]   # ... only from the second decade on
    assert rec["cells_differing"] == int(np.any(np.any(a.view(np.uint32) != b.view(np.uint32), axis=0), axis=0).sum())


def test_reference_depends_on_its_rank_split():
    """The reference's own result depends on its MPI decomposition: cut into
    two ranks (two chains), the same cells move (recorded by make_golden)."""
    meta, _, _ = load_golden("co_c1_30yr")
    two = meta["two_ranks_vs_one"]
    assert two["cells_differing"] >= 1 and two["annual"] > 1e-6


def test_reference_blocks_follow_init():
    """shard.reference_blocks against a loop restating INIT.f90:271-274 and
    the chunk assignment of :427-444 (1-based x, y; ids along longitude)."""
    from hybrid9_amd.shard import reference_blocks
    for nx, ny, P in ((10, 10, 4), (720, 360, 4), (720, 360, 9), (720, 360, 16), (12, 6, 9), (7, 5, 1)):
        nb = int(round(np.sqrt(P)))
        lon_c, lat_c = nx // nb, ny // nb
        chunk = np.full((ny, nx), -1)
        i_block_s = 0
        for y in range(1, ny + 1):
            i_block = i_block_s
            for x in range(1, nx + 1):
                chunk[y - 1, x - 1] = i_block
                if x % lon_c == 0:
                    i_block += 1
            if y % lat_c == 0:
                i_block_s += nb
        # cells outside the nb x nb blocks are never run by the reference
        run = np.zeros((ny, nx), bool)
        run[:nb * lat_c, :nb * lon_c] = True
        want = np.where(run, chunk, -1).ravel()
        assert np.array_equal(reference_blocks(np.arange(nx * ny), nx, ny, P), want), (nx, ny, P)


def test_blocks_golden_records_the_rank_dependence():
    """The reference's result depends on its decomposition: the 4-rank run
    of config 1's grid differs from the 1-rank run (recorded by make_golden
    from the reference itself)."""
    meta, _, _ = load_golden("co_c1_blocks4")
    rec = meta["blocks_vs_one_rank"]
    assert meta["num_procs"] == 4 and len(set(meta["rank"])) == 4
    assert rec["cells_differing"] >= 1


@pytest.mark.slow
def test_oracle_cell_order_blocks_match_reference_golden():
    """oracle.port.run_cell_order with one chain per reference block,
    bit for bit against the reference's 4-process run."""
    from oracle import port
    meta, inp, exp = load_golden("co_c1_blocks4")
    out = port.run_cell_order(chains=np.asarray(meta["rank"]), **inp)
    assert out["rc"] == 0
    assert same_bits(out["annual"], exp["annual"])


@pytest.mark.slow
def test_oracle_cell_order_matches_reference_golden():
    """oracle.port.run_cell_order restates the reference's order on the C
    oracle; bit for bit against the reference over two decades (the third
    adds minutes, not coverage)."""
    from oracle import port
    meta, inp, exp = load_golden("co_c1_30yr")
    ny = 20
    nd = sum(365 + (y % 4 == 0) for y in range(1901, 1901 + ny))
    out = port.run_cell_order(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"][:, :nd],
                              nisurf=inp["nisurf"], year0=inp["year0"], nyears=ny, grow_on=inp["grow_on"])
    assert out["rc"] == 0
    assert same_bits(out["annual"], exp["annual"][:ny])


# --------------------------------------------------------------------------
# GPU: the product in the reference's order (h9g_run_decade_ordered)
# --------------------------------------------------------------------------
CO_GOLDENS = ["co_c1_30yr", "co_band", "co_c2_band", "co_c5_band"]


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [True, False], ids=["run_ordered", "per_decade"])
@pytest.mark.parametrize("name", CO_GOLDENS)
def test_gpu_cell_order_matches_reference(name, pipelined):
    """h9g_run_ordered (the decades overlapping: a decade's re-runs ride in
    the next decade's year launches) and h9g_run_decade_ordered (one call
    per decade) both reproduce the reference's own order bit for bit: config
    1's grid (three decades), a GROW-on 0.5 deg row band, config 2's own
    settings (GROW off, NS=48) on a row band over 1901-1930 -- the bench's
    timed decades -- and config 5's (0.25 deg, L=10, NS=24, GROW on) on a row
    band over 1901-1920, which runs the L = 10 one-column and 11-column
    list kernels and the chain and merge logic at L = 10."""
    import hybrid9_amd as h
    meta, inp, exp = load_golden(name)
    out = h.run_cell_order(pipelined=pipelined, **inp)
    assert out["rc"] == 0, out["err"]
    assert same_bits(out["annual"], exp["annual"])
    assert same_bits(out["state"], exp["state"])
    yrs = [w["rerun_cell_years"] for w in out["work"]]
    print(f"{name}: {meta['ncell']} cells x {meta['nyears']} years bit-identical to the reference's cell order; "
          f"decade passes {out['passes']}, cell-years re-run {yrs}, re-run launches "
          f"{[w['rerun_launches'] for w in out['work']]}" + (f", overlap {out['overlap']}" if pipelined else ""))
    if pipelined and name in ("co_c1_30yr", "co_band", "co_c2_band"):
        assert out["overlap"]["rerun_years_riding"] > 0     # the overlap path ran


@pytest.mark.gpu
def test_gpu_ordered_call_refuses_shared_slots():
    """Every year of an ordered call keeps its own forcing slot: a decade's
    re-runs read their years while the next decade's first pass reads its
    own, so a slot named twice is refused before anything runs."""
    import hybrid9_amd as h
    meta, inp, _ = load_golden("co_c1_30yr")
    L, n = meta["L"], meta["ncell"]
    with h.Context(n, inp["zi"], nlayers=L, nisurf=inp["nisurf"], grow_on=inp["grow_on"], nslots=3) as ctx:
        ctx.set_params(inp["params"])
        ctx.init_state()
        d0 = 0
        for k in range(3):
            nt = h.days_in_year(1901 + k)
            ctx.push_forcing(k, inp["forcing"][:, d0:d0 + nt, :])
            d0 += nt
        with pytest.raises(h.H9GError):
            ctx.run_ordered([0, 1, 0], 1901)
        _, passes = ctx.run_ordered([0, 1, 2], 1901)      # distinct slots run
        assert len(passes) == 1


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["co_band", "co_c2_band"])
def test_gpu_cell_order_probe_keeps_results(name, monkeypatch):
    """The checks' day-1 probe (h9g_probe_cmp_kernel, round 6) drops from a
    re-run every cell whose first day from its new input equals the day
    from its old one; the results stay the reference's bit for bit, with
    and without it (H9G_NO_PROBE), and the probe re-runs fewer cell-years."""
    import hybrid9_amd as h
    meta, inp, exp = load_golden(name)
    out = h.run_cell_order(**inp)
    monkeypatch.setenv("H9G_NO_PROBE", "1")
    ref = h.run_cell_order(**inp)
    for o in (out, ref):
        assert o["rc"] == 0, o["err"]
        assert same_bits(o["annual"], exp["annual"])
        assert same_bits(o["state"], exp["state"])
    ov, ov0 = out["overlap"], ref["overlap"]
    yrs, yrs0 = out["work"][0]["rerun_cell_years"], ref["work"][0]["rerun_cell_years"]
    print(f"{name}: probe ran {ov['probed']} cells, kept {ov['probe_kept']} for a re-run; cell-years re-run "
          f"{yrs} (without the probe {yrs0}); passes {out['passes']} / {ref['passes']}")
    assert ov0["probed"] == 0 and 0 < ov["probe_kept"] < ov["probed"]
    assert yrs < yrs0


@pytest.mark.gpu
@pytest.mark.parametrize("pipelined", [True, False], ids=["run_ordered", "per_decade"])
def test_gpu_cell_order_blocks_match_reference(pipelined):
    """One context holding the 4 reference ranks' blocks as 4 chains
    (h9g_set_chains) reproduces the reference's 4-process run bit for bit;
    so does each rank's block run alone (one GPU per rank)."""
    import hybrid9_amd as h
    meta, inp, exp = load_golden("co_c1_blocks4")
    rank = np.asarray(meta["rank"])
    out = h.run_cell_order(chains=rank, pipelined=pipelined, **inp)
    assert out["rc"] == 0, out["err"]
    assert same_bits(out["annual"], exp["annual"])
    assert same_bits(out["state"], exp["state"])
    from oracle import refcase
    L, n = meta["L"], meta["ncell"]
    ex_st = refcase.unpack_state(exp["state"], n, L)
    for r in (0, 3):                        # two of the ranks, each on its own context
        sel = np.where(rank == r)[0]
        sub = dict(inp, params={k: v[sel] for k, v in inp["params"].items()},
                   forcing=np.ascontiguousarray(inp["forcing"][:, :, sel]))
        o = h.run_cell_order(pipelined=pipelined, **sub)
        assert o["rc"] == 0
        assert same_bits(o["annual"], exp["annual"][:, :, sel])
        got = refcase.unpack_state(o["state"], sel.size, L)
        assert all(same_bits(got[k], ex_st[k][sel]) for k in got)
    print(f"co_c1_blocks4: 4 reference ranks as chains: bit-identical; passes {out['passes']}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", CO_GOLDENS)
def test_gpu_isolated_contract_bound(name):
    """h9g_run_year (isolated cells) on the same inputs: its distance to the
    reference's order is exactly the one the reference's isolated run shows
    (recorded by make_golden), and the first decade is bit-identical."""
    import hybrid9_amd as h
    meta, inp, exp = load_golden(name)
    rec = meta["isolated_vs_cell_order"]
    out = h.run(**inp)
    assert out["rc"] == 0
    a, b = out["annual"], exp["annual"]
    p = pick(meta["L"])
    bound = rel_bound(a[:, p, :], b[:, p, :])
    diff = int(np.any(np.any(a.view(np.uint32) != b.view(np.uint32), axis=0), axis=0).sum())
    print(f"{name}: isolated-cell contract vs the reference's order: max rel {bound:.3e} over {FIELDS_CHECKED}, "
          f"{diff} of {meta['ncell']} cells not bitwise")
    assert bound == rec["annual"] and diff == rec["cells_differing"]
    assert same_bits(a[:10], b[:10]) == rec["first_decade_bitwise"]


def _stop_of(err):
    return {k: int(err[k]) for k in ("code", "cell", "day")}


def test_oracle_cell_order_reproduces_reference_stop():
    """A STOP inside the reference's order (co_stop: the reference's
    cell_order run of stop_ns24's soils, HYDROLOGY.f90:1244-1274): the
    oracle's restatement stops with the reference's site, cell and day, and
    the value it prints."""
    from oracle import port
    meta, inp, _ = load_golden("co_stop")
    s = meta["stop"]
    out = port.run_cell_order(**inp)
    assert out["rc"] == s["code"]
    assert _stop_of(out["err"]) == {k: s[k] for k in ("code", "cell", "day")}
    assert np.float32(out["err"]["value"]) == np.float32(s["value"])


@pytest.mark.gpu
def test_gpu_cell_order_reproduces_reference_stop():
    """The product in the reference's order (h9g_run_decade_ordered) returns
    the reference's STOP (site, cell, day, printed value) as the first
    failing cell in its order, and every cell that completes has the
    oracle's annual sums bit for bit."""
    import hybrid9_amd as h
    from oracle import port
    meta, inp, _ = load_golden("co_stop")
    s = meta["stop"]
    out = h.run_cell_order(**inp)
    assert out["rc"] == s["code"], out["err"]
    e = out["err"]
    assert (int(e["cell"]), int(e["day"])) == (s["cell"], s["day"])
    assert np.float32(e["value"]) == np.float32(s["value"])
    ref = port.run_cell_order(**inp)
    assert int(e["substep"]) == int(ref["err"]["substep"])      # not printed by the reference
    ok = np.isfinite(ref["annual"]).all(axis=(0, 1))
    assert not ok[s["cell"]] and ok.sum() == meta["ncell"] - 1
    assert np.array_equal(np.isfinite(out["annual"]).all(axis=(0, 1)), ok)
    assert same_bits(out["annual"][:, :, ok], ref["annual"][:, :, ok])
