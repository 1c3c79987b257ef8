"""The CPU oracle (oracle/h9_oracle.c) against the golden vectors that the
REFERENCE produced (tests/golden, made by oracle/_ref/h9ref from the
unmodified HYDROLOGY.f90/GROW.f90).  Bit-for-bit."""
import numpy as np
import pytest

from oracle import port, refcase
from tests.conftest import golden_names, load_golden, same_bits


@pytest.mark.parametrize("name", golden_names(kind=("synth", "explicit", "spinup")))
def test_oracle_matches_reference_golden(name):
    meta, inp, exp = load_golden(name)
    L, n = meta["L"], meta["ncell"]
    state0 = None if inp["state0"] is None else refcase.unpack_state(inp["state0"], n, L)
    out = port.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"],
                   nisurf=inp["nisurf"], year0=inp["year0"], nyears=inp["nyears"],
                   grow_on=inp["grow_on"], state0=state0,
                   trace_cells=meta.get("trace_cells", ()), nthreads=4)
    assert out["rc"] == 0, out["err"]
    assert same_bits(out["annual"], exp["annual"])
    assert same_bits(refcase.pack_state(out["state"], L), exp["state"])
    if "trace" in exp:
        k = exp["trace"].shape[1]
        assert same_bits(out["trace"][:, :k, :], exp["trace"])


@pytest.mark.parametrize("name", golden_names(kind=("stop",)))
def test_oracle_reproduces_reference_stop(name):
    meta, inp, _ = load_golden(name)
    out = port.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"],
                   nisurf=inp["nisurf"], year0=inp["year0"], nyears=1, grow_on=inp["grow_on"],
                   nthreads=4)
    s = meta["stop"]
    assert out["rc"] == s["code"]
    assert out["err"]["cell"] == s["cell"] and out["err"]["day"] == s["day"]
    assert f"{out['err']['value']:.9g}" == f"{s['value']:.9g}"


def test_oracle_is_cell_order_independent():
    """Isolated-cell semantics: a cell's results do not depend on its
    neighbours or on how cells are grouped."""
    meta, inp, exp = load_golden("c1_10x10")
    sub = np.arange(3, 100, 7)
    p = {k: v[sub] for k, v in inp["params"].items()}
    out = port.run(zi=inp["zi"], params=p, forcing=inp["forcing"][:, :, sub], nisurf=48,
                   year0=1901, nyears=1, grow_on=1)
    assert same_bits(out["annual"], exp["annual"][:, :, sub])


def test_oracle_matches_reference_l10_golden():
    """Config 5 (L = 10) against the reference rebuilt with
    nsoil_layers_max = 10 (oracle/_ref/h9ref_l10), including a cell that
    reaches the water-imbalance STOP: NaN means for it, its STOP record,
    and the other cells' annual means and end state bit for bit."""
    meta, inp, exp = load_golden("c5_l10_sample")
    L, ok = meta["L"], exp["ok"]
    out = port.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"], nisurf=inp["nisurf"],
                   year0=inp["year0"], nyears=inp["nyears"], grow_on=inp["grow_on"], nthreads=4)
    assert same_bits(out["annual"], exp["annual"])
    (s,) = meta["stops"]
    assert out["rc"] == s["code"] and out["err"]["cell"] == s["cell"] and out["err"]["day"] == s["day"]
    assert f"{out['err']['value']:.9g}" == f"{s['value']:.9g}"
    st = {k: (v[ok] if v.ndim else v) for k, v in out["state"].items()}
    assert same_bits(refcase.pack_state(st, L), exp["state_ok"])


def test_oracle_reproduces_bench_stop():
    """The config-2 bench's own STOP (land cell 20735, 1910, found by the
    GPU run of the driver's years; tests/golden make_golden.bench_stop_case):
    the reference STOPs there, and so does the oracle, with the same record;
    three cells of the same grid run through the 10 years bit for bit."""
    meta, inp, exp = load_golden("c2_bench_stop")
    ok = exp["ok"]
    out = port.run(zi=inp["zi"], params=inp["params"], forcing=inp["forcing"], nisurf=inp["nisurf"],
                   year0=inp["year0"], nyears=inp["nyears"], grow_on=inp["grow_on"], nthreads=4)
    (s,) = meta["stops"]
    c = s["cell"]
    assert out["rc"] == s["code"] and out["err"]["cell"] == c
    assert out["errors"]["code"][c] == s["code"] and out["errors"]["day"][c] == s["day"]
    assert out["errors"]["value"][c] == np.float32(s["value"])     # printed by the reference to 8 digits
    assert np.array_equal(np.nonzero(out["errors"]["code"])[0], [c])
    assert same_bits(out["annual"][:, :, ok], exp["annual"][:, :, ok])
    st = {k: (v[ok] if v.ndim else v) for k, v in out["state"].items()}
    assert same_bits(refcase.pack_state(st, meta["L"]), exp["state_ok"])
