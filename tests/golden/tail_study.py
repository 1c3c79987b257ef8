"""Where the cell order's re-runs come from, on a cell-order golden's band
(CPU, the C oracle as checker; round 6).  Not a test: the data behind
DESIGN.md §2's tail analysis (profiles/r06_tail_study_co_c2_band.txt).

For each decade after the first, every land cell's decade is run twice
from the reference's decade start (the oracle's cell order):
  A  from the cell's own smp -- h9g_run_ordered's first pass;
  B  from its predecessor's end-of-decade smp -- the reference's input
     (HYBRID9.f90:93-130, HYDROLOGY.f90:270-275).
Per year it prints how many cells' annual means differ between A and B,
how many cells' states still differ at the year end (a re-run cell leaves
the re-run at the first year end where they agree) and which state rows
differ.

    python tests/golden/tail_study.py [golden] [decades]

The decade-start states of the reference order are cached in
tests/_build/<golden>_states.npz (the oracle's cell order takes ~8 min per
decade of a 2,251-cell band)."""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from oracle import port, refcase  # noqa: E402
from tests.conftest import load_golden  # noqa: E402


def main() -> None:
    name = sys.argv[1] if len(sys.argv) > 1 else "co_c2_band"
    ndec = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    meta, inp, _ = load_golden(name)
    zi, p, f = inp["zi"], inp["params"], inp["forcing"]
    L, n, ns, grow = meta["L"], meta["ncell"], meta["nisurf"], meta["grow_on"]
    days = port._days
    d0s = [0]
    for k in range(ndec):
        d0s.append(d0s[-1] + sum(days(1901 + 10 * k + j) for j in range(10)))
    cache = ROOT / "tests" / "_build" / f"{name}_states.npz"
    cache.parent.mkdir(parents=True, exist_ok=True)
    if cache.exists():
        z = np.load(cache)
        S = [refcase.unpack_state(z[f"s{k}"], n, L) for k in range(ndec + 1)]
    else:
        S = [refcase.unpack_state(port.init_state(p, zi), n, L)]
        for k in range(ndec):
            t = time.time()
            r = port.run_cell_order(zi=zi, params=p, forcing=f[:, d0s[k]:d0s[k + 1]], nisurf=ns,
                                    year0=1901 + 10 * k, nyears=10, grow_on=grow, state0=S[-1])
            S.append(r["state"])
            print(f"reference order, decade {1901 + 10 * k}: {time.time() - t:.0f} s", flush=True)
        np.savez(cache, **{f"s{k}": refcase.pack_state(S[k], L) for k in range(ndec + 1)})
    land = [c for c in range(n) if port._mask_sum(p["theta_s"][c]) > np.float32(1e-8)]
    names = [k for k, _ in refcase.state_fields(L)]

    def bits(a):
        return np.asarray(a).view(np.uint32)

    for k in range(1, ndec):
        Sa, Se = S[k], S[k + 1]
        A = {kk: v.copy() for kk, v in Sa.items()}
        B = {kk: v.copy() for kk, v in Sa.items()}
        for i, c in enumerate(land):
            pred = land[i - 1]
            B["smp"][c] = Sa["smp"][pred] if i == 0 else Se["smp"][pred]
        d0 = d0s[k]
        alive = np.ones(n, bool)
        tails = []
        for y in range(10):
            yr = 1901 + 10 * k + y
            nd = days(yr)
            fa = np.ascontiguousarray(f[:, d0:d0 + nd])
            ra = port.run(zi=zi, params=p, forcing=fa, nisurf=ns, year0=yr, nyears=1, grow_on=grow, state0=A,
                          nthreads=8)
            rb = port.run(zi=zi, params=p, forcing=fa, nisurf=ns, year0=yr, nyears=1, grow_on=grow, state0=B,
                          nthreads=8)
            A, B = ra["state"], rb["state"]
            d0 += nd
            andiff = sum(not np.array_equal(bits(ra["annual"][0, :, c]), bits(rb["annual"][0, :, c])) for c in land)
            rows, still = {}, []
            for c in np.nonzero(alive)[0]:
                dif = [kk for kk in names if not np.array_equal(bits(A[kk][c]), bits(B[kk][c]))]
                if dif:
                    still.append(int(c))
                    rows[",".join(dif)] = rows.get(",".join(dif), 0) + 1
            alive[:] = False
            alive[still] = True
            tails.append(still)
            print(yr, "annual differs", andiff, "state differs", len(still),
                  sorted(rows.items(), key=lambda kv: -kv[1])[:6], flush=True)
        print("decade", 1901 + 10 * k, "tail at years 2/5/10:", tails[1], tails[4], tails[9], flush=True)


if __name__ == "__main__":
    main()
