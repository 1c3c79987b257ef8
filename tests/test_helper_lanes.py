"""The helper-lane task map of hydrology_pair (h9g_pair.h, round 5), restated
and checked on the host for every wave shape the library instantiates: the
per-layer phases of a wave with S pair lanes (C = S/2 columns) and H = 64 - S
helpers take R = ceil(NT S / 64) rounds; pair lanes evaluate their own slots
U .. NT-1 (U = NT - R), one per round, and helper S + tau % H evaluates task
tau = u S + k (slot u of pair lane k) in round tau // H.  The device code
fetches a helper's operands only for the slots its round can hold
(ulo..uhi) and returns a result only from the rounds that hold that slot's
tasks (qlo..qhi); a task outside those windows would silently read another
lane's value, so the windows are checked against the map itself."""
from __future__ import annotations

import pytest

# (L, columns per wave): h9g_pair_kernel / h9g_pair2_kernel (22),
# h9g_pair11_kernel (11), h9g_pair1_kernel (1)
SHAPES = [(L, C) for L in (8, 10) for C in (22, 11, 1)]


def plan(L, C):
    NT, S = L // 2, 2 * C
    H = 64 - S
    R = (NT * S + 63) // 64
    U = NT - R
    return NT, S, H, R, U


@pytest.mark.parametrize("L,C", SHAPES)
def test_every_slot_is_evaluated_once(L, C):
    NT, S, H, R, U = plan(L, C)
    assert U >= 1 and U * S <= R * H            # the static_assert of hydrology_pair
    done = {}
    for q in range(R):                           # pair lanes: own slots U + q
        for k in range(S):
            done.setdefault((U + q, k), []).append(("pair", q))
    TOT = U * S
    for q in range(R):                           # helpers: tasks tau = q H + j (clamped)
        for j in range(H):
            tau = min(q * H + j, TOT - 1)
            if q * H + j >= TOT:
                continue                         # a repeat of the last task: its result is never read
            u, k = divmod(tau, S)
            done.setdefault((u, k), []).append(("helper", S + j, q))
    assert sorted(done) == [(t, k) for t in range(NT) for k in range(S)]
    assert all(len(v) == 1 for v in done.values())


@pytest.mark.parametrize("L,C", SHAPES)
def test_result_and_operand_windows_hold_every_task(L, C):
    NT, S, H, R, U = plan(L, C)
    TOT = U * S

    def qlo(u):
        return (u * S) // H

    def qhi(u):
        return min((u * S + S - 1) // H, R - 1)

    def ulo(q):
        return min((q * H) // S, U - 1)

    def uhi(q):
        return min((q * H + H - 1) // S, U - 1)

    for k in range(S):                           # pair lane k gathers slot u from src in round qo
        for u in range(U):
            tau = u * S + k
            src, qo = S + tau % H, tau // H
            assert qlo(u) <= qo <= qhi(u)
            assert (src - S) + qo * H == tau         # that helper ran that task in that round
    for q in range(R):                           # a helper's task of round q has a fetched packet
        for j in range(H):
            tau = min(q * H + j, TOT - 1)
            assert ulo(q) <= tau // S <= uhi(q)


def test_round_counts():
    """The phases' rounds per wave shape: round 4's 22-column
    wave keeps its 3 rounds at L = 8; 11 columns take 2 at L = 10; one
    column takes one."""
    assert plan(8, 22)[3:] == (3, 1)
    assert plan(10, 22)[3:] == (4, 1)
    assert plan(10, 11)[3:] == (2, 3)
    assert plan(8, 1)[3:] == (1, 3)
    assert plan(10, 1)[3:] == (1, 4)
