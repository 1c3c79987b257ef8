"""The hardware ids behind the pair kernel's issue pacer (h9g_pair.h Pacer,
pace_key).  pace_key keys a wave's progress row by XCC/SE/SH/CU/SIMD from
HW_REG_HW_ID (wave slot 3:0, SIMD 5:4, CU 11:8, SH 12, SE 15:13) and
HW_REG_XCC_ID (3:0).  If that layout were wrong on gfx950, unrelated waves
would share a row and the pacer's priorities would be meaningless (results
stay bit-exact either way: priorities only order issue).  The probe launches
the config-2 pair kernel's shape and LDS footprint so that every wave is
resident at once, and checks that the decoded rows are exactly one per SIMD
of the device, each holding the pacer's RESIDENT (3) waves in distinct
slots."""
import ctypes as C

import numpy as np
import pytest

import hybrid9_amd as h

pytestmark = pytest.mark.gpu

PACE_ROWS = 16384     # h9g_pair.h H9G_PACE_ROWS
RESIDENT = 3          # h9g_pair.h pair_resident<8>()


def decode(hw, xcc):
    slot = hw & 15
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    row = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    return row.astype(np.int64), slot.astype(np.int64)


def test_pace_key_rows_are_the_simds():
    import torch
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nblocks = RESIDENT * ncu                  # every CU full: 3 workgroups of 4 waves
    out = np.zeros(nblocks * 4 * 3, np.uint32)
    rc = h.lib().h9g_pace_probe(0, nblocks, out.ctypes.data_as(C.POINTER(C.c_uint)))
    assert rc == 0
    hw, xcc, ok = out[0::3].astype(np.int64), out[1::3].astype(np.int64), out[2::3]
    if not ok.all():
        pytest.skip(f"{int((ok == 0).sum())} waves were not resident at once (shared GPU?)")
    row, slot = decode(hw, xcc)
    assert row.max() < PACE_ROWS
    rows, counts = np.unique(row, return_counts=True)
    print(f"{ncu} CUs, {rows.size} rows, waves per row {np.bincount(counts).tolist()}, "
          f"XCCs {np.unique(xcc).tolist()}")
    assert rows.size == 4 * ncu                       # one row per SIMD
    assert counts.max() <= RESIDENT and counts.min() == RESIDENT
    assert np.unique(row * 16 + slot).size == row.size   # the slots of a row are distinct
