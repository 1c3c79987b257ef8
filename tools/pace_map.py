#!/usr/bin/env python3
"""Which workgroups of a full config-2 launch share a SIMD: runs the pace
probe (h9g_pace_probe: the pair kernel's shape, every wave resident) and
prints, per SIMD row, the block indices of its waves (tests/test_pace.py
decodes the same ids)."""
import ctypes as C
import sys
from collections import Counter, defaultdict
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    import torch
    import hybrid9_amd as h
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nb = 3 * ncu
    out = np.zeros(nb * 4 * 3, np.uint32)
    assert h.lib().h9g_pace_probe(0, nb, out.ctypes.data_as(C.POINTER(C.c_uint))) == 0
    hw, xcc, ok = out[0::3].astype(np.int64), out[1::3].astype(np.int64), out[2::3]
    print("resident", int(ok.sum()), "of", ok.size)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    cuid = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    rows = defaultdict(list)
    cus = defaultdict(set)
    for i in range(nb * 4):
        rows[(cuid[i], simd[i])].append(i)
        cus[cuid[i]].add(i // 4)
    wave_in_block_vs_simd = Counter((i % 4, int(simd[i])) for i in range(nb * 4))
    print("wave-in-block -> SIMD:", sorted(wave_in_block_vs_simd.items())[:16])
    diffs = Counter()
    for c, bl in cus.items():
        bl = sorted(bl)
        diffs[tuple(b - bl[0] for b in bl)] += 1
    print("block-index offsets within a CU (top 10):", diffs.most_common(10))
    print("xcc of block b vs b % 8:", Counter((int(xcc[b * 4]), b % 8) for b in range(nb)).most_common(10))
    first = sorted(cus.items())[:8]
    for c, bl in first:
        print("cu", c, sorted(bl))


if __name__ == "__main__":
    main()
