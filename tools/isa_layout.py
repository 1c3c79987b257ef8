#!/usr/bin/env python3
"""Instruction-fetch footprint of the pair kernel's substep loop.

    bash tools/isa_pair.sh <tag>            # /tmp/isa/<tag>.{s,mir}
    python tools/isa_layout.py /tmp/isa/<tag>

Assembles the kernel's assembly with llvm-mc (block comments turned into
labels) to get every basic block's byte size and address, weighs the blocks
with tools/isa_mix.py's block frequencies (per wave-substep), and reports
the hot code's bytes and the 64-B instruction-cache lines it spans: the
inlined rare paths sit between the hot blocks, so the lines a substep
touches can far exceed its instruction bytes."""
from __future__ import annotations

import re
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import isa_mix  # noqa: E402

LLVM_MC = "/opt/rocm/lib/llvm/bin/llvm-mc"
FUNC = "_Z15h9g_pair_kernelILi8EN3h9k4GeoCILi8ELi48EEEEv5KArgsT0_"


def block_sizes(asm_path: Path, func: str):
    src = asm_path.read_text()
    a = src.index(f"{func}:")
    b = src.index(".Lfunc_end", a)
    body = src[a:b]
    lines = []
    for line in body.splitlines():
        m = re.match(r"^; %bb\.(\d+):", line)
        if m:
            lines.append(f".Lmirbb_{m.group(1)}:")
            continue
        m = re.match(r"^\.LBB\d+_(\d+):", line)
        if m:
            lines.append(f".Lmirbb_{m.group(1)}:")
            lines.append(line.split(";")[0])
            continue
        lines.append(line)
    text = "\t.amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n\t.text\n" + "\n".join(lines) + "\n"
    r = subprocess.run([LLVM_MC, "-triple=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-show-encoding"], input=text,
                       capture_output=True, text=True)
    sizes, order, cur = {}, [], None
    for line in r.stdout.splitlines():
        m = re.match(r"^\.Lmirbb_(\d+):", line)
        if m:
            cur = int(m.group(1))
            order.append(cur)
            sizes[cur] = 0
            continue
        m = re.search(r"encoding: \[([^\]]*)\]", line)
        if m and cur is not None:
            sizes[cur] += len(m.group(1).split(","))
    return order, sizes


def main():
    stem = Path(sys.argv[1])
    order, sizes = block_sizes(stem.with_suffix(".s"), FUNC)
    w, inloop, _, _, _ = isa_mix.weights(stem, FUNC)
    addr, a = {}, 0
    for bb in order:
        addr[bb] = a
        a += sizes[bb]
    print(f"kernel code {a / 1024:.1f} KB, {len(order)} blocks")
    for thr in (0.5, 0.1, 0.01, 0.001):
        hot = [bb for bb in order if bb in inloop and w.get(bb, 0) >= thr]
        byt = sum(sizes[bb] for bb in hot)
        lines = set()
        for bb in hot:
            lines.update(range(addr[bb] // 64, (addr[bb] + max(sizes[bb], 1) - 1) // 64 + 1))
        span = (max(addr[bb] + sizes[bb] for bb in hot) - min(addr[bb] for bb in hot)) if hot else 0
        print(f"blocks with freq >= {thr:<6}: {len(hot):4d} blocks, {byt / 1024:6.1f} KB of code, "
              f"{len(lines):5d} 64-B lines ({len(lines) * 64 / 1024:.1f} KB), spread over {span / 1024:.1f} KB")


if __name__ == "__main__":
    main()
