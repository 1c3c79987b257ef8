#!/usr/bin/env python3
"""Where the pair kernel's waves park in s_waitcnt lgkmcnt:
every LDS read of the substep loop, the distance from its issue to the
s_waitcnt that drains it, weighted by the compiler's block frequencies
(tools/isa_mix.py weights) and grouped by phase and by kind of read.

    bash tools/isa_pair.sh <tag> -DH9G_ISA_PHASES    # /tmp/isa/<tag>.{s,mir}
    python tools/isa_waits.py /tmp/isa/<tag> [--top N]

Model.  Within a basic block the LGKM counter drains in issue order (LDS
returns in order; the substep issues almost no scalar loads), so
`s_waitcnt lgkmcnt(N)` completes every read but the N youngest.  A read's
distance is the number of instructions the wave issued between the read and
the wait that needs it.  An LDS read takes ~64-128 shader cycles and a wave
issues at most one instruction per ~4-5 cycles on its own, so a read
drained after fewer than ~16-24 instructions stalls its wave unless the
SIMD's other waves fill the gap.  Reads still outstanding at the end of a
block are charged at the block end (the successor's first wait).
Reads are classed by their form: ds_read_b32/b64/read2 with a per-lane
computed address from a table (the powf/expf tables: b64/b128) or store
fields (b32, read2)."""
from __future__ import annotations

import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from isa_mix import weights  # noqa: E402

LBL = re.compile(r"^(?:\.LBB\d+_|; %bb\.)(\d+):")
WAIT = re.compile(r"s_waitcnt\s+(.*)")
LGKM = re.compile(r"lgkmcnt\((\d+)\)")
PHASE = re.compile(r"h9g-phase (\d+)")


def blocks_asm(stem: Path, func: str):
    asm = stem.with_suffix(".s").read_text()
    asm = asm[asm.index(f"{func}:"):]
    asm = asm[:asm.index(".Lfunc_end")]
    out, cur, order = {}, None, []
    for line in asm.splitlines():
        m = LBL.match(line)
        if m:
            cur = int(m.group(1))
            out[cur] = []
            order.append(cur)
            continue
        if cur is None:
            continue
        s = line.strip()
        if PHASE.search(s):
            out[cur].append(("PHASE", PHASE.search(s).group(1)))
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        out[cur].append(("I", s.split(";")[0].strip()))
    return out, order


def kind(ins: str) -> str:
    op = ins.split()[0]
    return op


def main() -> None:
    stem = Path(sys.argv[1])
    pos = [a for a in sys.argv[2:] if not a.startswith("--")]
    func = pos[0] if pos else "_Z15h9g_pair_kernelILi8EN3h9k4GeoCILi8ELi48EEEEv5KArgsT0_"
    top = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--top=")), 12))
    w, inloop, _, h, _ = weights(stem, func, [])
    blocks, order = blocks_asm(stem, func)
    # per (phase, kind): reads, weighted; distance histogram buckets
    reads = defaultdict(float)
    dist_sum = defaultdict(float)
    short = defaultdict(float)          # drained within 16 instructions
    waits = defaultdict(float)          # weighted s_waitcnt lgkmcnt per phase
    buckets = [4, 8, 16, 32, 64, 10 ** 9]
    hist = defaultdict(lambda: [0.0] * len(buckets))
    phase = "?"
    for b in order:
        ins = blocks[b]
        f = w.get(b, 0.0)
        q = []                           # outstanding LGKM ops: (index, kind, phase)
        n = 0
        for tag, s in ins:
            if tag == "PHASE":
                phase = s
                continue
            op = s.split()[0]
            if op.startswith("s_waitcnt"):
                m = LGKM.search(s)
                if m:
                    keep = int(m.group(1))
                    if b in inloop and len(q) > keep:
                        waits[phase] += f
                    while len(q) > keep:
                        i0, k, ph = q.pop(0)
                        d = n - i0
                        if b in inloop:
                            reads[(ph, k)] += f
                            dist_sum[(ph, k)] += f * d
                            if d < 16:
                                short[(ph, k)] += f
                            for j, lim in enumerate(buckets):
                                if d < lim:
                                    hist[ph][j] += f
                                    break
                continue
            if op.startswith("ds_read") or op.startswith("s_load") or op.startswith("s_buffer_load") or \
                    op.startswith("ds_bpermute"):
                q.append((n, op, phase))
            n += 1
        for i0, k, ph in q:              # drained after the block
            if b in inloop:
                d = n - i0
                reads[(ph, k)] += f
                dist_sum[(ph, k)] += f * d
                for j, lim in enumerate(buckets):
                    if d < lim:
                        hist[ph][j] += f
                        break
    tot = sum(reads.values())
    print(f"substep loop bb.{h}: {tot:.1f} LGKM reads per wave-substep; "
          f"{sum(waits.values()):.1f} draining s_waitcnt lgkmcnt")
    print("by phase: reads, draining waits, distance histogram (<4 <8 <16 <32 <64 >=64 instructions)")
    for ph in sorted(hist):
        r = sum(v for (p, _), v in reads.items() if p == ph)
        print(f"  phase {ph}: {r:7.1f} reads {waits[ph]:6.1f} waits  " +
              " ".join(f"{v:6.1f}" for v in hist[ph]))
    print(f"by phase and form (top {top} by reads drained within 16 instructions):")
    rows = sorted(reads, key=lambda k: -short[k])[:top]
    for k in rows:
        print(f"  phase {k[0]} {k[1]:18s} reads {reads[k]:6.1f}  mean distance {dist_sum[k] / reads[k]:5.1f}  "
              f"within 16: {short[k]:6.1f}")


if __name__ == "__main__":
    main()
