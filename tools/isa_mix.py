#!/usr/bin/env python3
"""Static instruction mix of the pair kernel's substep, weighted by the
compiler's own block frequencies.

    bash tools/isa_pair.sh [tag] [flags...]   # writes /tmp/isa/<tag>.{s,mir}
    python tools/isa_mix.py /tmp/isa/<tag>    # mix per substep

The final MIR (printed after branch relaxation) carries every edge's branch
probability, the rare paths' __builtin_expect weights included.  Block
frequencies follow from f = e_entry + P^T f; the substep loop is the
innermost loop header of the assembly's loop comments with the largest
frequency.  Counts are per execution of that header, i.e. per wave and
substep: comparable with the PMC counters per wave-substep
(profiles/pmc_*.json per_wave / 17,520).  Instructions are classed by MIR
opcode; 'other' VALU is everything the typed counters do not name
(compares, selects, moves, DPP, lane reads/writes, min/max ...)."""
from __future__ import annotations

import re
import sys
from collections import Counter, defaultdict
from pathlib import Path

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spl

BB = re.compile(r"^bb\.(\d+)")
SUCC = re.compile(r"%bb\.(\d+)\((0x[0-9a-f]+)\)")
FLAGS = {"renamable", "nofpexcept", "nnan", "ninf", "nsz", "arcp", "contract", "afn", "reassoc", "nuw", "nsw",
         "exact", "killed", "early-clobber", "undef", "dead", "internal"}


def opcode(line: str) -> str | None:
    s = line.strip()
    if not s or s.startswith(";") or s.startswith("successors") or s.startswith("liveins") or s == "}":
        return None
    if " = " in s:
        s = s.split(" = ", 1)[1]
    for tok in s.replace(",", " ").split():
        if tok in FLAGS:
            continue
        return tok
    return None


def parse(mir: str, func: str):
    blocks, succ, cur = {}, {}, None
    inside = False
    for line in mir.splitlines():
        if line.startswith("# Machine code for function"):
            inside = func in line
            continue
        if not inside:
            continue
        m = BB.match(line)
        if m:
            cur = int(m.group(1))
            blocks[cur] = []
            succ[cur] = []
            continue
        if cur is None:
            continue
        if line.strip().startswith("successors:"):
            succ[cur] = [(int(b), int(p, 16) / 2**31) for b, p in SUCC.findall(line.split(";")[0])]
            continue
        op = opcode(line)
        if op is not None and op.startswith("INLINEASM") and "h9g-substep" in line:
            blocks[cur].append("MARK")
            continue
        if op is not None and op.startswith("INLINEASM") and "h9g-phase" in line:
            m = re.search(r"\[imm\],\s*(\d+)", line)
            blocks[cur].append("PHASE" + (m.group(1) if m else "?"))
            continue
        if op is None or op == "BUNDLE" or op.startswith("INLINEASM") or op in ("DBG_VALUE", "KILL", "IMPLICIT_DEF",
                                                                                "SCHED_BARRIER"):
            continue
        blocks[cur].append(op)
    return blocks, succ


def classify(op: str) -> str:
    if op.startswith("V_"):
        o = op
        if "_F64" in o:
            if o.startswith("V_CVT"):
                return "valu.cvt"
            if o.startswith(("V_FMA_F64", "V_FMAC_F64")):
                return "valu.f64.fma"
            if o.startswith(("V_MUL_F64",)):
                return "valu.f64.mul"
            if o.startswith(("V_ADD_F64",)):
                return "valu.f64.add"
            if o.startswith(("V_RCP_F64", "V_RSQ_F64", "V_SQRT_F64")):
                return "valu.f64.trans"
        if o.startswith("V_CVT"):
            return "valu.cvt"
        if o.startswith(("V_FMA_F32", "V_FMAC_F32", "V_MAC_F32", "V_PK_FMA")):
            return "valu.f32.fma"
        if o.startswith(("V_MUL_F32",)):
            return "valu.f32.mul"
        if o.startswith(("V_ADD_F32", "V_SUB_F32", "V_SUBREV_F32")):
            return "valu.f32.add"
        if o.startswith(("V_RCP_F32", "V_EXP_F32", "V_LOG_F32", "V_RSQ_F32", "V_SQRT_F32")):
            return "valu.trans32"
        if o.startswith(("V_DIV_SCALE", "V_DIV_FMAS", "V_DIV_FIXUP")):
            return "valu.divsteps"
        if o.startswith(("V_CNDMASK",)):
            return "valu.cndmask"
        if o.startswith(("V_CMP",)):
            return "valu.cmp"
        if o.startswith(("V_READLANE", "V_WRITELANE", "V_READFIRSTLANE")):
            return "valu.lane"
        if "DPP" in o:
            return "valu.dpp"
        if o.startswith(("V_MOV",)):
            return "valu.mov"
        if o.startswith(("V_MAX", "V_MIN")):
            return "valu.minmax"
        if o.startswith(("V_LSHL_ADD_U64", "V_LSHLREV_B64", "V_LSHRREV_B64", "V_ASHRREV_I64", "V_ADD_U64",
                         "V_MAD_U64", "V_MAD_I64")):
            return "valu.int64"
        return "valu.int32/other"
    if op.startswith(("S_CBRANCH", "S_BRANCH")):
        return "branch"
    if op.startswith(("S_WAITCNT", "S_NOP", "S_SETPRIO", "S_SLEEP")):
        return "wait/nop"
    if op.startswith("S_LOAD") or op.startswith("S_BUFFER_LOAD"):
        return "smem"
    if op.startswith("S_"):
        return "salu"
    if op.startswith("DS_"):
        return "lds"
    if op.startswith(("GLOBAL_", "BUFFER_", "SCRATCH_", "FLAT_")):
        if "SPILL" in op or op.startswith("SCRATCH") or op.startswith("BUFFER"):
            return "vmem.scratch"
        return "vmem"
    if "SPILL" in op:
        return "spill." + op
    return "pseudo." + op


def weights(stem: Path, func: str, argv=()):
    """per-block frequency per wave-substep and the substep loop's blocks"""
    blocks, succ = parse(stem.with_suffix(".mir").read_text(), func)
    n = max(blocks) + 1
    rows, cols, vals = [], [], []
    for b, ss in succ.items():
        for t, p in ss:
            rows.append(t)
            cols.append(b)
            vals.append(p)
    P = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    e = np.zeros(n)
    e[0] = 1.0
    f = spl.spsolve((sp.identity(n, format="csr") - P).tocsc(), e)
    asm = stem.with_suffix(".s").read_text()
    asm = asm[asm.index(f"{func}:"):]
    asm = asm[:asm.index(".Lfunc_end")]
    hdr, last = [], None
    for line in asm.splitlines():
        m = re.match(r"^(?:\.LBB\d+_|; %bb\.)(\d+):", line)
        if m:
            last = int(m.group(1))
        m = re.search(r"This\s+Loop Header: Depth=(\d+)", line)
        if m and last is not None:
            hdr.append((last, int(m.group(1))))
    hdr = [h for h in hdr if h[0] in blocks]
    if "--headers" in argv:
        for b, d in hdr:
            print(f"  header bb.{b} depth {d} freq {f[b]:.4g} instrs {len(blocks[b])}")
    hsel = [a for a in argv if a.startswith("--header=")]
    h = int(hsel[0].split("=")[1]) if hsel else max(hdr, key=lambda x: (x[1] == 2, f[x[0]]))[0]
    mark = sum(f[b] for b, ins in blocks.items() for op in ins if op == "MARK")
    w = f / (mark if mark > 0 else f[h])
    inloop, last = set(), None
    tag = re.compile(rf"(Header=BB\d+_{h}\b|Parent Loop BB\d+_{h}\b)")
    for line in asm.splitlines():
        m = re.match(r"^(?:\.LBB\d+_|; %bb\.)(\d+):", line)
        if m:
            last = int(m.group(1))
            if last == h:
                inloop.add(last)
        if last is not None and tag.search(line):
            inloop.add(last)
    return {b: w[b] for b in blocks}, inloop, blocks, h, mark


def main() -> None:
    stem = Path(sys.argv[1])
    pos = [a for a in sys.argv[2:] if not a.startswith("--")]
    func = pos[0] if pos else "_Z15h9g_pair_kernelILi8EN3h9k4GeoCILi8ELi48EEEEv5KArgsT0_"
    w, inloop, blocks, h, mark = weights(stem, func, sys.argv[2:])
    if "--phases" in sys.argv:
        # blocks in layout (MIR number) order, each attributed to the last phase marker before it
        phase, per = "?", defaultdict(Counter)
        for b in sorted(blocks):
            for op in blocks[b]:
                if op.startswith("PHASE"):
                    phase = op[5:]
                    continue
                if b in inloop and op not in ("MARK",):
                    c = classify(op)
                    per[phase]["valu" if c.startswith("valu") else c] += w[b]
        for ph in sorted(per):
            print(f"  phase {ph}: " + "  ".join(f"{k} {v:.0f}" for k, v in sorted(per[ph].items(), key=lambda x: -x[1]) if v >= 1))
    mix, ops = Counter(), Counter()
    for b, ins in blocks.items():
        if b not in inloop:
            continue
        for op in ins:
            if op == "MARK" or op.startswith("PHASE"):
                continue
            c = classify(op)
            mix[c] += w[b]
            ops[op] += w[b]
    valu = sum(v for k, v in mix.items() if k.startswith("valu"))
    print(f"substep loop header bb.{h}; weighted per wave-substep ({'marker' if mark > 0 else 'header'})")
    print(f"  VALU {valu:8.1f}")
    for k, v in sorted(mix.items(), key=lambda x: -x[1]):
        if v >= 0.5:
            print(f"  {k:22s} {v:8.1f}")
    if "--ops" in sys.argv:
        print("top opcodes:")
        for k, v in ops.most_common(60):
            print(f"  {k:34s} {v:8.1f}")
    if "--blocks" in sys.argv:
        print("hottest blocks (freq, instrs):")
        for b in sorted(inloop, key=lambda b: -w[b] * len(blocks[b]))[:40]:
            print(f"  bb.{b:<5d} {w[b]:8.3f} {len(blocks[b]):5d}")


if __name__ == "__main__":
    main()
