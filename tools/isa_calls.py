#!/usr/bin/env python3
"""Calls in the device code of libh9g, and registers live across them.

    python tools/isa_calls.py [lib.so]          # calls per device function
    python tools/isa_calls.py --live x.s KERNEL # SGPRs live across calls

The first form extracts the gfx950 code object from the library's HIP fat
binary (objcopy, clang-offload-bundler) and counts s_swappc_b64 per function
of its disassembly: the product kernels make none (tests/test_abi.py).

The second form reads device assembly (hipcc --cuda-device-only -S) and, for
every call of KERNEL, runs a backward liveness analysis over the kernel's
basic blocks and reports the SGPRs that are live after the call although the
callee writes them (the callee's own code, minus the ABI's callee-saved
SGPRs s33-s105).  Round 2's out-of-line redo functions hit exactly this: in
the kernel built with a wave-uniform branch added to the equilibrium
profile, the low half of a lane mask stayed in s4 across calls of
powf_redo, whose first block writes s[4:5].  VGPR writes are
exec-masked, so the analysis treats them as partial (never killing) and
reports SGPRs only."""
from __future__ import annotations

import re
import subprocess
import sys
import tempfile
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = Path("/opt/rocm/lib/llvm/bin")


def disassemble(so: Path) -> str:
    with tempfile.TemporaryDirectory() as d:
        fat, co = Path(d) / "fat.bin", Path(d) / "co.elf"
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", str(so), str(Path(d) / "x.so")],
                       check=True, capture_output=True)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                       capture_output=True)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", str(co)], check=True,
                              capture_output=True, text=True).stdout


def calls_per_function(so: Path) -> dict:
    out, cur = defaultdict(int), None
    for line in disassemble(so).splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            out[cur] += 0
        elif cur and "s_swappc_b64" in line:
            out[cur] += 1
    return dict(out)


# ---------------------------------------------------------------- liveness
def _regs(op: str) -> set:
    out = set()
    for m in re.finditer(r"\b([vsa])(\d+)\b", op):
        out.add(m.group(1) + m.group(2))
    for m in re.finditer(r"\b([vsa])\[(\d+):(\d+)\]", op):
        out |= {m.group(1) + str(k) for k in range(int(m.group(2)), int(m.group(3)) + 1)}
    if re.search(r"\bvcc\b", op):
        out.add("vcc")
    if re.search(r"\bexec\b", op):
        out.add("exec")
    return out


_NODST = ("global_store", "scratch_store", "buffer_store", "ds_write", "s_cbranch", "s_branch", "s_waitcnt",
          "s_nop", "s_setprio", "flat_store", "s_setpc", "s_barrier", "s_cmp", "s_bitcmp", "global_atomic",
          "s_endpgm", "s_sleep", "s_swappc")


def _parse(t: str):
    parts = t.split(None, 1)
    mn, ops = parts[0], (parts[1] if len(parts) > 1 else "")
    opl = [o.strip() for o in ops.split(",")]
    if mn == "s_swappc_b64":                     # s_swappc_b64 s[30:31] (return address), target
        dst, src = _regs(opl[0]), _regs(",".join(opl[1:]))
    elif mn.startswith(_NODST):
        dst, src = set(), _regs(ops)
        if mn in ("s_cbranch_execz", "s_cbranch_execnz"):
            src.add("exec")
        if mn.startswith("s_cbranch_vcc"):
            src.add("vcc")
    elif mn.startswith("v_cmp") and mn.endswith("_e32"):
        dst, src = {"vcc"}, _regs(",".join(opl[1:]))
    elif mn.startswith(("v_div_scale", "v_add_co", "v_sub_co", "v_addc_co", "v_subb_co", "v_mad_u64", "v_mad_i64")):
        dst, src = _regs(opl[0]) | _regs(opl[1]), _regs(",".join(opl[2:]))
    else:
        dst, src = _regs(opl[0]), _regs(",".join(opl[1:]))
    if "saveexec" in mn:
        dst.add("exec")
        src.add("exec")
    if mn.startswith("v_"):
        src.add("exec")
    if mn.startswith("v_div_fmas") or (mn.endswith("_e32") and mn.startswith(("v_cndmask", "v_addc", "v_subb"))):
        src.add("vcc")
    return mn, dst, src


def _kills(mn: str, dst: set) -> set:
    if mn.startswith(("global_load", "scratch_load", "ds_read", "buffer_load", "flat_load")):
        return set()
    if mn.startswith("v_") and not mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp", "v_div_scale",
                                                    "v_add_co", "v_sub_co")):
        return {x for x in dst if not x.startswith("v")}        # exec-masked VGPR write: partial
    return dst


def _function(lines, name):
    st = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    return [l.split(";")[0].rstrip() for l in lines[st:en]], st


def live_across_calls(asm: Path, kernel: str):
    lines = asm.read_text().split("\n")
    body, base = _function(lines, kernel)
    blocks, cur = [], None
    for i, l in enumerate(body):
        t = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):$", t)
        if m or cur is None:
            cur = {"name": m.group(1) if m else "entry", "ins": []}
            blocks.append(cur)
            if m:
                continue
        if t and not t.startswith(".") and not t.endswith(":"):
            cur["ins"].append((i, t))
    idx = {b["name"]: k for k, b in enumerate(blocks)}
    clob = {}
    csr = {f"s{k}" for k in range(33, 106)}
    for k, b in enumerate(blocks):
        succ, term = [], False
        for _, t in b["ins"]:
            mn = t.split()[0]
            if mn.startswith("s_cbranch") or mn == "s_branch":
                succ.append(idx[re.search(r"(\.LBB\d+_\d+)", t).group(1)])
                term |= mn == "s_branch"
            elif mn in ("s_endpgm", "s_setpc_b64"):
                term = True
        if not term and k + 1 < len(blocks):
            succ.append(k + 1)
        b["succ"] = succ
        b["p"] = []
        for i, t in b["ins"]:
            mn, d, s = _parse(t)
            callee = None
            if mn == "s_swappc_b64":
                for j in range(i - 1, max(0, i - 400), -1):
                    m = re.search(r"(_ZN\w+)@rel32@lo", body[j])
                    if m:
                        callee = m.group(1)
                        break
                if callee not in clob:
                    cb, _ = _function(lines, callee)
                    w = set()
                    for l in cb:
                        t2 = l.strip()
                        if t2 and not t2.startswith(".") and not t2.endswith(":"):
                            w |= _parse(t2)[1]
                    clob[callee] = {x for x in w if x.startswith("s") and x not in csr}
                d = d | clob[callee] | {"s30", "s31"}
            b["p"].append((i, t, mn, d, s, callee))
    live_in = [set() for _ in blocks]
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks) - 1, -1, -1):
            L = set().union(*[live_in[s] for s in blocks[k]["succ"]]) if blocks[k]["succ"] else set()
            for _, _, mn, d, s, _ in reversed(blocks[k]["p"]):
                L = (L - _kills(mn, d)) | s
            if L != live_in[k]:
                live_in[k], changed = L, True
    hits = []
    for k, b in enumerate(blocks):
        L = set().union(*[live_in[s] for s in b["succ"]]) if b["succ"] else set()
        for i, t, mn, d, s, callee in reversed(b["p"]):
            if callee:
                bad = sorted(x for x in L & d if x.startswith("s"))
                if bad:
                    hits.append((base + i + 1, callee, bad))
            L = (L - _kills(mn, d)) | s
    return hits


def main(argv):
    if argv and argv[0] == "--live":
        hits = live_across_calls(Path(argv[1]), argv[2])
        for line, callee, regs in hits:
            print(f"line {line}: call of {callee}: live across and clobbered: {' '.join(regs)}")
        print(f"{len(hits)} call(s) with SGPRs live across and clobbered")
        return
    so = Path(argv[0]) if argv else ROOT / "hybrid9_amd" / "lib" / "libh9g.so"
    c = calls_per_function(so)
    for name, n in sorted(c.items()):
        if n:
            print(f"{n:5d} {name}")
    print(f"{sum(c.values())} call instruction(s) in {len(c)} device function(s) of {so.name}")


if __name__ == "__main__":
    main(sys.argv[1:])
