#!/bin/bash
# Device assembly and final MIR (with branch probabilities) of the config-2
# pair kernel alone (h9g.hip -DH9G_ISA_ONLY): ~15 s instead of the
# library's 4 minutes.  Usage: bash tools/isa_pair.sh <tag> [extra hipcc flags]
# Then: python tools/isa_mix.py /tmp/isa/<tag> [--ops] [--blocks]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-base}; shift || true
mkdir -p /tmp/isa
K=${ISA_K:-_Z15h9g_pair_kernelILi8EN3h9k4GeoCILi8ELi48EEEEv5KArgsT0_}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt --cuda-device-only -S -DH9G_ISA_ONLY -DH9G_ISA_MARK "$@" \
  -o /tmp/isa/$TAG.s "$ROOT/hybrid9_amd/csrc/h9g.hip" \
  -mllvm -print-after=branch-relaxation -mllvm -filter-print-funcs=$K 2> /tmp/isa/$TAG.mir
grep -A12 "\.name: *$K" /tmp/isa/$TAG.s | grep -E "spill_count|vgpr_count|sgpr_count" | tr -s ' ' | tr '\n' ' '
echo
