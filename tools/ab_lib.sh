#!/bin/bash
# A/B alternative builds of libh9g (hybrid9_amd/lib/libh9g_<tag>.so) on the
# config-2 bench.  Usage: bash tools/ab_lib.sh tag...   ("base" = libh9g.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  H9G_LIB=$lib timeout -k 10 300 python3 bench.py ${AB_ARGS:---steps 2 --warmup 1} --no-cpu-baseline > gpurun_out/ablib_$t.log 2>&1 || exit $?
  grep "stamps\|exact re-runs" gpurun_out/ablib_$t.log | tail -2
  python3 -c "import json; d=json.loads(open('gpurun_out/ablib_$t.log').read().strip().splitlines()[-1]); print('$t', d['roofline']['kernel'], '%.3e'%d['value'], '%.1f ms'%d['roofline']['kernel_ms_per_launch'])"
done
