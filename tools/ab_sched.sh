#!/bin/bash
# A/B library builds (hybrid9_amd/lib/libh9g_<tag>.so; "base" = libh9g.so) on
# the driver's config-2 years (warmup 5 = 1901-1905, then 10 timed years).
# Usage: bash tools/ab_sched.sh tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  H9G_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/abs_$t.log 2>&1 || { echo "$t failed"; tail -3 gpurun_out/abs_$t.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abs_$t.log').read().strip().splitlines()[-1]); print('$t', '%.4e'%d['value'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
done
