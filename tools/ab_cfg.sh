#!/bin/bash
# A/B library builds on one workload.  Usage: bash tools/ab_cfg.sh workload tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
w=$1; shift
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  H9G_LIB=$lib timeout -k 10 300 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/abcfg_${w}_$t.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/abcfg_${w}_$t.log').read().strip().splitlines()[-1]); print('$w $t', d['roofline']['kernel'], '%.3e'%d['value'], '%.1f ms'%d['roofline']['kernel_ms_per_launch'])"
done
