#!/bin/bash
# A/B the year-kernel variants on the config-2 bench (no CPU baseline).
# Usage: bash tools/ab.sh [variants...]   (default: pair solo)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for k in ${@:-pair solo}; do
  H9G_KERNEL=$k timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$k.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$k.log').read().strip().splitlines()[-1]); print('$k', d['roofline']['kernel'], '%.3e'%d['value'], '%.1f ms'%d['roofline']['kernel_ms_per_launch'])"
done
