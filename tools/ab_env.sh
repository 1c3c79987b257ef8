#!/bin/bash
# A/B environment settings on the driver's bench command (no CPU baseline).
# Usage: bash tools/ab_env.sh "H9G_SORT=0" "H9G_SORT=1" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abenv_$i.log 2>&1 || { tail -5 gpurun_out/abenv_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abenv_$i.log').read().strip().splitlines()[-1]); print('$e', '%.4e'%d['value'], '%.1f ms/step'%d['ms_per_step'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'], 'stopped', d['cells_stopped'])"
done
