#!/bin/bash
# A/B builds on config 2 (driver command) and config 3 (GROW on, 10 years).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  for wl in config2 config3; do
    a="--steps 20 --warmup 5"; [ $wl = config3 ] && a="--workload config3 --steps 10 --warmup 2"
    H9G_LIB=$lib timeout -k 10 300 python3 bench.py $a --no-cpu-baseline > gpurun_out/abg_${t}_$wl.log 2>&1 || { echo "$t $wl failed"; tail -3 gpurun_out/abg_${t}_$wl.log; continue; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abg_${t}_$wl.log').read().strip().splitlines()[-1]); print('$t $wl', '%.4e'%d['value'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
  done
done
