#!/bin/bash
# Round-3 bench lines of configs 3 and 4 (1 GPU) and the L=10 shard timings
# of strong scaling (tools/l10_shards.py: pair / solo / mixed / auto per shard).
# Usage (on the box): bash tools/r03_configs.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03e}
mkdir -p gpurun_out
run() { local tag=$1; shift; echo "== $tag: $*"; timeout -k 10 600 python3 -u bench.py "$@" > gpurun_out/bench_${TAG}_$tag.log 2>&1 || { tail -5 gpurun_out/bench_${TAG}_$tag.log; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_$tag.log').read().strip().splitlines()[-1]); print('$tag', '%.4e'%d['value'], '%.1f ms/step'%d['ms_per_step'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'], 'frac %.3f'%d['roofline']['frac'], 'stopped', d['cells_stopped'])"; }
run config3 --workload config3 --steps 10 --warmup 2 --no-cpu-baseline &&
run config4 --workload config4 --no-cpu-baseline &&
echo "== l10 shards" && timeout -k 10 900 python3 -u tools/l10_shards.py > gpurun_out/${TAG}_l10_shards.txt 2>&1; rc=$?; cat gpurun_out/${TAG}_l10_shards.txt; exit $rc
