#!/bin/bash
# Bench lines of every workload (1 GPU) after the driver's own command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() { local tag=$1; shift; echo "== $tag: $*"; timeout -k 10 600 python3 -u bench.py "$@" > gpurun_out/cfg_$tag.log 2>&1 || { tail -5 gpurun_out/cfg_$tag.log; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cfg_$tag.log').read().strip().splitlines()[-1]); print('$tag', '%.4e'%d['value'], '%.1f ms/step'%d['ms_per_step'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'], 'frac %.3f'%d['roofline']['frac'], 'stopped', d['cells_stopped'], 'cpu', d['cpu_baseline'] and '%.3e'%d['cpu_baseline']['value'])"; }
run config2 --gpus 1 --steps 20 --warmup 5 &&
run config3 --workload config3 --steps 10 --warmup 2 --no-cpu-baseline &&
run config4 --workload config4 --no-cpu-baseline &&
run config5 --workload config5 --steps 4 --warmup 1
