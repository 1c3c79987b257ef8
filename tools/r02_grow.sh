#!/bin/bash
# GROW-on workloads: per-year kernel time, exact re-run counts, round-1 library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in count r01 base; do
  l=hybrid9_amd/lib/libh9g_$lib.so; [ $lib = base ] && l=hybrid9_amd/lib/libh9g.so
  H9G_LIB=$l timeout -k 10 300 python3 -u bench.py --workload config3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/grow_$lib.log 2>&1 || { tail -3 gpurun_out/grow_$lib.log; exit 1; }
  grep "exact" gpurun_out/grow_$lib.log | tail -1
  python3 -c "import json; d=json.loads(open('gpurun_out/grow_$lib.log').read().strip().splitlines()[-1]); print('$lib', '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
done
H9G_LIB=hybrid9_amd/lib/libh9g_r01.so timeout -k 10 300 python3 -u bench.py --workload config3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/grow_r01_k3.log 2>&1 && python3 -c "import json; d=json.loads(open('gpurun_out/grow_r01_k3.log').read().strip().splitlines()[-1]); print('r01 K=3 W=1', '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
