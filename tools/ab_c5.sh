#!/bin/bash
# Per-kernel times of config 5 (solo + pair L=10) for A/B builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; srt=1
  [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  [ "$t" = nosort ] && lib=hybrid9_amd/lib/libh9g.so && srt=0
  H9G_SORT=$srt H9G_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5_$t -o c5 --output-format csv -- python3 bench.py --workload config5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$t.log 2>&1 || { echo "$t failed"; tail -3 gpurun_out/c5_$t.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5_$t.log').read().strip().splitlines()[-1]); print('$t', '%.4e'%d['value'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
  f=$(ls gpurun_out/c5_$t/*/c5_kernel_stats.csv 2>/dev/null || ls gpurun_out/c5_$t/c5_kernel_stats.csv); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'h9g' in r['Name']: print('   ', r['Name'][:60], r['Calls'], '%.1f ms avg'%(float(r['AverageNs'])/1e6))"
done
