#!/bin/bash
# A/B alternative builds (hybrid9_amd/lib/libh9g_<tag>.so, "base" = libh9g.so):
# bit-exact goldens + STOP reproduction on the pair kernel, then the
# driver's bench command.  Usage: bash tools/ab_libs.sh tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  H9G_LIB=$lib timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider \
     -k "(golden or stop or config2) and not solo and not mixed" > gpurun_out/abl_$t.pytest 2>&1
  p=$(tail -1 gpurun_out/abl_$t.pytest)
  H9G_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abl_$t.log 2>&1 || { echo "$t bench failed"; tail -3 gpurun_out/abl_$t.log; continue; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abl_$t.log').read().strip().splitlines()[-1]); print('$t', '%.4e'%d['value'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'], '| $p')"
done
