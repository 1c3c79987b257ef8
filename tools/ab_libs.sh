#!/bin/bash
# A/B alternative builds (hybrid9_amd/lib/libh9g_<tag>.so, "base" = libh9g.so):
# bit-exact goldens, STOP reproduction, the NaN-parameter cells and the soil
# build on the pair kernel, then the driver's bench command.  Stops at the
# first failing step.  Usage: bash tools/ab_libs.sh tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  H9G_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_soil.py -q -m gpu \
     -p no:cacheprovider --timeout 120 --timeout-method thread \
     -k "(golden or stop or config2 or nan or soil) and not solo and not mixed" > gpurun_out/abl_$t.pytest 2>&1
  rc=$?; p=$(tail -1 gpurun_out/abl_$t.pytest); echo "$t pytest rc=$rc: $p"
  if [ $rc -ne 0 ]; then
    grep -h "^FAILED" gpurun_out/abl_$t.pytest | head -5
    # plain test failures: go on with the next build; anything else (a GPU
    # fault, a crash, a time limit) ends the run here
    if [ $rc -eq 1 ] && ! grep -qi "illegal memory\|memory access fault\|hipError" gpurun_out/abl_$t.pytest; then continue; fi
    exit $rc
  fi
  H9G_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abl_$t.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$t bench rc=$rc"; tail -3 gpurun_out/abl_$t.log; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/abl_$t.log').read().strip().splitlines()[-1]); print('$t', '%.4e'%d['value'], '%.2f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
done
