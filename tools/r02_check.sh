#!/bin/bash
# Round-2 GPU check: smoke, the GPU tests, the driver's own bench command,
# and the list of PMC counters this box exposes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench (driver command)" && timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; rc=$?; tail -3 gpurun_out/bench_driver.log; [ $rc -eq 0 ] || exit $rc
echo "== counters" && timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "rc $?"; grep -c . gpurun_out/counters_list.txt
