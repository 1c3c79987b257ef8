#!/bin/bash
# The driver's bench command, timed, then the PMC counter list of the box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench (driver command)"; t0=$(date +%s.%N)
timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1; rc=$?
echo "wall $(echo "$(date +%s.%N) - $t0" | bc) s rc=$rc"; tail -c 3000 gpurun_out/bench_driver.log; [ $rc -eq 0 ] || exit $rc
echo "== counters"; timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "rc $?"
