#!/bin/bash
# One GPU pass over the committed tree: smoke, the -m gpu suite, then the
# driver's bench command.  Usage (on the box): bash tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-chk}; shift
BARGS=${@:---gpus 1 --steps 20 --warmup 5}
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu" && timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "== bench $BARGS" && timeout -k 10 600 python -u bench.py $BARGS > gpurun_out/bench_$TAG.log 2>&1; rc=$?; tail -c 1500 gpurun_out/bench_$TAG.log; exit $rc
