#!/bin/bash
# Round-5 GPU pass: smoke, the cell-order tests first (printing their decade
# passes), then the whole -m gpu suite and the driver's bench line.
# Usage (on the box): bash tools/r05_pass.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05}
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
echo "== cell order" && timeout -k 10 600 python -u -m pytest tests/test_cell_order.py -x -v -s -m gpu -p no:cacheprovider \
  --timeout 500 --timeout-method thread > gpurun_out/pytest_co_$TAG.txt 2>&1
rc=$?; grep -E "passes|bound|PASS|FAIL" gpurun_out/pytest_co_$TAG.txt | tail -8; [ $rc -eq 0 ] || exit $rc
bash tools/r05_gpu_tests.sh $TAG "${2:-not cell_order}" || exit $?
echo "== driver bench" && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_driver.log 2>&1
rc=$?; tail -c 800 gpurun_out/bench_${TAG}_driver.log; [ $rc -eq 0 ] || exit $rc
echo "== cell-order bench" && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 10 --order cell \
  --no-cpu-baseline > gpurun_out/bench_${TAG}_cellorder.log 2>&1
rc=$?; tail -c 1500 gpurun_out/bench_${TAG}_cellorder.log; [ $rc -eq 0 ] || exit $rc
if [ -f hybrid9_amd/lib/libh9g_aq.so ]; then     # day-level water-table record (tools/aq_sort.py)
  echo "== aq dump" && H9G_LIB=hybrid9_amd/lib/libh9g_aq.so H9G_AQ_DUMP=gpurun_out/aq_$TAG.bin timeout -k 10 300 \
    python -u bench.py --steps 8 --warmup 0 --no-cpu-baseline > gpurun_out/bench_${TAG}_aq.log 2>&1
  rc=$?; tail -c 300 gpurun_out/bench_${TAG}_aq.log; exit $rc
fi
