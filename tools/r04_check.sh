#!/bin/bash
# Round-4 GPU pass: the exhaustive Markstein sweep, the -m gpu suite, the
# driver's config-2 bench and the config-3 netCDF-4 ingest bench.
# Usage (on the box): bash tools/r04_check.sh <tag> [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out
[ "${MK:-1}" = 0 ] || { echo "== markstein" && timeout -k 10 300 tools/_build/markstein_exhaustive > gpurun_out/markstein_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/markstein_$TAG.txt; [ $rc -eq 0 ] || exit $rc; }
if [ "$2" != "skip-tests" ]; then
  echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_gpu_$TAG.txt 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu_$TAG.txt; [ $rc -eq 0 ] || exit $rc
fi
echo "== driver bench" && timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}_driver.log 2>&1
rc=$?; tail -c 300 gpurun_out/bench_${TAG}_driver.log; echo; [ $rc -eq 0 ] || exit $rc
if [ "${FETCH:-0}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $c" && timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/prof_${TAG}_$c -o $c --output-format csv -- \
      python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${TAG}_$c.log 2>&1 || exit $?
  done
fi
echo "== config3 nc4" && timeout -k 10 400 python -u bench.py --workload config3 --forcing nc4 --steps 3 --warmup 1 > gpurun_out/bench_${TAG}_config3_nc4.log 2>&1
rc=$?; tail -c 900 gpurun_out/bench_${TAG}_config3_nc4.log; echo; exit $rc
