#!/bin/bash
# Round-5 GPU pass over the final tree: smoke, the -m gpu suite (cell-order
# tests first), rocprofv3 kernel stats and PMC passes of config 2 and config 5
# with their summaries and the driver's bench line (tools/r03_final.sh), the
# configs 3/4 lines, the config-3 netCDF-4 ingest line (with the read's stage
# profile) and the L=10 shard table.
# Usage (on the box): bash tools/r05_final.sh <tag> [skip-tests]
# PART=1: up to the forced re-run suite; PART=2: the configs and the shard
# table only (two calls, each within gpurun's limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05}
mkdir -p gpurun_out
if [ "${PART:-1}" = 1 ]; then
if [ "$2" != "skip-tests" ]; then
  echo "== cell order" && timeout -k 10 600 python -u -m pytest tests/test_cell_order.py -x -v -s -m gpu \
    -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/pytest_co_$TAG.txt 2>&1
  rc=$?; grep -E "passes|bound" gpurun_out/pytest_co_$TAG.txt | tail -6; [ $rc -eq 0 ] || exit $rc
fi
bash tools/r03_final.sh "$TAG" "$2" || exit $?
if [ -f hybrid9_amd/lib/libh9g_frr.so ]; then
  echo "== forced re-run build" && H9G_LIB=hybrid9_amd/lib/libh9g_frr.so timeout -k 10 600 python -u -m pytest \
    tests/test_gpu_parity.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread \
    -k "golden or stop or nan or config5" > gpurun_out/pytest_frr_$TAG.txt 2>&1
  rc=$?; tail -2 gpurun_out/pytest_frr_$TAG.txt; [ $rc -eq 0 ] || exit $rc
fi
[ -n "$PART" ] && exit 0
fi
run() { local tag=$1; shift; echo "== $tag: $*"; timeout -k 10 600 python3 -u bench.py "$@" > gpurun_out/bench_${TAG}_$tag.log 2>&1 || { tail -5 gpurun_out/bench_${TAG}_$tag.log; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_$tag.log').read().strip().splitlines()[-1]); print('$tag', '%.4e'%d['value'], '%.1f ms/step'%d['ms_per_step'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'], 'frac %.3f'%d['roofline']['frac'], 'stopped', d['cells_stopped'])"; }
run config3 --workload config3 --steps 10 --warmup 2 --no-cpu-baseline &&
run config4 --workload config4 --no-cpu-baseline --no-cell-order-line &&
run config3_nc4 --workload config3 --forcing nc4 --steps 3 --warmup 1 &&
echo "== l10 shards" && L10_KINDS=pair,pair2,pair11,auto timeout -k 10 900 python3 -u tools/l10_shards.py > gpurun_out/${TAG}_l10_shards.txt 2>&1; rc=$?; cat gpurun_out/${TAG}_l10_shards.txt; exit $rc
