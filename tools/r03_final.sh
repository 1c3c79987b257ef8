#!/bin/bash
# Round-3 GPU pass over the current tree: smoke, the -m gpu suite, the
# rocprofv3 kernel stats and PMC passes of the driver's config-2 command
# (plus an instruction-cache pass), their summary (profiles/pmc_<tag>.json,
# copied to gpurun_out/), then the driver's bench line with those counters
# attached (same build), and config 5's line, kernel stats and PMC.
# Usage (on the box): bash tools/r03_final.sh <tag> [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03e}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  echo "== smoke" && timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
  echo "== pytest gpu" && timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_gpu_$TAG.txt 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu_$TAG.txt; [ $rc -eq 0 ] || exit $rc
fi
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-cell-order-line"
run() { # dir name, bench args, rocprof args...
  local name=$1 bargs=$2; shift 2
  echo "== $name"
  timeout -k 10 600 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $bargs \
    > $OUT/$name.log 2>&1
  local rc=$?; tail -c 300 $OUT/$name.log; echo; return $rc
}
run kt "$ARGS" --kernel-trace --stats &&
run sq1 "$ARGS" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU &&
run sq2 "$ARGS" --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SALU SQ_LDS_BANK_CONFLICT &&
run sq3 "$ARGS" --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 &&
run sq4 "$ARGS" --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES &&
run ic "$ARGS" --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH &&
run fetch "$ARGS" --pmc FETCH_SIZE &&
run write "$ARGS" --pmc WRITE_SIZE || exit 1
python3 tools/pmc_summary.py $TAG config2 > $OUT/summary.txt 2>&1 || { tail -5 $OUT/summary.txt; exit 1; }
cp profiles/pmc_$TAG.json profiles/${TAG}_kernel_stats.csv gpurun_out/
echo "== driver bench" && timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_driver.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_${TAG}_driver.log; echo; [ $rc -eq 0 ] || exit $rc
# config 5 (0.25 deg, L = 10): bench line, kernel stats and VALU counters
C5="--workload config5 --steps 2 --warmup 1 --no-cpu-baseline"
OUT=gpurun_out/prof_${TAG}_c5
mkdir -p $OUT
run kt "$C5" --kernel-trace --stats &&
run sq1 "$C5" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU &&
run sq4 "$C5" --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES &&
run fetch "$C5" --pmc FETCH_SIZE &&
run write "$C5" --pmc WRITE_SIZE || exit 1
python3 tools/pmc_summary.py ${TAG}_c5 config5 > $OUT/summary.txt 2>&1 || { tail -5 $OUT/summary.txt; exit 1; }
cp profiles/pmc_${TAG}_c5.json profiles/${TAG}_c5_kernel_stats.csv gpurun_out/
echo "== config5 bench" && timeout -k 10 600 python -u bench.py --workload config5 --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_config5.log 2>&1
rc=$?; tail -c 600 gpurun_out/bench_${TAG}_config5.log; echo; exit $rc
