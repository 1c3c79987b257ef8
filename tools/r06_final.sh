#!/bin/bash
# Round-6 GPU pass over the current tree (on the box, from the repo root).
#   PART=1  smoke, the -m gpu suite, the driver's bench line (reference cell
#           order, cpu_baseline) and a rocprofv3 kernel trace of the same
#           command (the ordered mode's launches, same build)
#   PART=2  rocprofv3 kernel stats and separate PMC passes of config 2's year
#           kernel (isolated year launches, the same kernel the ordered mode's
#           first passes run), summarised into profiles/pmc_<tag>.json, which
#           bench.py attaches to runs of the same build
#   PART=3  config 5: the L = 10 shard table, isolated and in cell order
#   PART=4  the forced-re-run build (H9G_FORCE_RERUN) on the parity and cell-order tests,
#           config 3 read from netCDF-4 files
# Usage: PART=n bash tools/r06_final.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r06}
mkdir -p gpurun_out
run() { # dir name, bench args, rocprof args...
  local name=$1 bargs=$2; shift 2
  echo "== $name"
  timeout -k 10 600 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $bargs \
    > $OUT/$name.log 2>&1
  local rc=$?; tail -c 200 $OUT/$name.log; echo; return $rc
}
case "${PART:-1}" in
1)
  echo "== smoke" && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1
  rc=$?; tail -2 gpurun_out/smoke_$TAG.txt; [ $rc -eq 0 ] || exit $rc
  echo "== pytest gpu" && timeout -k 10 700 python -u -m pytest tests -x -v -s -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_gpu_$TAG.txt 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu_$TAG.txt; [ $rc -eq 0 ] || exit $rc
  echo "== driver bench" && timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 \
    > gpurun_out/bench_${TAG}_driver.json 2> gpurun_out/bench_${TAG}_driver.err
  rc=$?; tail -c 400 gpurun_out/bench_${TAG}_driver.json; echo; [ $rc -eq 0 ] || exit $rc
  OUT=gpurun_out/prof_${TAG}_co
  mkdir -p $OUT
  run kt "--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated-line" --kernel-trace --stats || exit 1
  cp $OUT/kt/kt_kernel_stats.csv gpurun_out/${TAG}_cellorder_kernel_stats.csv
  ;;
2)
  OUT=gpurun_out/prof_$TAG
  mkdir -p $OUT
  ARGS=${PMC_ARGS:-"--order isolated --steps 20 --warmup 5 --no-cpu-baseline"}
  run kt "$ARGS" --kernel-trace --stats &&
  run sq1 "$ARGS" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU &&
  run sq2 "$ARGS" --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SALU SQ_LDS_BANK_CONFLICT &&
  run sq3 "$ARGS" --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 &&
  run sq4 "$ARGS" --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES &&
  run tcc "$ARGS" --pmc TCC_HIT_sum TCC_MISS_sum &&
  run fetch "$ARGS" --pmc FETCH_SIZE &&
  run write "$ARGS" --pmc WRITE_SIZE || exit 1
  python3 tools/pmc_summary.py $TAG config2 > $OUT/summary.txt 2>&1 || { tail -5 $OUT/summary.txt; exit 1; }
  cp profiles/pmc_$TAG.json profiles/${TAG}_kernel_stats.csv gpurun_out/
  ;;
3)
  echo "== l10 shards (isolated, chosen kernel)" && L10_KINDS=auto timeout -k 10 300 python3 -u tools/l10_shards.py \
    > gpurun_out/${TAG}_l10_shards.txt 2>&1
  rc=$?; cat gpurun_out/${TAG}_l10_shards.txt; [ $rc -eq 0 ] || exit $rc
  echo "== l10 shards (cell order)" && timeout -k 10 700 python3 -u tools/l10_shards.py --ordered \
    > gpurun_out/${TAG}_l10_shards_ordered.txt 2>&1
  rc=$?; cat gpurun_out/${TAG}_l10_shards_ordered.txt; exit $rc
  ;;
4)
  if [ -f hybrid9_amd/lib/libh9g_frr.so ]; then
    echo "== forced re-run build" && H9G_LIB=hybrid9_amd/lib/libh9g_frr.so timeout -k 10 700 python -u -m pytest \
      tests/test_gpu_parity.py tests/test_cell_order.py -x -v -m gpu -p no:cacheprovider --timeout 300 \
      --timeout-method thread -k "golden or stop or nan or config5 or cell_order" > gpurun_out/pytest_frr_$TAG.txt 2>&1
    rc=$?; tail -2 gpurun_out/pytest_frr_$TAG.txt; [ $rc -eq 0 ] || exit $rc
  fi
  echo "== config3 nc4" && timeout -k 10 400 python3 -u bench.py --workload config3 --forcing nc4 --steps 3 --warmup 1 \
    > gpurun_out/bench_${TAG}_config3_nc4.json 2> gpurun_out/bench_${TAG}_config3_nc4.err
  rc=$?; tail -c 600 gpurun_out/bench_${TAG}_config3_nc4.json; echo; exit $rc
  ;;
esac
