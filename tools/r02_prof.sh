#!/bin/bash
# rocprofv3 kernel stats + typed VALU / wait PMC passes over the driver's
# bench command (years 1906-1925 timed), then the phase-stamp and
# exact-re-run measurement builds.  Usage: bash tools/r02_prof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 20 --warmup 5 --no-cpu-baseline"
run() { # name, rocprof args...
  local name=$1; shift
  echo "== $name"
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; tail -c 400 $OUT/$name.log; echo; return $rc
}
run kt --kernel-trace --stats &&
run v1 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 &&
run v2 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES &&
run v3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
echo "== stamps" && H9G_LIB=hybrid9_amd/lib/libh9g_stamps.so timeout -k 10 300 python3 bench.py $ARGS > $OUT/stamps.log 2>&1 && grep "stamps" $OUT/stamps.log | tail -3 &&
echo "== count" && H9G_LIB=hybrid9_amd/lib/libh9g_count.so timeout -k 10 300 python3 bench.py $ARGS > $OUT/count.log 2>&1 && grep "exact" $OUT/count.log | tail -3
