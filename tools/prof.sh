#!/bin/bash
# rocprofv3 passes over the bench (kernel trace + stats, then separate PMC
# passes as MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes).
# Usage: bash tools/prof.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS=${@:---steps 2 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() { # name, rocprof args...
  local name=$1; shift
  echo "== $name"
  timeout -k 10 600 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; tail -2 $OUT/$name.log; return $rc
}
run kt --kernel-trace --stats &&
run sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU &&
run sq2 --pmc SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SALU SQ_LDS_BANK_CONFLICT &&
run sq3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 &&
run sq4 --pmc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_WAVES &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE
