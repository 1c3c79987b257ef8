#!/bin/bash
# Round-5 GPU test pass: the -m gpu suite (optionally a -k filter) to
# gpurun_out/pytest_gpu_<tag>.txt.  Usage (on the box):
#   bash tools/r05_gpu_tests.sh <tag> [pytest -k expression]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r05}
mkdir -p gpurun_out
K=()
[ -n "$2" ] && K=(-k "$2")
echo "== pytest gpu $TAG"
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread "${K[@]}" > gpurun_out/pytest_gpu_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.txt; exit $rc
