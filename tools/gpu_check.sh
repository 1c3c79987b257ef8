set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke" && timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; cat gpurun_out/smoke.log | tail -5; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu" && timeout -k 10 1200 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench" && timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; exit $rc
