#!/bin/bash
# Round-2 final GPU pass: same-box A/B of the last change (prev = previous
# commit's library), smoke + GPU tests, every workload's bench line (the
# driver's config-2 command first), then the rocprofv3 kernel stats, PMC
# passes, phase stamps and exact re-run counts of the config-2 run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r02e}
if [ -f hybrid9_amd/lib/libh9g_prev.so ]; then bash tools/ab_sched.sh prev base prev base || exit 1; fi
echo "== smoke" && timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "== pytest gpu" && timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/r02_configs.sh || exit 1
bash tools/r02_prof.sh $TAG
