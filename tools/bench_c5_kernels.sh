set -o pipefail
cd "$GRAFT_REPO_ROOT"
for k in pair solo mixed; do
  H9G_KERNEL=$k timeout -k 10 300 python3 -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$k.log 2>&1 || { echo "c5 $k failed"; tail -3 gpurun_out/c5_$k.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c5_$k.log').read().strip().splitlines()[-1]); print('config5 $k', d['roofline']['kernel'], '%.4e'%d['value'], '%.1f ms/step'%d['ms_per_step'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
done
