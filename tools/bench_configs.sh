set -o pipefail
cd "$GRAFT_REPO_ROOT"
for w in config3 config5; do
  for k in pair solo; do
    H9G_KERNEL=$k timeout -k 10 300 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${w}_$k.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_${w}_$k.log').read().strip().splitlines()[-1]); print('$w $k', d['roofline']['kernel'], '%.3e'%d['value'], '%.1f ms'%d['roofline']['kernel_ms_per_launch'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
