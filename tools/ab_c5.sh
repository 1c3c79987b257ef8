#!/bin/bash
# A/B of config 5's year kernel (isolated order, 2 timed years) between libraries, alternating.
# usage: tools/ab_c5.sh lib...
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for lib in "$@"; do
  H9G_LIB=$lib timeout -k 10 300 python -u bench.py --workload config5 --order isolated --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/ab_c5.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_c5.json').read().strip().splitlines()[-1]); print('$lib', round(d['ms_per_step'],1), round(d['roofline']['kernel_ms_per_launch'],1), d['diagnostics_last_year']['theta_total_sum'])"
done; done
