#!/bin/bash
# The GROW-on configurations in the reference's cell order (bench.py
# default order) on one GPU: config 3 (1911-1930 after 1901-1910), config 4
# (the 30-year spin-up 1901-1930), config 5 (0.25 deg, L = 10).
# usage: tools/ordered_configs.sh TAG [workloads...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
for wl in ${@:-config3 config4}; do
  timeout -k 10 500 python -u bench.py --workload $wl --no-cpu-baseline --no-isolated-line \
    > gpurun_out/bench_${tag}_${wl}_cell.json 2> gpurun_out/bench_${tag}_${wl}_cell.err || { tail gpurun_out/bench_${tag}_${wl}_cell.err; exit 1; }
  python - gpurun_out/bench_${tag}_${wl}_cell.json $wl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "%.4g cell-steps/s" % d["value"], "ms/yr %.1f" % d["ms_per_step"], "launches", d["launches"])
for c in d["cell_order"]["calls"]:
    print("  launch_cells", c["launch_cells"][:40], "overlap", c["overlap"])
PY
done
