#!/bin/bash
# One GPU pass on the box: the -m gpu suite, smoke, the default bench line.
# usage: tools/gpu_pass.sh TAG [extra bench args]
set -o pipefail
tag=$1; shift
out=gpurun_out
mkdir -p $out
TESTS=${TESTS:-tests}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread \
  > $out/pytest_gpu_$tag.txt 2>&1 || { tail -30 $out/pytest_gpu_$tag.txt; exit 1; }
tail -3 $out/pytest_gpu_$tag.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke_$tag.txt 2>&1 || { cat $out/smoke_$tag.txt; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $out/bench_${tag}_driver.json 2> $out/bench_${tag}_driver.err || { tail $out/bench_${tag}_driver.err; exit 1; }
python - "$out/bench_${tag}_driver.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value %.4g ms/yr %.1f kernel %s" % (d["value"], d["ms_per_step"], d["roofline"]["kernel_ms_per_launch"]))
print("launches", d.get("launches"))
print("cell_order", json.dumps(d.get("cell_order", {}))[:600])
print("isolated", d.get("isolated", {}).get("ms_per_step"))
PY
