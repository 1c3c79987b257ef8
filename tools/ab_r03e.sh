#!/bin/bash
# Round 3e: branch counts of the driver's years (H9G_COUNT_BRANCH builds named
# in CNT, e.g. CNT="cnt cntx"), then an A/B of the candidate builds on the
# config-2 bench.  Usage: CNT="..." bash tools/ab_r03e.sh tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in $CNT; do
  H9G_LIB=hybrid9_amd/lib/libh9g_$c.so timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 5 --no-cpu-baseline \
    > gpurun_out/cnt_$c.log 2>&1 || exit $?
  echo "$c: $(grep 'branch counts' gpurun_out/cnt_$c.log | tail -1)"
done
bash tools/ab_lib.sh "$@"
