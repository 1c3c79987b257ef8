#!/bin/bash
# A/B of the one-column kernel (the cell order's tail): tools/tail_probe.py
# on each library given, alternating.  usage: tools/ab_tail.sh ncell years lib...
set -o pipefail
n=$1; y=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib rep $rep"
    H9G_LIB=$lib H9G_KERNEL=pair1 timeout -k 10 200 python -u tools/tail_probe.py $n $y 2>&1 | grep -E "ms|probe" || exit 1
  done
done
