#!/bin/bash
# A/B of L=10 builds on the strong-scaling shards (tools/l10_shards.py):
# the product library and variants hybrid9_amd/lib/libh9g_<tag>.so.
# Usage: L10_KINDS=pair2 L10_WORLDS=8 bash tools/r04_l10ab.sh base tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  echo "== $t"
  H9G_LIB=$lib timeout -k 10 300 python3 -u tools/l10_shards.py > gpurun_out/l10ab_$t.txt 2>&1 || { cat gpurun_out/l10ab_$t.txt; exit 1; }
  cat gpurun_out/l10ab_$t.txt
done
