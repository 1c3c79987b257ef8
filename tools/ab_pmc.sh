#!/bin/bash
# A/B of alternative builds (hybrid9_amd/lib/libh9g_<tag>.so, "base" =
# libh9g.so) on the driver's bench command, with the HBM traffic of each:
# kernel time, then separate FETCH_SIZE and WRITE_SIZE rocprofv3 passes
# (MI355X_MICROARCH.md: one counter block per pass).
# Usage: bash tools/ab_pmc.sh tag...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ARGS="--steps 20 --warmup 5 --no-cpu-baseline"
for t in "$@"; do
  lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
  out=gpurun_out/abp_$t${AB_SUFFIX:-}; mkdir -p $out
  for c in FETCH_SIZE WRITE_SIZE; do
    H9G_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $c -d $out/$c -o $c --output-format csv -- python3 bench.py $ARGS \
      > $out/$c.log 2>&1 || { echo "$t $c pass failed"; tail -3 $out/$c.log; exit 1; }
  done
  python3 - "$t" "$out" <<'EOF'
import csv, glob, json, sys
t, out = sys.argv[1], sys.argv[2]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"{out}/{c}/*counter_collection.csv") + glob.glob(f"{out}/{c}/*/*counter_collection.csv")
         for r in csv.DictReader(open(f)) if "h9g_pair_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c]
    res[c] = sum(v) / len(v) * 1024 * (2 if c == "FETCH_SIZE" else 1) / 1e9 if v else None
line = [l for l in open(f"{out}/WRITE_SIZE.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"{t}{__import__('os').environ.get('AB_SUFFIX', '')}: {d['roofline']['kernel_ms_per_launch']:.2f} ms kernel, fetch {res['FETCH_SIZE']:.2f} GB, "
      f"write {res['WRITE_SIZE']:.2f} GB per launch")
EOF
done
