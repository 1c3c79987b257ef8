#!/bin/bash
# Alternating A/B of library builds on the config-2 bench, REPS rounds over
# the tags (hybrid9_amd/lib/libh9g_<tag>.so, "base" = libh9g.so); prints
# kernel ms per launch and the last year's diagnostics digest (bit-identical
# results give identical FP64 sums).  Usage: REPS=2 bash tools/ab_alt.sh tag[@VAR=val]...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for spec in "$@"; do
    t=${spec%%@*}; envs=""; [ "$spec" != "$t" ] && envs=${spec#*@}   # tag@VAR=val: run with that env
    lib=hybrid9_amd/lib/libh9g_$t.so; [ "$t" = base ] && lib=hybrid9_amd/lib/libh9g.so
    t=${spec//[@=]/_}
    env $envs H9G_LIB=$lib timeout -k 10 300 python3 bench.py ${AB_ARGS:---steps 6 --warmup 2} --no-cpu-baseline \
      > gpurun_out/abalt_${t}_$r.log 2>&1 || { tail -5 gpurun_out/abalt_${t}_$r.log; exit 1; }
    python3 -c "import json,hashlib; d=json.loads(open('gpurun_out/abalt_${t}_$r.log').read().strip().splitlines()[-1]); print('$r $t', '%.2f ms'%d['roofline']['kernel_ms_per_launch'], '%.2f ms/step'%d['ms_per_step'], hashlib.sha1(json.dumps(d['diagnostics_last_year'],sort_keys=True).encode()).hexdigest()[:10])"
  done
done
