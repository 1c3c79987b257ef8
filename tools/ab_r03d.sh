set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/ab_pmc.sh xcd && bash tools/ab_libs.sh xcd || exit 1
H9G_LIB=hybrid9_amd/lib/libh9g_p10.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "config5" > gpurun_out/p10.pytest 2>&1; rc=$?; echo "p10 pytest rc=$rc $(tail -1 gpurun_out/p10.pytest)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in pair mixed; do
H9G_LIB=hybrid9_amd/lib/libh9g_p10.so H9G_KERNEL=$k timeout -k 10 300 python3 -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_p10_$k.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/c5_p10_$k.log').read().strip().splitlines()[-1]); print('config5 p10 $k', d['roofline']['kernel'], '%.4e'%d['value'], '%.1f ms kernel'%d['roofline']['kernel_ms_per_launch'])"
done
