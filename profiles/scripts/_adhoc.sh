set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_adhoc.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_adhoc.log | head -20; tail -30 gpurun_out/pytest_gpu_adhoc.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_adhoc.log
export TMPDIR=/tmp
for cfg in c2 c3 c4 c1; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_adhoc_$cfg.json 2> gpurun_out/bench_adhoc_$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/bench_adhoc_$cfg.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_adhoc_$cfg.json'));r=d['roofline'];print('$cfg', round(d['value']), 'qps step', round(d['ms_per_step'],3), 'scan', round(r['avg_launch_ms'],3), 'pipe', round(d['pipeline_ms'],3), r['bound'], round(r['frac'],3), 'hbm', round(r['hbm_gbs']), 'tf', round(r['mfma_tflops']), 'fallback', d['fallback_queries_total'], 'ovf', d['fallback_list_overflow'])"
done
