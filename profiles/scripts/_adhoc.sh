set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_adhoc.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL|^E " gpurun_out/pytest_gpu_adhoc.log | head -30; tail -30 gpurun_out/pytest_gpu_adhoc.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_adhoc.log
for cfg in c2 c2 c3 c4; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 60 --no-cpu-baseline > gpurun_out/g_$cfg.json 2>gpurun_out/g_$cfg.err || { tail gpurun_out/g_$cfg.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/g_$cfg.json'));print('$cfg', round(r['value']), 'step', round(r['ms_per_step']*1e3,1), 'p50', round(r['p50_ms']*1e3,1), 'scan', round(r['roofline']['avg_launch_ms']*1e3,1), 'pipe', round(r['pipeline_ms']*1e3,1), 'fb', r['fallback_queries_total'])"
done
