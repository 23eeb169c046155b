set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_adhoc.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL|^E " gpurun_out/pytest_gpu_adhoc.log | head -40; tail -40 gpurun_out/pytest_gpu_adhoc.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_adhoc.log
for a in "c2 bf16x3 0"; do
  set -- $a
  timeout -k 10 200 python -u bench.py --config $1 --precision $2 --scan-variant $3 --steps 60 --no-cpu-baseline > gpurun_out/b_$1_$2_$3.json 2>gpurun_out/b_$1_$2_$3.err || { tail gpurun_out/b_$1_$2_$3.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/b_$1_$2_$3.json'));print('$a', round(r['value']), 'step', round(r['ms_per_step']*1e3,1), 'p50', round(r['p50_ms']*1e3,1), 'scan', round(r['roofline']['avg_launch_ms']*1e3,1), 'pipe', round(r['pipeline_ms']*1e3,1), 'fb', r['fallback_queries_total'])"
done
