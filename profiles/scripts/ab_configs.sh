#!/bin/bash
# GPU parity tests, then bench lines for C2, C3, C4 (N=1).  Usage: bash profiles/scripts/ab_configs.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
for c in c2 c3 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_${TAG}_$c.json 2> gpurun_out/bench_${TAG}_$c.err || { echo "bench $c failed"; tail -30 gpurun_out/bench_${TAG}_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_${TAG}_$c.json')); r=d['roofline']; print('$c', round(d['value']), 'qps p50', round(d['p50_ms'],3), 'scan ms', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],3), 'fb', d.get('fallback_queries_total'))"
done
