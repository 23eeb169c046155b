#!/bin/bash
# Pilot-bound rank A/B (Poisson rank vs the KP-th sample) + fast parity set.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'fallback', d['fallback_queries_total'])"
}
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for p in bf16x3 bf16; do
  run c2_${p}_poisson --precision $p || exit 1
  run c2_${p}_kp --precision $p --pilot-rank 256 || exit 1
done
run c3_poisson --config c3 || exit 1
run c3_kp --config c3 --pilot-rank 256 || exit 1
run c4_poisson --config c4 || exit 1
run c4_kp --config c4 --pilot-rank 256 || exit 1
