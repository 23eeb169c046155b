#!/bin/bash
# Sticky auto precision: parity + C2/C3/C4 with long timed regions.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02z
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'prec', r['precision'], r['searches_by_precision'], 'scan_ms', round(r['avg_launch_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'fallback', d['fallback_queries_total'])"
}
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run c2 --steps 60 || exit 1
run c3 --config c3 --steps 60 || exit 1
run c4 --config c4 --steps 60 || exit 1
run c2_b3 --precision bf16x3 --steps 60 || exit 1
bash profiles/scripts/r02_trace.sh z "c2:auto" || exit 1
