#!/bin/bash
# Fused gated fallback + split-K pilot: parity, bench, C4 sync A/B, finish stamps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'fallback', d['fallback_queries_total'])"
}
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run c2_bf16x3 --precision bf16x3 || exit 1
run c2_bf16 --precision bf16 || exit 1
run c4_flag --config c4 --scan-sync 2 || exit 1
run c4_lock --config c4 --scan-sync 1 || exit 1
timeout -k 10 120 python profiles/scripts/fin_stamp.py c2 bf16x3 > $O/fin_c2_bf16x3.txt 2>&1 && cat $O/fin_c2_bf16x3.txt || exit 1
timeout -k 10 120 python profiles/scripts/fin_stamp.py c2 bf16 > $O/fin_c2_bf16.txt 2>&1 && cat $O/fin_c2_bf16.txt || exit 1
timeout -k 10 200 python profiles/scripts/fin_stamp.py c4 bf16x3 > $O/fin_c4.txt 2>&1 && cat $O/fin_c4.txt || exit 1
