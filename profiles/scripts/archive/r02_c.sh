#!/bin/bash
# parity (fast set) + bench sweep of the split-bf16 pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'hbm', round(r['hbm_gbs']), 'mfma_tf', round(r['mfma_tflops']), 'fallback', d['fallback_queries_total'])"
}
run c2_b3 --precision bf16x3 && run c2_bf16 --precision bf16 && run c3_b3 --config c3 && run c4_b3 --config c4 && run c4_b3_lock --config c4 --scan-sync 1 && run c2_fp32 --precision fp32
