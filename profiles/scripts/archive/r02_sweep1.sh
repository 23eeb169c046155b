#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sw1
run() { # tag args...
  local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/sw1/$t.json 2> gpurun_out/sw1/$t.err || { echo "$t failed"; tail -5 gpurun_out/sw1/$t.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/sw1/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'p50', round(d['p50_ms'],4), 'hbm', round(r['hbm_gbs']), 'fallback', d['fallback_queries_total'])"
}
run b3_v0 --precision bf16x3 --scan-variant 0 &&
run bf16_v0 --precision bf16 --scan-variant 0 &&
run bf16_v1 --precision bf16 --scan-variant 1 &&
run bf16_v0_m48 --precision bf16 --scan-variant 0 --margin 48 &&
run bf16_v1_m48 --precision bf16 --scan-variant 1 --margin 48 &&
run c4_b3 --config c4 --precision bf16x3 &&
run c4_b3_pilot4k --config c4 --precision bf16x3 --pilot-tiles 4096 &&
run c3_b3 --config c3 --precision bf16x3 &&
run c3_bf16 --config c3 --precision bf16
