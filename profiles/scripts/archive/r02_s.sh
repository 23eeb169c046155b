#!/bin/bash
# KP-based pilot rank + pilot sample by k: C2 (both precisions), C3, C4; C2 k-rank A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02s
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'prec', r['precision'], 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'fallback', d['fallback_queries_total'])"
}
run c2 || exit 1
run c2_r5 --pilot-rank 5 || exit 1
run c2_p1024 --pilot-tiles 1024 || exit 1
run c2_b3 --precision bf16x3 || exit 1
run c2_b3_r5 --precision bf16x3 --pilot-rank 5 || exit 1
run c3 --config c3 || exit 1
run c4 --config c4 || exit 1
