#!/bin/bash
# A/B: pilot bound derived in the scan prologue vs a separate bound kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'prec', r['precision'], 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'fallback', d['fallback_queries_total'])"
}
for i in 1 2; do
run c2_fused_$i || exit 1
run c2_sep_$i --pilot-fused 0 || exit 1
run c2b3_fused_$i --precision bf16x3 || exit 1
run c2b3_sep_$i --precision bf16x3 --pilot-fused 0 || exit 1
done
run c3_fused --config c3 || exit 1
run c3_sep --config c3 --pilot-fused 0 || exit 1
