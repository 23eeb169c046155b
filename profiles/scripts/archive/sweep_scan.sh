#!/bin/bash
# Candidate-pass variant sweep on C2 (one process per variant; scan time from HIP events).
set -o pipefail
export TMPDIR=/tmp
for v in ${VARIANTS:-0 1 2}; do
  for nwg in ${NWGS:-0 256 512}; do
    extra=""; [ "$nwg" != "0" ] && extra="--n-wg $nwg"
    timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --scan-variant $v $extra > gpurun_out/sweep_v${v}_w${nwg}.json 2>gpurun_out/sweep_v${v}_w${nwg}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/sweep_v${v}_w${nwg}.json'));print('variant $v nwg $nwg', round(d['value']), 'qps scan_ms', round(d['roofline']['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'frac', round(d['roofline']['frac'],3), 'fallback', d['fallback_queries_total'])"
  done
done
