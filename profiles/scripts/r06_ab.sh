#!/bin/bash
# Round 6 same-box A/B lines: AB="label|[VAR=value ...] bench args;..." run ROUNDS times interleaved;
# each line -> gpurun_out/r06_ab/<label>_<round>.json, a one-line summary per run on stdout.
set -o pipefail
mkdir -p gpurun_out/r06_ab
IFS=';' read -ra CASES <<< "$AB"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${CASES[@]}"; do
    label=${c%%|*}; args=${c#*|}
    envs=""; while [[ "${args%% *}" == *=* ]]; do envs="$envs ${args%% *}"; args=${args#* }; done
    env $envs timeout -k 10 ${T:-240} python bench.py --no-cpu-baseline --no-serving --no-metric-workload --no-other-configs $args \
      > gpurun_out/r06_ab/${label}_$r.json 2> gpurun_out/r06_ab/${label}_$r.err || { echo "FAIL $label"; tail -5 gpurun_out/r06_ab/${label}_$r.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/r06_ab/${label}_$r.json')); r=d['roofline']
print('$label', $r, 'qps %.0f' % d['value'], 'step %.4f' % d['ms_per_step'], 'p50 %.4f' % d['p50_ms'], 'scan %.4f' % r['avg_launch_ms'], r['precision'], 'fb', d['fallback_queries_timed'])"
  done
done
