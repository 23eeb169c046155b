#!/bin/bash
# Round 6 final scan kernels: one-stream kernel trace + PMC passes (HBM bytes, SQ, clock / L2) of
# each bench config -> gpurun_out/prof_r06f_<cfg>/ (summarised by profiles/scripts/summarize.py).
set -o pipefail
for c in c2 c6 c3 c4; do
  STEPS=20 timeout -k 10 900 bash profiles/scripts/profile.sh r06f_$c --config $c --streams 1 --no-serving \
    --no-metric-workload --no-other-configs > gpurun_out/prof_r06f_$c.log 2>&1 || { tail -20 gpurun_out/prof_r06f_$c.log; exit 1; }
  echo "$c profiled"
done
