#!/bin/bash
# Round 6: one-stream trace + PMC passes of C3 with the long-row wide pass -> gpurun_out/prof_r06f_c3w/
set -o pipefail
STEPS=20 timeout -k 10 900 bash profiles/scripts/profile.sh r06f_c3w --config c3 --streams 1 --no-serving \
  --no-metric-workload --no-other-configs > gpurun_out/prof_r06f_c3w.log 2>&1 || { tail -20 gpurun_out/prof_r06f_c3w.log; exit 1; }
echo "c3 profiled"
