#!/bin/bash
# Round 6, last kernels: one-stream trace + PMC of C4 (short-row wide pass) -> gpurun_out/prof_r06g_c4/
set -o pipefail
STEPS=20 timeout -k 10 900 bash profiles/scripts/profile.sh r06g_c4 --config c4 --streams 1 --no-serving \
  --no-metric-workload --no-other-configs > gpurun_out/prof_r06g_c4.log 2>&1 || { tail -20 gpurun_out/prof_r06g_c4.log; exit 1; }
echo "c4 profiled"
