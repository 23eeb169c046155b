#!/bin/bash
# Round 6, last kernels: one-stream traces + PMC of C2 and C3 (both on the long-row wide pass now),
# then the whole GPU suite, smoke and the default line.
set -o pipefail
for c in c2 c3; do
  STEPS=20 timeout -k 10 600 bash profiles/scripts/profile.sh r06g_$c --config $c --streams 1 --no-serving \
    --no-metric-workload --no-other-configs > gpurun_out/prof_r06g_$c.log 2>&1 || { tail -20 gpurun_out/prof_r06g_$c.log; exit 1; }
  echo "$c profiled"
done
TAG=r06_final3 bash profiles/scripts/r06_suite.sh
