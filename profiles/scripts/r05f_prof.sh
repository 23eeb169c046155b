#!/bin/bash
# Round 5 final: rocprofv3 kernel trace + PMC passes of each config's default (profile.sh -> prof_r05f_<c>),
# then the one-stream per-kernel summaries (r05_side.sh).  Summaries: summarize.py r05f_<c> scan8_kernel.
set -o pipefail
export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c6 c4 c3}; do
  bash profiles/scripts/profile.sh r05f_$c --config $c --no-serving --no-metric-workload --no-other-configs || exit 1
  echo "profiled $c"
done
for c in ${SIDE:-c2 c6 c4 c3}; do
  bash profiles/scripts/r05_side.sh $c > gpurun_out/r05_side_$c.log 2>&1 || exit 1
  echo "side $c"
done
