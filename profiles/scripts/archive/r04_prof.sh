#!/bin/bash
# rocprofv3 kernel trace + PMC passes (profile.sh) of the round-4 defaults for each bench config.
set -o pipefail
export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c3 c6 c4}; do
  bash profiles/scripts/profile.sh r04_$c --config $c --no-serving --no-metric-workload || exit 1
  echo "profiled $c"
done
