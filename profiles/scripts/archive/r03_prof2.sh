#!/bin/bash
# rocprofv3 kernel trace + PMC passes (profile.sh) of the int8-era default for each bench config.
set -o pipefail
export TMPDIR=/tmp
for c in ${CONFIGS:-c2 c6 c3 c4}; do
  bash profiles/scripts/profile.sh r03i8_$c --config $c || exit 1
  echo "profiled $c"
done
