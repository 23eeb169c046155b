#!/bin/bash
# Round-2 rocprofv3 evidence: kernel trace + PMC passes for the BASELINE configs.
# Usage: bash profiles/scripts/r02_prof.sh SUFFIX "c2:bf16x3 c2:bf16 c4:bf16x3 ..."
set -o pipefail
SUF=$1; shift
for cp in $1; do
  c=${cp%%:*}; p=${cp##*:}
  STEPS=20 bash profiles/scripts/profile.sh r02_${c}_${p}${SUF} --config $c --precision $p || exit 1
done
