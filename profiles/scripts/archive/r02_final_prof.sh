#!/bin/bash
# Round-2 final rocprofv3 evidence (kernel trace + PMC passes) per BASELINE config and the
# precision auto runs there.  Usage: bash profiles/scripts/r02_final_prof.sh "c2:bf16 c2:bf16x3"
set -o pipefail
( while sleep 50; do date +%s >> gpurun_out/final_prof_heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for cp in $1; do
  c=${cp%%:*}; p=${cp##*:}
  STEPS=20 bash profiles/scripts/profile.sh r02f_${c}_${p} --config $c --precision $p || exit 1
done
