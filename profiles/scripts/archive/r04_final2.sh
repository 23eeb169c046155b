#!/bin/bash
# Round 4 (second session) final: guards, the whole GPU suite (full sizes), smoke, the default
# line and the other configs' lines (r04_final.sh), then the C2 kernel trace + HBM PMC passes.
set -o pipefail
export TMPDIR=/tmp
bash profiles/scripts/r04_final.sh ${1:-r04_final2} || exit 1
STEPS=20 bash profiles/scripts/profile.sh r04b_c2 --config c2 --no-serving --no-metric-workload || exit 1
echo "profiled c2"
