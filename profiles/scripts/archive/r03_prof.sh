#!/bin/bash
# Round-3 profiles: the C4 tests under the default (q4 auto), then rocprofv3 kernel trace + PMC
# passes (profile.sh) for each bench config.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "c4 or q4 or scan3" > gpurun_out/pytest_c4q4.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/pytest_c4q4.log | head; tail -20 gpurun_out/pytest_c4q4.log; exit 1; }
tail -1 gpurun_out/pytest_c4q4.log
for c in ${CONFIGS:-c2 c6 c3 c4}; do
  bash profiles/scripts/profile.sh r03_$c --config $c || exit 1
  echo "profiled $c"
done
