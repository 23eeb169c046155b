#!/bin/bash
# Round 5: rocprofv3 kernel trace + PMC passes (profile.sh) of the defaults for each bench config
# (the traffic of the kernels the lines run, incl. C4's 8-wave I8X3 pass), then
# the default bench line (C2 + the c6 / c3 / c4 sub-records).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05
for c in ${CONFIGS:-c2 c3 c4 c6}; do
  bash profiles/scripts/profile.sh r05_$c --config $c --no-serving --no-metric-workload || exit 1
  echo "profiled $c"
done
if [ -z "$NO_DEFAULT" ]; then
  timeout -k 10 600 python bench.py > gpurun_out/r05/bench_default.json 2> gpurun_out/r05/bench_default.err || exit 1
  echo "default line done"
fi
