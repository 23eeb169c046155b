#!/bin/bash
# Round 5: per-kernel times of one config with ONE stream (no overlap between a batch's kernels and
# another batch's scan), rocprofv3 kernel trace -> gpurun_out/r05_side_<config>/.
set -o pipefail
export TMPDIR=/tmp
c=${1:-c4}; O=gpurun_out/r05_side_$c; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config $c --streams 1 \
  --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-serving --no-metric-workload --no-other-configs \
  > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 profiles/scripts/rocpd_stats.py $(find $O/prof -name '*results.db' | head -1) 14 | tee $O/summary.md
