#!/bin/bash
# Round 6: three-stream kernel timelines (start/end per launch) of C2 and C3 for the gap analysis
# (profiles/scripts/timeline6.py): what runs while no scan does.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_tl; mkdir -p $O
for c in c2 c3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$c -o run -- python3 bench.py --config $c --steps 60 --warmup 10 --no-cpu-baseline --no-serving --no-metric-workload --no-other-configs > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
done
ls -R $O | head -20
