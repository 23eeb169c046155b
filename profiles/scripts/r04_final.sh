#!/bin/bash
# Round 4 final: guard tests, the whole GPU suite (full sizes included), smoke, the default bench
# line and the other configs' lines, all at the final commit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_final}; mkdir -p $O
bash profiles/scripts/r04_check.sh $(basename $O) || exit 1
for c in c3 c4 c6; do
  timeout -k 10 400 python bench.py --config $c --no-serving --no-metric-workload > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$c.json $c
done
