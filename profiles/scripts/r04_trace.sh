#!/bin/bash
# Single-stream kernel traces (isolated kernel durations) of the given configs.
# Usage: r04_trace.sh TAG "c4 c3" [extra bench args]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_trace}; mkdir -p $O
for c in $2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$c -o run -- python bench.py --config $c --streams 1 --steps 10 --warmup 3 --no-cpu-baseline --no-serving --no-metric-workload $3 > $O/bench_$c.json 2> $O/bench_$c.err || { echo "trace $c failed"; tail -20 $O/bench_$c.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$c.json $c
  python - $O/tr_$c/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f"  {r['Name'][:90]:90s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
done
