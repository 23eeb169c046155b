#!/bin/bash
# Round 6: per-kernel times of a small-batch (B = 2, one stream) C2 search: where the serving
# path's device latency goes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_b2; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c2 --batch 2 \
  --streams 1 --steps 200 --warmup 10 --no-cpu-baseline --no-serving > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - <<PY
import csv, glob
for f in glob.glob('$O/trace/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:70], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
