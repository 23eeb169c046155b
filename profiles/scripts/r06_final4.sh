#!/bin/bash
# Round 6 at the last kernel commit: the whole GPU suite, smoke, the default line, then the
# strong-scaled per-rank shard lines (c6 / c4 at 1.25M rows) with a one-stream trace of c6's.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r06_final4} bash profiles/scripts/r06_suite.sh || exit 1
O=gpurun_out/${TAG:-r06_final4}
for c in c6 c4; do
  timeout -k 10 200 python3 bench.py --config $c --rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline > $O/shard_${c}_line.json 2> $O/shard_${c}.err || { tail -5 $O/shard_${c}.err; exit 1; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_shard_c6 -o run -- python3 bench.py --config c6 --rows 1250000 --streams 1 --steps 50 --warmup 5 --no-cpu-baseline > $O/shard_c6_trace.json 2> $O/shard_c6_trace.err || { tail -5 $O/shard_c6_trace.err; exit 1; }
python3 - <<PY
import csv, glob, json
for c in ('c6', 'c4'):
    d = json.loads(open('$O/shard_%s_line.json' % c).read().strip().splitlines()[-1])
    print('shard', c, round(d['value']), d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['kernel'])
for f in glob.glob('$O/trace_shard_c6/**/run_kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:9]:
        print('c6 shard 1-stream', r['Name'][:50], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
