#!/bin/bash
# Round 6: the finish reads the wide passes' segments one per lane (one round of counts, then one
# round per entry slot): the wide tests, then C3 / C4 lines and a one-stream C3 trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_wl2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB="c3|--config c3 --steps 100;c4|--config c4 --steps 100" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 bench.py --config c3 \
  --streams 1 --steps 50 --warmup 5 --no-cpu-baseline --no-serving --no-metric-workload --no-other-configs > $O/c3_trace.json 2> $O/c3_trace.err || { tail -5 $O/c3_trace.err; exit 1; }
python3 - <<PY
import csv, glob
for f in glob.glob('$O/trace_c3/**/run_kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:6]:
        print('c3 1-stream', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
