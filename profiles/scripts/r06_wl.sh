#!/bin/bash
# Round 6: the long-row wide pass (vdb_scan8wl.hip): its parity tests, then C3 A/B against the
# 64-query shape (--scan-wide 0) and a one-stream kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_wl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -v -s --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
grep -E "passed|failed|long D" $O/pytest.txt | tail -16
AB="c3|--config c3 --steps 100;c3old|--config c3 --steps 100 --scan-wide 0" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 bench.py --config c3 \
  --streams 1 --steps 50 --warmup 5 --no-cpu-baseline --no-serving --no-metric-workload --no-other-configs > $O/c3_trace.json 2> $O/c3_trace.err || { tail -5 $O/c3_trace.err; exit 1; }
python3 - <<PY
import csv, glob
for f in glob.glob('$O/trace_c3/**/run_kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print('c3 1-stream', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
PY
