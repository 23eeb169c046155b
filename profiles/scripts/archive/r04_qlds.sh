#!/bin/bash
# A/B of the int8 query block in LDS whenever it fits (scan_qlds 2) vs the round-3 rule (1):
# parity first, then C2 / C3 / C6 lines with each setting (same box).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_qlds}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "lds or group_counts" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in c2 c3 c6; do for q in 1 2; do
  timeout -k 10 300 python bench.py --config $c --scan-qlds $q --no-cpu-baseline --no-serving --no-metric-workload > $O/bench_${c}_q$q.json 2> $O/bench_${c}_q$q.err || { echo "bench $c $q failed"; tail -30 $O/bench_${c}_q$q.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_${c}_q$q.json ${c}_qlds$q
done; done
