#!/bin/bash
# q4 (128-query shape of the split pass): parity, then C4 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-q4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "q4" > $O/pytest_q4.log 2>&1 || { echo "q4 parity failed"; grep -E "FAIL|Error|assert" $O/pytest_q4.log | head -20; tail -30 $O/pytest_q4.log; exit 1; }
tail -1 $O/pytest_q4.log
for q in 0 1; do
  VDB_SCAN_Q4=$q timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline --steps 50 > $O/bench_c4_q4$q.json 2> $O/bench_c4_q4$q.err || { echo "bench c4 q4=$q failed"; tail -20 $O/bench_c4_q4$q.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_c4_q4$q.json "c4_q4=$q"
done
VDB_SCAN_Q4=1 timeout -k 10 300 python bench.py --config c4 --precision bf16 --no-cpu-baseline --steps 30 > $O/bench_c4_q4_bf16.json 2> $O/bench_c4_q4_bf16.err && python profiles/scripts/ab_line.py $O/bench_c4_q4_bf16.json "c4_q4=1_bf16"
