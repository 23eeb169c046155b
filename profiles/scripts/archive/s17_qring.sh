#!/bin/bash
# Query operand through a per-workgroup LDS ring (scan_qring=1) vs per-wave L2 loads (default):
# parity with the ring on, then C2/C3 A/B on the same box, then the full-size C2/C3 tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s17; mkdir -p $O
VDB_SCAN_QRING=1 timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_qr.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_qr.log | head; tail -40 $O/pytest_qr.log; exit 1; }
tail -1 $O/pytest_qr.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
  run c2_def_s1_$rep --streams 1
  run c2_qr_s1_$rep --streams 1 --scan-qring 1
done
run c2_def_s3 
run c2_qr_s3 --scan-qring 1
run c3_def_s1 --config c3 --streams 1
run c3_qr_s1 --config c3 --streams 1 --scan-qring 1
run c3_def_s3 --config c3
run c3_qr_s3 --config c3 --scan-qring 1
run c2b3_def_s1 --streams 1 --precision bf16x3
run c2b3_qr_s1 --streams 1 --precision bf16x3 --scan-qring 1
VDB_SCAN_QRING=1 timeout -k 10 600 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 400 --timeout-method thread -k "c2 or c3" > $O/pytest_qr_slow.log 2>&1 || { tail -40 $O/pytest_qr_slow.log; exit 1; }
tail -1 $O/pytest_qr_slow.log
