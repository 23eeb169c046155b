#!/bin/bash
# Pacing of the query blocks of a row range (int8 pass, n_qb > 1): parity suite, C4 / C3 pace on
# vs off, C4 stamps (drift within a range).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pace}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 150 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -30; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c4_pace c4 && run c4_nopace c4 --scan-pace 0 && run c3_pace c3 && run c3_nopace c3 --scan-pace 0 || exit 1
timeout -k 10 200 python profiles/scripts/stamp_scan8.py c4 i8x3 > $O/stamp_c4.txt 2> $O/stamp_c4.err && cat $O/stamp_c4.txt || { tail -20 $O/stamp_c4.err; exit 1; }
