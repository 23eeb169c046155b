#!/bin/bash
# int8 + bf16 insertion: pass bits from independent tests + one round per hit (was a test-ballot-branch
# chain per register); pilot >= N/160.  Stamps (C6, C2, C3), parity suite, default lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8p}; mkdir -p $O
for c in c6 c2 c3; do
  timeout -k 10 200 python profiles/scripts/stamp_scan8.py $c > $O/stamp_$c.txt 2> $O/stamp_$c.err && cat $O/stamp_$c.txt || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 150 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -30; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c2 c2 && run c6 c6 && run c3 c3 && run c4 c4
