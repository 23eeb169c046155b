#!/bin/bash
# auto: k > 16 runs I8X3 (the int8 copy), BF16X3 for holds / re-passes / retries.  Parity suite,
# default lines C4 (k = 100) and C2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-x3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 150 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -30; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c4 c4 && run c2 c2
