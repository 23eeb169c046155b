#!/bin/bash
# I8 at KP 256 in 64-query blocks (KW 64): the parity suite, default lines C2 / C6 / C3, and a
# rocprofv3 kernel trace (one stream) of C2 and C6.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8e}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread \
  > $O/pytest_parity.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_parity.log | head -30; tail -40 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c2 c2 && run c6 c6 && run c3 c3 || exit 1
for c in c2 c6; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python bench.py --config $c --streams 1 --steps 30 --warmup 3 --no-cpu-baseline --no-serving > $O/trace_$c.json 2> $O/trace_$c.err || { echo "trace $c failed"; tail -20 $O/trace_$c.err; exit 1; }
done
find $O -name '*kernel_stats.csv'
