#!/bin/bash
# int8 pass, second cut (I8 = one accumulator set, RT 4; exact-key certificate in the finish):
# the parity suite, then C2 / C6 / C3 / C4 lines per precision on the same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8b}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_parity.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_parity.log | head -30; tail -40 $O/pytest_parity.log; exit 1; }
tail -1 $O/pytest_parity.log
grep -E "fallbacks" $O/pytest_parity.log | head -20
run() {  # config precision [extra args]
  c=$1; p=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --precision $p --no-cpu-baseline --no-serving "$@" > $O/bench_${c}_$p.json 2> $O/bench_${c}_$p.err || { echo "bench $c $p failed"; tail -30 $O/bench_${c}_$p.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_${c}_$p.json ${c}_$p
}
run c2 i8 && run c6 i8 && run c2 i8x3 && run c6 i8x3 && run c3 i8 && run c3 i8x3 && run c4 i8x3 && run c4 auto
