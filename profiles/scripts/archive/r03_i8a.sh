#!/bin/bash
# First GPU run of the int8 candidate pass: the int8 parity tests (small), then C2 / C6 lines in
# i8 against bf16 on the same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8a}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "i8 or golden or precision_switch" > $O/pytest_i8.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_i8.log | head -30; tail -40 $O/pytest_i8.log; exit 1; }
tail -1 $O/pytest_i8.log
for p in i8 bf16; do
  for c in c2 c6; do
    timeout -k 10 300 python bench.py --config $c --precision $p --no-cpu-baseline --no-serving > $O/bench_${c}_$p.json 2> $O/bench_${c}_$p.err || { echo "bench $c $p failed"; tail -30 $O/bench_${c}_$p.err; exit 1; }
    python profiles/scripts/ab_line.py $O/bench_${c}_$p.json ${c}_$p
  done
done
