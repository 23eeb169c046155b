#!/bin/bash
# Empty gated fallback launch size under the 3-stream pipeline: n_cu x 4 query slots (default)
# vs n_cu/4 and n_cu/8 row ranges with one slot; parity of the fallback tests with gate_div 8.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s21; mkdir -p $O
VDB_GATE_DIV=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fallback or duplicates or auto or exact_path or device_search" > $O/pytest_gd.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gd.log | head; tail -30 $O/pytest_gd.log; exit 1; }
tail -1 $O/pytest_gd.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
  run c2_gd1_$rep
  run c2_gd4_$rep --gate-div 4
  run c2_gd8_$rep --gate-div 8
done
run c3_gd1 --config c3
run c3_gd8 --config c3 --gate-div 8
