#!/bin/bash
# C4 (10M x 128 L2, k = 100, batch 512) by candidate-pass precision: bf16x3 (auto's choice for
# k > 16) against the int8 kernels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-c4prec}; mkdir -p $O
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c3_i8x3 c3 --precision i8x3 && run c3_b3 c3 --precision bf16x3 && run c2_i8x3 c2 --precision i8x3 && run c2_b3 c2 --precision bf16x3
