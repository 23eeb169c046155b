#!/bin/bash
# I8 at C2: KP = 256 (margin 246: a wider top-k gap for the 8-bit query bound) vs 128
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8c}; mkdir -p $O
run() {  # tag config precision [extra args]
  t=$1; c=$2; p=$3; shift 3
  timeout -k 10 300 python bench.py --config $c --precision $p --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c2_i8_kp256 c2 i8 --margin 246 && run c2_i8_kp128 c2 i8 && run c6_i8_kp256 c6 i8 --margin 246 && run c2_bf16 c2 bf16 && run c6_i8_kp64 c6 i8 --margin 54
