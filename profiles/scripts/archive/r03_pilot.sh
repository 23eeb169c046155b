#!/bin/bash
# Pilot sample size sweep for the int8 pass (C6, C2): a tighter pilot bound means fewer insertions
# in the scan's epilogue (C6 at 512 tiles: ~1.5 passing tiles per wave-step, ~45% of the step).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pilot}; mkdir -p $O
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c6_p1024 c6 --pilot-tiles 1024 || exit 1
for p in 512 1024 2048 4096; do run c2_p$p c2 --pilot-tiles $p || exit 1; done
for p in 512 1024 2048 4096; do run c3_p$p c3 --pilot-tiles $p || exit 1; done
