#!/bin/bash
# K-loop-only A/B of the int8 pass (VDB_SCAN8_KLOOP_ONLY: the epilogue skipped, results garbage,
# --no-fallback): how much of the C6 / C2 scan the epilogue costs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8k}; mkdir -p $O
run() {  # tag lib config [extra args]
  t=$1; l=$2; c=$3; shift 3
  VDB_LIB=$l timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving --no-fallback --streams 1 "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
L=mlx-vector-db_amd/lib
run c6_def $L/libvdb_amd.so c6 && run c6_kl $L/libvdb_amd_kl.so c6 && run c2_def $L/libvdb_amd.so c2 && run c2_kl $L/libvdb_amd_kl.so c2
