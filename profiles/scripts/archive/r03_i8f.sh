#!/bin/bash
# A/B: the shared-bound refresh of the int8 pass every step (default build) vs every 16 steps
# vs once (VDB_S8_GEVERY variants), C6 and C2, same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8f}; mkdir -p $O
run() {  # tag lib config [extra args]
  t=$1; l=$2; c=$3; shift 3
  VDB_LIB=$l timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
L=mlx-vector-db_amd/lib
for rep in 1 2; do
  run c6_def$rep $L/libvdb_amd.so c6 && run c6_g16_$rep $L/libvdb_amd_g16.so c6 && run c6_g1k_$rep $L/libvdb_amd_g1k.so c6 || exit 1
done
run c2_def $L/libvdb_amd.so c2 && run c2_g16 $L/libvdb_amd_g16.so c2 && run c2_g1k $L/libvdb_amd_g1k.so c2
