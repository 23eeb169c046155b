#!/bin/bash
# C2/C3 (bf16, global query operand) corpus prefetch depth A/B: PX 4 / PQ 4 (default) vs
# PX 8 with the query prefetch decoupled (PQ 2), PX 8 / PQ 4, PX 4 / PQ 2.  Bench only.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s13; mkdir -p $O
L=mlx-vector-db_amd/lib
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  VDB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
  for v in def b8q2 b4q2 b8q4; do
    lib=$L/libvdb_amd_$v.so; [ $v = def ] && lib=$L/libvdb_amd.so
    run c2_${v}_s1_$rep $lib --streams 1
  done
done
for v in def b8q2 b4q2; do
  lib=$L/libvdb_amd_$v.so; [ $v = def ] && lib=$L/libvdb_amd.so
  run c2_${v}_s3 $lib
  run c3_${v}_s1 $lib --config c3 --streams 1
done
