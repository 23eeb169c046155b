#!/bin/bash
# C3: K-loop-only build vs the full kernel (is the epilogue part of the C3 scan's cost?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s19; mkdir -p $O
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  VDB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
KL=mlx-vector-db_amd/lib/libvdb_amd_kl.so
D=mlx-vector-db_amd/lib/libvdb_amd.so
run c3_kl $KL --config c3 --streams 1 --precision bf16 --steps 4 --warmup 1
run c3_def $D --config c3 --streams 1 --precision bf16 --steps 20
