#!/bin/bash
# Session 3: K-loop-only variant (epilogue cost at C4 / C2), then rocprofv3 evidence at HEAD
# (one stream, so kernel durations are not inflated by concurrent batches).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s11; mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  VDB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
KL=mlx-vector-db_amd/lib/libvdb_amd_kl.so
D=mlx-vector-db_amd/lib/libvdb_amd.so
run c4_kl $KL --config c4 --streams 1 --precision bf16x3 --steps 3 --warmup 1
run c4_def $D --config c4 --streams 1 --precision bf16x3
run c2_kl $KL --config c2 --streams 1 --precision bf16 --steps 10 --warmup 2
run c2_def $D --config c2 --streams 1 --precision bf16
STEPS=20 bash profiles/scripts/profile.sh r02g_c2_bf16 --config c2 --streams 1 || exit 1
STEPS=10 bash profiles/scripts/profile.sh r02g_c4_bf16x3 --config c4 --streams 1 || exit 1
