#!/bin/bash
# scan2 shape A/B: 4 waves x 4 row tiles (default) vs 8 waves x 2 row tiles (two waves per SIMD,
# so one wave's epilogue can overlap the other's MFMAs).  Parity of the variant first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s10; mkdir -p $O
W8=mlx-vector-db_amd/lib/libvdb_amd_w8.so
VDB_LIB=$W8 timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_w8.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_w8.log | head; tail -40 $O/pytest_w8.log; exit 1; }
tail -1 $O/pytest_w8.log
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  VDB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
D=mlx-vector-db_amd/lib/libvdb_amd.so
for c in c4 c2 c3; do
  run ${c}_def_s1 $D --config $c --streams 1
  run ${c}_w8_s1 $W8 --config $c --streams 1
  run ${c}_def $D --config $c
  run ${c}_w8 $W8 --config $c
done
