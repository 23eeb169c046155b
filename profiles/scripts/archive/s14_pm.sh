#!/bin/bash
# Plane-major corpus copy (hi plane of a super tile contiguous) vs group-major (default):
# parity of the variant, then C2/C3/C4 A/B on the same box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s14; mkdir -p $O
PM=mlx-vector-db_amd/lib/libvdb_amd_pm.so
D=mlx-vector-db_amd/lib/libvdb_amd.so
VDB_LIB=$PM timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_pm.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_pm.log | head; tail -40 $O/pytest_pm.log; exit 1; }
tail -1 $O/pytest_pm.log
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  VDB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
  run c2_def_s1_$rep $D --streams 1
  run c2_pm_s1_$rep $PM --streams 1
done
run c2_def_s3 $D
run c2_pm_s3 $PM
run c2b3_def_s1 $D --streams 1 --precision bf16x3
run c2b3_pm_s1 $PM --streams 1 --precision bf16x3
run c3_def_s1 $D --config c3 --streams 1
run c3_pm_s1 $PM --config c3 --streams 1
run c4_def_s1 $D --config c4 --streams 1
run c4_pm_s1 $PM --config c4 --streams 1
VDB_LIB=$PM timeout -k 10 600 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 400 --timeout-method thread -k "not c5" > $O/pytest_pm_slow.log 2>&1 || { tail -40 $O/pytest_pm_slow.log; exit 1; }
tail -1 $O/pytest_pm_slow.log
