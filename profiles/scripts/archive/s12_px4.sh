#!/bin/bash
# C4 (query block in LDS) corpus prefetch depth: PX = 2 groups ahead (default) vs 4.
# The K-loop-only build showed the C4 scan is all K-loop (3.80 vs 3.79 ms): latency-bound loads.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s12; mkdir -p $O
P4=mlx-vector-db_amd/lib/libvdb_amd_px4.so
D=mlx-vector-db_amd/lib/libvdb_amd.so
VDB_LIB=$P4 timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_px4.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_px4.log | head; tail -40 $O/pytest_px4.log; exit 1; }
tail -1 $O/pytest_px4.log
run() {  # tag, lib, args
  local tag=$1 lib=$2; shift 2
  VDB_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
  run c4_def_s1_$rep $D --config c4 --streams 1
  run c4_px4_s1_$rep $P4 --config c4 --streams 1
done
run c4_def $D --config c4
run c4_px4 $P4 --config c4
VDB_LIB=$P4 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -m "gpu and slow" -x -q -k c4 --timeout 400 --timeout-method thread > $O/pytest_c4_px4.log 2>&1 || { tail -40 $O/pytest_c4_px4.log; exit 1; }
tail -1 $O/pytest_c4_px4.log
