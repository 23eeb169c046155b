#!/bin/bash
# L2 I8 tail waits counting the fresh start-value loads (A/B: lib/libvdb_amd_tf0.so = uncounted):
# parity suite, C4's rows at k = 10 (auto -> I8, query block in LDS) and the C4 line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-tf}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 150 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -30; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() {  # tag config [extra args]
  t=$1; c=$2; shift 2
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
run c4k10_new c4 --k 10 && VDB_LIB=$PWD/mlx-vector-db_amd/lib/libvdb_amd_tf0.so run c4k10_old c4 --k 10 && run c4k10_new2 c4 --k 10 && run c4 c4
