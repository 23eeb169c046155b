#!/bin/bash
# Same-box A/B: scan2 with / without IEEE NaN semantics; 2-rank sharded test on one GPU.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02x
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'prec', r['precision'], 'scan_ms', round(r['avg_launch_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'fallback', d['fallback_queries_total'])"
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 240 --timeout-method thread > $O/pytest_sharded.log 2>&1 || { echo "sharded test failed"; tail -40 $O/pytest_sharded.log; exit 1; }
tail -1 $O/pytest_sharded.log
for i in 1 2; do
  run c2_noieee_$i || exit 1
  VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_ieee.so run c2_ieee_$i || exit 1
  run c4_noieee_$i --config c4 || exit 1
  VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_ieee.so run c4_ieee_$i --config c4 || exit 1
done
