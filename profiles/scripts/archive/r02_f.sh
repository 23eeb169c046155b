#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'fallback', d['fallback_queries_total'])"
}
for p in bf16x3 bf16; do
  run c2_${p}_lock --precision $p --scan-sync 1 || exit 1
  run c2_${p}_flag --precision $p --scan-sync 2 || exit 1
  VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_nopub.so run c2_${p}_nopub --precision $p || exit 1
  VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_kl.so run c2_${p}_kl --precision $p --no-fallback || exit 1
  run c2_${p}_pilot0 --precision $p --pilot-tiles 0 || exit 1
  run c2_${p}_pilot2k --precision $p --pilot-tiles 2048 || exit 1
done
