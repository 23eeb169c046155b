#!/bin/bash
# A/B of the split pass's insertion scheme and LDS-query prefetch depth (same box)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', round(d['value']), 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'fallback', d['fallback_queries_total'])"
}
for lib in libvdb_amd libvdb_amd_bat libvdb_amd_px4 libvdb_amd_batpx4; do
  for cfg in c4 c2 c3; do
    VDB_LIB=mlx-vector-db_amd/lib/$lib.so run ${lib}_$cfg --config $cfg || exit 1
  done
done
