#!/bin/bash
# Same-box A/B of the scan step end: previous library (lib/libvdb_amd_old.so) vs the current
# one in auto / lockstep / flag mode, C2 C3 C4.  Usage: bash profiles/scripts/ab_sync.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_sync
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value']), 'p50', round(d['p50_ms'],3), 'scan ms', round(r['avg_launch_ms'],4))" "$@"; }
for c in c2 c3 c4; do
  for mode in old 0 1 2; do
    out=gpurun_out/ab_sync/${c}_$mode.json
    if [ $mode = old ]; then
      VDB_LIB=$PWD/mlx-vector-db_amd/lib/libvdb_amd_old.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 40 > $out 2> $out.err || { tail -20 $out.err; exit 1; }
    else
      timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 40 --scan-sync $mode > $out 2> $out.err || { tail -20 $out.err; exit 1; }
    fi
    summ $out "$c $mode"
  done
done
