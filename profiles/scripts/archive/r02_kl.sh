#!/bin/bash
# K-loop-only timing of the split pass (diagnostic library) vs the product library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02kl
mkdir -p $O
run() { local t=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-fallback "$@" > $O/$t.json 2> $O/$t.err || { echo "$t failed"; tail -5 $O/$t.err; return 1; }
  python -c "import json;d=json.load(open('$O/$t.json'));r=d['roofline'];print('$t', 'scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'hbm', round(r['hbm_gbs']), 'mfma_tf', round(r['mfma_tflops']))"
}
for cfg in "c2 --precision bf16x3" "c2 --precision bf16" "c3" "c4" "c4 --scan-sync 1"; do
  tag=$(echo $cfg | tr ' ' _ | tr -d '-')
  VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_kl.so run kl_$tag --config $cfg || exit 1
  run full_$tag --config $cfg || exit 1
done
