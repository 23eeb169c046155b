#!/bin/bash
# Directional bf16 bound (C3 in bf16), maximum3 vs IEEE max, publish at C3, streams at C3/C4, stamps C2/C3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
run c3_bf16 --config c3 --precision bf16
run c3_bf16_cs --config c3 --precision bf16 --dir-bound 0
run c3_auto --config c3
run c3_b3 --config c3 --precision bf16x3
VDB_LIB=$PWD/mlx-vector-db_amd/lib/libvdb_amd_im.so run c3_b3_im --config c3 --precision bf16x3
run c3_b3_pub0 --config c3 --precision bf16x3 --scan-publish 0
run c2_def
run c2_str2 --streams 2
VDB_LIB=$PWD/mlx-vector-db_amd/lib/libvdb_amd_im.so run c2_im
run c4_def --config c4
run c4_str2 --config c4 --streams 2
for a in "c2 bf16" "c3 bf16x3"; do
  timeout -k 10 240 python profiles/scripts/stamp_scan2.py $a >> $O/stamp.txt 2>> $O/stamp.err || { tail -20 $O/stamp.err; exit 1; }
done
cat $O/stamp.txt
