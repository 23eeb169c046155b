#!/bin/bash
# scan3 RT=4 variant (lib/libvdb_amd_s3d.so): parity, then C3 / C4 against the default scan2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-s3b}; mkdir -p $O
export VDB_LIB=$PWD/mlx-vector-db_amd/lib/libvdb_amd_s3d.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -k "scan3" > $O/pytest_s3.log 2>&1 || { echo "scan3 parity failed"; grep -E "FAIL|Error|assert" $O/pytest_s3.log | head -20; tail -30 $O/pytest_s3.log; exit 1; }
tail -1 $O/pytest_s3.log
for c in c3 c4; do
  for s3 in 0 1; do
    VDB_SCAN3=$s3 timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 30 > $O/bench_${c}_s3$s3.json 2> $O/bench_${c}_s3$s3.err || { echo "bench $c s3=$s3 failed"; tail -20 $O/bench_${c}_s3$s3.err; exit 1; }
    python profiles/scripts/ab_line.py $O/bench_${c}_s3$s3.json "${c}_s3d_scan3=$s3"
  done
done
