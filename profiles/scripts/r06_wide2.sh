#!/bin/bash
# Round 6: wide-pass variants -- 16 waves x 32 queries (parity first), K-loop only, checksum off.
set -o pipefail
mkdir -p gpurun_out/r06_wide2
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_w16.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py \
  > gpurun_out/r06_wide2/pytest_w16.txt 2>&1 || { tail -40 gpurun_out/r06_wide2/pytest_w16.txt; exit 1; }
tail -2 gpurun_out/r06_wide2/pytest_w16.txt
export AB="wide|--config c4;w16|VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_w16.so --config c4;wkl|VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_wkl.so --config c4 --no-fallback;ck0|--config c4 --scan-checksum 0"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
