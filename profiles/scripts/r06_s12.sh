#!/bin/bash
# Round 6: the split short-row wide pass at c6 (10M x 128, B = 64) with a 12-tile small stage
# (s12: 48 KiB slots, still room for the finish's small form) against 8 tiles and the 64-query shape.
set -o pipefail
O=gpurun_out/r06_s12; mkdir -p $O
L=mlx-vector-db_amd/lib/libvdb_amd_s12.so
VDB_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q -k "small_batches_split or mask_and_chunked" --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB="c6|--config c6 --steps 100;c6w|--config c6 --steps 100 --scan-wide 1;c6w12|VDB_LIB=$L --config c6 --steps 100 --scan-wide 1;sh12|VDB_LIB=$L --config c6 --rows 1250000 --steps 400;sh|--config c6 --rows 1250000 --steps 400" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
