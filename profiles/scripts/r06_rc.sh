#!/bin/bash
# Round 6: wide passes' segment counters in registers (no LDS atomic on the insertion path) vs the
# previous commit's library (old): wide tests, then C4, C3, C2 rows at B = 32 / 64 (forced wide).
set -o pipefail
O=gpurun_out/r06_rc; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
AB="c4|--config c4 --steps 100;c4o|VDB_LIB=$L --config c4 --steps 100;c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100;w64|--config c2 --steps 200 --scan-wide 1;w64o|VDB_LIB=$L --config c2 --steps 200 --scan-wide 1;w32|--config c2 --batch 32 --streams 1 --steps 200 --scan-wide 1;w32o|VDB_LIB=$L --config c2 --batch 32 --streams 1 --steps 200 --scan-wide 1" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
