#!/bin/bash
# Round 6: long-row wide pass, final form (round-based RL = 2 kernel for <= 128 queries at <= 1024
# dims, the per-tile kernel otherwise): wide tests, then C2 / C3 default lines against the 64-query
# shape and the previous library (old).
set -o pipefail
O=gpurun_out/r06_rl5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
AB="c2|--config c2 --steps 200;c2s|--config c2 --steps 200 --scan-wide 0;c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
