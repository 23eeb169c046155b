#!/bin/bash
# Round 6: the long-row wide pass (ring of <= 4 tiles, counters in LDS only for RL = 2): wide tests,
# then where it wins: C2 rows at B = 64 (3 streams), C3 rows at B = 32 / 64 / 128 (one stream), C3.
set -o pipefail
O=gpurun_out/r06_rl4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
S="--streams 1 --steps 200"
AB="c2|--config c2 --steps 200;c2w|--config c2 --steps 200 --scan-wide 1;l32|--config c3 --batch 32 $S;l32w|--config c3 --batch 32 $S --scan-wide 1;l64|--config c3 --batch 64 $S;l64w|--config c3 --batch 64 $S --scan-wide 1;l128|--config c3 --batch 128 $S;l128w|--config c3 --batch 128 $S --scan-wide 1;c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
