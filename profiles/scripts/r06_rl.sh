#!/bin/bash
# Round 6: the long-row wide pass with RL = 2 waves per query tile for batches of <= 128 (rows of
# <= 1024 dims): wide tests, then C2 (B = 64) forced wide against the 64-query shape, small
# batches, and C3 against the previous library (old).
set -o pipefail
O=gpurun_out/r06_rl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
S="--streams 1 --steps 200"
AB="c2|--config c2 --steps 200;c2w|--config c2 --steps 200 --scan-wide 1;b2w|--config c2 --batch 2 $S --scan-wide 1;b2wo|VDB_LIB=$L --config c2 --batch 2 $S --scan-wide 1;b32|--config c2 --batch 32 $S;b32w|--config c2 --batch 32 $S --scan-wide 1;b128|--config c2 --batch 128 --steps 200;b128w|--config c2 --batch 128 --steps 200 --scan-wide 1;c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
