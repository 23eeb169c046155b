#!/bin/bash
# Round 6: the long-row wide pass without 64-bit remainders in its ring indexing, and a 4-slot ring
# (s4: LDS left for the other streams' side kernels) at C2 forced wide; C3 and B = 2 against the
# library before the round-based change (old).
set -o pipefail
O=gpurun_out/r06_rl2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
L4=mlx-vector-db_amd/lib/libvdb_amd_s4.so
S="--streams 1 --steps 200"
AB="c2w|--config c2 --steps 200 --scan-wide 1;c2ws4|VDB_LIB=$L4 --config c2 --steps 200 --scan-wide 1;b2w|--config c2 --batch 2 $S --scan-wide 1;b2ws4|VDB_LIB=$L4 --config c2 --batch 2 $S --scan-wide 1;b2wo|VDB_LIB=$L --config c2 --batch 2 $S --scan-wide 1;c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
