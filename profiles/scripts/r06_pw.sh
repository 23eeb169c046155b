#!/bin/bash
# Round 6: the pilot with four waves per sampled tile beside a long-row wide scan (C3; C2 rows
# already had it), against the previous library (old); pilot-touching tests first.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_pw; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_guards.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
AB="c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100;l2|--config c3 --batch 2 --streams 1 --steps 200;l2o|VDB_LIB=$L --config c3 --batch 2 --streams 1 --steps 200" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
