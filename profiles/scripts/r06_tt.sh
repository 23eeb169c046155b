#!/bin/bash
# Round 6: the pilot with two sampled tiles per wave beside a long-row wide pass (VDB_PILOT8_TT=2,
# query operands loaded once for both) against one (tt1): wide + parity tests on the default
# build, then same-box A/B at C3 and C2.
set -o pipefail
O=gpurun_out/r06_tt; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd
AB="c3|--config c3 --steps 100;c3t1|VDB_LIB=${L}_tt1.so --config c3 --steps 100;c2|--steps 200;c2t1|VDB_LIB=${L}_tt1.so --steps 200" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
