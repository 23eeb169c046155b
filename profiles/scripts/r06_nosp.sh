#!/bin/bash
# Round 6: each finish form compiled with its own exact-key path only (no scratch spills in the
# 16- and 4-wave forms: 212 -> 0 bytes per lane) against the previous build (old): the finish and
# parity tests on the new build, then same-box A/B at C2, c6, C4, C3 and the c6 / c4 shards.
set -o pipefail
O=gpurun_out/r06_nosp; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
L=mlx-vector-db_amd/lib/libvdb_amd_old.so
AB="c2|--steps 200;c2o|VDB_LIB=$L --steps 200;c6|--config c6 --steps 100;c6o|VDB_LIB=$L --config c6 --steps 100;c4|--config c4 --steps 60;c4o|VDB_LIB=$L --config c4 --steps 60;c3|--config c3 --steps 100;c3o|VDB_LIB=$L --config c3 --steps 100;s6|--config c6 --rows 1250000 --steps 200;s6o|VDB_LIB=$L --config c6 --rows 1250000 --steps 200;s4|--config c4 --rows 1250000 --steps 200;s4o|VDB_LIB=$L --config c4 --rows 1250000 --steps 200" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
