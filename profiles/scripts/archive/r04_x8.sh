#!/bin/bash
# 8-wave I8X3 L2 pass (VDB_S8_NW_X3L=8, one row tile per wave; lib/libvdb_amd_x8.so): guard,
# parity and full-size C4 tests first, then the same-box A/B against the base library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_x8}; mkdir -p $O
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_x8.so VDB_TEST_REPORT_DIR=$O/reports timeout -k 10 700 python -u -m pytest tests/test_gpu_guards.py tests/test_gpu_parity.py "tests/test_gpu_fullsize.py::test_c4_10m_x_128_l2_b512_top100" -m "gpu" -x -q --timeout 400 --timeout-method thread > $O/pytest_x8.log 2>&1 || { echo "x8 tests failed"; grep -E "FAIL|Error" $O/pytest_x8.log | head -20; tail -20 $O/pytest_x8.log; exit 1; }
tail -1 $O/pytest_x8.log
bash profiles/scripts/r04_ab.sh $(basename $O) "c4 c2" "base x8"
