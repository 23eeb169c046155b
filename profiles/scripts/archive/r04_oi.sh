#!/bin/bash
# Insertions with the step's thresholds and a wave-uniform register index (VDB_S8_INS2=1 on top of
# the one-loop step, lib/libvdb_amd_oi.so): its parity tests first, then the same-box A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_oi}; mkdir -p $O
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_oi.so timeout -k 10 600 python -u -m pytest tests/test_gpu_guards.py tests/test_gpu_parity.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_oi.log 2>&1 || { echo "oi tests failed"; grep -E "FAIL|Error" $O/pytest_oi.log | head -20; tail -20 $O/pytest_oi.log; exit 1; }
tail -1 $O/pytest_oi.log
bash profiles/scripts/r04_ab.sh $(basename $O) "${CONFIGS:-c2 c6 c3 c4}" "${VARIANTS:-ol oi}"
