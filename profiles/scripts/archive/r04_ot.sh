#!/bin/bash
# Insertions with the step's thresholds in the first round (VDB_S8_INSTHR=1, per-lane select kept;
# lib/libvdb_amd_ot.so): its parity tests first, then the same-box A/B against the base library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_ot}; mkdir -p $O
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_ot.so timeout -k 10 600 python -u -m pytest tests/test_gpu_guards.py tests/test_gpu_parity.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_ot.log 2>&1 || { echo "ot tests failed"; grep -E "FAIL|Error" $O/pytest_ot.log | head -20; tail -20 $O/pytest_ot.log; exit 1; }
tail -1 $O/pytest_ot.log
bash profiles/scripts/r04_ab.sh $(basename $O) "${CONFIGS:-c2 c6 c3 c4}" "${VARIANTS:-ol oi}"
