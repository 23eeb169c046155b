#!/bin/bash
# One-loop step of the int8 and bf16 passes (VDB_S8_ONELOOP=1 VDB_S2_ONELOOP=1, lib/libvdb_amd_ol.so): its parity tests first, then the
# same-box A/B against the base library on C2 / C3 / C6 / C4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_ol}; mkdir -p $O
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_ol.so timeout -k 10 600 python -u -m pytest tests/test_gpu_guards.py tests/test_gpu_parity.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_ol.log 2>&1 || { echo "ol tests failed"; grep -E "FAIL|Error" $O/pytest_ol.log | head -20; tail -20 $O/pytest_ol.log; exit 1; }
tail -1 $O/pytest_ol.log
bash profiles/scripts/r04_ab.sh $(basename $O) "c2 c3 c6 c4" "base ol"
bash profiles/scripts/r04_ab.sh $(basename $O)_x3 "c2" "base ol" "--precision bf16x3"
