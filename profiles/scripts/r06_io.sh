#!/bin/bash
# Round 6: host-memory searches through pinned staging (one synchronisation): parity / store /
# REST / guard tests, then the serving diagnosis and the store-level serving A/B.
set -o pipefail
O=gpurun_out/r06_io; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_store.py tests/test_gpu_rest.py tests/test_gpu_guards.py \
  tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -u profiles/scripts/serving_diag6.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
timeout -k 10 400 python -u profiles/scripts/serving_ab6.py 1600 > $O/serving.txt 2>&1 || { tail -20 $O/serving.txt; exit 1; }
cat $O/serving.txt
