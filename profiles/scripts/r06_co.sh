#!/bin/bash
# Round 6: the coalescer with per-caller wake events and slot hand-off: store / REST GPU tests,
# then the store-level serving A/B (C2, 4 threads).
set -o pipefail
O=gpurun_out/r06_co; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_store.py tests/test_gpu_rest.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 400 python -u profiles/scripts/serving_ab6.py 1600 > $O/serving.txt 2>&1 || { tail -20 $O/serving.txt; exit 1; }
cat $O/serving.txt
