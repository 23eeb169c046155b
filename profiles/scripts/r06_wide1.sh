#!/bin/bash
# Round 6: the wide int8 pass -- its parity tests, then C4 with it (auto) against the 64-query shape.
set -o pipefail
mkdir -p gpurun_out/r06_wide1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wide.py \
  > gpurun_out/r06_wide1/pytest.txt 2>&1 || { tail -40 gpurun_out/r06_wide1/pytest.txt; exit 1; }
tail -3 gpurun_out/r06_wide1/pytest.txt
export AB="wide|--config c4;old|--config c4 --scan-wide 0"
ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
