#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_store.py tests/test_gpu_rest.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/r02b/pytest.log; exit 1; }
tail -1 gpurun_out/r02b/pytest.log
bash profiles/scripts/r02_stamp.sh
