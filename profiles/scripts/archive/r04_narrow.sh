#!/bin/bash
# auto's I8 KP = 128 on small indexes (i8_narrow): the non-full-size GPU suite, then the per-rank
# shapes of weak-scaled C2 runs (rows / N, batch x N) and the default lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_narrow}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash profiles/scripts/r04_matrix.sh $(basename $O)_ab "c2" "base base:rows=500000:batch=128 base:rows=250000:batch=256 base:rows=125000:batch=512"
