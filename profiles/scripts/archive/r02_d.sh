#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -30; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/scripts/r02_kl.sh
