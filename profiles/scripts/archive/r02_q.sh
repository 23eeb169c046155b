#!/bin/bash
# Graph: incremental insertion parity + C5 bench (row-major rows of the index).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py --config c5 --steps 100 --warmup 5 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail -20 $O/c5.err; exit 1; }
python -c "import json;d=json.load(open('$O/c5.json'));print({k:d[k] for k in ('value','p50_ms','recall_at_10','build_s','exact_b1_p50_ms','teams_sweep')})"
