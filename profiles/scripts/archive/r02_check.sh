#!/bin/bash
# Round-2 GPU check: parity tests (fast set, then the full-size BASELINE configs), smoke.
# Usage: bash profiles/scripts/r02_check.sh TAG [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
export VDB_TEST_REPORT_DIR=$O/reports
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 900 python -u -m pytest tests -m "gpu and slow" -x -v -s --timeout 400 --timeout-method thread ${K:+-k "$K"} > $O/pytest_slow.log 2>&1 || { echo "slow pytest failed"; tail -60 $O/pytest_slow.log; exit 1; }
grep -E "PASSED|FAILED|json" $O/pytest_slow.log | tail -20
tail -1 $O/pytest_slow.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
