#!/bin/bash
# Round-end evidence in one call: GPU parity tests, smoke, default bench line (C2 with CPU
# baseline), C4 bench line.  Usage: bash profiles/scripts/final_check.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -30 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { echo "bench c4 failed"; tail -30 $O/bench_c4.err; exit 1; }
cat $O/bench_c4.json
