#!/bin/bash
# Session-3 round-2 check at HEAD: every GPU test (fast + full-size), smoke, the default bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -30 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
