#!/bin/bash
# Evidence at HEAD: all GPU tests (full sizes included), smoke, the default bench line (C2 + the
# metric's c6 sub-record, CPU baseline, serving), the c3 / c4 / c6 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-final}; mkdir -p $O
VDB_TEST_REPORT_DIR=$O/reports timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -30 $O/bench_default.err; exit 1; }
python profiles/scripts/ab_line.py $O/bench_default.json default_c2
for c in c6 c3 c4; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -30 $O/bench_$c.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$c.json $c
done
