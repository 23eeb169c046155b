#!/bin/bash
# Session-3 round-end evidence at HEAD: all GPU tests (full sizes included), smoke, the default
# bench line (C2, CPU baseline), C3 and C4 lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -30 $O/bench_c2.err; exit 1; }
python profiles/scripts/ab_line.py $O/bench_c2.json c2_default
for c in c3 c4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { echo "bench $c failed"; tail -30 $O/bench_$c.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$c.json ${c}_default
done
