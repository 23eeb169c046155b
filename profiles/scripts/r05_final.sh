#!/bin/bash
# Round 5 final evidence at one commit: guard tests (fresh-process first searches, the consistency
# guard, the checksum's planted under-scoring fault -- printed with -s), the whole GPU suite (full
# sizes unless $2 = quick), smoke, and the default bench line (C2 + c6 / c3 / c4 sub-records).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r05_final}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_guards.py -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/pytest_guards.log 2>&1 || { echo "guards failed"; grep -E "FAIL|Error" $O/pytest_guards.log | head -40; tail -30 $O/pytest_guards.log; exit 1; }
grep -E "checksum off" $O/pytest_guards.log | head; tail -1 $O/pytest_guards.log
SEL="gpu"; [ "$2" = quick ] && SEL="gpu and not slow"
VDB_TEST_REPORT_DIR=$O/reports timeout -k 10 900 python -u -m pytest tests -m "$SEL" -x -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "default bench failed"; tail -30 $O/bench_default.err; exit 1; }
python profiles/scripts/ab_line.py $O/bench_default.json default_c2
