#!/bin/bash
# Round-3 check: GPU tests (optionally a -k filter), smoke, bench lines for the given configs.
# usage: r03_check.sh TAG [pytest -k expr or ""] [configs...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-a}; K=${2:-}; shift 2; CONFIGS="$@"
O=gpurun_out/$TAG; mkdir -p $O
if [ "$K" != "skip" ]; then
  if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
  timeout -k 10 900 python -u -m pytest tests -m "${MARK:-gpu}" -x -v --timeout 300 --timeout-method thread "${KARG[@]}" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
for c in $CONFIGS; do
  name=${c%%:*}; extra=""; [ "$c" != "$name" ] && extra=$(echo ${c#*:} | tr ',' ' ')
  timeout -k 10 500 python bench.py --config $name $extra > $O/bench_${name}.json 2> $O/bench_${name}.err || { echo "bench $c failed"; tail -30 $O/bench_${name}.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_${name}.json "$c"
done
