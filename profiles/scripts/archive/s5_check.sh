#!/bin/bash
# Full GPU suite (incl. full-size C2-C5) + C2/C3/C4 bench lines at 1 and 2 streams.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for c in c2 c3 c4; do
  run ${c}_s1 --config $c --streams 1
  run ${c}_s2 --config $c --streams 2
done
run c2_s3 --config c2 --streams 3
