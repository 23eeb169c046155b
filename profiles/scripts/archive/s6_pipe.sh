#!/bin/bash
# Pipelined short-row scan (scan2p_kernel): parity + C4 A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s6; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
run c4_pipe1 --config c4 --streams 1
run c4_pipe0 --config c4 --streams 1 --scan-pipe 0
run c4_pipe1_s3 --config c4
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m "gpu and slow" -x -q -k c4 --timeout 400 --timeout-method thread > $O/pytest_c4.log 2>&1 || { tail -40 $O/pytest_c4.log; exit 1; }
tail -2 $O/pytest_c4.log
