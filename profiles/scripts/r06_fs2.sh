#!/bin/bash
# Round 6: the finish's small form only while another search is in flight: tests, then C2 and the
# c6 shard (QPS under three streams, p50 one batch at a time) against finish_small 1 / 0.
set -o pipefail
O=gpurun_out/r06_fs2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_guards.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
A="--config c2 --steps 300"; H="--config c6 --rows 1250000 --steps 400"
AB="c2|$A;c2f1|$A --finish-small 1;c2f0|$A --finish-small 0;sh|$H;shf1|$H --finish-small 1" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
