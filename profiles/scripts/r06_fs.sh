#!/bin/bash
# Round 6: the finish's small form beside the long-row wide scan: wide tests + parity, then C2 and
# small batches with and without it.
set -o pipefail
O=gpurun_out/r06_fs; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
S="--streams 1 --steps 200"
AB="c2|--config c2 --steps 200;c2f0|--config c2 --steps 200 --finish-small 0;b2|--config c2 --batch 2 $S;b2f0|--config c2 --batch 2 $S --finish-small 0;sh|--config c6 --rows 1250000 --steps 400" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
