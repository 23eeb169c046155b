#!/bin/bash
# Round 6: the short-row wide pass with a 64-query block's stage tiles split over 8 waves (rw = 8)
# forced on for c6 (10M x 128 cosine, B = 64) and its shard shape, against the 64-query shape.
set -o pipefail
O=gpurun_out/r06_c6w2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB="c6|--config c6 --steps 100;c6w|--config c6 --steps 100 --scan-wide 1;sh|--config c6 --rows 1250000 --steps 400;shw|--config c6 --rows 1250000 --steps 400 --scan-wide 1;c4|--config c4 --steps 100" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
