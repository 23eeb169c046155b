#!/bin/bash
# Round 6: the long-row wide pass with a deeper ring for shorter rows (up to 6 tiles), forced on
# for C2's 64-query batches (--scan-wide 1) against the 64-query shape; C3 unchanged (3 tiles).
set -o pipefail
O=gpurun_out/r06_wl3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB="c2|--config c2 --steps 200;c2w|--config c2 --steps 200 --scan-wide 1;c3|--config c3 --steps 100;b2|--config c2 --batch 2 --streams 1 --steps 200;b2w|--config c2 --batch 2 --streams 1 --steps 200 --scan-wide 1" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
