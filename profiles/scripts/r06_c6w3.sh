#!/bin/bash
# Round 6: the split short-row wide pass with a small stage (8 tiles, 32 KiB slots) and the
# finish's small form beside it: tests, then c6 (forced) and its shard.
set -o pipefail
O=gpurun_out/r06_c6w3; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
AB="c6|--config c6 --steps 100;c6w|--config c6 --steps 100 --scan-wide 1;c6wf0|--config c6 --steps 100 --scan-wide 1 --finish-small 0;sh|--config c6 --rows 1250000 --steps 400;shf0|--config c6 --rows 1250000 --steps 400 --finish-small 0" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
