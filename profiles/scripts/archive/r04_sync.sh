#!/bin/bash
# int8 pass flag-gated step ends by default: the sync-mode / refinement parity tests and the
# full-size C2 / C3 tests, then same-box lines of the configs against the lockstep knob.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_sync2}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "sync_modes or refinement_modes" > $O/pytest_sync.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest_sync.log | head -20; tail -30 $O/pytest_sync.log; exit 1; }
tail -1 $O/pytest_sync.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -k "c2 or c3" > $O/pytest_full.log 2>&1 || { echo "pytest full failed"; grep -E "FAIL|Error" $O/pytest_full.log | head -20; tail -30 $O/pytest_full.log; exit 1; }
tail -1 $O/pytest_full.log
bash profiles/scripts/r04_matrix.sh $(basename $O)_ab "c2 c3 c6 c4" "base base:scan-sync=1"
