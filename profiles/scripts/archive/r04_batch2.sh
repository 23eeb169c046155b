#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_batch2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_guards.py -m gpu -x -v --timeout 200 --timeout-method thread -k "repass or auto or q4 or consistency or i8 or golden" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 0 1; do for c in c2 c3 c6; do VDB_FIN_REFINE=$r timeout -k 10 200 python profiles/scripts/fin_stamp.py $c auto 2>/dev/null | sed "s/^/refine $r: /" || exit 1; done; done
bash profiles/scripts/r04_knob.sh r04_refine2 "c2 c6 c3" --i8-refine "0 1" || exit 1
bash profiles/scripts/r04_knob.sh r04_plant2 "c2" --device-repass "0 1" "--plant-close 1"
