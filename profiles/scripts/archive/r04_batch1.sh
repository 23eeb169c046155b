#!/bin/bash
# Round-4 batch: correctness of the new paths first (device re-pass, int8 q4 shape, I8
# refinement, guards, the two-step variant), then same-box A/B lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04_batch1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_guards.py -m gpu -x -v --timeout 200 --timeout-method thread -k "repass or device or auto or q4 or guard or first or consistency or add_waits or i8 or golden or random_uniform" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log; grep -E "re-passed" $O/pytest.log | head -3
VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_two.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_guards.py -m gpu -x -q --timeout 200 --timeout-method thread -k "i8 or golden or random_uniform or first" > $O/pytest_two.log 2>&1 || { echo "pytest two failed"; grep -E "FAIL|Error" $O/pytest_two.log | head -20; tail -30 $O/pytest_two.log; exit 1; }
tail -1 $O/pytest_two.log
bash profiles/scripts/r04_ab.sh r04_two "c6 c2" "base two" || exit 1
bash profiles/scripts/r04_knob.sh r04_refine "c2 c6 c3" --i8-refine "0 1" || exit 1
bash profiles/scripts/r04_ab.sh r04_fw8 "c2 c3" "base fw8" || exit 1
bash profiles/scripts/r04_knob.sh r04_rep "c2" --device-repass "0 1" || exit 1
bash profiles/scripts/r04_knob.sh r04_q48 "c4" --scan-q4 "0 -1" || exit 1
bash profiles/scripts/r04_knob.sh r04_plant "c2" --device-repass "0 1" "--plant-close 1"
