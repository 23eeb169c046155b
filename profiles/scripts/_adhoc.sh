set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_store.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_adhoc.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL|^E " gpurun_out/pytest_gpu_adhoc.log | head -40; tail -40 gpurun_out/pytest_gpu_adhoc.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_adhoc.log
