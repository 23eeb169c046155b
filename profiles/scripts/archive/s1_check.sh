set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > gpurun_out/s1_pytest.log 2>&1 || { tail -40 gpurun_out/s1_pytest.log; exit 1; }
tail -2 gpurun_out/s1_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/s1_bench.json 2> gpurun_out/s1_bench.err || { tail -20 gpurun_out/s1_bench.err; exit 1; }
cat gpurun_out/s1_bench.json
