set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_adhoc.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu_adhoc.log | head -20; tail -30 gpurun_out/pytest_gpu_adhoc.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_adhoc.log
bash profiles/scripts/sweep.sh bf16x3 c2 "0 1" "0" || exit 1
bash profiles/scripts/sweep.sh fp32 c2 "0" "0" || exit 1
OUT=gpurun_out/prof_adhoc
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
