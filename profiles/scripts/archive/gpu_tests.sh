#!/bin/bash
# GPU parity tests + smoke + bench lines for both candidate-pass precisions.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_$TAG.log | head -30; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke_$TAG.log; exit 1; }
for prec in bf16x3 fp32; do
  timeout -k 10 300 python bench.py --precision $prec --no-cpu-baseline > gpurun_out/bench_${TAG}_$prec.json 2> gpurun_out/bench_${TAG}_$prec.err || { echo "bench $prec failed"; tail -30 gpurun_out/bench_${TAG}_$prec.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$prec.json
done
