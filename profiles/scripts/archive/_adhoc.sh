set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r01_c5b
timeout -k 10 900 python -u bench.py --config c5 --steps 300 --warmup 20 > gpurun_out/r01_c5b/bench.json 2> gpurun_out/r01_c5b/bench.err || { tail -20 gpurun_out/r01_c5b/bench.err; exit 1; }
cat gpurun_out/r01_c5b/bench.json
