#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/stamp
for a in "0 0 bf16 c2" "1 0 bf16 c2" "0 0 bf16x3 c2" "0 0 bf16x3 c4"; do
  timeout -k 10 200 python profiles/scripts/stamp_scan.py $a > "gpurun_out/stamp/$(echo $a | tr ' ' _).txt" 2>&1 || { echo "stamp $a failed"; tail -20 "gpurun_out/stamp/$(echo $a | tr ' ' _).txt"; exit 1; }
  cat "gpurun_out/stamp/$(echo $a | tr ' ' _).txt"
done
