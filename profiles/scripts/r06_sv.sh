#!/bin/bash
# Round 6: store serving modes (in flight, linger us) with the final kernels.
set -o pipefail
O=gpurun_out/r06_sv; mkdir -p $O
timeout -k 10 400 python -u profiles/scripts/serving_ab6.py 1600 > $O/serving.txt 2>&1 || { tail -20 $O/serving.txt; exit 1; }
cat $O/serving.txt
