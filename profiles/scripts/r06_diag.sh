#!/bin/bash
# Round 6: serving diagnosis (store / native host / native device layers, 1 and 4 threads) at C2.
set -o pipefail
O=gpurun_out/r06_diag; mkdir -p $O
timeout -k 10 400 python -u profiles/scripts/serving_diag6.py > $O/diag.txt 2>&1 || { tail -20 $O/diag.txt; exit 1; }
cat $O/diag.txt
