#!/bin/bash
# Round 6: store-level serving A/B (coalescer inflight x linger) and finish-kernel phase stamps at
# the c6 shard shape (1.25M x 128, B = 64), C2 and C3 (diagnostic stamp build).
set -o pipefail
O=gpurun_out/r06_serve; mkdir -p $O
timeout -k 10 400 python -u profiles/scripts/serving_ab6.py 1600 > $O/serving.txt 2>&1 || { tail -20 $O/serving.txt; exit 1; }
cat $O/serving.txt
FIN_ROWS=1250000 timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c6 auto > $O/fin_c6shard.txt 2>&1 || { tail -20 $O/fin_c6shard.txt; exit 1; }
timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c2 auto > $O/fin_c2.txt 2>&1 || { tail -20 $O/fin_c2.txt; exit 1; }
timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c3 auto > $O/fin_c3.txt 2>&1 || { tail -20 $O/fin_c3.txt; exit 1; }
cat $O/fin_*.txt
