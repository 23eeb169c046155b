#!/bin/bash
# Round 6: finish sub-phase stamps (certificate, refinement) at C2, B = 64 and B = 2.
set -o pipefail
O=gpurun_out/r06_st2; mkdir -p $O
timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c2 auto > $O/fin_c2.txt 2>&1 || { tail -20 $O/fin_c2.txt; exit 1; }
FIN_B=2 timeout -k 10 120 python -u profiles/scripts/fin_stamp.py c2 auto > $O/fin_c2_b2.txt 2>&1 || { tail -20 $O/fin_c2_b2.txt; exit 1; }
grep -v amdgpu $O/fin_*.txt
