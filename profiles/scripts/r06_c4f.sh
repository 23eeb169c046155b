#!/bin/bash
# Round 6: C4's finish in its small form (4 waves, 3 workgroups per CU instead of 1) vs the 16-wave.
set -o pipefail
A="--config c4 --steps 100"
AB="d|$A;f1|$A --finish-small 1;s4d|--config c4 --rows 1250000 --steps 200;s4f1|--config c4 --rows 1250000 --steps 200 --finish-small 1" ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
