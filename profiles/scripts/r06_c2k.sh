#!/bin/bash
# Round 6, final kernels: C2 (the headline line) streams and pilot sample re-checked.
set -o pipefail
AB="d|--steps 200;st2|--steps 200 --streams 2;st4|--steps 200 --streams 4;pt256|--steps 200 --pilot-tiles 256;pt1k|--steps 200 --pilot-tiles 1024" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
