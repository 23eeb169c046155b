#!/bin/bash
# Round 6, final kernels (spill-free finish forms): the finish's small form under auto against
# the 16-wave form (--finish-small 0) at C4, the c4 shard and C2.
set -o pipefail
AB="c4|--config c4 --steps 60;c4f0|--config c4 --steps 60 --finish-small 0;s4|--config c4 --rows 1250000 --steps 200;s4f0|--config c4 --rows 1250000 --steps 200 --finish-small 0;c2|--steps 200;c2f0|--steps 200 --finish-small 0" \
  ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
