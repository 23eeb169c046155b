#!/bin/bash
# Round 6: finish latency knobs at small batches (one stream, p50 = one batch at a time): the I8
# refinement off and several workgroups per query (finish_split), C2 B = 2 and the c6 shard (B = 64).
set -o pipefail
B2="--config c2 --batch 2 --streams 1 --steps 300"
SH="--config c6 --rows 1250000 --streams 1 --steps 300"
AB="b2|$B2;b2r0|$B2 --i8-refine 0;b2s4|$B2 --finish-split 4;b2s8|$B2 --finish-split 8;b2r0s8|$B2 --i8-refine 0 --finish-split 8;sh|$SH;shs2|$SH --finish-split 2;shs4|$SH --finish-split 4" \
  ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
