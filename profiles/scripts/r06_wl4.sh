#!/bin/bash
# Round 6: where the long-row wide pass beats the 64-query shape for small batches (one stream):
# C2 rows at B = 4 / 8 / 16 / 32, C3 rows at B = 2 / 16.
set -o pipefail
A="--streams 1 --steps 200"
AB="b4|--config c2 --batch 4 $A;b4w|--config c2 --batch 4 $A --scan-wide 1;b8|--config c2 --batch 8 $A;b8w|--config c2 --batch 8 $A --scan-wide 1;b16|--config c2 --batch 16 $A;b16w|--config c2 --batch 16 $A --scan-wide 1;b32|--config c2 --batch 32 $A;b32w|--config c2 --batch 32 $A --scan-wide 1;l2|--config c3 --batch 2 $A;l2w|--config c3 --batch 2 $A --scan-wide 1;l16|--config c3 --batch 16 $A;l16w|--config c3 --batch 16 $A --scan-wide 1" ROUNDS=1 T=200 bash profiles/scripts/r06_ab.sh
