#!/bin/bash
# Round 6: C2 on the long-row wide pass: streams (2 / 3 / 4) and scan workgroups (256 / 240 / 224,
# leaving CUs to the other streams' side kernels).
set -o pipefail
A="--config c2 --steps 300"
AB="s3|$A;s2|$A --streams 2;s4|$A --streams 4;n240|$A --n-wg 240;n224|$A --n-wg 224;n192|$A --n-wg 192" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
