#!/bin/bash
# Round 6: the pilot bound's rank at C2 (B = 64) for the 64-query shape and the long-row wide pass
# (whose lists take every row above the bound): default rank (Poisson + 2 KP rule: 9) vs 5 / 3,
# fallbacks counted.
set -o pipefail
A="--config c2 --steps 200"
AB="c2|$A;c2p5|$A --pilot-rank 5;c2w|$A --scan-wide 1;c2wp5|$A --scan-wide 1 --pilot-rank 5;c2wp3|$A --scan-wide 1 --pilot-rank 3" ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
