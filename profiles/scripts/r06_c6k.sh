#!/bin/bash
# Round 6: c6 (10M x 128 cosine, B = 64, the 64-query shape) knobs once more on the final
# kernels: two workgroups per CU (--n-wg 512) and the pilot sample (1953 tiles by default).
set -o pipefail
A="--config c6 --steps 150"
AB="d|$A;w512|$A --n-wg 512;pt4k|$A --pilot-tiles 4096;pt1k|$A --pilot-tiles 1024" ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
