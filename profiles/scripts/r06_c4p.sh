#!/bin/bash
# Round 6: C4's pilot sample with the wide pass: default (8192 tiles) vs 4096 / 6144 / 12288.
set -o pipefail
A="--config c4 --steps 100"
AB="d|$A;p4k|$A --pilot-tiles 4096;p6k|$A --pilot-tiles 6144;p12k|$A --pilot-tiles 12288" ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
