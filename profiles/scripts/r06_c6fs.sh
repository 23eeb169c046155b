#!/bin/bash
# Round 6: c6 (10M x 128 cosine B = 64, the 64-query shape, whose scans overlap each other 100%
# of the loop) with the finish's small form forced (43 KiB: beside a scan workgroup of 57 KiB)
# against auto (the 16-wave form, 134 KiB: waits for a CU no scan holds).
set -o pipefail
AB="d|--config c6 --steps 150;fs1|--config c6 --steps 150 --finish-small 1" ROUNDS=2 T=240 bash profiles/scripts/r06_ab.sh
