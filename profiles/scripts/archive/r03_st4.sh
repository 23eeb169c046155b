#!/bin/bash
# Per-phase stamps of the I8X3 L2 pass on C4 (stamp build lib/libvdb_amd_st8.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-st4}; mkdir -p $O
timeout -k 10 200 python profiles/scripts/stamp_scan8.py c4 i8x3 > $O/stamp_c4.txt 2> $O/stamp_c4.err && cat $O/stamp_c4.txt || { tail -20 $O/stamp_c4.err; exit 1; }
