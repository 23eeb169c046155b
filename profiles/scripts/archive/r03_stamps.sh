#!/bin/bash
# Per-phase stamps of the int8 pass (stamp build lib/libvdb_amd_st8.so) on C6, C2, C3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-stamps}; mkdir -p $O
for c in c6 c2 c3; do
  timeout -k 10 200 python profiles/scripts/stamp_scan8.py $c > $O/stamp_$c.txt 2> $O/stamp_$c.err && cat $O/stamp_$c.txt || exit 1
done
