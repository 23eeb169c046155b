#!/bin/bash
# scan2 per-wave phase stamps (diagnostic build lib/libvdb_amd_st.so) for C2 bf16 / bf16x3, C3, C4.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "c2 bf16" "c2 bf16x3" "c4 bf16x3" "c3 bf16x3"; do
  timeout -k 10 240 python profiles/scripts/stamp_scan2.py $a >> gpurun_out/s2_stamp.txt 2>> gpurun_out/s2_stamp.err || { tail -20 gpurun_out/s2_stamp.err; exit 1; }
done
cat gpurun_out/s2_stamp.txt
