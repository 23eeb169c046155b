#!/bin/bash
# C2 step-end A/B: lockstep vs flag-gated with a realign barrier every n steps (one stream).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s8; mkdir -p $O
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
run c2_lock_$rep --streams 1
run c2_fs_r0_$rep --streams 1 --scan-sync 2
run c2_fs_r2_$rep --streams 1 --scan-sync 2 --scan-realign 2
run c2_fs_r4_$rep --streams 1 --scan-sync 2 --scan-realign 4
done
run c3_lock --config c3 --streams 1
run c3_fs_r2 --config c3 --streams 1 --scan-sync 2 --scan-realign 2
run c3_fs_r8 --config c3 --streams 1 --scan-sync 2 --scan-realign 8
