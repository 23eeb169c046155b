#!/bin/bash
# Slot publishing A/B (scan_publish auto = on with >= 16 steps per workgroup) and step ends.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-pub}; mkdir -p $O
run() { c=$1; name=$2; shift 2; timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 40 "$@" > $O/${c}_$name.json 2> $O/${c}_$name.err || { echo "bench $c $name failed"; tail -20 $O/${c}_$name.err; exit 1; }; python profiles/scripts/ab_line.py $O/${c}_$name.json "${c}_$name"; }
run c6 def
run c6 pub0 --scan-publish 0
run c6 pub0_sync1 --scan-publish 0 --scan-sync 1
run c3 def
run c3 pub0 --scan-publish 0
run c4 def
run c4 sync1 --scan-sync 1
run c4 q40 --scan-q4 0
run c4 q40_pub0 --scan-q4 0 --scan-publish 0
run c2 def
run c2 pub1 --scan-publish 1
