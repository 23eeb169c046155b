#!/bin/bash
# Default-run shape: streams (batches in flight) and timed steps for the C2 line, C4 streams.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s15; mkdir -p $O
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python profiles/scripts/ab_line.py $O/$tag.json $tag
}
for rep in 1 2; do
  for s in 2 3 4 6; do run c2_str${s}_k20_$rep --streams $s; done
  for s in 3 4; do run c2_str${s}_k100_$rep --streams $s --steps 100; done
done
run c4_str3 --config c4
run c4_str4 --config c4 --streams 4
run c3_str3 --config c3
run c3_str4 --config c3 --streams 4
