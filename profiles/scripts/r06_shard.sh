#!/bin/bash
# Round 6: one rank's share of the strong-scaled 8-GPU runs, on one GPU: c6 (1.25M x 128, B = 64)
# and c4 (1.25M x 128, B = 512) -- the bench line (3 streams) and a one-stream kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_shard; mkdir -p $O
for c in c6 c4; do
  timeout -k 10 200 python3 bench.py --config $c --rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline > $O/${c}_line.json 2> $O/${c}_line.err || { tail -5 $O/${c}_line.err; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$c -o run -- python3 bench.py --config $c --rows 1250000 --streams 1 --steps 50 --warmup 5 --no-cpu-baseline > $O/${c}_trace.json 2> $O/${c}_trace.err || { tail -5 $O/${c}_trace.err; exit 1; }
  echo "$c done"
done
