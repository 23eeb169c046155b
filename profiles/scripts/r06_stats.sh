#!/bin/bash
# Round 6, final binary: rocprofv3 --kernel-trace --stats of the default bench command (C2 line +
# the c6 sub-record), for the per-kernel averages beside the line's HIP-event scan time.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_stats; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 50 --warmup 5 --no-serving --no-other-configs --no-cpu-baseline > $O/line.json 2> $O/line.err || { tail -5 $O/line.err; exit 1; }
tail -1 $O/line.json | cut -c1-300
