#!/bin/bash
# Session-2 round-2 evidence: smoke, the default bench line, rocprofv3 kernel trace + PMC for C2/C3/C4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s7; mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python profiles/scripts/ab_line.py $O/bench_default.json default
for cp in c2:bf16 c3:bf16 c4:bf16x3; do
  c=${cp%%:*}; p=${cp##*:}
  STEPS=20 bash profiles/scripts/profile.sh r02s_${c}_${p} --config $c || exit 1
done
