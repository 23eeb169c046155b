#!/bin/bash
# Same-box sweep of one bench knob: r04_knob.sh TAG "configs" "--flag" "values" [extra args]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_knob}; mkdir -p $O
for rep in 1 2; do for c in $2; do for v in $4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving --no-metric-workload $3 $v $5 > $O/${c}_${v}_$rep.json 2> $O/${c}_${v}_$rep.err || { echo "bench $c $v failed"; tail -20 $O/${c}_${v}_$rep.err; exit 1; }
  python profiles/scripts/ab_line.py $O/${c}_${v}_$rep.json "${c} $3 $v #$rep"
done; done; done
