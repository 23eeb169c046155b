#!/bin/bash
# Same-box A/B of library variants: r04_ab.sh TAG "configs" "variants" [extra bench args]
# variant "base" = lib/libvdb_amd.so, otherwise lib/libvdb_amd_<variant>.so; two rounds, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_ab}; mkdir -p $O
for rep in 1 2; do for c in $2; do for v in $3; do
  if [ $v = base ]; then L=""; else L="VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_$v.so"; fi
  env $L timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving --no-metric-workload $4 > $O/${c}_${v}_$rep.json 2> $O/${c}_${v}_$rep.err || { echo "bench $c $v failed"; tail -20 $O/${c}_${v}_$rep.err; exit 1; }
  python profiles/scripts/ab_line.py $O/${c}_${v}_$rep.json ${c}_${v}_$rep
done; done; done
