#!/bin/bash
# Same-box matrix: r04_matrix.sh TAG "configs" "entry entry ..."
# entry = variant[:flag=value[:flag=value]]; variant "base" = lib/libvdb_amd.so, otherwise
# lib/libvdb_amd_<variant>.so; flags are bench.py flags without the leading "--".  Two rounds, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_matrix}; mkdir -p $O
for rep in 1 2; do for c in $2; do for e in $3; do
  IFS=: read -r v rest <<< "$e"
  if [ $v = base ]; then L=""; else L="VDB_LIB=mlx-vector-db_amd/lib/libvdb_amd_$v.so"; fi
  args=""
  if [ -n "$rest" ]; then for kv in ${rest//:/ }; do args="$args --${kv%%=*} ${kv#*=}"; done; fi
  n=$(echo "${c}_$e" | tr ':=' '__')
  env $L timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving --no-metric-workload $args > $O/${n}_$rep.json 2> $O/${n}_$rep.err || { echo "bench $c $e failed"; tail -20 $O/${n}_$rep.err; exit 1; }
  python profiles/scripts/ab_line.py $O/${n}_$rep.json "${c} $e #$rep"
done; done; done
