set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
for v in base nt; do
  if [ $v = nt ]; then export VDB_LIB=$PWD/mlx-vector-db_amd/lib/libvdb_amd_nt.so; else unset VDB_LIB; fi
  timeout -k 10 200 python -u bench.py --config c2 --steps 100 --no-cpu-baseline > gpurun_out/ab_$v$i.json 2>gpurun_out/ab_$v$i.err || { tail gpurun_out/ab_$v$i.err; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/ab_$v$i.json'));print('$v$i', round(r['value']), 'scan', round(r['roofline']['avg_launch_ms']*1e3,1), 'pipe', round(r['pipeline_ms']*1e3,1))"
done
done
