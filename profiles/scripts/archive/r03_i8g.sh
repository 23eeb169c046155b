#!/bin/bash
# A/B: plane-major corpus copies (VDB_PLANE_MAJOR: the I8 hi plane of a super tile contiguous)
# vs the default group-major order; FETCH_SIZE of the scan per launch for both at C6.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-i8g}; mkdir -p $O
run() {  # tag lib config [extra args]
  t=$1; l=$2; c=$3; shift 3
  VDB_LIB=$l timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-serving "$@" > $O/bench_$t.json 2> $O/bench_$t.err || { echo "bench $t failed"; tail -30 $O/bench_$t.err; exit 1; }
  python profiles/scripts/ab_line.py $O/bench_$t.json $t
}
L=mlx-vector-db_amd/lib
run c6_def $L/libvdb_amd.so c6 && run c6_pm $L/libvdb_amd_pm.so c6 && run c2_def $L/libvdb_amd.so c2 && run c2_pm $L/libvdb_amd_pm.so c2 || exit 1
for v in def pm; do
  l=$L/libvdb_amd.so; [ $v = pm ] && l=$L/libvdb_amd_pm.so
  VDB_LIB=$l timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run -- python bench.py --config c6 --streams 1 --steps 20 --warmup 3 --no-cpu-baseline --no-serving > $O/pmc_$v.json 2> $O/pmc_$v.err || { echo "pmc $v failed"; tail -20 $O/pmc_$v.err; exit 1; }
done
O=$O python3 - <<'PY'
import csv, glob, os
O = os.environ['O']
for v in ("def", "pm"):
    f = glob.glob(f"{O}/pmc_{v}/**/*counter_collection.csv", recursive=True)
    if not f: print(v, "no csv"); continue
    rows = [r for r in csv.DictReader(open(f[0])) if "scan8_kernel" in r.get("Kernel_Name", "")]
    vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == "FETCH_SIZE"]
    print(v, "scan8 launches", len(vals), "FETCH_SIZE KB avg", sum(vals) / max(len(vals), 1))
PY
