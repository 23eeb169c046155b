#!/bin/bash
# Kernel trace only (per-kernel averages) for a list of bench configs: TAG "cfg:prec ..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
for cp in $1; do
  c=${cp%%:*}; p=${cp##*:}
  OUT=gpurun_out/trace_${TAG}_${c}_${p}
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --config $c --precision $p > $OUT/bench.json 2> $OUT/err.txt || { echo "trace $cp failed"; tail -5 $OUT/err.txt; exit 1; }
  python - "$OUT" <<'PY'
import csv, sys, json
out = sys.argv[1]
b = json.load(open(out + "/bench.json"))
print(out, "value", round(b["value"]), "step_ms", round(b["ms_per_step"], 4))
for r in csv.DictReader(open(out + "/run_kernel_stats.csv")):
    if int(r["Calls"]) >= 20:
        print("   %-60s %6s %9.1f us" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
