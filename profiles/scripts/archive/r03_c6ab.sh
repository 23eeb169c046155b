#!/bin/bash
# C6 (10M x 128 cosine, B = 64) step-end / query-operand A/B, plus the default bench line (c2 + c6 sub-record)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-c6ab}; mkdir -p $O
run() { name=$1; shift; timeout -k 10 300 python bench.py --config c6 --no-cpu-baseline --steps 40 "$@" > $O/$name.json 2> $O/$name.err || { echo "bench $name failed"; tail -20 $O/$name.err; exit 1; }; python profiles/scripts/ab_line.py $O/$name.json "$name"; }
run def
run sync1 --scan-sync 1
run qlds0 --scan-qlds 0
run qlds0_sync1 --scan-qlds 0 --scan-sync 1
run pub0 --scan-publish 0
run str1 --streams 1
timeout -k 10 400 python bench.py --no-serving > $O/default.json 2> $O/default.err || { echo "default bench failed"; tail -20 $O/default.err; exit 1; }
python - $O/default.json <<'PY'
import json,sys
r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m=r.get("metric_workload_10m_x_128",{})
print("default c2", round(r["value"]), "c6 sub", round(m.get("value",0)), m.get("p50_ms"), m.get("roofline",{}).get("frac"))
PY
