#!/bin/bash
# Session-3 A/B: finish cut, slot publishing, flag-gated step ends with nt loads, streams, timing events.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
O=gpurun_out/s3
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "bench $tag failed"; tail -20 $O/$tag.err; exit 1; }
  python - $O/$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:24s} qps {r['value']:9.0f} ms/step {r['ms_per_step']:.4f} p50 {r['p50_ms']:.4f} scan {r['roofline']['avg_launch_ms']:.4f} pipe {r['pipeline_ms']:.4f} frac {r['roofline']['frac']:.3f} prec {r['roofline']['precision']} fb {r['fallback_queries_timed']}")
PY
}
run c2_def
run c2_pub1 --scan-publish 1
run c2_fs --scan-sync 2
run c2_fs_pub1 --scan-sync 2 --scan-publish 1
run c2_str2 --streams 2
run c2_tim0 --timing 0
run c2_b3 --precision bf16x3
run c2_b3_fs --precision bf16x3 --scan-sync 2
run c3_def --config c3
run c4_def --config c4
