"""One summary line of a bench.py JSON result (A/B scripts)."""
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ro = r["roofline"]
print(f"{sys.argv[2]:24s} qps {r['value']:9.0f} ms/step {r['ms_per_step']:.4f} p50 {r['p50_ms']:.4f} "
      f"scan {ro['avg_launch_ms']:.4f} pipe {r['pipeline_ms']:.4f} frac {ro['frac']:.3f} prec {ro['precision']} "
      f"fb {r['fallback_queries_timed']}")
