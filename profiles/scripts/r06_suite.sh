#!/bin/bash
# Round 6: the whole GPU suite, smoke, then the default bench line (with every sub-record's CPU baseline).
set -o pipefail
O=gpurun_out/${TAG:-r06_suite}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
cat $O/smoke.txt
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('c2', round(d['value']), d['ms_per_step'], d['roofline']['avg_launch_ms'], 'cpu', d.get('cpu_baseline',{}).get('value'))
for k in ('metric_workload_10m_x_128','config_c3','config_c4'):
  s=d.get(k); print(k, round(s['value']), s['ms_per_step'], s['roofline']['avg_launch_ms'], round(s['roofline']['frac'],3), 'cpu', s.get('cpu_baseline',{}).get('value'))
c5=d.get('config_c5') or {}; print('c5', {k: c5.get(k) for k in ('value','p50_ms','recall_at_10','exact_b1_p50_ms')}, 'cpu', (c5.get('cpu_baseline') or {}).get('value'))
print(d['serving'])"
