#!/bin/bash
# Round 6: the full-size certificate tests on hostile data, then the default bench line (now with c5).
set -o pipefail
O=gpurun_out/r06_hostile; mkdir -p $O
VDB_TEST_REPORT_DIR=$O timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -k hostile -v -s --timeout 900 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
grep -E "passed|failed|hostile_" $O/pytest.txt | tail -5
timeout -k 10 480 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('c2', round(d['value']), d['ms_per_step'])
for k in ('metric_workload_10m_x_128','config_c3','config_c4'):
  s=d.get(k); print(k, round(s['value']), s['ms_per_step'], 'cpu', s.get('cpu_baseline',{}).get('value'))
c5=d.get('config_c5'); print('c5', {k: c5.get(k) for k in ('value','p50_ms','recall_at_10','exact_b1_p50_ms','visited_per_query','build_s')}, 'cpu', c5.get('cpu_baseline',{}).get('value'))"
