#!/bin/bash
# Round 6: the gated exact scan without LDS (global scratch) -- its parity tests, a one-stream C3
# trace (the empty gated launch's duration) -- then finish-wave A/B (16 default, 8, 4) on C3, C2 and
# the c6 shard shape (1.25M x 128, B = 64).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_gate; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_guards.py -x -v \
  --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 bench.py --config c3 \
  --streams 1 --steps 50 --warmup 5 --no-cpu-baseline > $O/c3_trace.json 2> $O/c3_trace.err || { tail -5 $O/c3_trace.err; exit 1; }
python3 - <<EOF
import csv, glob
for f in glob.glob('$O/trace_c3/**/run_kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print('c3 1-stream', r['Name'][:60], r['Calls'], '%.1f us' % (float(r['AverageNs']) / 1e3))
EOF
L4=mlx-vector-db_amd/lib/libvdb_amd_fw4.so; L8=mlx-vector-db_amd/lib/libvdb_amd_fw8.so
AB="c3|--config c3 --steps 100;c3fw8|VDB_LIB=$L8 --config c3 --steps 100;c2|--config c2 --steps 200;c2fw8|VDB_LIB=$L8 --config c2 --steps 200;c2fw4|VDB_LIB=$L4 --config c2 --steps 200;sh|--config c6 --rows 1250000 --steps 400;shfw8|VDB_LIB=$L8 --config c6 --rows 1250000 --steps 400;shfw4|VDB_LIB=$L4 --config c6 --rows 1250000 --steps 400" \
  ROUNDS=2 T=200 bash profiles/scripts/r06_ab.sh
