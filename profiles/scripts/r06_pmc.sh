#!/bin/bash
# Round 6: one-stream kernel trace + PMC passes of one bench config (optionally another library):
#   TAG=... LIB=... bash profiles/scripts/r06_pmc.sh [bench args]   ->  gpurun_out/pmc_$TAG/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_$TAG; mkdir -p $O
ARGS="--streams 1 --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-serving --no-metric-workload --no-other-configs $*"
[ -n "$LIB" ] && export VDB_LIB=$LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py $ARGS > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/pmc_sq -o run -- python3 bench.py $ARGS > $O/pmc_sq_bench.json 2> $O/pmc_sq.err || { tail -20 $O/pmc_sq.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM --output-format csv -d $O/pmc_b -o run -- python3 bench.py $ARGS > $O/pmc_b_bench.json 2> $O/pmc_b.err || { tail -20 $O/pmc_b.err; exit 1; }
echo "pmc $TAG done"
