#!/bin/bash
# rocprofv3 evidence for one bench config: kernel-trace stats (csv) + separate
# PMC passes (HBM FETCH_SIZE / WRITE_SIZE, SQ busy/MFMA).  Counters never share
# a run with tracing domains (pool rule).  Usage: bash profiles/scripts/profile.sh TAG [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
ARGS="--steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $*"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || { echo "trace failed"; tail -20 $OUT/trace.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py $ARGS > $OUT/pmc_fetch_bench.json 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed"; tail -20 $OUT/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py $ARGS > $OUT/pmc_write_bench.json 2> $OUT/pmc_write.err || { echo "pmc write failed"; tail -20 $OUT/pmc_write.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/pmc_sq -o run -- python bench.py $ARGS > $OUT/pmc_sq_bench.json 2> $OUT/pmc_sq.err || { echo "pmc sq failed"; tail -20 $OUT/pmc_sq.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc_clk -o run -- python bench.py $ARGS > $OUT/pmc_clk_bench.json 2> $OUT/pmc_clk.err || { echo "pmc clk failed"; tail -20 $OUT/pmc_clk.err; exit 1; }
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
find $OUT -name '*.csv'
