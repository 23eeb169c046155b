set -o pipefail
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD -d gpurun_out/pmc_sq -o run --output-format csv -- $B > gpurun_out/pmc_sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B > gpurun_out/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_tcc -o run --output-format csv -- $B > gpurun_out/pmc_tcc.log 2>&1
echo rc=$?
