#!/bin/bash
# C4 diagnosis: PMC passes on the scan kernel, flag-gated vs lockstep step ends.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c4diag
mkdir -p $O
B="python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline"
pass() { local tag=$1; shift; local sync=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $O/$tag -o run -- $B --scan-sync $sync > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; return 1; }
}
for sync in 2 1; do
  pass sq1_s$sync $sync SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
  pass sq2_s$sync $sync SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU || exit 1
  pass ta_s$sync $sync TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_CACHE_MISS GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum || exit 1
  pass fetch_s$sync $sync FETCH_SIZE || exit 1
done
python - <<'PY'
import csv, glob, os, collections
O = "gpurun_out/c4diag"
for f in sorted(glob.glob(O + "/*/run_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "scan2_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(os.path.dirname(f)), {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
