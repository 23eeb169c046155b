#!/bin/bash
# Candidate-pass variant sweep: bash profiles/scripts/sweep.sh PREC CONFIG "VARIANTS" "NWGS"
set -o pipefail
export TMPDIR=/tmp
PREC=${1:-bf16x3}; CFG=${2:-c2}; VARIANTS=${3:-"0 1 2"}; NWGS=${4:-"0"}
mkdir -p gpurun_out
for v in $VARIANTS; do
  for nwg in $NWGS; do
    extra=""; [ "$nwg" != "0" ] && extra="--n-wg $nwg"
    f=gpurun_out/sweep_${PREC}_${CFG}_v${v}_w${nwg}
    timeout -k 10 300 python bench.py --config $CFG --precision $PREC --steps 30 --warmup 3 --no-cpu-baseline --scan-variant $v $extra > $f.json 2> $f.err || { echo "variant $v nwg $nwg failed"; tail -5 $f.err; exit 1; }
    python -c "import json;d=json.load(open('$f.json'));r=d['roofline'];print('$PREC $CFG variant $v nwg $nwg', round(d['value']), 'qps scan_ms', round(r['avg_launch_ms'],4), 'pipe_ms', round(d['pipeline_ms'],4), 'step_ms', round(d['ms_per_step'],4), 'hbm', round(r['hbm_gbs']), 'mfma_tf', round(r['mfma_tflops'],1), 'fallback', d['fallback_queries_total'])"
  done
done
