#!/bin/bash
# Diagnostic: where the config-2 program kernel's time goes (results of DIAG runs are wrong).
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline "${EXTRA[@]}" > gpurun_out/diag/$tag.json 2> gpurun_out/diag/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/diag/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/diag/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2; do
EXTRA=(--probe); run probe_$rep DICE_X=0
EXTRA=()
run full_$rep DICE_X=0
run noacc_$rep DICE_PROG_DIAG=noacc
run noepi_$rep DICE_PROG_DIAG=noepi
done
