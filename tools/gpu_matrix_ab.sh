#!/bin/bash
# Interleaved A/B of library builds on the T = 600 matrix + top-3 workload (config 5-T600):
#   tools/gpu_matrix_ab.sh <reps> <name>...   (name "base" = licensee_amd/lib/liblicensee_dice.so,
#   others licensee_amd/lib/var/<name>.so from tools/build_variant.sh)
export TMPDIR=/tmp
REPS=$1; shift
mkdir -p gpurun_out
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    if [ "$v" = base ]; then unset LICENSEE_DICE_LIB; else export LICENSEE_DICE_LIB=licensee_amd/lib/var/$v.so; fi
    timeout -k 10 240 python bench.py --config 5-T600 --steps 10 --warmup 2 --no-cpu-baseline --no-extras \
      --extra-configs= > gpurun_out/mab_${v}_$rep.json 2> gpurun_out/mab_${v}_$rep.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/mab_${v}_$rep.json'));print('$v rep$rep', round(d['roofline']['launch_ms'],3), 'ms frac', round(d['roofline']['frac'],3))"
  done
done
