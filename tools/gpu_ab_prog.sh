#!/bin/bash
# A/B of quad orders x burst sizes on config 2 (interleaved, one box).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3; do
run zip5_$rep DICE_X=0
run snake5_$rep DICE_PROG_QORDER=snake
run zip4_$rep DICE_PROG_BURST=4
run zip6_$rep DICE_PROG_BURST=6
run snake4_$rep DICE_PROG_QORDER=snake DICE_PROG_BURST=4
done
