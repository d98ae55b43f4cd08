#!/bin/bash
# A/B of sparse-program occupancy/burst knobs on config 2 (interleaved, one box).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['value']/1e9,3), 'Gfiles/s', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3; do
run b3_$rep DICE_X=0
run b2_$rep DICE_PROG_BURST=2
run b2w6_$rep DICE_PROG_BURST=2 DICE_PROG_WAVES=6
run b4_$rep DICE_PROG_BURST=4
done
