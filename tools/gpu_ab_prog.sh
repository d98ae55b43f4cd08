#!/bin/bash
# A/B of sparse-program burst size / asm block size on config 2 (interleaved, one box).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3 4; do
run b3_$rep DICE_X=0
run b4_$rep DICE_PROG_BURST=4
run b5_$rep DICE_PROG_BURST=5
run b4a16_$rep DICE_PROG_BURST=4 DICE_PROG_ACC_BLOCK=16
run b4a4_$rep DICE_PROG_BURST=4 DICE_PROG_ACC_BLOCK=4
done
