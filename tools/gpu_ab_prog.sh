#!/bin/bash
# A/B of sparse-program load schedules on config 2 (one box session; variants interleaved
# twice so box-to-box clock differences do not enter the comparison).
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['value']/1e9,3), 'Gfiles/s', round(d['roofline']['launch_ms']*1000,1), 'us', round(d['roofline']['frac'],3))"
}
for rep in 1 2; do
run ring8_$rep DICE_PROG_SCHED=ring
run ring4_$rep DICE_PROG_SCHED=ring DICE_PROG_PREFETCH=4
run ring4nt_$rep DICE_PROG_SCHED=ring DICE_PROG_PREFETCH=4 DICE_PROG_NT=1
run b3x1_$rep DICE_PROG_BURST=3 DICE_PROG_TILES=1
run b3x1nt_$rep DICE_PROG_BURST=3 DICE_PROG_TILES=1 DICE_PROG_NT=1
run b2x1_$rep DICE_PROG_BURST=2 DICE_PROG_TILES=1
run b2x1nt_$rep DICE_PROG_BURST=2 DICE_PROG_TILES=1 DICE_PROG_NT=1
run b3x2_$rep DICE_PROG_BURST=3 DICE_PROG_TILES=2
run b2x2_$rep DICE_PROG_BURST=2 DICE_PROG_TILES=2
done
