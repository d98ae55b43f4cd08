#!/bin/bash
# A/B: vocabulary packing (entries 1347 -> 1088) on config 2, interleaved.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['value']/1e9,3), 'Gfiles/s', round(d['roofline']['launch_ms']*1000,1), 'us', d['config']['program_entries'])"
}
for rep in 1 2 3; do
run base_$rep DICE_PROG_SCHED=ring
run perm_$rep DICE_PROG_SCHED=ring DICE_EXP_VOCAB_PERM=tools/exp/order47.bin
run permb3_$rep DICE_PROG_BURST=3 DICE_PROG_TILES=1 DICE_PROG_NT=1 DICE_EXP_VOCAB_PERM=tools/exp/order47.bin
done
DICE_PROG_SCHED=ring DICE_EXP_VOCAB_PERM=tools/exp/order47.bin timeout -k 10 300 python bench.py --steps 20 --warmup 2 > gpurun_out/ab/perm_parity.json 2> gpurun_out/ab/perm_parity.err || exit 2
python -c "import json;d=json.load(open('gpurun_out/ab/perm_parity.json'));print('parity', d['parity'])"
