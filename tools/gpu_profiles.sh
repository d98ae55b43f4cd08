#!/bin/bash
# Round profiles: rocprofv3 kernel trace + PMC passes for configs 2-5 (tools/profile_round.sh),
# then an interleaved A/B of the matrix kernels' load schedule (config 5).
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_round.sh r1c_config2 || exit 1
bash tools/profile_round.sh r1c_config3 --config 3 || exit 2
bash tools/profile_round.sh r1c_config4 --config 4 || exit 3
bash tools/profile_round.sh r1c_config5 --config 5 || exit 4
echo profiles_ok
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config 5 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['value']/1e9,3), 'Gfiles/s', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
mkdir -p gpurun_out/ab
for rep in 1 2; do
run c5burst_$rep DICE_X=0
run c5ring_$rep DICE_PROG_SCHED=ring DICE_PROG_NT=0
run c5ringnt_$rep DICE_PROG_SCHED=ring
done
