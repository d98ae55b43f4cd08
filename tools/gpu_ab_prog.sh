#!/bin/bash
# A/B of the quad processing order (memory order vs costliest-first vs zipped) on config 2.
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err || { echo "$tag failed"; tail -3 gpurun_out/ab/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$tag.json'));print('$tag', round(d['roofline']['launch_ms']*1000,1), 'us')"
}
for rep in 1 2 3; do
run asc_$rep DICE_X=0
run desc_$rep DICE_PROG_QORDER=desc
run zip_$rep DICE_PROG_QORDER=zip
run desc4_$rep DICE_PROG_QORDER=desc DICE_PROG_BURST=4
done
