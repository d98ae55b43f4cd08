#!/bin/bash
# Sparse-program burst depth A/B on config 2 (DICE_PROG_BURST; hiprtc compiles each variant once).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${BURSTS:-5}; do
  DICE_PROG_BURST=$b timeout -k 10 300 python bench.py --steps 50 --warmup 5 --extra-configs= --no-cpu-baseline > gpurun_out/burst$b.json 2> gpurun_out/burst$b.err || exit 10
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['roofline']['launch_ms']*1e3,2), 'us', round(d['roofline']['frac'],4))" gpurun_out/burst$b.json
done
