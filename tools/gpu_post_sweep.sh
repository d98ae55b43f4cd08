#!/bin/bash
# Postings-kernel A/B on config 3: dense-prefix sizes and phase-skip diagnostics (results wrong
# under DICE_POST_DIAG), then one PMC pass. Run under gpurun from the repo root.
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
run() {  # tag, env...
  local tag=$1; shift
  env "$@" DICE_LARGE_KERNEL=post timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline --extra-configs= > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || exit 7
  python -c "import json;d=json.load(open('gpurun_out/sweep/$tag.json'));print('$tag', round(d['roofline']['launch_ms'],3), 'ms')"
}
for D in ${SWEEP_D:-8 13 16}; do run d$D DICE_POST_DENSE=$D; done
for G in ${SWEEP_DIAG:-1 2 4 6}; do run diag$G DICE_POST_DIAG=$G; done
